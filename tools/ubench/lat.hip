// Micro-benchmarks (diagnostic): cycles of the solver's building blocks on one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../colaborativempc-_amd/csrc/wave_ops.h"
using namespace cmpc;
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); asm volatile("" ::: "memory"); }
constexpr int NX = 4, NU = 2, N = 30;

// (a) readlane-broadcast forward recursion (current kernels)
__global__ __launch_bounds__(64,1) void k_fwd_readlane(const double* gA, const double* gB, double* out, unsigned long long* cyc) {
  __shared__ double A[N*NX*NX], B[N*NX*NU], U[64], X[(N+1)*NX];
  int l = threadIdx.x;
  for (int i = l; i < N*NX*NX; i += 64) A[i] = gA[i];
  for (int i = l; i < N*NX*NU; i += 64) B[i] = gB[i];
  U[l] = 0.01 * l;
  __syncthreads();
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) {
    const int s = l < NX ? l : 0;
    double xr = 1.0 + rep;
    for (int k = 0; k < N; ++k) {
      const double* Ak = A + (k * NX + s) * NX;
      const double* Bk = B + (k * NX + s) * NU;
      double v = 0.0;
#pragma unroll
      for (int i = 0; i < NU; ++i) v = fma(Bk[i], U[k * NU + i], v);
#pragma unroll
      for (int t = 0; t < NX; ++t) v = fma(Ak[t], readlane_d(xr, t), v);
      xr = v;
      if (l < NX) X[(k + 1) * NX + l] = v;
    }
    wsync();
  }
  unsigned long long t1 = stamp();
  if (l == 0) { cyc[blockIdx.x] = (t1 - t0) / 10; }
  out[blockIdx.x * 64 + l] = X[(N * NX + l) % ((N+1)*NX)];
}

// (b) replicated state, A/B from LDS broadcast, prefetch one stage ahead
__global__ __launch_bounds__(64,1) void k_fwd_repl(const double* gA, const double* gB, double* out, unsigned long long* cyc) {
  __shared__ double A[N*NX*NX], B[N*NX*NU], U[64], X[(N+1)*NX];
  int l = threadIdx.x;
  for (int i = l; i < N*NX*NX; i += 64) A[i] = gA[i];
  for (int i = l; i < N*NX*NU; i += 64) B[i] = gB[i];
  U[l] = 0.01 * l;
  __syncthreads();
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) {
    double x[NX];
#pragma unroll
    for (int s = 0; s < NX; ++s) x[s] = 1.0 + rep;
    double a[NX*NX], bb[NX];
#pragma unroll
    for (int i = 0; i < NX*NX; ++i) a[i] = A[i];
#pragma unroll
    for (int s = 0; s < NX; ++s) { double v = 0; for (int i = 0; i < NU; ++i) v = fma(B[s*NU+i], U[i], v); bb[s] = v; }
    for (int k = 0; k < N; ++k) {
      double xn[NX];
#pragma unroll
      for (int s = 0; s < NX; ++s) {
        double v = bb[s];
#pragma unroll
        for (int t = 0; t < NX; ++t) v = fma(a[s*NX+t], x[t], v);
        xn[s] = v;
      }
      if (k + 1 < N) {
#pragma unroll
        for (int i = 0; i < NX*NX; ++i) a[i] = A[(k+1)*NX*NX + i];
#pragma unroll
        for (int s = 0; s < NX; ++s) { double v = 0; for (int i = 0; i < NU; ++i) v = fma(B[(k+1)*NX*NU + s*NU+i], U[(k+1)*NU+i], v); bb[s] = v; }
      }
#pragma unroll
      for (int s = 0; s < NX; ++s) x[s] = xn[s];
      if (l < NX) X[(k + 1) * NX + l] = x[l & 3];
    }
    wsync();
  }
  unsigned long long t1 = stamp();
  if (l == 0) { cyc[blockIdx.x] = (t1 - t0) / 10; }
  out[blockIdx.x * 64 + l] = X[(N * NX + l) % ((N+1)*NX)];
}

// (c) 16x16 Cholesky diag block, readlane version (current)
__global__ __launch_bounds__(64,1) void k_chol_readlane(const double* gK, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double rw0[16];
  for (int cc = 0; cc < 16; ++cc) rw0[cc] = gK[(l & 15) * 16 + cc];
  double acc = 0;
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) {
    double rw[16];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) rw[cc] = rw0[cc] + rep;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double djj = readlane_d(rw[j], j);
      const double d = sqrt(djj);
      const double lj = (l > j) ? rw[j] / d : ((l == j) ? d : rw[j]);
      rw[j] = lj;
#pragma unroll
      for (int cc = j + 1; cc < 16; ++cc) rw[cc] = fma(-lj, readlane_d(lj, cc), rw[cc]);
    }
    acc += rw[l & 15];
  }
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0) / 10;
  out[blockIdx.x * 64 + l] = acc;
}

// (d) 16x16 Cholesky diag block: rsqrt pivot, lower triangle only, column broadcast through LDS
__global__ __launch_bounds__(64,1) void k_chol_lds(const double* gK, double* out, unsigned long long* cyc) {
  __shared__ double col[16 * 16];
  int l = threadIdx.x;
  double rw0[16];
  for (int cc = 0; cc < 16; ++cc) rw0[cc] = gK[(l & 15) * 16 + cc];
  double acc = 0;
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) {
    double rw[16];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) rw[cc] = rw0[cc] + rep;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double djj = readlane_d(rw[j], j);
      double y = __builtin_amdgcn_rsq(djj);            // ~ 2^-? accurate
      y = y * (1.5 - 0.5 * djj * y * y);
      y = y * (1.5 - 0.5 * djj * y * y);
      const double lj = (l > j) ? rw[j] * y : ((l == j) ? djj * y : 0.0);
      rw[j] = lj;
      if (l < 16) col[j * 16 + l] = lj;
      wsync();
#pragma unroll
      for (int cc = j + 1; cc < 16; ++cc) rw[cc] = fma(-lj, col[j * 16 + cc], rw[cc]);
    }
    acc += rw[l & 15];
  }
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0) / 10;
  out[blockIdx.x * 64 + l] = acc;
}

// (e) MFMA f64 16x16x4: 10 independent accumulators, 10 rounds
__global__ __launch_bounds__(64,1) void k_mfma(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  v4d acc[10];
  for (int q = 0; q < 10; ++q) acc[q] = v4d{0,0,0,0};
  double a = gA[l], b = gA[64 + l];
  double av[10];
  for (int q = 0; q < 10; ++q) av[q] = a + q;
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) {
#pragma unroll
    for (int q = 0; q < 10; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], b, acc[q], 0, 0, 0);
  }
  double s0 = acc[9][0]; asm volatile("v_mov_b64 %0, %0" : "+v"(s0));
  unsigned long long t1 = stamp();
  double s = 0; for (int q = 0; q < 10; ++q) s += acc[q][0] + acc[q][3];
  if (l == 0) cyc[blockIdx.x] = (t1 - t0) / 10;
  out[blockIdx.x * 64 + l] = s;
}

// (f) dependent f64 FMA chain of 64
__global__ __launch_bounds__(64,1) void k_fma(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double x = gA[l], y = gA[64 + l];
  unsigned long long t0 = stamp();
#pragma unroll
  for (int i = 0; i < 64; ++i) x = fma(x, y, 0.5);
  asm volatile("v_mov_b64 %0, %0" : "+v"(x));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = x;
}

// (g) LDS round trip: write then dependent read chain of 32
__global__ __launch_bounds__(64,1) void k_lds(const double* gA, double* out, unsigned long long* cyc) {
  __shared__ double buf[128];
  int l = threadIdx.x;
  buf[l] = gA[l]; buf[64 + l] = 0;
  __syncthreads();
  int idx = l;
  double v = 0;
  unsigned long long t0 = stamp();
#pragma unroll
  for (int i = 0; i < 32; ++i) { v = buf[idx]; idx = ((int)v + l) & 63; }
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = v;
}

// (h) readlane_d -> fma dependent chain of 32
__global__ __launch_bounds__(64,1) void k_readlane(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double v = gA[l];
  unsigned long long t0 = stamp();
#pragma unroll
  for (int i = 0; i < 32; ++i) v = fma(readlane_d(v, i & 63), 0.5, v);
  asm volatile("v_mov_b64 %0, %0" : "+v"(v));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = v;
}

// (i) f64 divide and sqrt dependent chains of 16
__global__ __launch_bounds__(64,1) void k_div(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double v = gA[l] + 2.0, w = gA[64+l] + 3.0;
  unsigned long long t0 = stamp();
#pragma unroll
  for (int i = 0; i < 16; ++i) v = w / v + 1.0;
  asm volatile("v_mov_b64 %0, %0" : "+v"(v));
  unsigned long long t1 = stamp();
#pragma unroll
  for (int i = 0; i < 16; ++i) w = sqrt(w) + 1.0;
  asm volatile("v_mov_b64 %0, %0" : "+v"(w));
  unsigned long long t2 = stamp();
  if (l == 0) { cyc[blockIdx.x] = (t1 - t0); cyc[1024 + blockIdx.x] = t2 - t1; }
  out[blockIdx.x * 64 + l] = v + w;
}


__global__ __launch_bounds__(64,1) void k_mfma_dep(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  v4d acc = {0,0,0,0};
  double a = gA[l], b = gA[64 + l];
  unsigned long long t0 = stamp();
#pragma unroll
  for (int rep = 0; rep < 32; ++rep) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  double s0 = acc[0]; asm volatile("v_mov_b64 %0, %0" : "+v"(s0));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = s0;
}

__global__ __launch_bounds__(64,1) void k_mfma_tp(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  v4d acc[10];
  for (int q = 0; q < 10; ++q) acc[q] = v4d{0,0,0,0};
  double a = gA[l], b = gA[64 + l];
  double av[10];
  for (int q = 0; q < 10; ++q) av[q] = a + q;
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 32; ++rep) {
#pragma unroll
    for (int q = 0; q < 10; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], b, acc[q], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 10; ++q) s += acc[q][0];
  asm volatile("v_mov_b64 %0, %0" : "+v"(s));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = s;
}
__global__ __launch_bounds__(64,1) void k_fma_tp(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double x[16];
  for (int q = 0; q < 16; ++q) x[q] = gA[l] + q;
  double y = gA[64 + l];
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 32; ++rep) {
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = fma(x[q], y, 0.5);
  }
  double s = 0;
  for (int q = 0; q < 16; ++q) s += x[q];
  asm volatile("v_mov_b64 %0, %0" : "+v"(s));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = s;
}
__global__ __launch_bounds__(64,1) void k_dpp(const double* gA, double* out, unsigned long long* cyc) {
  int l = threadIdx.x;
  double v = gA[l];
  unsigned long long t0 = stamp();
#pragma unroll
  for (int i = 0; i < 32; ++i) v = fma(cmpc::bcast16<3>(v), 0.5, v);
  asm volatile("v_mov_b64 %0, %0" : "+v"(v));
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0);
  out[blockIdx.x * 64 + l] = v;
}
int main() {
  const int nb = 1024;
  std::vector<double> hA(N*NX*NX*1 + 4096), hK(256);
  for (size_t i = 0; i < hA.size(); ++i) hA[i] = ((i * 37) % 11) * 0.01 + ((i % 5) == 0);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) hK[i*16+j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
  double *dA, *dK, *out; unsigned long long* cyc;
  hipMalloc(&dA, hA.size() * 8); hipMalloc(&dK, 256 * 8); hipMalloc(&out, nb * 64 * 8); hipMalloc(&cyc, 2048 * 8);
  hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice); hipMemcpy(dK, hK.data(), 256 * 8, hipMemcpyHostToDevice);
  std::vector<unsigned long long> hc(2048);
  auto rep = [&](const char* nm, int div) {
    hipDeviceSynchronize(); hipMemcpy(hc.data(), cyc, 2048 * 8, hipMemcpyDeviceToHost);
    double s = 0; for (int i = 0; i < nb; ++i) s += hc[i];
    printf("%-28s %10.1f cyc (mean over %d waves)%s\n", nm, s / nb / div, nb, div > 1 ? " per unit" : "");
  };
  for (int w = 0; w < 2; ++w) {
    hipLaunchKernelGGL(k_fwd_readlane, dim3(nb), dim3(64), 0, 0, dA, dA, out, cyc); rep("fwd readlane (30 stages)", 1);
    hipLaunchKernelGGL(k_fwd_repl, dim3(nb), dim3(64), 0, 0, dA, dA, out, cyc); rep("fwd replicated (30 stages)", 1);
    hipLaunchKernelGGL(k_chol_readlane, dim3(nb), dim3(64), 0, 0, dK, out, cyc); rep("chol16 readlane", 1);
    hipLaunchKernelGGL(k_chol_lds, dim3(nb), dim3(64), 0, 0, dK, out, cyc); rep("chol16 rsq+lds", 1);
    hipLaunchKernelGGL(k_mfma, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("mfma f64 x10 indep (per mfma)", 100);
    hipLaunchKernelGGL(k_mfma_dep, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("mfma f64 dependent chain", 32);
    hipLaunchKernelGGL(k_mfma_tp, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("mfma f64 throughput (10 indep, drained)", 320);
    hipLaunchKernelGGL(k_fma_tp, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("fma f64 throughput (16 indep)", 512);
    hipLaunchKernelGGL(k_dpp, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("dpp bcast -> fma dep chain", 32);
    hipLaunchKernelGGL(k_fma, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("fma f64 dep chain", 64);
    hipLaunchKernelGGL(k_lds, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("lds dep read", 32);
    hipLaunchKernelGGL(k_readlane, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("readlane_d->fma dep", 32);
    hipLaunchKernelGGL(k_div, dim3(nb), dim3(64), 0, 0, dA, out, cyc); rep("f64 div dep", 16);
    { double s = 0; for (int i = 0; i < nb; ++i) s += hc[1024 + i]; printf("%-28s %10.1f cyc per unit\n", "f64 sqrt dep", s / nb / 16); }
  }
  return 0;
}
