// Diagnostic: cycles of the v3 forward recursion alone (NX=4, NU=2, N=30), one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../../colaborativempc-_amd/csrc/wave_ops.h"
using namespace cmpc;
constexpr int NX = 4, NU = 2, N = 30;
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
template <int NX, int NU>
__device__ __forceinline__ void fwd3(int l, int N, const double* A, const double* B, const double* x0,
                                     const double* U, double* X) {
    const int s = (l & 15) < NX ? (l & 15) : 0;
    double xr = x0 ? x0[s] : 0.0;
    if (l < NX) X[l] = xr;
    double a[NX], bu = 0.0;
    auto fetch = [&](int k, double* av, double& b) {
#pragma unroll
        for (int t = 0; t < NX; ++t) av[t] = A[(k * NX + s) * NX + t];
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < NU; ++i) v = fma(B[(k * NX + s) * NU + i], U[k * NU + i], v);
        b = v;
    };
    if (N > 0) fetch(0, a, bu);
    for (int k = 0; k < N; ++k) {
        double an[NX], bn = 0.0;
        if (k + 1 < N) fetch(k + 1, an, bn);
        double v0 = bu, v1 = 0.0;
        static_for<0, NX>([&](auto t) __attribute__((always_inline)) {
            constexpr int tt = decltype(t)::value;
            if constexpr (tt & 1) v1 = fma(a[tt], bcast16<tt>(xr), v1);
            else v0 = fma(a[tt], bcast16<tt>(xr), v0);
        });
        xr = v0 + v1;
        if (l < NX) X[(k + 1) * NX + l] = xr;
#pragma unroll
        for (int t = 0; t < NX; ++t) a[t] = an[t];
        bu = bn;
    }
}
__global__ __launch_bounds__(64,1) void k_fwd(const double* gA, double* out, unsigned long long* cyc) {
  __shared__ double A[N*NX*NX], B[N*NX*NU], U[64], X[(N+1)*NX], x0[4];
  int l = threadIdx.x;
  for (int i = l; i < N*NX*NX; i += 64) A[i] = gA[i] * 0.1;
  for (int i = l; i < N*NX*NU; i += 64) B[i] = gA[i];
  U[l] = 0.01 * l; if (l < 4) x0[l] = 1.0;
  __syncthreads();
  unsigned long long t0 = stamp();
  for (int rep = 0; rep < 10; ++rep) { fwd3<NX, NU>(l, N, A, B, x0, U, X); __syncthreads(); }
  unsigned long long t1 = stamp();
  if (l == 0) cyc[blockIdx.x] = (t1 - t0) / 10;
  out[blockIdx.x * 64 + l] = X[(N * NX + l) % ((N+1)*NX)];
}
int main() {
  const int nb = 1024;
  std::vector<double> h(4096, 0.5);
  double *dA, *out; unsigned long long* cyc;
  hipMalloc(&dA, 4096 * 8); hipMalloc(&out, nb * 64 * 8); hipMalloc(&cyc, nb * 8);
  hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  std::vector<unsigned long long> hc(nb);
  for (int w = 0; w < 3; ++w) {
    hipLaunchKernelGGL(k_fwd, dim3(nb), dim3(64), 0, 0, dA, out, cyc);
    hipDeviceSynchronize(); hipMemcpy(hc.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
    double s = 0; for (int i = 0; i < nb; ++i) s += hc[i];
    printf("fwd3 dpp (30 stages): %.1f cyc  (%.1f / stage)\n", s / nb, s / nb / N);
  }
}
