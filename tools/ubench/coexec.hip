// Micro-benchmark (diagnostic): does an f64 MFMA (V_MFMA_F64_16X16X4_F64) co-execute with independent f64
// VALU work issued by the same wave?  One wave per SIMD; per loop trip: NM independent MFMAs (distinct
// accumulators) and NV independent FMAs (8 chains).  Variants: (a) grouped — every MFMA, then every FMA
// (sched_barrier between the groups); (b) interleaved — {1 MFMA, NV/NM FMAs} x NM by sched_group_barrier;
// (c) MFMAs only; (d) FMAs only.  Prints clocks per trip.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

constexpr int NM = 8, NC = 8, NPER = 5, NV = NC * NPER, TRIPS = 200;

template <int MODE>
__global__ __launch_bounds__(64, 1) void k(const double* in, double* out, unsigned long long* cyc) {
    const int l = threadIdx.x;
    double a = in[l], b = in[64 + l];
    v4d acc[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(0.0, 0.0, (v4d){0, 0, 0, 0}, 0, 0, 0);
    double x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = in[128 + c * 64 + l];
    const double m = in[1000 + l], q = in[1100 + l];
    const unsigned long long t0 = stamp();
    for (int t = 0; t < TRIPS; ++t) {
        if constexpr (MODE != 3) {
#pragma unroll
            for (int i = 0; i < NM; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
        }
        if constexpr (MODE == 0) __builtin_amdgcn_sched_barrier(0);
        if constexpr (MODE != 2) {
#pragma unroll
            for (int j = 0; j < NPER; ++j)
#pragma unroll
                for (int c = 0; c < NC; ++c) x[c] = fma(x[c], m, q);
        }
        if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, NV / NM, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = stamp();
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NM; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
    for (int c = 0; c < NC; ++c) s += x[c];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = (t1 - t0);
}

int main() {
    double *in, *out;
    unsigned long long* cyc;
    hipMalloc(&in, 4096 * 8);
    hipMalloc(&out, 64 * 1024 * 8);
    hipMalloc(&cyc, 1024 * 8);
    double h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0 + 1e-3 * (i % 97);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[4] = {"grouped (MFMAs, then FMAs)", "interleaved (1 MFMA : 5 FMA)", "MFMA only", "FMA only"};
    void (*ks[4])(const double*, double*, unsigned long long*) = {k<0>, k<1>, k<2>, k<3>};
    for (int v = 0; v < 4; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(ks[v], dim3(1024), dim3(64), 0, 0, in, out, cyc);
            hipDeviceSynchronize();
        }
        unsigned long long hc[1024];
        hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 1024; ++i) s += hc[i];
        // s_memtime counts at the constant 100 MHz reference on gfx950? report raw units per trip
        printf("%-32s %8.1f units/trip (NM=%d MFMA, NV=%d FMA)\n", names[v], s / 1024 / TRIPS, NM, NV);
    }
    return 0;
}
