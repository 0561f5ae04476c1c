// Calibration (diagnostic): FETCH_SIZE / WRITE_SIZE against a known byte count for the access
// widths and patterns of the solver kernels (MI355X_MICROARCH.md: only 16 B/lane streaming reads and
// stores are calibrated; "calibrate other widths on a known byte count").  Every kernel touches
// exactly `bytes` of a 512 MiB buffer (past the 256 MiB Infinity Cache), once:
//   rd16      16 B per lane, coalesced (double2)                    — the guide's calibrated case
//   rd8       8 B per lane, coalesced (one double per lane)
//   rd8_agent 8 B per lane in 64 KiB per-wave regions, lane l reading elements l, l + 64, ... of its
//             wave's region (the Riccati kernel's per-agent scratch / stage images)
//   wr8       8 B per lane stores, coalesced
//   wr8_agent 8 B per lane stores in per-wave regions (as rd8_agent)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench/fetch_cal tools/ubench/fetch_cal.hip
// Run under rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (another); the program prints
// the bytes each dispatch touches.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = 512ull << 20;
constexpr int kRegion = 64 << 10;  // bytes per wave region (rd8_agent / wr8_agent)

__global__ void rd16(const double2* __restrict__ x, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = x[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[0] = s;  // (never true for zero data: keeps the loads)
}
__global__ void rd8(const double* __restrict__ x, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += x[i];
    if (s == 1.2345) out[0] = s;
}
// one 64-lane workgroup per region
__global__ void rd8_agent(const double* __restrict__ x, double* out) {
    const double* r = x + (size_t)blockIdx.x * (kRegion / 8);
    double s = 0.0;
    for (int i = threadIdx.x; i < kRegion / 8; i += 64) s += r[i];
    if (s == 1.2345) out[0] = s;
}
__global__ void wr8(double* __restrict__ x, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x[i] = 1.0;
}
__global__ void wr8_agent(double* __restrict__ x) {
    double* r = x + (size_t)blockIdx.x * (kRegion / 8);
    for (int i = threadIdx.x; i < kRegion / 8; i += 64) r[i] = 1.0;
}

int main() {
    double *x = nullptr, *out = nullptr;
    if (hipMalloc(&x, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(x, 0, kBytes) != hipSuccess) return 1;
    const size_t n8 = kBytes / 8, n16 = kBytes / 16;
    const int regions = (int)(kBytes / kRegion);
    for (int rep = 0; rep < 3; ++rep) {  // the first dispatch of each kernel is a warm-up
        hipLaunchKernelGGL(rd16, dim3(4096), dim3(256), 0, 0, (const double2*)x, n16, out);
        hipLaunchKernelGGL(rd8, dim3(4096), dim3(256), 0, 0, (const double*)x, n8, out);
        hipLaunchKernelGGL(rd8_agent, dim3(regions), dim3(64), 0, 0, (const double*)x, out);
        hipLaunchKernelGGL(wr8, dim3(4096), dim3(256), 0, 0, x, n8);
        hipLaunchKernelGGL(wr8_agent, dim3(regions), dim3(64), 0, 0, x);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::printf("{\"bytes_per_dispatch\": %zu, \"kernels\": [\"rd16\", \"rd8\", \"rd8_agent\", \"wr8\", \"wr8_agent\"]}\n",
                kBytes);
    (void)hipFree(x);
    (void)hipFree(out);
    return 0;
}
