// exec_half.hip -- diagnostic: does a wave64 fp64 VALU instruction run faster when half of its
// lanes are masked off (EXEC upper 32 bits zero) on gfx950?  Times a dependent-free fp64 FMA
// stream per wave (8 independent chains) with 64 and 32 active lanes, at 1, 2 and 4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/exec_half.hip -o tools/micro/exec_half
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64, 2) void fma_stream(double *out, int iters, int active) {
    const int lane = threadIdx.x;
    if (lane >= active) return;  // EXEC mask for the rest of the kernel
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = lane * 0.001 + k;
    const double b = 1.0000001, c = 1e-9;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fma(a[k], b, c);
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    out[blockIdx.x * 64 + lane] = s;
}

int main() {
    double *out;
    if (hipMalloc(&out, 4096 * 64 * 8) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 100000;
    for (int waves : {1024, 2048, 4096})
        for (int active : {64, 32}) {
            hipLaunchKernelGGL(fma_stream, dim3(waves), dim3(64), 0, 0, out, 1000, active);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(fma_stream, dim3(waves), dim3(64), 0, 0, out, iters, active);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double cyc = ms * 1e-3 * 2.4e9 / (iters * 8.0) / (waves / 1024);
            printf("%d waves (%d per SIMD), active lanes %2d: %.3f ms  ~%.2f SIMD cycles per wave fp64 FMA\n", waves,
                   waves / 1024, active, ms, cyc);
        }
    return 0;
}
