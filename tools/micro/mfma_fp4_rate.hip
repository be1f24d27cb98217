// mfma_fp4_rate.hip -- diagnostic: v_mfma_scale_f32_32x32x64_f8f6f4 (FP4 x FP4) issue rate with one
// wave per SIMD (256-thread blocks, one per CU: the level-0 Gram's shape, ci_gram_mfma.hip), and
// what the Gram kernel's per-stage extras cost on top of 32 MFMAs per stage:
//   kind 0: 16 accumulators, 32 MFMAs per stage, operands from registers
//   kind 1: + 16 ds_read_b128 per stage (the fragment reads), waited once per 16 MFMAs
//   kind 2: kind 1 + one s_barrier per stage
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_fp4_rate.hip -o tools/micro/mfma_fp4_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16f mm(v4i a, v4i b, v16f c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{a[0], a[1], a[2], a[3], 0, 0, 0, 0},
                                                           v8i{b[0], b[1], b[2], b[3], 0, 0, 0, 0}, c, 4, 4, 0, 0, 0, 0);
}

template <int KIND>
__global__ __launch_bounds__(256, 1) void rate(float *out, int stages, int seed) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<int *>(lds)[i] = (i * 2654435761u) & 0x22222222;
    __syncthreads();
    v16f acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[m][n][j] = 0.f;
    v4i a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = v4i{seed + k, lane, 0x22, k}, b[k] = v4i{lane, seed, k, 0x20};
    const int off = (threadIdx.x >> 6) * 8192 + lane * 16;
    for (int t = 0; t < stages; ++t) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if (KIND >= 1) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a[k] = *reinterpret_cast<const v4i *>(lds + off + ((t + s) & 3) * 1024 + k * 2048 % 8192);
                    b[k] = *reinterpret_cast<const v4i *>(lds + off + 4096 % 8192 + k * 1024);
                }
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = mm(a[m], b[n], acc[m][n]);
        }
        if (KIND >= 2) __builtin_amdgcn_s_barrier();
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j) s += acc[m][n][j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
static float run(float *out, int blocks, int stages) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, stages, 1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, stages, 1);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    if (hipMalloc(&out, (size_t)cus * 256 * 4) != hipSuccess) return 1;
    const int stages = 112;
    const double flops = (double)cus * 4 * stages * 32 * 32.0 * 32 * 64 * 2;
    const float t0 = run<0>(out, cus, stages), t1 = run<1>(out, cus, stages), t2 = run<2>(out, cus, stages);
    printf("blocks %d stages %d: regs-only %.1f us (%.2f PF/s)  +ds_reads %.1f us (%.2f)  +barrier %.1f us (%.2f)\n", cus,
           stages, 1e3 * t0, flops / t0 / 1e12, 1e3 * t1, flops / t1 / 1e12, 1e3 * t2, flops / t2 / 1e12);
    return 0;
}
