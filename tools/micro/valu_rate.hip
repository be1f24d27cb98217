// valu_rate.hip -- diagnostic: int32 VALU issue rate on gfx950 for the bit-sliced CI kernels' inner
// ops, 16 independent chains per lane, 8 waves per SIMD (8192 blocks of 256 threads):
//   kind 0: xor + v_bcnt_u32_b32 (popcount + accumulate)   2 instructions per chain step
//   kind 1: (a & b) ^ k -- the compiler emits ONE v_bitop3_b32   1 instruction per step
//   kind 2: and + bcnt (the CI kernels' inner pair)            2 instructions per step
// Measured (round 2): kind 1 70 T instr-lanes/s (0.89 of the 78.6 T issue peak: 2 cycles per wave64
// instruction), kind 0 / 2: 29 / 34 ms vs 9.6 ms -- v_bcnt_u32_b32 issues at half rate (4 cycles).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rate.hip -o tools/micro/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(256) void stream(unsigned *out, int iters, unsigned seed) {
    unsigned a[16], b = seed ^ threadIdx.x;
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = seed * (k + 1) + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (KIND == 0) a[k] += __builtin_popcount(b ^ (unsigned)k);  // bcnt with accumulate (+ xor folded?)
            if (KIND == 1) a[k] = (a[k] & b) ^ (unsigned)k;              // and + xor
            if (KIND == 2) a[k] += __builtin_popcount(a[(k + 1) & 15] & b);  // and + bcnt
        }
        b += 0x9E3779B9u;
    }
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    unsigned *out;
    const int blocks = 8192, iters = 20000;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[3] = {"bcnt(xor) ", "and+xor   ", "and+bcnt  "};
    for (int kind = 0; kind < 3; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0, 0);
            if (kind == 0) hipLaunchKernelGGL(stream<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
            if (kind == 1) hipLaunchKernelGGL(stream<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
            if (kind == 2) hipLaunchKernelGGL(stream<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 7u);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double steps = 16.0 * iters * (double)blocks * 256;  // chain steps (lanes)
            if (rep) printf("%s %.3f ms  %.1f T chain-steps/s\n", names[kind], ms, steps / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
