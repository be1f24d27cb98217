// gather_rate.hip -- per-CU cost of the memory operations a C-cases-per-wave JT layout would use
// (round 4 design study): 8-B LDS gathers, 8-B global gathers with 8 / 64 distinct addresses per
// wave-instruction (L1/L2-resident), LDS fp64 atomic adds with 8-way and no address conflicts.
// Build: hipcc -O3 --offload-arch=gfx950 -o gather_rate gather_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096;
constexpr int UNR = 8;

template <int MODE>
__global__ __launch_bounds__(256) void k(const double *__restrict__ g, double *__restrict__ out, int salt) {
    __shared__ double s[4096];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4096; i += 256) s[i] = (double)(i ^ salt);
    __syncthreads();
    double acc = 0.0;
    // per-lane address components: slot = lane % 8 (8 distinct rows), case = lane / 8
    const int slot = lane & 7, cse = lane >> 3;
    unsigned a = (unsigned)(slot * 37 + blockIdx.x) & 511u;
    for (int it = 0; it < ITERS; it += UNR) {
        double v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const unsigned step = (unsigned)(it + u) * 13u;
            if (MODE == 0) {  // LDS gather: 8 rows x 8 cases (64-B rows), ds_read_b64
                const unsigned row = (a + step) & 255u;
                v[u] = s[row * 8 + cse];
            } else if (MODE == 1) {  // global gather: 8 distinct 64-B rows per wave, L1/L2 resident (32 KB)
                const unsigned row = (a + step) & 511u;
                v[u] = g[row * 8 + cse];
            } else if (MODE == 2) {  // global: one contiguous 512-B segment per wave (coalesced)
                const unsigned row = (step + blockIdx.x) & 63u;
                v[u] = g[row * 64 + lane];
            } else if (MODE == 3) {  // global: 8 lanes share one address, 8 distinct 8-B addresses (one 64-B line)
                const unsigned row = (step + blockIdx.x) & 511u;
                v[u] = g[row * 8 + slot];
            } else {  // MODE 4: LDS atomic add fp64, 8 distinct addresses (lanes of a case collide)
                const unsigned row = (a + step) & 255u;
                atomicAdd(&s[row * 8 + slot], 1.0);
                v[u] = 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc += v[u];
    }
    if (MODE == 4) {
        __syncthreads();
        acc = s[threadIdx.x];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void k5(double *__restrict__ out) {  // LDS atomic, 64 distinct addresses
    __shared__ double s[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) s[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int it = 0; it < ITERS; ++it) {
        const unsigned row = ((unsigned)it * 13u + w) & 63u;
        atomicAdd(&s[row * 64 + lane], 1.0);
    }
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = s[threadIdx.x];
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double *g, *out;
    hipMalloc(&g, 64 << 20);
    hipMemset(g, 0, 64 << 20);
    hipMalloc(&out, (size_t)ncu * 16 * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"lds gather b64 (8 rows x 8 cases)", "global gather (8 x 64-B rows, L1/L2)",
                           "global coalesced 512 B", "global 8 addresses x 8 lanes each", "lds atomic add f64 (8-way)",
                           "lds atomic add f64 (no conflict)"};
    for (int wpcu : {4, 8, 16}) {
        const int blocks = ncu * wpcu / 4;  // 4 waves per block
        for (int m = 0; m < 6; ++m) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                switch (m) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, g, out, rep); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, g, out, rep); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, g, out, rep); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, g, out, rep); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, g, out, rep); break;
                default: hipLaunchKernelGGL(k5<0>, dim3(blocks), dim3(256), 0, 0, out); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            const double winstr_per_cu = (double)wpcu * ITERS;
            const double cyc = best * 1e-3 * 2.4e9 / winstr_per_cu;
            printf("waves/CU %2d  %-42s %.3f ms  %.2f CU-cycles per wave-instruction\n", wpcu, names[m], best, cyc);
        }
    }
    return 0;
}
