// fp64 VALU dependent-chain latency vs independent issue rate, one wave per SIMD (s_memtime)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void chain(double *out, unsigned long long *cyc, double a) {
    double x[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) x[k] = threadIdx.x + k;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1024; ++i) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) x[k] = x[k] + a;
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) s += x[k];
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
void run(double *d, unsigned long long *c) {
    hipLaunchKernelGGL(chain<CHAINS>, dim3(1), dim3(64), 0, 0, d, c, 1.000001);
    hipLaunchKernelGGL(chain<CHAINS>, dim3(1), dim3(64), 0, 0, d, c, 1.000001);
    unsigned long long h;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("chains %2d: %8.2f cycles per add per chain-step, %6.2f cycles per add\n", CHAINS, h / 1024.0,
           h / 1024.0 / CHAINS);
}

int main() {
    double *d;
    unsigned long long *c;
    (void)hipMalloc(&d, 1 << 20);
    (void)hipMalloc(&c, 4096);
    run<1>(d, c);
    run<2>(d, c);
    run<4>(d, c);
    run<8>(d, c);
    run<16>(d, c);
    return 0;
}
