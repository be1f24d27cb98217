// fp64_ilp.hip -- diagnostic for the ALARM specialized kernel's latency bound (one wave per SIMD):
// (1) wall-clock SIMD cycles per fp64 add / mul at 1 and 2 waves per SIMD as the number of
//     independent dependency chains per wave grows (1 .. 32): dependent latency vs issue rate;
// (2) the same for a 32-bit integer op (v_and) and a 64-bit select (2 x v_cndmask_b32);
// (3) accuracy of v_rcp_f64 and of one / two Newton steps against IEEE 1/x and a/x, over 4M
//     random operands spanning 2^-60 .. 2^60 (the fast-order division candidates).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/fp64_ilp.hip -o tools/micro/fp64_ilp
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdio>
#include <random>
#include <vector>

template <int K, int OP>
__global__ __launch_bounds__(64) void chains(double *out, int iters, double a) {
    const int lane = threadIdx.x;
    double x[K];
    unsigned u[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = lane * 1e-3 + k, u[k] = lane * 7 + k;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (OP == 0) x[k] = x[k] + a;
            else if (OP == 1) x[k] = x[k] * a;
            else if (OP == 2) u[k] = (u[k] & 0x7fffffffu) ^ (unsigned)i;  // v_and + v_xor: 2 int ops
            else x[k] = (u[k] & (1u << (i & 31))) ? x[k] : a;            // 64-bit select
        }
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k] + (double)u[k];
    out[blockIdx.x * 64 + lane] = s;
}

template <int K, int OP>
void run(double *out, hipEvent_t e0, hipEvent_t e1, int wps, const char *name) {
    const int iters = 20000, waves = 1024 * wps;
    hipLaunchKernelGGL((chains<K, OP>), dim3(waves), dim3(64), 0, 0, out, 100, 1.0000001);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((chains<K, OP>), dim3(waves), dim3(64), 0, 0, out, iters, 1.0000001);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double per = ms * 1e-3 * 2.4e9 / ((double)iters * K) / wps;
    printf("%-10s waves/SIMD %d chains %2d: %7.3f ms  %6.2f SIMD cycles per op (aggregate)\n", name, wps, K, ms, per);
}

__global__ void rcp_acc(const double *x, const double *a, long n, unsigned long long *worst) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i], q0 = a[i] / d, r = 1.0 / d;
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0), r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0), r2 = __builtin_fma(r1, e1, r1);
    const double q1 = a[i] * r1, q2 = a[i] * r2;
    const double t = __builtin_fma(-d, q1, a[i]), q1m = __builtin_fma(t, r1, q1);  // Markstein on r1
    const double errs[6] = {fabs(r0 - r) / r, fabs(r1 - r) / r, fabs(r2 - r) / r,
                            fabs(q1 - q0) / fabs(q0), fabs(q2 - q0) / fabs(q0), fabs(q1m - q0) / fabs(q0)};
    for (int k = 0; k < 6; ++k) {
        // relative errors are >= 0: their bit patterns order like the values
        atomicMax(worst + k, (unsigned long long)__double_as_longlong(errs[k]));
    }
    if (q1m != q0) atomicAdd(worst + 6, 1ull);
    if (q2 != q0) atomicAdd(worst + 7, 1ull);
}

int main() {
    double *out;
    if (hipMalloc(&out, 2048 * 64 * 8) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int wps : {1, 2}) {
        run<1, 0>(out, e0, e1, wps, "f64 add");
        run<2, 0>(out, e0, e1, wps, "f64 add");
        run<4, 0>(out, e0, e1, wps, "f64 add");
        run<8, 0>(out, e0, e1, wps, "f64 add");
        run<16, 0>(out, e0, e1, wps, "f64 add");
        run<32, 0>(out, e0, e1, wps, "f64 add");
        run<1, 1>(out, e0, e1, wps, "f64 mul");
        run<8, 1>(out, e0, e1, wps, "f64 mul");
        run<32, 1>(out, e0, e1, wps, "f64 mul");
        run<1, 2>(out, e0, e1, wps, "i32 and+xor");
        run<8, 2>(out, e0, e1, wps, "i32 and+xor");
        run<32, 2>(out, e0, e1, wps, "i32 and+xor");
        run<8, 3>(out, e0, e1, wps, "f64 select");
        run<32, 3>(out, e0, e1, wps, "f64 select");
    }
    const long n = 1 << 22;
    std::vector<double> hx(n), ha(n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> ex(-60, 60), mant(1, 2);
    for (long i = 0; i < n; ++i) hx[i] = std::ldexp(mant(g), (int)ex(g)), ha[i] = std::ldexp(mant(g), (int)ex(g));
    double *dx, *da;
    unsigned long long *w;
    (void)hipMalloc(&dx, n * 8);
    (void)hipMalloc(&da, n * 8);
    (void)hipMalloc(&w, 64);
    (void)hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(da, ha.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemset(w, 0, 64);
    hipLaunchKernelGGL(rcp_acc, dim3((n + 255) / 256), dim3(256), 0, 0, dx, da, n, w);
    unsigned long long hw[8];
    (void)hipMemcpy(hw, w, 64, hipMemcpyDeviceToHost);
    const char *names[6] = {"rcp", "rcp+1NR", "rcp+2NR", "a*(rcp+1NR)", "a*(rcp+2NR)", "Markstein(rcp+1NR)"};
    for (int k = 0; k < 6; ++k) {
        double v;
        std::memcpy(&v, &hw[k], 8);
        printf("max rel err %-20s %.3e\n", names[k], v);
    }
    printf("quotients != IEEE a/x of %ld: Markstein(rcp+1NR) %llu, a*(rcp+2NR) %llu\n", n, hw[6], hw[7]);
    return 0;
}
