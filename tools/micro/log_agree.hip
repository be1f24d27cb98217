// log_agree.hip -- diagnostic: how often does the device's fp64 log differ from the host libm's
// (glibc) std::log on the quotients G^2 takes the log of (observed / expected, expected =
// col * row / total, src/IndependenceTest.cpp:134-135)?  Compares the ocml log and a double-double
// (correctly rounded in practice) log against std::log.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/log_agree.hip -o tools/micro/log_agree
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

struct dd {
    double hi, lo;
};
__device__ __forceinline__ dd two_sum(double a, double b) {
    double s = a + b, bb = s - a, e = (a - (s - bb)) + (b - bb);
    return {s, e};
}
__device__ __forceinline__ dd quick_two_sum(double a, double b) {
    double s = a + b;
    return {s, b - (s - a)};
}
__device__ __forceinline__ dd dd_add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi), t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
    double p = a.hi * b.hi, e = fma(a.hi, b.hi, -p);
    e += a.hi * b.lo + a.lo * b.hi;
    return quick_two_sum(p, e);
}
__device__ __forceinline__ dd dd_div(dd a, dd b) {
    double q1 = a.hi / b.hi;
    dd r = dd_add(a, dd_mul({-q1, 0.0}, b));
    double q2 = r.hi / b.hi;
    r = dd_add(r, dd_mul({-q2, 0.0}, b));
    double q3 = r.hi / b.hi;
    dd q = quick_two_sum(q1, q2);
    return dd_add(q, {q3, 0.0});
}

__constant__ double c_inv_hi[24], c_inv_lo[24];

__device__ double log_dd(double x) {
    int k;
    double m = frexp(x, &k);  // x = m 2^k, m in [0.5, 1)
    if (m < 0.70710678118654752) m *= 2.0, k -= 1;
    const double num = m - 1.0;  // exact (Sterbenz)
    dd den = two_sum(m, 1.0);
    dd s = dd_div({num, 0.0}, den);
    dd s2 = dd_mul(s, s);
    dd P = {c_inv_hi[22], c_inv_lo[22]};
    for (int n = 21; n >= 0; --n) P = dd_add(dd_mul(P, s2), {c_inv_hi[n], c_inv_lo[n]});
    dd lm = dd_mul(dd_mul(s, P), {2.0, 0.0});
    const dd ln2 = {0x1.62e42fefa39efp-1, 0x1.abc9e3b39803fp-56};
    dd kl = dd_mul({(double)k, 0.0}, ln2);
    dd r = dd_add(kl, lm);
    return r.hi + r.lo;
}

__global__ void logs(const double *in, double *o1, double *o2, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
        o1[i] = log(in[i]);
        o2[i] = log_dd(in[i]);
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 4000000;
    std::mt19937_64 rng(12345);
    std::vector<double> x(n), h(n), d1(n), d2(n);
    for (long i = 0; i < n; ++i) {
        if (i % 4 == 3) {  // generic doubles
            x[i] = std::exp(std::uniform_real_distribution<double>(-20, 20)(rng));
            continue;
        }
        long total = 100 + (long)(rng() % 200000);
        long sr = 1 + (long)(rng() % total), sc = 1 + (long)(rng() % total);
        long obs = 1 + (long)(rng() % std::min(sr, sc));
        double expected = (double)sc * (double)sr / (double)total;
        x[i] = obs / expected;
    }
    for (long i = 0; i < n; ++i) h[i] = std::log(x[i]);
    double hi[24], lo[24];
    for (int k = 0; k < 24; ++k) {
        const double q = 2.0 * k + 1.0;
        hi[k] = 1.0 / q;
        lo[k] = -std::fma(hi[k], q, -1.0) / q;
    }
    hipMemcpyToSymbol(HIP_SYMBOL(c_inv_hi), hi, sizeof hi);
    hipMemcpyToSymbol(HIP_SYMBOL(c_inv_lo), lo, sizeof lo);
    double *dx, *e1, *e2;
    hipMalloc(&dx, n * 8);
    hipMalloc(&e1, n * 8);
    hipMalloc(&e2, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(logs, dim3(2048), dim3(256), 0, nullptr, dx, e1, e2, n);
    hipMemcpy(d1.data(), e1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(d2.data(), e2, n * 8, hipMemcpyDeviceToHost);
    long m1 = 0, m2 = 0, m12 = 0, m1q = 0, m2q = 0;
    for (long i = 0; i < n; ++i) {
        const bool a = memcmp(&d1[i], &h[i], 8) != 0, b = memcmp(&d2[i], &h[i], 8) != 0;
        m1 += a, m2 += b, m12 += memcmp(&d1[i], &d2[i], 8) != 0;
        if (i % 4 != 3) m1q += a, m2q += b;
        if (b && m2 <= 5) printf("  cr-dd vs libm: x=%a libm=%a dd=%a ocml=%a\n", x[i], h[i], d2[i], d1[i]);
    }
    printf("n=%ld  ocml!=libm %ld (quotients %ld)  dd!=libm %ld (quotients %ld)  ocml!=dd %ld\n", n, m1, m1q, m2, m2q,
           m12);
    return 0;
}
