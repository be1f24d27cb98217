// ci_chisq.h -- the chi-square p-value of a G^2 test, shared by ci_kernels.hip and ci_bits.hip.
//
// The reference computes p = 1.0 - stats::pchisq(g2, df) (src/IndependenceTest.cpp:146,268,355);
// pchisq lives in the un-vendored lib/stats submodule (parity unpinned).  Restated
// as the regularized lower incomplete gamma P(df/2, g2/2) (series below a + 1, modified Lentz
// continued fraction for Q = 1 - P above), and p = 1.0 - P exactly as the reference forms it, so a
// CDF that rounds to 1 gives p = 0 as in the reference (alpha = 0 keeps its meaning).  The oracle
// restatement (oracle/pc_oracle.cpp ChiSquarePValue) is the same algorithm.
#ifndef FBN_CI_CHISQ_H
#define FBN_CI_CHISQ_H

#include <hip/hip_runtime.h>

__host__ __device__ inline double fbn_gamma_p(double a, double x) {
    if (x <= 0.0) return 0.0;
    const double lg = lgamma(a);
    if (x < a + 1.0) {
        double ap = a, sum = 1.0 / a, del = sum;
        for (int n = 0; n < 2000; ++n) {
            ap += 1.0;
            del *= x / ap;
            sum += del;
            if (fabs(del) < fabs(sum) * 1e-17) break;
        }
        return sum * exp(-x + a * log(x) - lg);
    }
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 2000; ++i) {
        const double an = -i * (i - a);
        b += 2.0;
        d = an * d + b;
        if (fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < 1e-17) break;
    }
    return 1.0 - exp(-x + a * log(x) - lg) * h;
}

// p = 1 - pchisq(g2, df) (df > 0)
__host__ __device__ inline double fbn_chisq_pvalue(double g2, int df) { return 1.0 - fbn_gamma_p(0.5 * df, 0.5 * g2); }

// Decision band (skeleton-search batches, which need only the decision p > alpha and the margin
// log, not p itself): per df, lo < hi with p(lo) > alpha + delta and p(hi) < alpha - delta, found by
// bisection on this same function.  p is monotone in G^2 and the CDF's rounding error is ~1e-15, far
// below delta, so G^2 < lo decides "independent" and G^2 > hi "dependent" exactly as evaluating p
// would; only tests inside [lo, hi] evaluate p.  Skipped tests are >= delta from alpha.
inline void fbn_chisq_band(double alpha, double delta, int df, double *lo, double *hi) {
    auto bracket = [&](double target, bool want_lo) {
        double a = 0.0, b = df + 10.0 * sqrt(2.0 * df) + 10.0;
        while (fbn_chisq_pvalue(b, df) >= target) a = b, b *= 2.0;  // p(a) >= target > p(b)
        for (int i = 0; i < 40; ++i) {
            const double m = 0.5 * (a + b);
            (fbn_chisq_pvalue(m, df) >= target ? a : b) = m;
        }
        return want_lo ? a : b;
    };
    double l = bracket(alpha + delta, true);
    while (l > 0.0 && !(fbn_chisq_pvalue(l, df) > alpha + delta)) l *= 0.999;  // strict
    double h = bracket(alpha - delta, false);
    while (!(fbn_chisq_pvalue(h, df) < alpha - delta)) h *= 1.001;
    *lo = l, *hi = h;
}

#endif
