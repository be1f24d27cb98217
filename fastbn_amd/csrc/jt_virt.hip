// jt_virt.hip -- streamed ("virtual table") junction-tree kernel for large trees (Munin class).
//
// One lane = one evidence case, 64 cases per wave, persistent waves (as jt_kernels.hip).  No
// clique table is ever stored: every pass over a clique recomputes each entry it needs as
//     c_0(e) = mask(e) ? init(e) : 0,     c_j(e) = (c_{j-1}(e) / D_{j-1}) * M_j(e)
// from the constant initial potentials (scalar loads shared by the 64 cases), the lane's evidence
// mask, the messages received so far (M_1..M_k: child Collect messages in multiplication order,
// M_{k+1}: the parent's Distribute message) and the per-step normalization sums D_j.  Those are the
// values the reference stores after each `parent *= ext; Normalize()` (src/JunctionTree.cpp:829-941,
// 1150-1238): the recomputation repeats the same IEEE operations on the same operands, so every
// value is bit-identical, while HBM only sees separator messages (written once per case and
// phase) instead of whole tables read and written once per operation.
//
// Passes per clique (entry order inside every bin = the reference's summation order):
//   Collect:     SUM(L) for L = 0..k -> D_L  (post-evidence Normalize, then one per child round)
//                SEPCOL: message to the parent, bins = upstream separator entries, e = q*Ts + j
//                (SeparatorLevelCollectionOptimized, :1056-1148; the old separator is all ones)
//   Distribute:  SUM(k+1) -> D_{k+1} after the parent's message (CliqueLevelDistributionOptimized)
//                SEPDIS per child: bins = that separator's entries, divided by its Collect message
//                with the reference's zero guard (SeparatorLevelDistribution, :700-816)
//                MARG per variable and case whose chosen clique this is (GetProbabilitiesOneNode,
//                :1392-1454; ArgMax, src/Inference.cpp:92-102)
// Division by D_j uses Markstein's correctly rounded sequence (see jt_kernels.hip); a block any of
// whose denominators leaves [2^-600, 2^600] is flagged and recomputed by the exact interpreter.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "jt_program.h"

namespace {

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) char gchar;
typedef __attribute__((address_space(1))) int gint;

struct Den {
    double den, y;
};
constexpr int kVFast = 1 << 12;  // launch flag (dbg word): one-pass Collect denominators (vsum_all)
// fast order: a label whose top two normalized values are within 1e-12 (relative) of each other
// may differ from the reference's ArgMax (strict '>' from 0, src/Inference.cpp:92-102), so its
// block is flagged and recomputed by the exact pass
__device__ __forceinline__ bool near_tie(double mx, double m2) { return mx - m2 <= 1e-12 * mx; }
__device__ __forceinline__ double mdiv(double x, const Den &d) {
    const double q = x * d.y;
    const double r = __builtin_fma(-d.den, q, x);
    return __builtin_fma(r, d.y, q);
}
__device__ __forceinline__ bool den_ok(double d) { return d >= 0x1p-600 && d <= 0x1p+600; }

// The wave's store is addressed through a buffer resource: row offsets are the loads' scalar
// soffset (no per-load 64-bit address arithmetic), the lane's byte offset the VGPR offset.
struct Store {
    __amdgpu_buffer_rsrc_t r;
    unsigned lo;
    __device__ __forceinline__ double ld(int byte_off) const {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo, byte_off, 0));
    }
    __device__ __forceinline__ double row(int row) const { return ld(row * 512); }
    __device__ __forceinline__ void st(int byte_off, double v) const {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                              lo, byte_off, 0);
    }
    __device__ __forceinline__ void st_row(int row, double v) const { st(row * 512, v); }
    // scratch-table accesses with an explicit cache policy (aux bits: 1 sc0, 2 nt, 16 sc1)
    template <int AUX>
    __device__ __forceinline__ double ldp(int byte_off) const {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo, byte_off, AUX));
    }
    template <int AUX>
    __device__ __forceinline__ void stp(int byte_off, double v) const {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), r,
                                              lo, byte_off, AUX);
    }
};
// scratch policy SP of the kernel instance: low byte = aux of scratch stores, next byte = aux of
// scratch loads
#define IROW(r) (*(gint *)((gchar *)(Ib + (long long)(r) * 64) + lo4))

// uniform entry-sequence generators: entries bin by bin, each bin in increasing entry order
struct SeqCol {  // bin j = upstream separator entry, e = q * Ts + j
    int e, q, j, Ts, per;
    __device__ __forceinline__ int next() {
        const int r = e;
        if (++q == per) q = 0, ++j, e = j;
        else e += Ts;
        return r;
    }
};
struct SeqList {  // bins of `per` entries listed in aux
    const int32_t *__restrict__ l;
    int n;
    __device__ __forceinline__ int next() { return l[n++]; }
};
struct SeqMarg {  // bin d = value of the variable: e = hi * bw + d * cum + lo
    int e, lo, hi, d, cum, bw, nhi;
    __device__ __forceinline__ int next() {
        const int r = e;
        if (++lo == cum) {
            lo = 0;
            if (++hi == nhi) hi = 0, ++d, e = d * cum;
            else e += bw - cum + 1;
        } else {
            ++e;
        }
        return r;
    }
};

struct Clq {
    const double *__restrict__ iv;
    const uint32_t *__restrict__ dg32;
    const uint64_t *__restrict__ dg64;
    const int32_t *__restrict__ mp;
    int T, nw;
    uint32_t M32, W32;                                  // this lane's evidence pattern (packed digits)
    uint64_t M[JT_MAX_DIG_WORDS], W[JT_MAX_DIG_WORDS];  // (8-bit digits)
};
// The step denominators D_0 .. D_{k+1} of a clique.  Eight named members, not an array, and the
// runtime-index accessors (pick / put, wave-uniform j) are bit-mask selects / blends over VALUES: as
// an array -- or with a switch returning a member, which becomes a select of member addresses -- the
// compiler turned them into a dynamically indexed load and kept the whole set in per-thread scratch
// (144 B per lane, stored every clique, reloaded on every pick).  Accesses whose index is known after
// unrolling (operator[] in the entry loops) fold to one member.
struct Dens {
    Den a0, a1, a2, a3, a4, a5, a6, a7;
    __device__ __forceinline__ Den operator[](int j) const;
};
static_assert(JT_V_MAX_CHILDREN + 2 == 8, "Dens holds 8 denominators");
__device__ __forceinline__ unsigned long long dbits(double x) { return __builtin_bit_cast(unsigned long long, x); }
__device__ __forceinline__ double dfrom(unsigned long long b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ Den pick(const Dens &D, int j) {
    unsigned long long rd = 0ull, ry = 0ull;
#define FBN_PK(i)                                                             \
    {                                                                         \
        const unsigned long long m = 0ull - (unsigned long long)(j == i);    \
        rd |= dbits(D.a##i.den) & m;                                          \
        ry |= dbits(D.a##i.y) & m;                                            \
    }
    FBN_PK(0) FBN_PK(1) FBN_PK(2) FBN_PK(3) FBN_PK(4) FBN_PK(5) FBN_PK(6) FBN_PK(7)
#undef FBN_PK
    return Den{dfrom(rd), dfrom(ry)};
}
__device__ __forceinline__ Den Dens::operator[](int j) const { return pick(*this, j); }
__device__ __forceinline__ void put(Dens &D, int j, const Den &v) {
#define FBN_PT(i)                                                                         \
    {                                                                                     \
        const unsigned long long m = 0ull - (unsigned long long)(j == i);                \
        D.a##i.den = dfrom((dbits(D.a##i.den) & ~m) | (dbits(v.den) & m));                \
        D.a##i.y = dfrom((dbits(D.a##i.y) & ~m) | (dbits(v.y) & m));                      \
    }
    FBN_PT(0) FBN_PT(1) FBN_PT(2) FBN_PT(3) FBN_PT(4) FBN_PT(5) FBN_PT(6) FBN_PT(7)
#undef FBN_PT
}

// entry e of the clique after L message multiplies (divided by D_L when FINAL), 0 if the entry
// contradicts this lane's evidence
template <int L, bool FINAL, bool P32>
__device__ __forceinline__ double entry(const Store &S, const Clq &C, const Dens &D, int e) {
    double w = C.iv[e];
    bool ok;
    if (P32) {
        ok = (C.dg32[e] & C.M32) == C.W32;
    } else {
        const uint64_t *d = C.dg64 + (size_t)e * C.nw;
        ok = (d[0] & C.M[0]) == C.W[0];
#pragma unroll
        for (int i = 1; i < JT_MAX_DIG_WORDS; ++i)
            if (i < C.nw) ok = ok && ((d[i] & C.M[i]) == C.W[i]);
    }
#pragma unroll
    for (int j = 0; j < L; ++j) w = mdiv(w, D[j]) * S.ld(C.mp[(size_t)j * C.T + e]);
    if (FINAL) w = mdiv(w, D[L]);
    return ok ? w : 0.0;
}

template <int L>
struct Unroll {
    static constexpr int U = L <= 2 ? 4 : 2;  // entries in flight together (SGPR budget)
};

// one entry's operands, loaded ahead of its arithmetic: the masked initial potential and the L
// messages (masking first is equivalent: 0 / D * m == +0 for the finite values involved)
template <int L>
struct Pre {
    double w0;
    double m[L > 0 ? L : 1];
};
template <int L, bool P32>
__device__ __forceinline__ void pre_load(const Store &S, const Clq &C, int e, Pre<L> &p) {
    const double iv = C.iv[e];
    bool ok;
    if (P32) {
        ok = (C.dg32[e] & C.M32) == C.W32;
    } else {
        const uint64_t *d = C.dg64 + (size_t)e * C.nw;
        ok = (d[0] & C.M[0]) == C.W[0];
#pragma unroll
        for (int i = 1; i < JT_MAX_DIG_WORDS; ++i)
            if (i < C.nw) ok = ok && ((d[i] & C.M[i]) == C.W[i]);
    }
    p.w0 = ok ? iv : 0.0;
#pragma unroll
    for (int j = 0; j < L; ++j) p.m[j] = S.ld(C.mp[(size_t)j * C.T + e]);
}
template <int L>
__device__ __forceinline__ double pre_eval(const Pre<L> &p, const Dens &D) {
    double w = p.w0;
#pragma unroll
    for (int j = 0; j < L; ++j) w = mdiv(w, D[j]) * p.m[j];
    return w;
}

// normalization sum D_L = sum_e c_L(e), entry order (Normalize, src/PotentialTableBase.cpp:433-445);
// STORE: c_L(e) is also written to the scratch rows starting at byte offset scr.  Software
// pipelined: the operands of chunk c+1 are in flight while chunk c is evaluated.
template <int L, bool P32, bool STORE = false, int SP = 0>
__device__ __forceinline__ double vsum(const Store &S, const Clq &C, const Dens &D, int scr = 0) {
    constexpr int U = Unroll<L>::U;
    double acc = 0.0;
    const int T = C.T;
    int n0 = 0;
    for (; n0 + U <= T; n0 += U) {
        Pre<L> X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pre_load<L, P32>(S, C, n0 + u, X[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double v = pre_eval<L>(X[u], D);
            acc += v;
            if (STORE) S.template stp<(SP & 255)>(scr + (n0 + u) * 512, v);
        }
    }
    for (; n0 < T; ++n0) {
        Pre<L> X;
        pre_load<L, P32>(S, C, n0, X);
        const double v = pre_eval<L>(X, D);
        acc += v;
        if (STORE) S.template stp<(SP & 255)>(scr + n0 * 512, v);
    }
    return acc;
}

constexpr int kFuseVars = 4, kFuseBins = 16;
// fast mode: the Distribute normalization pass (vsum) also accumulates the fused marginal bins of
// up to kFuseVars variables from the entries before their division by D_L (vmarg_fused's bins, each
// in increasing entry order): the caller divides the bins by D_L afterwards (one rounding apart
// from the exact order's per-entry division), and the separate marginal sweep is gone.
template <int L, bool P32, bool STORE, int SP>
__device__ __forceinline__ double vsum_m(const Store &S, const Clq &C, const Dens &D, int scr, int nf,
                                         const int (&cum)[kFuseVars], const int (&dim)[kFuseVars],
                                         const int (&base)[kFuseVars], double *__restrict__ macc, int lane) {
    constexpr int U = Unroll<L>::U;
    double acc = 0.0;
    const int T = C.T;
    int lo[kFuseVars], dd[kFuseVars];
#pragma unroll
    for (int i = 0; i < kFuseVars; ++i) lo[i] = 0, dd[i] = 0;
    for (int n0 = 0; n0 < T; n0 += U) {
        Pre<L> X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pre_load<L, P32>(S, C, n0 + u < T ? n0 + u : n0, X[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (n0 + u >= T) continue;
            const double v = pre_eval<L>(X[u], D);
            acc += v;
            if (STORE) S.template stp<(SP & 255)>(scr + (n0 + u) * 512, v);
#pragma unroll
            for (int i = 0; i < kFuseVars; ++i) {
                if (i >= nf) continue;
                macc[(base[i] + dd[i]) * 64 + lane] += v;
                if (++lo[i] == cum[i]) {
                    lo[i] = 0;
                    if (++dd[i] == dim[i]) dd[i] = 0;
                }
            }
        }
    }
    return acc;
}

// fast mode (kVFast): every Collect normalization sum of a clique in ONE pass.  c_L(e) = init(e)
// M_1(e) ... M_L(e) / (D_0 ... D_{L-1}), so D_L = P_L / (D_0 ... D_{L-1}) with P_L = sum_e init(e)
// M_1(e) ... M_L(e): one sweep accumulates P_0 .. P_K from prefix products (K message loads per
// entry instead of 1 + 2 + ... + K over K + 1 sweeps).  Same values up to rounding (a few ulp per
// operation: well inside north_star's 1e-6 on potentials); not bit-identical to the reference's
// sequential Normalize, hence opt-in per plan (fbn_jt_set_exact).
// STORE: the full product init(e) M_1(e) ... M_K(e) also goes to the scratch rows at byte offset scr
// (SEPCOL then divides by D_0 ... D_K).
template <int K, bool P32, bool STORE = false, int SP = 0>
__device__ __forceinline__ void vsum_all(const Store &S, const Clq &C, double (&P)[JT_V_MAX_CHILDREN + 2],
                                         int scr = 0) {
    constexpr int U = Unroll<K>::U;
#pragma unroll
    for (int j = 0; j < JT_V_MAX_CHILDREN + 2; ++j) P[j] = 0.0;
    const int T = C.T;
    for (int n0 = 0; n0 < T; n0 += U) {
        Pre<K> X[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pre_load<K, P32>(S, C, n0 + u < T ? n0 + u : n0, X[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (n0 + u >= T) continue;
            double w = X[u].w0;
            P[0] += w;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                w *= X[u].m[j];
                P[j + 1] += w;
            }
            if (STORE) S.template stp<(SP & 255)>(scr + (n0 + u) * 512, w);
        }
    }
}

// binned pass over the stored table (scratch rows at byte offset scr), divided by Df
template <int SP, class Seq, class Flush>
__device__ __forceinline__ void vbins_scr(const Store &S, int scr, const Den &Df, int total, Seq seq, int per,
                                          Flush flush) {
    constexpr int U = 16;
    double acc = 0.0;
    int q = 0, bin = 0;
    for (int n0 = 0; n0 < total; n0 += U) {
        const int cnt = total - n0 < U ? total - n0 : U;
        double val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) val[u] = mdiv(S.template ldp<(SP >> 8)>(scr + ((u < cnt) ? seq.next() : 0) * 512), Df);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < cnt) {
                acc += val[u];
                if (++q == per) {
                    flush(bin, acc);
                    ++bin;
                    q = 0;
                    acc = 0.0;
                }
            }
        }
    }
}

// binned pass over the final table (after L multiplies, divided by D_L): bins of `per`
// consecutive sequence entries; flush(bin, sum) consumes each finished bin
template <int L, bool P32, class Seq, class Flush>
__device__ __forceinline__ void vbins(const Store &S, const Clq &C, const Dens &D, Seq seq, int per, Flush flush) {
    constexpr int U = Unroll<L>::U;
    const int total = C.T;
    double acc = 0.0;
    int q = 0, bin = 0;
    for (int n0 = 0; n0 < total; n0 += U) {
        const int cnt = total - n0 < U ? total - n0 : U;
        int e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = (u < cnt) ? seq.next() : 0;
        double val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) val[u] = entry<L, true, P32>(S, C, D, e[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < cnt) {
                acc += val[u];
                if (++q == per) {
                    flush(bin, acc);
                    ++bin;
                    q = 0;
                    acc = 0.0;
                }
            }
        }
    }
}

// The marginals of up to kFuseVars variables of one clique in ONE in-order sweep over the final table
// (stored scratch rows when MAT, else recomputed entries): entry e adds into bin (variable i, value
// (e / cum_i) % dim_i) of an LDS accumulator [bin][64 lanes].  Every bin receives its entries in
// increasing e -- the order of the per-variable SeqMarg pass it replaces -- starting from 0.0, so
// each bin sum is bit-identical; one pass instead of one per variable.
template <int L, bool P32, int SP, bool MAT>
__device__ __forceinline__ void vmarg_fused(const Store &S, const Clq &C, const Dens &D, int scr, const Den &Df,
                                            int T, int nf, const int (&cum)[kFuseVars],
                                            const int (&dim)[kFuseVars], const int (&base)[kFuseVars],
                                            double *__restrict__ acc, int lane) {
    constexpr int U = MAT ? 16 : Unroll<L>::U;
    int lo[kFuseVars], dd[kFuseVars];
#pragma unroll
    for (int i = 0; i < kFuseVars; ++i) lo[i] = 0, dd[i] = 0;
    for (int n0 = 0; n0 < T; n0 += U) {
        const int cnt = T - n0 < U ? T - n0 : U;
        double val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = u < cnt ? n0 + u : 0;
            if (MAT) val[u] = mdiv(S.template ldp<(SP >> 8)>(scr + e * 512), Df);
            else val[u] = entry<L, true, P32>(S, C, D, e);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u >= cnt) continue;
#pragma unroll
            for (int i = 0; i < kFuseVars; ++i) {
                if (i >= nf) continue;
                double *a = acc + (base[i] + dd[i]) * 64 + lane;
                *a += val[u];
                if (++lo[i] == cum[i]) {
                    lo[i] = 0;
                    if (++dd[i] == dim[i]) dd[i] = 0;
                }
            }
        }
    }
}

// dispatch on the (wave-uniform) chain length and digit packing
#define FBN_VDISPATCH(Lv, P32v, CALL)                                  \
    do {                                                               \
        if (P32v) {                                                    \
            switch (Lv) {                                              \
            case 0: CALL(0, true); break;                              \
            case 1: CALL(1, true); break;                              \
            case 2: CALL(2, true); break;                              \
            case 3: CALL(3, true); break;                              \
            case 4: CALL(4, true); break;                              \
            case 5: CALL(5, true); break;                              \
            case 6: CALL(6, true); break;                              \
            default: CALL(7, true); break;                             \
            }                                                          \
        } else {                                                       \
            switch (Lv) {                                              \
            case 0: CALL(0, false); break;                             \
            case 1: CALL(1, false); break;                             \
            case 2: CALL(2, false); break;                             \
            case 3: CALL(3, false); break;                             \
            case 4: CALL(4, false); break;                             \
            case 5: CALL(5, false); break;                             \
            case 6: CALL(6, false); break;                             \
            default: CALL(7, false); break;                            \
            }                                                          \
        }                                                              \
    } while (0)

// A workgroup = JT_V_WAVES waves sharing one 64-case block: each runs the Collect (then the
// Distribute) of its own disjoint subtrees in parallel, one wave runs the "top" cliques above them
// (jt_virt_plan.cpp: order / sched segments), barriers between the stages.  More waves per block
// = more memory-level parallelism for a kernel that is latency-bound at ~2 blocks per SIMD.
template <int SP>
__global__ __launch_bounds__(64 * JT_V_WAVES) __attribute__((amdgpu_waves_per_eu(4)))
void jt_virt_kernel(
    const JtVClique *__restrict__ cls, const int32_t *__restrict__ aux, const double *__restrict__ initv,
    const uint64_t *__restrict__ dig, const int32_t *__restrict__ order, const int32_t *__restrict__ sched,
    const int32_t *__restrict__ vsel, const int8_t *__restrict__ evid, double *__restrict__ marg,
    int32_t *__restrict__ labels, double *__restrict__ ws, int32_t *__restrict__ wsi, int *__restrict__ flags,
    long long ncases, long long store_rows, long long scratch_row, long long scratch_rows, int nc, int V, int SD,
    int dbg) {
    __shared__ int sbad[JT_V_WAVES];
    const bool fast = (dbg & kVFast) != 0;
    __shared__ double macc[JT_V_WAVES][kFuseBins * 64];  // fused marginal bins, per wave
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    Store S;  // the block's store (messages, denominators, one scratch table per wave)
    S.r = __builtin_amdgcn_make_buffer_rsrc((double *)ws + (size_t)blockIdx.x * (size_t)store_rows * 64, 0,
                                            (int)(store_rows * 512), 0x00020000);
    S.lo = (unsigned)lane * 8u;
    gint *Ib = (gint *)wsi + (size_t)blockIdx.x * (size_t)(nc + V) * 64;  // rows: red[c], then sel[v]
    const unsigned lo4 = (unsigned)lane * 4u;
    const int scr = (int)((scratch_row + (long long)wv * scratch_rows) * 512);

    for (long long blk = blockIdx.x; blk * 64 < ncases; blk += gridDim.x) {
        const long long cs = blk * 64 + lane;
        const bool act = cs < ncases;
        const long long csr = act ? cs : ncases - 1;
        const int8_t *__restrict__ ev = evid + csr * V;
        double *__restrict__ out = marg + csr * SD;
        bool bad = false;

        auto setup = [&](const JtVClique &q, Clq &C, int &nobs) {
            C.iv = initv + q.iv_off;
            C.dg32 = reinterpret_cast<const uint32_t *>(dig + q.dig_off);
            C.dg64 = dig + q.dig_off;
            C.mp = aux + q.map_off;
            C.T = q.T;
            C.nw = q.nw;
            C.M32 = 0u, C.W32 = 0u;
#pragma unroll
            for (int i = 0; i < JT_MAX_DIG_WORDS; ++i) C.M[i] = 0ull, C.W[i] = 0ull;
            nobs = 0;
            const int32_t *__restrict__ vr = aux + q.vars_off;
            for (int j = 0; j < q.nv; ++j) {
                const int x = ev[vr[3 * j]];
                const int sh = vr[3 * j + 1];
                const uint32_t fm = (uint32_t)vr[3 * j + 2];
                nobs += x >= 0;
                if (q.nw == 0) {
                    C.M32 |= x >= 0 ? fm << sh : 0u;
                    C.W32 |= x >= 0 ? (uint32_t)x << sh : 0u;
                } else {
                    const uint64_t m = x >= 0 ? ((uint64_t)fm << sh) : 0ull;
                    const uint64_t w = x >= 0 ? ((uint64_t)x << sh) : 0ull;
                    const int wi = j >> 3;
                    if (wi == 0) C.M[0] |= m, C.W[0] |= w;
                    else if (wi == 1) C.M[1] |= m, C.W[1] |= w;
                    else if (wi == 2) C.M[2] |= m, C.W[2] |= w;
                    else C.M[3] |= m, C.W[3] |= w;
                }
            }
        };

        // ---------------- Collect of one clique (children first)
        auto collect = [&](int cid) {
            const JtVClique q = cls[cid];
            Clq C;
            int nobs;
            setup(q, C, nobs);
            IROW(q.id) = q.nv - nobs;  // variables left after the reference's table reduction
            const bool p32 = q.nw == 0;
            Dens D;
#pragma unroll
            for (int j = 0; j < JT_V_MAX_CHILDREN + 2; ++j) put(D, j, Den{1.0, 1.0});
            // the last normalization pass of a clique with children also stores the table for SEPCOL
            // (exact mode; fast mode recomputes the SEPCOL entries with its one-pass denominators)
            const bool cmat = q.cmat && !(dbg & 32);
            double prod = 1.0;  // fast mode: D_0 ... D_k (the stored products' divisor)
            if (fast) {
                double P[JT_V_MAX_CHILDREN + 2];
                if (cmat) {
#define FBN_ALLCALL(Lc, Pc) vsum_all<Lc, Pc, true, SP>(S, C, P, scr)
                    FBN_VDISPATCH(q.k, p32, FBN_ALLCALL);
#undef FBN_ALLCALL
                } else {
#define FBN_ALLCALL(Lc, Pc) vsum_all<Lc, Pc>(S, C, P)
                    FBN_VDISPATCH(q.k, p32, FBN_ALLCALL);
#undef FBN_ALLCALL
                }
#pragma unroll
                for (int L = 0; L < JT_V_MAX_CHILDREN + 2; ++L) {
                    if (L > q.k) continue;
                    const double s = P[L] / prod;
                    // a product chain that leaves the normal range: the block goes to the exact pass
                    bad |= !den_ok(s) || !(P[L] >= 0x1p-960 && P[L] <= 0x1p+960);
                    S.st_row(q.den_row + L, s);
                    put(D, L, Den{s, 1.0 / s});
                    prod *= s;
                }
            }
            for (int L = 0; L <= (fast ? -1 : q.k); ++L) {
                double s = 0.0;
                if (cmat && L == q.k) {
#define FBN_SUMCALL(Lc, P) s = vsum<Lc, P, true, SP>(S, C, D, scr)
                    FBN_VDISPATCH(L, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                } else {
#define FBN_SUMCALL(Lc, P) s = vsum<Lc, P>(S, C, D)
                    FBN_VDISPATCH(L, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                }
                bad |= !den_ok(s);
                S.st_row(q.den_row + L, s);
                // D is indexed by the uniform L: write every slot under a uniform compare so the
                // array stays in registers
                put(D, L, Den{s, 1.0 / s});
            }
            if (!q.root && !(dbg & 1)) {
                const int Ts = q.up_Ts, per = q.T / Ts, dst = q.up_col_row;
                auto fl = [&](int j, double acc) { S.st_row(dst + j, acc); };
                if (cmat) {
                    const Den Dc = fast ? Den{prod, 1.0 / prod} : pick(D, q.k);
                    vbins_scr<SP>(S, scr, Dc, q.T, SeqCol{0, 0, 0, Ts, per}, per, fl);
                } else {
#define FBN_COLCALL(Lc, P) vbins<Lc, P>(S, C, D, SeqCol{0, 0, 0, Ts, per}, per, fl)
                    FBN_VDISPATCH(q.k, p32, FBN_COLCALL);
#undef FBN_COLCALL
                }
            }
        };

        // ---------------- per variable: the clique GetProbabilitiesOneNode would use for this case
        // (first candidate with the fewest remaining variables, src/JunctionTree.cpp:1412-1434)
        auto select = [&](int v) {
            const int32_t *__restrict__ cd = aux + vsel[4 * v];
            const int ncand = vsel[4 * v + 1];
            int sel = 0, best = 0x7fffffff;
            for (int k = 0; k < ncand; ++k) {
                const int r = IROW(cd[k]);
                if (r < best) best = r, sel = cd[k];
            }
            IROW(nc + v) = sel | (best << 24);
        };

        // ---------------- Distribute of one clique (parent first) and its outputs
        auto distribute = [&](int cid) {
            const JtVClique q = cls[cid];
            Clq C;
            int nobs;
            setup(q, C, nobs);
            const bool p32 = q.nw == 0;
            Dens D;
#pragma unroll
            for (int j = 0; j < JT_V_MAX_CHILDREN + 2; ++j) {
                Den v = Den{1.0, 1.0};
                if (j <= q.k) {
                    const double s = S.row(q.den_row + j);
                    v = Den{s, 1.0 / s};
                }
                put(D, j, v);
            }
            // marginals of the variables whose chosen clique (for this case) is this one: up to
            // kFuseVars of them (kFuseBins values in total) in one fused sweep, the rest one pass each
            const bool fuse = !(dbg & 1024);
            int fv[kFuseVars], fcum[kFuseVars], fdim[kFuseVars], fbase[kFuseVars];
#pragma unroll
            for (int i = 0; i < kFuseVars; ++i) fv[i] = 0, fcum[i] = 1, fdim[i] = 1, fbase[i] = 0;
            int nf = 0, nb = 0;
            uint32_t fmask = 0;  // marginal records fused
            auto pick_fused = [&]() {
                for (int mi = 0; mi < ((dbg & 4) ? 0 : q.nmarg); ++mi) {
                    const int32_t *__restrict__ rec = aux + q.marg_off + 4 * mi;
                    const int dim = rec[1], var = rec[2], cum = rec[3];
                    const int sb = IROW(nc + var);
                    const bool mine = ((sb & 0xFFFFFF) == q.id) && ev[var] < 0;
                    if (__ballot(mine) == 0ull) continue;
                    if (fuse && nf < kFuseVars && nb + dim <= kFuseBins && mi < 32) {
#pragma unroll
                        for (int i = 0; i < kFuseVars; ++i)
                            if (i == nf) fv[i] = mi, fcum[i] = cum, fdim[i] = dim, fbase[i] = nb;
                        ++nf, nb += dim;
                        fmask |= 1u << mi;
                    }
                }
            };
            // fast mode: the marginal bins ride on the Distribute normalization pass (vsum_m)
            const bool mfused = fast && !q.root && !(dbg & 8);
            double *macc_w = macc[wv];
            if (mfused) {
                pick_fused();
                for (int b = 0; b < nb; ++b) macc_w[b * 64 + lane] = 0.0;
            }
            int Lf = q.k;
            if (!q.root && !(dbg & 8)) {
                double s = 0.0;
                if (mfused && nf > 0) {
                    const bool st = q.mat && !(dbg & 64) && !((dbg & 512) && q.k < 2);
                    if (st) {
#define FBN_SUMCALL(Lc, P) s = vsum_m<Lc, P, true, SP>(S, C, D, scr, nf, fcum, fdim, fbase, macc_w, lane)
                        FBN_VDISPATCH(q.k + 1, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                    } else {
#define FBN_SUMCALL(Lc, P) s = vsum_m<Lc, P, false, SP>(S, C, D, scr, nf, fcum, fdim, fbase, macc_w, lane)
                        FBN_VDISPATCH(q.k + 1, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                    }
                } else if (q.mat && !(dbg & 64) && !((dbg & 512) && q.k < 2)) {
#define FBN_SUMCALL(Lc, P) s = vsum<Lc, P, true, SP>(S, C, D, scr)
                    FBN_VDISPATCH(q.k + 1, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                } else {
#define FBN_SUMCALL(Lc, P) s = vsum<Lc, P>(S, C, D)
                    FBN_VDISPATCH(q.k + 1, p32, FBN_SUMCALL);
#undef FBN_SUMCALL
                }
                bad |= !den_ok(s);
                Lf = q.k + 1;
                put(D, Lf, Den{s, 1.0 / s});
            }
            // messages to the children
            for (int ci = 0; ci < ((dbg & 2) ? 0 : q.k); ++ci) {
                const int32_t *__restrict__ rec = aux + q.child_off + 5 * ci;
                const int Ts = rec[0], per = rec[1], col = rec[3], dis = rec[4];
                const int32_t *__restrict__ lst = aux + rec[2];
                // sep = tmp / old at each bin's flush (diagnostic dbg & 256: bin sums first, then
                // a separate division sweep)
                const bool direct = !(dbg & 256);
                auto fl = [&](int j, double acc) {
                    if (direct) {
                        const double old = S.row(col + j);
                        S.st_row(dis + j, (old == 0.0) ? 0.0 : acc / old);
                    } else {
                        S.st_row(dis + j, acc);
                    }
                };
                if (q.mat && !(dbg & 64) && !((dbg & 512) && q.k < 2)) {
                    vbins_scr<SP>(S, scr, pick(D, Lf), q.T, SeqList{lst, 0}, per, fl);
                } else {
#define FBN_DISCALL(Lc, P) vbins<Lc, P>(S, C, D, SeqList{lst, 0}, per, fl)
                    FBN_VDISPATCH(Lf, p32, FBN_DISCALL);
#undef FBN_DISCALL
                }
                // sep = tmp / old, zero-guarded (src/JunctionTree.cpp:700-816)
                for (int j0 = 0; j0 < (direct ? 0 : Ts); j0 += 8) {
                    double a[8], o[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int j = j0 + u < Ts ? j0 + u : Ts - 1;
                        a[u] = S.row(dis + j);
                        o[u] = S.row(col + j);
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (j0 + u < Ts) S.st_row(dis + j0 + u, (o[u] == 0.0) ? 0.0 : a[u] / o[u]);
                }
            }
            const bool mat = q.mat && !(dbg & 64) && !((dbg & 512) && q.k < 2);
            auto finish = [&](int mi, auto bin_of) {  // outputs of marginal record mi from its bins
                const int32_t *__restrict__ rec = aux + q.marg_off + 4 * mi;
                const int off = rec[0], dim = rec[1], var = rec[2];
                const int sb = IROW(nc + var);
                const bool mine = ((sb & 0xFFFFFF) == q.id) && ev[var] < 0;
                const int best = sb >> 24;
                double *__restrict__ o = out + off;
                const bool wr = mine && act;
                double tot = 0.0;
                for (int d = 0; d < dim; ++d) {  // bins in value order; tot = their sum in order
                    const double acc = bin_of(d);
                    if (wr) o[d] = acc;
                    tot += acc;
                }
                if (wr) {
                    if (var == 0) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                        int lab = 0;
                        double mx = 0.0, m2 = 0.0;
                        for (int d = 0; d < dim; ++d) {
                            const double p = (best == 1) ? o[d] : o[d] / tot;
                            if (p > mx) m2 = mx, mx = p, lab = d;
                            else if (p > m2) m2 = p;
                        }
                        labels[cs] = lab;
                        bad |= fast && near_tie(mx, m2);
                    }
                    for (int d = 0; d < dim; ++d) o[d] = o[d] / tot;
                }
            };
            for (int mi = 0; mi < ((dbg & 4) ? 0 : q.nmarg); ++mi) {
                const int32_t *__restrict__ rec = aux + q.marg_off + 4 * mi;
                const int dim = rec[1], var = rec[2], cum = rec[3];
                const int sb = IROW(nc + var);
                const bool mine = ((sb & 0xFFFFFF) == q.id) && ev[var] < 0;
                if (__ballot(mine) == 0ull) continue;
                if (mfused ? ((fmask >> mi) & 1u) != 0 : (fuse && nf < kFuseVars && nb + dim <= kFuseBins)) {
                    if (mfused) continue;  // accumulated by the normalization pass
                    // into the fused sweep
#pragma unroll
                    for (int i = 0; i < kFuseVars; ++i)
                        if (i == nf) fv[i] = mi, fcum[i] = cum, fdim[i] = dim, fbase[i] = nb;
                    ++nf, nb += dim;
                    continue;
                }
                const int bw = dim * cum;
                double *__restrict__ o = out + (aux + q.marg_off + 4 * mi)[0];
                const bool wr = mine && act;
                const int best = sb >> 24;
                double tot = 0.0;
                auto fl = [&](int d, double acc) {
                    if (wr) o[d] = acc;
                    tot += acc;
                };
                if (mat) {
                    vbins_scr<SP>(S, scr, pick(D, Lf), q.T, SeqMarg{0, 0, 0, 0, cum, bw, q.T / bw}, q.T / dim, fl);
                } else {
#define FBN_MARGCALL(Lc, P) vbins<Lc, P>(S, C, D, SeqMarg{0, 0, 0, 0, cum, bw, q.T / bw}, q.T / dim, fl)
                    FBN_VDISPATCH(Lf, p32, FBN_MARGCALL);
#undef FBN_MARGCALL
                }
                if (wr) {
                    if (var == 0) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                        int lab = 0;
                        double mx = 0.0, m2 = 0.0;
                        for (int d = 0; d < dim; ++d) {
                            const double p = (best == 1) ? o[d] : o[d] / tot;
                            if (p > mx) m2 = mx, mx = p, lab = d;
                            else if (p > m2) m2 = p;
                        }
                        labels[cs] = lab;
                        bad |= fast && near_tie(mx, m2);
                    }
                    for (int d = 0; d < dim; ++d) o[d] = o[d] / tot;
                }
            }
            if (nf > 0 && mfused) {  // bins from the normalization pass, divided by its sum D_Lf
                const Den Df = pick(D, Lf);
#pragma unroll
                for (int i = 0; i < kFuseVars; ++i)
                    if (i < nf) finish(fv[i], [&](int d) { return mdiv(macc_w[(fbase[i] + d) * 64 + lane], Df); });
            } else if (nf > 0) {
                double *acc = macc[wv];
                for (int b = 0; b < nb; ++b) acc[b * 64 + lane] = 0.0;
                const Den Df = pick(D, Lf);
                if (mat) {
                    vmarg_fused<0, true, SP, true>(S, C, D, scr, Df, q.T, nf, fcum, fdim, fbase, acc, lane);
                } else {
#define FBN_FUSECALL(Lc, P) vmarg_fused<Lc, P, SP, false>(S, C, D, scr, Df, q.T, nf, fcum, fdim, fbase, acc, lane)
                    FBN_VDISPATCH(Lf, p32, FBN_FUSECALL);
#undef FBN_FUSECALL
                }
#pragma unroll
                for (int i = 0; i < kFuseVars; ++i)
                    if (i < nf) finish(fv[i], [&](int d) { return acc[(fbase[i] + d) * 64 + lane]; });
            }
        };

        // ---------------- the schedule: subtrees in parallel, the top by wave 0
        // (one call site per lambda, so each is inlined)
        for (int stage = 0; stage < 2; ++stage) {
            const int b = stage == 0 ? sched[wv] : (wv == 0 ? sched[JT_V_WAVES] : 0);
            const int e = stage == 0 ? sched[wv + 1] : (wv == 0 ? sched[JT_V_WAVES + 1] : 0);
            for (int i = b; i < e; ++i) collect(order[i]);
            __syncthreads();
        }
        for (int v = wv; v < V; v += JT_V_WAVES) select(v);
        __syncthreads();
        for (int stage = 0; stage < ((dbg & 16) ? 0 : 2); ++stage) {
            const int b = stage == 0 ? (wv == 0 ? sched[JT_V_WAVES + 1] : 0) : sched[JT_V_WAVES + 2 + wv];
            const int e = stage == 0 ? (wv == 0 ? sched[JT_V_WAVES + 2] : 0) : sched[JT_V_WAVES + 3 + wv];
            for (int i = b; i < e; ++i) distribute(order[i]);
            if (stage == 0) __syncthreads();
        }
        // evidence variables: probabilities stay 0 (their first slot is compared with -1 by the scorer)
        if (act)
            for (int v = wv; v < V; v += JT_V_WAVES)
                if (ev[v] >= 0) {
                    const int off = vsel[4 * v + 2], dim = vsel[4 * v + 3];
                    for (int d = 0; d < dim; ++d) out[off + d] = 0.0;
                }
        const unsigned long long b = __ballot(bad);
        if (lane == 0) sbad[wv] = b != 0ull;
        __syncthreads();  // also: no wave starts the next block while another still reads this one
        if (wv == 0 && lane == 0) {
            int f = 0;
            for (int w = 0; w < JT_V_WAVES; ++w) f |= sbad[w];
            flags[blk] = f;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" hipError_t fbn_jt_virt_launch(const JtVClique *cls, const int32_t *aux, const double *initv,
                                         const uint64_t *dig, const int32_t *order, const int32_t *sched,
                                         const int32_t *vsel, const int8_t *evid, double *marg, int32_t *labels,
                                         double *ws, int32_t *wsi, int *flags, long long ncases, long long store_rows,
                                         long long scratch_row, long long scratch_rows, int nc, int V, int SD,
                                         int grid, int dbg, hipStream_t stream) {
    // scratch-table cache policy (diagnostic override FBN_JT_VPOL; results do not depend on it)
    static const int pol = getenv("FBN_JT_VPOL") ? atoi(getenv("FBN_JT_VPOL")) : 1;
#define FBN_VLAUNCH(SPv)                                                                                          \
    hipLaunchKernelGGL(jt_virt_kernel<SPv>, dim3(grid), dim3(64 * JT_V_WAVES), 0, stream, cls, aux, initv, dig, \
                       order, sched, vsel, evid, marg, labels, ws, wsi, flags, ncases, store_rows, scratch_row,  \
                       scratch_rows, nc, V, SD, dbg)
    switch (pol) {
    case 1: FBN_VLAUNCH(2 | (2 << 8)); break;     // nt stores, nt loads
    case 2: FBN_VLAUNCH(16 | (2 << 8)); break;    // sc1 stores (line dropped from L2), nt loads
    case 3: FBN_VLAUNCH(18 | (18 << 8)); break;   // sc1|nt both ways
    default: FBN_VLAUNCH(0); break;
    }
#undef FBN_VLAUNCH
    return hipGetLastError();
}
