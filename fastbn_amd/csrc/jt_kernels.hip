// jt_kernels.hip -- batched junction-tree sum-product on gfx950.
//
// One lane = one evidence case.  A 64-lane wave walks the case-independent device program
// (jt_program.h) in lock-step, so every branch and loop bound is wave-uniform and every op
// descriptor / index map / initial potential is a scalar (SMEM) load shared by the 64 cases.
// The per-case state lives in a persistent workspace laid out [wave][entry][64 lanes] (fp64):
// touching one table entry is one fully coalesced 512-byte wave access.  Waves are persistent
// (grid = CUs x waves-per-CU) and recycle their workspace block for the next 64 cases, so the
// whole in-flight state stays small enough to be served from L2 / Infinity Cache.
//
// Numerics: each lane performs the reference's per-case operations in the reference's order
// (src/JunctionTree.cpp:1473-1502) on masked tables with a lazily applied normalization
// denominator (see jt_program.h) -- results are bit-identical to the reference's fp64 path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jt_program.h"

namespace {

struct JtArgs {
    const JtOp *ops;
    const int32_t *aux;
    const double *initv;
    const uint64_t *dig;
    const int8_t *evid;  // [ncases][V]
    double *marg;        // [ncases][SD]
    int32_t *labels;     // [ncases]
    double *ws;          // [grid][NE][64]
    int32_t *wsi;        // [grid][nc][64]
    long long ncases;
    long long NE;
    int nops, V, SD, nc;
    int vmajor;  // marginals variable-major [SD][ncases] (fbn_jt_set_output_layout)
};

// one case's marginal outputs: a case-major row (vs = 1) or a column stride of the variable-major
// layout (vs = ncases); value d of the output at index k is o[d] of `out + k`
struct MOut {
    double *p;
    long long vs;
    __device__ __forceinline__ double &operator[](long long d) const { return p[d * vs]; }
    __device__ __forceinline__ MOut operator+(long long k) const { return MOut{p + k * vs, vs}; }
};

#define AT(e) S[(size_t)(e) * 64]

// Division by the pending denominator.  Markstein: with y = RN(1/den) and q = RN(x*y) within one
// ulp of x/den, q + RN(x - den*q)*y (two fmas) is the correctly rounded quotient -- the same bits as
// the reference's `potentials[i] /= denominator` -- as long as nothing under/overflows.  The fast form
// is used when den lies in [2^-600, 2^600] for every lane of the wave (then any table value >= 2^-400
// keeps every intermediate normal); otherwise the op runs with the IEEE division sequence.
struct Den {
    double den, y;
};
template <bool EXACT>
__device__ __forceinline__ double dv(double x, const Den &d) {
    if (EXACT) return x / d.den;
    const double q = x * d.y;
    const double r = __builtin_fma(-d.den, q, x);
    return __builtin_fma(r, d.y, q);
}
__device__ __forceinline__ bool den_fast_all(double den) {
    return __ballot(!(den >= 0x1p-600 && den <= 0x1p+600)) == 0ull;
}



#ifndef FBN_G_UNROLL
#define FBN_G_UNROLL 8
#endif
// global-variant op bodies, instantiated for the fast (Markstein) and the exact division
// Separator sweeps keep up to kGJ results in registers and store them together, so the loads of a
// chunk of separator entries are not serialized behind per-entry stores (vmcnt is in issue order).
constexpr int kGJ = 32;
template <bool EXACT>
__device__ __forceinline__ void g_sepcol(double *__restrict__ S, const JtOp &op, const Den &D) {
    const int Ts = op.b, Q = op.d / op.b;
    for (int j0 = 0; j0 < Ts; j0 += kGJ) {
        const int nj = Ts - j0 < kGJ ? Ts - j0 : kGJ;
        double res[kGJ];
#pragma unroll
        for (int jj = 0; jj < kGJ; ++jj) {
            res[jj] = 0.0;
            if (jj >= nj) continue;
            const int j = j0 + jj;
            double acc = 0.0;
#pragma unroll FBN_G_UNROLL
            for (int q = 0; q < Q; ++q) acc += dv<EXACT>(AT(op.c + q * Ts + j), D);
            const double old = AT(op.a + j);
            res[jj] = (old == 0.0) ? 0.0 : acc / old;
        }
#pragma unroll
        for (int jj = 0; jj < kGJ; ++jj)
            if (jj < nj) AT(op.a + j0 + jj) = res[jj];
    }
}
// Read-modify-write sweeps are software-pipelined: the loads of chunk k+1 are issued before the
// stores of chunk k, so a wait for loaded data never includes this sweep's own stores (vmcnt
// counts loads and stores together, in issue order).  Element order and the sum order are the
// reference's.
constexpr int kGChunk = 16;
template <bool EXACT>
__device__ __forceinline__ double g_clqmul(double *__restrict__ S, const JtOp &op, const int32_t *__restrict__ mp,
                                           const Den &D) {
    const int T = op.b, nfull = T / kGChunk;
    double sum = 0.0;
    double ta[kGChunk], ma[kGChunk];
    if (nfull > 0) {
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) ta[k] = AT(op.a + k), ma[k] = AT(op.d + mp[k]);
    }
    for (int c = 0; c < nfull; ++c) {
        const int e0 = c * kGChunk, e1 = e0 + kGChunk;
        double tb[kGChunk], mb[kGChunk];
        if (c + 1 < nfull) {
#pragma unroll
            for (int k = 0; k < kGChunk; ++k) tb[k] = AT(op.a + e1 + k), mb[k] = AT(op.d + mp[e1 + k]);
        }
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) {
            const double v = dv<EXACT>(ta[k], D) * ma[k];
            AT(op.a + e0 + k) = v;
            sum += v;
        }
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) ta[k] = tb[k], ma[k] = mb[k];
    }
    for (int e = nfull * kGChunk; e < T; ++e) {
        const double v = dv<EXACT>(AT(op.a + e), D) * AT(op.d + mp[e]);
        AT(op.a + e) = v;
        sum += v;
    }
    return sum;
}
template <bool EXACT>
__device__ __forceinline__ void g_sepdis(double *__restrict__ S, const JtOp &op, const int32_t *__restrict__ ls,
                                         const Den &D) {
    const int per = op.f, Ts = op.b;
    for (int j0 = 0; j0 < Ts; j0 += kGJ) {
        const int nj = Ts - j0 < kGJ ? Ts - j0 : kGJ;
        double res[kGJ];
#pragma unroll
        for (int jj = 0; jj < kGJ; ++jj) {
            res[jj] = 0.0;
            if (jj >= nj) continue;
            const int j = j0 + jj;
            double acc = 0.0;
#pragma unroll FBN_G_UNROLL
            for (int q = 0; q < per; ++q) acc += dv<EXACT>(AT(op.c + ls[j * per + q]), D);
            const double old = AT(op.a + j);
            res[jj] = (old == 0.0) ? 0.0 : acc / old;
        }
#pragma unroll
        for (int jj = 0; jj < kGJ; ++jj)
            if (jj < nj) AT(op.a + j0 + jj) = res[jj];
    }
}
template <bool EXACT>
__device__ __forceinline__ double g_clqdis(double *__restrict__ S, const JtOp &op, const Den &D) {
    const int T = op.b, Ts = op.e, nfull = T / kGChunk;
    double sum = 0.0;
    double ta[kGChunk], ma[kGChunk];
    if (nfull > 0) {
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) ta[k] = AT(op.a + k), ma[k] = AT(op.d + k % Ts);
    }
    for (int c = 0; c < nfull; ++c) {
        const int e0 = c * kGChunk, e1 = e0 + kGChunk;
        double tb[kGChunk], mb[kGChunk];
        if (c + 1 < nfull) {
#pragma unroll
            for (int k = 0; k < kGChunk; ++k) tb[k] = AT(op.a + e1 + k), mb[k] = AT(op.d + (e1 + k) % Ts);
        }
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) {
            const double v = dv<EXACT>(ta[k], D) * ma[k];
            AT(op.a + e0 + k) = v;
            sum += v;
        }
#pragma unroll
        for (int k = 0; k < kGChunk; ++k) ta[k] = tb[k], ma[k] = mb[k];
    }
    for (int e = nfull * kGChunk; e < T; ++e) {
        const double v = dv<EXACT>(AT(op.a + e), D) * AT(op.d + e % Ts);
        AT(op.a + e) = v;
        sum += v;
    }
    return sum;
}
template <bool EXACT>
__device__ __forceinline__ double g_marg(double *__restrict__ S, int toff, int dim, int cum, int T, const Den &D,
                                         const MOut &o, bool act) {
    const int bw = dim * cum, nhi = T / bw;
    double tot = 0.0;
    for (int d = 0; d < dim; ++d) {
        double acc = 0.0;
        for (int hi = 0; hi < nhi; ++hi)
#pragma unroll FBN_G_UNROLL
            for (int lo = 0; lo < cum; ++lo) acc += dv<EXACT>(AT(toff + hi * bw + d * cum + lo), D);
        if (act) o[d] = acc;
        tot += acc;
    }
    return tot;
}

__global__ __launch_bounds__(64) void jt_interp_kernel(JtArgs A) {
    const int lane = threadIdx.x;
    double *__restrict__ S = A.ws + (size_t)blockIdx.x * (size_t)A.NE * 64 + lane;
    int32_t *__restrict__ red = A.wsi + (size_t)blockIdx.x * (size_t)A.nc * 64 + lane;
    const JtOp *__restrict__ ops = A.ops;
    const int32_t *__restrict__ aux = A.aux;
    const double *__restrict__ initv = A.initv;
    const uint64_t *__restrict__ dig = A.dig;

    for (long long blk = blockIdx.x; blk * 64 < A.ncases; blk += gridDim.x) {
        const long long cs = blk * 64 + lane;
        const bool act = cs < A.ncases;
        const long long csr = act ? cs : A.ncases - 1;
        const int8_t *__restrict__ ev = A.evid + csr * A.V;
        const MOut out{A.marg + csr * (A.vmajor ? 1 : A.SD), A.vmajor ? A.ncases : 1};

        for (int i = 0; i < A.nops; ++i) {
            const JtOp op = ops[i];
            switch (op.type) {
            case JT_OP_INIT: {
                // evidence pattern of this table for this lane: mask/value words over the slots
                const int nv = op.d;
                uint64_t M0 = 0, M1 = 0, M2 = 0, M3 = 0, W0 = 0, W1 = 0, W2 = 0, W3 = 0;
                int nobs = 0;
                for (int j = 0; j < nv; ++j) {
                    const int x = ev[aux[op.c + j]];
                    const uint64_t m = x >= 0 ? (0xFFull << (8 * (j & 7))) : 0ull;
                    const uint64_t w = x >= 0 ? ((uint64_t)x << (8 * (j & 7))) : 0ull;
                    nobs += x >= 0;
                    if (j < 8) M0 |= m, W0 |= w;
                    else if (j < 16) M1 |= m, W1 |= w;
                    else if (j < 24) M2 |= m, W2 |= w;
                    else M3 |= m, W3 |= w;
                }
                const int nw = nv > 8 ? (nv + 7) / 8 : 1;
                const uint64_t *__restrict__ dg = dig + op.e;
                const double *__restrict__ iv = initv + op.h;
                double sum = 0.0;
#pragma unroll 4
                for (int e = 0; e < op.b; ++e) {
                    const uint64_t *d = dg + (size_t)e * nw;
                    bool cons = (d[0] & M0) == W0;
                    if (nw > 1) cons = cons && ((d[1] & M1) == W1);
                    if (nw > 2) cons = cons && ((d[2] & M2) == W2);
                    if (nw > 3) cons = cons && ((d[3] & M3) == W3);
                    const double val = cons ? iv[e] : 0.0;
                    AT(op.a + e) = val;
                    sum += val;
                }
                if (op.f >= 0) {  // clique: post-evidence Normalize (src/JunctionTree.cpp:1479-1483)
                    AT(op.f) = sum;
                    red[(size_t)op.g * 64] = nv - nobs;
                }
                break;
            }
            case JT_OP_SEPCOL: {  // src/JunctionTree.cpp:1056-1148
                const double den = AT(op.e);
                const Den D{den, 1.0 / den};
                if (den_fast_all(den)) g_sepcol<false>(S, op, D);
                else g_sepcol<true>(S, op, D);
                break;
            }
            case JT_OP_CLQMUL: {  // src/JunctionTree.cpp:829-941 (extension + multiply + Normalize)
                const double den = AT(op.c);
                const Den D{den, 1.0 / den};
                const int32_t *__restrict__ mp = aux + op.e;
                AT(op.c) = den_fast_all(den) ? g_clqmul<false>(S, op, mp, D) : g_clqmul<true>(S, op, mp, D);
                break;
            }
            case JT_OP_SEPDIS: {  // src/JunctionTree.cpp:700-816
                const double den = AT(op.d);
                const Den D{den, 1.0 / den};
                const int32_t *__restrict__ ls = aux + op.e;
                if (den_fast_all(den)) g_sepdis<false>(S, op, ls, D);
                else g_sepdis<true>(S, op, ls, D);
                break;
            }
            case JT_OP_CLQDIS: {  // src/JunctionTree.cpp:1150-1238
                const double den = AT(op.c);
                const Den D{den, 1.0 / den};
                AT(op.c) = den_fast_all(den) ? g_clqdis<false>(S, op, D) : g_clqdis<true>(S, op, D);
                break;
            }
            case JT_OP_MARG: {  // src/JunctionTree.cpp:1339-1454, src/Inference.cpp:92-102
                const int dim = op.b;
                const MOut o = out + op.a;
                if (ev[op.e] >= 0) {  // evidence node: probabilities stay 0
                    if (act)
                        for (int d = 0; d < dim; ++d) o[d] = 0.0;
                    break;
                }
                const int32_t *__restrict__ cd = aux + op.c;
                int sel = 0, best = 0x7fffffff;
                for (int k = 0; k < op.d; ++k) {  // first clique with the fewest reduced variables
                    const int r = red[(size_t)cd[6 * k] * 64];
                    if (r < best) best = r, sel = k;
                }
                for (int k = 0; k < op.d; ++k) {
                    if (k != sel) continue;
                    const int toff = cd[6 * k + 1], cum = cd[6 * k + 4], T = cd[6 * k + 5];
                    const double den = AT(cd[6 * k + 2]);
                    const Den D{den, 1.0 / den};
                    const double tot = den_fast_all(den) ? g_marg<false>(S, toff, dim, cum, T, D, o, act)
                                                         : g_marg<true>(S, toff, dim, cum, T, D, o, act);
                    if (act) {
                        if (op.f) {  // label: ArgMax, strict '>' from 0
                            int lab = 0;
                            double mp = 0.0;
                            for (int d = 0; d < dim; ++d) {
                                const double v = (best == 1) ? o[d] : o[d] / tot;
                                if (v > mp) mp = v, lab = d;
                            }
                            A.labels[cs] = lab;
                        }
                        for (int d = 0; d < dim; ++d) o[d] = o[d] / tot;
                    }
                }
                break;
            }
            default:
                break;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// LDS-resident variant: the clique in flight is held in LDS ([entry][64 lanes], rows >= cap spill
// to a per-wave global buffer), its pending denominator in a register.  HBM sees each clique table
// once when parked after Collect and once when reloaded in Distribute, plus the separator messages.
struct JtLParams {
    long long ncases;
    long long wave_entries;  // store + nc + sep + spill
    long long store_off, den_off, sep_off, spill_off;
    int nops, V, SD, nc, cap;
    int force_exact;  // ablation/testing: always take the IEEE division path
    int vmajor;        // marginals variable-major [SD][ncases]
    const int *flags;  // fixup mode (non-null): only the blocks the specialized kernel flagged
};

// Pointers are separate __restrict__ kernel arguments (not a struct): the compiler can then prove
// that the program arrays are never written and turns their wave-uniform reads into SMEM loads.
// the clique in flight: LDS rows [0, cap), spilled rows in per-wave global memory
template <bool SPILL>
struct Tab {
    double *__restrict__ lds;
    double *__restrict__ spill;
    int cap;
    __device__ __forceinline__ double &operator[](int e) const {
        return (!SPILL || e < cap) ? lds[(size_t)e * 64] : spill[(size_t)(e - cap) * 64];
    }
};

// parent *= extended child message, then the normalization sum in entry order (:829-941).
// By separator entry: one message load per separator entry, parent entries from the inverse map.
template <bool SPILL, bool EXACT>
__device__ void op_mul(const Tab<SPILL> &T, Den &D, const double *__restrict__ sp, const int32_t *__restrict__ ls,
                       int Ts, int Tn) {
    const int per = Tn / Ts;
    for (int j = 0; j < Ts; ++j) {
        const double m = sp[(size_t)j * 64];
        const int32_t *__restrict__ l = ls + j * per;
#pragma unroll 8
        for (int q = 0; q < per; ++q) {
            const int e = l[q];
            T[e] = dv<EXACT>(T[e], D) * m;
        }
    }
    double sum = 0.0;
#pragma unroll 8
    for (int e = 0; e < Tn; ++e) sum += T[e];
    D.den = sum;
    D.y = 1.0 / sum;
}

// child *= parent message broadcast over k % Ts, then Normalize (:1150-1238)
template <bool SPILL, bool EXACT>
__device__ void op_dmul(const Tab<SPILL> &T, Den &D, const double *__restrict__ sp, int Ts, int Tn) {
    const int Q = Tn / Ts;
    for (int j = 0; j < Ts; ++j) {
        const double m = sp[(size_t)j * 64];
#pragma unroll 8
        for (int q = 0; q < Q; ++q) {
            const int e = q * Ts + j;
            T[e] = dv<EXACT>(T[e], D) * m;
        }
    }
    double sum = 0.0;
#pragma unroll 8
    for (int e = 0; e < Tn; ++e) sum += T[e];
    D.den = sum;
    D.y = 1.0 / sum;
}

// message to the parent: tmp[k % Ts] += child[k]; the separator's old value is its masked all-ones
// table (x / 1.0 == x; its zero entries face child entries that are masked to zero) (:1056-1148)
template <bool SPILL, bool EXACT>
__device__ void op_sepcol(const Tab<SPILL> &T, const Den &D, double *__restrict__ sp, int Ts, int Tn) {
    const int Q = Tn / Ts;
    for (int j = 0; j < Ts; ++j) {
        double acc = 0.0;
#pragma unroll 8
        for (int q = 0; q < Q; ++q) acc += dv<EXACT>(T[q * Ts + j], D);
        sp[(size_t)j * 64] = acc;
    }
}

// tmp[map(k)] += parent[k]; sep = tmp / old, zero-guarded (:700-816)
template <bool SPILL, bool EXACT>
__device__ void op_sepdis(const Tab<SPILL> &T, const Den &D, double *__restrict__ sp, const int32_t *__restrict__ ls,
                          int Ts, int per) {
    for (int j = 0; j < Ts; ++j) {
        const int32_t *__restrict__ l = ls + j * per;
        double acc = 0.0;
#pragma unroll 8
        for (int q = 0; q < per; ++q) acc += dv<EXACT>(T[l[q]], D);
        const double old = sp[(size_t)j * 64];
        sp[(size_t)j * 64] = (old == 0.0) ? 0.0 : acc / old;
    }
}

// marginal of one variable from the clique (TableMarginalization in entry order), un-normalized
template <bool SPILL, bool EXACT>
__device__ void op_marg(const Tab<SPILL> &T, const Den &D, const MOut &o, bool act, int dim, int cum,
                        int Tn, double &tot) {
    const int bw = dim * cum, nhi = Tn / bw;
    tot = 0.0;
    for (int d = 0; d < dim; ++d) {
        double acc = 0.0;
        for (int hi = 0; hi < nhi; ++hi) {
            const int base = hi * bw + d * cum;
#pragma unroll 8
            for (int lo = 0; lo < cum; ++lo) acc += dv<EXACT>(T[base + lo], D);
        }
        if (act) o[d] = acc;
        tot += acc;
    }
}

// PROF: diagnostic build that accumulates s_memtime cycles per op type (prof[wave][32])
template <bool SPILL, bool PROF = false>
__global__ __launch_bounds__(64) void jt_lds_kernel(const JtOp *__restrict__ ops, const int32_t *__restrict__ aux,
                                                   const double *__restrict__ initv,
                                                   const uint64_t *__restrict__ dig,
                                                   const int8_t *__restrict__ evid, double *__restrict__ marg,
                                                   int32_t *__restrict__ labels, double *__restrict__ ws,
                                                   int32_t *__restrict__ wsi, const JtLParams A,
                                                   unsigned long long *__restrict__ prof = nullptr) {
    unsigned long long pc[24] = {0};
    extern __shared__ double lds[];
    const int lane = threadIdx.x;
    double *__restrict__ W = ws + (size_t)blockIdx.x * (size_t)A.wave_entries * 64 + lane;
    double *__restrict__ store = W + (size_t)A.store_off * 64;
    double *__restrict__ dens = W + (size_t)A.den_off * 64;
    double *__restrict__ sep = W + (size_t)A.sep_off * 64;
    int32_t *__restrict__ red = wsi + (size_t)blockIdx.x * (size_t)A.nc * 64 + lane;
    const Tab<SPILL> T{lds + lane, W + (size_t)A.spill_off * 64, A.cap};

    // blocks: grid stride; fixup mode (flags): each wave scans 64 flags per step (one load per lane +
    // a ballot) and runs only the flagged blocks -- a one-flag-per-step scan is a chain of dependent
    // scalar loads, ~80 ns each, which made a small fixup grid cost more than the kernel it checks
    long long blk = -1, cbase = (long long)blockIdx.x * 64 - (long long)gridDim.x * 64;
    unsigned long long pend = 0ull;
    for (;;) {
        if (A.flags) {
            while (pend == 0ull) {
                cbase += (long long)gridDim.x * 64;
                if (cbase * 64 >= A.ncases) break;
                const long long b = cbase + lane;
                pend = __ballot(b * 64 < A.ncases && A.flags[b] != 0);
            }
            if (pend == 0ull) break;
            blk = cbase + __builtin_ctzll(pend);
            pend &= pend - 1ull;
        } else {
            blk = blk < 0 ? (long long)blockIdx.x : blk + gridDim.x;
            if (blk * 64 >= A.ncases) break;
        }
        const long long cs = blk * 64 + lane;
        const bool act = cs < A.ncases;
        const long long csr = act ? cs : A.ncases - 1;
        const int8_t *__restrict__ ev = evid + csr * A.V;
        const MOut out{marg + csr * (A.vmajor ? 1 : A.SD), A.vmajor ? A.ncases : 1};
        Den D{1.0, 1.0};  // the clique in LDS is T[e] / D.den
        bool fast = true;

        for (int i = 0; i < A.nops; ++i) {
            const JtOp op = ops[i];
            unsigned long long t0 = 0;
            if (PROF) t0 = __builtin_amdgcn_s_memtime();
            switch (op.type) {
            case JT_L_INIT: {  // masked initial potential + post-evidence Normalize (:1479-1483)
                const int nv = op.d;
                uint64_t M0 = 0, M1 = 0, M2 = 0, M3 = 0, W0 = 0, W1 = 0, W2 = 0, W3 = 0;
                int nobs = 0;
                for (int j = 0; j < nv; ++j) {
                    const int x = ev[aux[op.c + j]];
                    const uint64_t m = x >= 0 ? (0xFFull << (8 * (j & 7))) : 0ull;
                    const uint64_t w = x >= 0 ? ((uint64_t)x << (8 * (j & 7))) : 0ull;
                    nobs += x >= 0;
                    if (j < 8) M0 |= m, W0 |= w;
                    else if (j < 16) M1 |= m, W1 |= w;
                    else if (j < 24) M2 |= m, W2 |= w;
                    else M3 |= m, W3 |= w;
                }
                const int nw = nv > 8 ? (nv + 7) / 8 : 1;
                const uint64_t *__restrict__ dg = dig + op.e;
                const double *__restrict__ iv = initv + op.h;
                double sum = 0.0;
#pragma unroll 8
                for (int e = 0; e < op.b; ++e) {
                    const uint64_t *d = dg + (size_t)e * nw;
                    bool cons = (d[0] & M0) == W0;
                    if (nw > 1) cons = cons && ((d[1] & M1) == W1);
                    if (nw > 2) cons = cons && ((d[2] & M2) == W2);
                    if (nw > 3) cons = cons && ((d[3] & M3) == W3);
                    const double val = cons ? iv[e] : 0.0;
                    T[e] = val;
                    sum += val;
                }
                D.den = sum;
                D.y = 1.0 / sum;
                fast = !A.force_exact && den_fast_all(sum);
                red[(size_t)op.g * 64] = nv - nobs;
                break;
            }
            case JT_L_MUL: {
                const double *sp = sep + (size_t)op.d * 64;
                if (fast) op_mul<SPILL, false>(T, D, sp, aux + op.e, op.c, op.b);
                else op_mul<SPILL, true>(T, D, sp, aux + op.e, op.c, op.b);
                fast = !A.force_exact && den_fast_all(D.den);
                break;
            }
            case JT_L_SEPCOL: {
                double *sp = sep + (size_t)op.a * 64;
                if (fast) op_sepcol<SPILL, false>(T, D, sp, op.b, op.c);
                else op_sepcol<SPILL, true>(T, D, sp, op.b, op.c);
                break;
            }
            case JT_L_STORE: {
                double *__restrict__ st = store + (size_t)op.a * 64;
#pragma unroll 8
                for (int e = 0; e < op.b; ++e) st[(size_t)e * 64] = T[e];
                dens[(size_t)op.c * 64] = D.den;
                break;
            }
            case JT_L_LOAD: {
                const double *__restrict__ st = store + (size_t)op.a * 64;
#pragma unroll 8
                for (int e = 0; e < op.b; ++e) T[e] = st[(size_t)e * 64];
                D.den = dens[(size_t)op.c * 64];
                D.y = 1.0 / D.den;
                fast = !A.force_exact && den_fast_all(D.den);
                break;
            }
            case JT_L_DMUL: {
                const double *sp = sep + (size_t)op.d * 64;
                if (fast) op_dmul<SPILL, false>(T, D, sp, op.e, op.b);
                else op_dmul<SPILL, true>(T, D, sp, op.e, op.b);
                fast = !A.force_exact && den_fast_all(D.den);
                break;
            }
            case JT_L_SEPDIS: {
                double *sp = sep + (size_t)op.a * 64;
                if (fast) op_sepdis<SPILL, false>(T, D, sp, aux + op.e, op.b, op.f);
                else op_sepdis<SPILL, true>(T, D, sp, aux + op.e, op.b, op.f);
                break;
            }
            case JT_L_MARG: {  // GetProbabilitiesOneNode / InferenceUsingJT (:1339-1454)
                if (ev[op.e] >= 0) break;
                const int32_t *__restrict__ cd = aux + op.c;
                int sel = -1, best = 0x7fffffff;
                for (int k = 0; k < op.d; ++k) {  // first clique with the fewest reduced variables
                    const int r = red[(size_t)cd[k] * 64];
                    if (r < best) best = r, sel = cd[k];
                }
                if (sel != op.g) break;
                const MOut o = out + op.a;
                double tot;
                if (fast) op_marg<SPILL, false>(T, D, o, act, op.b, op.h, op.pad, tot);
                else op_marg<SPILL, true>(T, D, o, act, op.b, op.h, op.pad, tot);
                if (act) {
                    if (op.f) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                        int lab = 0;
                        double mp = 0.0;
                        for (int d = 0; d < op.b; ++d) {
                            const double v = (best == 1) ? o[d] : o[d] / tot;
                            if (v > mp) mp = v, lab = d;
                        }
                        labels[cs] = lab;
                    }
                    for (int d = 0; d < op.b; ++d) o[d] = o[d] / tot;
                }
                break;
            }
            case JT_L_EVZERO: {
                if (act && ev[op.e] >= 0)
                    for (int d = 0; d < op.b; ++d) out[op.a + d] = 0.0;
                break;
            }
            default:
                break;
            }
            if (PROF) {
                __builtin_amdgcn_s_waitcnt(0);
                const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
                for (int k = 0; k < 10; ++k)
                    if (op.type == 11 + k) pc[k] += t1 - t0;
            }
        }
    }
    if (PROF && lane == 0)
        for (int k = 0; k < 10; ++k) prof[(size_t)blockIdx.x * 16 + k] = pc[k];
}

}  // namespace

extern "C" hipError_t fbn_jt_lds_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                        const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                        double *marg, int32_t *labels, double *ws, int32_t *wsi, long long wave_entries,
                                        long long store_off, long long den_off, long long sep_off,
                                        long long spill_off, int nc, int cap, bool spill, int force_exact,
                                        const int *flags, int grid, unsigned long long *prof, int vmajor,
                                        hipStream_t stream) {
    JtLParams a;
    a.force_exact = force_exact;
    a.vmajor = vmajor;
    a.flags = flags;
    a.ncases = ncases;
    a.wave_entries = wave_entries;
    a.store_off = store_off;
    a.den_off = den_off;
    a.sep_off = sep_off;
    a.spill_off = spill_off;
    a.nops = nops;
    a.V = V;
    a.SD = SD;
    a.nc = nc;
    a.cap = cap;
    const size_t lds = (size_t)cap * 64 * sizeof(double);
    if (prof) {
        if (spill)
            hipLaunchKernelGGL((jt_lds_kernel<true, true>), dim3(grid), dim3(64), lds, stream, ops, aux, initv, dig,
                               evid, marg, labels, ws, wsi, a, prof);
        else
            hipLaunchKernelGGL((jt_lds_kernel<false, true>), dim3(grid), dim3(64), lds, stream, ops, aux, initv, dig,
                               evid, marg, labels, ws, wsi, a, prof);
    } else if (spill) {
        hipLaunchKernelGGL((jt_lds_kernel<true, false>), dim3(grid), dim3(64), lds, stream, ops, aux, initv, dig,
                           evid, marg, labels, ws, wsi, a, nullptr);
    } else {
        hipLaunchKernelGGL((jt_lds_kernel<false, false>), dim3(grid), dim3(64), lds, stream, ops, aux, initv, dig,
                           evid, marg, labels, ws, wsi, a, nullptr);
    }
    return hipGetLastError();
}

// launch wrapper (called from capi.hip)
extern "C" hipError_t fbn_jt_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                    const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                    double *marg, int32_t *labels, double *ws, int32_t *wsi, long long NE, int nc,
                                    int grid, int vmajor, hipStream_t stream) {
    JtArgs a;
    a.vmajor = vmajor;
    a.ops = ops;
    a.aux = aux;
    a.initv = initv;
    a.dig = dig;
    a.evid = evid;
    a.marg = marg;
    a.labels = labels;
    a.ws = ws;
    a.wsi = wsi;
    a.ncases = ncases;
    a.NE = NE;
    a.nops = nops;
    a.V = V;
    a.SD = SD;
    a.nc = nc;
    hipLaunchKernelGGL(jt_interp_kernel, dim3(grid), dim3(64), 0, stream, a);
    return hipGetLastError();
}

// evidence range check of a host-supplied batch, on the device: *first = smallest flat index
// [case * V + v] whose value is outside -1 .. dom[v] - 1 (left at INT64_MAX when all are valid)
static __global__ __launch_bounds__(256) void jt_evidence_check(const int8_t *__restrict__ ev, long long n, int V,
                                                                const int32_t *__restrict__ dom,
                                                                unsigned long long *__restrict__ first) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int x = ev[i];
        const int v = (int)(i % V);
        if (x < -1 || x >= dom[v]) atomicMin(first, (unsigned long long)i);
    }
}

extern "C" hipError_t fbn_jt_evidence_check(const int8_t *ev, long long n, int V, const int32_t *dom,
                                            unsigned long long *first, hipStream_t s) {
    const long long b = (n + 255) / 256;
    hipLaunchKernelGGL(jt_evidence_check, dim3((unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096)), dim3(256), 0, s, ev, n,
                       V, dom, first);
    return hipGetLastError();
}

// ------------------------------------------------------------------ output layout / scoring
// case-major [n][SD] -> variable-major [SD][n] (the kernels without a variable-major store path
// write case-major scratch; fbn_jt_set_output_layout): 32 x 32 tiles through LDS, both sides coalesced
static __global__ __launch_bounds__(256) void jt_marg_transpose(const double *__restrict__ in, double *__restrict__ out,
                                                                long long n, int SD) {
    __shared__ double tile[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    const long long c0 = (long long)blockIdx.x * 32;  // cases on x (up to 2^31 - 1 tiles), values on y
    const int k0 = blockIdx.y * 32;
    for (int r = ty; r < 32; r += 8) {
        const long long c = c0 + r;
        const int k = k0 + tx;
        if (c < n && k < SD) tile[r][tx] = in[c * SD + k];
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int k = k0 + r;
        const long long c = c0 + tx;
        if (c < n && k < SD) out[(long long)k * n + c] = tile[tx][r];
    }
}

extern "C" hipError_t fbn_jt_marg_transpose(const double *in, double *out, long long n, int SD, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const long long gx = (n + 31) / 32, gy = (SD + 31) / 32;
    if (gx > 0x7FFFFFFFLL || gy > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(jt_marg_transpose, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, s, in, out, n, SD);
    return hipGetLastError();
}

// Round(x, 7) of src/Inference.cpp:195-206, the operations of fbn_jt_score's host lambda
__device__ __forceinline__ double jt_round7(double number) {
    const long long integerpart = (long long)number;
    number -= integerpart;
    for (int i = 0; i < 7; ++i) number *= 10;
    number = (double)(long long)(number + 0.5);
    for (int i = 0; i < 7; ++i) number /= 10;
    return integerpart + number;
}

// correctly rounded sqrt (the host's sqrtsd): the device estimate and its two neighbours, the one
// whose square is nearest x (exact fma residuals; sqrt never lands on a midpoint)
__device__ __forceinline__ double jt_sqrt_rn(double x) {
    if (!(x > 0.0) || __builtin_isinf(x)) return __builtin_sqrt(x);
    const double s = __builtin_sqrt(x);
    const long long b = __double_as_longlong(s);  // s > 0, finite: neighbours by the bit pattern
    const double sm = __longlong_as_double(b - 1), sp = __longlong_as_double(b + 1);
    const double r = __builtin_fabs(__builtin_fma(-s, s, x)), rm = __builtin_fabs(__builtin_fma(-sm, sm, x)),
                 rp = __builtin_fabs(__builtin_fma(-sp, sp, x));
    return rm < r ? (rm < rp ? sm : sp) : (rp < r ? sp : s);
}

// per-case MSE / HD terms (CalculateMSE / CalculateHellingerDistance, src/Inference.cpp:153-193),
// one thread per case; no contraction, so every term equals the host's fbn_jt_score term bit for bit
static __global__ __launch_bounds__(256) void jt_score_terms(const double *__restrict__ marg,
                                                             const double *__restrict__ golden, long long n, int SD,
                                                             long long mcs, long long mvs,
                                                             const int32_t *__restrict__ dom, int V,
                                                             double *__restrict__ terms) {
#pragma clang fp contract(off)
    for (long long c = (long long)blockIdx.x * 256 + threadIdx.x; c < n; c += (long long)gridDim.x * 256) {
        const double *__restrict__ a = marg + c * mcs;
        const double *__restrict__ x = golden + c * SD;
        int num = 0, off = 0;
        double e1 = 0.0, e2 = 0.0;
        for (int v = 0; v < V; ++v) {
            const int dv = dom[v];
            if (x[off] > 0) {
                num += dv;
                for (int j = 0; j < dv; ++j) {
                    const double r = jt_round7(a[(long long)(off + j) * mvs]);
                    const double d1 = r - x[off + j];
                    e1 += d1 * d1;
                    const double d2 = jt_sqrt_rn(r) - jt_sqrt_rn(x[off + j]);
                    e2 += d2 * d2;
                }
            }
            off += dv;
        }
        terms[2 * c] = jt_sqrt_rn(e1 / num);
        terms[2 * c + 1] = jt_sqrt_rn(e2 / num);
    }
}

extern "C" hipError_t fbn_jt_score_terms(const double *marg, const double *golden, long long n, int SD, int vmajor,
                                         const int32_t *dom, int V, double *terms, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const long long b = (n + 255) / 256;
    hipLaunchKernelGGL(jt_score_terms, dim3((unsigned)(b < 8192 ? b : 8192)), dim3(256), 0, s, marg, golden, n, SD,
                       vmajor ? 1LL : (long long)SD, vmajor ? n : 1LL, dom, V, terms);
    return hipGetLastError();
}
