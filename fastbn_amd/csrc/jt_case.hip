// jt_case.hip -- per-case junction-tree kernel for large trees (Munin class), fast arithmetic order.
//
// One wave (one workgroup) = one evidence case at a time; persistent waves stride over the cases.
// Lanes run over the case's EVIDENCE-REDUCED clique entries: observed variables have one fixed
// digit (the reference's TableReduction, src/PotentialTable.cpp:309-396, with the evidence of
// src/JunctionTree.cpp:1150-1238), so only the consistent entries -- on the Munin-like tree 43 % of
// them on average -- are ever formed.  The unobserved variables of a clique split into
//   inner: the least significant ones, product >= 64 -- the lane index decodes into their digits
//          once per 64-entry chunk (per-lane offsets v_*),
//   outer: the rest -- 64 outer indices decode in parallel into "records" held one per lane, and
//          the entry loop fetches record r with v_readlane (scalar offsets s_*),
// so entry (record r, lane) has table index s_e + v_e and separator index s_t + v_t for every
// adjacent separator t (strides from jt_case_plan.cpp; no per-entry index arithmetic beyond adds).
//
// Per clique and direction ONE pass forms
//     w(e) = init(e) * M_1(s_1(e)) * ... * M_k(s_k(e)) [* D(s_up(e))]
// (child Collect messages in the reference's multiplication order, then the parent's Distribute
// message) and accumulates sum_e w(e) plus the bins of the separators / marginals fed by it:
//   Collect (post-order):     message to the parent  C(u) = bin_u / sum      (SeparatorLevelCollection,
//                                                                             src/JunctionTree.cpp:1056-1148)
//   Distribute (pre-order):   message to child j     D_j(s) = (bin_s / sum) / C_j(s), 0 if C_j(s) == 0
//                                                    (SeparatorLevelDistribution, :700-816)
//                             marginals of the variables this case reads from this clique
//                             (GetProbabilitiesOneNode, :1392-1454: the candidate with the fewest
//                             unobserved variables; ArgMax, src/Inference.cpp:92-102)
// The reference normalizes after every `parent *= ext`; those divisions cancel in the normalized
// result, so each message and marginal equals the reference's up to rounding (fp64, relative
// ~1e-15 per operation; north_star allows 1e-6).  Bins are fp64 atomics into the wave's own LDS
// (global memory for bin sets beyond the LDS budget): one wave per case keeps their order fixed.
// A case whose normalization sum leaves [2^-960, 2^960] flags its 64-case block for the exact
// interpreter (fixup pass, as variants 3 / 4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jt_program.h"

namespace {

constexpr int kMaxM = 4;  // marginals riding on one Distribute pass
constexpr int kMaxC = JT_C_MAX_CHILDREN;

__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double rdld(double v, int l) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// wave sum in a fixed pattern: quad swaps and row mirrors (DPP) leave the row sum in all 16
// lanes of each row (every step adds a + b on one lane and b + a on its partner: IEEE addition
// commutes), then the four row sums are added in order -- the same, run-independent value on
// every lane; all 64 lanes must be active
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror
    return (rdld(v, 0) + rdld(v, 16)) + (rdld(v, 32) + rdld(v, 48));
}
// floor(i / d) for 0 <= i < 2^26, 2 <= d <= 64 with M = ceil(2^32 / d): i * M / 2^32 exceeds i / d
// by less than i / 2^32 < 1/64 <= 1/d, never reaching the next integer (d == 1: M = 0, q = i)
__device__ __forceinline__ int udiv_small(int i, int d, int M) { return d == 1 ? i : (int)__umulhi((unsigned)i, (unsigned)M); }
__device__ __forceinline__ bool range_ok(double s) { return s >= 0x1p-960 && s <= 0x1p+960; }
__device__ __forceinline__ int top_bit(uint64_t m) { return 63 - __builtin_clzll(m); }

// lane j < nv: clique variable j (JT_C_VREC record) and this case's evidence for it
struct Cv {
    int var, dim, cum, up, out, x, mg;
    int cs[kMaxC];
};

// the case's index space of one clique: partition, observed offsets, sizes
struct Space {
    uint64_t inner, outer;
    int nin, nout;
    int be, bu;        // observed digits' offsets: table (incl. iv_off), upstream separator
    int bc[kMaxC];     // ... child separators
};

__device__ __forceinline__ void load_vars(const JtCClique &q, const int32_t *__restrict__ vrec,
                                          const signed char *ev, int lane, Cv &v) {
    v.var = 0, v.dim = 1, v.cum = 0, v.up = 0, v.out = 0, v.x = -1, v.mg = 0;
#pragma unroll
    for (int i = 0; i < kMaxC; ++i) v.cs[i] = 0;
    if (lane < q.nv) {
        const int32_t *__restrict__ r = vrec + (size_t)(q.var_off + lane) * JT_C_VREC;
        v.var = r[0], v.dim = r[1], v.cum = r[2], v.up = r[3];
#pragma unroll
        for (int i = 0; i < kMaxC; ++i) v.cs[i] = r[4 + i];
        v.out = r[4 + kMaxC];
        v.mg = r[5 + kMaxC];
        v.x = ev[v.var];  // (LDS copy of the case's evidence row)
    }
}

template <int K>
__device__ __forceinline__ void make_space(const JtCClique &q, const Cv &v, int lane, Space &sp) {
    const uint64_t live = __ballot(lane < q.nv);
    const uint64_t obs = __ballot(lane < q.nv && v.x >= 0);
    sp.be = q.iv_off, sp.bu = 0;
#pragma unroll
    for (int i = 0; i < kMaxC; ++i) sp.bc[i] = 0;
    for (uint64_t m = obs; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        const int x = rdl(v.x, j);
        sp.be += x * rdl(v.cum, j);
        sp.bu += x * rdl(v.up, j);
#pragma unroll
        for (int i = 0; i < K; ++i) sp.bc[i] += x * rdl(v.cs[i], j);
    }
    uint64_t un = live & ~obs;
    sp.inner = 0;
    sp.nin = 1;
    while (un && sp.nin < 64) {  // least significant unobserved variables first
        const int j = top_bit(un);
        un &= ~(1ull << j);
        sp.inner |= 1ull << j;
        sp.nin *= rdl(v.dim, j);
    }
    sp.outer = un;
    sp.nout = 1;
    for (uint64_t m = un; m; m &= m - 1) sp.nout *= rdl(v.dim, __builtin_ctzll(m));
}

typedef __attribute__((address_space(3))) double ldouble;
typedef __attribute__((address_space(1))) double gdouble;
// bins in LDS, or in the wave's global bin area for bin sets beyond the LDS budget (uniform choice)
__device__ __forceinline__ void bin_add(bool glob, double *b, double w) {
    if (glob) __hip_atomic_fetch_add((gdouble *)b, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add((ldouble *)b, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr int kU = 2;  // records in flight together (their loads issued before any product)
constexpr int kDbgNoAtomics = 1, kDbgNoGather = 2, kDbgNoInit = 4;  // ablations (wrong results)
constexpr int kDbgProf = 8;  // per-phase s_memtime totals into the prof array (diagnostic)
constexpr int kProf = 10;  // 0 case set-up, 1 Collect set-up, 2-4 Collect inner decode / records / entries,
                            // 5 Distribute set-up, 6-8 its decode / records / entries, 9 finishing
#define FBN_TP(k)                                         \
    do {                                                  \
        if (prof) {                                       \
            const unsigned long long t1_ = clock64();     \
            tp[k] += t1_ - t0;                            \
            t0 = t1_;                                     \
        }                                                 \
    } while (0)

// One pass over the clique's reduced entries (see the file comment).  DIST = Distribute pass:
// gathers the K child Collect messages (+ the parent's Distribute message unless root) and adds into
// the K child bins (when sepdis) and the m marginal bins; Collect: gathers the K child messages and
// adds into the upstream separator's bins (unless root).  Returns this lane's partial sum.
template <int K, bool DIST>
__device__ __forceinline__ double clique_pass(bool glob, const double *__restrict__ iv, const double *msg, double *bins,
                                              const Cv &v, const Space &sp, int lane, bool root, const int (&ccol)[kMaxC],
                                              int up_dis, bool sepdis, const int (&cb)[kMaxC], int m,
                                              const int (&mpos)[kMaxM], const int (&mb)[kMaxM], int dbg,
                                              unsigned long long (&tp)[kProf], unsigned long long &t0) {
    const bool gp = DIST && !root, bu = !DIST && !root;
    const bool prof = (dbg & kDbgProf) != 0;
    double acc = 0.0;
    for (int ch = 0; ch * 64 < sp.nin; ++ch) {
        int i = ch * 64 + lane;
        const bool act = i < sp.nin;
        int ve = 0, vu = 0, vc[kMaxC], vm[kMaxM];
#pragma unroll
        for (int k = 0; k < kMaxC; ++k) vc[k] = 0;
#pragma unroll
        for (int t = 0; t < kMaxM; ++t) vm[t] = 0;
        for (uint64_t msk = sp.inner; msk;) {
            const int j = top_bit(msk);
            msk &= ~(1ull << j);
            const int d = rdl(v.dim, j);
            const int qd = udiv_small(i, d, rdl(v.mg, j));
            const int dig = i - qd * d;
            i = qd;
            ve += dig * rdl(v.cum, j);
            vu += dig * rdl(v.up, j);
#pragma unroll
            for (int k = 0; k < K; ++k) vc[k] += dig * rdl(v.cs[k], j);
            if (DIST) {
#pragma unroll
                for (int t = 0; t < kMaxM; ++t)
                    if (t < m && mpos[t] == j) vm[t] = dig;
            }
        }
        FBN_TP(DIST ? 6 : 2);
        for (int sg = 0; sg * 64 < sp.nout; ++sg) {
            // records: outer index sg * 64 + lane -> scalar-side offsets
            int o = sg * 64 + lane;
            int re = sp.be, ru = sp.bu, rc[kMaxC], rm[kMaxM];
#pragma unroll
            for (int k = 0; k < kMaxC; ++k) rc[k] = sp.bc[k];
#pragma unroll
            for (int t = 0; t < kMaxM; ++t) rm[t] = 0;
            for (uint64_t msk = sp.outer; msk;) {
                const int j = top_bit(msk);
                msk &= ~(1ull << j);
                const int d = rdl(v.dim, j);
                const int qd = udiv_small(o, d, rdl(v.mg, j));
                const int dig = o - qd * d;
                o = qd;
                re += dig * rdl(v.cum, j);
                ru += dig * rdl(v.up, j);
#pragma unroll
                for (int k = 0; k < K; ++k) rc[k] += dig * rdl(v.cs[k], j);
                if (DIST) {
#pragma unroll
                    for (int t = 0; t < kMaxM; ++t)
                        if (t < m && mpos[t] == j) rm[t] = dig;
                }
            }
            const int nr = min(64, sp.nout - sg * 64);
            FBN_TP(DIST ? 7 : 3);
            for (int r0 = 0; r0 < nr; r0 += kU) {
                // kU records: all loads first, then the products and the bins
                double w[kU];
                int su[kU], sc[kU][kMaxC], sm[kU][kMaxM];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int r = min(r0 + u, nr - 1);
                    const int se = rdl(re, r);
                    su[u] = rdl(ru, r);
#pragma unroll
                    for (int k = 0; k < K; ++k) sc[u][k] = rdl(rc[k], r);
                    if (DIST) {
#pragma unroll
                        for (int t = 0; t < kMaxM; ++t) sm[u][t] = t < m ? rdl(rm[t], r) : 0;
                    }
                    w[u] = (dbg & kDbgNoInit) ? 1.0 : iv[se + ve];
                }
                double g[kU][kMaxC + 1];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
#pragma unroll
                    for (int k = 0; k < K; ++k) g[u][k] = (dbg & kDbgNoGather) ? 1.0 : msg[ccol[k] + sc[u][k] + vc[k]];
                    g[u][K] = (gp && !(dbg & kDbgNoGather)) ? msg[up_dis + su[u] + vu] : 1.0;
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    if (!act || r0 + u >= nr) continue;
                    double x = w[u];
#pragma unroll
                    for (int k = 0; k < K; ++k) x *= g[u][k];
                    if (gp) x *= g[u][K];
                    acc += x;
                    if (dbg & kDbgNoAtomics) continue;
                    if (bu) bin_add(glob, bins + su[u] + vu, x);
                    if (DIST) {
                        if (sepdis) {
#pragma unroll
                            for (int k = 0; k < K; ++k) bin_add(glob, bins + cb[k] + sc[u][k] + vc[k], x);
                        }
#pragma unroll
                        for (int t = 0; t < kMaxM; ++t)
                            if (t < m) bin_add(glob, bins + mb[t] + sm[u][t] + vm[t], x);
                    }
                }
            }
            FBN_TP(DIST ? 8 : 4);
        }
    }
    return acc;
}

// bins visible to every lane after the pass: LDS atomics are ordered within the wave; global ones
// (bin sets beyond the LDS budget) are read back with L1-bypassing loads after the wait
__device__ __forceinline__ double bin_read(const double *b, bool global) {
    return global ? __hip_atomic_load(b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *b;
}

#define FBN_CDISPATCH(Kv, CALL)        \
    do {                               \
        switch (Kv) {                  \
        case 0: CALL(0); break;        \
        case 1: CALL(1); break;        \
        case 2: CALL(2); break;        \
        case 3: CALL(3); break;        \
        case 4: CALL(4); break;        \
        case 5: CALL(5); break;        \
        default: CALL(6); break;       \
        }                              \
    } while (0)

__global__ __launch_bounds__(64) void jt_case_kernel(
    const JtCClique *__restrict__ cls, const int32_t *__restrict__ vrec, const int32_t *__restrict__ aux,
    const double *__restrict__ initv, const int32_t *__restrict__ post, const int32_t *__restrict__ pre,
    const int32_t *__restrict__ vsel, const int8_t *__restrict__ evid, double *__restrict__ marg,
    int32_t *__restrict__ labels, double *__restrict__ ws, int *__restrict__ flags, long long ncases,
    long long msg_doubles, long long gbin_doubles, int nc, int V, int SD, int lds_bins, int dbg,
    unsigned long long *__restrict__ prof_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: bins | the case's evidence row | unobserved count per clique | chosen clique per variable
    double *lbins = reinterpret_cast<double *>(smem);
    signed char *ev_s = reinterpret_cast<signed char *>(smem + (size_t)lds_bins * 8);
    unsigned char *red_s = reinterpret_cast<unsigned char *>(ev_s + ((V + 7) & ~7));
    unsigned short *sel_s = reinterpret_cast<unsigned short *>(red_s + ((nc + 7) & ~7));
    const int lane = threadIdx.x;
    double *msg = ws + (size_t)blockIdx.x * (size_t)(msg_doubles + gbin_doubles);
    double *gbins = msg + msg_doubles;
    const bool prof = (dbg & kDbgProf) != 0;
    unsigned long long tp[kProf];
#pragma unroll
    for (int k = 0; k < kProf; ++k) tp[k] = 0;
    unsigned long long t0 = prof ? clock64() : 0;
    // A workgroup is one wave: its LDS and vector-memory operations complete in program order, so no
    // barrier is needed between producing and consuming lanes -- only the compiler must not move
    // memory operations across these points.
#define FBN_WAVE_ORDER() __builtin_amdgcn_wave_barrier()

    for (long long cs = blockIdx.x; cs < ncases; cs += gridDim.x) {
        const int8_t *__restrict__ ev = evid + cs * V;
        double *__restrict__ out = marg + cs * SD;
        bool bad = false;
        for (int v = lane; v < V; v += 64) ev_s[v] = ev[v];
        FBN_WAVE_ORDER();

        // remaining (unobserved) variables per clique, then each variable's clique
        // (first candidate with the fewest, src/JunctionTree.cpp:1412-1434)
        for (int c = lane; c < nc; c += 64) {
            const JtCClique q = cls[c];
            int cnt = 0;
            for (int j = 0; j < q.nv; ++j) cnt += ev_s[vrec[(size_t)(q.var_off + j) * JT_C_VREC]] < 0;
            red_s[c] = (unsigned char)cnt;
        }
        FBN_WAVE_ORDER();
        int best0 = 0;
        for (int v = lane; v < V; v += 64) {
            const int32_t *__restrict__ cd = aux + vsel[4 * v];
            const int n = vsel[4 * v + 1];
            int sel = 0, best = 0x7fffffff;
            for (int k = 0; k < n; ++k) {
                const int r = red_s[cd[k]];
                if (r < best) best = r, sel = cd[k];
            }
            sel_s[v] = (unsigned short)sel;
            if (v == 0) best0 = best;
        }
        best0 = rdl(best0, 0);
        FBN_WAVE_ORDER();
        FBN_TP(0);

        // ---------------- Collect (children first; the root needs no pass of its own).  The next
        // clique's variable records are loaded while this one runs.
        for (int n = 0; n < nc - 1; ++n) {
            const JtCClique q = cls[post[n]];
            Cv v;
            load_vars(q, vrec, ev_s, lane, v);
            FBN_TP(1);
            const bool glob = q.up_Ts > lds_bins;
            double *B = glob ? gbins : lbins;
            for (int b = lane; b < q.up_Ts; b += 64) B[b] = 0.0;
            int ccol[kMaxC], cb[kMaxC], mpos[kMaxM] = {0, 0, 0, 0}, mb[kMaxM] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < kMaxC; ++k) {
                ccol[k] = k < q.k ? aux[q.child_off + 3 * k + 1] : 0;
                cb[k] = 0;
            }
            if (glob) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
            FBN_WAVE_ORDER();
            double a = 0.0;
            Space sp;
#define FBN_CCALL(Kc)                                                                                          \
    make_space<Kc>(q, v, lane, sp);                                                                             \
    a = clique_pass<Kc, false>(glob, initv, msg, B, v, sp, lane, false, ccol, 0, false, cb, 0, mpos, mb, dbg, tp, t0)
            FBN_CDISPATCH(q.k, FBN_CCALL);
#undef FBN_CCALL
            const double S = wave_sum(a);
            bad |= !range_ok(S);
            if (glob) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
            FBN_WAVE_ORDER();
            for (int u = lane; u < q.up_Ts; u += 64) msg[q.up_col + u] = bin_read(B + u, glob) / S;
            FBN_WAVE_ORDER();
            FBN_TP(9);
        }

        // ---------------- Distribute (parents first) and the marginals
        for (int n = 0; n < nc; ++n) {
            const int c = pre[n];
            const JtCClique q = cls[c];
            Cv v;
            load_vars(q, vrec, ev_s, lane, v);
            uint64_t mine = __ballot(lane < q.nv && v.x < 0 && sel_s[v.var] == c);
            if (q.k == 0 && mine == 0) continue;  // a leaf nobody reads a marginal from
            bool first = true;
            int ccol[kMaxC], cb[kMaxC], cts[kMaxC], cdis[kMaxC];
            int sep_bins = 0;
#pragma unroll
            for (int k = 0; k < kMaxC; ++k) {
                const bool on = k < q.k;
                cts[k] = on ? aux[q.child_off + 3 * k] : 0;
                ccol[k] = on ? aux[q.child_off + 3 * k + 1] : 0;
                cdis[k] = on ? aux[q.child_off + 3 * k + 2] : 0;
                cb[k] = sep_bins;
                sep_bins += cts[k];
            }
            Space sp;
#define FBN_SCALL(Kc) make_space<Kc>(q, v, lane, sp)
            FBN_CDISPATCH(q.k, FBN_SCALL);
#undef FBN_SCALL
            FBN_TP(5);
            while (first || mine) {
                const bool sepdis = first && q.k > 0;
                int m = 0, mpos[kMaxM] = {0, 0, 0, 0}, mb[kMaxM] = {0, 0, 0, 0};
                int nb = sepdis ? sep_bins : 0;
                while (mine && m < kMaxM) {
                    const int j = __builtin_ctzll(mine);
                    mine &= mine - 1;
#pragma unroll
                    for (int t = 0; t < kMaxM; ++t)
                        if (t == m) mpos[t] = j, mb[t] = nb;
                    nb += rdl(v.dim, j);
                    ++m;
                }
                const bool glob = nb > lds_bins;
                double *B = glob ? gbins : lbins;
                for (int b = lane; b < nb; b += 64) B[b] = 0.0;
                if (glob) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
                FBN_WAVE_ORDER();
                double a = 0.0;
#define FBN_DCALL(Kc)                                                                                               \
    a = clique_pass<Kc, true>(glob, initv, msg, B, v, sp, lane, q.root != 0, ccol, q.up_dis, sepdis, cb, m, mpos, mb, \
                              dbg, tp, t0)
                FBN_CDISPATCH(q.k, FBN_DCALL);
#undef FBN_DCALL
                const double R = wave_sum(a);
                bad |= !range_ok(R);
                if (glob) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
                FBN_WAVE_ORDER();
                if (sepdis) {
                    for (int k = 0; k < q.k; ++k) {
                        const int Ts = rdl(cts[k], 0);
                        for (int s = lane; s < Ts; s += 64) {
                            const double old = msg[ccol[k] + s];
                            const double nw = bin_read(B + cb[k] + s, glob) / R;
                            msg[cdis[k] + s] = (old == 0.0) ? 0.0 : nw / old;
                        }
                    }
                }
                for (int t = 0; t < m; ++t) {
                    const int j = mpos[t];
                    const int dim = rdl(v.dim, j), var = rdl(v.var, j), off = rdl(v.out, j);
                    const double o = lane < dim ? bin_read(B + mb[t] + lane, glob) / R : 0.0;
                    double tot = 0.0;
                    for (int d = 0; d < dim; ++d) tot += rdld(o, d);  // bins in value order
                    if (var == 0) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                        int lab = 0;
                        double mx = 0.0;
                        for (int d = 0; d < dim; ++d) {
                            const double od = rdld(o, d);
                            const double p = (best0 == 1) ? od : od / tot;
                            if (p > mx) mx = p, lab = d;
                        }
                        if (lane == 0) labels[cs] = lab;
                    }
                    if (lane < dim) out[off + lane] = o / tot;
                }
                first = false;
                FBN_WAVE_ORDER();
                FBN_TP(9);
            }
        }
        // evidence variables: probabilities stay 0 (their first slot is compared with -1 by the scorer)
        for (int v = lane; v < V; v += 64)
            if (ev_s[v] >= 0) {
                const int off = vsel[4 * v + 2], dim = vsel[4 * v + 3];
                for (int d = 0; d < dim; ++d) out[off + d] = 0.0;
            }
        if (__ballot(bad) != 0ull && lane == 0) flags[cs >> 6] = 1;
        FBN_WAVE_ORDER();
        FBN_TP(0);
    }
    if (prof && lane == 0)
        for (int k = 0; k < kProf; ++k) atomicAdd(prof_out + k, tp[k]);
}

}  // namespace

extern "C" hipError_t fbn_jt_case_launch(const JtCClique *cls, const int32_t *vrec, const int32_t *aux,
                                         const double *initv, const int32_t *post, const int32_t *pre,
                                         const int32_t *vsel, const int8_t *evid, double *marg, int32_t *labels,
                                         double *ws, int *flags, long long ncases, long long msg_doubles,
                                         long long gbin_doubles, int nc, int V, int SD, int lds_bins, int grid,
                                         int dbg, unsigned long long *prof, hipStream_t stream) {
    const size_t lds = (size_t)lds_bins * 8 + (size_t)((V + 7) & ~7) + (size_t)((nc + 7) & ~7) + (size_t)V * 2;
    hipLaunchKernelGGL(jt_case_kernel, dim3(grid), dim3(64), lds, stream, cls, vrec, aux, initv, post, pre, vsel,
                       evid, marg, labels, ws, flags, ncases, msg_doubles, gbin_doubles, nc, V, SD, lds_bins, dbg, prof);
    return hipGetLastError();
}
