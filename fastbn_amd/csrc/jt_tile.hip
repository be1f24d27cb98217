// jt_tile.hip -- tiled junction-tree kernel (variant 5, fast arithmetic order): the Munin-class
// default.  Passes and tables: jt_tile_plan.cpp; layout: jt_program.h (JtTPass).
//
// One wave = JT_T_C evidence cases x JT_T_L entry slots (lane = slot * JT_T_C + case), persistent
// over groups of JT_T_C cases (one wave per workgroup by default; FBN_JT_TW = 2 / 4 lets that many
// waves share a case group, its store and its LDS stage, splitting every pass by rounds or by
// blocks of outer configurations).  A pass walks one clique: slot s of round r takes G-configuration
// r * JT_T_L + s, every lane walks the same R stream, and entry e = G-part + R-part gives
//     w(e) = init(e) * prod_j M_j(s_j(e))        (0 if e contradicts the lane's case's evidence)
// -- the clique's table after all its child multiplications [and the parent's], up to the
// normalizations, which cancel (fast order; the reference multiplies and normalizes step by step,
// src/JunctionTree.cpp:829-941, 1150-1238).  Messages are stored un-normalized, each with a per-case
// scale row (normalized message = values / scale); a pass multiplies its lanes' sums by
// sigma = 1 / (product of its factors' scales).  The inner R stream sums into one register, and at
// the end of every inner run the sum (times sigma) is written straight to its output bin U(b):
//   Collect:     the upstream separator's message U, scale S = sum_b U(b)  (src/JunctionTree.cpp:1056-1148)
//   Distribute:  a child separator's message U, scale sum_b U(b)                       (:700-816)
// The reference's Distribute message is (U / S') / old, 0 where old == 0, S' = sum_b old U: the
// child's own Collect message `old` cancels in it (it is left out of the pass's factors), S' is a
// per-case constant that cancels in every normalized result, and where old(b) == 0 every entry of
// the child that b reaches is 0 already -- so U / sum U serves.  Marginals whose source is this pass
// (GetProbabilitiesOneNode, :1392-1454; ArgMax, src/Inference.cpp:92-102) sum old(b) U(b) by value.
// Outputs with fewer than JT_T_L bins take extra lane variables: their partial bins are added by a
// post sweep first.  Every sum runs in a fixed order (per lane, then a butterfly over the slots), so
// results are run-to-run identical.  Messages are rows [entry][JT_T_C cases] in the wave's store; a
// clique's factors are staged into LDS when they fit the per-wave budget.  A case group whose pass
// totals or factor scales leave [2^-900, 2^900] flags its 64-case block; the exact interpreter
// recomputes flagged blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jt_program.h"

namespace {

constexpr int C = JT_T_C, L = JT_T_L, kMaxW = JT_T_W;
static_assert(C * L == 64, "one wave = C cases x L slots");
constexpr int kValChunks = 2;  // marginal sweep: value d in slot d % L, chunk (d % kGrp) / L
constexpr int kGrp = kValChunks * L;  // values per bin sweep (more states: one sweep per group)
constexpr int kBinRows = JT_T_LDS_BIN_ROWS;  // bin sets up to this many rows live in LDS
#ifndef FBN_TILE_REUSE
#define FBN_TILE_REUSE 0  // 1: skip the load of a factor row equal to the step before's (bit 0 of its soffset)
#endif
#ifndef FBN_TILE_U
#define FBN_TILE_U 4  // steps per load batch
#endif
#ifndef FBN_TILE_VREC
#define FBN_TILE_VREC 0  // 1: step records by vector loads one chunk ahead (else scalar loads one batch ahead)
#endif
#ifndef FBN_TILE_STEPBRK
#define FBN_TILE_STEPBRK 1  // leave the unrolled batch at the step range's end (else: bin ends masked)
#endif
constexpr int kMaxCliqueVars = 10;           // evidence bytes loaded together; wider cliques (up to 32
                                             // digit bits, jt_tile_plan.cpp) take the rest in a loop

typedef __attribute__((ext_vector_type(2))) unsigned u2;

__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, int voff, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, voff, 0, 0);
}
// sum over the L slots of a case (lanes g, g + C, ...): a butterfly, identical in every lane
__device__ __forceinline__ double slot_sum(double x) {
#pragma unroll
    for (int o = C; o < 64; o <<= 1) x += __shfl_xor(x, o);
    return x;
}

// diagnostic phase clock: drains the wave's outstanding memory operations first, so a phase's
// loads are charged to it (prof mode only: slows the kernel down)
__device__ __forceinline__ unsigned long long dclock() {
    __builtin_amdgcn_s_waitcnt(0);
    return clock64();
}

// lane n of every 16-lane DPP row (row_newbcast:n): the value slot s's lane n loaded, to all 16
// lanes of the slot
template <int N>
__device__ __forceinline__ double row_bcast(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x150 + N, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x150 + N, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// n is a constant after unrolling: the switch folds to one row_bcast
__device__ __forceinline__ double row_bcast_n(double x, int n) {
    switch (n & 15) {
    case 0: return row_bcast<0>(x);
    case 1: return row_bcast<1>(x);
    case 2: return row_bcast<2>(x);
    case 3: return row_bcast<3>(x);
    case 4: return row_bcast<4>(x);
    case 5: return row_bcast<5>(x);
    case 6: return row_bcast<6>(x);
    case 7: return row_bcast<7>(x);
    case 8: return row_bcast<8>(x);
    case 9: return row_bcast<9>(x);
    case 10: return row_bcast<10>(x);
    case 11: return row_bcast<11>(x);
    case 12: return row_bcast<12>(x);
    case 13: return row_bcast<13>(x);
    case 14: return row_bcast<14>(x);
    default: return row_bcast<15>(x);
    }
}

// where a pass's inner-run sums go: straight to the output bins (direct: one bin per run, times
// sigma; LDS for a small private-variable output) or to the partial bins of the post sweep
struct PassOut {
    bool direct, out_lds, bins_lds;
    int out_b;   // output rows (bytes: wave store, or LDS for out_lds)
    int part_b;  // partial bins (bytes: LDS for bins_lds, else the wave store)
    double sig;
    int r0, rs;  // this wave's rounds: r0, r0 + rs, ...
    int kb, ke;  // and its steps of each round's R stream [kb, ke) (whole inner runs)
};

// the entry work of one pass: rounds of G-configurations x the flattened R stream (outer x inner
// configurations) -> partial bins; returns the lane's share of the pass total.  The stream runs in
// chunks of 16 steps = the 16 lanes (cases) of a slot: lane (s, g) loads the initial potential of
// ITS slot's entry at step k0 + g (one fully used gather per chunk instead of one per step), and
// step k0 + u takes it from lane u of the slot's DPP row.  Per step: a scalar step record (factor
// soffsets, digit word, the bin of the inner run ending there), one digit test and NF factor loads
// (LDS: one address add; wave store: voffset + soffset).  The sum of an inner run goes to its bin
// (LDS rows for small bin sets, else the wave store).  Factors 0 .. NL-1 are in LDS, the rest in the
// wave store.  Every factor is loaded at every step (round 6): a batch's loads are then one
// straight-line block the compiler can issue back to back and wait for one step at a time.  Bit 0 of
// a factor's soffset (set by the plan, which orders the R stream to make it common) marks "the same
// row as the step before"; skipping that load (FBN_TILE_REUSE=1, the round-4 form) costs a scalar
// branch per factor and step, splits the batch into basic blocks and measured 203 ms against 181-185
// ms for the branch-free loads (125k Munin-like cases; the repeated row is an L1 hit).  Build-time
// switches measured the same day and not kept: FBN_TILE_VREC=1 (step records as vector loads one chunk
// ahead, read out by v_readlane, so an LDS wait no longer waits for scalar record loads: 206 ms, VGPR
// spills), FBN_TILE_U=2 (190 ms), FBN_TILE_STEPBRK=0 (184 vs 185 ms, noise)
template <int NF, int NL>
__device__ __forceinline__ double pass_entries(const JtTPass &P, const int32_t *__restrict__ tab,
                                               __amdgpu_buffer_rsrc_t ivrs, __amdgpu_buffer_rsrc_t st,
                                               char *__restrict__ ldsb, int s, int g, uint32_t M, uint32_t Wd,
                                               const PassOut &O) {
    static_assert(C == 16, "a chunk = the 16 lanes of a DPP row");
    constexpr int RS = NF + 2, GS = 4 + NF, NFA = NF > 0 ? NF : 1;
    constexpr int U = FBN_TILE_U;  // steps with their loads in flight together
    const int g8 = g * 8;
    double tot = 0.0;
    const uint32_t gf = (uint32_t)P.gfields;
    const uint32_t MR = M & ~gf, WR = Wd & MR;  // evidence on the R digits
    const int kb = O.kb, ke = O.ke;
    const int32_t *__restrict__ sr = tab + P.st_off;
    const int32_t *__restrict__ et = tab + P.et_off;
    for (int r = O.r0; r < P.rounds; r += O.rs) {
        const int cfg = r * L + s;
        const bool la = cfg < P.nG;
        const int32_t *__restrict__ gr = tab + P.g_off + (size_t)(la ? cfg : 0) * GS;
        const int ivb = (P.iv_off + gr[0]) * 8;  // this lane's G part of the entry (bytes)
        const uint32_t dwG = (uint32_t)gr[1];
        const int xG = gr[2];
        int fG[NFA];
#pragma unroll
        for (int j = 0; j < NF; ++j) fG[j] = gr[4 + j] + g8;
        const bool okG = la && (((dwG ^ Wd) & M & gf) == 0u);
        double acc = 0.0;
        double fe[NFA];  // the factor values of the step before
#pragma unroll
        for (int j = 0; j < NFA; ++j) fe[j] = 0.0;
        // slot s's entry at step k0 + g, one chunk ahead (the tables are padded by one chunk)
        double wn = bld(ivrs, ivb + et[kb + g], 0);
#if FBN_TILE_VREC
        // the step records of a chunk (C steps x RS words) arrive one chunk ahead as VECTOR loads (lane
        // l holds word l + 64 v) and are read out with v_readlane per batch: vector loads complete in
        // order, so waiting for a batch's LDS factors (lgkmcnt) no longer waits for record loads too
        constexpr int RW = C * RS, NV = (RW + 63) / 64;
        const int ln = s * C + g;
        int32_t rc[NV], rn[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) rc[v] = v * 64 + ln < RW ? sr[(size_t)kb * RS + v * 64 + ln] : 0;
#else
        // the step records of the batch in flight (qc) and of the next one (qn): the next batch's
        // scalar loads are issued before this batch computes, so a scalar-cache miss is not on the
        // batch's critical path (the records are padded past every wave's last step)
        int32_t qc[U][RS];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < RS; ++i) qc[u][i] = sr[(size_t)(kb + u) * RS + i];
#endif
        for (int k0 = kb; k0 < ke; k0 += C) {
            const double wl = wn;
            if (k0 + C < ke) wn = bld(ivrs, ivb + et[k0 + C + g], 0);
#if FBN_TILE_VREC
            if (k0 + C < ke) {
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    rn[v] = v * 64 + ln < RW ? sr[(size_t)(k0 + C) * RS + v * 64 + ln] : 0;
            }
#endif
#pragma unroll
            for (int u0 = 0; u0 < C; u0 += U) {
                if (k0 + u0 >= ke) break;  // (uniform)
                double w[U], f[U][NFA];
                bool ok[U];
#if FBN_TILE_VREC
                int32_t qc[U][RS];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int i = 0; i < RS; ++i) {
                        const int wi = (u0 + u) * RS + i;
                        qc[u][i] = __builtin_amdgcn_readlane(rc[wi / 64], wi % 64);
                    }
#endif
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    ok[u] = (((uint32_t)qc[u][NF]) & MR) == WR;
#pragma unroll
                    for (int j = 0; j < NF; ++j) {
#if FBN_TILE_REUSE
                        if (qc[u][j] & 1) continue;  // (uniform) the row of the step before
#endif
                        const int qo = FBN_TILE_REUSE ? qc[u][j] : qc[u][j] & ~1;
                        if (j < NL) f[u][j] = *reinterpret_cast<const double *>(ldsb + (fG[j] + qo));  // bytes
                        else f[u][j] = bld(st, fG[j], qo);
                    }
                }
#if !FBN_TILE_VREC
                int32_t qn[U][RS];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int i = 0; i < RS; ++i) qn[u][i] = sr[(size_t)(k0 + u0 + U + u) * RS + i];
#endif
#pragma unroll
                for (int u = 0; u < U; ++u) w[u] = row_bcast_n(wl, u0 + u);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = k0 + u0 + u;
#if FBN_TILE_STEPBRK
                    if (k >= ke) break;
#endif
                    double x = w[u];
#pragma unroll
                    for (int j = 0; j < NF; ++j) {
#if FBN_TILE_REUSE
                        if (!(qc[u][j] & 1)) fe[j] = f[u][j];
#else
                        fe[j] = f[u][j];
#endif
                        x *= fe[j];
                    }
                    acc += ok[u] ? x : 0.0;
                    const int xo = qc[u][NF + 1];
                    // (steps past ke, up to the batch's end: padding, or the next wave's share -- summed
                    // into acc, never written: acc restarts with the next round)
                    if (xo != -1 && (FBN_TILE_STEPBRK || k < ke)) {  // end of an inner run (or of its chunk, loop-tiled): its bin
                        const bool add = xo < -1;  // (a later chunk: add into the bin, which this
                        const int xb = add ? -xo - 2 : xo;  // lane wrote in an earlier chunk)
                        const double a = okG ? acc : 0.0;
                        if (la) {
                            const int x8 = (xG + xb) * (C * 8) + g8;
                            if (O.direct) {
                                const double v = a * O.sig;
                                if (O.out_lds) {
                                    double *p = reinterpret_cast<double *>(ldsb + O.out_b + x8);
                                    *p = add ? *p + v : v;
                                } else {
                                    bst(st, O.out_b + x8, add ? bld(st, O.out_b + x8, 0) + v : v);
                                }
                                tot += v;
                            } else if (O.bins_lds) {
                                double *p = reinterpret_cast<double *>(ldsb + O.part_b + x8);
                                *p = add ? *p + a : a;
                            } else {
                                bst(st, O.part_b + x8, add ? bld(st, O.part_b + x8, 0) + a : a);
                            }
                        }
                        acc = 0.0;
                    }
                }
#if !FBN_TILE_VREC
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int i = 0; i < RS; ++i) qc[u][i] = qn[u][i];
#endif
            }
#if FBN_TILE_VREC
#pragma unroll
            for (int v = 0; v < NV; ++v) rc[v] = rn[v];
#endif
        }
    }
    return tot;
}

// the post sweep of a pass whose output has fewer than JT_T_L bins (extra lane variables E):
// output bin b = its nE partial bins added in order, times sigma, written like a direct pass's bin.
// Returns the wave's share of the pass total (lane partials in bin order, then the slot butterfly).
__device__ __forceinline__ double post_sweep(const JtTPass &P, __amdgpu_buffer_rsrc_t st, char *__restrict__ ldsb,
                                             int wv, int W, int s, int g8, const PassOut &O) {
    const int nE = P.nE, nb = P.nbins;
    double tot = 0.0;
    for (int b = wv * L + s; b < nb; b += W * L) {  // bins over the workgroup's slots
        double v = 0.0;
        for (int e = 0; e < nE; ++e) {
            const int x8 = (b * nE + e) * (C * 8) + g8;
            v += O.bins_lds ? *reinterpret_cast<const double *>(ldsb + O.part_b + x8) : bld(st, O.part_b + x8, 0);
        }
        v *= O.sig;
        const int o8 = b * (C * 8) + g8;
        if (O.out_lds) *reinterpret_cast<double *>(ldsb + O.out_b + o8) = v;
        else bst(st, O.out_b + o8, v);
        tot += v;
    }
    return slot_sum(tot);
}

template <int NF>
__device__ __forceinline__ double pass_entries_nl(const JtTPass &P, const int32_t *__restrict__ tab,
                                                  __amdgpu_buffer_rsrc_t ivrs, __amdgpu_buffer_rsrc_t st,
                                                  char *__restrict__ ldsb, int s, int g, uint32_t M, uint32_t Wd,
                                                  const PassOut &O) {
#define FBN_TNL(n)                                                                                        \
    case n:                                                                                               \
        if constexpr (n <= NF) return pass_entries<NF, n>(P, tab, ivrs, st, ldsb, s, g, M, Wd, O);    \
        else return 0.0;
    switch (P.nl) {
        FBN_TNL(1) FBN_TNL(2) FBN_TNL(3) FBN_TNL(4) FBN_TNL(5) FBN_TNL(6) FBN_TNL(7)
    default: return pass_entries<NF, 0>(P, tab, ivrs, st, ldsb, s, g, M, Wd, O);
    }
#undef FBN_TNL
}

__global__ __launch_bounds__(64 * kMaxW, 16 / kMaxW) void jt_tile_kernel(const JtTPass *__restrict__ passes, int npass,
                                                         const int32_t *__restrict__ tab, const double *__restrict__ iv,
                                                         const int8_t *__restrict__ evid, double *__restrict__ marg,
                                                         int32_t *__restrict__ labels, double *__restrict__ ws,
                                                         int *__restrict__ flags, long long ncases, long long store_rows,
                                                         long long scr_row, long long red_row, int V, int SD,
                                                         int fac_bytes, unsigned long long *__restrict__ prof) {
    extern __shared__ double lds[];
    char *ldsb = reinterpret_cast<char *>(lds);
    // (wv through readfirstlane: the compiler then knows it is wave-uniform, so the step records of
    // every wave's share stay scalar loads)
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid & 63;
    const int W = blockDim.x / 64;  // waves sharing the case group (the plan's split assumes this many)
    const int s = lane / C, g = lane % C, g8 = g * 8;
    // the workgroup's message store (its case group's messages, partial and reduced bins)
    __amdgpu_buffer_rsrc_t st = __builtin_amdgcn_make_buffer_rsrc(
        ws + (size_t)blockIdx.x * (size_t)store_rows * C, 0, (int)(store_rows * C * 8), 0x00020000);
    const int scr_b = (int)(scr_row * C * 8), red_b = (int)(red_row * C * 8);
    // LDS: [factors: fac_bytes][partial bins x nbuf][reduced bins x nbuf][wave totals x nbuf] -- with
    // several waves the bin and total regions alternate with the parity of the pass barrier, so a
    // wave one pass ahead never writes what a slower wave still reads
    constexpr int kBinBytes = kBinRows * C * 8;
    const int nbuf = W > 1 ? 2 : 1;
    const int bin0 = fac_bytes, red0 = fac_bytes + nbuf * kBinBytes, tot0 = fac_bytes + 2 * nbuf * kBinBytes;
    // initial potentials through a buffer resource: entry = per-lane G part (voffset) + the R
    // record's part (soffset, scalar) -- no per-step address arithmetic
    const __amdgpu_buffer_rsrc_t ivrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(iv), 0, 0x7FFFFFF8, 0x00020000);
    // diagnostic (prof != nullptr): s_memtime cycles per phase, summed over the waves -- [0] staging,
    // [1..3] entry work with every factor in LDS / in the wave store / mixed, [4] pass totals, scales
    // and the post sweep (incl. the barrier wait), [5] marginal sweeps, [6] all
    unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t_all = prof ? clock64() : 0ull;
    int par = 0;  // parity of the pass barriers so far (uniform over the workgroup)
    for (long long cg = blockIdx.x; cg * C < ncases; cg += gridDim.x) {
        const long long cs = cg * C + g;
        const bool act = cs < ncases;
        const long long csr = act ? cs : ncases - 1;
        const int8_t *__restrict__ ev = evid + csr * V;
        double *__restrict__ out = marg + csr * SD;
        uint32_t M = 0u, Wd = 0u;  // the case's evidence in the clique's digit fields
        bool bad = false;
        for (int p = 0; p < npass; ++p) {
            const JtTPass P = passes[p];
            unsigned long long t0 = prof ? dclock() : 0ull;
            if (P.first) {
                M = 0u, Wd = 0u;
                const int32_t *__restrict__ vr = tab + P.vars_off;
                int xs[kMaxCliqueVars];  // every evidence byte in flight at once
#pragma unroll
                for (int j = 0; j < kMaxCliqueVars; ++j) xs[j] = j < P.nv ? ev[vr[3 * j]] : -1;
#pragma unroll
                for (int j = 0; j < kMaxCliqueVars; ++j)
                    if (xs[j] >= 0) M |= (uint32_t)vr[3 * j + 2] << vr[3 * j + 1], Wd |= (uint32_t)xs[j] << vr[3 * j + 1];
                for (int j = kMaxCliqueVars; j < P.nv; ++j) {  // (wider cliques: the rest one at a time)
                    const int x = ev[vr[3 * j]];
                    if (x >= 0) M |= (uint32_t)vr[3 * j + 2] << vr[3 * j + 1], Wd |= (uint32_t)x << vr[3 * j + 1];
                }
                // the clique's LDS factors, staged by the whole workgroup (every wave is past the last
                // pass barrier, after which no wave reads the previous phase's factors)
                for (int k = 0; k < P.nstage; ++k) {
                    const int32_t *__restrict__ sg = tab + P.stage_off + 3 * k;
                    const int src = sg[0] * (C * 8), n = sg[1] * C, dst = sg[2] >> 3;
                    int i = tid;
                    for (; i + 3 * 64 * W < n; i += 4 * 64 * W) {  // four loads in flight
                        const double a0 = bld(st, i * 8, src), a1 = bld(st, (i + 64 * W) * 8, src),
                                     a2 = bld(st, (i + 128 * W) * 8, src), a3 = bld(st, (i + 192 * W) * 8, src);
                        lds[dst + i] = a0, lds[dst + i + 64 * W] = a1, lds[dst + i + 128 * W] = a2, lds[dst + i + 192 * W] = a3;
                    }
                    for (; i < n; i += 64 * W) lds[dst + i] = bld(st, i * 8, src);
                }
                // the staged factors, and the messages / scales the previous phase wrote (other lanes /
                // waves), become visible
                if (W > 1 || P.nstage > 0) __syncthreads();
                else __threadfence_block();
            }
            if (prof) {
                const unsigned long long t1 = dclock();
                pc[0] += t1 - t0;
                t0 = t1;
            }
            // a private-variable pass runs only if some case of the group lacks evidence on one of them
            bool need_entries = true;
            if (P.kind == JT_T_MARG) {
                bool any = false;
                for (int m = 0; m < P.nmv; ++m) any |= act && ev[tab[P.mv_off + 5 * m]] < 0;
                need_entries = __ballot(any) != 0ull;  // (the same cases in every wave)
            }
            // output: Collect / Distribute -> the message rows (wave store); private variables -> the
            // reduced rows (LDS when they fit); partial bins (outputs with extra lane variables) in LDS
            // when they fit
            const bool marg_pass = P.kind == JT_T_MARG;
            PassOut O;
            O.direct = P.nE == 1;
            O.bins_lds = P.nbins * P.nE <= kBinRows;
            O.part_b = O.bins_lds ? bin0 + par * kBinBytes : scr_b;
            O.out_lds = marg_pass && P.nbins <= kBinRows;
            O.out_b = marg_pass ? (O.out_lds ? red0 + par * kBinBytes : red_b) : P.dest_row * (C * 8);
            if (need_entries) {
                // this wave's share: rounds r = wv (mod W), or a contiguous block of outer configurations
                const int nRi = P.nRi;
                if (P.split == 0) {
                    O.r0 = wv, O.rs = W, O.kb = 0, O.ke = P.nRo * nRi;
                } else {
                    O.r0 = 0, O.rs = 1, O.kb = (P.nRo * wv) / W * nRi, O.ke = (P.nRo * (wv + 1)) / W * nRi;
                }
                // sigma = 1 / product of the factors' scales (this lane's case)
                double prod = 1.0;
                for (int j = 0; j < P.nf; ++j) prod *= bld(st, tab[P.fsc_off + j] * (C * 8) + g8, 0);
                bad |= act && !(prod >= 0x1p-900 && prod <= 0x1p+900);
                O.sig = 1.0 / prod;
                double tot = 0.0;
#define FBN_TNF(n) \
    case n: tot = pass_entries_nl<n>(P, tab, ivrs, st, ldsb, s, g, M, Wd, O); break;
                switch (P.nf) {
                    FBN_TNF(0) FBN_TNF(1) FBN_TNF(2) FBN_TNF(3) FBN_TNF(4) FBN_TNF(5) FBN_TNF(6)
                    default: tot = pass_entries_nl<7>(P, tab, ivrs, st, ldsb, s, g, M, Wd, O);
                }
#undef FBN_TNF
                if (prof) {
                    const unsigned long long t1 = dclock();
                    pc[P.nl == P.nf ? 1 : P.nl == 0 ? 2 : 3] += t1 - t0;
                    t0 = t1;
                }
                double Sw;
                if (O.direct) {
                    Sw = slot_sum(tot);
                } else {  // the partial bins (every wave's) become visible; then the post sweep
                    __syncthreads();
                    Sw = post_sweep(P, st, ldsb, wv, W, s, g8, O);
                }
                // pass total = the waves' shares in wave order; the barrier also makes the output bins
                // visible to the marginal sweep
                double S = Sw;
                if (W > 1) {
                    double *tw = reinterpret_cast<double *>(ldsb + tot0 + par * (W * C * 8));
                    if (s == 0) tw[wv * C + g] = Sw;
                    __syncthreads();
                    S = tw[g];
                    for (int w = 1; w < W; ++w) S += tw[w * C + g];
                } else if (P.nmv > 0) {  // one wave: the output bins (other lanes) become visible
                    if (O.out_lds) __syncthreads();
                    else __threadfence_block();
                }
                bad |= act && !(S >= 0x1p-900 && S <= 0x1p+900);
                if (!marg_pass && wv == 0 && s == 0) bst(st, P.dest_sc * (C * 8) + g8, S);  // the message's scale
                par ^= nbuf - 1;
                if (prof) {
                    const unsigned long long t1 = dclock();
                    pc[4] += t1 - t0;
                    t0 = t1;
                }
            }
            // marginals whose source is this pass (wave m % W): value d of the variable in slot d % L
            // (chunk d / L), summed over the bins in bin order, normalized by their total (evidence
            // variables: zeros).  Variables of more than kGrp states: one bin sweep per group of kGrp
            // values, the total from a first sweep over all bins
            for (int m = wv; m < P.nmv; m += W) {
                const int32_t *__restrict__ mr = tab + P.mv_off + 5 * m;
                const int var = mr[0], off = mr[1], dim = mr[2], sh = mr[3];
                const uint32_t fm = (uint32_t)mr[4];
                const bool obs = ev[var] >= 0;
                const bool need = need_entries && __ballot(act && !obs) != 0ull;
                const int32_t *__restrict__ bd = tab + P.bdig_off;
                const int nb = P.nbins;
                // bin values: old(b) U(b) (Distribute: the calibrated separator up to a per-case
                // constant), U(b) (private variables)
                auto bins4 = [&](int b0, double *v) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int bc = b0 + t < nb ? b0 + t : nb - 1;
                        const int o8 = bc * (C * 8) + g8;
                        if (marg_pass) v[t] = O.out_lds ? *reinterpret_cast<const double *>(ldsb + O.out_b + o8)
                                                        : bld(st, O.out_b + o8, 0);
                        else v[t] = bld(st, P.col_row * (C * 8) + o8, 0) * bld(st, O.out_b + o8, 0);
                    }
                };
                double tm = 0.0;
                if (need && dim > kGrp)
                    for (int b0 = 0; b0 < nb; b0 += 4) {
                        double v[4];
                        bins4(b0, v);
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            if (b0 + t < nb) tm += v[t];
                    }
                int lab = 0;
                double mx = 0.0, m2 = 0.0;
                for (int q0 = 0; q0 < dim; q0 += kGrp) {
                    double a[kValChunks];
#pragma unroll
                    for (int c = 0; c < kValChunks; ++c) a[c] = 0.0;
                    if (need) {
                        for (int b0 = 0; b0 < nb; b0 += 4) {
                            double v[4];
                            bins4(b0, v);
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                if (b0 + t >= nb) break;
                                const int dg = (int)(((uint32_t)bd[b0 + t] >> sh) & fm) - q0;
#pragma unroll
                                for (int c = 0; c < kValChunks; ++c) a[c] += dg == c * L + s ? v[t] : 0.0;
                            }
                        }
                    }
                    if (dim <= kGrp) {  // the lane's values in chunk order, then the slot butterfly
                        double am = 0.0;
#pragma unroll
                        for (int c = 0; c < kValChunks; ++c) am += a[c];
                        tm = slot_sum(am);
                    }
#pragma unroll
                    for (int c = 0; c < kValChunks; ++c)
                        if (act && q0 + c * L + s < dim) out[off + q0 + c * L + s] = obs ? 0.0 : a[c] / tm;
                    if (var == 0 && need)  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                        for (int d = q0; d < dim && d < q0 + kGrp; ++d) {
                            double ad = 0.0;
#pragma unroll
                            for (int c = 0; c < kValChunks; ++c) {
                                const double t = __shfl(a[c], (d % L) * C + g);
                                ad = (d - q0) / L == c ? t : ad;
                            }
                            const double pd = ad / tm;
                            if (pd > mx) m2 = mx, mx = pd, lab = d;
                            else if (pd > m2) m2 = pd;
                        }
                }
                if (var == 0 && need) {
                    if (act && !obs && s == 0) labels[cs] = lab;
                    // a near-tie (top two within 1e-12 relative) may break differently from the
                    // reference's exact values: the block goes to the exact pass
                    bad |= act && !obs && mx - m2 <= 1e-12 * mx;
                }
            }
            if (prof) pc[5] += dclock() - t0;
        }
        const unsigned long long fb = __ballot(bad);
        if (fb && lane == 0) atomicOr(flags + (cg * C) / 64, 1);
    }
    if (prof && lane == 0) {
        pc[6] = clock64() - t_all;
        for (int k = 0; k < 8; ++k) atomicAdd(prof + k, pc[k]);
    }
}

}  // namespace

extern "C" hipError_t fbn_jt_tile_launch(const JtTPass *passes, int npass, const int32_t *tab, const double *iv,
                                         const int8_t *evid, double *marg, int32_t *labels, double *ws, int *flags,
                                         long long ncases, long long store_rows, long long scr_row, long long red_row,
                                         int V, int SD, int lds_bytes, int grid, int waves,
                                         unsigned long long *prof, hipStream_t stream) {
    // workgroups of JT_T_W waves (one case group each); LDS per workgroup: the staged factors, the
    // small bin sets (partial, reduced; two parities each), the waves' pass totals (two parities)
    const int fac = (lds_bytes + 15) & ~15;
    const size_t nbuf = waves > 1 ? 2 : 1;
    const size_t total = (size_t)fac + 2 * nbuf * (size_t)kBinRows * C * 8 + nbuf * (size_t)waves * C * 8;
    hipLaunchKernelGGL(jt_tile_kernel, dim3(grid), dim3(64 * waves), total, stream, passes, npass, tab, iv, evid, marg,
                       labels, ws, flags, ncases, store_rows, scr_row, red_row, V, SD, fac, prof);
    return hipGetLastError();
}
