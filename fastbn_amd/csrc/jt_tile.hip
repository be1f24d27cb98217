// jt_tile.hip -- tiled junction-tree kernel (variant 5, fast arithmetic order): the Munin-class
// default.  Passes and tables: jt_tile_plan.cpp; layout: jt_program.h (JtTPass).
//
// One wave = JT_T_C evidence cases x JT_T_L entry slots (lane = slot * JT_T_C + case), persistent
// over groups of JT_T_C cases.  A pass walks one clique: slot s of round r takes G-configuration
// r * JT_T_L + s, every lane walks the same R stream, and entry e = G-part + R-part gives
//     w(e) = init(e) * prod_j M_j(s_j(e))        (0 if e contradicts the lane's case's evidence)
// -- the clique's table after all its child multiplications [and the parent's], up to the
// normalizations, which cancel (fast order; the reference multiplies and normalizes step by step,
// src/JunctionTree.cpp:829-941, 1150-1238).  The inner R stream sums into one register, stored once
// per outer configuration into the pass's partial-bin rows; the post sweep adds the E partials of
// every output bin in order, normalizes by the pass total S and writes
//   Collect:     the upstream separator's message  tmp / S          (src/JunctionTree.cpp:1056-1148)
//   Distribute:  a child separator's message  (tmp / S) / old, 0 where old == 0       (:700-816)
// and the marginals whose source is this pass (GetProbabilitiesOneNode, :1392-1454; ArgMax,
// src/Inference.cpp:92-102).  Every sum runs in a fixed order (per lane, then a butterfly over the
// slots), so results are run-to-run identical.  Messages are 64-byte rows [entry][JT_T_C cases] in
// the wave's store; a clique's factors are staged into LDS when they fit the per-wave budget.
// A case group whose pass totals leave [2^-900, 2^900] flags its 64-case block; the exact
// interpreter recomputes flagged blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jt_program.h"

namespace {

constexpr int C = JT_T_C, L = JT_T_L;
constexpr int U = 4;  // R steps with their loads in flight together
static_assert(C * L == 64, "one wave = C cases x L slots");
static_assert(JT_T_MAXDIM <= L, "the marginal sweep gives each value one slot");

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

// the entry work of one pass: rounds of G-configurations x the R stream -> partial bins; returns
// the lane's share of the pass total.  MODE 0: every factor in LDS, 1: every factor in the wave
// store, 2: all but the last (the parent message) in LDS
template <int NF, int MODE>
__device__ __forceinline__ double pass_entries(const JtTPass &P, const int32_t *__restrict__ tab,
                                               const double *__restrict__ iv, __amdgpu_buffer_rsrc_t st,
                                               const double *__restrict__ lds, int s, int g8, uint32_t M, uint32_t W,
                                               int scr_b) {
    constexpr int RS = 2 + NF, GS = 4 + NF;
    double tot = 0.0;
    const uint32_t MR = M & ~(uint32_t)P.gfields, WR = W & MR;
    const int nRi = P.nRi;
    for (int r = 0; r < P.rounds; ++r) {
        const int cfg = r * L + s;
        const bool la = cfg < P.nG;
        const int32_t *__restrict__ gr = tab + P.g_off + (size_t)(la ? cfg : 0) * GS;
        const int eG = gr[0];
        const uint32_t dwG = (uint32_t)gr[1];
        const int xG = gr[2];
        int fG[NF > 0 ? NF : 1];
#pragma unroll
        for (int j = 0; j < NF; ++j) fG[j] = gr[4 + j] + g8;
        const bool okG = la && (((dwG ^ W) & M & (uint32_t)P.gfields) == 0u);
        const double *__restrict__ ivg = iv + P.iv_off + eG;
        for (int o = 0; o < P.nRo; ++o) {
            const int32_t *__restrict__ rr = tab + P.r_off + (size_t)o * nRi * RS;
            double acc = 0.0;
            int i = 0;
            auto step = [&](const int32_t *__restrict__ q, double &w, double (&f)[NF > 0 ? NF : 1], bool &ok) {
                w = ivg[q[0]];
                ok = (((uint32_t)q[1]) & MR) == WR;
#pragma unroll
                for (int j = 0; j < NF; ++j) {
                    if (MODE == 0 || (MODE == 2 && j < NF - 1)) f[j] = lds[(fG[j] + q[2 + j]) >> 3];
                    else f[j] = bld(st, fG[j], q[2 + j]);
                }
            };
            for (; i + U <= nRi; i += U) {
                double w[U], f[U][NF > 0 ? NF : 1];
                bool ok[U];
#pragma unroll
                for (int u = 0; u < U; ++u) step(rr + (size_t)(i + u) * RS, w[u], f[u], ok[u]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    double x = w[u];
#pragma unroll
                    for (int j = 0; j < NF; ++j) x *= f[u][j];
                    acc += ok[u] ? x : 0.0;
                }
            }
            for (; i < nRi; ++i) {
                double w, f[NF > 0 ? NF : 1];
                bool ok;
                step(rr + (size_t)i * RS, w, f, ok);
                double x = w;
#pragma unroll
                for (int j = 0; j < NF; ++j) x *= f[j];
                acc += ok ? x : 0.0;
            }
            const double a = okG ? acc : 0.0;
            if (la) bst(st, scr_b + (xG + tab[P.o_off + o]) * (C * 8) + g8, a);
            tot += a;
        }
    }
    return tot;
}

#define FBN_TCASE(NFv)                                                                                    \
    case NFv:                                                                                             \
        if (P.mode == 0) tot = pass_entries<NFv, 0>(P, tab, iv, st, lds, s, g8, M, W, scr_b);             \
        else if (P.mode == 1) tot = pass_entries<NFv, 1>(P, tab, iv, st, lds, s, g8, M, W, scr_b);        \
        else tot = pass_entries<NFv, 2>(P, tab, iv, st, lds, s, g8, M, W, scr_b);                         \
        break;

__global__ __launch_bounds__(64) void jt_tile_kernel(const JtTPass *__restrict__ passes, int npass,
                                                     const int32_t *__restrict__ tab, const double *__restrict__ iv,
                                                     const int8_t *__restrict__ evid, double *__restrict__ marg,
                                                     int32_t *__restrict__ labels, double *__restrict__ ws,
                                                     int *__restrict__ flags, long long ncases, long long store_rows,
                                                     long long scr_row, long long red_row, int V, int SD) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x & 63;
    const int s = lane / C, g = lane % C, g8 = g * 8;
    __amdgpu_buffer_rsrc_t st = __builtin_amdgcn_make_buffer_rsrc(
        ws + (size_t)blockIdx.x * (size_t)store_rows * C, 0, (int)(store_rows * C * 8), 0x00020000);
    const int scr_b = (int)(scr_row * C * 8), red_b = (int)(red_row * C * 8);
    for (long long cg = blockIdx.x; cg * C < ncases; cg += gridDim.x) {
        const long long cs = cg * C + g;
        const bool act = cs < ncases;
        const long long csr = act ? cs : ncases - 1;
        const int8_t *__restrict__ ev = evid + csr * V;
        double *__restrict__ out = marg + csr * SD;
        uint32_t M = 0u, W = 0u;  // the case's evidence in the clique's digit fields
        bool bad = false;
        for (int p = 0; p < npass; ++p) {
            const JtTPass P = passes[p];
            if (P.first) {
                M = 0u, W = 0u;
                const int32_t *__restrict__ vr = tab + P.vars_off;
                for (int j = 0; j < P.nv; ++j) {
                    const int x = ev[vr[3 * j]];
                    if (x >= 0) M |= (uint32_t)vr[3 * j + 2] << vr[3 * j + 1], W |= (uint32_t)x << vr[3 * j + 1];
                }
                if (P.nstage > 0) {
                    __syncthreads();  // (one wave per workgroup: orders the LDS writes after earlier reads)
                    for (int k = 0; k < P.nstage; ++k) {
                        const int32_t *__restrict__ sr = tab + P.stage_off + 3 * k;
                        const int src = sr[0] * (C * 8), n = sr[1] * C, dst = sr[2] >> 3;
                        for (int i = lane; i < n; i += 64) lds[dst + i] = bld(st, i * 8, src);
                    }
                    __syncthreads();
                }
            }
            // a private-variable pass runs only if some case of the group lacks evidence on one of them
            bool need_entries = true;
            if (P.kind == JT_T_MARG) {
                bool any = false;
                for (int m = 0; m < P.nmv; ++m) any |= act && ev[tab[P.mv_off + 5 * m]] < 0;
                need_entries = __ballot(any) != 0ull;
            }
            double S = 1.0;
            if (need_entries) {
                double tot = 0.0;
                switch (P.nf) {
                    FBN_TCASE(0) FBN_TCASE(1) FBN_TCASE(2) FBN_TCASE(3) FBN_TCASE(4) FBN_TCASE(5) FBN_TCASE(6)
                    default: {
                        if (P.mode == 0) tot = pass_entries<7, 0>(P, tab, iv, st, lds, s, g8, M, W, scr_b);
                        else if (P.mode == 1) tot = pass_entries<7, 1>(P, tab, iv, st, lds, s, g8, M, W, scr_b);
                        else tot = pass_entries<7, 2>(P, tab, iv, st, lds, s, g8, M, W, scr_b);
                    }
                }
                S = slot_sum(tot);
                bad |= act && !(S >= 0x1p-900 && S <= 0x1p+900);
                __threadfence_block();  // the partial bins, stored by other lanes, become visible
                // post sweep: output bin b = sum of its nE partial bins (in order)
                const int nE = P.nE;
                for (int b = s; b < P.nbins; b += L) {
                    double v = 0.0;
                    for (int e = 0; e < nE; ++e) v += bld(st, scr_b + (b * nE + e) * (C * 8) + g8, 0);
                    if (P.kind == JT_T_COL) {
                        bst(st, (P.dest_row + b) * (C * 8) + g8, v / S);
                    } else if (P.kind == JT_T_DIS) {
                        const double old = bld(st, (P.col_row + b) * (C * 8) + g8, 0);
                        bst(st, (P.dest_row + b) * (C * 8) + g8, old == 0.0 ? 0.0 : (v / S) / old);
                    }
                    if (P.nmv > 0) bst(st, red_b + b * (C * 8) + g8, v);
                }
                __threadfence_block();
            }
            // marginals whose source is this pass: value d of the variable in slot d, summed over the
            // bins in bin order, normalized by their total (evidence variables: zeros)
            for (int m = 0; m < P.nmv; ++m) {
                const int32_t *__restrict__ mr = tab + P.mv_off + 5 * m;
                const int var = mr[0], off = mr[1], dim = mr[2], sh = mr[3];
                const uint32_t fm = (uint32_t)mr[4];
                const bool obs = ev[var] >= 0;
                const bool need = need_entries && __ballot(act && !obs) != 0ull;
                double a = 0.0;
                if (need) {
                    const int32_t *__restrict__ bd = tab + P.bdig_off;
                    for (int b = 0; b < P.nbins; ++b) {
                        const int dg = (int)(((uint32_t)bd[b] >> sh) & fm);
                        const double v = bld(st, red_b + b * (C * 8) + g8, 0);
                        a += dg == s ? v : 0.0;
                    }
                }
                const double tm = slot_sum(a);
                if (act && s < dim) out[off + s] = obs ? 0.0 : a / tm;
                if (var == 0 && need) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
                    int lab = 0;
                    double mx = 0.0;
                    for (int d = 0; d < dim; ++d) {
                        const double pd = __shfl(a, d * C + g) / tm;
                        if (pd > mx) mx = pd, lab = d;
                    }
                    if (act && !obs && s == 0) labels[cs] = lab;
                }
            }
        }
        const unsigned long long fb = __ballot(bad);
        if (fb && lane == 0) atomicOr(flags + (cg * C) / 64, 1);
    }
}

}  // namespace

extern "C" hipError_t fbn_jt_tile_launch(const JtTPass *passes, int npass, const int32_t *tab, const double *iv,
                                         const int8_t *evid, double *marg, int32_t *labels, double *ws, int *flags,
                                         long long ncases, long long store_rows, long long scr_row, long long red_row,
                                         int V, int SD, int lds_bytes, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(jt_tile_kernel, dim3(grid), dim3(64), (size_t)(lds_bytes > 0 ? lds_bytes : 8), stream, passes,
                       npass, tab, iv, evid, marg, labels, ws, flags, ncases, store_rows, scr_row, red_row, V, SD);
    return hipGetLastError();
}
