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
};

#define AT(e) S[(size_t)(e) * 64]

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
        double *__restrict__ out = A.marg + csr * A.SD;

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
                const int Ts = op.b, Q = op.d / op.b;
                for (int j = 0; j < Ts; ++j) {
                    double acc = 0.0;
#pragma unroll 4
                    for (int q = 0; q < Q; ++q) acc += AT(op.c + q * Ts + j) / den;
                    const double old = AT(op.a + j);
                    AT(op.a + j) = (old == 0.0) ? 0.0 : acc / old;
                }
                break;
            }
            case JT_OP_CLQMUL: {  // src/JunctionTree.cpp:829-941 (extension + multiply + Normalize)
                const double den = AT(op.c);
                const int32_t *__restrict__ mp = aux + op.e;
                double sum = 0.0;
#pragma unroll 4
                for (int e = 0; e < op.b; ++e) {
                    const double v = (AT(op.a + e) / den) * AT(op.d + mp[e]);
                    AT(op.a + e) = v;
                    sum += v;
                }
                AT(op.c) = sum;
                break;
            }
            case JT_OP_SEPDIS: {  // src/JunctionTree.cpp:700-816
                const double den = AT(op.d);
                const int32_t *__restrict__ ls = aux + op.e;
                const int per = op.f;
                for (int j = 0; j < op.b; ++j) {
                    double acc = 0.0;
#pragma unroll 4
                    for (int q = 0; q < per; ++q) acc += AT(op.c + ls[j * per + q]) / den;
                    const double old = AT(op.a + j);
                    AT(op.a + j) = (old == 0.0) ? 0.0 : acc / old;
                }
                break;
            }
            case JT_OP_CLQDIS: {  // src/JunctionTree.cpp:1150-1238
                const double den = AT(op.c);
                const int Ts = op.e, Q = op.b / op.e;
                double sum = 0.0;
                for (int q = 0; q < Q; ++q) {
#pragma unroll 4
                    for (int j = 0; j < Ts; ++j) {
                        const int e = q * Ts + j;
                        const double v = (AT(op.a + e) / den) * AT(op.d + j);
                        AT(op.a + e) = v;
                        sum += v;
                    }
                }
                AT(op.c) = sum;
                break;
            }
            case JT_OP_MARG: {  // src/JunctionTree.cpp:1339-1454, src/Inference.cpp:92-102
                const int dim = op.b;
                double *__restrict__ o = out + op.a;
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
                    const int bw = dim * cum, nhi = T / bw;
                    double tot = 0.0;
                    for (int d = 0; d < dim; ++d) {
                        double acc = 0.0;
                        for (int hi = 0; hi < nhi; ++hi)
#pragma unroll 4
                            for (int lo = 0; lo < cum; ++lo) acc += AT(toff + hi * bw + d * cum + lo) / den;
                        if (act) o[d] = acc;
                        tot += acc;
                    }
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
struct JtLArgs {
    const JtOp *ops;
    const int32_t *aux;
    const double *initv;
    const uint64_t *dig;
    const int8_t *evid;
    double *marg;
    int32_t *labels;
    double *ws;     // per wave: [store][dens nc][sep][spill] x 64
    int32_t *wsi;   // per wave: [nc] x 64 (reduced variable counts)
    long long ncases;
    long long wave_entries;  // store + nc + sep + spill
    long long store_off, den_off, sep_off, spill_off;
    int nops, V, SD, nc, cap;
};

template <bool SPILL>
__global__ __launch_bounds__(64) void jt_lds_kernel(JtLArgs A) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x;
    double *__restrict__ W = A.ws + (size_t)blockIdx.x * (size_t)A.wave_entries * 64 + lane;
    double *__restrict__ store = W + (size_t)A.store_off * 64;
    double *__restrict__ dens = W + (size_t)A.den_off * 64;
    double *__restrict__ sep = W + (size_t)A.sep_off * 64;
    double *__restrict__ spill = W + (size_t)A.spill_off * 64;
    int32_t *__restrict__ red = A.wsi + (size_t)blockIdx.x * (size_t)A.nc * 64 + lane;
    double *__restrict__ T = lds + lane;
    const JtOp *__restrict__ ops = A.ops;
    const int32_t *__restrict__ aux = A.aux;
    const int cap = A.cap;
#define TT(e) (*((!SPILL || (e) < cap) ? &T[(size_t)(e) * 64] : &spill[(size_t)((e) - cap) * 64]))
#define SP(e) sep[(size_t)(e) * 64]

    for (long long blk = blockIdx.x; blk * 64 < A.ncases; blk += gridDim.x) {
        const long long cs = blk * 64 + lane;
        const bool act = cs < A.ncases;
        const long long csr = act ? cs : A.ncases - 1;
        const int8_t *__restrict__ ev = A.evid + csr * A.V;
        double *__restrict__ out = A.marg + csr * A.SD;
        double den = 1.0;  // pending normalization denominator of the clique in LDS

        for (int i = 0; i < A.nops; ++i) {
            const JtOp op = ops[i];
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
                const uint64_t *__restrict__ dg = A.dig + op.e;
                const double *__restrict__ iv = A.initv + op.h;
                double sum = 0.0;
#pragma unroll 4
                for (int e = 0; e < op.b; ++e) {
                    const uint64_t *d = dg + (size_t)e * nw;
                    bool cons = (d[0] & M0) == W0;
                    if (nw > 1) cons = cons && ((d[1] & M1) == W1);
                    if (nw > 2) cons = cons && ((d[2] & M2) == W2);
                    if (nw > 3) cons = cons && ((d[3] & M3) == W3);
                    const double val = cons ? iv[e] : 0.0;
                    TT(e) = val;
                    sum += val;
                }
                den = sum;
                red[(size_t)op.g * 64] = nv - nobs;
                break;
            }
            case JT_L_MUL: {  // parent *= extended child message; Normalize (:829-941)
                const int32_t *__restrict__ mp = aux + op.e;
                const double *__restrict__ sp = sep + (size_t)op.d * 64;
                double sum = 0.0;
#pragma unroll 4
                for (int e = 0; e < op.b; ++e) {
                    const double v = (TT(e) / den) * sp[(size_t)mp[e] * 64];
                    TT(e) = v;
                    sum += v;
                }
                den = sum;
                break;
            }
            case JT_L_SEPCOL: {  // message to the parent: tmp[k % Ts] += child[k] (:1056-1148)
                // the separator's old value is its masked all-ones table, and x / 1.0 == x, while
                // its zero entries face child entries that are themselves masked to zero
                const int Ts = op.b, Q = op.c / op.b;
                for (int j = 0; j < Ts; ++j) {
                    double acc = 0.0;
#pragma unroll 4
                    for (int q = 0; q < Q; ++q) acc += TT(q * Ts + j) / den;
                    SP(op.a + j) = acc;
                }
                break;
            }
            case JT_L_STORE: {
                double *__restrict__ st = store + (size_t)op.a * 64;
#pragma unroll 8
                for (int e = 0; e < op.b; ++e) st[(size_t)e * 64] = TT(e);
                dens[(size_t)op.c * 64] = den;
                break;
            }
            case JT_L_LOAD: {
                const double *__restrict__ st = store + (size_t)op.a * 64;
#pragma unroll 8
                for (int e = 0; e < op.b; ++e) TT(e) = st[(size_t)e * 64];
                den = dens[(size_t)op.c * 64];
                break;
            }
            case JT_L_DMUL: {  // child *= parent message (k % Ts); Normalize (:1150-1238)
                const double *__restrict__ sp = sep + (size_t)op.d * 64;
                const int Ts = op.e, Q = op.b / op.e;
                double sum = 0.0;
                for (int q = 0; q < Q; ++q) {
#pragma unroll 4
                    for (int j = 0; j < Ts; ++j) {
                        const int e = q * Ts + j;
                        const double v = (TT(e) / den) * sp[(size_t)j * 64];
                        TT(e) = v;
                        sum += v;
                    }
                }
                den = sum;
                break;
            }
            case JT_L_SEPDIS: {  // tmp[map(k)] += parent[k]; sep = tmp / old, zero-guarded (:700-816)
                const int32_t *__restrict__ ls = aux + op.e;
                const int per = op.f;
                for (int j = 0; j < op.b; ++j) {
                    double acc = 0.0;
#pragma unroll 4
                    for (int q = 0; q < per; ++q) acc += TT(ls[j * per + q]) / den;
                    const double old = SP(op.a + j);
                    SP(op.a + j) = (old == 0.0) ? 0.0 : acc / old;
                }
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
                const int dim = op.b, cum = op.h, bw = dim * cum, nhi = op.pad / bw;
                double *__restrict__ o = out + op.a;
                double tot = 0.0;
                for (int d = 0; d < dim; ++d) {
                    double acc = 0.0;
                    for (int hi = 0; hi < nhi; ++hi)
#pragma unroll 4
                        for (int lo = 0; lo < cum; ++lo) acc += TT(hi * bw + d * cum + lo) / den;
                    if (act) o[d] = acc;
                    tot += acc;
                }
                if (act) {
                    if (op.f) {  // label: ArgMax, strict '>' from 0 (src/Inference.cpp:92-102)
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
        }
    }
#undef TT
#undef SP
}

}  // namespace

extern "C" hipError_t fbn_jt_lds_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                        const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                        double *marg, int32_t *labels, double *ws, int32_t *wsi, long long wave_entries,
                                        long long store_off, long long den_off, long long sep_off,
                                        long long spill_off, int nc, int cap, bool spill, int grid,
                                        hipStream_t stream) {
    JtLArgs a;
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
    if (spill)
        hipLaunchKernelGGL(jt_lds_kernel<true>, dim3(grid), dim3(64), lds, stream, a);
    else
        hipLaunchKernelGGL(jt_lds_kernel<false>, dim3(grid), dim3(64), lds, stream, a);
    return hipGetLastError();
}

// launch wrapper (called from capi.hip)
extern "C" hipError_t fbn_jt_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                    const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                    double *marg, int32_t *labels, double *ws, int32_t *wsi, long long NE, int nc,
                                    int grid, hipStream_t stream) {
    JtArgs a;
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
