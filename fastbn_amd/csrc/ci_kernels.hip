// ci_kernels.hip -- batched G^2 conditional-independence tests on gfx950.
//
// One 256-thread workgroup per test (grid-stride over the batch).  The column store is uint8
// [var][sample]; each thread streams 4 samples per load (one dword per column).  Tables of <= 16
// cells are counted in per-lane packed 16-bit counters held in registers (4 x u64, no LDS traffic
// in the sample loop) and wave-reduced once per test; larger tables N[z][x][y] use per-wave LDS
// sub-histograms (LDS atomics without cross-wave contention), merged once per test.  Marginals, the
// adjusted degrees of freedom and the G^2 terms (one per cell: the logs) are then evaluated by
// parallel threads; one lane adds the terms in cell order -- the reference's single running sum
// over z -> x -> y -- and evaluates p = 1 - P(df/2, G^2/2) (ci_chisq.h).
//
// Reference: Counts2D/Counts3D (src/CellTable.cpp:23-91,226-291,430-455) and
// ComputeGSquareXY/XYZ (src/IndependenceTest.cpp:65-155,295-364).  Counts and df are exact; G^2
// is the reference's sum of the same terms in the same order (skipped cells contribute +0.0,
// which leaves a running sum unchanged).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "ci_chisq.h"

namespace {

// G^2 terms buffered per chunk of cells (LDS doubles) before the in-order sum
constexpr int kTermChunk = 1024;
constexpr long long kWideTests = 512;  // batches up to this size: 1024-thread workgroups
constexpr int kDerivedInts = 256;      // MODE 3: the four full 3-way tables (4 x 64 ints) after the terms
// MODE 3 / 4: the derived d = 2 counting with the register allocation unconstrained (2 waves per
// SIMD) / allowing 3 waves per SIMD (the default; only the widest state-count instantiations spill)
__host__ __device__ constexpr int der2_waves(int mode) { return mode == 4 ? 3 : 1; }

// sub-histogram copies per wave for a table of `cells` > 16 cells (0: one shared table, beyond
// 64 KB of LDS for the 4 waves' copies): 4 for small tables (config-5 level 2, <= 256 cells:
// 0.589 -> 0.519 ms), 2 up to 512 cells, else 1 -- on larger tables the extra copies' zeroing and
// merging cost more than the atomic conflicts they remove (level 3: 0.100 -> 0.138 ms with 4)
__device__ __host__ inline int sub_lanes(int cells) {
    return cells <= 16 ? 0 : cells <= 256 ? 4 : cells <= 512 ? 2 : cells <= 4096 ? 1 : 0;
}

struct CiArgs {
    const uint8_t *cols;  // [nvars][N]
    const int32_t *dims;
    const int32_t *items;  // [n][2+D]
    long long N;
    long long n;
    double alpha;
    double *g2;
    int32_t *df;
    double *p;
    uint8_t *indep;
    int32_t *counts;  // optional: histogram of item 0
    int32_t *gscratch;  // non-null: tables too large for LDS live in global memory, one region per
    long long gstride;  // workgroup of gstride ints (same layout as the LDS one)
    // decision-margin log: [0] = min over tests of |p - alpha| as IEEE bits
    // (non-negative doubles order like their bit patterns), [1] = #tests with |p - alpha| < 1e-9
    unsigned long long *stats;
    // non-null: count from the bit-sliced store instead (every variable of every test has <= 4
    // states; all value rows of variable v start at row0[v], W words per row)
    const uint32_t *bits;
    const int32_t *row0;
    long long W;
    // decisions only (p == nullptr): [lo, hi] per df 1..nband then delta (ci_chisq.h fbn_chisq_band)
    const double *band;
    int nband;
    // PK instantiation: the columns packed 2 bits per sample (every state count <= 4), 16 samples
    // per word, PW words per variable (fbn_ci_pack2_build)
    const uint32_t *pk;
    long long PW;
    // counts != nullptr: cstride == 0 -> the table of test 0 only; cstride > 0 -> every test's table
    // at counts + test * cstride (fbn_ci_debug_counts)
    long long cstride;
    // split mode (small batches, MODE 1 / 2): test t's table at tab + t * tstride (zeroed), its
    // packed words divided among `split` workgroups
    int32_t *tab;
    long long tstride;
    int split;
    // MODE 3 (d = 2, bit-sliced, derived): the pair tables of this PC run's level 0 (every pair u < v
    // of the nvars variables, [value of u][value of v], ci_bits.hip pair_table)
    const int32_t *pairtab;
    int nvars;
    int dbg;  // diagnostic ablations (FBN_CI_DER2_DBG): bit 0 = MODE 3 skips its counting
};

// ---- MODE 3: tests with two conditioning variables (z1, z2), every state count <= 4, from the
// bit-sliced store, counting only LEADING cells (values 0 .. d-2 of each variable; the masks of a
// variable partition the samples, so the last value of any variable follows by subtraction):
//   L4[c1][c2][a][b] = sum popcount(x_a & y_b & z1_c1 & z2_c2)      the 4-way table's leading cells
//   the leading cells of the four 3-way tables (x, y | z1), (x, y | z2), (z1, z2, x), (z1, z2, y)
// then every 3-way table is completed from its leading cells and the pair tables level 0 recorded
// (full 2-way tables), and the 4-way table from its leading cells and the four 3-way tables --
// each step fills the cells whose last index is at its last value from cells already known:
//   G[i][j][MK] = P_ij - sum_k<MK G[i][j][k];  G[i][MJ][k] = P_ik - sum_j<MJ;  G[MI][j][k] = P_jk - sum_i<MI
// Exact integers: the table is Counts3D's (src/CellTable.cpp:268-291, z = c1 * dz2 + c2) cell for
// cell, so the G^2 epilogue is the histogram kernel's own.  Per 32 samples: <= 54 AND + popcount
// pairs per wave (wave c1 < 3: the 4-way and three 3-way tables of its z1 value; wave 3: (x, y | z2))
// instead of 32 LDS-atomic binnings.
__device__ __forceinline__ int pair_at(const int32_t *__restrict__ pairtab, int nvars, const int32_t *__restrict__ dims,
                                       int u, int a, int v, int b) {
    const int i = u < v ? u : v, j = u < v ? v : u;
    const int32_t *T = pairtab + 16 * ((long long)i * nvars - (long long)i * (i + 1) / 2 + (j - i - 1));
    return u < v ? T[a * dims[v] + b] : T[b * dims[u] + a];
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// the leading cells of one test (see above) for MX = dx - 1, MY = dy - 1, M2 = dz2 - 1 values: wave
// c1 < M1 counts the 4-way cells and three 3-way tables of its z1 value, wave 3 the (x, y | z2)
// table; wave totals into the 4-way table (hist) and the 3-way tables (F..., [i][j][k] at (4i+j)4+k)
template <int MX, int MY, int M2>
__device__ __forceinline__ void lead4(const uint32_t *__restrict__ px, const uint32_t *__restrict__ py,
                                      const uint32_t *__restrict__ p1, const uint32_t *__restrict__ p2, long long W,
                                      int M1, int wv, int lane, int32_t *__restrict__ hist, int d2, int dx, int dy,
                                      int32_t *__restrict__ Fxy1, int32_t *__restrict__ Fxy2,
                                      int32_t *__restrict__ F12x, int32_t *__restrict__ F12y) {
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    constexpr int AX = MX > 0 ? MX : 1, AY = MY > 0 ? MY : 1, A2 = M2 > 0 ? M2 : 1;
    constexpr int kQU = MX * MY * A2 > 8 ? 1 : 4;  // sub-words unrolled (see the word loop)
    // waves 0-2: (z1 value c1, word part) units -- with fewer than 3 z1 leading values the words are
    // split between waves (M1 = 1: 3 parts), so a binary z1 does not leave two waves idle; wave 3
    // counts (x, y | z2) over all words.  Parts add into the (zeroed) LDS tables atomically.
    const int P = M1 > 0 ? 3 / M1 : 0;
    const bool c1wave = wv < M1 * P, ywave = wv == 3;  // (uniform per wave)
    if (!c1wave && !ywave) return;
    const int c1 = c1wave ? wv % M1 : 0, part = c1wave ? wv / M1 : 0, nparts = c1wave ? P : 1;
    uint32_t k4[A2][AX][AY], ka[AX][AY], kc[A2][AX], kd[A2][AY];
#pragma unroll
    for (int a = 0; a < AX; ++a) {
#pragma unroll
        for (int b = 0; b < AY; ++b) {
            ka[a][b] = 0u;
#pragma unroll
            for (int c = 0; c < A2; ++c) k4[c][a][b] = 0u;
        }
#pragma unroll
        for (int c = 0; c < A2; ++c) kc[c][a] = 0u;
    }
#pragma unroll
    for (int c = 0; c < A2; ++c)
#pragma unroll
        for (int b = 0; b < AY; ++b) kd[c][b] = 0u;
    if (c1wave) {
        const uint32_t *pz1 = p1 + (size_t)c1 * W;
        for (long long w4 = lane + 64 * part; 4 * w4 < W; w4 += 64 * nparts) {
            u4 X[AX], Y[AY], Z[A2];
#pragma unroll
            for (int a = 0; a < MX; ++a) X[a] = *reinterpret_cast<const u4 *>(px + a * W + 4 * w4);
#pragma unroll
            for (int b = 0; b < MY; ++b) Y[b] = *reinterpret_cast<const u4 *>(py + b * W + 4 * w4);
#pragma unroll
            for (int c = 0; c < M2; ++c) Z[c] = *reinterpret_cast<const u4 *>(p2 + c * W + 4 * w4);
            const u4 Z1 = *reinterpret_cast<const u4 *>(pz1 + 4 * w4);
            // (the four sub-words one after the other for the wide tables: all four in flight
            // needed 238 VGPRs, i.e. 2 waves per SIMD)
#pragma unroll kQU
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int a = 0; a < MX; ++a) {
                    const uint32_t xm = X[a][q] & Z1[q];
#pragma unroll
                    for (int c = 0; c < M2; ++c) kc[c][a] += __builtin_popcount(xm & Z[c][q]);
#pragma unroll
                    for (int b = 0; b < MY; ++b) {
                        const uint32_t xy = xm & Y[b][q];
                        ka[a][b] += __builtin_popcount(xy);
#pragma unroll
                        for (int c = 0; c < M2; ++c) k4[c][a][b] += __builtin_popcount(xy & Z[c][q]);
                    }
                }
#pragma unroll
                for (int b = 0; b < MY; ++b) {
                    const uint32_t ym = Y[b][q] & Z1[q];
#pragma unroll
                    for (int c = 0; c < M2; ++c) kd[c][b] += __builtin_popcount(ym & Z[c][q]);
                }
            }
        }
    } else {  // wave 3: (x, y | z2)'s leading cells
        for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
            u4 X[AX], Y[AY], Z[A2];
#pragma unroll
            for (int a = 0; a < MX; ++a) X[a] = *reinterpret_cast<const u4 *>(px + a * W + 4 * w4);
#pragma unroll
            for (int b = 0; b < MY; ++b) Y[b] = *reinterpret_cast<const u4 *>(py + b * W + 4 * w4);
#pragma unroll
            for (int c = 0; c < M2; ++c) Z[c] = *reinterpret_cast<const u4 *>(p2 + c * W + 4 * w4);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int a = 0; a < MX; ++a)
#pragma unroll
                    for (int b = 0; b < MY; ++b) {
                        const uint32_t xy = X[a][q] & Y[b][q];
#pragma unroll
                        for (int c = 0; c < M2; ++c) k4[c][a][b] += __builtin_popcount(xy & Z[c][q]);
                    }
        }
    }
    auto I3 = [](int i, int j, int k) { return (i * 4 + j) * 4 + k; };
#pragma unroll
    for (int c = 0; c < M2; ++c)
#pragma unroll
        for (int a = 0; a < MX; ++a)
#pragma unroll
            for (int b = 0; b < MY; ++b) {
                const uint32_t v = wave_sum(k4[c][a][b]);
                if (lane == 0) {
                    if (c1wave) atomicAdd(&hist[((c1 * d2 + c) * dx + a) * dy + b], (int32_t)v);
                    else Fxy2[I3(c, a, b)] = (int32_t)v;
                }
            }
    if (c1wave) {
#pragma unroll
        for (int a = 0; a < MX; ++a)
#pragma unroll
            for (int b = 0; b < MY; ++b) {
                const uint32_t v = wave_sum(ka[a][b]);
                if (lane == 0) atomicAdd(&Fxy1[I3(c1, a, b)], (int32_t)v);
            }
#pragma unroll
        for (int c = 0; c < M2; ++c) {
#pragma unroll
            for (int a = 0; a < MX; ++a) {
                const uint32_t v = wave_sum(kc[c][a]);
                if (lane == 0) atomicAdd(&F12x[I3(c1, c, a)], (int32_t)v);
            }
#pragma unroll
            for (int b = 0; b < MY; ++b) {
                const uint32_t v = wave_sum(kd[c][b]);
                if (lane == 0) atomicAdd(&F12y[I3(c1, c, b)], (int32_t)v);
            }
        }
    }
}

// hist: the test's table (zeroed); F: 4 x 64 ints of LDS for the 3-way tables
__device__ __forceinline__ void derived4(const CiArgs &A, int x, int y, int z1, int z2, int dx, int dy,
                                      int32_t *__restrict__ hist, int32_t *__restrict__ F, int tid) {
    const long long W = A.W;
    const int32_t *dims = A.dims;
    const int d1 = dims[z1], d2 = dims[z2];
    const int MX = dx - 1, MY = dy - 1, M1 = d1 - 1, M2 = d2 - 1;
    const int wv = tid >> 6, lane = tid & 63;
    const uint32_t *px = A.bits + (size_t)A.row0[x] * W, *py = A.bits + (size_t)A.row0[y] * W,
                   *p1 = A.bits + (size_t)A.row0[z1] * W, *p2 = A.bits + (size_t)A.row0[z2] * W;
    // F[0] = (z1, x, y), F[1] = (z2, x, y), F[2] = (z1, z2, x), F[3] = (z1, z2, y): [i][j][k] at
    // (i * 4 + j) * 4 + k; the 4-way table in hist at ((c1 * d2 + c2) * dx + a) * dy + b
    int32_t *Fxy1 = F, *Fxy2 = F + 64, *F12x = F + 128, *F12y = F + 192;
    auto H = [&](int c1, int c2, int a, int b) -> int32_t & { return hist[((c1 * d2 + c2) * dx + a) * dy + b]; };
    auto I3 = [](int i, int j, int k) { return (i * 4 + j) * 4 + k; };
    for (int i = tid; i < 256; i += 256) F[i] = 0;  // (parts of the 3-way tables add atomically)
    __syncthreads();
    // the leading cells by popcount: static loops per (MX, MY, M2) (runtime guards inside unrolled
    // loops measured no faster than the histogram kernel: a branch per cell and word)
    switch (A.dbg & 1 ? -1 : MX * 16 + MY * 4 + M2) {  // (dbg bit 0: counting skipped, diagnostic)
#define FBN_L4(A_, B_, C_) \
    case A_ * 16 + B_ * 4 + C_: \
        lead4<A_, B_, C_>(px, py, p1, p2, W, M1, wv, lane, hist, d2, dx, dy, Fxy1, Fxy2, F12x, F12y); \
        break;
#define FBN_L4B(A_, B_) FBN_L4(A_, B_, 0) FBN_L4(A_, B_, 1) FBN_L4(A_, B_, 2) FBN_L4(A_, B_, 3)
#define FBN_L4A(A_) FBN_L4B(A_, 0) FBN_L4B(A_, 1) FBN_L4B(A_, 2) FBN_L4B(A_, 3)
        FBN_L4A(0) FBN_L4A(1) FBN_L4A(2) FBN_L4A(3)
#undef FBN_L4A
#undef FBN_L4B
#undef FBN_L4
    default: break;
    }
    __syncthreads();
    // the four 3-way tables, one per wave: G[i][j][k] over (vi, vj, vk) with dims (DI, DJ, DK)
    {
        const int t = wv;
        int vi, vj, vk;
        int32_t *G;
        if (t == 0) vi = z1, vj = x, vk = y, G = Fxy1;
        else if (t == 1) vi = z2, vj = x, vk = y, G = Fxy2;
        else if (t == 2) vi = z1, vj = z2, vk = x, G = F12x;
        else vi = z1, vj = z2, vk = y, G = F12y;
        const int DI = dims[vi], DJ = dims[vj], DK = dims[vk], MI = DI - 1, MJ = DJ - 1, MK = DK - 1;
        auto P = [&](int u, int a, int v, int b) { return pair_at(A.pairtab, A.nvars, dims, u, a, v, b); };
        // step 1: G[i][j][MK], i < MI, j < MJ
        if (lane < MI * MJ) {
            const int i = lane / MJ, j = lane % MJ;
            int32_t r = P(vi, i, vj, j);
            for (int k = 0; k < MK; ++k) r -= G[I3(i, j, k)];
            G[I3(i, j, MK)] = r;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done (one wave per table)
        __builtin_amdgcn_wave_barrier();
        // step 2: G[i][MJ][k], i < MI, every k
        if (lane < MI * DK) {
            const int i = lane / DK, k = lane % DK;
            int32_t r = P(vi, i, vk, k);
            for (int j = 0; j < MJ; ++j) r -= G[I3(i, j, k)];
            G[I3(i, MJ, k)] = r;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // step 3: G[MI][j][k], every j, k
        if (lane < DJ * DK) {
            const int j = lane / DK, k = lane % DK;
            int32_t r = P(vj, j, vk, k);
            for (int i = 0; i < MI; ++i) r -= G[I3(i, j, k)];
            G[I3(MI, j, k)] = r;
        }
    }
    __syncthreads();
    // the 4-way table T[c1][c2][a][b] from its leading cells and the 3-way tables (wave 0)
    if (wv == 0) {
        // step 1: T[c1][c2][a][MY] = F12x[c1][c2][a] - sum_b<MY
        if (lane < M1 * M2 * MX) {
            const int c1 = lane / (M2 * MX), c2 = (lane / MX) % M2, a = lane % MX;
            int32_t r = F12x[I3(c1, c2, a)];
            for (int b = 0; b < MY; ++b) r -= H(c1, c2, a, b);
            H(c1, c2, a, MY) = r;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // step 2: T[c1][c2][MX][b] = F12y[c1][c2][b] - sum_a<MX (every b)
        if (lane < M1 * M2 * dy) {
            const int c1 = lane / (M2 * dy), c2 = (lane / dy) % M2, b = lane % dy;
            int32_t r = F12y[I3(c1, c2, b)];
            for (int a = 0; a < MX; ++a) r -= H(c1, c2, a, b);
            H(c1, c2, MX, b) = r;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // step 3: T[c1][M2][a][b] = Fxy1[c1][a][b] - sum_c2<M2 (every a, b)
        if (lane < M1 * dx * dy) {
            const int c1 = lane / (dx * dy), a = (lane / dy) % dx, b = lane % dy;
            int32_t r = Fxy1[I3(c1, a, b)];
            for (int c2 = 0; c2 < M2; ++c2) r -= H(c1, c2, a, b);
            H(c1, M2, a, b) = r;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // step 4: T[M1][c2][a][b] = Fxy2[c2][a][b] - sum_c1<M1 (every c2, a, b: up to 64 cells)
        if (lane < d2 * dx * dy) {
            const int c2 = lane / (dx * dy), a = (lane / dy) % dx, b = lane % dy;
            int32_t r = Fxy2[I3(c2, a, b)];
            for (int c1 = 0; c1 < M1; ++c1) r -= H(c1, c2, a, b);
            H(M1, c2, a, b) = r;
        }
    }
}

// BITS: count from the bit-sliced store (A.bits); a separate instantiation, so the byte-column
// kernel keeps its register budget (74 VGPRs vs 178 with the bit-sliced counters compiled in).
// PK: count from the 2-bit packed columns (A.pk): a quarter of the byte columns' bytes, the same
// per-sample binning (one field extract per variable and sample, as the byte extract)
// MODE (2-bit packed columns only): 0 = one workgroup counts and decides a test; 1 = workgroup
// (t, part) counts part `part` of test t's packed words and adds its histogram into the global table
// of t; 2 = one workgroup per test reads the table and decides.  Small batches (the deep levels of
// config 5: 30-1056 tests of 100k samples each, one workgroup per test leaves most CUs idle) run as
// 1 then 2.  Counts are integers: the same in any order.
template <int D, bool BITS, bool PK = false, int BS = 256, int MODE = 0>
__global__ __launch_bounds__(BS, der2_waves(MODE)) void ci_g2_kernel(CiArgs A) {
    constexpr int NW = BS / 64;  // waves per workgroup (sub-histogram copies exist for 4 of them)
    extern __shared__ __align__(16) int32_t lds_base[];
    int32_t *smem = A.gscratch ? A.gscratch + (size_t)blockIdx.x * A.gstride : lds_base;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const long long nwork = MODE == 1 ? A.n * A.split : A.n;
    for (long long iw = blockIdx.x; iw < nwork; iw += gridDim.x) {
        const long long it = MODE == 1 ? iw / A.split : iw;
        const int part = MODE == 1 ? (int)(iw % A.split) : 0, nparts = MODE == 1 ? A.split : 1;
        const int32_t *item = A.items + it * (2 + D);
        const int x = item[0], y = item[1];
        const int dx = A.dims[x], dy = A.dims[y];
        int zv[D > 0 ? D : 1], cum[D > 0 ? D : 1];
        int dimz = 1;
#pragma unroll
        for (int j = D - 1; j >= 0; --j) {
            zv[j] = item[2 + j];
            cum[j] = dimz;  // last conditioning variable fastest (src/CellTable.cpp:39-51)
            dimz *= A.dims[zv[j]];
        }
        const int dxy = dx * dy;
        const int cells = dimz * dxy;
        // small tables (<= 16 cells): per-lane packed 16-bit counters in registers, no LDS traffic
        // in the sample loop; larger tables: LDS sub-histograms, kLanes per wave (lane l of wave w
        // adds into copy w * kl + l % kl): no cross-wave contention, and kl-fold fewer same-address
        // atomics within a wave on skewed tables (a popular cell's lanes serialize in one copy);
        // copies at an odd stride, so one cell's copies fall in different banks
        const bool packed = cells <= 16 && A.N <= (1ll << 24);
        const int kl = sub_lanes(cells);
        const int nsub = kl ? 4 * kl : 1;  // = fbn_ci_lds_bytes
        const int sstr = cells | 1;
        // LDS layout (ints): hist[cells] | sub[nsub][sstr] | ni | nj | nk | dfp | (even) term[tc] f64
        // (tc = min(cells, kTermChunk): the G^2 terms of one chunk of cells)
        const int tc = cells < kTermChunk ? cells : kTermChunk;
        int32_t *hist = smem;
        int32_t *sub = hist + ((cells + 3) & ~3);
        int32_t *ni = sub + (nsub > 1 ? nsub * sstr : 0);
        int32_t *nj = ni + dimz * dx;
        int32_t *nk = nj + dimz * dy;
        int32_t *dfp = nk + dimz;
        const int term_off = (int)((dfp + dimz) - smem + 1) & ~1;
        double *term = reinterpret_cast<double *>(smem + term_off);

        for (int c = tid; c < cells; c += BS) hist[c] = MODE == 2 ? A.tab[it * A.tstride + c] : 0;
        if (nsub > 1 && !BITS && MODE != 2)
            for (int c = tid; c < nsub * sstr; c += BS) sub[c] = 0;
        __syncthreads();
        if (BITS && MODE >= 3) {
            if constexpr (D == 2) derived4(A, x, y, zv[0], zv[1], dx, dy, hist, smem + term_off + 2 * tc, tid);
        } else if (BITS) {
            // bit-sliced counting: wave w takes the prefixes p = w, w + 4, ... of the z-configuration
            // (values of z_1 .. z_{d-1}; the last conditioning variable is the fastest digit, so
            // configuration k = p * dl + c for its value c).  Per 4-word step: m = AND of the prefix's
            // z rows, then for each value c of the last z (<= 4), every x value row ANDed with
            // m & z_last[c] and popcounted against every y value row -- the x, y and last-z rows are
            // loaded once per step for all dl configurations; one wave total per (k, cell)
            typedef __attribute__((ext_vector_type(4))) unsigned u4;
            const long long W = A.W;
            const uint32_t *px = A.bits + (size_t)A.row0[x] * W, *py = A.bits + (size_t)A.row0[y] * W;
            const int dl = A.dims[zv[D > 0 ? D - 1 : 0]];
            const uint32_t *pl = A.bits + (size_t)A.row0[zv[D > 0 ? D - 1 : 0]] * W;
            for (int pfx = tid >> 6; pfx < dimz / dl; pfx += NW) {
                const uint32_t *pz[D > 1 ? D - 1 : 1];
#pragma unroll
                for (int j = 0; j + 1 < D; ++j) {
                    const int v = (pfx * dl / cum[j]) % A.dims[zv[j]];
                    pz[j] = A.bits + (size_t)(A.row0[zv[j]] + v) * W;
                }
                uint32_t cnt[4][16];
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int e = 0; e < 16; ++e) cnt[c][e] = 0u;
                for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
                    u4 m = {~0u, ~0u, ~0u, ~0u};
#pragma unroll
                    for (int j = 0; j + 1 < D; ++j) m &= *reinterpret_cast<const u4 *>(pz[j] + 4 * w4);
                    u4 xv[4], yv[4], zl[4];
#pragma unroll
                    for (int a = 0; a < 4; ++a)
                        xv[a] = a < dx ? *reinterpret_cast<const u4 *>(px + a * W + 4 * w4) & m : u4{0u, 0u, 0u, 0u};
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        yv[b] = b < dy ? *reinterpret_cast<const u4 *>(py + b * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        zl[c] = c < dl ? *reinterpret_cast<const u4 *>(pl + c * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        if (c >= dl) continue;
#pragma unroll
                        for (int a = 0; a < 4; ++a) {
                            if (a >= dx) continue;
                            const u4 xm = xv[a] & zl[c];
#pragma unroll
                            for (int b = 0; b < 4; ++b) {
                                if (b >= dy) continue;
#pragma unroll
                                for (int q = 0; q < 4; ++q) cnt[c][a * 4 + b] += __builtin_popcount(xm[q] & yv[b][q]);
                            }
                        }
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int a = 0; a < 4; ++a)
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            if (c >= dl || a >= dx || b >= dy) continue;
                            uint32_t v = cnt[c][a * 4 + b];
#pragma unroll
                            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
                            if (lane == 0) hist[(pfx * dl + c) * dxy + a * dy + b] = (int32_t)v;
                        }
            }
        }
        if (!BITS && MODE != 2) {
        int32_t *myhist = nsub > 1 ? sub + (((tid >> 6) & 3) * kl + (lane & (kl - 1))) * sstr : hist;
        unsigned long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;  // cell c: a[c >> 2] bits [16 (c & 3), +16)
        auto bin = [&](int cell, bool valid) {
            if (packed) {
                const unsigned long long inc = valid ? (1ull << ((cell & 3) << 4)) : 0ull;
                const int q = cell >> 2;
                a0 += q == 0 ? inc : 0ull;
                a1 += q == 1 ? inc : 0ull;
                a2 += q == 2 ? inc : 0ull;
                a3 += q == 3 ? inc : 0ull;
            } else if (valid) {
                atomicAdd(&myhist[cell], 1);
            }
        };
        if (PK) {
            // full words (16 samples each) unchecked, kU in flight per thread; the tail word's
            // samples beyond N (zero padding) excluded
            const uint32_t *px = A.pk + (size_t)x * A.PW, *py = A.pk + (size_t)y * A.PW;
            const uint32_t *pz[D > 0 ? D : 1];
#pragma unroll
            for (int j = 0; j < D; ++j) pz[j] = A.pk + (size_t)zv[j] * A.PW;
            const long long full = A.N / 16;
            // this workgroup's words [w0, w1) (all of them unless MODE 1)
            const long long w0 = full * part / nparts, w1 = full * (part + 1) / nparts;
            auto bin16 = [&](uint32_t wx, uint32_t wy, const uint32_t *wz, int lim) {
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    int zi = 0;
#pragma unroll
                    for (int j = 0; j < D; ++j) zi += (int)((wz[j] >> (2 * s)) & 3u) * cum[j];
                    const int cell = (zi * dx + (int)((wx >> (2 * s)) & 3u)) * dy + (int)((wy >> (2 * s)) & 3u);
                    bin(s < lim ? cell : 0, s < lim);
                }
            };
            constexpr int kU = 2;
            for (long long kb = w0 + tid; kb < w1; kb += BS * kU) {
                uint32_t wx[kU], wy[kU], wz[kU][D > 0 ? D : 1];
                bool v[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const long long k = kb + u * BS;
                    v[u] = k < w1;
                    const long long kk = v[u] ? k : 0;
                    wx[u] = px[kk], wy[u] = py[kk];
#pragma unroll
                    for (int j = 0; j < D; ++j) wz[u][j] = pz[j][kk];
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) bin16(wx[u], wy[u], wz[u], v[u] ? 16 : 0);
            }
            if (A.N % 16 && tid == 0 && part == nparts - 1) {
                uint32_t wz[D > 0 ? D : 1];
#pragma unroll
                for (int j = 0; j < D; ++j) wz[j] = pz[j][full];
                bin16(px[full], py[full], wz, (int)(A.N % 16));
            }
        } else {
        const uint8_t *cx = A.cols + (size_t)x * A.N;
        const uint8_t *cy = A.cols + (size_t)y * A.N;
        const uint8_t *cz[D > 0 ? D : 1];
#pragma unroll
        for (int j = 0; j < D; ++j) cz[j] = A.cols + (size_t)zv[j] * A.N;

        const long long N4 = (A.N % 4 == 0) ? A.N / 4 : 0;
        // kU words per column in flight per thread: one memory latency per kU steps, not per step
        constexpr int kU = 4;
        for (long long kb = tid; kb < N4; kb += BS * kU) {
            uint32_t wx[kU], wy[kU], wz[kU][D > 0 ? D : 1];
            bool v4[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const long long k4 = kb + u * BS;
                v4[u] = k4 < N4;
                const long long kk = v4[u] ? k4 : 0;
                wx[u] = reinterpret_cast<const uint32_t *>(cx)[kk];
                wy[u] = reinterpret_cast<const uint32_t *>(cy)[kk];
#pragma unroll
                for (int j = 0; j < D; ++j) wz[u][j] = reinterpret_cast<const uint32_t *>(cz[j])[kk];
            }
#pragma unroll
            for (int u = 0; u < kU; ++u)
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    int zi = 0;
#pragma unroll
                    for (int j = 0; j < D; ++j) zi += (int)((wz[u][j] >> (8 * s)) & 0xFF) * cum[j];
                    const int cell =
                        (zi * dx + (int)((wx[u] >> (8 * s)) & 0xFF)) * dy + (int)((wy[u] >> (8 * s)) & 0xFF);
                    bin(v4[u] ? cell : 0, v4[u]);
                }
        }
        for (long long k = 4 * N4 + tid; k < ((A.N - 4 * N4 + BS - 1) / BS) * BS + 4 * N4; k += BS) {
            const bool v = k < A.N;
            int cell = 0;
            if (v) {
                int zi = 0;
#pragma unroll
                for (int j = 0; j < D; ++j) zi += (int)cz[j][k] * cum[j];
                cell = (zi * dx + cx[k]) * dy + cy[k];
            }
            bin(cell, v);
        }
        }  // byte / 2-bit columns
        if (packed) {  // wave reduction of the packed counters, one LDS add per cell per wave
            for (int c = 0; c < cells; ++c) {
                const unsigned long long w = (c >> 2) == 0 ? a0 : (c >> 2) == 1 ? a1 : (c >> 2) == 2 ? a2 : a3;
                int v = (int)((w >> ((c & 3) << 4)) & 0xFFFFull);
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
                if (lane == 0 && v) atomicAdd(&hist[c], v);
            }
        }
        }  // !BITS
        __syncthreads();
        if (nsub > 1 && !BITS && MODE != 2) {
            for (int c = tid; c < cells; c += BS) {
                int v = 0;
                for (int w = 0; w < nsub; ++w) v += sub[w * sstr + c];
                hist[c] = v;
            }
            __syncthreads();
        }
        if (MODE == 1) {  // this part's counts into the test's global table
            for (int c = tid; c < cells; c += BS)
                if (hist[c]) atomicAdd(&A.tab[it * A.tstride + c], hist[c]);
            __syncthreads();  // LDS reused by the next work item
            continue;
        }
        if (A.counts && (A.cstride > 0 || it == 0))
            for (int c = tid; c < cells; c += BS) A.counts[it * A.cstride + c] = hist[c];

        // marginals N_{x+z}, N_{+yz}, N_{++z} (src/CellTable.cpp:242-250)
        for (int r = tid; r < dimz * dx; r += BS) {
            const int k = r / dx, i = r % dx;
            int s = 0;
            for (int j = 0; j < dy; ++j) s += hist[k * dxy + i * dy + j];
            ni[r] = s;
        }
        for (int r = tid; r < dimz * dy; r += BS) {
            const int k = r / dy, j = r % dy;
            int s = 0;
            for (int i = 0; i < dx; ++i) s += hist[k * dxy + i * dy + j];
            nj[r] = s;
        }
        __syncthreads();
        // N_{++z} and the adjusted df per z (src/IndependenceTest.cpp:96-112)
        for (int k = tid; k < dimz; k += BS) {
            int alx = 0, aly = 0, total = 0;
            for (int i = 0; i < dx; ++i) alx += ni[k * dx + i] > 0, total += ni[k * dx + i];
            for (int j = 0; j < dy; ++j) aly += nj[k * dy + j] > 0;
            alx = alx >= 1 ? alx : 1;
            aly = aly >= 1 ? aly : 1;
            dfp[k] = (alx - 1) * (aly - 1);
            nk[k] = total;
        }
        __syncthreads();
        // decision-only batches (no G^2 / p returned, band present): the terms summed as a block tree
        // first.  Tree and in-order sums of the same terms differ by at most (cells + 64) u sum|t|, so
        // a tree sum that clears the band [lo, hi] by that much decides exactly as the reference's
        // ordered sum would (past the band's df range: p at both ends of that interval); only the
        // rest (near alpha) add in order below.
        auto term_of = [&](int c) {
            const int k = c / dxy, i = (c / dy) % dx, j = c % dy;
            const long total = nk[k], sum_row = ni[k * dx + i], sum_col = nj[k * dy + j], observed = hist[c];
            double t = 0.0;
            if (total != 0 && sum_row != 0 && sum_col != 0 && observed != 0) {
                const double expected = (double)sum_col * (double)sum_row / (double)total;
                t = 2.0 * observed * log(observed / expected);
            }
            return t;
        };
        __shared__ double sred[2 * NW];
        __shared__ int sdf[NW], sdec;
        if (!A.p && !A.g2 && A.band) {
            double ps = 0.0, pa = 0.0;
            int pdf = 0;
            for (int c = tid; c < cells; c += BS) {
                const double t = term_of(c);
                ps += t;
                pa += fabs(t);
            }
            for (int k = tid; k < dimz; k += BS) pdf += dfp[k];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                ps += __shfl_xor(ps, o);
                pa += __shfl_xor(pa, o);
                pdf += __shfl_xor(pdf, o);
            }
            if (lane == 0) sred[2 * (tid >> 6)] = ps, sred[2 * (tid >> 6) + 1] = pa, sdf[tid >> 6] = pdf;
            __syncthreads();
            if (tid == 0) {
                double gs = (sred[0] + sred[2]) + (sred[4] + sred[6]);
                double ga = (sred[1] + sred[3]) + (sred[5] + sred[7]);
                int df = sdf[0] + sdf[1] + sdf[2] + sdf[3];
#pragma unroll
                for (int w = 4; w < NW; ++w) gs += sred[2 * w], ga += sred[2 * w + 1], df += sdf[w];
                const double err = (cells + 64) * 2.3e-16 * ga;
                int dec = -1;  // 0 dependent, 1 independent, -1 in-order sum
                double pd = -1.0;  // p of a decision past the band's df range
                if (df == 0) dec = 1;  // src/IndependenceTest.cpp:140-142
                else if (df <= A.nband && gs + err < A.band[2 * df - 2]) dec = 1;
                else if (df <= A.nband && gs - err > A.band[2 * df - 1]) dec = 0;
                else if (df > A.nband) {
                    // p decreases in G^2 and the in-order sum lies in [gs - err, gs + err]: p at
                    // both ends on the same side of alpha (by a relative 1e-12 more than the
                    // evaluation's own rounding) decides as the in-order sum would
                    const double phi = fbn_chisq_pvalue(gs - err > 0.0 ? gs - err : 0.0, df), plo = fbn_chisq_pvalue(gs + err, df);
                    if (plo > A.alpha * (1.0 + 1e-12)) dec = 1, pd = plo;
                    else if (phi < A.alpha * (1.0 - 1e-12)) dec = 0, pd = phi;
                }
                if (dec >= 0) {
                    const double p = df == 0 ? 1.0 : pd >= 0.0 ? pd
                                                 : dec ? A.alpha + A.band[2 * A.nband] : A.alpha - A.band[2 * A.nband];
                    if (A.df) A.df[it] = df;
                    if (A.indep) A.indep[it] = dec;
                    if (A.stats) {
                        const double m = fabs(p - A.alpha);
                        atomicMin(A.stats, (unsigned long long)__double_as_longlong(m));
                        if (m < 1e-9) atomicAdd(A.stats + 1, 1ull);
                    }
                }
                sdec = dec;
            }
            __syncthreads();
            const bool done = sdec >= 0;
            __syncthreads();  // sdec / sred reused by the next test
            if (done) continue;
        }
        // G^2: the terms of a chunk of cells in parallel (cell c = (k * dx + i) * dy + j, the
        // reference's loop order), then one lane adds them in order (src/IndependenceTest.cpp:112-137)
        double g2 = 0.0;
        for (int c0 = 0; c0 < cells; c0 += tc) {
            const int c1 = c0 + tc < cells ? c0 + tc : cells;
            for (int c = c0 + tid; c < c1; c += BS) term[c - c0] = term_of(c);
            __syncthreads();
            if (tid == 0) {  // loads batched ahead of the dependent adds (LDS latency off the chain)
                const int m = c1 - c0;
                int c = 0;
                for (; c + 8 <= m; c += 8) {
                    double t[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) t[u] = term[c + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) g2 += t[u];
                }
                for (; c < m; ++c) g2 += term[c];
            }
            __syncthreads();
        }
        if (tid == 0) {
            int df = 0;
            for (int k = 0; k < dimz; ++k) df += dfp[k];
            double p;
            bool ind;
            if (df == 0) {  // src/IndependenceTest.cpp:140-142, 349-351
                p = 1.0;
                ind = true;
            } else if (!A.p && A.band && df <= A.nband && g2 < A.band[2 * df - 2]) {
                p = A.alpha + A.band[2 * A.nband];  // p > alpha + delta: logged as margin delta
                ind = true;
            } else if (!A.p && A.band && df <= A.nband && g2 > A.band[2 * df - 1]) {
                p = A.alpha - A.band[2 * A.nband];
                ind = false;
            } else {
                p = fbn_chisq_pvalue(g2, df);
                ind = p > A.alpha;
            }
            if (A.g2) A.g2[it] = g2;
            if (A.df) A.df[it] = df;
            if (A.p) A.p[it] = p;
            if (A.indep) A.indep[it] = ind;
            if (A.stats) {
                const double m = fabs(p - A.alpha);
                atomicMin(A.stats, (unsigned long long)__double_as_longlong(m));
                if (m < 1e-9) atomicAdd(A.stats + 1, 1ull);
            }
        }
        __syncthreads();
    }
}

}  // namespace

// LDS bytes needed for a test with `cells` = dimz*dx*dy
extern "C" size_t fbn_ci_lds_bytes(int dimz, int dx, int dy) {
    // must match the kernel's layout
    const size_t cells = (size_t)dimz * dx * dy;
    const size_t kl = cells > (1u << 30) ? 0 : sub_lanes((int)cells);
    const size_t nsub = 4 * kl;
    size_t ints = ((cells + 3) & ~(size_t)3) + nsub * (cells | 1) + (size_t)dimz * (dx + dy + 2);
    ints = (ints + 1) & ~(size_t)1;
    return ints * 4 + std::min<size_t>(cells, kTermChunk) * 8 + kDerivedInts * 4;
}

extern "C" hipError_t fbn_ci_launch(const uint8_t *cols, const int32_t *dims, const int32_t *items, long long N,
                                    long long n, int d, double alpha, double *g2, int32_t *df, double *p,
                                    uint8_t *indep, int32_t *counts, size_t lds_bytes, int grid,
                                    int32_t *gscratch, unsigned long long *stats, const uint32_t *bits,
                                    const int32_t *row0, long long W, const double *band, int nband,
                                    const uint32_t *pk, long long PW, long long cstride, int32_t *tab,
                                    long long tstride, int split, int split_grid, const int32_t *pairtab, int nvars,
                                    hipStream_t stream) {
    CiArgs a{cols, dims, items, N, n, alpha, g2, df, p, indep, counts, gscratch, (long long)(lds_bytes / 4 + 1) & ~1ll,
             stats, bits, row0, W, band, nband, pk, PW, cstride, tab, tstride, split, pairtab, nvars,
             getenv("FBN_CI_DER2_DBG") ? atoi(getenv("FBN_CI_DER2_DBG")) : 0};
    if (gscratch) lds_bytes = 0;
    if (pairtab && bits && d == 2) {  // MODE 3: derived bit-sliced counting (every state count <= 4)
        // registers for 3 waves per SIMD (config-5 level 2: 0.47 / 0.42 / 0.49 ms at 2 / 3 / 4 waves;
        // FBN_CI_DER2_WAVES = 2 selects the unconstrained allocation)
        static const int w = getenv("FBN_CI_DER2_WAVES") ? atoi(getenv("FBN_CI_DER2_WAVES")) : 3;
        if (w == 2) hipLaunchKernelGGL((ci_g2_kernel<2, true, false, 256, 3>), dim3(grid), dim3(256), lds_bytes, stream, a);
        else hipLaunchKernelGGL((ci_g2_kernel<2, true, false, 256, 4>), dim3(grid), dim3(256), lds_bytes, stream, a);
        return hipGetLastError();
    }
    if (split > 1 && pk && !bits && !gscratch) {  // small batch: count in parts, then decide
        hipError_t e = hipMemsetAsync(tab, 0, (size_t)n * tstride * 4, stream);
        if (e != hipSuccess) return e;
        switch (d) {
#define FBN_CI_SPLIT(DD)                                                                                      \
    case DD:                                                                                                  \
        hipLaunchKernelGGL((ci_g2_kernel<DD, false, true, 256, 1>), dim3(split_grid), dim3(256), lds_bytes, stream, a); \
        hipLaunchKernelGGL((ci_g2_kernel<DD, false, true, 1024, 2>), dim3(grid), dim3(1024), lds_bytes, stream, a); \
        break;
            FBN_CI_SPLIT(0)
            FBN_CI_SPLIT(1)
            FBN_CI_SPLIT(2)
            FBN_CI_SPLIT(3)
            FBN_CI_SPLIT(4)
            FBN_CI_SPLIT(5)
            FBN_CI_SPLIT(6)
            FBN_CI_SPLIT(7)
            FBN_CI_SPLIT(8)
#undef FBN_CI_SPLIT
        default:
            return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    // batches of at most kWideTests tests (deep PC levels: a few hundred tests or fewer, one
    // workgroup per test on part of the chip): 16 waves per test instead of 4, so each test's
    // sample loop and epilogue have 4x the waves to hide latency (FBN_CI_NO_WIDE: always 4)
    static const bool no_wide = getenv("FBN_CI_NO_WIDE") != nullptr;
    const bool wide = n <= kWideTests && !no_wide;
    switch (d) {
#define FBN_CI_CASE(DD)                                                                              \
    case DD:                                                                                         \
        if (bits && DD >= 2)                                                                         \
            hipLaunchKernelGGL((ci_g2_kernel<DD, true>), dim3(grid), dim3(256), lds_bytes, stream, a);  \
        else if (wide && pk)                                                                         \
            hipLaunchKernelGGL((ci_g2_kernel<DD, false, true, 1024>), dim3(grid), dim3(1024), lds_bytes, stream, a); \
        else if (wide)                                                                               \
            hipLaunchKernelGGL((ci_g2_kernel<DD, false, false, 1024>), dim3(grid), dim3(1024), lds_bytes, stream, a); \
        else if (pk)                                                                                 \
            hipLaunchKernelGGL((ci_g2_kernel<DD, false, true>), dim3(grid), dim3(256), lds_bytes, stream, a); \
        else                                                                                         \
            hipLaunchKernelGGL((ci_g2_kernel<DD, false>), dim3(grid), dim3(256), lds_bytes, stream, a); \
        break;
        FBN_CI_CASE(0)
        FBN_CI_CASE(1)
        FBN_CI_CASE(2)
        FBN_CI_CASE(3)
        FBN_CI_CASE(4)
        FBN_CI_CASE(5)
        FBN_CI_CASE(6)
        FBN_CI_CASE(7)
        FBN_CI_CASE(8)
#undef FBN_CI_CASE
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the 2-bit packed column store: word w of variable v holds samples 16w .. 16w + 15 (sample 16w + s
// in bits 2s, 2s + 1); samples past N are zero (the kernel excludes them)
__global__ __launch_bounds__(256) void ci_pack2_build(const uint8_t *__restrict__ cols, long long N, long long PW,
                                                      long long total, uint32_t *__restrict__ pk) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
        const long long v = i / PW, w = i % PW;
        const uint8_t *c = cols + v * N + 16 * w;
        const long long left = N - 16 * w;
        uint32_t r = 0;
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (s < left) r |= (uint32_t)(c[s] & 3u) << (2 * s);
        pk[i] = r;
    }
}

extern "C" hipError_t fbn_ci_pack2_build(const uint8_t *cols, int nvars, long long N, long long PW, uint32_t *pk,
                                         hipStream_t stream) {
    const long long total = (long long)nvars * PW;
    const int grid = (int)std::min<long long>((total + 255) / 256, 65536);
    if (total > 0) hipLaunchKernelGGL(ci_pack2_build, dim3(grid), dim3(256), 0, stream, cols, N, PW, total, pk);
    return hipGetLastError();
}
