// ci_bits.hip -- G^2 tests with at most one conditioning variable on bit-sliced columns, gfx950.
//
// The level-0 sweep tests every pair of variables (499,500 tests at 1000 variables), each a
// 2-D contingency table N[x][y] over all samples (Counts2D::FillTable, src/CellTable.cpp:430-455).
// Instead of re-reading two byte columns and binning sample by sample, every column is stored
// once as one bit mask per value (bit s of mask (v, a) = [sample s of v has value a], 32 samples
// per word): N[a][b] = sum over words of popcount(mask(x, a) & mask(y, b)).  One wave per test,
// lanes stride over the words, one v_bcnt (popcount + accumulate) per cell per 32 samples; the
// masks are 1/8 of the byte columns per value (HBM / Infinity-cache traffic per test: (dx + dy
// [+ dz]) rows of N/8 bytes), counts are exact integers.  Level 1 (one conditioning variable z)
// adds z's masks: N[c][a][b] = sum popcount(x_a & y_b & z_c) (Counts3D, src/CellTable.cpp:226-291).
//
// Phase 2 evaluates marginals, the adjusted df and G^2 with one lane per test (no idle lanes in
// the log / incomplete-gamma code), in the reference's operation order (one running G^2 sum):
// ComputeGSquareXY,
// src/IndependenceTest.cpp:295-364 (same arithmetic as ci_kernels.hip, so the two kernels agree
// bit for bit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdlib.h>

#include "ci_chisq.h"


namespace {

// bits[(row0[v] + a) * W + w]: samples 32w .. 32w+31 of variable v equal to a
__global__ __launch_bounds__(256) void ci_bits_build(const uint8_t *__restrict__ cols, const int32_t *__restrict__ dims,
                                                     const int32_t *__restrict__ row0, long long N, long long W,
                                                     int nvars, uint32_t *__restrict__ bits) {
    const long long total = (long long)nvars * W;
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
        const int v = (int)(t / W);
        const long long w = t % W;
        const uint8_t *c = cols + (size_t)v * N + 32 * w;
        const int n = (int)((N - 32 * w) < 32 ? (N - 32 * w) : 32);
        uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int d = dims[v];
        for (int s = 0; s < n; ++s) {
            const int a = c[s];
#pragma unroll
            for (int k = 0; k < 8; ++k) m[k] |= (a == k ? 1u : 0u) << s;
        }
        for (int a = 0; a < d; ++a) bits[(size_t)(row0[v] + a) * W + w] = m[a];
    }
}

// counts of one test: N[z][a][b] += popcount(x_a & y_b & z_c) over this lane's words, then a
// wave reduction; cells (c * DX + a) * DY + b (Counts3D layout, src/CellTable.cpp:277-281).
// DZ = 1 for marginal tests; conditional tests (one conditioning variable) use DZ = 4 with the
// masks of absent values zero (their cells stay 0 and are never read).
template <int DX, int DY, int DZ>
__device__ __forceinline__ void count_test(const uint32_t *__restrict__ bx, const uint32_t *__restrict__ by,
                                           const uint32_t *__restrict__ bz, int dz, long long W, int lane,
                                           int32_t *__restrict__ out) {
    constexpr int NC = DX * DY * DZ;
    uint32_t cnt[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) cnt[c] = 0u;
    // four consecutive words per lane per step, one 16-byte load per mask row (W is a multiple
    // of 4, padding words are zero)
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    auto quad = [&](long long w4) {
        u4 x[DX], y[DY], z[DZ];
#pragma unroll
        for (int a = 0; a < DX; ++a) x[a] = *reinterpret_cast<const u4 *>(bx + a * W + 4 * w4);
#pragma unroll
        for (int b = 0; b < DY; ++b) y[b] = *reinterpret_cast<const u4 *>(by + b * W + 4 * w4);
#pragma unroll
        for (int c = 0; c < DZ; ++c) {
            if (DZ == 1) z[c] = u4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            else z[c] = c < dz ? *reinterpret_cast<const u4 *>(bz + c * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int a = 0; a < DX; ++a)
#pragma unroll
                for (int b = 0; b < DY; ++b) {
                    const uint32_t xy = x[a][k] & y[b][k];
#pragma unroll
                    for (int c = 0; c < DZ; ++c) cnt[(c * DX + a) * DY + b] += __builtin_popcount(xy & z[c][k]);
                }
    };
    for (long long w4 = lane; 4 * w4 < W; w4 += 64) quad(w4);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        uint32_t v = cnt[c];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        cnt[c] = v;
    }
    const int ncells = DX * DY * (DZ == 1 ? 1 : dz);
    if (lane < ncells) {
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) v = lane == c ? cnt[c] : v;
        out[lane] = (int32_t)v;
    }
}

// marginal test N[a][b] (Counts2D::FillTable, src/CellTable.cpp:430-455) from (DX-1)(DY-1)
// popcounts per word: the masks of a variable partition the samples, so the last value's row and
// column follow exactly from the per-value sample counts nx / ny of x and y (test-independent,
// ci_bits_rowcount) -- N[a][DY-1] = nx[a] - sum_b N[a][b], N[DX-1][b] = ny[b] - sum_a N[a][b];
// only DX-1 and DY-1 mask rows are read
template <int DX, int DY>
__device__ __forceinline__ void count_pair(const uint32_t *__restrict__ bx, const uint32_t *__restrict__ by,
                                           const int32_t *__restrict__ nx, const int32_t *__restrict__ ny,
                                           long long W, int lane, int32_t *__restrict__ out,
                                           int32_t *__restrict__ rec) {
    constexpr int MX = DX - 1, MY = DY - 1, NC = MX * MY > 0 ? MX * MY : 1;
    uint32_t cnt[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) cnt[c] = 0u;
    if (MX > 0 && MY > 0) {
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
            u4 x[MX > 0 ? MX : 1], y[MY > 0 ? MY : 1];
#pragma unroll
            for (int a = 0; a < MX; ++a) x[a] = *reinterpret_cast<const u4 *>(bx + a * W + 4 * w4);
#pragma unroll
            for (int b = 0; b < MY; ++b) y[b] = *reinterpret_cast<const u4 *>(by + b * W + 4 * w4);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int a = 0; a < MX; ++a)
#pragma unroll
                    for (int b = 0; b < MY; ++b) cnt[a * MY + b] += __builtin_popcount(x[a][k] & y[b][k]);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint32_t v = cnt[c];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            cnt[c] = v;
        }
    }
    // every lane now holds the wave totals: complete the table with the marginals
    int32_t full[DX * DY];
#pragma unroll
    for (int a = 0; a < MX; ++a) {
        int32_t r = nx[a];
#pragma unroll
        for (int b = 0; b < MY; ++b) full[a * DY + b] = (int32_t)cnt[a * MY + b], r -= (int32_t)cnt[a * MY + b];
        full[a * DY + MY] = r;
    }
#pragma unroll
    for (int b = 0; b < DY; ++b) {
        int32_t r = ny[b];
#pragma unroll
        for (int a = 0; a < MX; ++a) r -= full[a * DY + b];
        full[MX * DY + b] = r;
    }
    if (lane < DX * DY) {
        int32_t v = 0;
#pragma unroll
        for (int c = 0; c < DX * DY; ++c) v = lane == c ? full[c] : v;
        out[lane] = v;
        if (rec) rec[lane] = v;
    }
}

// conditional test N[c][a][b] (one conditioning variable z) from (DZ-1)(DX-1)(DY-1) popcounts per
// word: the pair tables N_xy, N_xz, N_yz this run's level 0 recorded (every pair of the complete
// graph, table of (u < v) stored [value of u][value of v]) give the last value of each variable
// exactly -- N[c][a][DY-1] = N_xz[a][c] - sum_b, N[c][DX-1][b] = N_yz[b][c] - sum_a,
// N[DZ-1][a][b] = N_xy[a][b] - sum_c; only DX-1, DY-1, DZ-1 mask rows are read
template <int DX, int DY, int DZ>
__device__ __forceinline__ void derived_finish(uint32_t (&cnt)[(DX - 1) * (DY - 1) * (DZ - 1) > 0 ? (DX - 1) * (DY - 1) * (DZ - 1) : 1],
                                               const int32_t *__restrict__ Txy, bool txy,
                                               const int32_t *__restrict__ Txz, bool txz,
                                               const int32_t *__restrict__ Tyz, bool tyz,
                                               int32_t (&full)[DZ * DX * DY]);
template <int DX, int DY, int DZ>
__device__ __forceinline__ void count_test_derived_full(const uint32_t *__restrict__ bx,
                                                        const uint32_t *__restrict__ by,
                                                        const uint32_t *__restrict__ bz, long long W, int lane,
                                                        const int32_t *__restrict__ Txy, bool txy,
                                                        const int32_t *__restrict__ Txz, bool txz,
                                                        const int32_t *__restrict__ Tyz, bool tyz,
                                                        int32_t (&full)[DZ * DX * DY]) {
    constexpr int MX = DX - 1, MY = DY - 1, MZ = DZ - 1, M = MX * MY * MZ, NC = M > 0 ? M : 1;
    uint32_t cnt[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) cnt[c] = 0u;
    if (M > 0) {
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
            u4 x[MX > 0 ? MX : 1], y[MY > 0 ? MY : 1], z[MZ > 0 ? MZ : 1];
#pragma unroll
            for (int a = 0; a < MX; ++a) x[a] = *reinterpret_cast<const u4 *>(bx + a * W + 4 * w4);
#pragma unroll
            for (int b = 0; b < MY; ++b) y[b] = *reinterpret_cast<const u4 *>(by + b * W + 4 * w4);
#pragma unroll
            for (int c = 0; c < MZ; ++c) z[c] = *reinterpret_cast<const u4 *>(bz + c * W + 4 * w4);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int a = 0; a < MX; ++a)
#pragma unroll
                    for (int b = 0; b < MY; ++b) {
                        const uint32_t xy = x[a][k] & y[b][k];
#pragma unroll
                        for (int c = 0; c < MZ; ++c) cnt[(c * MX + a) * MY + b] += __builtin_popcount(xy & z[c][k]);
                    }
        }
    }
    derived_finish<DX, DY, DZ>(cnt, Txy, txy, Txz, txz, Tyz, tyz, full);
}

// the wave totals of the leading cells (butterfly) and the derived rest of the table
template <int DX, int DY, int DZ>
__device__ __forceinline__ void derived_finish(uint32_t (&cnt)[(DX - 1) * (DY - 1) * (DZ - 1) > 0 ? (DX - 1) * (DY - 1) * (DZ - 1) : 1],
                                               const int32_t *__restrict__ Txy, bool txy,
                                               const int32_t *__restrict__ Txz, bool txz,
                                               const int32_t *__restrict__ Tyz, bool tyz,
                                               int32_t (&full)[DZ * DX * DY]) {
    constexpr int MX = DX - 1, MY = DY - 1, MZ = DZ - 1, M = MX * MY * MZ, NC = M > 0 ? M : 1;
    if (M > 0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint32_t v = cnt[c];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            cnt[c] = v;
        }
    }
    auto nxy = [&](int a, int b) { return txy ? Txy[b * DX + a] : Txy[a * DY + b]; };
    auto nxz = [&](int a, int c) { return txz ? Txz[c * DX + a] : Txz[a * DZ + c]; };
    auto nyz = [&](int b, int c) { return tyz ? Tyz[c * DY + b] : Tyz[b * DZ + c]; };
#pragma unroll
    for (int c = 0; c < MZ; ++c) {
#pragma unroll
        for (int a = 0; a < MX; ++a) {
            int32_t r = nxz(a, c);
#pragma unroll
            for (int b = 0; b < MY; ++b) {
                const int32_t v = (int32_t)cnt[(c * MX + a) * MY + b];
                full[(c * DX + a) * DY + b] = v;
                r -= v;
            }
            full[(c * DX + a) * DY + MY] = r;
        }
#pragma unroll
        for (int b = 0; b < DY; ++b) {
            int32_t r = nyz(b, c);
#pragma unroll
            for (int a = 0; a < MX; ++a) r -= full[(c * DX + a) * DY + b];
            full[(c * DX + MX) * DY + b] = r;
        }
    }
#pragma unroll
    for (int a = 0; a < DX; ++a)
#pragma unroll
        for (int b = 0; b < DY; ++b) {
            int32_t r = nxy(a, b);
#pragma unroll
            for (int c = 0; c < MZ; ++c) r -= full[(c * DX + a) * DY + b];
            full[(MZ * DX + a) * DY + b] = r;
        }
}

template <int DX, int DY, int DZ>
__device__ __forceinline__ void count_test_derived(const uint32_t *__restrict__ bx, const uint32_t *__restrict__ by,
                                                   const uint32_t *__restrict__ bz, long long W, int lane,
                                                   int32_t *__restrict__ out, const int32_t *__restrict__ Txy, bool txy,
                                                   const int32_t *__restrict__ Txz, bool txz,
                                                   const int32_t *__restrict__ Tyz, bool tyz) {
    int32_t full[DZ * DX * DY];
    count_test_derived_full<DX, DY, DZ>(bx, by, bz, W, lane, Txy, txy, Txz, txz, Tyz, tyz, full);
    if (lane < DZ * DX * DY) {
        int32_t v = 0;
#pragma unroll
        for (int c = 0; c < DZ * DX * DY; ++c) v = lane == c ? full[c] : v;
        out[lane] = v;
    }
}

// items == nullptr for a marginal batch: test t is the (t0 + t)-th pair (x < y) of the complete graph
// over nv variables in lexicographic order (a PC run's level 0, or one rank's range of it), decoded
// instead of read
__device__ __forceinline__ void pair_of(long long t, int nv, int &x, int &y) {
    const double b = 2.0 * nv - 1.0;
    long long i = (long long)((b - sqrt(b * b - 8.0 * (double)t)) * 0.5);
    auto off = [&](long long r) { return r * nv - r * (r + 1) / 2; };
    if (i < 0) i = 0;
    while (i > 0 && off(i) > t) --i;
    while (i + 1 < nv && off(i + 1) <= t) ++i;
    x = (int)i;
    y = (int)(t - off(i) + i + 1);
}

constexpr int kBitsCells = 64;  // count slots per test

// ---- register-blocked marginal tests (a PC run's level 0, all pairs of a pair-index range)
// One wave per task = a block of BX x-variables x BY y-variables of one state-count class each
// (tasks built on the host, CiPairTasks in capi.hip): per 4-word step every mask row of the block's
// variables is loaded once and feeds every pair of the block, so L2 / fabric traffic per pair drops
// from (dx-1 + dy-1) rows to (BX (dx-1) + BY (dy-1)) / (BX BY) rows.  A pair is the block's
// (x, y) with x < y and its index in [t0, t1) (each pair of the range exactly once); the counts
// and the derived last row / column are exactly count_pair's (Counts2D, src/CellTable.cpp:430-455).
template <int DX, int DY>
struct PairBlock {
    static constexpr int MX = DX - 1, MY = DY - 1;
    static constexpr int BX = MX <= 1 ? 4 : (MX == 2 ? 3 : 2), BY = MY <= 1 ? 4 : (MY == 2 ? 3 : 2);
    static constexpr int NCC = MX * MY > 0 ? MX * MY : 1;
};
constexpr int kPairTaskInts = 12;  // dx, dy, nx, ny, xs[4], ys[4]

template <int DX, int DY>
__device__ __forceinline__ void pair_block(const uint32_t *__restrict__ bits, const int32_t *__restrict__ row0,
                                           const int32_t *__restrict__ rowcnt, long long W,
                                           const int32_t *__restrict__ task, int nvars, long long t0, long long t1,
                                           int32_t *__restrict__ counts, int32_t *__restrict__ pairtab, int lane) {
    using PB = PairBlock<DX, DY>;
    constexpr int MX = PB::MX, MY = PB::MY, BX = PB::BX, BY = PB::BY, NCC = PB::NCC;
    const int nx = task[2], ny = task[3];
    int xs[BX], ys[BY];
#pragma unroll
    for (int a = 0; a < BX; ++a) xs[a] = task[4 + (a < nx ? a : 0)];  // padding repeats the first
#pragma unroll
    for (int b = 0; b < BY; ++b) ys[b] = task[8 + (b < ny ? b : 0)];
    uint32_t cnt[BX][BY][NCC];
#pragma unroll
    for (int a = 0; a < BX; ++a)
#pragma unroll
        for (int b = 0; b < BY; ++b)
#pragma unroll
            for (int c = 0; c < NCC; ++c) cnt[a][b][c] = 0u;
    if (MX > 0 && MY > 0) {
        typedef __attribute__((ext_vector_type(4))) unsigned u4;
        const uint32_t *px[BX], *py[BY];
#pragma unroll
        for (int a = 0; a < BX; ++a) px[a] = bits + (size_t)row0[xs[a]] * W;
#pragma unroll
        for (int b = 0; b < BY; ++b) py[b] = bits + (size_t)row0[ys[b]] * W;
        for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
            u4 xv[BX][MX > 0 ? MX : 1], yv[BY][MY > 0 ? MY : 1];
#pragma unroll
            for (int a = 0; a < BX; ++a)
#pragma unroll
                for (int r = 0; r < MX; ++r) xv[a][r] = *reinterpret_cast<const u4 *>(px[a] + r * W + 4 * w4);
#pragma unroll
            for (int b = 0; b < BY; ++b)
#pragma unroll
                for (int r = 0; r < MY; ++r) yv[b][r] = *reinterpret_cast<const u4 *>(py[b] + r * W + 4 * w4);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int a = 0; a < BX; ++a)
#pragma unroll
                    for (int r = 0; r < MX; ++r)
#pragma unroll
                        for (int b = 0; b < BY; ++b)
#pragma unroll
                            for (int q = 0; q < MY; ++q) cnt[a][b][r * MY + q] += __builtin_popcount(xv[a][r][k] & yv[b][q][k]);
        }
#pragma unroll
        for (int a = 0; a < BX; ++a)
#pragma unroll
            for (int b = 0; b < BY; ++b)
#pragma unroll
                for (int c = 0; c < NCC; ++c) {
                    uint32_t v = cnt[a][b][c];
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
                    cnt[a][b][c] = v;
                }
    }
#pragma unroll
    for (int a = 0; a < BX; ++a)
#pragma unroll
        for (int b = 0; b < BY; ++b) {
            const int x = xs[a], y = ys[b];
            const int u = x < y ? x : y, v = x < y ? y : x;
            const long long t = (long long)u * nvars - (long long)u * (u + 1) / 2 + (v - u - 1);
            if (!(a < nx && b < ny && x < y && t >= t0 && t < t1)) continue;  // wave-uniform
            const int32_t *cx = rowcnt + row0[x], *cy = rowcnt + row0[y];
            int32_t full[DX * DY];
#pragma unroll
            for (int i = 0; i < MX; ++i) {
                int32_t r = cx[i];
#pragma unroll
                for (int j = 0; j < MY; ++j) full[i * DY + j] = (int32_t)cnt[a][b][i * MY + j], r -= full[i * DY + j];
                full[i * DY + MY] = r;
            }
#pragma unroll
            for (int j = 0; j < DY; ++j) {
                int32_t r = cy[j];
#pragma unroll
                for (int i = 0; i < MX; ++i) r -= full[i * DY + j];
                full[MX * DY + j] = r;
            }
            if (lane < DX * DY) {
                int32_t val = 0;
#pragma unroll
                for (int c = 0; c < DX * DY; ++c) val = lane == c ? full[c] : val;
                // x < y here: the table is N[value of x][value of y] (Counts2D of the pair (u, v))
                int32_t *out = counts + (t - t0) * kBitsCells;
                out[lane] = val;
                if (pairtab) pairtab[16 * t + lane] = val;
            }
        }
}

__global__ __launch_bounds__(256) void ci_bits_pairs_tiled(const uint32_t *__restrict__ bits,
                                                           const int32_t *__restrict__ row0,
                                                           const int32_t *__restrict__ rowcnt, long long W,
                                                           const int32_t *__restrict__ tasks, long long ntasks,
                                                           int nvars, long long t0, long long t1,
                                                           int32_t *__restrict__ counts, int32_t *__restrict__ pairtab) {
    const int lane = threadIdx.x & 63;
    for (long long k = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); k < ntasks; k += (long long)gridDim.x * 4) {
        const int32_t *task = tasks + k * kPairTaskInts;
        switch (task[0] * 8 + task[1]) {
#define FBN_PB(A, B)                                                                                       \
    case A * 8 + B:                                                                                        \
        pair_block<A, B>(bits, row0, rowcnt, W, task, nvars, t0, t1, counts, pairtab, lane);               \
        break;
            FBN_PB(1, 1) FBN_PB(1, 2) FBN_PB(1, 3) FBN_PB(1, 4)
            FBN_PB(2, 1) FBN_PB(2, 2) FBN_PB(2, 3) FBN_PB(2, 4)
            FBN_PB(3, 1) FBN_PB(3, 2) FBN_PB(3, 3) FBN_PB(3, 4)
            FBN_PB(4, 1) FBN_PB(4, 2) FBN_PB(4, 3) FBN_PB(4, 4)
#undef FBN_PB
        default: break;
        }
    }
}


// phase 1: counts[t][64] of every test, one wave per test; D = 0 (x, y) or 1 (x, y, z)
template <int D>
__global__ __launch_bounds__(256) void ci_bits_count(const uint32_t *__restrict__ bits, const int32_t *__restrict__ dims,
                                                     const int32_t *__restrict__ row0, const int32_t *__restrict__ items,
                                                     long long W, long long n, int32_t *__restrict__ counts,
                                                     const int32_t *__restrict__ rowcnt, int32_t *__restrict__ pairtab,
                                                     int nvars, long long t0) {
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    for (long long t = wave; t < n; t += (long long)gridDim.x * 4) {
        int x, y;
        if (D == 0 && !items) pair_of(t0 + t, nvars, x, y);
        else x = items[(2 + D) * t], y = items[(2 + D) * t + 1];
        const int dx = dims[x], dy = dims[y];
        const uint32_t *bx = bits + (size_t)row0[x] * W, *by = bits + (size_t)row0[y] * W;
        const uint32_t *bz = bx;
        int dz = 1;
        if (D == 1) {
            const int z = items[3 * t + 2];
            dz = dims[z];
            bz = bits + (size_t)row0[z] * W;
        }
        int32_t *out = counts + t * kBitsCells;
        constexpr int DZ = D == 1 ? 4 : 1;
        const int32_t *nx = rowcnt + row0[x], *ny = rowcnt + row0[y];
        // level 0 of a PC run records every pair's table (pair index of x < y, 16 slots)
        int32_t *rec = (D == 0 && pairtab && x < y)
                           ? pairtab + 16 * ((long long)x * nvars - (long long)x * (x + 1) / 2 + (y - x - 1))
                           : nullptr;
        switch (dx * 8 + dy) {
#define FBN_PAIR(A, B)                                                             \
    case A * 8 + B:                                                                \
        if (D == 0) count_pair<A, B>(bx, by, nx, ny, W, lane, out, rec);           \
        else count_test<A, B, DZ>(bx, by, bz, dz, W, lane, out);                   \
        break;
            FBN_PAIR(1, 1) FBN_PAIR(1, 2) FBN_PAIR(1, 3) FBN_PAIR(1, 4)
            FBN_PAIR(2, 1) FBN_PAIR(2, 2) FBN_PAIR(2, 3) FBN_PAIR(2, 4)
            FBN_PAIR(3, 1) FBN_PAIR(3, 2) FBN_PAIR(3, 3) FBN_PAIR(3, 4)
            FBN_PAIR(4, 1) FBN_PAIR(4, 2) FBN_PAIR(4, 3) FBN_PAIR(4, 4)
#undef FBN_PAIR
        default: break;  // the host only routes tests with dims <= 4 here
        }
    }
}

// level >= 1 of a PC run, one conditioning variable, pair tables recorded: derived counting
__device__ __forceinline__ const int32_t *pair_table(const int32_t *pairtab, int nvars, int u, int v) {
    const int i = u < v ? u : v, j = u < v ? v : u;
    return pairtab + 16 * ((long long)i * nvars - (long long)i * (i + 1) / 2 + (j - i - 1));
}
// XCD-contiguous work split: workgroups are dispatched round-robin over the 8 XCDs (block b on XCD
// b % 8), each with its own L2.  Cutting the n units into 8 contiguous ranges, range j worked by
// XCD j's blocks in order, keeps consecutive units -- an edge's candidate conditioning variables,
// which share the x and y mask rows -- in one L2 at about the same time.  xcd = 0: plain grid stride.
struct XcdSplit {
    long long first, end, stride;
};
__device__ __forceinline__ XcdSplit xcd_split(long long n, int wave, int per_block, int xcd) {
    const long long G = gridDim.x, b = blockIdx.x;
    if (!xcd || G < 8) return {b * per_block + wave, n, G * per_block};
    const long long j = b % 8, nb = (G - j + 7) / 8, i = b / 8;
    return {n * j / 8 + i * per_block + wave, n * (j + 1) / 8, nb * per_block};
}

__device__ __forceinline__ void count_derived_items(const uint32_t *__restrict__ bits,
                                                             const int32_t *__restrict__ dims,
                                                             const int32_t *__restrict__ row0,
                                                             const int32_t *__restrict__ items, long long W, long long n,
                                                             int32_t *__restrict__ counts,
                                                             const int32_t *__restrict__ pairtab, int nvars,
                                                             int xcd) {
    const int lane = threadIdx.x & 63;
    const XcdSplit sp = xcd_split(n, threadIdx.x >> 6, 4, xcd);
    for (long long t = sp.first; t < sp.end; t += sp.stride) {
        const int x = items[3 * t], y = items[3 * t + 1], z = items[3 * t + 2];
        const int dx = dims[x], dy = dims[y], dz = dims[z];
        const uint32_t *bx = bits + (size_t)row0[x] * W, *by = bits + (size_t)row0[y] * W,
                       *bz = bits + (size_t)row0[z] * W;
        const int32_t *Txy = pair_table(pairtab, nvars, x, y), *Txz = pair_table(pairtab, nvars, x, z),
                      *Tyz = pair_table(pairtab, nvars, y, z);
        int32_t *out = counts + t * kBitsCells;
        switch (dz * 64 + dx * 8 + dy) {
#define FBN_TRIPLE(C, A, B)                                                                                  \
    case C * 64 + A * 8 + B:                                                                                 \
        count_test_derived<A, B, C>(bx, by, bz, W, lane, out, Txy, x > y, Txz, x > z, Tyz, y > z);          \
        break;
#define FBN_ROW(C)                                                                                           \
    FBN_TRIPLE(C, 1, 1) FBN_TRIPLE(C, 1, 2) FBN_TRIPLE(C, 1, 3) FBN_TRIPLE(C, 1, 4)                          \
    FBN_TRIPLE(C, 2, 1) FBN_TRIPLE(C, 2, 2) FBN_TRIPLE(C, 2, 3) FBN_TRIPLE(C, 2, 4)                          \
    FBN_TRIPLE(C, 3, 1) FBN_TRIPLE(C, 3, 2) FBN_TRIPLE(C, 3, 3) FBN_TRIPLE(C, 3, 4)                          \
    FBN_TRIPLE(C, 4, 1) FBN_TRIPLE(C, 4, 2) FBN_TRIPLE(C, 4, 3) FBN_TRIPLE(C, 4, 4)
            FBN_ROW(1) FBN_ROW(2) FBN_ROW(3) FBN_ROW(4)
#undef FBN_ROW
#undef FBN_TRIPLE
        default: break;
        }
    }
}

// n_dev != nullptr: the test count is read on the device (batches generated on the device)
__global__ __launch_bounds__(256) void ci_bits_count_derived(const uint32_t *__restrict__ bits,
                                                             const int32_t *__restrict__ dims,
                                                             const int32_t *__restrict__ row0,
                                                             const int32_t *__restrict__ items, long long W, long long n,
                                                             int32_t *__restrict__ counts,
                                                             const int32_t *__restrict__ pairtab, int nvars, int xcd,
                                                             const long long *__restrict__ n_dev) {
    count_derived_items(bits, dims, row0, items, W, n_dev ? *n_dev : n, counts, pairtab, nvars, xcd);
}



// ---- row Gram matrices (levels 0 and 1 of a PC run on the bit-sliced store)
// A PC run's level 0 needs popcount(r_i & r_j) for every pair of leading mask rows (values 0..d-2
// of every variable; the last value is derived), and level 1 needs popcount(x_a & r_i & r_j) for
// the rows of every pair of x's neighbours: both are Gram matrices of mask rows over the sample
// bits.  One wave per task = an 8 x 8 tile of (i, j) row pairs (optionally every row ANDed with a
// mask row x_a): per 4-word step 16 (17) 16-byte loads feed 256 popcounts, counters in registers,
// then a butterfly reduction that leaves counter l's wave total in lane l (63 shuffles instead of
// 64 x 6).  Tasks are built on the host (capi.hip CiGram*): one block of one wave per task so the
// task fields and row pointers are wave-uniform (scalar registers).
constexpr int kGramTaskInts = 8;  // mask row (-1: none), i0, ni, j0, nj, out offset (lo, hi), ld

template <bool MASKED>
__global__ __launch_bounds__(64) void ci_bits_gram(const uint32_t *__restrict__ bits, long long W,
                                                   const int32_t *__restrict__ rl, const int32_t *__restrict__ tasks,
                                                   long long ntasks, int32_t *__restrict__ out, int xcd) {
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    const int lane = threadIdx.x;
    // consecutive tiles (the same i-block of rows) on one XCD: the rows stay in that XCD's L2
    const XcdSplit sp = xcd_split(ntasks, 0, 1, xcd);
    for (long long k = sp.first; k < sp.end; k += sp.stride) {
        const int32_t *t = tasks + k * kGramTaskInts;
        const int mrow = t[0], i0 = t[1], ni = t[2], j0 = t[3], nj = t[4], ld = t[7];
        const long long off = (long long)(uint32_t)t[5] | ((long long)t[6] << 32);
        const uint32_t *pi[8], *pj[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) pi[r] = bits + (size_t)rl[i0 + (r < ni ? r : 0)] * W;
#pragma unroll
        for (int r = 0; r < 8; ++r) pj[r] = bits + (size_t)rl[j0 + (r < nj ? r : 0)] * W;
        const uint32_t *pm = bits + (size_t)(MASKED ? mrow : 0) * W;
        uint32_t v[64];
#pragma unroll
        for (int c = 0; c < 64; ++c) v[c] = 0u;
        for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
            u4 xi[8], yj[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) xi[r] = *reinterpret_cast<const u4 *>(pi[r] + 4 * w4);
#pragma unroll
            for (int r = 0; r < 8; ++r) yj[r] = *reinterpret_cast<const u4 *>(pj[r] + 4 * w4);
            if (MASKED) {
                const u4 m = *reinterpret_cast<const u4 *>(pm + 4 * w4);
#pragma unroll
                for (int r = 0; r < 8; ++r) xi[r] &= m;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int a = 0; a < 8; ++a)
#pragma unroll
                    for (int b = 0; b < 8; ++b) v[a * 8 + b] += __builtin_popcount(xi[a][q] & yj[b][q]);
        }
        // butterfly: at distance o each lane keeps the half of its counters selected by lane bit o
        // and adds its partner's copy of that half; lane l ends with counter l's total
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const bool hi = (lane & o) != 0;
#pragma unroll
            for (int c = 0; c < o; ++c) {
                const uint32_t send = hi ? v[c] : v[c + o], keep = hi ? v[c + o] : v[c];
                v[c] = keep + (uint32_t)__shfl_xor((int)send, o);
            }
        }
        const int a = lane >> 3, b = lane & 7;
        if (a < ni && b < nj) out[off + (long long)a * ld + b] = (int32_t)v[0];
    }
}

// level 0 from the Gram G of all leading rows (ld x ld, lead0[v] = v's first leading row): the
// (x < y) pair table of test t (pair t0 + t of the complete graph), last row / column derived from
// the per-row sample counts exactly as pair_block / count_pair; the 64-slot record and, when
// recording, the pair table
template <int DX, int DY>
__device__ __forceinline__ void gram_pair(const int32_t *__restrict__ G, long long ld, int x, int y,
                                          const int32_t *__restrict__ lead0, const int32_t *__restrict__ cx,
                                          const int32_t *__restrict__ cy, int32_t *__restrict__ out,
                                          int32_t *__restrict__ ptab) {
    constexpr int MX = DX - 1, MY = DY - 1;
    int32_t full[DX * DY];
    const int32_t *g = G + (long long)lead0[x] * ld + lead0[y];
#pragma unroll
    for (int i = 0; i < MX; ++i) {
        int32_t r = cx[i];
#pragma unroll
        for (int j = 0; j < MY; ++j) full[i * DY + j] = g[i * ld + j], r -= full[i * DY + j];
        full[i * DY + MY] = r;
    }
#pragma unroll
    for (int j = 0; j < DY; ++j) {
        int32_t r = cy[j];
#pragma unroll
        for (int i = 0; i < MX; ++i) r -= full[i * DY + j];
        full[MX * DY + j] = r;
    }
#pragma unroll
    for (int c = 0; c < DX * DY; ++c) out[c] = full[c];
    if (ptab)
#pragma unroll
        for (int c = 0; c < DX * DY; ++c) ptab[c] = full[c];
}

__global__ __launch_bounds__(256) void ci_bits_gram_pairs(const int32_t *__restrict__ G, long long ld,
                                                          const int32_t *__restrict__ lead0,
                                                          const int32_t *__restrict__ dims,
                                                          const int32_t *__restrict__ row0,
                                                          const int32_t *__restrict__ rowcnt, long long t0, long long n,
                                                          int nvars, int32_t *__restrict__ counts,
                                                          int32_t *__restrict__ pairtab) {
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < n; t += (long long)gridDim.x * 256) {
        int x, y;
        pair_of(t0 + t, nvars, x, y);
        int32_t *out = counts + t * kBitsCells, *ptab = pairtab ? pairtab + 16 * (t0 + t) : nullptr;
        const int32_t *cx = rowcnt + row0[x], *cy = rowcnt + row0[y];
        switch (dims[x] * 8 + dims[y]) {
#define FBN_GP(A, B)                                                                                         \
    case A * 8 + B:                                                                                          \
        gram_pair<A, B>(G, ld, x, y, lead0, cx, cy, out, ptab);                                              \
        break;
            FBN_GP(1, 1) FBN_GP(1, 2) FBN_GP(1, 3) FBN_GP(1, 4)
            FBN_GP(2, 1) FBN_GP(2, 2) FBN_GP(2, 3) FBN_GP(2, 4)
            FBN_GP(3, 1) FBN_GP(3, 2) FBN_GP(3, 3) FBN_GP(3, 4)
            FBN_GP(4, 1) FBN_GP(4, 2) FBN_GP(4, 3) FBN_GP(4, 4)
#undef FBN_GP
        default: break;
        }
    }
}

// position of v in the sorted list a[0..n) (present by construction)
__device__ __forceinline__ int find_sorted(const int32_t *__restrict__ a, int n, int v) {
    int lo = 0, hi = n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] <= v) lo = mid;
        else hi = mid;
    }
    return lo < n && a[lo] == v ? lo : -1;
}

// level 1 from the per-variable masked Grams: item (x, y, z) reads its (dx-1)(dy-1)(dz-1) leading
// cells popcount(x_a & y_b & z_c) from G_u, u = x if z is x's neighbour, else y (then x and z are
// y's neighbours); G_u[a] is R_u x R_u over u's neighbours' leading rows (upper tiles only: the
// entry is read as (row of the earlier neighbour, row of the later one)).  The rest of the table
// is derived from the pair tables exactly as count_test_derived; every value is an integer.
__global__ __launch_bounds__(256) void ci_bits_gram_triples(
    const int32_t *__restrict__ G, const long long *__restrict__ goff, const int32_t *__restrict__ gR,
    const int32_t *__restrict__ adj, const int32_t *__restrict__ adj_off, const int32_t *__restrict__ loff,
    const int32_t *__restrict__ dims, const int32_t *__restrict__ items, long long n, int32_t *__restrict__ counts,
    const int32_t *__restrict__ pairtab, int nvars) {
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < n; t += (long long)gridDim.x * 256) {
        const int x = items[3 * t], y = items[3 * t + 1], z = items[3 * t + 2];
        const int DX = dims[x], DY = dims[y], DZ = dims[z], MX = DX - 1, MY = DY - 1, MZ = DZ - 1;
        int pzx = find_sorted(adj + adj_off[x], adj_off[x + 1] - adj_off[x], z);
        const bool ux = pzx >= 0;
        const int u = ux ? x : y, o = ux ? y : x;
        const int32_t *au = adj + adj_off[u];
        const int nu = adj_off[u + 1] - adj_off[u];
        const int po = find_sorted(au, nu, o), pz = ux ? pzx : find_sorted(au, nu, z);
        if (po < 0 || pz < 0) continue;  // not a level-1 item of this skeleton (never generated)
        const int32_t *lu = loff + adj_off[u];
        const int Ru = gR[u], ro = lu[po], rz = lu[pz];
        const bool oz = po < pz;
        const int32_t *Gu = G + goff[u];
        // leading cells cnt[c][a][b] (a: value of x, b: value of y, c: value of z)
        int32_t cnt[3][3][3];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    int32_t v = 0;
                    if (c < MZ && a < MX && b < MY) {
                        const int ua = ux ? a : b, ob = ux ? b : a;  // u's value, the other's value
                        const long long ri = ro + ob, rj = rz + c;
                        v = Gu[((long long)ua * Ru + (oz ? ri : rj)) * Ru + (oz ? rj : ri)];
                    }
                    cnt[c][a][b] = v;
                }
        const int32_t *Txy = pair_table(pairtab, nvars, x, y), *Txz = pair_table(pairtab, nvars, x, z),
                      *Tyz = pair_table(pairtab, nvars, y, z);
        const bool txy = x > y, txz = x > z, tyz = y > z;
        auto nxy = [&](int a, int b) { return txy ? Txy[b * DX + a] : Txy[a * DY + b]; };
        auto nxz = [&](int a, int c) { return txz ? Txz[c * DX + a] : Txz[a * DZ + c]; };
        auto nyz = [&](int b, int c) { return tyz ? Tyz[c * DY + b] : Tyz[b * DZ + c]; };
        // N[c][a][b] for c < MZ: leading cells, then the last y value, then the last x value
        auto fz = [&](int c, int a, int b) {
            auto row_last = [&](int aa) {  // N[c][aa][MY], aa < MX
                int32_t r = nxz(aa, c);
#pragma unroll
                for (int bb = 0; bb < 3; ++bb)
                    if (bb < MY) r -= cnt[c][aa][bb];
                return r;
            };
            if (a < MX) return b < MY ? cnt[c][a][b] : row_last(a);
            int32_t r = nyz(b, c);
#pragma unroll
            for (int aa = 0; aa < 3; ++aa)
                if (aa < MX) r -= b < MY ? cnt[c][aa][b] : row_last(aa);
            return r;
        };
        int32_t *out = counts + t * kBitsCells;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (a >= DX || b >= DY) continue;
                int32_t last = nxy(a, b);
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    if (c < MZ) {
                        const int32_t v = fz(c, a, b);
                        out[(c * DX + a) * DY + b] = v;
                        last -= v;
                    }
                out[(MZ * DX + a) * DY + b] = last;
            }
    }
}

// phase 2, large launches (ci_bits_g2): one lane per test -- per z: marginals, adjusted df; G^2 as one running sum in the
// reference's z -> x -> y order (ComputeGSquareXY / XYZ, src/IndependenceTest.cpp:65-155,
// 295-364; the same arithmetic as ci_g2_kernel), p = 1 - P(df/2, G^2/2) (ci_chisq.h).  With no p
// output and a decision band (band != nullptr: [lo, hi] per df 1..nband, then delta), p is only
// evaluated for G^2 inside the band (fbn_chisq_band).  The margin log is reduced per wave (one
// atomic per wave, not per test).  (Measured and not kept: 16 lanes per test with the terms in
// LDS, 10x slower at level 0; per-class instantiations with the table in registers, 1.7x slower.)
template <int D>
__global__ __launch_bounds__(256) void ci_bits_g2(const int32_t *__restrict__ counts, const int32_t *__restrict__ dims,
                                                  const int32_t *__restrict__ items, long long n, double alpha,
                                                  double *__restrict__ g2o, int32_t *__restrict__ dfo,
                                                  double *__restrict__ po, uint8_t *__restrict__ indep,
                                                  int32_t *__restrict__ counts0, unsigned long long *__restrict__ stats,
                                                  int nvars, long long t0, const double *__restrict__ band,
                                                  int nband, const long long *__restrict__ n_dev) {
    if (n_dev) n = *n_dev;
    const long long stride = (long long)gridDim.x * 256;
    // wave-uniform trip count (the margin reduction below is a whole-wave operation)
    for (long long wb = (long long)blockIdx.x * 256 + (threadIdx.x & ~63); wb < n; wb += stride) {
        const long long t = wb + (threadIdx.x & 63);
        unsigned long long mbits = ~0ull;  // this lane's |p - alpha| (as ordered bits), none = max
        bool near = false;
        if (t < n) {
            int px, py;
            if (D == 0 && !items) pair_of(t0 + t, nvars, px, py);
            else px = items[(2 + D) * t], py = items[(2 + D) * t + 1];
            const int dx = dims[px], dy = dims[py];
            const int dimz = D == 1 ? dims[items[3 * t + 2]] : 1;
            const int dxy = dx * dy;
            const int32_t *hz = counts + t * kBitsCells;
            // the record unpacked into a fixed KZ x 4 x 4 register table (absent cells 0): every load
            // is independent (one memory latency per test, not one per loop step) and every index
            // below is static.  Absent rows / columns / z values have zero counts, so they add
            // nothing to df (max(0, 1) - 1 = 0) or G^2 (their terms are skipped) -- the sums are the
            // reference's over the real table, in its order.
            constexpr int KZ = D == 1 ? 4 : 1;
            int h[KZ][4][4];
#pragma unroll
            for (int k = 0; k < KZ; ++k)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const bool in = k < dimz && i < dx && j < dy;
                        const int v = hz[in ? k * dxy + i * dy + j : 0];
                        h[k][i][j] = in ? v : 0;
                    }
            // one running sum over z -> x -> y, exactly the reference's loop (no per-z partials)
            double g2 = 0.0;
            int df = 0;
#pragma unroll
            for (int k = 0; k < KZ; ++k) {
                int ni[4], nj[4], alx = 0, aly = 0;
                long total = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    ni[i] = (h[k][i][0] + h[k][i][1]) + (h[k][i][2] + h[k][i][3]);
                    alx += ni[i] > 0;
                    total += ni[i];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    nj[j] = (h[k][0][j] + h[k][1][j]) + (h[k][2][j] + h[k][3][j]);
                    aly += nj[j] > 0;
                }
                df += ((alx >= 1 ? alx : 1) - 1) * ((aly >= 1 ? aly : 1) - 1);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const long sum_row = ni[i];
                    if (total == 0 || sum_row == 0) continue;
                    // the row's four terms side by side (independent latency chains), then the present
                    // ones added in order
                    double tm[4];
                    bool on[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        on[j] = nj[j] != 0 && h[k][i][j] != 0;
                        const long o1 = on[j] ? h[k][i][j] : 1, c1 = on[j] ? nj[j] : 1;
                        const double expected = (double)c1 * (double)sum_row / (double)total;
                        tm[j] = 2.0 * o1 * log(o1 / expected);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (on[j]) g2 += tm[j];
                }
            }
            double p = 1.0, m;
            bool ind;
            if (df == 0) {  // src/IndependenceTest.cpp:149-151, 349-351
                ind = true;
                m = fabs(p - alpha);
            } else if (!po && band && df <= nband && g2 < band[2 * df - 2]) {
                ind = true, m = band[2 * nband];  // p > alpha + delta
            } else if (!po && band && df <= nband && g2 > band[2 * df - 1]) {
                ind = false, m = band[2 * nband];  // p < alpha - delta
            } else {
                p = fbn_chisq_pvalue(g2, df);
                ind = p > alpha;
                m = fabs(p - alpha);
            }
            if (g2o) g2o[t] = g2;
            dfo[t] = df;
            if (po) po[t] = p;
            indep[t] = ind;
            if (counts0 && t == 0)
                for (int c = 0; c < dimz * dxy; ++c) counts0[c] = hz[c];
            mbits = (unsigned long long)__double_as_longlong(m);
            near = m < 1e-9;
        }
        if (stats) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned long long v = __shfl_xor(mbits, o);
                mbits = v < mbits ? v : mbits;
            }
            const unsigned long long nn = __popcll(__ballot(near));
            if ((threadIdx.x & 63) == 0) {
                if (mbits != ~0ull) atomicMin(stats, mbits);
                if (nn) atomicAdd(stats + 1, nn);
            }
        }
    }
}

// phase 2, small launches (ci_bits_g2q): four lanes per test -- marginals, adjusted df; G^2 as one running sum in the reference's
// z -> x -> y order (ComputeGSquareXY / XYZ, src/IndependenceTest.cpp:65-155, 295-364; the same
// arithmetic as ci_g2_kernel), p = 1 - P(df/2, G^2/2) (ci_chisq.h).  Lane q of a test's group owns z
// value q (D = 1: a 4 x 4 slice) or x value q (D = 0: a row of 4): it unpacks its part of the 256-B
// count record into a zero-padded register table (independent loads, static indices; absent rows,
// columns and z values add nothing to df or G^2), evaluates its terms -- the costly part, a division
// chain and a log each -- in parallel with the other three lanes, and then the four lanes add
// their terms into the one running sum in turn.  With no p output and a decision band (band !=
// nullptr: [lo, hi] per df 1..nband, then delta), p is only evaluated for G^2 inside the band
// (fbn_chisq_band).  The margin log is reduced per wave (one atomic per wave, not per test).
constexpr int kG2Lanes = 4;
constexpr int kG2TestsPerBlock = 256 / kG2Lanes;
constexpr long long kG2QuadMax = 16384;  // launches of at most this many tests use ci_bits_g2q
template <int D>
__global__ __launch_bounds__(256) void ci_bits_g2q(const int32_t *__restrict__ counts, const int32_t *__restrict__ dims,
                                                  const int32_t *__restrict__ items, long long n, double alpha,
                                                  double *__restrict__ g2o, int32_t *__restrict__ dfo,
                                                  double *__restrict__ po, uint8_t *__restrict__ indep,
                                                  int32_t *__restrict__ counts0, unsigned long long *__restrict__ stats,
                                                  int nvars, long long t0, const double *__restrict__ band,
                                                  int nband, const long long *__restrict__ n_dev) {
    if (n_dev) n = *n_dev;
    const int lane = threadIdx.x & 63, q = lane & (kG2Lanes - 1), g0 = lane & ~(kG2Lanes - 1);
    const long long stride = (long long)gridDim.x * kG2TestsPerBlock;
    // wave-uniform trip count (the shuffles and the margin reduction are whole-wave operations)
    for (long long wb = (long long)blockIdx.x * kG2TestsPerBlock + (threadIdx.x >> 6) * (64 / kG2Lanes); wb < n;
         wb += stride) {
        const long long t = wb + lane / kG2Lanes;
        const bool live = t < n;
        int px = 0, py = 0, pz = 0;
        if (live) {
            if (D == 0 && !items) pair_of(t0 + t, nvars, px, py);
            else px = items[(2 + D) * t], py = items[(2 + D) * t + 1];
            if (D == 1) pz = items[3 * t + 2];
        }
        const int dx = live ? dims[px] : 1, dy = live ? dims[py] : 1;
        const int dimz = D == 1 && live ? dims[pz] : 1;
        const int dxy = dx * dy;
        const int32_t *hz = counts + (live ? t : 0) * kBitsCells;
        constexpr int NR = D == 1 ? 4 : 1;  // rows this lane owns
        int h[NR][4];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = D == 1 ? q : 0, i = D == 1 ? r : q;
                const bool in = live && k < dimz && i < dx && j < dy;
                const int v = hz[in ? k * dxy + i * dy + j : 0];
                h[r][j] = in ? v : 0;
            }
        // this lane's slice (D = 1) or the test's only slice (D = 0): marginals, total, df
        int ni[NR], nj[4], df;
        long total = 0;
        {
            int alx = 0, aly = 0;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                ni[r] = (h[r][0] + h[r][1]) + (h[r][2] + h[r][3]);
                alx += ni[r] > 0;
                total += ni[r];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int c = 0;
#pragma unroll
                for (int r = 0; r < NR; ++r) c += h[r][j];
                nj[j] = c;
            }
            if (D == 0) {  // the slice's rows are spread over the group
#pragma unroll
                for (int o = 1; o < kG2Lanes; o <<= 1) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) nj[j] += __shfl_xor(nj[j], o);
                    alx += __shfl_xor(alx, o);
                    total += __shfl_xor(total, o);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) aly += nj[j] > 0;
            df = ((alx >= 1 ? alx : 1) - 1) * ((aly >= 1 ? aly : 1) - 1);
            if (D == 1)
#pragma unroll
                for (int o = 1; o < kG2Lanes; o <<= 1) df += __shfl_xor(df, o);
        }
        // this lane's terms, side by side (independent latency chains)
        double tm[NR][4];
        bool on[NR][4];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const long sum_row = ni[r];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                on[r][j] = total != 0 && sum_row != 0 && nj[j] != 0 && h[r][j] != 0;
                tm[r][j] = 0.0;
            }
            if (total != 0 && sum_row != 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const long o1 = on[r][j] ? h[r][j] : 1, c1 = on[r][j] ? nj[j] : 1;
                    const double expected = (double)c1 * (double)sum_row / (double)total;
                    tm[r][j] = 2.0 * o1 * log(o1 / expected);
                }
            }
        }
        // the running sum, lane 0's cells first: z (D = 1) or x (D = 0) is the group's outer digit
        double g2 = 0.0;
#pragma unroll
        for (int s = 0; s < kG2Lanes; ++s) {
            if (q == s)
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (on[r][j]) g2 += tm[r][j];
            g2 = __shfl(g2, g0 + s);
        }
        unsigned long long mbits = ~0ull;  // this test's |p - alpha| (as ordered bits), none = max
        bool near = false;
        if (live) {
            double p = 1.0, m;
            bool ind;
            if (df == 0) {  // src/IndependenceTest.cpp:149-151, 349-351
                ind = true;
                m = fabs(p - alpha);
            } else if (!po && band && df <= nband && g2 < band[2 * df - 2]) {
                ind = true, m = band[2 * nband];  // p > alpha + delta
            } else if (!po && band && df <= nband && g2 > band[2 * df - 1]) {
                ind = false, m = band[2 * nband];  // p < alpha - delta
            } else {
                p = fbn_chisq_pvalue(g2, df);
                ind = p > alpha;
                m = fabs(p - alpha);
            }
            if (q == 0) {
                if (g2o) g2o[t] = g2;
                dfo[t] = df;
                if (po) po[t] = p;
                indep[t] = ind;
                if (counts0 && t == 0)
                    for (int c = 0; c < dimz * dxy; ++c) counts0[c] = hz[c];
                mbits = (unsigned long long)__double_as_longlong(m);
                near = m < 1e-9;
            }
        }
        if (stats) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned long long v = __shfl_xor(mbits, o);
                mbits = v < mbits ? v : mbits;
            }
            const unsigned long long nn = __popcll(__ballot(near));
            if (lane == 0) {
                if (mbits != ~0ull) atomicMin(stats, mbits);
                if (nn) atomicAdd(stats + 1, nn);
            }
        }
    }
}

// ---- device-resident level-1 search (a PC run's level 1, group size 1)
// Edge e = (x < y) of the level's range; its candidate k walks the combined list adj(x)\{y} then
// adj(y)\{x} in sorted order (CheckEdge's two sides, src/PCStable.cpp:402-470 with d = 1); pos =
// next candidate, st = 0 open / 1 removed (sep = z of its first independent test) / 2 kept
// (exhausted).  Every round takes the next `chunk` candidates of each open edge, counts and tests
// them (ci_bits_count_derived + ci_bits_g2<1> with the test count read on the device) and resolves
// each edge's prefix in order: counted = tests up to and including the first independent one.  The
// host only enqueues rounds; nothing per test crosses PCIe.
struct L1Edge {
    int32_t x, y, m0, L, skx, sky, ax, ay;  // ax / ay: adjacency offsets, skx / sky: position of y / x
    // the candidates the information screen keeps (below): P of them, positions plist[pl .. pl + P)
    // (pl = -1: no screen, every candidate k = its own position)
    int32_t P, pl;
};

// ---- the information screen of level 1 (exact: it only skips tests whose answer is known)
// With empirical (plug-in) mutual information I over the same N samples, the chain rule holds
// exactly: I(X;Y) + I(X;Z|Y) = I(X;Z) + I(X;Y|Z), so I(X;Y) <= I(X;Z) + I(X;Y|Z) (and likewise for
// Y).  G^2 of a test is 2N I(X;Y|Z) (src/IndependenceTest.cpp:94-138: the sum of 2 O log(O / E)),
// and "independent" needs G^2 <= hi(df), the upper end of the decision band for its df (df <=
// (dx-1)(dy-1)dz; hi grows with df).  Hence a candidate z with
//     I(X;Z) < I(X;Y) - tau   or   I(Y;Z) < I(X;Y) - tau,   tau = hi((dx-1)(dy-1)dz) / 2N (+ margins)
// can never be the independent one: its test is dependent whatever its counts.  Level 1 runs only
// the other candidates; counted tests stay the reference's (every candidate up to the first
// independent one, src/PCStable.cpp:465-551), launched tests are the ones run.  The pairwise I come
// from the level-0 pair tables.  (The margins, 1e-9 relative on hi and 1e-9 absolute in nats, are
// orders above the rounding of either side: a few 1e-16 relative on values <= log 4.)
__device__ __forceinline__ long long l1_pidx(int u, int v, int nv) {
    const int i = u < v ? u : v, j = u < v ? v : u;
    return (long long)i * nv - (long long)i * (i + 1) / 2 + (j - i - 1);
}
// (in G^2 units: g2[pair] = 2N I of the pair's level-0 table; the margin 1e-9 nats = two_n * 1e-9)
__device__ __forceinline__ bool l1_plausible(const double *__restrict__ g2, int nv, const int32_t *__restrict__ dims,
                                             const double *__restrict__ band, int nband, double two_n, int x, int y,
                                             int z, double gxy) {
    const int df = (dims[x] - 1) * (dims[y] - 1) * dims[z];
    if (df <= 0 || df > nband) return true;
    const double lim = gxy - (band[2 * df - 1] * (1.0 + 1e-9) + two_n * 1e-9);
    if (lim <= 0.0) return true;
    return g2[l1_pidx(x, z, nv)] >= lim && g2[l1_pidx(y, z, nv)] >= lim;
}
// G^2 = 2N I(X;Y) of every pair of the complete graph from its level-0 table (pairtab, 16 counts:
// N[a][b] at a * dy + b for x < y), one thread per pair -- when level 0's own G^2 values are not all
// on this device (a rank of the distributed session ran part of level 0 and imported the others'
// tables).  The screen reads pairs that need not be edges: (y, z) for z a neighbour of x.
__global__ __launch_bounds__(256) void ci_pair_g2(const int32_t *__restrict__ pairtab, const int32_t *__restrict__ dims,
                                                  int nv, long long P, double *__restrict__ g2) {
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < P; t += (long long)gridDim.x * 256) {
        int x, y;
        pair_of(t, nv, x, y);
        const int dx = dims[x], dy = dims[y];
        const int32_t *T = pairtab + 16 * t;
        double r[4] = {0, 0, 0, 0}, c[4] = {0, 0, 0, 0}, n = 0.0;
        for (int a = 0; a < dx; ++a)  // (dims <= 4 on this path)
            for (int b = 0; b < dy; ++b) {
                const double w = T[a * dy + b];
                r[a] += w, c[b] += w, n += w;
            }
        double acc = 0.0;
        for (int a = 0; a < dx; ++a)
            for (int b = 0; b < dy; ++b) {
                const double w = T[a * dy + b];
                if (w > 0.0) acc += w * log(w * n / (r[a] * c[b]));
            }
        g2[t] = 2.0 * acc;
    }
}

// The rounds' test offsets: a single-pass exclusive scan of the edges' lengths inside the kernel
// that computes them (ci_l1_setup for round 0, ci_l1_resolve for the next round), 256-edge tiles
// taken in ticket order (so every earlier tile belongs to a running workgroup) with a decoupled
// look-back over the earlier tiles' published aggregates / prefixes, then the round's clip at cap
// (edges past it continue next round).  Status word per tile: epoch << 34 | flag << 32 | value
// (flag 1 = tile aggregate, 2 = inclusive prefix); the epoch (1 = setup, r + 2 = round r's resolve)
// makes stale words of earlier kernels invisible without a memset.  scal: [0] total, [1] launched,
// [2] rows read, [3] scan-timeout flag, then two ticket counters (kernel of epoch k uses k & 1 and
// zeroes the other for the next kernel).
constexpr long long kScanSpin = 1ll << 24;  // look-back spins before giving up (never reached)

__device__ __forceinline__ int l1_ticket(unsigned *tickets, unsigned epoch) {
    __shared__ int t_sh;
    if (threadIdx.x == 0) t_sh = (int)atomicAdd(tickets + (epoch & 1u), 1u);
    __syncthreads();
    const int t = t_sh;
    __syncthreads();
    return t;
}

// exclusive offset of this thread's edge (len: this round's length, clipped in place)
__device__ __forceinline__ int32_t l1_tile_scan(int tile, int ntiles, int32_t &len, unsigned long long *sstat,
                                                unsigned epoch, long long cap, long long *scal) {
    __shared__ int wsum[4];
    __shared__ long long ex_sh;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int v = len;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int wbase = 0, agg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) wbase += k < w ? wsum[k] : 0, agg += wsum[k];
    if (w == 0) {  // wave 0: publish the aggregate, then look back 64 tiles at a time
        const unsigned long long tag = (unsigned long long)epoch << 34;
        long long ex = 0;
        if (tile > 0) {
            if (lane == 0)
                __hip_atomic_store(sstat + tile, tag | (1ull << 32) | (unsigned)agg, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
            long long spins = 0;
            for (int j0 = tile - 1; j0 >= 0; j0 -= 64) {
                const int j = j0 - lane;  // lane l looks at tile j0 - l
                unsigned long long st = 0;
                for (;;) {  // until every looked-at tile has published
                    st = j >= 0 ? __hip_atomic_load(sstat + j, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                : tag | (2ull << 32);
                    if (__ballot((st >> 34) != epoch) == 0ull) break;
                    if (++spins > kScanSpin) {  // cannot happen (tiles are taken in order by running
                        scal[3] = 1;            // workgroups); reported instead of hanging
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                // the nearest inclusive prefix among them ends the look-back: add the values of the
                // lanes up to and including it
                const unsigned long long pre = __ballot(((st >> 32) & 3ull) == 2ull && j >= 0);
                const int stop = pre ? __builtin_ctzll(pre) : 64;
                long long val = (lane <= stop && j >= 0) ? (long long)(st & 0xFFFFFFFFull) : 0;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) val += __shfl_xor(val, o);
                ex += val;
                if (pre || spins > kScanSpin) break;
            }
        }
        if (lane == 0) {
            __hip_atomic_store(sstat + tile, tag | (2ull << 32) | (unsigned long long)(ex + agg), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
            ex_sh = ex;
            if (tile == ntiles - 1) {
                const long long t = ex + agg < cap ? ex + agg : cap;
                scal[0] = t;
                scal[1] += t;
            }
        }
    }
    __syncthreads();
    long long run = ex_sh + wbase + inc - v;
    if (run + v > cap) {  // the clip: this round holds at most cap tests
        len = (int32_t)(run >= cap ? 0 : cap - run);
        run = run < cap ? run : cap;
    }
    return (int32_t)run;
}

// candidate k of an edge: adj(x)\{y} then adj(y)\{x}, each ascending
__device__ __forceinline__ int l1_cand(const L1Edge &g, const int32_t *__restrict__ adj, int k) {
    return k < g.m0 ? adj[g.ax + k + (k >= g.skx)] : adj[g.ay + (k - g.m0) + ((k - g.m0) >= g.sky)];
}

// the screen, one wave per edge (64 candidates per step, ballots): count the candidates it keeps ...
__device__ __forceinline__ L1Edge l1_edge_of(const int32_t *__restrict__ pairs, const int32_t *__restrict__ adj,
                                             const int32_t *__restrict__ adj_off, int e) {
    const int x = pairs[2 * e], y = pairs[2 * e + 1];
    const int ax = adj_off[x], nx = adj_off[x + 1] - ax, ay = adj_off[y], ny = adj_off[y + 1] - ay;
    int skx = find_sorted(adj + ax, nx, y), sky = find_sorted(adj + ay, ny, x);
    const int m0 = skx >= 0 ? nx - 1 : nx, m1 = sky >= 0 ? ny - 1 : ny;
    skx = skx >= 0 ? skx : nx + 1, sky = sky >= 0 ? sky : ny + 1;
    return L1Edge{x, y, m0, m0 + m1, skx, sky, ax, ay, m0 + m1, -1};
}
__global__ __launch_bounds__(256) void ci_l1_screen_count(const int32_t *__restrict__ pairs, int E,
                                                          const int32_t *__restrict__ adj,
                                                          const int32_t *__restrict__ adj_off,
                                                          const double *__restrict__ mi, const int32_t *__restrict__ dims,
                                                          const double *__restrict__ band, int nband, int nv,
                                                          double two_n, int32_t *__restrict__ pcnt) {
    const int lane = threadIdx.x & 63;
    for (int e = blockIdx.x * 4 + (threadIdx.x >> 6); e < E; e += gridDim.x * 4) {  // (whole waves)
        const L1Edge g = l1_edge_of(pairs, adj, adj_off, e);
        const double gxy = mi[l1_pidx(g.x, g.y, nv)];
        int n = 0;
        for (int k0 = 0; k0 < g.L; k0 += 64) {
            const int k = k0 + lane;
            n += __popcll(__ballot(k < g.L && l1_plausible(mi, nv, dims, band, nband, two_n, g.x, g.y, l1_cand(g, adj, k), gxy)));
        }
        if (lane == 0) pcnt[e] = n;
    }
}
// ... and, once ci_l1_setup has placed every edge's list, write the kept positions in order
__global__ __launch_bounds__(256) void ci_l1_screen_fill(const L1Edge *__restrict__ ed, int E,
                                                         const int32_t *__restrict__ adj, const double *__restrict__ mi,
                                                         const int32_t *__restrict__ dims,
                                                         const double *__restrict__ band, int nband, int nv,
                                                         double two_n, int32_t *__restrict__ plist) {
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int e = blockIdx.x * 4 + (threadIdx.x >> 6); e < E; e += gridDim.x * 4) {
        const L1Edge g = ed[e];
        const double gxy = mi[l1_pidx(g.x, g.y, nv)];
        int q = g.pl;
        for (int k0 = 0; k0 < g.L; k0 += 64) {
            const int k = k0 + lane;
            const bool keep = k < g.L && l1_plausible(mi, nv, dims, band, nband, two_n, g.x, g.y, l1_cand(g, adj, k), gxy);
            const unsigned long long m = __ballot(keep);
            if (keep) plist[q + __popcll(m & below)] = k;
            q += __popcll(m);
        }
    }
}

// (also the first round's lengths, chunk0 candidates per edge, and their offsets; both open-count
// ring slots zeroed; with pcnt -- the screen's counts -- each edge's list offset pl first)
__global__ __launch_bounds__(256) void ci_l1_setup(const int32_t *__restrict__ pairs, int E,
                                                   const int32_t *__restrict__ adj,
                                                   const int32_t *__restrict__ adj_off, L1Edge *__restrict__ ed,
                                                   int32_t *__restrict__ pos, uint8_t *__restrict__ st,
                                                   int32_t *__restrict__ sep, long long *__restrict__ counted,
                                                   int chunk0, int32_t *__restrict__ len, int32_t *__restrict__ off,
                                                   unsigned *__restrict__ ring, unsigned long long *__restrict__ sstat,
                                                   long long cap, long long *__restrict__ scal,
                                                   const int32_t *__restrict__ pcnt,
                                                   unsigned long long *__restrict__ sstat2, long long *__restrict__ scal2) {
    constexpr unsigned epoch = 1;
    unsigned *tickets = reinterpret_cast<unsigned *>(scal + 4);
    if (blockIdx.x == 0 && threadIdx.x < 2) ring[threadIdx.x] = 0u;
    if (blockIdx.x == 0 && threadIdx.x == 0) tickets[(epoch + 1) & 1u] = 0u;
    const int ntiles = (E + 255) / 256;
    for (;;) {
        const int tile = l1_ticket(tickets, epoch);
        if (tile >= ntiles) break;
        const int e = tile * 256 + threadIdx.x;
        int32_t l = 0;
        L1Edge g{};
        if (e < E) {
            const int x = pairs[2 * e], y = pairs[2 * e + 1];
            const int ax = adj_off[x], nx = adj_off[x + 1] - ax, ay = adj_off[y], ny = adj_off[y + 1] - ay;
            int skx = find_sorted(adj + ax, nx, y), sky = find_sorted(adj + ay, ny, x);
            const int m0 = skx >= 0 ? nx - 1 : nx, m1 = sky >= 0 ? ny - 1 : ny;
            skx = skx >= 0 ? skx : nx + 1, sky = sky >= 0 ? sky : ny + 1;
            g = L1Edge{x, y, m0, m0 + m1, skx, sky, ax, ay, m0 + m1, -1};
            if (pcnt) g.P = pcnt[e];  // the candidates the screen keeps (ci_l1_screen_count)
        }
        if (pcnt) {  // their positions go to plist[pl .. pl + P) (ci_l1_screen_fill, after this kernel)
            int32_t pcount = e < E ? g.P : 0;
            const int32_t pl = l1_tile_scan(tile, ntiles, pcount, sstat2, epoch, 1ll << 62, scal2);
            if (e < E) g.pl = pl;
        }
        if (e < E) {
            ed[e] = g;
            pos[e] = 0;
            // no candidate left to run: kept, every candidate counted (a dependent test each)
            st[e] = g.P == 0 ? 2 : 0;
            sep[e] = -1;
            counted[e] = g.P == 0 ? g.L : 0;
            l = g.P < chunk0 ? g.P : chunk0;
        }
        const int32_t o = l1_tile_scan(tile, ntiles, l, sstat, epoch, cap, scal);
        if (e < E) len[e] = l, off[e] = o;
    }
}

// one thread per generated test: its edge by binary search over off (edges with len 0 share an
// offset with the next one; the last edge whose off <= t owns t)
__global__ __launch_bounds__(256) void ci_l1_gen(const L1Edge *__restrict__ ed, const int32_t *__restrict__ pos,
                                                 const int32_t *__restrict__ off, int E,
                                                 const long long *__restrict__ total,
                                                 const int32_t *__restrict__ adj, int32_t *__restrict__ items,
                                                 const int32_t *__restrict__ dims,
                                                 unsigned long long *__restrict__ rows_read,
                                                 const int32_t *__restrict__ plist) {
    const long long n = *total;
    // wave-uniform trip count (the row tally below is reduced per wave)
    for (long long wb = (long long)blockIdx.x * 256 + (threadIdx.x & ~63); wb < n; wb += (long long)gridDim.x * 256) {
        const long long t = wb + (threadIdx.x & 63);
        unsigned rows = 0;
        if (t < n) {
        int lo = 0, hi = E;  // last e with off[e] <= t
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (off[mid] <= t) lo = mid;
            else hi = mid;
        }
        const L1Edge g = ed[lo];
        const int j = pos[lo] + (int)(t - off[lo]);
        const int z = l1_cand(g, adj, g.pl < 0 ? j : plist[g.pl + j]);
        items[3 * t] = g.x, items[3 * t + 1] = g.y, items[3 * t + 2] = z;
        rows = dims[g.x] + dims[g.y] + dims[z] - 3;  // mask rows the derived count reads
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) rows += __shfl_xor(rows, o);
        if ((threadIdx.x & 63) == 0 && rows) atomicAdd(rows_read, (unsigned long long)rows);
    }
}

__global__ __launch_bounds__(256) void ci_l1_resolve(const L1Edge *__restrict__ ed, int32_t *__restrict__ pos,
                                                     int32_t *__restrict__ len, int32_t *__restrict__ off,
                                                     uint8_t *__restrict__ st, int32_t *__restrict__ sep,
                                                     long long *__restrict__ counted, const uint8_t *__restrict__ indep,
                                                     const int32_t *__restrict__ items, int E,
                                                     unsigned *__restrict__ open_cnt, unsigned *__restrict__ open_next,
                                                     int next_chunk, unsigned long long *__restrict__ sstat,
                                                     unsigned epoch, long long cap, long long *__restrict__ scal,
                                                     const int32_t *__restrict__ plist) {
    unsigned *tickets = reinterpret_cast<unsigned *>(scal + 4);
    // the next round's open-count slot (its previous value went to the host before this round) and
    // the next kernel's ticket counter
    if (blockIdx.x == 0 && threadIdx.x == 0) *open_next = 0u, tickets[(epoch + 1) & 1u] = 0u;
    const int ntiles = (E + 255) / 256;
    for (;;) {
        const int tile = l1_ticket(tickets, epoch);
        if (tile >= ntiles) break;
        const int e = tile * 256 + threadIdx.x;
        bool open = false;
        if (e < E && st[e] == 0) {
            const int n = len[e], o = off[e];
            int found = -1;
            for (int i = 0; i < n; ++i)
                if (indep[o + i]) {
                    found = i;
                    break;
                }
            const L1Edge g = ed[e];
            if (found >= 0) {  // counted: every candidate up to its position (the screened-out ones dependent)
                st[e] = 1;
                sep[e] = items[3 * (o + found) + 2];
                const int j = pos[e] + found;
                counted[e] = (g.pl < 0 ? j : plist[g.pl + j]) + 1;
            } else {
                pos[e] += n;
                if (pos[e] >= g.P) st[e] = 2, counted[e] = g.L;
                else open = true;
            }
        }
        // the next round's length of this edge and, through the tile scan, its offset
        int32_t l = 0;
        if (e < E && open) {
            const int left = ed[e].P - pos[e];
            l = left < next_chunk ? left : next_chunk;
        }
        const int32_t o = l1_tile_scan(tile, ntiles, l, sstat, epoch, cap, scal);
        if (e < E) len[e] = l, off[e] = o;
        const unsigned nopen = (unsigned)__popcll(__ballot(open));  // one atomic per wave
        if ((threadIdx.x & 63) == 0 && nopen) atomicAdd(open_cnt, nopen);
    }
}

}  // namespace

// bad[0] = 1 and bad[1] = v + 1 (some such v) if any code of variable v is >= dims[v]
static __global__ __launch_bounds__(256) void ci_cols_check(const uint8_t *__restrict__ cols, const int32_t *__restrict__ dims,
                                                     int nvars, long long N, int *__restrict__ bad) {
    for (int v = blockIdx.y; v < nvars; v += gridDim.y) {
        const uint8_t *c = cols + (size_t)v * N;
        const int d = dims[v];
        bool b = false;
        for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < N; k += (long long)gridDim.x * 256)
            b |= c[k] >= d;
        if (b) {
            bad[0] = 1;
            bad[1] = v + 1;
        }
    }
}

extern "C" hipError_t fbn_ci_cols_check(const uint8_t *cols, const int32_t *dims, int nvars, long long N, int *bad,
                                        hipStream_t s) {
    const long long bx = (N + 255) / 256;
    const dim3 grid((unsigned)(bx < 16 ? bx : 16), (unsigned)(nvars < 4096 ? nvars : 4096));
    hipLaunchKernelGGL(ci_cols_check, grid, dim3(256), 0, s, cols, dims, nvars, N, bad);
    return hipGetLastError();
}

// sample count of every mask row (variable v, value a): one wave per row
static __global__ __launch_bounds__(256) void ci_bits_rowcount(const uint32_t *__restrict__ bits, long long rows,
                                                               long long W, int32_t *__restrict__ rowcnt) {
    const int lane = threadIdx.x & 63;
    for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
        uint32_t v = 0;
        for (long long w = lane; w < W; w += 64) v += __builtin_popcount(bits[r * W + w]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) rowcnt[r] = (int32_t)v;
    }
}

extern "C" hipError_t fbn_ci_bits_rowcount(const uint32_t *bits, long long rows, long long W, int32_t *rowcnt,
                                           hipStream_t s) {
    const long long g = (rows + 3) / 4;
    hipLaunchKernelGGL(ci_bits_rowcount, dim3((unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096)), dim3(256), 0, s, bits,
                       rows, W, rowcnt);
    return hipGetLastError();
}

extern "C" hipError_t fbn_ci_bits_build(const uint8_t *cols, const int32_t *dims, const int32_t *row0, long long N,
                                        long long W, int nvars, uint32_t *bits, hipStream_t s) {
    const long long total = (long long)nvars * W;
    const int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
    hipLaunchKernelGGL(ci_bits_build, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, cols, dims, row0, N, W, nvars, bits);
    return hipGetLastError();
}

// block size per state-count class (the host builds tasks with these)
extern "C" int fbn_ci_pair_block(int d) { return d - 1 <= 1 ? 4 : (d - 1 == 2 ? 3 : 2); }

extern "C" hipError_t fbn_ci_bits_pairs_tiled(const uint32_t *bits, const int32_t *row0, const int32_t *rowcnt,
                                              long long W, const int32_t *tasks, long long ntasks, int nvars,
                                              long long t0, long long t1, int32_t *counts, int32_t *pairtab,
                                              int num_cu, hipStream_t s) {
    const long long g = (ntasks + 3) / 4, cap = (long long)num_cu * 8;
    if (ntasks > 0)
        hipLaunchKernelGGL(ci_bits_pairs_tiled, dim3((unsigned)(g < cap ? g : cap)), dim3(256), 0, s, bits, row0,
                           rowcnt, W, tasks, ntasks, nvars, t0, t1, counts, pairtab);
    return hipGetLastError();
}

extern "C" size_t fbn_ci_l1_edge_bytes(void) { return sizeof(L1Edge); }

// ---- level 0 -> level 1 without the host: the pairs level 0 kept (decision flag 0 over the
// implicit complete graph, pair (i < j) at i*n - i(i+1)/2 + j-i-1) become the level-1 edge list
// (lexicographic, as the host's vec_edges) and the CSR adjacency (each list ascending: the lower
// neighbours, then the upper ones -- the order the host builds from the edge list).  One wave per
// variable, 64 flags per step with a ballot.
__device__ __forceinline__ long long kept_pidx(int i, int j, int n) {
    return (long long)i * n - (long long)i * (i + 1) / 2 + (j - i - 1);
}
__global__ __launch_bounds__(256) void ci_kept_count(const uint8_t *__restrict__ indep, int n, int32_t *__restrict__ low,
                                                     int32_t *__restrict__ up) {
    const int lane = threadIdx.x & 63, v = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= n) return;  // (whole wave)
    int lo = 0, hi = 0;
    for (int u0 = 0; u0 < v; u0 += 64) {
        const int u = u0 + lane;
        lo += __popcll(__ballot(u < v && indep[kept_pidx(u, v, n)] == 0));
    }
    for (int w0 = v + 1; w0 < n; w0 += 64) {
        const int w = w0 + lane;
        hi += __popcll(__ballot(w < n && indep[kept_pidx(v, w, n)] == 0));
    }
    if (lane == 0) low[v] = lo, up[v] = hi;
}
// one workgroup: off = exclusive scan of the degrees (off[n] = 2E), upoff = exclusive scan of the
// upper counts; scal[0] = E, scal[1] = the level's candidate sets sum_e (deg x + deg y - 2) =
// sum_v deg(v)^2 - 2E
__global__ __launch_bounds__(1024) void ci_kept_scan(const int32_t *__restrict__ low, const int32_t *__restrict__ up,
                                                     int n, int32_t *__restrict__ off, int32_t *__restrict__ upoff,
                                                     long long *__restrict__ scal) {
    __shared__ long long sd[1024], su[1024];
    __shared__ long long carry_d, carry_u, sq;
    const int t = threadIdx.x;
    if (t == 0) carry_d = carry_u = sq = 0;
    __syncthreads();
    for (int b = 0; b < n; b += 1024) {
        const int v = b + t;
        const long long d = v < n ? (long long)low[v] + up[v] : 0, u = v < n ? up[v] : 0;
        sd[t] = d, su[t] = u;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
            const long long xd = t >= o ? sd[t - o] : 0, xu = t >= o ? su[t - o] : 0;
            __syncthreads();
            sd[t] += xd, su[t] += xu;
            __syncthreads();
        }
        if (v < n) off[v] = (int32_t)(carry_d + sd[t] - d), upoff[v] = (int32_t)(carry_u + su[t] - u);
        if (d) atomicAdd((unsigned long long *)&sq, (unsigned long long)(d * d));
        __syncthreads();
        if (t == 1023) carry_d += sd[1023], carry_u += su[1023];
        __syncthreads();
    }
    if (t == 0) {
        off[n] = (int32_t)carry_d;
        scal[0] = carry_u;
        scal[1] = sq - 2 * carry_u;
    }
}
__global__ __launch_bounds__(256) void ci_kept_fill(const uint8_t *__restrict__ indep, int n,
                                                    const int32_t *__restrict__ off, const int32_t *__restrict__ upoff,
                                                    int32_t *__restrict__ adj, int32_t *__restrict__ pairs) {
    const int lane = threadIdx.x & 63, v = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= n) return;
    const unsigned long long below = (1ull << lane) - 1ull;
    int r = off[v], q = upoff[v];
    for (int u0 = 0; u0 < v; u0 += 64) {
        const int u = u0 + lane;
        const bool k = u < v && indep[kept_pidx(u, v, n)] == 0;
        const unsigned long long m = __ballot(k);
        if (k) adj[r + __popcll(m & below)] = u;
        r += __popcll(m);
    }
    for (int w0 = v + 1; w0 < n; w0 += 64) {
        const int w = w0 + lane;
        const bool k = w < n && indep[kept_pidx(v, w, n)] == 0;
        const unsigned long long m = __ballot(k);
        if (k) {
            const int i = __popcll(m & below);
            adj[r + i] = w;
            pairs[2 * (q + i)] = v, pairs[2 * (q + i) + 1] = w;
        }
        r += __popcll(m), q += __popcll(m);
    }
}
// level-1 results straight into pinned host memory (one kernel instead of four DMA copies): the
// removal flag (status 1) and the sepset (or -1) of every edge, per-workgroup sums of the counted
// tests in `part`; ci_l1_results_tail adds them up and copies the launched count and the scan flag
__global__ __launch_bounds__(256) void ci_l1_results(const uint8_t *__restrict__ st, const int32_t *__restrict__ sep,
                                                     const long long *__restrict__ cnt, int E, char *__restrict__ h_rm,
                                                     int32_t *__restrict__ h_sep, long long *__restrict__ part) {
    __shared__ long long ws[4];
    long long acc = 0;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) {
        const bool rm = st[e] == 1;
        h_rm[e] = rm ? 1 : 0;
        h_sep[e] = rm ? sep[e] : -1;
        acc += cnt[e];
    }
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(64) void ci_l1_results_tail(const long long *__restrict__ part, int nparts,
                                                         const long long *__restrict__ scal, long long *__restrict__ h_sc) {
    long long acc = 0;
    for (int i = threadIdx.x; i < nparts; i += 64) acc += part[i];
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    // (scal[11]: the information screen's scan flag, ci_l1_setup's second scan at scal + 8)
    if (threadIdx.x == 0) h_sc[0] = acc, h_sc[1] = scal[1], h_sc[2] = scal[2], h_sc[3] = scal[3] | scal[11];
}
// h_sc: 4 long longs (counted, launched, rows read, scan flag); part: >= 256 long longs of scratch
extern "C" hipError_t fbn_ci_l1_results(const uint8_t *st, const int32_t *sep, const long long *cnt, int E,
                                        const long long *scal, char *h_rm, int32_t *h_sep, long long *h_sc,
                                        long long *part, hipStream_t s) {
    const int g = std::max(1, std::min(256, (E + 255) / 256));
    hipLaunchKernelGGL(ci_l1_results, dim3(g), dim3(256), 0, s, st, sep, cnt, E, h_rm, h_sep, part);
    hipLaunchKernelGGL(ci_l1_results_tail, dim3(1), dim3(64), 0, s, part, g, scal, h_sc);
    return hipGetLastError();
}

// low / up: n ints of scratch each; scal: 2 long longs (E, candidate sets)
extern "C" hipError_t fbn_ci_kept_csr(const uint8_t *indep, int n, int32_t *low, int32_t *up, int32_t *off,
                                      int32_t *upoff, int32_t *adj, int32_t *pairs, long long *scal, hipStream_t s) {
    const dim3 g((unsigned)((n + 3) / 4));
    hipLaunchKernelGGL(ci_kept_count, g, dim3(256), 0, s, indep, n, low, up);
    hipLaunchKernelGGL(ci_kept_scan, dim3(1), dim3(1024), 0, s, low, up, n, off, upoff, scal);
    hipLaunchKernelGGL(ci_kept_fill, g, dim3(256), 0, s, indep, n, off, upoff, adj, pairs);
    return hipGetLastError();
}

// mi != nullptr: the information screen first over mi = every pair's level-0 G^2 (indexed by pair;
// computed here from the pair tables when mi_from_tables), band for the level's alpha, two_n = 2N,
// pcnt >= E ints, plist >= the level's candidate sets, sstat2 / scal2 a second tile-status array
// (>= tiles) and 4 long longs)
extern "C" hipError_t fbn_ci_l1_setup(const int32_t *pairs, int E, const int32_t *adj, const int32_t *adj_off,
                                      void *ed, int32_t *pos, uint8_t *st, int32_t *sep, long long *counted,
                                      int chunk0, int32_t *len, int32_t *off, unsigned *ring,
                                      unsigned long long *sstat, long long cap, long long *scal, int num_cu,
                                      const int32_t *pairtab, double *mi, int mi_from_tables, const int32_t *dims,
                                      const double *band, int nband, int nv, double two_n, int32_t *pcnt,
                                      int32_t *plist, unsigned long long *sstat2, long long *scal2, hipStream_t s) {
    const int ntiles = (E + 255) / 256;
    if (E <= 0) return hipSuccess;
    const unsigned gw = (unsigned)std::min((E + 3) / 4, num_cu * 8);  // one wave per edge
    if (mi) {
        const long long P = (long long)nv * (nv - 1) / 2, b = (P + 255) / 256;
        if (mi_from_tables)
            hipLaunchKernelGGL(ci_pair_g2, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, s, pairtab, dims, nv, P, mi);
        hipLaunchKernelGGL(ci_l1_screen_count, dim3(gw), dim3(256), 0, s, pairs, E, adj, adj_off, (const double *)mi,
                           dims, band, nband, nv, two_n, pcnt);
    }
    hipLaunchKernelGGL(ci_l1_setup, dim3((unsigned)std::min(ntiles, num_cu * 4)), dim3(256), 0, s, pairs, E, adj,
                       adj_off, (L1Edge *)ed, pos, st, sep, counted, chunk0, len, off, ring, sstat, cap, scal,
                       mi ? (const int32_t *)pcnt : nullptr, sstat2, scal2);
    if (mi)
        hipLaunchKernelGGL(ci_l1_screen_fill, dim3(gw), dim3(256), 0, s, (const L1Edge *)ed, E, adj, (const double *)mi,
                           dims, band, nband, nv, two_n, plist);
    return hipGetLastError();
}

// one round (its lengths and offsets come from ci_l1_setup or the previous round's resolve):
// generation, counting, G^2 / decisions, resolution + the next round's lengths and offsets for
// next_chunk; scal[0] = the round's test count (device), open_cnt += edges still open after it,
// *open_next = 0; epoch = round + 2
extern "C" hipError_t fbn_ci_l1_round(const uint32_t *bits, const int32_t *dims, const int32_t *row0, long long W,
                                      const int32_t *adj, const int32_t *pairtab, int nvars, void *edv, int32_t *pos,
                                      uint8_t *st, int32_t *sep, long long *counted, int32_t *len, int32_t *off,
                                      int E, long long cap, long long *scal, int32_t *items, int32_t *counts,
                                      int32_t *df, uint8_t *indep, double alpha, unsigned long long *stats,
                                      const double *band, int nband, unsigned *open_cnt, int num_cu,
                                      unsigned *open_next, int next_chunk, unsigned long long *sstat, unsigned epoch,
                                      const int32_t *plist, hipStream_t s) {
    const L1Edge *ed = (const L1Edge *)edv;
    const long long gcap = (long long)num_cu * 8;
    const long long gt = (cap + 255) / 256;
    const dim3 gT((unsigned)(gt < gcap ? gt : gcap));
    const long long gw = (cap + 3) / 4;
    const dim3 gW((unsigned)(gw < gcap ? gw : gcap));
    const int ntiles = (E + 255) / 256;
    const long long *total = scal;
    unsigned long long *rows_read = reinterpret_cast<unsigned long long *>(scal + 2);
    hipLaunchKernelGGL(ci_l1_gen, gT, dim3(256), 0, s, ed, pos, off, E, total, adj, items, dims, rows_read, plist);
    hipLaunchKernelGGL(ci_bits_count_derived, gW, dim3(256), 0, s, bits, dims, row0, (const int32_t *)items, W, cap,
                       counts, pairtab, nvars, 1, total);
    // four lanes per test: the screened rounds are small (a few thousand to ~27k tests on config 5),
    // where the lane-per-test kernel's single latency chain per test dominated (config 5: 0.22 ->
    // 0.13 ms of G^2 per run; FBN_PC_L1_G2Q=0: lane per test)
    static const bool quad = !(getenv("FBN_PC_L1_G2Q") && atoi(getenv("FBN_PC_L1_G2Q")) == 0);
    const long long gq = (cap + kG2TestsPerBlock - 1) / kG2TestsPerBlock;
    hipLaunchKernelGGL((quad ? ci_bits_g2q<1> : ci_bits_g2<1>), quad ? dim3((unsigned)(gq < gcap ? gq : gcap)) : gT,
                       dim3(256), 0, s, (const int32_t *)counts, dims, (const int32_t *)items, cap, alpha,
                       (double *)nullptr, df, (double *)nullptr, indep, (int32_t *)nullptr, stats, nvars, 0ll, band,
                       nband, total);
    hipLaunchKernelGGL(ci_l1_resolve, dim3((unsigned)std::min(ntiles, num_cu * 4)), dim3(256), 0, s, ed, pos, len,
                       off, st, sep, counted, (const uint8_t *)indep, (const int32_t *)items, E, open_cnt, open_next,
                       next_chunk, sstat, epoch, cap, scal, plist);
    return hipGetLastError();
}

// one byte per (leading row, sample): out[r][s] = [cols[v][s] == a] for leading row r = lead0[v] + a
// (a < dims[v] - 1), samples N..Npad-1 zero -- the int8 operand of the level-0 Gram as a library
// GEMM (capi.hip); 4 samples per thread
__global__ __launch_bounds__(256) void ci_onehot_build(const uint8_t *__restrict__ cols, const int32_t *__restrict__ dims,
                                                       const int32_t *__restrict__ lead0, long long N, long long Npad,
                                                       int nvars, int8_t *__restrict__ out) {
    const long long n4 = Npad / 4;
    for (int v = blockIdx.y; v < nvars; v += gridDim.y) {
        const int m = dims[v] - 1;
        if (m <= 0) continue;
        const uint8_t *c = cols + (size_t)v * N;
        int8_t *o = out + (size_t)lead0[v] * Npad;
        for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long long)gridDim.x * 256) {
            uint8_t b[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) b[k] = 4 * q + k < N ? c[4 * q + k] : 0xFF;
            for (int a = 0; a < m; ++a) {
                uint32_t w = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) w |= (uint32_t)(b[k] == a) << (8 * k);
                reinterpret_cast<uint32_t *>(o + (size_t)a * Npad)[q] = w;
            }
        }
    }
}

extern "C" hipError_t fbn_ci_onehot_build(const uint8_t *cols, const int32_t *dims, const int32_t *lead0, long long N,
                                          long long Npad, int nvars, int8_t *out, hipStream_t s) {
    const long long g = (Npad / 4 + 255) / 256;
    hipLaunchKernelGGL(ci_onehot_build, dim3((unsigned)(g < 64 ? g : 64), (unsigned)(nvars < 1024 ? nvars : 1024)),
                       dim3(256), 0, s, cols, dims, lead0, N, Npad, nvars, out);
    return hipGetLastError();
}

// out[i] = sum over np planes of planes[p * n + i] (split-K partial Grams; integers)
__global__ __launch_bounds__(256) void ci_sum_planes(const int4 *__restrict__ planes, int np, long long n4,
                                                     int4 *__restrict__ out) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        int4 a = planes[i];
        for (int p = 1; p < np; ++p) {
            const int4 b = planes[p * n4 + i];
            a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
        }
        out[i] = a;
    }
}
__global__ __launch_bounds__(256) void ci_sum_planes_tail(const int32_t *__restrict__ planes, int np, long long n,
                                                          long long from, int32_t *__restrict__ out) {
    const long long i = from + (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int32_t a = 0;
    for (int p = 0; p < np; ++p) a += planes[p * n + i];
    out[i] = a;
}

extern "C" hipError_t fbn_ci_sum_planes(const int32_t *planes, int np, long long n, int32_t *out, hipStream_t s) {
    // the int4 path needs every plane 16-byte aligned: n % 4 == 0 (and 16-byte aligned bases)
    const bool vec = n % 4 == 0 && ((uintptr_t)planes % 16) == 0 && ((uintptr_t)out % 16) == 0;
    const long long n4 = vec ? n / 4 : 0;
    if (n4) {
        const long long g = (n4 + 255) / 256;
        hipLaunchKernelGGL(ci_sum_planes, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, s,
                           (const int4 *)planes, np, n4, (int4 *)out);
    }
    const long long rest = n - 4 * n4;
    if (rest > 0)
        hipLaunchKernelGGL(ci_sum_planes_tail, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, s, planes, np, n,
                           4 * n4, out);
    return hipGetLastError();
}

extern "C" int fbn_ci_gram_task_ints(void) { return kGramTaskInts; }

extern "C" hipError_t fbn_ci_gram(const uint32_t *bits, long long W, const int32_t *rl, const int32_t *tasks,
                                  long long ntasks, int masked, int32_t *out, int num_cu, hipStream_t s) {
    const long long cap = (long long)num_cu * 32;
    const dim3 g((unsigned)(ntasks < cap ? ntasks : cap));
    if (ntasks <= 0) return hipSuccess;
    static const int xcd = getenv("FBN_CI_GRAM_XCD") ? atoi(getenv("FBN_CI_GRAM_XCD")) : 1;
    if (masked) hipLaunchKernelGGL(ci_bits_gram<true>, g, dim3(64), 0, s, bits, W, rl, tasks, ntasks, out, xcd);
    else hipLaunchKernelGGL(ci_bits_gram<false>, g, dim3(64), 0, s, bits, W, rl, tasks, ntasks, out, xcd);
    return hipGetLastError();
}

extern "C" hipError_t fbn_ci_gram_pairs(const int32_t *G, long long ld, const int32_t *lead0, const int32_t *dims,
                                        const int32_t *row0, const int32_t *rowcnt, long long t0, long long n,
                                        int nvars, int32_t *counts, int32_t *pairtab, int num_cu, hipStream_t s) {
    const long long g = (n + 255) / 256, cap = (long long)num_cu * 8;
    if (n > 0)
        hipLaunchKernelGGL(ci_bits_gram_pairs, dim3((unsigned)(g < cap ? g : cap)), dim3(256), 0, s, G, ld, lead0,
                           dims, row0, rowcnt, t0, n, nvars, counts, pairtab);
    return hipGetLastError();
}

extern "C" hipError_t fbn_ci_gram_triples(const int32_t *G, const long long *goff, const int32_t *gR,
                                          const int32_t *adj, const int32_t *adj_off, const int32_t *loff,
                                          const int32_t *dims, const int32_t *items, long long n, int32_t *counts,
                                          const int32_t *pairtab, int nvars, int num_cu, hipStream_t s) {
    const long long g = (n + 255) / 256, cap = (long long)num_cu * 8;
    if (n > 0)
        hipLaunchKernelGGL(ci_bits_gram_triples, dim3((unsigned)(g < cap ? g : cap)), dim3(256), 0, s, G, goff, gR,
                           adj, adj_off, loff, dims, items, n, counts, pairtab, nvars);
    return hipGetLastError();
}

extern "C" hipError_t fbn_ci_bits_launch(const uint32_t *bits, const int32_t *dims, const int32_t *row0,
                                         const int32_t *items, long long W, long long n, int d, double alpha,
                                         double *g2, int32_t *df, double *p, uint8_t *indep, int32_t *counts,
                                         int32_t *counts0, unsigned long long *stats, const int32_t *rowcnt,
                                         int32_t *pairtab, int pmode, int nvars, int num_cu, long long t0,
                                         int counted, const double *band, int nband, hipStream_t s) {
    const long long g1 = (n + 3) / 4, cap = (long long)num_cu * 8;
    // launches too small to fill the chip with a lane per test (ALARM's 8.7k level-1 tests: 137
    // waves on 1024 SIMDs) take four lanes per test, which cuts each test's latency chain ~4x
    const bool quad = n <= kG2QuadMax;
    const long long g2g = quad ? (n + kG2TestsPerBlock - 1) / kG2TestsPerBlock : (n + 255) / 256;
    const dim3 b1((unsigned)(g1 < cap ? g1 : cap)), b2((unsigned)(g2g < cap ? g2g : cap));
    if (d == 0) {
        if (!counted)  // counted = 1: the counts are already in place (ci_bits_pairs_tiled)
            hipLaunchKernelGGL(ci_bits_count<0>, b1, dim3(256), 0, s, bits, dims, row0, items, W, n, counts, rowcnt,
                               pmode == 1 ? pairtab : nullptr, nvars, t0);
        hipLaunchKernelGGL((quad ? ci_bits_g2q<0> : ci_bits_g2<0>), b2, dim3(256), 0, s, counts, dims, items, n,
                           alpha, g2, df, p, indep, counts0, stats, nvars, t0, band, nband, (const long long *)nullptr);
    } else if (d == 1) {
        // FBN_CI_L1MODE = 0: plain grid stride instead of the XCD-contiguous split
        static const int l1mode = getenv("FBN_CI_L1MODE") ? atoi(getenv("FBN_CI_L1MODE")) : 1;
        if (counted) {
            // the counts are already in place (ci_bits_gram_triples)
        } else if (pmode == 2) {
            hipLaunchKernelGGL(ci_bits_count_derived, b1, dim3(256), 0, s, bits, dims, row0, items, W, n, counts,
                               (const int32_t *)pairtab, nvars, l1mode == 1 ? 1 : 0, (const long long *)nullptr);
        }
        else
            hipLaunchKernelGGL(ci_bits_count<1>, b1, dim3(256), 0, s, bits, dims, row0, items, W, n, counts, rowcnt,
                               nullptr, nvars, 0ll);
        hipLaunchKernelGGL((quad ? ci_bits_g2q<1> : ci_bits_g2<1>), b2, dim3(256), 0, s, counts, dims, items, n,
                           alpha, g2, df, p, indep, counts0, stats, nvars, 0ll, band, nband, (const long long *)nullptr);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
