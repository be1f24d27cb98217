// pc_small.hip -- the whole PC-stable skeleton search of a small graph in ONE launch (gfx950).
//
// Why: on ALARM-5000 (37 variables, 5000 samples; BASELINE config 3) a level is a few microseconds
// of CI tests, and the host-driven level loop spent more time in round trips (event wait, host
// bookkeeping, next launch) than in kernels.  Here the level loop itself runs on the device:
//
//   for d = 0, 1, ...:                                    (src/PCStable.cpp:49-200, SearchAtDepth
//     every workgroup rebuilds the level's edge list from the adjacency snapshot in LDS   :209-328)
//       (vec_edges order = lexicographic (x < y) pairs of the skeleton, src/Network.cpp:346-358);
//     every candidate set of every edge is a test t (edge-major, then side, then ChoiceGenerator
//       order: the d-subsets of adj(x)\{y} in lexicographic order, then those of adj(y)\{x},
//       CheckEdge src/PCStable.cpp:339-470, ChoiceGenerator src/ChoiceGenerator.cpp:14-85);
//     tests are counted and decided (d <= 1: one wave per test on the bit-sliced store, level 1
//       deriving the last value of x, y and z from the level-0 pair tables; d = 2: one wave per
//       test, d = 3, 4: one workgroup per test, LDS histograms of the 2-bit packed columns -- Counts2D/Counts3D,
//       src/CellTable.cpp:23-91,226-291,430-455; G^2 / df / p as ComputeGSquareXY/XYZ,
//       src/IndependenceTest.cpp:65-155,295-364);
//     an independent test does atomicMax(first[d][edge], ~its index within the edge): the edge's
//       first independent set in the reference's sequential order is the minimum (speculative
//       tests beyond it are evaluated but not counted: counted = first + 1, else every set);
//     ONE grid barrier; every workgroup applies the removals to its own LDS adjacency (removals
//       after the level, src/PCStable.cpp:310-326) and evaluates FreeDegree (:557-563);
//       workgroup 0 writes the level's counts, adjacency and sepsets into the pinned result.
//
// Sizes: <= 64 variables (adjacency = one u64 each), every state count <= 4, levels <= 4 and
// <= 2^22 candidate sets per level; a level outside those hands the search to the host driver
// (pc_driver.cpp) at that level.  Synchronisation follows MI355X_MICROARCH.md's barrier-xcd form:
// per-group arrival counters (group = blockIdx % 8), the last arriver of a group adds to the top
// counter, every workgroup polls relaxed with s_sleep; the data crossing workgroups moves through
// agent-coherent accesses, so the barrier carries no cache-maintenance fence (see grid_barrier);
// every spin bounded (a timed-out launch reports status 1 and exits; the host then runs the search
// on its level loop).  The launch is plain by default: the host checks first that the grid fits
// the occupancy (hipOccupancyMaxActiveBlocksPerMultiprocessor) and falls back to its level loop if
// not, and the bounded spin covers a grid that is still not co-resident; FBN_PC_SMALL_COOP=1 selects
// hipLaunchCooperativeKernel, which refuses such a grid at launch.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ci_chisq.h"
#include "pc_small.h"

using namespace fbn;

namespace {

constexpr int BS = 512;             // threads per workgroup, one workgroup per CU
constexpr int NWAVE = BS / 64;
constexpr int kHistCells = 4096;    // 4^(kSmallMaxD + 2)
constexpr int kMaxZ = 256;          // 4^kSmallMaxD conditioning configurations
constexpr int kTermChunk = 1024;
constexpr int kGroups = 8;          // barrier groups (blockIdx % 8: the XCD when dispatch is round-robin)
constexpr long long kSpinTicks = 200000000ll;  // wall_clock64 ticks (100 MHz): 2 s per barrier (default)

typedef __attribute__((ext_vector_type(4))) unsigned u4;

constexpr int kWaveHist = 2048;    // per-wave region of the one-wave histogram tests (d = 2, 3)
// One-wave levels (1, 2) run in two parts: A = the first spec_a candidate sets of every edge
// (about one round of the grid's waves on ALARM-5000), then B = the rest, edge-major.  A part-B test
// first checks whether its edge already has an independent set at a lower index (published by
// every independent test as it happens, not at the end of the level) and is skipped if so: it
// could never be the edge's first.  Counts, removals and sepsets are those of full speculation.
// (part-A width: PcSmallArgs::spec_a, 8 candidate sets per edge by default)

struct Lds {
    // per-run constants staged once: state counts, first mask row and per-row sample counts of
    // every variable, the decision band
    int32_t dims[kSmallMaxVars], row0[kSmallMaxVars], rowcnt[4 * kSmallMaxVars];
    double band[2 * 256 + 1];
    uint64_t adj[kSmallMaxVars];
    int32_t rowoff[kSmallMaxVars + 1];     // edges of rows before x
    int32_t eoff[kSmallMaxEdges + 1];      // part A: first test of each edge (its first spec_a candidates)
    int32_t eoffB[kSmallMaxEdges + 1];     // part B: first test of each edge's remaining candidates
    int32_t TA;                            // tests in part A
    int32_t next;                          // one-wave levels: this workgroup's next test (dynamic)
    uint8_t ex[kSmallMaxEdges], ey[kSmallMaxEdges], rm[kSmallMaxEdges];
    int32_t binom[kSmallMaxVars + 1][kSmallMaxD + 1];
    int32_t wscan[NWAVE];
    long long wsum[NWAVE];
    unsigned long long wst[NWAVE][3];  // per-wave statistics of a level: min margin bits, near, launched
    int32_t E;
    long long T;
    int flag;
    // one workgroup-wide test (d >= 2)
    int32_t hist[kHistCells];
    int32_t ni[kMaxZ * 4], nj[kMaxZ * 4], nk[kMaxZ], dfp[kMaxZ];
    double term[kTermChunk];
    double red[2 * NWAVE];
    int redi[NWAVE];
    int32_t whist[NWAVE][kWaveHist];  // one test per wave (d = 2, 3): table + margins
    unsigned bfirst[kSmallMaxEdges];   // this workgroup's first independent candidate per edge
    unsigned long long ph[NWAVE][4];   // diagnostic (trace): cycles per test phase, per wave
    int32_t wtab[NWAVE][64];  // one test per wave (d <= 1): the wave's table
    int32_t waux[NWAVE][64];  // ... and its margins (sample counts / pair tables)
    int dec;
    double g2;
};

__device__ __forceinline__ int popc64(uint64_t v) { return __popcll(v); }
// agent-coherent (sc1) accesses of data one workgroup hands to another (see grid_barrier)
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- wave-wide reductions on DPP (VALU lane moves, no LDS round trip): an inclusive scan inside
// each 16-lane row (row_shr 1, 2, 4, 8 with zeros shifted in), then row_bcast:15 / :31 carry the
// row totals up, lane 63 holds the wave total; readlane broadcasts it (a wave-uniform value)
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i32(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWS, 0xf, CTRL < 0x140);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = dpp_i32<CTRL, ROWS>((int)(unsigned)b), hi = dpp_i32<CTRL, ROWS>((int)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ int wsum_i32(int x) {
    x += dpp_i32<0x111, 0xf>(x);
    x += dpp_i32<0x112, 0xf>(x);
    x += dpp_i32<0x114, 0xf>(x);
    x += dpp_i32<0x118, 0xf>(x);
    x += dpp_i32<0x142, 0xa>(x);
    x += dpp_i32<0x143, 0xc>(x);
    return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ double wsum_f64(double x) {
    x += dpp_f64<0x111, 0xf>(x);
    x += dpp_f64<0x112, 0xf>(x);
    x += dpp_f64<0x114, 0xf>(x);
    x += dpp_f64<0x118, 0xf>(x);
    x += dpp_f64<0x142, 0xa>(x);
    x += dpp_f64<0x143, 0xc>(x);
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63),
                   hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ long long wsum_i64(long long x) {
    // 64-bit sums of small per-lane values: the two halves summed separately, carries folded
    const unsigned long long u = (unsigned long long)x;
    const long long lo = (long long)(unsigned)wsum_i32((int)(u & 0xFFFFu)) +
                         ((long long)wsum_i32((int)((u >> 16) & 0xFFFFu)) << 16);
    return lo + ((long long)wsum_i32((int)(u >> 32)) << 32);
}

// the k-th (0-based) set bit of m
__device__ __forceinline__ int select_bit(uint64_t m, int k) {
    for (int j = 0; j < k; ++j) m &= m - 1;
    return __ffsll((unsigned long long)m) - 1;
}

__device__ __forceinline__ int binom_l(const Lds &L, int m, int k) {
    return (m < 0 || k < 0 || m < k) ? 0 : L.binom[m][k];
}

// test k of edge (x, y) at level d >= 1 -> its conditioning set z[0..d-1] (ascending): sets of
// adj(x)\{y} first, then of adj(y)\{x}; lexicographic unranking = ChoiceGenerator::Next order
__device__ __forceinline__ void unrank(const Lds &L, int x, int y, int d, int k, int *z) {
    const uint64_t ax = L.adj[x] & ~(1ull << y), ay = L.adj[y] & ~(1ull << x);
    const int m0 = popc64(ax);
    const int c0 = binom_l(L, m0, d);
    uint64_t base = ax;
    int m = m0;
    if (k >= c0) base = ay, m = popc64(ay), k -= c0;
    int p = 0;
    for (int i = 0; i < d; ++i) {
        while (true) {
            const int cnt = binom_l(L, m - p - 1, d - i - 1);
            if (k < cnt) break;
            k -= cnt;
            ++p;
        }
        const int v = select_bit(base, p);
        z[i] = v < 0 ? 0 : v;  // (never: k < C(m, d) by construction; no out-of-range variable either way)
        ++p;
    }
}

__device__ __forceinline__ int pair_index(int n, int x, int y) {  // x < y
    return x * n - x * (x + 1) / 2 + (y - x - 1);
}

// ---- grid barrier (barrier-xcd form), phase = 1, 2, ...
// Everything one workgroup hands to another crosses through agent-coherent accesses (sc1: the
// first[] atomics, the level-0 pair tables and the statistics slots as relaxed agent-scope atomic
// stores / loads), so the barrier needs no release / acquire fence: on MI355X those are an L2
// writeback and an L2 invalidate per arriving workgroup (each XCD has its own L2), ~4 us per level
// and a cold L2 for the next level's column reads.  What it does need is that every such store has
// completed (vmcnt(0) in every wave) before the workgroup arrives.
struct Barrier {
    unsigned *grp;   // kGroups arrival counters, each on its own 64-B line (stride 16)
    unsigned *top;   // groups done
    int nblocks;
    long long spin;  // wall_clock64 ticks a workgroup waits at one barrier before giving up
};

__device__ bool grid_barrier(const Barrier &B, unsigned phase, Lds &L) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int g = blockIdx.x % kGroups;
        const int ngroups = B.nblocks < kGroups ? B.nblocks : kGroups;
        const unsigned gsize = (unsigned)((B.nblocks - g + kGroups - 1) / kGroups);
        const unsigned old = __hip_atomic_fetch_add(B.grp + 16 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == phase * gsize - 1)  // last of its group in this phase: the group arrives
            __hip_atomic_fetch_add(B.top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = phase * (unsigned)ngroups;
        const long long t0 = wall_clock64();
        int ok = 1;
        while (__hip_atomic_load(B.top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > B.spin) {
                ok = 0;
                break;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        L.flag = ok;
    }
    __syncthreads();
    return L.flag != 0;
}

// this launch's first independent candidate of edge e at level d (~0u: none): first[] words of
// earlier launches carry another epoch
__device__ __forceinline__ unsigned first_of(const PcSmallArgs &A, int d, int e) {
    const unsigned long long v =
        __hip_atomic_load(A.first + (size_t)d * kSmallMaxEdges + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (unsigned)(v >> 32) == A.epoch ? ~(unsigned)v : ~0u;
}

// ---- block-wide helpers
__device__ __forceinline__ long long block_sum_ll(long long v, Lds &L) {
    v = wsum_i64(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) L.wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    long long s = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) s += L.wsum[w];
    return s;
}

__device__ __forceinline__ unsigned long long block_min_u64(unsigned long long v, Lds &L) {
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long u = __shfl_xor(v, o);
        v = u < v ? u : v;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) L.wsum[threadIdx.x >> 6] = (long long)v;
    __syncthreads();
    unsigned long long m = ~0ull;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) m = (unsigned long long)L.wsum[w] < m ? (unsigned long long)L.wsum[w] : m;
    return m;
}

// exclusive scan of v over the workgroup (thread order); returns the thread's offset, *total
__device__ __forceinline__ int block_excl_scan(int v, Lds &L, int *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) L.wscan[w] = x;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; ++i) {
        before += i < w ? L.wscan[i] : 0;
        tot += L.wscan[i];
    }
    *total = tot;
    return before + x - v;
}

// g + t(lane 0) + t(lane 1) + ... + t(lane 63), one add at a time in lane order (the reference's
// running sum), skipping the terms that are 0.0 (empty cells, unit ratios): x + 0.0 == x for every
// running sum that can occur (never -0.0: it starts at +0.0 and round-to-nearest gives +0.0 for
// a + (-a)), so the result is the full in-order sum bit for bit; v_readlane with a uniform lane
// index, no LDS round trip
__device__ __forceinline__ double wave_inorder_add(double g, double t) {
    unsigned long long m = __ballot(t != 0.0);
    const long long bits = __double_as_longlong(t);
    const int lo = (int)(bits & 0xffffffffll), hi = (int)(bits >> 32);
    while (m) {
        const int l = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const unsigned long long b = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(hi, l) << 32) |
                                     (unsigned)__builtin_amdgcn_readlane(lo, l);
        g += __longlong_as_double((long long)b);
    }
    return g;
}

// ---- G^2 decision, shared by the wave and workgroup paths.  The reference (src/IndependenceTest.cpp
// :94-155, 295-364) forms G^2 as one running sum over cells z -> x -> y and p = 1 - pchisq(G^2, df),
// independent iff p > alpha (df == 0: independent, p = 1).  `gs` / `ga` = tree sum of the terms and
// of their magnitudes: with the decision band [lo, hi] (ci_chisq.h) a tree sum clearing it by the
// tree-vs-in-order error bound decides exactly; otherwise *need_inorder and the caller sums in order.
struct Decision {
    int ind;        // -1: undecided (in-order sum needed)
    double margin;  // |p - alpha| as logged
};

__device__ __forceinline__ Decision decide_tree(double gs, double ga, int df, int cells, const PcSmallArgs &A,
                                                const double *band) {
    if (df == 0) return Decision{1, fabs(1.0 - A.alpha)};
    if (A.band && df <= A.nband) {
        const double err = (cells + 64) * 2.3e-16 * ga;
        if (gs + err < band[2 * df - 2]) return Decision{1, band[2 * A.nband]};
        if (gs - err > band[2 * df - 1]) return Decision{0, band[2 * A.nband]};
    }
    return Decision{-1, 0.0};
}

__device__ __noinline__ Decision decide_exact(double g2, int df, const PcSmallArgs &A, const double *band) {
    if (df == 0) return Decision{1, fabs(1.0 - A.alpha)};
    if (A.band && df <= A.nband && g2 < band[2 * df - 2]) return Decision{1, band[2 * A.nband]};
    if (A.band && df <= A.nband && g2 > band[2 * df - 1]) return Decision{0, band[2 * A.nband]};
    const double p = fbn_chisq_pvalue(g2, df);
    return Decision{p > A.alpha ? 1 : 0, fabs(p - A.alpha)};
}

__device__ __forceinline__ double g2_term(long observed, long sum_row, long sum_col, long total) {
    if (total == 0 || sum_row == 0 || sum_col == 0 || observed == 0) return 0.0;
    const double expected = (double)sum_col * (double)sum_row / (double)total;
    return 2.0 * observed * log(observed / expected);
}

// ---- one test per wave on the bit-sliced store (d = 0: marginal; d = 1: one conditioning
// variable).  Leading-value popcounts only: the last value of every variable follows from the
// per-row sample counts (d = 0) or from the level-0 pair tables (d = 1), integers, exact.  The
// table is completed in the wave's LDS slot, cell l = (c * dx + a) * dy + b (Counts3D layout,
// src/CellTable.cpp:277-281), in dependency order: leading cells, then the last y value of every
// leading (z, x) row, then the last x value of every leading z slice, then the last z slice.
// LDS written by some lanes of a wave, then read by others: the wave's LDS operations complete in
// order, so waiting for its own LDS counter suffices (no vector-memory wait: a pending global atomic
// or store must not stall the table passes); the clobber keeps the compiler from moving LDS
// accesses across it
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

template <int D>
__device__ __forceinline__ Decision wave_test(const PcSmallArgs &A, const Lds &L, int x, int y, int z, int lane,
                                           bool record_pair, int32_t *tab, int32_t *aux, unsigned long long *ph) {
    const unsigned long long c0 = A.trace ? clock64() : 0;
    const int n = A.nvars;
    const int dx = L.dims[x], dy = L.dims[y], dz = D == 1 ? L.dims[z] : 1;
    // the margins, staged into the wave's LDS slot by one load per lane (issued ahead of the
    // popcount loop): d = 0 the per-value sample counts of x and y, d = 1 the pair tables
    // N_xy, N_xz, N_yz (16 ints each, u < v stored [u value][v value])
    {
        const int32_t *src = nullptr;
        int k = 0;
        if (D == 0) {
            if (lane < dx) aux[lane] = L.rowcnt[L.row0[x] + lane];
            else if (lane >= 4 && lane < 4 + dy) aux[lane] = L.rowcnt[L.row0[y] + lane - 4];
        } else if (lane < 48) {
            const int u = lane < 32 ? x : y, v = lane < 16 ? y : z;
            src = A.pairtab + 16 * (size_t)pair_index(n, u < v ? u : v, u < v ? v : u);
            k = lane & 15;
        }
        if (src) aux[lane] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int mx = dx - 1, my = dy - 1, mz = D == 1 ? dz - 1 : 1;
    const long long W = A.W;
    const uint32_t *bx = A.bits + (size_t)L.row0[x] * W, *by = A.bits + (size_t)L.row0[y] * W;
    const uint32_t *bz = D == 1 ? A.bits + (size_t)L.row0[z] * W : bx;
    constexpr int MZ = D == 1 ? 3 : 1;
    uint32_t cnt[MZ][3][3];
#pragma unroll
    for (int c = 0; c < MZ; ++c)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) cnt[c][a][b] = 0u;
    for (long long w4 = lane; 4 * w4 < W; w4 += 64) {
        u4 xv[3], yv[3], zv[MZ];
#pragma unroll
        for (int a = 0; a < 3; ++a) xv[a] = a < mx ? *reinterpret_cast<const u4 *>(bx + a * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int b = 0; b < 3; ++b) yv[b] = b < my ? *reinterpret_cast<const u4 *>(by + b * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int c = 0; c < MZ; ++c) {
            if (D == 1) zv[c] = c < mz ? *reinterpret_cast<const u4 *>(bz + c * W + 4 * w4) : u4{0u, 0u, 0u, 0u};
            else zv[c] = u4{~0u, ~0u, ~0u, ~0u};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const uint32_t xy = xv[a][k] & yv[b][k];
#pragma unroll
                    for (int c = 0; c < MZ; ++c) cnt[c][a][b] += __builtin_popcount(xy & zv[c][k]);
                }
    }
    // leading cells: wave totals straight into the table.  Transposing butterfly over the 32
    // (padded) counters: at distance o every lane keeps one half of its counters and adds its
    // partner's copy of that half (32 shuffles in 6 independent stages, instead of 6 dependent
    // shuffles per counter); lane l ends with the total of counter l >> 1 = (c * 3 + a) * 3 + b
    {
        // every counter reduced on DPP (independent chains, interleaved), totals wave-uniform; lane
        // i writes counter i = (c * 3 + a) * 3 + b
        int mine = 0;
#pragma unroll
        for (int c = 0; c < MZ; ++c)
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const int tot = wsum_i32((int)cnt[c][a][b]);
                    mine = lane == (c * 3 + a) * 3 + b ? tot : mine;
                }
        const int i = lane, c = i / 9, a = (i / 3) % 3, b = i % 3;
        if (i < 9 * MZ && c < mz && a < mx && b < my) tab[(c * dx + a) * dy + b] = mine;
    }
    // margins of the full table, all exact integers
    //   d = 0: N_x[a] = rowcnt(x, a), N_y[b] = rowcnt(y, b)
    //   d = 1: N_xz(a, c), N_yz(b, c), N_xy(a, b) from the pair tables (u < v stored [u value][v value])
    const int32_t *Txy = aux, *Txz = aux + 16, *Tyz = aux + 32;
    auto nxz = [&](int a, int c) -> int {
        if (D == 0) return aux[a];
        return x < z ? Txz[a * dz + c] : Txz[c * dx + a];
    };
    auto nyz = [&](int b, int c) -> int {
        if (D == 0) return aux[4 + b];
        return y < z ? Tyz[b * dz + c] : Tyz[c * dy + b];
    };
    const int dxy = dx * dy, cells = dz * dxy;
    const int c = lane / dxy, a = (lane / dy) % dx, b = lane % dy;
    const bool live = lane < cells;
    wave_lds_sync();
    const unsigned long long c1 = A.trace ? clock64() : 0;
    // last y value of the leading (z, x) rows: N_xz(a, c) - sum of the row
    if (live && c < mz && a < mx && b == my) {
        int s = nxz(a, c);
        for (int j = 0; j < my; ++j) s -= tab[(c * dx + a) * dy + j];
        tab[lane] = s;
    }
    wave_lds_sync();
    // last x value of the leading z slices: N_yz(b, c) - sum of the column
    if (live && c < mz && a == mx) {
        int s = nyz(b, c);
        for (int i = 0; i < mx; ++i) s -= tab[(c * dx + i) * dy + b];
        tab[lane] = s;
    }
    wave_lds_sync();
    // last z slice (d = 1): N_xy(a, b) - the other slices
    if (D == 1 && live && c == mz) {
        int s = Txy[a * dy + b];  // x < y: N_xy stored [x value][y value]
        for (int k = 0; k < mz; ++k) s -= tab[(k * dx + a) * dy + b];
        tab[lane] = s;
    }
    wave_lds_sync();
    const int ob = live ? tab[lane] : 0;
    if (D == 0 && record_pair && live)
        __hip_atomic_store(A.pairtab + 16 * (size_t)pair_index(n, x, y) + lane, ob, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long c2 = A.trace ? clock64() : 0;
    // marginals: N_{x+z} = N_xz, N_{+yz} = N_yz, N_{++z} = sum_a N_xz; adjusted df per z
    // (src/IndependenceTest.cpp:96-112, 309-322)
    // nonzero margins as wave ballots: lane l < dz * dx holds N_xz(l % dx, l / dx), lane l < dz * dy
    // N_yz(l % dy, l / dy); alx(c) / aly(c) = set bits in slice c's lane range
    const int mxz = lane < dz * dx ? nxz(lane % dx, lane / dx) : 0;
    const int myz = lane < dz * dy ? nyz(lane % dy, lane / dy) : 0;
    const unsigned long long nzx = __ballot(mxz > 0), nzy = __ballot(myz > 0);
    int df = 0;
    for (int k = 0; k < dz; ++k) {  // wave-uniform
        const int alx = __popcll((nzx >> (k * dx)) & ((1ull << dx) - 1)),
                  aly = __popcll((nzy >> (k * dy)) & ((1ull << dy) - 1));
        df += ((alx >= 1 ? alx : 1) - 1) * ((aly >= 1 ? aly : 1) - 1);
    }
    double t = 0.0;
    if (live) {
        long tot = 0;
        if (D == 0) {
            tot = A.N;
        } else {
            int q[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = i < dx ? nxz(i, c) : 0;  // independent loads
            tot = (long)q[0] + q[1] + q[2] + q[3];
        }
        t = g2_term(ob, nxz(a, c), nyz(b, c), tot);
    }
    const double gs = wsum_f64(t), ga = wsum_f64(fabs(t));
    if (D == 0 && record_pair && A.pg2 && lane == 0)  // G^2 = 2N I(X;Y): the level-1 screen's input
        __hip_atomic_store(A.pg2 + pair_index(n, x, y), (unsigned long long)__double_as_longlong(gs), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    Decision r = decide_tree(gs, ga, df, cells, A, L.band);
    if (r.ind < 0) {  // in the band: the reference's in-order running sum, then p
        r = decide_exact(wave_inorder_add(0.0, t), df, A, L.band);  // lane l = cell l (t = 0 beyond)
    }
    wave_lds_sync();  // the slot is reused by the wave's next test
    if (A.trace && lane == 0) {
        const unsigned long long c3 = clock64();
        ph[0] += c1 - c0, ph[1] += c2 - c1, ph[2] += c3 - c2, ph[3] += 1;
    }
    return r;
}

// ---- the level-1 information screen (the argument: ci_bits.hip, l1_plausible).  In G^2 units:
// with G^2_uv = 2N I(U;V) from level 0, the test (x, y | z) can be independent only if G^2_xz and
// G^2_yz are both >= G^2_xy - hi(df) - margins, df = (dx-1)(dy-1)dz (hi: the decision band's upper
// end, which every independent test's G^2 stays below).  false = certainly dependent (not run).
__device__ __forceinline__ bool screen_plausible(const PcSmallArgs &A, const Lds &L, int x, int y, int z) {
    if (!A.pg2 || !A.band) return true;
    const int df = (L.dims[x] - 1) * (L.dims[y] - 1) * L.dims[z];
    if (df <= 0 || df > A.nband) return true;
    auto g2 = [&](int u, int v) {
        return __longlong_as_double((long long)__hip_atomic_load(
            A.pg2 + pair_index(A.nvars, u < v ? u : v, u < v ? v : u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    };
    const double lim = g2(x, y) - (L.band[2 * df - 1] * (1.0 + 1e-9) + 2e-9 * (double)A.N);
    return lim <= 0.0 || (g2(x, z) >= lim && g2(y, z) >= lim);
}

// ---- one test per wave on the 2-bit packed columns (d = 2, 3: tables of <= 4^5 = 1024 cells): the
// wave's histogram, margins and adjusted df in its LDS region (wh: hist[1024] ni[256] nj[256]
// nk[64] dfp[64]); z index with the LAST conditioning variable fastest (src/CellTable.cpp:39-51,
// 277-281); G^2 as block_test, the in-order fallback 64 terms at a time
template <int D>
__device__ __noinline__ Decision wave_hist_test(const PcSmallArgs &A, const Lds &L, int x, int y, const int *z,
                                                int lane, int32_t *wh, unsigned long long *ph) {
    const unsigned long long c0 = A.trace ? clock64() : 0;
    const int dx = L.dims[x], dy = L.dims[y];
    int cum[D], dimz = 1;
#pragma unroll
    for (int j = D - 1; j >= 0; --j) cum[j] = dimz, dimz *= L.dims[z[j]];
    const int dxy = dx * dy, cells = dimz * dxy;
    int32_t *hist = wh, *ni = wh + 1024, *nj = ni + 256, *nk = nj + 256, *dfp = nk + 64;
    // up to 4 sub-histogram copies (lane l adds into copy l mod copies, copies at an odd stride: a
    // popular cell's same-address LDS atomics serialize copies-fold less), merged after the sweep
    int copies = 1;
    while (copies < 4 && 2 * copies * (cells | 1) <= 1024) copies *= 2;
    const int cstr = copies > 1 ? (cells | 1) : cells;
    for (int c = lane; c < copies * cstr; c += 64) hist[c] = 0;
    int32_t *myh = hist + (lane & (copies - 1)) * cstr;
    wave_lds_sync();
    const long long PW = A.PW, N = A.N;
    const uint32_t *px = A.pk + (size_t)x * PW, *py = A.pk + (size_t)y * PW;
    const uint32_t *pz[D];
#pragma unroll
    for (int j = 0; j < D; ++j) pz[j] = A.pk + (size_t)z[j] * PW;
    // kU words of every column in flight per lane: one memory latency per kU words, not per word
    constexpr int kU = 4;
    for (long long w0 = lane; w0 < PW; w0 += 64 * kU) {
        uint32_t wx[kU], wy[kU], wz[kU][D];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const long long w = w0 + 64 * u < PW ? w0 + 64 * u : w0;
            wx[u] = px[w], wy[u] = py[w];
#pragma unroll
            for (int j = 0; j < D; ++j) wz[u][j] = pz[j][w];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const long long w = w0 + 64 * u;
            const long long left = w < PW ? N - 16 * w : 0;
            const int lim = left < 16 ? (int)left : 16;
            // consecutive samples of the word in the same cell fold into one atomic (skewed data)
            int prev = -1, run = 0;
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                int zi = 0;
#pragma unroll
                for (int j = 0; j < D; ++j) zi += (int)((wz[u][j] >> (2 * s)) & 3u) * cum[j];
                const int cl = (zi * dx + (int)((wx[u] >> (2 * s)) & 3u)) * dy + (int)((wy[u] >> (2 * s)) & 3u);
                if (s < lim) {
                    if (cl == prev) {
                        ++run;
                    } else {
                        if (run) atomicAdd(&myh[prev], run);
                        prev = cl, run = 1;
                    }
                }
            }
            if (run) atomicAdd(&myh[prev], run);
        }
    }
    wave_lds_sync();
    if (copies > 1) {
        for (int c = lane; c < cells; c += 64) {
            int v = 0;
            for (int k = 0; k < copies; ++k) v += hist[k * cstr + c];
            hist[c] = v;  // copy 0 in place: cell c of copy 0 is read only by this lane
        }
        wave_lds_sync();
    }
    const unsigned long long c1 = A.trace ? clock64() : 0;
    // marginals N_{x+z}, N_{+yz} (src/CellTable.cpp:242-250)
    for (int r = lane; r < dimz * dx; r += 64) {
        const int k = r / dx, i = r % dx;
        int sm = 0;
        for (int j = 0; j < dy; ++j) sm += hist[k * dxy + i * dy + j];
        ni[r] = sm;
    }
    for (int r = lane; r < dimz * dy; r += 64) {
        const int k = r / dy, j = r % dy;
        int sm = 0;
        for (int i = 0; i < dx; ++i) sm += hist[k * dxy + i * dy + j];
        nj[r] = sm;
    }
    wave_lds_sync();
    // N_{++z}, adjusted df per z (src/IndependenceTest.cpp:96-112)
    for (int k = lane; k < dimz; k += 64) {
        int alx = 0, aly = 0, tot = 0;
        for (int i = 0; i < dx; ++i) alx += ni[k * dx + i] > 0, tot += ni[k * dx + i];
        for (int j = 0; j < dy; ++j) aly += nj[k * dy + j] > 0;
        dfp[k] = ((alx >= 1 ? alx : 1) - 1) * ((aly >= 1 ? aly : 1) - 1);
        nk[k] = tot;
    }
    wave_lds_sync();
    const unsigned long long c2 = A.trace ? clock64() : 0;
    auto term_of = [&](int c) {
        const int k = c / dxy, i = (c / dy) % dx, j = c % dy;
        return g2_term(hist[c], ni[k * dx + i], nj[k * dy + j], nk[k]);
    };
    double ps = 0.0, pa = 0.0;
    int df = 0;
    for (int c = lane; c < cells; c += 64) {
        const double t = term_of(c);
        ps += t;
        pa += fabs(t);
    }
    for (int k = lane; k < dimz; k += 64) df += dfp[k];
    ps = wsum_f64(ps);
    pa = wsum_f64(pa);
    df = wsum_i32(df);
    Decision r = decide_tree(ps, pa, df, cells, A, L.band);
    if (r.ind < 0) {  // in-order running sum over z -> x -> y, 64 terms at a time
        double g2 = 0.0;
        for (int c0 = 0; c0 < cells; c0 += 64) {
            const double t = c0 + lane < cells ? term_of(c0 + lane) : 0.0;
            g2 = wave_inorder_add(g2, t);
        }
        r = decide_exact(g2, df, A, L.band);
    }
    wave_lds_sync();  // the region is reused by the wave's next test
    if (A.trace && lane == 0) {
        const unsigned long long c3 = clock64();
        ph[0] += c1 - c0, ph[1] += c2 - c1, ph[2] += c3 - c2, ph[3] += 1;
    }
    return r;
}

// ---- one test per workgroup (d >= 2): LDS histogram of the 2-bit packed columns.  z index with
// the LAST conditioning variable fastest (src/CellTable.cpp:39-51, 277-281).
template <int D>
__device__ __noinline__ Decision block_test(const PcSmallArgs &A, int x, int y, const int *z, Lds &L) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long c0 = A.trace ? clock64() : 0;
    const int dx = L.dims[x], dy = L.dims[y];
    int cum[D], dimz = 1;
#pragma unroll
    for (int j = D - 1; j >= 0; --j) cum[j] = dimz, dimz *= L.dims[z[j]];
    const int dxy = dx * dy, cells = dimz * dxy;
    // sub-histogram copies: each wave adds into copy (wave mod copies), fewer same-cell conflicts
    int copies = 1;
    while (copies < NWAVE && 2 * copies * cells <= kHistCells) copies *= 2;
    int32_t *hist = L.hist;
    for (int i = tid; i < copies * cells; i += BS) hist[i] = 0;
    __syncthreads();
    int32_t *my = hist + (wv & (copies - 1)) * cells;
    const long long PW = A.PW, N = A.N;
    const uint32_t *px = A.pk + (size_t)x * PW, *py = A.pk + (size_t)y * PW;
    const uint32_t *pz[D];
#pragma unroll
    for (int j = 0; j < D; ++j) pz[j] = A.pk + (size_t)z[j] * PW;
    for (long long w = tid; w < PW; w += BS) {
        const uint32_t wx = px[w], wy = py[w];
        uint32_t wz[D];
#pragma unroll
        for (int j = 0; j < D; ++j) wz[j] = pz[j][w];
        const long long left = N - 16 * w;
        const int lim = left < 16 ? (int)left : 16;
        int prev = -1, run = 0;  // consecutive samples in the same cell: one atomic
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            int zi = 0;
#pragma unroll
            for (int j = 0; j < D; ++j) zi += (int)((wz[j] >> (2 * s)) & 3u) * cum[j];
            const int cl = (zi * dx + (int)((wx >> (2 * s)) & 3u)) * dy + (int)((wy >> (2 * s)) & 3u);
            if (s < lim) {
                if (cl == prev) {
                    ++run;
                } else {
                    if (run) atomicAdd(&my[prev], run);
                    prev = cl, run = 1;
                }
            }
        }
        if (run) atomicAdd(&my[prev], run);
    }
    __syncthreads();
    if (copies > 1) {
        for (int i = tid; i < cells; i += BS) {
            int v = 0;
            for (int k = 0; k < copies; ++k) v += hist[k * cells + i];
            hist[i] = v;
        }
        __syncthreads();
    }
    const unsigned long long c1 = A.trace ? clock64() : 0;
    // marginals N_{x+z}, N_{+yz}, N_{++z}, adjusted df per z (src/CellTable.cpp:242-250,
    // src/IndependenceTest.cpp:96-112)
    for (int r = tid; r < dimz * dx; r += BS) {
        const int k = r / dx, i = r % dx;
        int s = 0;
        for (int j = 0; j < dy; ++j) s += hist[k * dxy + i * dy + j];
        L.ni[r] = s;
    }
    for (int r = tid; r < dimz * dy; r += BS) {
        const int k = r / dy, j = r % dy;
        int s = 0;
        for (int i = 0; i < dx; ++i) s += hist[k * dxy + i * dy + j];
        L.nj[r] = s;
    }
    __syncthreads();
    for (int k = tid; k < dimz; k += BS) {
        int alx = 0, aly = 0, tot = 0;
        for (int i = 0; i < dx; ++i) alx += L.ni[k * dx + i] > 0, tot += L.ni[k * dx + i];
        for (int j = 0; j < dy; ++j) aly += L.nj[k * dy + j] > 0;
        L.dfp[k] = ((alx >= 1 ? alx : 1) - 1) * ((aly >= 1 ? aly : 1) - 1);
        L.nk[k] = tot;
    }
    __syncthreads();
    const unsigned long long c2 = A.trace ? clock64() : 0;
    auto term_of = [&](int c) {
        const int k = c / dxy, i = (c / dy) % dx, j = c % dy;
        return g2_term(hist[c], L.ni[k * dx + i], L.nj[k * dy + j], L.nk[k]);
    };
    double ps = 0.0, pa = 0.0;
    int pdf = 0;
    for (int c = tid; c < cells; c += BS) {
        const double t = term_of(c);
        ps += t;
        pa += fabs(t);
    }
    for (int k = tid; k < dimz; k += BS) pdf += L.dfp[k];
    ps = wsum_f64(ps);
    pa = wsum_f64(pa);
    pdf = wsum_i32(pdf);
    if (lane == 0) L.red[2 * wv] = ps, L.red[2 * wv + 1] = pa, L.redi[wv] = pdf;
    __syncthreads();
    double gs = 0.0, ga = 0.0;
    int df = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) gs += L.red[2 * w], ga += L.red[2 * w + 1], df += L.redi[w];
    Decision r = decide_tree(gs, ga, df, cells, A, L.band);
    if (r.ind < 0) {  // in-order running sum over z -> x -> y, chunk by chunk (terms in LDS)
        double g2 = 0.0;
        for (int c0 = 0; c0 < cells; c0 += kTermChunk) {
            const int c1 = c0 + kTermChunk < cells ? c0 + kTermChunk : cells;
            __syncthreads();
            for (int c = c0 + tid; c < c1; c += BS) L.term[c - c0] = term_of(c);
            __syncthreads();
            if (wv == 0)  // wave 0: 64 terms per step, zero terms skipped
                for (int c = 0; c < c1 - c0; c += 64) g2 = wave_inorder_add(g2, c + lane < c1 - c0 ? L.term[c + lane] : 0.0);
        }
        if (tid == 0) L.g2 = g2;
        __syncthreads();
        r = decide_exact(L.g2, df, A, L.band);
    }
    if (A.trace && tid == 0) {
        const unsigned long long c3 = clock64();
        L.ph[0][0] += c1 - c0, L.ph[0][1] += c2 - c1, L.ph[0][2] += c3 - c2, L.ph[0][3] += 1;
    }
    __syncthreads();  // LDS reused by the next test
    return r;
}

// workgroup 0, at the end of the device's part of the search: the run's decision-margin log (over
// every workgroup's slot) into the result and into the ctx's log, the level count, hand-off flag
__device__ void finalize(const PcSmallArgs &A, Lds &L, int nb, int levels, int handoff) {
    const int tid = threadIdx.x;
    unsigned long long mm = ~0ull;
    long long nn = 0;
    for (int b = tid; b < nb; b += BS) {
        const unsigned long long v = ld_agent(A.acc + 8 * (size_t)b);
        mm = v < mm ? v : mm;
        nn += (long long)ld_agent(A.acc + 8 * (size_t)b + 1);
    }
    mm = block_min_u64(mm, L);
    nn = block_sum_ll(nn, L);
    PcSmallOut *o = A.dout;
    for (int d = 0; d < levels; ++d) {  // tests evaluated per level, over every workgroup's slot
        long long la = 0;
        for (int b = tid; b < nb; b += BS) la += (long long)ld_agent(A.acc + 8 * (size_t)b + 2 + d);
        la = block_sum_ll(la, L);
        if (tid == 0) o->launched[d] = la;
    }
    if (tid == 0) {
        o->margin_bits = mm;
        o->near = (unsigned long long)nn;
        A.ctx_stats[0] = mm;
        A.ctx_stats[1] = (unsigned long long)nn;
        o->levels = levels;
        o->handoff = handoff;
        o->status = 0;
        o->pad = 0;
        for (int d = levels; d <= kSmallMaxD; ++d) o->sep_off[d + 1] = o->sep_off[d > 0 ? d : 0];
    }
    __syncthreads();
    // the record, built in device memory during the run, goes to the pinned host copy in one
    // parallel pass: everything before the sepset pool, then the pool's used part
    const uint32_t *src = reinterpret_cast<const uint32_t *>(o);
    uint32_t *dst = reinterpret_cast<uint32_t *>(A.out);
    const int head = (int)(offsetof(PcSmallOut, pool) / 4);
    const int used = head + (levels > 0 ? o->sep_off[levels] : 0);
    for (int i = tid; i < used; i += BS) dst[i] = src[i];
    // every thread's part of the copy reaches the host before the completion word
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&A.out->done, A.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(BS) void pc_small_kernel(PcSmallArgs Ak, Barrier B) {
    __shared__ Lds L;
    // the arguments staged in LDS: the out-of-line test functions take them by reference, and a
    // reference to the kernel parameter made the compiler copy the struct into per-thread scratch
    // (176 B per thread, ~23 MB of writes per launch, a scratch load per field access)
    __shared__ PcSmallArgs SA;
    if (threadIdx.x == 0) SA = Ak;
    __syncthreads();
    const PcSmallArgs &A = SA;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = A.nvars;
    const int nb = gridDim.x;
    const int bid = blockIdx.x;
    if (A.trace && bid == 0 && tid == 0) A.trace[63] = (unsigned long long)wall_clock64();
    // prologue: every constant staged in ONE round of independent loads (no load depends on
    // another), binomials in 32-bit arithmetic (C(64, 4) < 2^20)
    for (int i = tid; i < (kSmallMaxVars + 1) * (kSmallMaxD + 1); i += BS) {
        const int m = i / (kSmallMaxD + 1), k = i % (kSmallMaxD + 1);
        int r = 1;
        for (int j = 1; j <= k; ++j) r = r * (m - k + j) / j;
        L.binom[m][k] = m < k ? 0 : r;
    }
    for (int v = tid; v < kSmallMaxVars; v += BS) {
        const uint64_t all = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
        L.adj[v] = v < n ? (all & ~(1ull << v)) : 0ull;
        L.dims[v] = v < n ? A.dims[v] : 1;
        L.row0[v] = v < n ? A.row0[v] : 0;
    }
    for (int r = tid; r < 4 * kSmallMaxVars; r += BS) L.rowcnt[r] = r < A.nrows ? A.rowcnt[r] : 0;
    if (A.band)
        for (int i = tid; i <= 2 * A.nband; i += BS) L.band[i] = A.band[i];
    __syncthreads();
    // this workgroup's statistics slot: [0] min margin bits, [1] near, [2 + d] tests evaluated
    unsigned long long wmin = ~0ull, wnear = 0ull;
    unsigned long long *slot = A.acc + 8 * (size_t)bid;
    unsigned phase = 0;
    int32_t sep_cursor = 0;
    for (int d = 0;; ++d) {
        // ---- the level's edges (lexicographic pairs of the snapshot) and their test offsets
        if (tid < 64) {  // rowoff[x] = edges (x' < y) of rows x' < x: one wave's inclusive scan
            int c = tid < n && tid + 1 < 64 ? popc64(L.adj[tid] >> (tid + 1)) : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(c, o);
                if (tid >= o) c += y;
            }
            L.rowoff[tid + 1] = c;
            if (tid == 0) L.rowoff[0] = 0;
            if (tid == 63) L.E = c;
        }
        __syncthreads();
        const int E = L.E;
        if (tid < n) {
            const int x = tid;
            uint64_t m = x + 1 < 64 ? (L.adj[x] >> (x + 1)) << (x + 1) : 0ull;
            int e = L.rowoff[x];
            while (m) {
                const int y = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                L.ex[e] = (uint8_t)x, L.ey[e] = (uint8_t)y;
                ++e;
            }
        }
        __syncthreads();
        // tests per edge (level 0: one marginal test; level d: C(|adj(x)|-1, d) + C(|adj(y)|-1, d))
        // -> exclusive offsets: thread tid owns a contiguous run of edges, one workgroup scan
        long long tot64 = 0;
        {
            const int seg = (E + BS - 1) / BS, e0 = tid * seg, e1 = e0 + seg < E ? e0 + seg : E;
            auto ntests = [&](int e) {
                const int x = L.ex[e], y = L.ey[e];
                return d == 0 ? 1 : binom_l(L, popc64(L.adj[x]) - 1, d) + binom_l(L, popc64(L.adj[y]) - 1, d);
            };
            const int KA = (d == 1 || d == 2) ? A.spec_a : 0x40000000;  // part A per edge
            long long mine = 0, mineA = 0;  // (int64: a level's total may exceed 2^31 -> hand-off below)
            for (int e = e0; e < e1; ++e) {
                const int nt = ntests(e);
                mine += nt;
                mineA += nt < KA ? nt : KA;
            }
            tot64 = block_sum_ll(mine, L);
            if (tot64 <= kSmallMaxTests) {  // (workgroup-uniform) int32 offsets
                int totalA = 0, totalB = 0;
                int runA = block_excl_scan((int)mineA, L, &totalA);
                int runB = block_excl_scan((int)(mine - mineA), L, &totalB);
                for (int e = e0; e < e1; ++e) {
                    const int nt = ntests(e), na = nt < KA ? nt : KA;
                    L.eoff[e] = runA, runA += na;
                    L.eoffB[e] = runB, runB += nt - na;
                }
                if (tid == 0) L.eoff[E] = totalA, L.eoffB[E] = totalB, L.TA = totalA;
            }
        }
        __syncthreads();
        const bool fits = d <= kSmallMaxD && tot64 <= kSmallMaxTests;
        if (!fits) {
            // hand the search to the host driver at this level (its snapshot = adj after d - 1)
            if (bid == 0) finalize(A, L, nb, d, 1);
            return;
        }
        const int T = (int)tot64;
        for (int e = tid; e < E; e += BS) L.bfirst[e] = ~0u;
        if (tid < NWAVE * 4) (&L.ph[0][0])[tid] = 0ull;
        if (tid == 0) L.next = 0;
        __syncthreads();
        if (A.trace && bid == 0 && tid == 0) A.trace[8 * d + 0] = (unsigned long long)wall_clock64();
        if (A.trace && tid == 0) A.trace[64 + 5 * 1024 + (size_t)d * 1024 + bid] = (unsigned long long)wall_clock64();
        // ---- the tests
        unsigned long long launched = 0;
        if (d <= 2) {
            // workgroup b takes tests t = b' + nb j (b' = nb - 1 - b: workgroup 0, which builds the
            // result record between levels, the last and lightest share); its waves claim j
            // dynamically, so part-B skips do not leave some waves with more tests than others
            const int b0 = nb - 1 - bid;
            const int TA = L.TA;
            // test t -> (edge, candidate index): part A, then part B (see spec_a)
            auto locate = [&](int t, int &e, int &k) {
                const bool b = t >= TA;
                const int32_t *off = b ? L.eoffB : L.eoff;
                const int tt = b ? t - TA : t;
                int lo = 0, hi = E;  // last edge whose first test <= tt
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (off[mid] <= tt) lo = mid;
                    else hi = mid;
                }
                e = lo;
                k = tt - off[lo] + (b ? A.spec_a : 0);
            };
            while (true) {
                int j = 0;
                if (lane == 0) j = atomicAdd(&L.next, 1);
                const int t = b0 + nb * __shfl(j, 0);
                if (t >= T) break;
                int e, k;
                locate(t, e, k);
                if (t >= TA) {  // part B: skip a candidate behind an independent one (read just before
                                // the test: a check loaded a test earlier sees too little of part A)
                    const unsigned fl = L.bfirst[e], fg = first_of(A, d, e);
                    if ((fg != ~0u && fg < (unsigned)k) || (fl != ~0u && fl < (unsigned)k)) continue;
                }
                const int x = L.ex[e], y = L.ey[e];
                Decision r;
                if (d == 0) {
                    r = wave_test<0>(A, L, x, y, 0, lane, true, L.wtab[wv], L.waux[wv], L.ph[wv]);
                } else {
                    int zz[3];
                    unrank(L, x, y, d, k, zz);
                    if (d == 1 && !screen_plausible(A, L, x, y, zz[0])) continue;  // dependent: not run
                    if (d == 1) r = wave_test<1>(A, L, x, y, zz[0], lane, false, L.wtab[wv], L.waux[wv], L.ph[wv]);
                    else r = wave_hist_test<2>(A, L, x, y, zz, lane, L.whist[wv], L.ph[wv]);  // (d == 2)
                }
                ++launched;
                const unsigned long long mb = (unsigned long long)__double_as_longlong(r.margin);
                wmin = mb < wmin ? mb : wmin;
                wnear += r.margin < 1e-9;
                if (r.ind == 1 && lane == 0) {
                    atomicMin(&L.bfirst[e], (unsigned)k);
                    if (d >= 1)  // published at once for the part-B checks of every workgroup
                        __hip_atomic_fetch_max(A.first + (size_t)d * kSmallMaxEdges + e,
                                               ((unsigned long long)A.epoch << 32) | (unsigned)~(unsigned)k,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        } else {
            for (int t = nb - 1 - bid; t < T; t += nb) {
                int lo = 0, hi = E;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (L.eoff[mid] <= t) lo = mid;
                    else hi = mid;
                }
                const int e = lo, k = t - L.eoff[e];
                const int x = L.ex[e], y = L.ey[e];
                int zz[kSmallMaxD];
                unrank(L, x, y, d, k, zz);
                Decision r;
                r = d == 3 ? block_test<3>(A, x, y, zz, L) : block_test<4>(A, x, y, zz, L);
                if (tid == 0) {
                    ++launched;
                    const unsigned long long mb = (unsigned long long)__double_as_longlong(r.margin);
                    wmin = mb < wmin ? mb : wmin;
                    wnear += r.margin < 1e-9;
                    if (r.ind == 1) atomicMin(&L.bfirst[e], (unsigned)k);
                }
            }
        }
        // per-wave statistics (lane 0 holds the wave's; the workgroup path's are thread 0's)
        if (lane == 0) L.wst[wv][0] = wmin, L.wst[wv][1] = wnear, L.wst[wv][2] = launched;
        // this workgroup's first independent candidates -> the global per-edge words (first[] holds
        // ~min k, 0 = none: an atomic max of the complements), all in flight together
        __syncthreads();
        for (int e = tid; e < E; e += BS)
            if (L.bfirst[e] != ~0u)
                __hip_atomic_fetch_max(A.first + (size_t)d * kSmallMaxEdges + e,
                                       ((unsigned long long)A.epoch << 32) | (unsigned)~L.bfirst[e], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        // this workgroup's statistics into its slot (agent-coherent stores, published by the barrier)
        if (tid == 0) {
            unsigned long long mm = ~0ull, nn = 0, ll = 0;
#pragma unroll
            for (int w = 0; w < NWAVE; ++w) {
                mm = L.wst[w][0] < mm ? L.wst[w][0] : mm;
                nn += L.wst[w][1], ll += L.wst[w][2];
            }
            st_agent(slot, mm);
            st_agent(slot + 1, nn);
            st_agent(slot + 2 + d, ll);
        }
        if (A.trace && tid == 0) A.trace[64 + (size_t)d * 1024 + bid] = (unsigned long long)wall_clock64();
        if (A.trace && tid < 4) {  // phase cycles summed over the workgroup's waves -> trace[8d + 4 + k]
            unsigned long long sum = 0;
            for (int w = 0; w < NWAVE; ++w) sum += L.ph[w][tid];
            atomicAdd(A.trace + 8 * d + 4 + tid, sum);
        }
        if (!grid_barrier(B, A.phase_base + ++phase, L)) {
            if (tid == 0) {  // the host sees the failure (and stops waiting) without a stream sync
                A.out->status = 1;
                __threadfence_system();
                __hip_atomic_store(&A.out->done, A.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
        if (A.trace && bid == 0 && tid == 0) A.trace[8 * d + 2] = (unsigned long long)wall_clock64();
        // ---- apply: removed = some independent set found; counted = first + 1, else all sets
        long long counted = 0;
        for (int e = tid; e < E; e += BS) {
            const unsigned f = first_of(A, d, e);
            const bool rmv = f != ~0u;
            L.rm[e] = rmv;
            counted += rmv ? (long long)f + 1
                           : (long long)(L.eoff[e + 1] - L.eoff[e]) + (long long)(L.eoffB[e + 1] - L.eoffB[e]);
        }
        __syncthreads();
        if (bid == 0) {  // the result record (the other workgroups go straight on to the next level)
            counted = block_sum_ll(counted, L);
            // sepsets of the removed edges in edge order (unranked against the level's snapshot)
            int carry = 0;
            for (int e0 = 0; e0 < E; e0 += BS) {
                const int e = e0 + tid;
                const int r = e < E ? L.rm[e] : 0;
                int total = 0;
                const int off = block_excl_scan(r, L, &total);
                if (r && d > 0) {
                    const unsigned f = first_of(A, d, e);
                    int zz[kSmallMaxD];
                    unrank(L, L.ex[e], L.ey[e], d, (int)f, zz);
                    for (int j = 0; j < d; ++j) A.dout->pool[sep_cursor + (carry + off) * d + j] = zz[j];
                }
                carry += total;
                __syncthreads();
            }
            if (tid == 0) {  // (launched[d]: summed over the workgroups' slots in finalize)
                A.dout->sep_off[d] = sep_cursor;
                A.dout->sep_off[d + 1] = sep_cursor + carry * d;
                A.dout->counted[d] = counted;
            }
            sep_cursor += carry * d;
        }
        __syncthreads();
        for (int e = tid; e < E; e += BS)
            if (L.rm[e]) {
                const int x = L.ex[e], y = L.ey[e];
                atomicAnd((unsigned long long *)&L.adj[x], ~(1ull << y));
                atomicAnd((unsigned long long *)&L.adj[y], ~(1ull << x));
            }
        __syncthreads();
        if (A.trace && bid == 0 && tid == 0) A.trace[8 * d + 3] = (unsigned long long)wall_clock64();
        int maxdeg = 0;
        for (int v = 0; v < n; ++v) maxdeg = maxdeg > popc64(L.adj[v]) ? maxdeg : popc64(L.adj[v]);
        if (bid == 0 && tid < kSmallMaxVars) A.dout->adj[d][tid] = L.adj[tid];
        const bool cont = d + 1 < A.depth && (d == 0 || maxdeg - 1 > d);  // FreeDegree (src/PCStable.cpp:557-563)
        if (!cont) {
            if (bid == 0) finalize(A, L, nb, d + 1, 0);
            return;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" int fbn_pc_small_block_threads(void) { return BS; }

extern "C" hipError_t fbn_pc_small_occupancy(int *blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, pc_small_kernel, BS, 0);
}

// a->bar: (kGroups * 16 + 16) unsigned words, zeroed once (see kSmallZeroBytes).  spin_ticks <= 0:
// the default barrier limit.  cooperative: hipLaunchCooperativeKernel, which refuses a grid that
// cannot be resident at once (hipErrorCooperativeLaunchTooLarge) instead of letting it spin.
extern "C" hipError_t fbn_pc_small_launch(const PcSmallArgs *a, int grid, long long spin_ticks, int cooperative,
                                          hipStream_t s) {
    Barrier b{a->bar, a->bar + 16 * kGroups, grid, spin_ticks > 0 ? spin_ticks : kSpinTicks};
    if (cooperative) {
        PcSmallArgs ak = *a;
        void *params[2] = {&ak, &b};
        return hipLaunchCooperativeKernel(reinterpret_cast<const void *>(pc_small_kernel), dim3(grid), dim3(BS),
                                          params, 0, s);
    }
    hipLaunchKernelGGL(pc_small_kernel, dim3(grid), dim3(BS), 0, s, *a, b);
    return hipGetLastError();
}
