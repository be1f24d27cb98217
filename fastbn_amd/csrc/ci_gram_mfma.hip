// ci_gram_mfma.hip -- the level-0 Gram of PC-stable on the gfx950 matrix cores, hand-written.
//
// Level 0 of the skeleton search tests every pair of the complete graph marginally
// (reference: src/PCStable.cpp level-0 loop -> IndependenceTest::IsIndependent -> Counts2D::FillTable,
// src/CellTable.cpp:23-91).  Every pair's table follows from popcount(r_i & r_j) over the leading
// value rows r of the two variables (ci_bits.hip), i.e. from the Gram G = O O^T of the 0/1 matrix
// O[leading row][sample].  Here O is stored as FP4 (E2M1: 1.0 = nibble 0x2, 0.0 = 0x0, two
// samples per byte) and G is formed with v_mfma_scale_f32_32x32x64_f8f6f4 (FP4 x FP4, fp32
// accumulate: products are 0/1 and a K-slice of <= 65535 samples sums exactly in fp32), the
// densest MFMA of CDNA4 (4x the bf16 rate, 2x int8).
//
//  * Only the tiles the pairs need: 256 x 256 output tiles (I, J) with J >= I (x < y puts every
//    needed entry above the diagonal).  A diagonal tile stages one panel (A = B); its four waves
//    compute their whole quadrants anyway -- the upper-right wave bounds the block's time, and no
//    branch around the MFMAs keeps the accumulators in AGPRs -- and the lower-left one stores nothing.
//  * Split-K: tile x K-slice blocks, about one per CU.  Consecutive (XCD-remapped) block ids share
//    the K-slice and walk the same 128-sample stages of all row panels, so one XCD's L2 serves a
//    panel to the ~8 tiles that read it.  Each block writes its slice's partial counts as uint16 to a
//    slab; ci_gram_reduce sums the slabs into the int32 Gram (upper entries only).
//  * 256 threads = 4 waves (2 x 2), 128 x 128 per wave = 4 x 4 MFMA tiles of 32 x 32 (256
//    accumulator registers).  Stages of 128 samples (64 B per row, 16 KB per 256-row panel) arrive
//    by global_load_lds (dwordx4) into 5 LDS buffers, 4 stages in flight; one raw s_barrier per
//    stage; every LDS byte in one __shared__ array (hipcc otherwise waits vmcnt(0) at ds_reads);
//    the fragments of K-step k + 1 are read while the MFMAs of K-step k run.
//  * The FP4 store is stage-major ([stage][row][64 B]): a panel's stage is one contiguous 16 KB.
//  * LDS rows are 64 B = 4 chunks of 16 B; chunk c of row r lives at c ^ ((r >> 2) & 3), so each
//    16-lane group of a ds_read_b128 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...: rows with every
//    (r & 3, (r >> 2) & 3) pair once) hits 16 distinct 4-bank slots (SQ_LDS_BANK_CONFLICT = 0).
//    global_load_lds writes lane L at base + 16 L, so the swizzle is applied to the global source.
//  * Measured (config 5, 2000 rows x 100k samples, S = 7, 252 blocks): 0.100-0.110 ms for the
//    tiles + 0.013-0.018 ms for the reduce (rocBLAS int8 split-K: 0.26 ms).  MFMA busy 47 % of the
//    kernel (PMC); an MFMA-only loop of the same shape reaches 7.9 PF/s (61 us), with the fragment
//    reads and barrier 6.7 PF/s (72 us, tools/micro/mfma_fp4_rate.hip); the restaging costs
//    ~17 us more (no change from 4 -> 5 stages in flight or from full-line staging: L2 bandwidth,
//    ~2.2 TB/s per XCD at 32 KB per CU per stage), the uint16 slab stores ~6 us.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kTile = 256;                 // output tile edge (rows of O per panel)
constexpr int kStageS = 128;               // samples per stage
constexpr int kRowB = kStageS / 2;         // bytes per row per stage (fp4)
constexpr int kPanelB = kTile * kRowB;     // 16 KB
constexpr int kBufB = 2 * kPanelB;         // A + B panel
constexpr int kNBuf = 5;                   // stages resident (4 in flight + 1 computing)
constexpr int kLdsB = kNBuf * kBufB;       // 160 KB: the whole LDS of the CU
constexpr int kInstPerPanelWave = kPanelB / 1024 / 4;  // glds dwordx4 per wave per panel: 4

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void glds16(const uint8_t *g, uint8_t *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

// one panel-stage: 256 rows x 64 B.  Wave w stages rows [64 w, 64 w + 64): 4 instructions of 16 rows
// (lane L: row 16 i + L / 4, LDS chunk L % 4 = global chunk (L % 4) ^ ((row >> 2) & 3))
__device__ __forceinline__ void stage_panel(const uint8_t *__restrict__ src, uint8_t *dst, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < kInstPerPanelWave; ++i) {
        const int row0 = wave * 64 + i * 16;
        const int row = row0 + (lane >> 2);
        const int c = (lane & 3) ^ ((row >> 2) & 3);
        glds16(src + row * kRowB + c * 16, dst + row0 * kRowB);
    }
}

__device__ __forceinline__ v4i frag(const uint8_t *buf, int row, int c) {
    return *reinterpret_cast<const v4i *>(buf + row * kRowB + ((c ^ ((row >> 2) & 3)) << 4));
}

__device__ __forceinline__ v16f mfma_fp4(v4i a, v4i b, v16f acc) {
    // cbsz = blgp = 4: both operands FP4 E2M1; scales 0 select the unscaled operation
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{a[0], a[1], a[2], a[3], 0, 0, 0, 0},
                                                           v8i{b[0], b[1], b[2], b[3], 0, 0, 0, 0}, acc, 4, 4, 0, 0,
                                                           0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt left outstanding when stage t must have landed: the loads of the `ahead` stages issued after
// it (0..4), 8 instructions per stage (A + B panel) or 4 (diagonal tile: one panel)
__device__ __forceinline__ void wait_stage(int ahead, bool diag) {
    if (diag) {
        if (ahead >= 4) wait_vm<16>();
        else if (ahead == 3) wait_vm<12>();
        else if (ahead == 2) wait_vm<8>();
        else if (ahead == 1) wait_vm<4>();
        else wait_vm<0>();
    } else {
        if (ahead >= 4) wait_vm<32>();
        else if (ahead == 3) wait_vm<24>();
        else if (ahead == 2) wait_vm<16>();
        else if (ahead == 1) wait_vm<8>();
        else wait_vm<0>();
    }
}

struct Frags {
    v4i a[4], b[4];
};

// the wave's fragments of K-step s (64 samples) of a staged buffer: lane (r, h) holds 32 samples of
// A row ra + 32 m and of B row rb + 32 n, chunk 2 s + h of the 64-B stage row
__device__ __forceinline__ void load_frags(Frags &f, const uint8_t *bufA, const uint8_t *bufB, int ra, int rb, int c) {
#pragma unroll
    for (int n = 0; n < 4; ++n) f.b[n] = frag(bufB, rb + 32 * n, c);
#pragma unroll
    for (int m = 0; m < 4; ++m) f.a[m] = frag(bufA, ra + 32 * m, c);
}

template <int M0 = 0, int M1 = 4>
__device__ __forceinline__ void mfma_step(v16f (&acc)[4][4], const Frags &f) {
#pragma unroll
    for (int m = M0; m < M1; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_fp4(f.a[m], f.b[n], acc[m][n]);
}

// tasks[t] = (I, J) tile coordinates; block b (XCD-remapped to w) computes tile w % nt over stages
// [split * KS / S, (split + 1) * KS / S) with split = w / nt; slab[w][256][256] uint16 partials.
__global__ __launch_bounds__(256, 1) void ci_gram_fp4(const uint8_t *__restrict__ O4, long long Rp,
                                                        const int2 *__restrict__ tasks, int nt, int S, int KS,
                                                        uint16_t *__restrict__ slab) {
    __shared__ __attribute__((aligned(1024))) uint8_t lds[kLdsB];
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    const int split = w / nt, tile = w - split * nt;
    const int st0 = (int)((long long)split * KS / S), st1 = (int)((long long)(split + 1) * KS / S);
    const int2 IJ = tasks[tile];
    const bool diag = IJ.x == IJ.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    const bool idle = diag && wm > wn;
    const uint8_t *Ag = O4 + (long long)IJ.x * kTile * kRowB;
    const uint8_t *Bg = O4 + (long long)IJ.y * kTile * kRowB;

    v16f acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[m][n][j] = 0.f;

    auto buf_of = [&](int t) { return lds + ((t - st0) % kNBuf) * kBufB; };
    auto issue = [&](int t) {
        uint8_t *buf = buf_of(t);
        const long long off = (long long)t * Rp * kRowB;  // stage t of every row: one contiguous block
        stage_panel(Ag + off, buf, wave, lane);
        if (!diag) stage_panel(Bg + off, buf + kPanelB, wave, lane);
    };
    // Software pipeline (one wave per SIMD, so the MFMA pipe must never wait on LDS): the fragments
    // of the next K-step are read while the MFMAs of the current one run.  Iteration t: read K-step
    // 1 of stage t, MFMAs of K-step 0; then (every wave's reads of stage t retired) wait for stage
    // t + 1's loads, barrier, restage buffer t with stage t + kNBuf, read K-step 0 of stage t + 1,
    // MFMAs of K-step 1 of stage t.  kNBuf - 1 stages stay in flight.
    const int ra = wm * 128 + (lane & 31), rb = wn * 128 + (lane & 31), h = lane >> 5;
    for (int t = st0; t < st0 + kNBuf && t < st1; ++t) issue(t);
    wait_stage(min(kNBuf - 1, st1 - 1 - st0), diag);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    Frags f0, f1;
    {
        const uint8_t *bA = buf_of(st0);
        load_frags(f0, bA, diag ? bA : bA + kPanelB, ra, rb, h);
    }
    for (int t = st0; t + 1 < st1; ++t) {  // the last stage is peeled: no branch inside the body
        const uint8_t *bA = buf_of(t);
        // (the reads go out after the first MFMAs: f0's own reads retire with nothing queued behind)
        mfma_step<0, 1>(acc, f0);
        __builtin_amdgcn_sched_barrier(0);
        load_frags(f1, bA, diag ? bA : bA + kPanelB, ra, rb, 2 + h);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step<1, 4>(acc, f0);
        __builtin_amdgcn_sched_barrier(0);
        // stage t's reads retired (buffer t reusable); the builtin (not asm) lets hipcc's own wait
        // accounting see it, so the MFMAs of f1 below do not wait for f0's new reads
        __builtin_amdgcn_s_waitcnt(0xC07F);             // lgkmcnt(0)
        wait_stage(min(kNBuf - 2, st1 - 2 - t), diag);  // stage t + 1 landed
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");  // no LDS read of stage t + 1 above the barrier
        const uint8_t *nA = buf_of(t + 1);
        load_frags(f0, nA, diag ? nA : nA + kPanelB, ra, rb, h);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step<0, 1>(acc, f1);  // the MFMA pipe restarts before the restaging goes out
        __builtin_amdgcn_sched_barrier(0);
        if (t + kNBuf < st1) issue(t + kNBuf);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step<1, 4>(acc, f1);
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        const uint8_t *bA = buf_of(st1 - 1);
        load_frags(f1, bA, diag ? bA : bA + kPanelB, ra, rb, 2 + h);
        mfma_step(acc, f0);
        mfma_step(acc, f1);
    }
    if (idle) return;  // lower-left quadrant of a diagonal tile: the transpose of the upper-right
    // C/D layout of the 32 x 32 MFMA: column lane & 31, row (j & 3) + 8 (j >> 2) + 4 (lane >> 5)
    uint16_t *out = slab + (long long)w * kTile * kTile;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int row = wm * 128 + 32 * m + (j & 3) + 8 * (j >> 2) + 4 * h;
                const int col = wn * 128 + 32 * n + (lane & 31);
                out[row * kTile + col] = (uint16_t)(uint32_t)acc[m][n][j];
            }
        }
}

// gram[i * ld + j] = sum over the S slices of tile (I, J)'s partials, for i < j < R (the entries the
// pair tables read).  Block (tile, 16-row band); thread: 4 consecutive columns per row.
__global__ __launch_bounds__(256) void ci_gram_reduce(const uint16_t *__restrict__ slab, const int2 *__restrict__ tasks,
                                                      int nt, int S, int R, long long ld, int32_t *__restrict__ gram) {
    const int tile = blockIdx.x, band = blockIdx.y;
    const int2 IJ = tasks[tile];
    const int lr = threadIdx.x >> 6, cq = threadIdx.x & 63;  // 4 rows x 64 column quads per pass
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int ii = band * 16 + p * 4 + lr, jj = cq * 4;
        const int i = IJ.x * kTile + ii, j0 = IJ.y * kTile + jj;
        if (i >= R) continue;
        int sum[4] = {0, 0, 0, 0};
        for (int s = 0; s < S; ++s) {
            const uint2 v = *reinterpret_cast<const uint2 *>(slab + ((long long)(s * nt + tile) * kTile + ii) * kTile + jj);
            sum[0] += (int)(v.x & 0xffff), sum[1] += (int)(v.x >> 16);
            sum[2] += (int)(v.y & 0xffff), sum[3] += (int)(v.y >> 16);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = j0 + k;
            if (j > i && j < R) gram[(long long)i * ld + j] = sum[k];
        }
    }
}

// O4 in stage-major layout: byte (t * Rp + r) * 64 + b holds samples 128 t + 2 b (low nibble) and
// 128 t + 2 b + 1 (high nibble) of leading row r = lead0[v] + a (a < dims[v] - 1): FP4 1.0 (0x2)
// where column v holds value a; samples >= N zero.  A 256-row panel's stage is one contiguous 16 KB
// (full-line global_load_lds).  Rows >= R are left as they are (the caller zeroes them once).
// Thread: 8 samples -> one 32-bit word per row.
__global__ __launch_bounds__(256) void ci_onehot4_build(const uint8_t *__restrict__ cols, const int32_t *__restrict__ dims,
                                                        const int32_t *__restrict__ lead0, long long N, long long KS,
                                                        long long Rp, int nvars, uint8_t *__restrict__ O4) {
    const long long n8 = KS * (kStageS / 8);
    for (int v = blockIdx.y; v < nvars; v += gridDim.y) {
        const int m = dims[v] - 1;
        if (m <= 0) continue;
        const uint8_t *c = cols + (size_t)v * N;
        for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n8; q += (long long)gridDim.x * 256) {
            uint8_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = 8 * q + k < N ? c[8 * q + k] : 0xFF;
            const long long t = q / (kStageS / 8), wq = q % (kStageS / 8);
            for (int a = 0; a < m; ++a) {
                uint32_t word = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) word |= (uint32_t)(x[k] == a ? 2u : 0u) << (4 * k);
                reinterpret_cast<uint32_t *>(O4 + (t * Rp + lead0[v] + a) * kRowB)[wq] = word;
            }
        }
    }
}

}  // namespace

extern "C" int fbn_ci_gram4_tile(void) { return kTile; }
extern "C" int fbn_ci_gram4_stage(void) { return kStageS; }

extern "C" hipError_t fbn_ci_onehot4_build(const uint8_t *cols, const int32_t *dims, const int32_t *lead0, long long N,
                                           long long KS, long long Rp, int nvars, uint8_t *O4, hipStream_t s) {
    const long long g = (KS * (kStageS / 8) + 255) / 256;
    hipLaunchKernelGGL(ci_onehot4_build, dim3((unsigned)(g < 64 ? g : 64), (unsigned)(nvars < 1024 ? nvars : 1024)),
                       dim3(256), 0, s, cols, dims, lead0, N, KS, Rp, nvars, O4);
    return hipGetLastError();
}

// O4: KS stages x Rp rows x 64 bytes (Rp a multiple of 256); tasks: nt device (I, J) pairs; slab:
// nt * S * 256 * 256 uint16.  The host checks KS * 128 / S < 65536 (uint16 partials) and I, J < Rp / 256.
extern "C" hipError_t fbn_ci_gram4(const uint8_t *O4, long long Rp, const int2 *tasks, int nt, int S, int KS,
                                   uint16_t *slab, int R, long long ld, int32_t *gram, hipStream_t s) {
    if (nt <= 0) return hipSuccess;
    hipLaunchKernelGGL(ci_gram_fp4, dim3((unsigned)(nt * S)), dim3(256), 0, s, O4, Rp, tasks, nt, S, KS, slab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ci_gram_reduce, dim3((unsigned)nt, kTile / 16), dim3(256), 0, s, (const uint16_t *)slab, tasks,
                       nt, S, R, ld, gram);
    return hipGetLastError();
}
