// pc_small.h -- the device-resident PC-stable skeleton search for small graphs (pc_small.hip):
// host <-> kernel seam, internal to libfastbn.
//
// One cooperative launch runs every level of the skeleton search (src/PCStable.cpp:49-328): the
// adjacency snapshot lives on the chip, each level's candidate sets are enumerated, counted and
// decided on the device, the first independent set of every edge is found with one atomic per
// independent test, removals are applied after the level (PC-stable) and the FreeDegree rule decides the
// next level -- with one grid barrier per level and no host round trip.  The result record is
// written straight into pinned host memory.
#ifndef FBN_PC_SMALL_H
#define FBN_PC_SMALL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fbn {

constexpr int kSmallMaxVars = 64;                                  // adjacency = one u64 per variable
constexpr int kSmallMaxEdges = kSmallMaxVars * (kSmallMaxVars - 1) / 2;  // 2016
constexpr int kSmallMaxD = 4;           // levels 0..4 on the device; a level d >= 5 hands off to the host
constexpr int kSmallMaxLevels = kSmallMaxD + 1;
constexpr int64_t kSmallMaxTests = 1 << 22;  // a level with more candidate sets hands off to the host

constexpr int kSmallBarWords = 256;  // 8 group counters 64 B apart + the top counter (1 KB)
// barrier words + epoch-tagged first-independent words: zeroed once when the scratch is allocated
// (never per launch: the barrier counts phases across launches, first[] values carry the launch epoch)
constexpr size_t kSmallZeroBytes = (size_t)kSmallBarWords * 4 + (size_t)kSmallMaxLevels * kSmallMaxEdges * 8;

// result record (int32 words; 64-bit values little-endian in two words)
struct PcSmallOut {
    int32_t status;      // 0 ok, 1 grid barrier timed out (kernel gave up), 2 bad argument
    int32_t levels;      // levels completed on the device (0..levels-1)
    int32_t handoff;     // 1: the host continues at level `levels` from adj[levels - 1]
    int32_t pad;
    uint64_t margin_bits;                  // min |p - alpha| over every evaluated test (IEEE bits)
    uint64_t near;                         // tests with |p - alpha| < 1e-9
    int64_t counted[kSmallMaxLevels];      // reference (t = 1) test counts
    int64_t launched[kSmallMaxLevels];     // tests evaluated (speculative ones included)
    uint64_t adj[kSmallMaxLevels][kSmallMaxVars];  // adjacency after each completed level
    int32_t sep_off[kSmallMaxLevels + 1];  // removed edges' sepsets of level d: pool[sep_off[d] ..)
    int32_t pool[kSmallMaxEdges * kSmallMaxD];     // level d: d ints per removed edge, edge order
    // written last (after the record, system-scope release): the launch epoch -- the host polls it
    // instead of synchronizing the stream; never part of the record copy
    uint32_t done;
    uint32_t pad2;
};

struct PcSmallArgs {
    const uint32_t *bits;    // bit-sliced masks: row (row0[v] + a), W words (multiple of 4)
    const int32_t *row0;
    const int32_t *rowcnt;   // samples per mask row
    int nrows;               // mask rows (rowcnt entries)
    long long W;
    const uint32_t *pk;      // 2-bit packed columns: PW words per variable, 16 samples per word
    long long PW;
    const int32_t *dims;
    int nvars;
    long long N;
    double alpha;
    const double *band;      // decision band [lo, hi] per df 1..nband, then delta (or nullptr)
    int nband;
    int depth;               // levels 0 .. depth - 1 at most
    int spec_a;              // levels 1-2: candidate sets per edge in part A (default 8, FBN_PC_SPEC_A)
    // scratch: bar and first zeroed once at allocation (kSmallZeroBytes from its start)
    unsigned *bar;           // grid barrier arrivals (kSmallBarWords), counting phases across launches
    unsigned long long *first;  // [kSmallMaxLevels][kSmallMaxEdges] (epoch << 32) | ~(first independent
                                // candidate); a word of another epoch = none
    unsigned epoch;          // this launch's number (1, 2, ...; never 0)
    unsigned phase_base;     // grid barrier phases completed by the earlier launches on this scratch
    unsigned long long *acc; // [0] margin bits (min), [1] near, [2 + d] launched at level d
    int32_t *pairtab;        // [kSmallMaxEdges][16] level-0 tables (derived level-1 counting)
    unsigned long long *pg2; // [kSmallMaxEdges] level-0 G^2 (fp64 bits) of every pair: the level-1
                             // information screen (nullptr: off)
    unsigned long long *ctx_stats;  // the ctx's margin log, set to this run's at the end
    PcSmallOut *dout;        // the record, built in device memory during the run
    PcSmallOut *out;         // pinned host memory: the record's used part, copied at the end
    // diagnostic (FBN_PC_SMALL_TRACE): wall_clock64 stamps -- [8d + 0] level d's tests start,
    // [8d + 2] its barrier passed, [8d + 3] applied (workgroup 0), [63] kernel start,
    // [64 + 1024 d + b] workgroup b done with level d's tests
    unsigned long long *trace;
};

}  // namespace fbn

extern "C" hipError_t fbn_pc_small_launch(const fbn::PcSmallArgs *a, int grid, long long spin_ticks, int cooperative,
                                          hipStream_t s);
extern "C" int fbn_pc_small_block_threads(void);
extern "C" hipError_t fbn_pc_small_occupancy(int *blocks_per_cu);

#endif
