// capi.hip -- the extern "C" boundary (include/fastbn.h): handles, device memory, uploads, launches.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocblas/rocblas.h>
#include <dlfcn.h>
#include <chrono>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <new>
#include <string>

#include "fbn_internal.h"
#include "pc_internal.h"
#include "ci_chisq.h"
#include "pc_small.h"

extern "C" hipError_t fbn_jt_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                    const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                    double *marg, int32_t *labels, double *ws, int32_t *wsi, long long NE, int nc,
                                    int grid, int vmajor, hipStream_t stream);
extern "C" hipError_t fbn_jt_marg_transpose(const double *in, double *out, long long n, int SD, hipStream_t s);
extern "C" hipError_t fbn_jt_score_terms(const double *marg, const double *golden, long long n, int SD, int vmajor,
                                         const int32_t *dom, int V, double *terms, hipStream_t s);
extern "C" hipError_t fbn_ci_launch(const uint8_t *cols, const int32_t *dims, const int32_t *items, long long N,
                                    long long n, int d, double alpha, double *g2, int32_t *df, double *p,
                                    uint8_t *indep, int32_t *counts, size_t lds_bytes, int grid,
                                    int32_t *gscratch, unsigned long long *stats, const uint32_t *bits,
                                    const int32_t *row0, long long W, const double *band, int nband,
                                    const uint32_t *pk, long long PW, long long cstride, int32_t *tab,
                                    long long tstride, int split, int split_grid, const int32_t *pairtab,
                                    int nvars, hipStream_t stream);
extern "C" hipError_t fbn_ci_pack2_build(const uint8_t *cols, int nvars, long long N, long long PW, uint32_t *pk,
                                         hipStream_t stream);
extern "C" size_t fbn_ci_lds_bytes(int dimz, int dx, int dy);
extern "C" hipError_t fbn_jt_evidence_check(const int8_t *ev, long long n, int V, const int32_t *dom,
                                            unsigned long long *first, hipStream_t s);
extern "C" hipError_t fbn_ci_cols_check(const uint8_t *cols, const int32_t *dims, int nvars, long long N, int *bad,
                                        hipStream_t s);
extern "C" hipError_t fbn_ci_bits_build(const uint8_t *cols, const int32_t *dims, const int32_t *row0, long long N,
                                        long long W, int nvars, uint32_t *bits, hipStream_t s);
extern "C" hipError_t fbn_ci_bits_launch(const uint32_t *bits, const int32_t *dims, const int32_t *row0,
                                         const int32_t *items, long long W, long long n, int d, double alpha,
                                         double *g2, int32_t *df, double *p, uint8_t *indep, int32_t *counts,
                                         int32_t *counts0, unsigned long long *stats, const int32_t *rowcnt,
                                         int32_t *pairtab, int pmode, int nvars, int num_cu, long long t0,
                                         int counted, const double *band, int nband, hipStream_t s);
extern "C" hipError_t fbn_ci_bits_rowcount(const uint32_t *bits, long long rows, long long W, int32_t *rowcnt,
                                           hipStream_t s);
extern "C" int fbn_ci_pair_block(int d);
extern "C" int fbn_ci_gram_task_ints(void);
extern "C" hipError_t fbn_ci_onehot4_build(const uint8_t *cols, const int32_t *dims, const int32_t *lead0, long long N,
                                           long long KS, long long Rp, int nvars, uint8_t *O4, hipStream_t s);
extern "C" hipError_t fbn_ci_gram4(const uint8_t *O4, long long Rp, const int2 *tasks, int nt, int S, int KS,
                                   uint16_t *slab, int R, long long ld, int32_t *gram, hipStream_t s);
extern "C" int fbn_ci_gram4_tile(void);
extern "C" int fbn_ci_gram4_stage(void);
extern "C" hipError_t fbn_ci_sum_planes(const int32_t *planes, int np, long long n, int32_t *out, hipStream_t s);
extern "C" hipError_t fbn_ci_onehot_build(const uint8_t *cols, const int32_t *dims, const int32_t *lead0, long long N,
                                          long long Npad, int nvars, int8_t *out, hipStream_t s);
extern "C" size_t fbn_ci_l1_edge_bytes(void);
extern "C" hipError_t fbn_ci_l1_results(const uint8_t *st, const int32_t *sep, const long long *cnt, int E,
                                        const long long *scal, char *h_rm, int32_t *h_sep, long long *h_sc,
                                        long long *part, hipStream_t s);
extern "C" hipError_t fbn_ci_kept_csr(const uint8_t *indep, int n, int32_t *low, int32_t *up, int32_t *off,
                                      int32_t *upoff, int32_t *adj, int32_t *pairs, long long *scal, hipStream_t s);
extern "C" hipError_t fbn_ci_l1_setup(const int32_t *pairs, int E, const int32_t *adj, const int32_t *adj_off,
                                      void *ed, int32_t *pos, uint8_t *st, int32_t *sep, long long *counted,
                                      int chunk0, int32_t *len, int32_t *off, unsigned *ring,
                                      unsigned long long *sstat, long long cap, long long *scal, int num_cu,
                                      const int32_t *pairtab, double *mi, int mi_from_tables, const int32_t *dims,
                                      const double *band, int nband, int nv, double two_n, int32_t *pcnt,
                                      int32_t *plist, unsigned long long *sstat2, long long *scal2, hipStream_t s);
extern "C" hipError_t fbn_ci_l1_round(const uint32_t *bits, const int32_t *dims, const int32_t *row0, long long W,
                                      const int32_t *adj, const int32_t *pairtab, int nvars, void *edv, int32_t *pos,
                                      uint8_t *st, int32_t *sep, long long *counted, int32_t *len, int32_t *off,
                                      int E, long long cap, long long *scal, int32_t *items, int32_t *counts,
                                      int32_t *df, uint8_t *indep, double alpha, unsigned long long *stats,
                                      const double *band, int nband, unsigned *open_cnt, int num_cu,
                                      unsigned *open_next, int next_chunk, unsigned long long *sstat, unsigned epoch,
                                      const int32_t *plist, hipStream_t s);
extern "C" hipError_t fbn_ci_gram(const uint32_t *bits, long long W, const int32_t *rl, const int32_t *tasks,
                                  long long ntasks, int masked, int32_t *out, int num_cu, hipStream_t s);
extern "C" hipError_t fbn_ci_gram_pairs(const int32_t *G, long long ld, const int32_t *lead0, const int32_t *dims,
                                        const int32_t *row0, const int32_t *rowcnt, long long t0, long long n,
                                        int nvars, int32_t *counts, int32_t *pairtab, int num_cu, hipStream_t s);
extern "C" hipError_t fbn_ci_gram_triples(const int32_t *G, const long long *goff, const int32_t *gR,
                                          const int32_t *adj, const int32_t *adj_off, const int32_t *loff,
                                          const int32_t *dims, const int32_t *items, long long n, int32_t *counts,
                                          const int32_t *pairtab, int nvars, int num_cu, hipStream_t s);
extern "C" hipError_t fbn_ci_bits_pairs_tiled(const uint32_t *bits, const int32_t *row0, const int32_t *rowcnt,
                                              long long W, const int32_t *tasks, long long ntasks, int nvars,
                                              long long t0, long long t1, int32_t *counts, int32_t *pairtab,
                                              int num_cu, hipStream_t s);
extern "C" hipError_t fbn_jt_tile_launch(const JtTPass *passes, int npass, const int32_t *tab, const double *iv,
                                         const int8_t *evid, double *marg, int32_t *labels, double *ws, int *flags,
                                         long long ncases, long long store_rows, long long scr_row, long long red_row,
                                         int V, int SD, int lds_bytes, int grid, int waves,
                                         unsigned long long *prof, hipStream_t stream);
extern "C" hipError_t fbn_jt_virt_launch(const JtVClique *cls, const int32_t *aux, const double *initv,
                                         const uint64_t *dig, const int32_t *order, const int32_t *sched,
                                         const int32_t *vsel, const int8_t *evid, double *marg, int32_t *labels,
                                         double *ws, int32_t *wsi, int *flags, long long ncases, long long store_rows,
                                         long long scratch_row, long long scratch_rows, int nc, int V, int SD,
                                         int grid, int dbg, hipStream_t stream);
extern "C" hipError_t fbn_jt_lds_launch(const JtOp *ops, int nops, const int32_t *aux, const double *initv,
                                        const uint64_t *dig, const int8_t *evid, int V, long long ncases, int SD,
                                        double *marg, int32_t *labels, double *ws, int32_t *wsi, long long wave_entries,
                                        long long store_off, long long den_off, long long sep_off,
                                        long long spill_off, int nc, int cap, bool spill, int force_exact,
                                        const int *flags, int grid, unsigned long long *prof, int vmajor,
                                        hipStream_t stream);

namespace fbn {
const char *LastError();
extern const char *kJitOptions[];
extern const int kJitNumOptions;
std::string JitCachePath(const std::string &src);
int JitCodeObject(const std::string &src, std::vector<char> &code);
}
using fbn::SetError;

#define FBN_HIP(call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) return SetError(FBN_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

namespace {

// growable device buffer
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t b) {
        if (b <= bytes) return FBN_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (b == 0) return FBN_OK;
        hipError_t e = hipMalloc(&p, b);
        if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipMalloc(%zu): %s", b, hipGetErrorString(e));
        bytes = b;
        return FBN_OK;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

int CheckDevice(int device, int *num_cu) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return SetError(FBN_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return SetError(FBN_ERR_NODEV, "device %d out of range (%d visible)", device, n);
    FBN_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    FBN_HIP(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return SetError(FBN_ERR_NODEV, "device %d is %s; libfastbn is built for gfx950 only", device, prop.gcnArchName);
    if (num_cu) *num_cu = prop.multiProcessorCount;
    return FBN_OK;
}

}  // namespace

// =============================================================================================

struct fbn_jt_plan {
    fbn::JTPlanHost host;
    fbn::JTProgram prog;      // variant 1: whole case state in a global workspace
    fbn::JTProgramLDS lprog;  // variant 0 (default): clique in flight resident in LDS
    fbn::JTProgramV vprog;    // variant 4: streamed (virtual) tables, large trees
    bool v_ok = false;
    DevBuf vcl, vaux, viv, vdig, vorder, vsched, vsel;
    fbn::JTProgramT tprog;    // variant 5: tiled, JT_T_C cases x JT_T_L entry slots per wave (fast order)
    bool t_ok = false;
    DevBuf tpass, ttab, tiv;
    int device = 0, num_cu = 0, waves_per_cu = 0, variant = -1, last_variant = -1;
    // plan-specialized kernel (variant 3)
    bool gen_eligible = false;
    // one loaded module (and initial-potential buffer) per arithmetic order, [0] exact, [1] fast:
    // switching the order never unloads a module or rewrites a buffer a queued run may still use
    struct GenKernel {
        int state = 0;  // 0 not tried, 1 loaded, -1 failed
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr;
        int64_t we = 0, lds = 0;
        DevBuf iv;
    } gen[4];  // [fast + 2 * variable-major output]
    int64_t last_nblk = 0;  // 64-case blocks of the last run (flags of variants 3-5)
    DevBuf flags, ws_fix;
    bool force_fixup = false;
    // arithmetic order of the specialized / streamed kernels: 1 = the reference's (bit-identical),
    // 0 = fast (normalizations that cancel left out, within 1e-12), -1 = auto (fast)
    int exact = -1;
    DevBuf ops, aux, initv, dig;
    DevBuf lops, laux, linitv, ldig;
    DevBuf prof;       // diagnostic per-op-type cycle counters
    bool prof_on = false;
    int last_grid = 0;
    DevBuf evid, labels, marg, ws;
    // fbn_jt_set_output_layout: 1 = d_marginals variable-major [SD][ncases]; kernels without a
    // variable-major store path (4, 5) write case-major into mtmp, transposed into place after
    int out_layout = 0;
    DevBuf mtmp;
    DevBuf ddom, evcheck;  // device-side evidence range check (fbn_jt_run, fbn_jt_run_device)
    bool ev_check = true;  // fbn_jt_set_evidence_check
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false, ktiming = true;
    // the caller streams runs were queued on (fbn_jt_run_device returns before its kernels end):
    // fbn_jt_plan_destroy drains these, not the whole device
    std::vector<hipStream_t> streams_used;
    void note_stream(hipStream_t s) {
        for (hipStream_t u : streams_used)
            if (u == s) return;
        streams_used.push_back(s);
    }
    ~fbn_jt_plan() {
        for (auto &k : gen)
            if (k.mod) (void)hipModuleUnload(k.mod);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
    }
};

// per-slot state of the CI launches: the PC driver keeps two batches in flight (one per half of
// the level's edges) on the ctx stream, so every buffer a launch (re)sizes or writes is per slot
struct CiSlot {
    DevBuf items, indep, df, bcounts, scratch;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;  // kernel start / end, batch results ready
    int64_t last_bytes = 0;  // input bytes of the last launch in the kernel's own format (roofline)
    // pinned host staging of the driver's batches
    void *h_items = nullptr, *h_res = nullptr;
    size_t h_items_bytes = 0, h_res_bytes = 0;
    int64_t n = 0;  // batch in flight
    bool zc = false, want_df = false;
    ~CiSlot() {
        if (h_items) (void)hipHostFree(h_items);
        if (h_res) (void)hipHostFree(h_res);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (done) (void)hipEventDestroy(done);
    }
};

struct fbn_ci_ctx {
    int device = 0, num_cu = 0, nvars = 0;
    int64_t N = 0;
    std::vector<int32_t> dims;
    DevBuf cols, ddims, g2, p, counts;
    DevBuf stats;  // decision-margin log: {min |p - alpha| bits, #tests within 1e-9 of alpha}
    // bit-sliced columns for marginal tests (ci_bits.hip), built on first use
    DevBuf bits, brow, browcnt;  // masks, first row of each variable, sample count per row
    DevBuf pack2;                // 2-bit packed columns (every state count <= 4), built on first use
    bool pack2_ready = false;
    int64_t pack2_W = 0;
    // pair tables of every (i < j), 16 counts each, recorded by level 0 of a PC run and used by its
    // level-1 tests (pair_mode: 0 off, 1 record at the next marginal batch, 2 use if recorded)
    DevBuf pairtab;
    // register-blocked level-0 tasks (ci_bits_pairs_tiled) of the pair range [ptask_t0, ptask_t1)
    DevBuf ptasks;
    int64_t ptask_t0 = -1, ptask_t1 = -1, ptask_n = 0;
    int pair_mode = 0;
    bool pairs_recorded = false;
    // row Grams (ci_bits.hip ci_bits_gram): leading rows = values 0..d-2 of every variable;
    // lead0[v] = v's first leading row, leadrows[r] = the bits row of leading row r
    std::vector<int32_t> row0_host, lead0_host, leadrows_host;
    DevBuf lead0, leadrows;
    bool lead_ready = false;
    // level 0: the Gram of all leading rows (ld = leading-row count) and its tile tasks for the
    // pair range [g0_t0, g0_t1)
    DevBuf gram0, g0tasks;
    int64_t g0_t0 = -1, g0_t1 = -1, g0_ntasks = 0;
    // level 1: per-variable masked Grams over the neighbours' leading rows (CiTriplePrepare), used
    // by the next d = 1 batches while triples_ready
    DevBuf g1, g1tasks, g1rl, g1goff, g1R, g1adj, g1adjoff, g1loff;
    bool triples_ready = false;
    // device-resident level-1 search (CiLevel1Device): edge state, round buffers, per-round open
    // counts (pinned mirror), round events
    DevBuf l1pairs, l1adj, l1adjoff, l1ed, l1pos, l1st, l1sep, l1cnt, l1len, l1off, l1scal, l1open;
    DevBuf l1items, l1counts, l1df, l1indep, l1sstat;  // l1sstat: the offset scan's per-tile status words
    // the level-1 information screen (ci_bits.hip): pairwise I of the complete graph, the kept
    // candidates' positions, the screen's scan status words
    DevBuf l1mi, l1pcnt, l1plist, l1sstat2;
    // level 0's G^2 of every pair written into l1mi by the recording batches (pairs [0, covered) in
    // order; == all pairs: the screen needs no recomputation from the pair tables)
    int64_t l1mi_covered = 0;
    DevBuf keptidx, kepttmp;  // level-0 kept pair indices (CiAllPairsKept)
    // level 0 -> level 1 on the device (CiL0L1Device): per-variable kept counts, upper-part offsets,
    // (E, candidate sets); the side stream copies the flags / edge list to the host meanwhile
    DevBuf kcnt, kupoff, kscal, l1part;
    hipStream_t side = nullptr;
    hipEvent_t side_ev = nullptr, main_ev = nullptr;
    void *h_pairs = nullptr;
    size_t h_pairs_bytes = 0;
    // level-0 Gram on the matrix cores (ci_gram_mfma.hip): FP4 one-hot store (Rp x Kb bytes, built
    // once, stage-major), the tile list of row range [g4_r0, g4_r1), split-K slabs
    DevBuf onehot4, g4tasks, g4slab;
    int64_t g4_r0 = -1, g4_r1 = -1;
    int g4_nt = 0;
    bool onehot4_ready = false;
    // level-0 Gram as an int8 library GEMM (FBN_CI_GRAM_ROCBLAS=1 only: the measured alternative)
    DevBuf onehot, gram0split;
    int64_t onehot_Npad = 0;
    bool onehot_ready = false, blas_failed = false;
    void *blas = nullptr;
    int *h_kept = nullptr;
    unsigned *h_open = nullptr;
    void *h_xfer = nullptr;  // pinned staging of level-0 kept pairs / level-1 results (read-back)
    size_t h_xfer_bytes = 0;
    unsigned long long *h_margin = nullptr;  // pinned: reset value, read-back (CiResetMargin)
    hipEvent_t l1ev[2] = {nullptr, nullptr};
    // device-resident skeleton search of small graphs (pc_small.hip): scratch (barrier counters +
    // first-independent words, zeroed once; statistics slots; level-0 pair tables) and the
    // pinned result record the kernel writes
    DevBuf small_scr;
    void *small_zeroed = nullptr;       // scratch whose barrier / first[] words are zeroed (and its size)
    size_t small_zeroed_bytes = 0;
    unsigned small_epoch = 0, small_phase = 0;  // launches so far, grid-barrier phases so far
    fbn::PcSmallOut *h_small = nullptr;
    // fbn_ci_debug_counts: the histogram kernel writes every test's table (stride in ints), 0 off
    int64_t counts_stride = 0;
    // decision band of the bit-sliced G^2 kernel for alpha = band_alpha (ci_chisq.h fbn_chisq_band):
    // [lo, hi] per df 1..kBandDf, then delta; host copy kept alive for the async upload
    DevBuf band;
    std::vector<double> band_host;
    double band_alpha = -1.0;
    int band_n = 0;
    bool bits_ready = false;
    int64_t bits_W = 0;
    CiSlot slot[2];
    hipStream_t stream = nullptr;  // the PC driver's rounds (pinned staging, one sync per round)
    std::vector<hipStream_t> streams_used;  // caller streams of fbn_ci_run (drained by fbn_ci_ctx_destroy)
    float last_ms = 0.f;
    bool timing = true;  // HIP events around every CI kernel (fbn_ci_set_kernel_timing)
    ~fbn_ci_ctx();
    void destroy_() {
        if (h_open) (void)hipHostFree(h_open);
        if (h_margin) (void)hipHostFree(h_margin);
        if (h_kept) (void)hipHostFree(h_kept);
        if (h_xfer) (void)hipHostFree(h_xfer);
        if (h_small) (void)hipHostFree(h_small);
        for (auto &e : l1ev)
            if (e) (void)hipEventDestroy(e);
        if (h_pairs) (void)hipHostFree(h_pairs);
        if (side_ev) (void)hipEventDestroy(side_ev);
        if (main_ev) (void)hipEventDestroy(main_ev);
        if (side) (void)hipStreamDestroy(side);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

static int64_t EnvOr0(const char *name, int64_t dflt) {
    const char *v = getenv(name);
    return v ? atoll(v) : dflt;
}

// Wait for a PC round's event: hipEventSynchronize, or with FBN_CI_SPIN = 1 by polling it from
// this thread (measured on ALARM-5000 / config 5: no faster than HIP's own wait, so off)
static hipError_t EventWaitSpin(hipEvent_t ev) {
    static const bool spin = EnvOr0("FBN_CI_SPIN", 0) != 0;
    if (!spin) return hipEventSynchronize(ev);
    hipError_t e;
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
    }
    return e;
}

// df <= 36 covers every bit-sliced test (<= 4 states, <= 1 conditioning variable: 4 * 3 * 3)
constexpr int kBandDf = 36;
constexpr int kBandDfMax = 256;  // larger df (few tests, deep levels): p evaluated

// the band for `alpha` (delta = alpha / 1024: few tests fall inside, so few evaluate p) over df 1..max(want_df, kBandDf) (at most kBandDfMax),
// computed on the host per ctx and alpha and extended on demand; *out = nullptr (p evaluated for
// every test) when alpha is outside (0, 1) or FBN_CI_NO_BAND is set
static int CiBand(fbn_ci_ctx *c, double alpha, hipStream_t s, const double **out, int *nband, int want_df = 0) {
    *out = nullptr;
    *nband = 0;
    if (!(alpha > 0.0 && alpha < 1.0) || getenv("FBN_CI_NO_BAND")) return FBN_OK;
    const int want = std::min(kBandDfMax, std::max(kBandDf, want_df));
    if (c->band_alpha != alpha || c->band_n < want) {
        const double delta = alpha / 1024;
        const int have = c->band_alpha == alpha ? c->band_n : 0;
        FBN_HIP(hipStreamSynchronize(s));  // the previous upload of the host table has completed
        c->band_host.resize(2 * (size_t)want + 1);
        for (int df = have + 1; df <= want; ++df)
            fbn_chisq_band(alpha, delta, df, &c->band_host[2 * df - 2], &c->band_host[2 * df - 1]);
        c->band_host[2 * (size_t)want] = delta;
        if (int rc = c->band.ensure(c->band_host.size() * 8)) return rc;
        FBN_HIP(hipMemcpyAsync(c->band.p, c->band_host.data(), c->band_host.size() * 8, hipMemcpyHostToDevice, s));
        c->band_alpha = alpha;
        c->band_n = want;
    }
    *out = c->band.as<double>();
    *nband = c->band_n;
    return FBN_OK;
}

// rocBLAS, resolved at first use (dlopen): the level-0 Gram is a plain int8 GEMM (O O^T of the
// one-hot leading rows); without the library the popcount Gram kernel computes it
struct BlasLib {
    bool ok = false;
    rocblas_status (*create)(rocblas_handle *) = nullptr;
    rocblas_status (*destroy)(rocblas_handle) = nullptr;
    rocblas_status (*set_stream)(rocblas_handle, hipStream_t) = nullptr;
    rocblas_status (*gemm_ex)(rocblas_handle, rocblas_operation, rocblas_operation, rocblas_int, rocblas_int,
                              rocblas_int, const void *, const void *, rocblas_datatype, rocblas_int, const void *,
                              rocblas_datatype, rocblas_int, const void *, const void *, rocblas_datatype, rocblas_int,
                              void *, rocblas_datatype, rocblas_int, rocblas_datatype, rocblas_gemm_algo, int32_t,
                              uint32_t) = nullptr;
    rocblas_status (*gemm_sb_ex)(rocblas_handle, rocblas_operation, rocblas_operation, rocblas_int, rocblas_int,
                                 rocblas_int, const void *, const void *, rocblas_datatype, rocblas_int, rocblas_stride,
                                 const void *, rocblas_datatype, rocblas_int, rocblas_stride, const void *,
                                 const void *, rocblas_datatype, rocblas_int, rocblas_stride, void *,
                                 rocblas_datatype, rocblas_int, rocblas_stride, rocblas_int, rocblas_datatype,
                                 rocblas_gemm_algo, int32_t, uint32_t) = nullptr;
};
static BlasLib &Blas() {
    static BlasLib b = [] {
        BlasLib r;
        void *h = dlopen("librocblas.so.5", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librocblas.so.5", RTLD_NOW);
        if (!h) return r;
        r.create = (decltype(r.create))dlsym(h, "rocblas_create_handle");
        r.destroy = (decltype(r.destroy))dlsym(h, "rocblas_destroy_handle");
        r.set_stream = (decltype(r.set_stream))dlsym(h, "rocblas_set_stream");
        r.gemm_ex = (decltype(r.gemm_ex))dlsym(h, "rocblas_gemm_ex");
        r.gemm_sb_ex = (decltype(r.gemm_sb_ex))dlsym(h, "rocblas_gemm_strided_batched_ex");
        r.ok = r.create && r.destroy && r.set_stream && r.gemm_ex;
        return r;
    }();
    return b;
}
fbn_ci_ctx::~fbn_ci_ctx() {
    if (blas) (void)Blas().destroy((rocblas_handle)blas);
    destroy_();
}

static int PinnedEnsure(void *&ptr, size_t &have, size_t want) {
    if (want <= have) return FBN_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    have = 0;
    want = std::max<size_t>(want, 1 << 16) * 2;
    hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocDefault);
    if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc(%zu): %s", want, hipGetErrorString(e));
    have = want;
    return FBN_OK;
}

// The margin log lives on the device (atomics of every batch kernel); reset and read are
// stream-ordered copies through a pinned 32-byte buffer ([0..1] the reset value, constant; [2..3]
// the read-back).  Work the caller queued on its own streams (fbn_ci_run_device) is drained first.
static int CiMarginPinned(fbn_ci_ctx *c) {
    if (c->h_margin) return FBN_OK;
    hipError_t e = hipHostMalloc((void **)&c->h_margin, 32, hipHostMallocDefault);
    if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc: %s", hipGetErrorString(e));
    c->h_margin[0] = 0x7FF0000000000000ull;  // +inf
    c->h_margin[1] = 0;
    return FBN_OK;
}

static int CiResetMargin(fbn_ci_ctx *c) {
    if (int rc = CiMarginPinned(c)) return rc;
    FBN_HIP(hipDeviceSynchronize());
    FBN_HIP(hipMemcpyAsync(c->stats.p, c->h_margin, 16, hipMemcpyHostToDevice, c->stream));
    return FBN_OK;
}

static int CiReadMargin(fbn_ci_ctx *c, double *min_margin, int64_t *near_alpha, bool own_stream_only = false) {
    if (int rc = CiMarginPinned(c)) return rc;
    if (!own_stream_only) FBN_HIP(hipDeviceSynchronize());
    FBN_HIP(hipMemcpyAsync(c->h_margin + 2, c->stats.p, 16, hipMemcpyDeviceToHost, c->stream));
    FBN_HIP(hipStreamSynchronize(c->stream));
    double m;
    memcpy(&m, &c->h_margin[2], 8);
    if (min_margin) *min_margin = m;
    if (near_alpha) *near_alpha = (int64_t)c->h_margin[3];
    return FBN_OK;
}

// =============================================================================================
extern "C" {

const char *fbn_last_error(void) { return fbn::LastError(); }

int fbn_version(int *major, int *minor) {
    if (major) *major = 0;
    if (minor) *minor = 1;
    return FBN_OK;
}

int fbn_device_count(int *n) {
    if (!n) return SetError(FBN_ERR_ARG, "null pointer");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return FBN_OK;
}

// ------------------------------------------------------------------ networks & data
int fbn_network_load_xmlbif(const char *path, fbn_network **out) {
    if (!path || !out) return SetError(FBN_ERR_ARG, "null pointer");
    auto h = std::unique_ptr<fbn_network>(new (std::nothrow) fbn_network());
    if (!h) return SetError(FBN_ERR_NOMEM, "out of memory");
    int rc = fbn::LoadXmlbif(path, h->net);
    if (rc) return rc;
    *out = h.release();
    return FBN_OK;
}
int fbn_network_create(int nvars, const int32_t *dims, const int32_t *parent_off, const int32_t *parents,
                       const int64_t *counts, const char *const *names, fbn_network **out) {
    if (!out) return SetError(FBN_ERR_ARG, "null pointer");
    auto h = std::unique_ptr<fbn_network>(new (std::nothrow) fbn_network());
    if (!h) return SetError(FBN_ERR_NOMEM, "out of memory");
    int rc = fbn::BuildNetwork(nvars, dims, parent_off, parents, counts, names, h->net);
    if (rc) return rc;
    *out = h.release();
    return FBN_OK;
}
int fbn_network_node_counts(const fbn_network *net, int node, int32_t *parents, int64_t *counts, int *nparents,
                            int64_t *ncounts) {
    if (!net) return SetError(FBN_ERR_ARG, "null pointer");
    return fbn::NodeCounts(net->net, node, parents, counts, nparents, ncounts);
}
int fbn_network_num_nodes(const fbn_network *net, int *n) {
    if (!net || !n) return SetError(FBN_ERR_ARG, "null pointer");
    *n = net->net.n();
    return FBN_OK;
}
int fbn_network_dims(const fbn_network *net, int32_t *dims) {
    if (!net || !dims) return SetError(FBN_ERR_ARG, "null pointer");
    for (int i = 0; i < net->net.n(); ++i) dims[i] = net->net.dom[i];
    return FBN_OK;
}
int fbn_network_name(const fbn_network *net, int node, char *buf, int cap) {
    if (!net || !buf || cap <= 0 || node < 0 || node >= net->net.n()) return SetError(FBN_ERR_ARG, "bad argument");
    snprintf(buf, cap, "%s", net->net.names[node].c_str());
    return FBN_OK;
}
int fbn_network_destroy(fbn_network *net) {
    delete net;
    return FBN_OK;
}

int fbn_evidence_load_libsvm(const char *path, int num_nodes, int8_t *evidence, int32_t *labels, int64_t cap,
                             int64_t *ncases) {
    if (!path || num_nodes <= 0) return SetError(FBN_ERR_ARG, "bad argument");
    // streaming parse straight into the caller's rows (no intermediate copy)
    return fbn::LoadLibsvm(path, num_nodes, evidence && cap > 0 ? evidence : nullptr, labels, cap, ncases);
}

int fbn_dataset_load_csv(const char *path, fbn_dataset **out) {
    if (!path || !out) return SetError(FBN_ERR_ARG, "null pointer");
    auto h = std::unique_ptr<fbn_dataset>(new (std::nothrow) fbn_dataset());
    if (!h) return SetError(FBN_ERR_NOMEM, "out of memory");
    int rc = fbn::LoadCsv(path, h->ds);
    if (rc) return rc;
    *out = h.release();
    return FBN_OK;
}
int fbn_dataset_shape(const fbn_dataset *ds, int *nvars, int64_t *nsamples) {
    if (!ds) return SetError(FBN_ERR_ARG, "null pointer");
    if (nvars) *nvars = ds->ds.nvars;
    if (nsamples) *nsamples = ds->ds.nsamples;
    return FBN_OK;
}
int fbn_dataset_dims(const fbn_dataset *ds, int32_t *dims) {
    if (!ds || !dims) return SetError(FBN_ERR_ARG, "null pointer");
    std::copy(ds->ds.dims.begin(), ds->ds.dims.end(), dims);
    return FBN_OK;
}
int fbn_dataset_columns(const fbn_dataset *ds, uint8_t *cols) {
    if (!ds || !cols) return SetError(FBN_ERR_ARG, "null pointer");
    std::copy(ds->ds.cols.begin(), ds->ds.cols.end(), cols);
    return FBN_OK;
}
int fbn_dataset_var_name(const fbn_dataset *ds, int v, char *buf, int cap) {
    if (!ds || !buf || cap <= 0 || v < 0 || v >= ds->ds.nvars) return SetError(FBN_ERR_ARG, "bad argument");
    snprintf(buf, cap, "%s", ds->ds.names[v].c_str());
    return FBN_OK;
}
int fbn_dataset_destroy(fbn_dataset *ds) {
    delete ds;
    return FBN_OK;
}

// ------------------------------------------------------------------ junction tree
static int JtUpload(fbn_jt_plan *p) {
    auto up = [](DevBuf &b, const void *src, size_t bytes) -> int {
        int rc = b.ensure(std::max<size_t>(bytes, 8));
        if (rc) return rc;
        if (bytes) FBN_HIP(hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
        return FBN_OK;
    };
    const auto &g = p->prog;
    int rc;
    if ((rc = up(p->ops, g.ops.data(), g.ops.size() * sizeof(JtOp)))) return rc;
    if ((rc = up(p->aux, g.aux.data(), g.aux.size() * 4))) return rc;
    if ((rc = up(p->initv, g.initv.data(), g.initv.size() * 8))) return rc;
    if ((rc = up(p->dig, g.dig.data(), g.dig.size() * 8))) return rc;
    const auto &l = p->lprog;
    if ((rc = up(p->lops, l.ops.data(), l.ops.size() * sizeof(JtOp)))) return rc;
    if ((rc = up(p->laux, l.aux.data(), l.aux.size() * 4))) return rc;
    if ((rc = up(p->linitv, l.initv.data(), l.initv.size() * 8))) return rc;
    if ((rc = up(p->ldig, l.dig.data(), l.dig.size() * 8))) return rc;
    if (p->v_ok) {
        const auto &v = p->vprog;
        if ((rc = up(p->vcl, v.cl.data(), v.cl.size() * sizeof(JtVClique)))) return rc;
        if ((rc = up(p->vaux, v.aux.data(), v.aux.size() * 4))) return rc;
        if ((rc = up(p->viv, v.initv.data(), v.initv.size() * 8))) return rc;
        if ((rc = up(p->vdig, v.dig.data(), v.dig.size() * 8))) return rc;
        if ((rc = up(p->vorder, v.order.data(), v.order.size() * 4))) return rc;
        if ((rc = up(p->vsched, v.sched.data(), v.sched.size() * 4))) return rc;
        if ((rc = up(p->vsel, v.vsel.data(), v.vsel.size() * 4))) return rc;
    }
    if (p->t_ok) {
        const auto &t = p->tprog;
        if ((rc = up(p->tpass, t.passes.data(), t.passes.size() * sizeof(JtTPass)))) return rc;
        if ((rc = up(p->ttab, t.tab.data(), t.tab.size() * 4))) return rc;
        if ((rc = up(p->tiv, t.initv.data(), t.initv.size() * 8))) return rc;
    }
    return FBN_OK;
}

int fbn_jt_plan_create(const fbn_network *net, int device, fbn_jt_plan **out) {
    if (!net || !out) return SetError(FBN_ERR_ARG, "null pointer");
    auto p = std::unique_ptr<fbn_jt_plan>(new (std::nothrow) fbn_jt_plan());
    if (!p) return SetError(FBN_ERR_NOMEM, "out of memory");
    static const bool ptime = getenv("FBN_PLAN_TIMING") != nullptr;  // diagnostic: plan phases
    auto tp0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!ptime) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "plan %s: %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - tp0).count());
        tp0 = t;
    };
    int rc = fbn::BuildJTPlan(net->net, p->host);
    if (rc) return rc;
    lap("structure");
    rc = fbn::CompileJTProgram(p->host, p->prog);
    if (rc) return rc;
    rc = fbn::CompileJTProgramLDS(p->host, p->lprog);
    if (rc) return rc;
    lap("interpreter programs");
    rc = fbn::CompileJTProgramV(p->host, p->vprog);
    if (rc && rc != FBN_ERR_LIMIT) return rc;
    p->v_ok = rc == FBN_OK;
    if (!p->v_ok) p->vprog = fbn::JTProgramV();
    lap("streamed program");
    // tiled variant: factors of a clique phase staged in LDS up to this many bytes per wave
    // LDS factor budget per workgroup (tuning knob): 6016 B + the bin and total rows = 10 KB, so 16
    // one-wave workgroups fit a CU's 160 KB
    static const int t_lds = getenv("FBN_JT_TLDS") ? atoi(getenv("FBN_JT_TLDS")) : 6016;
    rc = fbn::CompileJTProgramT(p->host, p->tprog, t_lds);
    if (rc && rc != FBN_ERR_LIMIT) return rc;
    p->t_ok = rc == FBN_OK;
    if (!p->t_ok) p->tprog = fbn::JTProgramT();
    lap("tiled program");
    p->gen_eligible = fbn::JTCodegenEligible(p->host, nullptr);
    p->device = device;
    if (device >= 0) {  // device < 0: host-only plan (info / dump), runs fail with FBN_ERR_NODEV
        rc = CheckDevice(device, &p->num_cu);
        if (rc) return rc;
        rc = JtUpload(p.get());
        if (rc) return rc;
        FBN_HIP(hipEventCreate(&p->ev0));
        FBN_HIP(hipEventCreate(&p->ev1));
    }
    *out = p.release();
    return FBN_OK;
}

int fbn_jt_plan_info_get(const fbn_jt_plan *p, fbn_jt_plan_info *info) {
    if (!p || !info) return SetError(FBN_ERR_ARG, "null pointer");
    memset(info, 0, sizeof *info);
    info->num_nodes = p->host.num_nodes;
    info->num_cliques = (int32_t)p->host.cliques.size();
    info->num_separators = (int32_t)p->host.seps.size();
    info->num_levels = (int32_t)p->host.levels.size();
    info->root = p->host.root;
    info->sum_dom = p->prog.sum_dom;
    for (auto &t : p->host.cliques) info->clique_entries += t.size();
    for (auto &t : p->host.seps) info->separator_entries += t.size();
    info->algorithmic_bytes_per_case =
        16 * (info->clique_entries + info->separator_entries) + 8 * (int64_t)info->sum_dom + info->num_nodes;
    info->num_ops = (int32_t)p->prog.ops.size();
    info->max_vars_per_table = p->prog.max_vars;
    info->specialized_eligible = p->gen_eligible ? 1 : 0;
    info->variant = p->variant >= 0 ? p->variant : p->last_variant;
    info->streamed_eligible = p->v_ok ? 1 : 0;
    info->streamed_waves = JT_V_WAVES;
    info->streamed_split_efficiency = p->v_ok ? p->vprog.split_efficiency : 0.0;
    info->tiled_eligible = p->t_ok ? 1 : 0;
    info->tiled_passes = (int32_t)p->tprog.passes.size();
    info->tiled_entry_visits = p->tprog.entry_visits;
    info->tiled_lds_bytes = p->tprog.lds_bytes;
    info->tiled_table_bytes = (int64_t)p->tprog.tab.size() * 4;
    return FBN_OK;
}

int fbn_jt_stream_schedule(const fbn_jt_plan *p, int32_t *order, int64_t order_cap, int32_t *sched,
                           int64_t sched_cap, int64_t *n_order, int64_t *n_sched) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    if (!p->v_ok) return SetError(FBN_ERR_LIMIT, "plan not eligible for the streamed kernel");
    const auto &v = p->vprog;
    if (n_order) *n_order = (int64_t)v.order.size();
    if (n_sched) *n_sched = (int64_t)v.sched.size();
    if (order) {
        if (order_cap < (int64_t)v.order.size()) return SetError(FBN_ERR_ARG, "order buffer too small");
        std::copy(v.order.begin(), v.order.end(), order);
    }
    if (sched) {
        if (sched_cap < (int64_t)v.sched.size()) return SetError(FBN_ERR_ARG, "sched buffer too small");
        std::copy(v.sched.begin(), v.sched.end(), sched);
    }
    return FBN_OK;
}

int fbn_jt_tile_program(const fbn_jt_plan *p, int32_t *passes, int32_t *tab, double *initv, int64_t *geometry) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    if (!p->t_ok) return SetError(FBN_ERR_LIMIT, "plan not eligible for the tiled kernel");
    static_assert(sizeof(JtTPass) == 33 * 4, "JtTPass = 33 int32");
    const auto &t = p->tprog;
    if (passes) memcpy(passes, t.passes.data(), t.passes.size() * sizeof(JtTPass));
    if (tab) memcpy(tab, t.tab.data(), t.tab.size() * 4);
    if (initv) memcpy(initv, t.initv.data(), t.initv.size() * 8);
    if (geometry) {
        const int64_t g[8] = {(int64_t)t.passes.size(), (int64_t)t.tab.size(), (int64_t)t.initv.size(), t.scr_row,
                              t.red_row, t.store_rows, JT_T_C, JT_T_L};
        memcpy(geometry, g, sizeof g);
    }
    return FBN_OK;
}

int fbn_jt_plan_dump(const fbn_jt_plan *p, const char *plan_path, const char *init_path) {
    if (!p || !plan_path || !init_path) return SetError(FBN_ERR_ARG, "null pointer");
    const auto &h = p->host;
    FILE *f = fopen(plan_path, "w");
    if (!f) return SetError(FBN_ERR_IO, "cannot write %s", plan_path);
    fprintf(f, "cliques %zu\n", h.cliques.size());
    for (size_t i = 0; i < h.cliques.size(); ++i) {
        const auto &t = h.cliques[i];
        fprintf(f, "c %zu %zu %lld", i, t.vars.size(), (long long)t.size());
        for (int v : t.vars) fprintf(f, " %d", v);
        fprintf(f, " | up %d | down", h.clique_up[i]);
        for (int d : h.clique_down[i]) fprintf(f, " %d", d);
        fprintf(f, "\n");
    }
    fprintf(f, "seps %zu\n", h.seps.size());
    for (size_t i = 0; i < h.seps.size(); ++i) {
        const auto &t = h.seps[i];
        fprintf(f, "s %zu %zu %lld", i, t.vars.size(), (long long)t.size());
        for (int v : t.vars) fprintf(f, " %d", v);
        fprintf(f, " | up %d | down %d\n", h.sep_up[i], h.sep_down[i]);
    }
    fprintf(f, "root %d\n", h.root);
    fprintf(f, "levels %zu\n", h.levels.size());
    for (size_t l = 0; l < h.levels.size(); ++l) {
        fprintf(f, "level %zu %c", l, (l % 2) ? 's' : 'c');
        for (int x : h.levels[l]) fprintf(f, " %d", x);
        fprintf(f, "\n");
    }
    fclose(f);
    f = fopen(init_path, "w");
    if (!f) return SetError(FBN_ERR_IO, "cannot write %s", init_path);
    for (size_t i = 0; i < h.cliques.size(); ++i) {
        fprintf(f, "c %zu %lld", i, (long long)h.cliques[i].size());
        for (double v : h.cliques[i].pot) fprintf(f, " %.17g", v);
        fprintf(f, "\n");
    }
    fclose(f);
    return FBN_OK;
}

constexpr int kJtVFast = 1 << 12;  // jt_virt.hip kVFast
// auto (-1) = the fast arithmetic order for every kernel that has one; exact (1) on request
static bool JtFast(const fbn_jt_plan *p) { return p->exact != 1; }

int fbn_jt_set_waves_per_cu(fbn_jt_plan *p, int waves) {
    if (!p || waves < 0 || waves > 32) return SetError(FBN_ERR_ARG, "waves per CU must be 0..32");
    p->waves_per_cu = waves;
    return FBN_OK;
}

int fbn_jt_set_variant(fbn_jt_plan *p, int variant) {
    if (!p || variant < -1 || variant > 5)
        return SetError(FBN_ERR_ARG, "variant must be -1 (auto), 0 (LDS), 1 (global), 2 (LDS, IEEE division), "
                                     "3 (specialized), 4 (streamed) or 5 (tiled)");
    if (variant == 3 && !p->gen_eligible) return SetError(FBN_ERR_ARG, "plan not eligible for the specialized kernel");
    if (variant == 4 && !p->v_ok) return SetError(FBN_ERR_ARG, "plan not eligible for the streamed kernel");
    if (variant == 5 && !p->t_ok) return SetError(FBN_ERR_ARG, "plan not eligible for the tiled kernel");
    p->variant = variant;
    return FBN_OK;
}

// the plan-specialized kernel of the current arithmetic order, loaded (cache) or compiled (hiprtc)
// once per plan and order; both orders stay loaded
static fbn_jt_plan::GenKernel &GenCur(fbn_jt_plan *p, bool vm) { return p->gen[(JtFast(p) ? 1 : 0) + (vm ? 2 : 0)]; }
static int GenEnsure(fbn_jt_plan *p, bool vm) {
    const bool fast = JtFast(p);
    auto &k = GenCur(p, vm);
    if (k.state == 1) return FBN_OK;
    if (k.state == -1) return FBN_ERR_HIP;
    k.state = -1;
    std::string src;
    std::vector<double> iv;
    int rc = fbn::GenerateJTKernel(p->host, src, &k.we, iv, &k.lds, fast, vm);
    if (rc) return rc;
    std::vector<char> code;
    if ((rc = fbn::JitCodeObject(src, code))) return rc;
    FBN_HIP(hipModuleLoadData(&k.mod, code.data()));
    FBN_HIP(hipModuleGetFunction(&k.fn, k.mod, "fbn_jt_gen"));
    if ((rc = k.iv.ensure(std::max<size_t>(iv.size() * 8, 8)))) return rc;
    FBN_HIP(hipMemcpy(k.iv.p, iv.data(), iv.size() * 8, hipMemcpyHostToDevice));  // (a new buffer: no run uses it yet)
    k.state = 1;
    return FBN_OK;
}

// diagnostic: per-op-type cycle totals of the LDS variant (s_memtime, summed over waves)
int fbn_jt_debug_op_cycles(fbn_jt_plan *p, int enable, unsigned long long *cycles /* [10] or NULL */) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    if (cycles && p->prof_on && p->last_grid > 0) {
        std::vector<unsigned long long> h((size_t)p->last_grid * 16);
        FBN_HIP(hipDeviceSynchronize());
        FBN_HIP(hipMemcpy(h.data(), p->prof.p, h.size() * 8, hipMemcpyDeviceToHost));
        for (int k = 0; k < 10; ++k) {
            cycles[k] = 0;
            for (int w = 0; w < p->last_grid; ++w) cycles[k] += h[(size_t)w * 16 + k];
        }
    }
    p->prof_on = enable != 0;
    return FBN_OK;
}

int fbn_jt_kernel_source(const fbn_jt_plan *p, char *buf, int64_t cap, int64_t *len) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    if (!p->gen_eligible) return SetError(FBN_ERR_ARG, "plan not eligible for codegen");
    std::string src;
    std::vector<double> iv;
    int64_t we = 0;
    int rc = fbn::GenerateJTKernel(p->host, src, &we, iv, nullptr, JtFast(p), p->out_layout == 1);
    if (rc) return rc;
    if (len) *len = (int64_t)src.size() + 1;
    if (buf && cap > 0) {
        const size_t n = std::min<size_t>((size_t)cap - 1, src.size());
        memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return FBN_OK;
}

int fbn_jt_kernel_cache_path(const fbn_jt_plan *p, char *buf, int64_t cap) {
    if (!p || !buf || cap <= 0) return SetError(FBN_ERR_ARG, "bad argument");
    if (!p->gen_eligible) return SetError(FBN_ERR_ARG, "plan not eligible for codegen");
    std::string src;
    std::vector<double> iv;
    int64_t we = 0;
    int rc = fbn::GenerateJTKernel(p->host, src, &we, iv, nullptr, JtFast(p), p->out_layout == 1);
    if (rc) return rc;
    snprintf(buf, (size_t)cap, "%s", fbn::JitCachePath(src).c_str());
    return FBN_OK;
}

int fbn_jt_set_exact(fbn_jt_plan *p, int exact) {
    if (!p || exact < -1 || exact > 1) return SetError(FBN_ERR_ARG, "exact must be -1 (auto), 0 (fast) or 1 (exact)");
    p->exact = exact;
    return FBN_OK;
}

int fbn_jt_debug_force_fixup(fbn_jt_plan *p, int enable) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    p->force_fixup = enable != 0;
    return FBN_OK;
}

int fbn_jt_debug_flagged_blocks(fbn_jt_plan *p, int64_t *count) {
    if (!p || !count) return SetError(FBN_ERR_ARG, "null pointer");
    *count = 0;
    if (p->last_nblk <= 0 || !p->flags.p) return FBN_OK;
    std::vector<int> h((size_t)p->last_nblk);
    FBN_HIP(hipDeviceSynchronize());
    FBN_HIP(hipMemcpy(h.data(), p->flags.p, h.size() * 4, hipMemcpyDeviceToHost));
    for (int f : h) *count += f != 0;
    return FBN_OK;
}

int fbn_jt_kernel_build(const fbn_jt_plan *p) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    if (!p->gen_eligible) return SetError(FBN_ERR_ARG, "plan not eligible for codegen");
    std::string src;
    std::vector<double> iv;
    int64_t we = 0;
    int rc = fbn::GenerateJTKernel(p->host, src, &we, iv, nullptr, JtFast(p), p->out_layout == 1);
    if (rc) return rc;
    std::vector<char> code;
    return fbn::JitCodeObject(src, code);
}

int fbn_jt_kernel_options(char *buf, int64_t cap) {
    if (!buf || cap <= 0) return SetError(FBN_ERR_ARG, "bad argument");
    std::string o;
    for (int i = 0; i < fbn::kJitNumOptions; ++i) o += std::string(fbn::kJitOptions[i]) + "\n";
    snprintf(buf, (size_t)cap, "%s", o.c_str());
    return FBN_OK;
}

static const size_t kLdsBytes = 160 * 1024;

// LDS variant geometry: waves per CU and the number of LDS table rows (64 lanes x 8 B each)
static void LdsGeometry(const fbn_jt_plan *p, int *waves, int *cap) {
    const int64_t row = 64 * 8, tmax = std::max<int64_t>(1, p->lprog.max_table);
    int w = p->waves_per_cu;
    if (w <= 0) w = (int)std::max<int64_t>(1, std::min<int64_t>(8, (int64_t)kLdsBytes / (tmax * row)));
    int64_t c = std::min<int64_t>(tmax, (int64_t)(kLdsBytes / w) / row);
    *waves = w;
    *cap = (int)std::max<int64_t>(1, c);
}

// LDS interpreter launch (variants 0/2, and the exact fixup of variant 3 when flags != NULL)
static int LaunchLds(fbn_jt_plan *p, DevBuf &ws, const int8_t *d_evidence, int64_t ncases, int32_t *labels,
                     double *marg, const int *flags, bool force_exact, hipStream_t s, bool vm = false) {
    const auto &l = p->lprog;
    const int V = p->host.num_nodes, SD = l.sum_dom, nc = l.num_cliques;
    const int64_t nblk = (ncases + 63) / 64;
    int wpc, cap, rc;
    LdsGeometry(p, &wpc, &cap);
    const bool spill = cap < l.max_table;
    // fixup mode: flagged blocks are rare; one wave per CU scans the flags 64 at a time (the launch
    // follows every specialized / tiled launch: ~3 us per call on ALARM, grids of 4 / 16 / 256 waves
    // measured alike; FBN_JT_FIX_GRID: tuning)
    static const int fix_grid = getenv("FBN_JT_FIX_GRID") ? std::max(1, atoi(getenv("FBN_JT_FIX_GRID"))) : 0;
    int grid = (int)std::min<int64_t>(nblk, flags ? (int64_t)(fix_grid > 0 ? fix_grid : p->num_cu) : (int64_t)p->num_cu * wpc);
    const int64_t store_off = 0, den_off = l.store_entries, sep_off = den_off + nc, spill_off = sep_off + l.sep_entries;
    const int64_t wave_entries = spill_off + (spill ? l.max_table - cap : 0);
    if (flags)  // fixup mode: at most ~2 GiB of workspace (large trees need ~100 MB per wave)
        grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, ((int64_t)2 << 30) / (wave_entries * 64 * 8 + nc * 64 * 4)));
    const size_t ws_d = (size_t)grid * wave_entries * 64 * 8;
    const size_t ws_i = (size_t)grid * nc * 64 * 4;
    if ((rc = ws.ensure(ws_d + ws_i))) return rc;
    const bool prof = p->prof_on && !flags;
    if (prof) {
        if ((rc = p->prof.ensure((size_t)grid * 16 * 8))) return rc;
        FBN_HIP(hipMemsetAsync(p->prof.p, 0, (size_t)grid * 16 * 8, s));
        p->last_grid = grid;
    }
    hipError_t e = fbn_jt_lds_launch(p->lops.as<JtOp>(), (int)l.ops.size(), p->laux.as<int32_t>(),
                                     p->linitv.as<double>(), p->ldig.as<uint64_t>(), d_evidence, V, ncases, SD, marg,
                                     labels, ws.as<double>(), reinterpret_cast<int32_t *>(ws.as<char>() + ws_d),
                                     wave_entries, store_off, den_off, sep_off, spill_off, nc, cap, spill, force_exact,
                                     flags, grid, prof ? p->prof.as<unsigned long long>() : nullptr, vm ? 1 : 0, s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt kernel launch: %s", hipGetErrorString(e));
    return FBN_OK;
}

// out-of-domain evidence has no reference meaning (a code >= the node's state count would shift
// bits into the neighbouring digit fields of the kernels' evidence masks): checked on the device
// before any kernel indexes with it; one stream sync (the host loop cost ~1 ns per value)
static int JtCheckEvidence(fbn_jt_plan *p, const int8_t *d_ev, int64_t ncases, hipStream_t s) {
    const int V = p->host.num_nodes;
    int rc;
    if (!p->ddom.p) {
        if ((rc = p->ddom.ensure((size_t)V * 4))) return rc;
        if ((rc = p->evcheck.ensure(8))) return rc;
        FBN_HIP(hipMemcpy(p->ddom.p, p->host.dom.data(), (size_t)V * 4, hipMemcpyHostToDevice));
    }
    FBN_HIP(hipMemsetAsync(p->evcheck.p, 0xFF, 8, s));
    hipError_t e = fbn_jt_evidence_check(d_ev, (long long)ncases * V, V, p->ddom.as<int32_t>(),
                                         p->evcheck.as<unsigned long long>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "evidence check: %s", hipGetErrorString(e));
    unsigned long long first = 0;
    FBN_HIP(hipMemcpyAsync(&first, p->evcheck.p, 8, hipMemcpyDeviceToHost, s));
    FBN_HIP(hipStreamSynchronize(s));
    if (first == ~0ull) return FBN_OK;
    int8_t code = 0;
    FBN_HIP(hipMemcpy(&code, d_ev + first, 1, hipMemcpyDeviceToHost));
    const long long c = (long long)(first / V);
    const int v = (int)(first % V);
    return SetError(FBN_ERR_ARG, "case %lld: evidence %d for node %d (domain %d)", c, (int)code, v, p->host.dom[v]);
}

int fbn_jt_evidence_validate(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, void *hip_stream) {
    if (!p || (!d_evidence && ncases > 0) || ncases < 0) return SetError(FBN_ERR_ARG, "bad argument");
    if (ncases == 0) return FBN_OK;
    if (p->device < 0) return SetError(FBN_ERR_NODEV, "host-only plan (created with device < 0)");
    FBN_HIP(hipSetDevice(p->device));
    p->note_stream(static_cast<hipStream_t>(hip_stream));
    return JtCheckEvidence(p, d_evidence, ncases, static_cast<hipStream_t>(hip_stream));
}

int fbn_jt_set_kernel_timing(fbn_jt_plan *p, int enable) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    p->ktiming = enable != 0;
    return FBN_OK;
}

int fbn_jt_set_evidence_check(fbn_jt_plan *p, int enable) {
    if (!p) return SetError(FBN_ERR_ARG, "null pointer");
    p->ev_check = enable != 0;
    return FBN_OK;
}

static int JtRunDevice(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, int32_t *d_labels,
                       double *d_marginals, hipStream_t s, bool check, bool vm);

int fbn_jt_run_device(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, int32_t *d_labels,
                      double *d_marginals, void *hip_stream) {
    if (!p || (!d_evidence && ncases > 0) || ncases < 0) return SetError(FBN_ERR_ARG, "bad argument");
    if (ncases == 0) return FBN_OK;
    if (p->device < 0) return SetError(FBN_ERR_NODEV, "host-only plan (created with device < 0)");
    FBN_HIP(hipSetDevice(p->device));
    p->note_stream(static_cast<hipStream_t>(hip_stream));
    return JtRunDevice(p, d_evidence, ncases, d_labels, d_marginals, static_cast<hipStream_t>(hip_stream),
                       p->ev_check, p->out_layout == 1 && d_marginals);
}

static int JtRunDevice(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, int32_t *d_labels,
                       double *d_marginals, hipStream_t s, bool check, bool vm) {
    if (check)
        if (int rc = JtCheckEvidence(p, d_evidence, ncases, s)) return rc;
    const auto &g = p->prog;
    const int V = p->host.num_nodes, SD = g.sum_dom, nc = g.num_cliques;
    const int64_t nblk = (ncases + 63) / 64;
    int rc;
    double *marg = d_marginals;
    if (!marg) {
        if ((rc = p->marg.ensure((size_t)ncases * SD * 8))) return rc;
        marg = p->marg.as<double>();
    }
    int32_t *labels = d_labels;
    if (!labels) {
        if ((rc = p->labels.ensure((size_t)ncases * 4))) return rc;
        labels = p->labels.as<int32_t>();
    }
    int variant = p->variant;
    // the specialized kernel stores variable-major columns with 32-bit byte offsets
    const bool vm3 = vm && (int64_t)ncases * SD * 8 < INT32_MAX;
    if (variant == -1) {
        // specialized kernel when eligible; else the streamed kernel (1.5-2x the interpreters on
        // ALARM and the Munin-like network); the interpreters only for plans it cannot take
        if (p->gen_eligible && GenEnsure(p, vm3) == FBN_OK) variant = 3;
        else if (p->t_ok && JtFast(p)) variant = 5;  // (fast arithmetic order only)
        else if (p->v_ok) variant = 4;
        else variant = (p->lprog.max_table * 64 * 8 * 2 <= (int64_t)kLdsBytes) ? 0 : 1;
    }
    else if (variant == 3 && (rc = GenEnsure(p, vm3))) return rc;
    p->last_variant = variant;
    // variable-major output: kernels 0-3 store it directly; 4 and 5 write case-major scratch that is
    // transposed into the caller's buffer at the end (same values)
    double *const marg_out = marg;
    // (the specialized kernel addresses columns with 32-bit byte offsets: larger batches transpose too)
    const bool vm_scratch = vm && (variant == 4 || variant == 5 || (variant == 3 && !vm3));
    if (vm_scratch) {
        if ((rc = p->mtmp.ensure((size_t)ncases * SD * 8))) return rc;
        marg = p->mtmp.as<double>();
    }
    const bool vm_direct = vm && !vm_scratch;
    p->last_nblk = variant >= 3 ? nblk : 0;

    if (variant == 1) {
        const int wpc = p->waves_per_cu > 0 ? p->waves_per_cu : 8;
        int grid = (int)std::min<int64_t>(nblk, (int64_t)p->num_cu * wpc);
        // persistent waves: cap the per-wave workspaces at 80 % of the free HBM (more resident waves
        // = more memory-level parallelism: this variant is latency bound on large plans)
        const size_t per_wave = (size_t)g.state_entries * 64 * 8 + (size_t)nc * 64 * 4;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && per_wave > 0) {
            const size_t have = free_b / 10 * 8 + (p->ws.bytes);
            grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (int64_t)(have / per_wave)));
        }
        const size_t ws_d = (size_t)grid * g.state_entries * 64 * 8;
        const size_t ws_i = (size_t)grid * nc * 64 * 4;
        if ((rc = p->ws.ensure(ws_d + ws_i))) return rc;
        if (p->ktiming) FBN_HIP(hipEventRecord(p->ev0, s));
        hipError_t e = fbn_jt_launch(p->ops.as<JtOp>(), (int)g.ops.size(), p->aux.as<int32_t>(), p->initv.as<double>(),
                                     p->dig.as<uint64_t>(), d_evidence, V, ncases, SD, marg, labels,
                                     p->ws.as<double>(), reinterpret_cast<int32_t *>(p->ws.as<char>() + ws_d),
                                     g.state_entries, nc, grid, vm_direct ? 1 : 0, s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt kernel launch: %s", hipGetErrorString(e));
    } else if (variant == 4) {
        // streamed tables: small register footprint, many resident waves; the per-wave store holds
        // only separator messages and denominators
        // workgroups of JT_V_WAVES waves, one 64-case block per workgroup (persistent)
        const int W = JT_V_WAVES;
        const int wpc = p->waves_per_cu > 0 ? p->waves_per_cu : 16;
        int grid = (int)std::min<int64_t>(nblk, std::max<int64_t>(1, (int64_t)p->num_cu * wpc / W));
        const auto &v = p->vprog;
        const size_t per_blk_d = (size_t)v.store_rows * 64 * 8, per_blk_i = (size_t)(nc + V) * 64 * 4;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const size_t have = free_b / 10 * 8 + p->ws.bytes;
            grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (int64_t)(have / (per_blk_d + per_blk_i))));
        }
        const size_t ws_d = (size_t)grid * per_blk_d;
        if ((rc = p->ws.ensure(ws_d + (size_t)grid * per_blk_i))) return rc;
        if ((rc = p->flags.ensure((size_t)nblk * 4))) return rc;
        if (p->ktiming) FBN_HIP(hipEventRecord(p->ev0, s));
        hipError_t e = fbn_jt_virt_launch(p->vcl.as<JtVClique>(), p->vaux.as<int32_t>(), p->viv.as<double>(),
                                          p->vdig.as<uint64_t>(), p->vorder.as<int32_t>(), p->vsched.as<int32_t>(),
                                          p->vsel.as<int32_t>(), d_evidence, marg, labels, p->ws.as<double>(),
                                          reinterpret_cast<int32_t *>(p->ws.as<char>() + ws_d), p->flags.as<int>(),
                                          ncases, v.store_rows, v.scratch_row, v.scratch_rows, nc, V, SD, grid,
                                          // diagnostic ablation only (tools/): skip pass types, wrong results
                                          (getenv("FBN_JT_VDEBUG") ? atoi(getenv("FBN_JT_VDEBUG")) : 0) |
                                              (JtFast(p) ? kJtVFast : 0),
                                          s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt kernel launch: %s", hipGetErrorString(e));
        if (p->force_fixup) FBN_HIP(hipMemsetAsync(p->flags.p, 1, (size_t)nblk * 4, s));  // testing only
        // exact recomputation of the blocks whose denominators left the fast-division range
        if (!getenv("FBN_JT_VDEBUG") &&
            (rc = LaunchLds(p, p->ws_fix, d_evidence, ncases, labels, marg, p->flags.as<int>(), false, s)))
            return rc;
    } else if (variant == 5) {
        const auto &t = p->tprog;
        // workgroups of JT_T_W waves, one case group (JT_T_C cases) each, persistent; per workgroup
        // its message store
        const int64_t ncg = (ncases + JT_T_C - 1) / JT_T_C;
        const int wpc = p->waves_per_cu > 0 ? p->waves_per_cu : 16;
        int grid = (int)std::min<int64_t>(ncg, std::max<int64_t>(1, (int64_t)p->num_cu * wpc / t.waves));
        const size_t per_wg = (size_t)t.store_rows * JT_T_C * 8;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const size_t have = free_b / 10 * 8 + p->ws.bytes;
            grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (int64_t)(have / per_wg)));
        }
        if ((rc = p->ws.ensure((size_t)grid * per_wg))) return rc;
        if ((rc = p->flags.ensure((size_t)nblk * 4))) return rc;
        FBN_HIP(hipMemsetAsync(p->flags.p, 0, (size_t)nblk * 4, s));
        unsigned long long *tprof = nullptr;  // diagnostic: per-phase cycles (fbn_jt_debug_op_cycles)
        if (p->prof_on) {
            if ((rc = p->prof.ensure(16 * 8))) return rc;
            FBN_HIP(hipMemsetAsync(p->prof.p, 0, 16 * 8, s));
            p->last_grid = 1;
            tprof = p->prof.as<unsigned long long>();
        }
        if (p->ktiming) FBN_HIP(hipEventRecord(p->ev0, s));
        hipError_t e = fbn_jt_tile_launch(p->tpass.as<JtTPass>(), (int)t.passes.size(), p->ttab.as<int32_t>(),
                                          p->tiv.as<double>(), d_evidence, marg, labels, p->ws.as<double>(),
                                          p->flags.as<int>(), ncases, t.store_rows, t.scr_row, t.red_row, V, SD,
                                          (int)t.lds_bytes, grid, t.waves, tprof, s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt kernel launch: %s", hipGetErrorString(e));
        if (p->force_fixup) FBN_HIP(hipMemsetAsync(p->flags.p, 1, (size_t)nblk * 4, s));  // testing only
        // exact recomputation of the blocks holding a case group whose pass totals left the checked range
        // (FBN_JT_NO_FIXUP: diagnostic only -- flagged blocks keep the tiled kernel's values)
        static const bool no_fix = getenv("FBN_JT_NO_FIXUP") != nullptr;
        if (!no_fix && (rc = LaunchLds(p, p->ws_fix, d_evidence, ncases, labels, marg, p->flags.as<int>(), false, s)))
            return rc;
    } else if (variant == 3) {
        // one wave (64 cases) per SIMD: the clique in flight occupies the register file (+ LDS tail)
        const auto &gk = GenCur(p, vm3);
        int wpc = p->waves_per_cu > 0 ? p->waves_per_cu : 4;
        if (gk.lds > 0) wpc = std::max<int>(1, std::min<int64_t>(wpc, (int64_t)kLdsBytes / gk.lds));
        const int grid = (int)std::min<int64_t>(nblk, (int64_t)p->num_cu * wpc);
        if ((rc = p->ws.ensure((size_t)grid * gk.we * 64 * 8))) return rc;
        if ((rc = p->flags.ensure((size_t)nblk * 4))) return rc;
        if (p->ktiming) FBN_HIP(hipEventRecord(p->ev0, s));

        const int8_t *a_ev = d_evidence;
        double *a_marg = marg, *a_ws = p->ws.as<double>();
        int32_t *a_lab = labels;
        int *a_flags = p->flags.as<int>();
        const double *a_iv = gk.iv.as<double>();
        long long a_n = ncases;
        unsigned long long *a_prof = nullptr;
        if (p->prof_on) {  // diagnostic: only kernels generated with FBN_JT_PROFILE=1 write it
            if ((rc = p->prof.ensure((size_t)grid * 16 * 8))) return rc;
            FBN_HIP(hipMemsetAsync(p->prof.p, 0, (size_t)grid * 16 * 8, s));
            p->last_grid = grid;
            a_prof = p->prof.as<unsigned long long>();
        }
        void *args[] = {&a_ev, &a_marg, &a_lab, &a_ws, &a_flags, &a_iv, &a_n, &a_prof};
        FBN_HIP(hipModuleLaunchKernel(gk.fn, grid, 1, 1, 64, 1, 1, (unsigned)gk.lds, s, args, nullptr));
        if (p->force_fixup) FBN_HIP(hipMemsetAsync(p->flags.p, 1, (size_t)nblk * 4, s));  // testing only
        // exact recomputation of the blocks whose denominators left the fast-division range
        // (FBN_JT_NO_FIXUP: diagnostic only, as above)
        static const bool no_fix3 = getenv("FBN_JT_NO_FIXUP") != nullptr;
        if (!no_fix3 && (rc = LaunchLds(p, p->ws_fix, d_evidence, ncases, labels, marg, p->flags.as<int>(), false, s, vm_direct)))
            return rc;
    } else {
        if (p->ktiming) FBN_HIP(hipEventRecord(p->ev0, s));
        if ((rc = LaunchLds(p, p->ws, d_evidence, ncases, labels, marg, nullptr, variant == 2, s, vm_direct))) return rc;
    }
    if (vm_scratch) {
        hipError_t e = fbn_jt_marg_transpose(marg, marg_out, ncases, SD, s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt marginal transpose: %s", hipGetErrorString(e));
    }
    if (p->ktiming) FBN_HIP(hipEventRecord(p->ev1, s));
    p->timed = p->ktiming;
    return FBN_OK;
}

int fbn_jt_run(fbn_jt_plan *p, const int8_t *evidence, int64_t ncases, int32_t *labels_out, double *marginals_out,
               void *hip_stream) {
    if (!p || (!evidence && ncases > 0) || ncases < 0 || (!labels_out && ncases > 0))
        return SetError(FBN_ERR_ARG, "bad argument");
    if (ncases == 0) return FBN_OK;
    if (p->device < 0) return SetError(FBN_ERR_NODEV, "host-only plan (created with device < 0)");
    const int V = p->host.num_nodes, SD = p->prog.sum_dom;
    FBN_HIP(hipSetDevice(p->device));
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    int rc;
    if ((rc = p->evid.ensure((size_t)ncases * V))) return rc;
    if ((rc = p->labels.ensure((size_t)ncases * 4))) return rc;
    if ((rc = p->marg.ensure((size_t)ncases * SD * 8))) return rc;
    FBN_HIP(hipMemcpyAsync(p->evid.p, evidence, (size_t)ncases * V, hipMemcpyHostToDevice, s));
    rc = JtRunDevice(p, p->evid.as<int8_t>(), ncases, p->labels.as<int32_t>(), p->marg.as<double>(), s, true, false);
    if (rc) return rc;
    FBN_HIP(hipMemcpyAsync(labels_out, p->labels.p, (size_t)ncases * 4, hipMemcpyDeviceToHost, s));
    if (marginals_out)
        FBN_HIP(hipMemcpyAsync(marginals_out, p->marg.p, (size_t)ncases * SD * 8, hipMemcpyDeviceToHost, s));
    FBN_HIP(hipStreamSynchronize(s));
    return FBN_OK;
}

int fbn_jt_score(const fbn_jt_plan *p, const double *marginals, const double *golden, int64_t ncases, double *mse_sum,
                 double *hd_sum) {
    if (!p || !marginals || !golden || !mse_sum || !hd_sum) return SetError(FBN_ERR_ARG, "null pointer");
    const auto &dom = p->host.dom;
    const int SD = p->prog.sum_dom;
    auto round7 = [](double number) {  // Round(x, 7), src/Inference.cpp:195-206
        long long integerpart = (long long)number;
        number -= integerpart;
        for (int i = 0; i < 7; ++i) number *= 10;
        number = (double)(long long)(number + 0.5);
        for (int i = 0; i < 7; ++i) number /= 10;
        return integerpart + number;
    };
    double mse = 0.0, hd = 0.0;
    for (int64_t c = 0; c < ncases; ++c) {  // CalculateMSE / CalculateHellingerDistance (:153-193)
        const double *a = marginals + c * SD, *x = golden + c * SD;
        int num = 0, off = 0;
        double e1 = 0.0, e2 = 0.0;
        for (size_t v = 0; v < dom.size(); ++v) {
            if (x[off] > 0) {
                num += dom[v];
                for (int j = 0; j < dom[v]; ++j) {
                    double r = round7(a[off + j]);
                    e1 += pow(r - x[off + j], 2);
                    e2 += pow(sqrt(r) - sqrt(x[off + j]), 2);
                }
            }
            off += dom[v];
        }
        mse += sqrt(e1 / num);
        hd += sqrt(e2 / num);
    }
    *mse_sum = mse;
    *hd_sum = hd;
    return FBN_OK;
}

int fbn_jt_set_output_layout(fbn_jt_plan *p, int layout) {
    if (!p || layout < 0 || layout > 1)
        return SetError(FBN_ERR_ARG, "layout must be 0 (case-major) or 1 (variable-major)");
    p->out_layout = layout;
    return FBN_OK;
}

int fbn_jt_score_terms_device(fbn_jt_plan *p, const double *d_marginals, const double *d_golden, int64_t ncases,
                              double *d_terms, void *hip_stream) {
    if (!p || ncases < 0 || (ncases > 0 && (!d_marginals || !d_golden || !d_terms)))
        return SetError(FBN_ERR_ARG, "bad argument");
    if (ncases == 0) return FBN_OK;
    if (p->device < 0) return SetError(FBN_ERR_NODEV, "host-only plan (created with device < 0)");
    FBN_HIP(hipSetDevice(p->device));
    const int V = p->host.num_nodes;
    int rc;
    if (!p->ddom.p) {
        if ((rc = p->ddom.ensure((size_t)V * 4))) return rc;
        if ((rc = p->evcheck.ensure(8))) return rc;
        FBN_HIP(hipMemcpy(p->ddom.p, p->host.dom.data(), (size_t)V * 4, hipMemcpyHostToDevice));
    }
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    p->note_stream(s);
    hipError_t e = fbn_jt_score_terms(d_marginals, d_golden, ncases, p->prog.sum_dom, p->out_layout == 1 ? 1 : 0,
                                      p->ddom.as<int32_t>(), V, d_terms, s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "jt score terms: %s", hipGetErrorString(e));
    return FBN_OK;
}

int fbn_jt_last_kernel_ms(const fbn_jt_plan *p, float *ms) {
    if (!p || !ms || !p->timed) return SetError(FBN_ERR_ARG, "no timed launch");
    FBN_HIP(hipEventSynchronize(p->ev1));
    FBN_HIP(hipEventElapsedTime(ms, p->ev0, p->ev1));
    return FBN_OK;
}

int fbn_jt_plan_destroy(fbn_jt_plan *p) {
    if (!p) return FBN_OK;
    if (p->device >= 0) {  // runs are queued on caller streams: drain those before the buffers go
        (void)hipSetDevice(p->device);
        for (hipStream_t s : p->streams_used) (void)hipStreamSynchronize(s);
    }
    delete p;
    return FBN_OK;
}

// ------------------------------------------------------------------ CI tests
// the column store from host memory (cols_on_device = false) or from a device buffer of the same
// device, e.g. one filled by an RCCL broadcast (true); every code is checked < dims[v] on the
// device before any kernel bins with it
static int CiCreate(const uint8_t *cols, bool cols_on_device, int nvars, int64_t nsamples, const int32_t *dims,
                    int device, fbn_ci_ctx **out) {
    if (!cols || !dims || !out || nvars <= 0 || nsamples <= 0) return SetError(FBN_ERR_ARG, "bad argument");
    for (int v = 0; v < nvars; ++v)
        if (dims[v] < 1 || dims[v] > 256) return SetError(FBN_ERR_ARG, "dims[%d] = %d out of 1..256", v, dims[v]);
    auto c = std::unique_ptr<fbn_ci_ctx>(new (std::nothrow) fbn_ci_ctx());
    if (!c) return SetError(FBN_ERR_NOMEM, "out of memory");
    int rc = CheckDevice(device, &c->num_cu);
    if (rc) return rc;
    FBN_HIP(hipSetDevice(device));
    c->device = device;
    c->nvars = nvars;
    c->N = nsamples;
    c->dims.assign(dims, dims + nvars);
    if ((rc = c->cols.ensure((size_t)nvars * nsamples))) return rc;
    if ((rc = c->ddims.ensure((size_t)nvars * 4))) return rc;
    if ((rc = c->stats.ensure(16))) return rc;
    FBN_HIP(hipMemcpy(c->cols.p, cols, (size_t)nvars * nsamples,
                      cols_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
    FBN_HIP(hipMemcpy(c->ddims.p, dims, (size_t)nvars * 4, hipMemcpyHostToDevice));
    {
        FBN_HIP(hipMemset(c->stats.p, 0, 16));
        hipError_t e = fbn_ci_cols_check(c->cols.as<uint8_t>(), c->ddims.as<int32_t>(), nvars, nsamples,
                                         c->stats.as<int>(), nullptr);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "column check: %s", hipGetErrorString(e));
        int bad[2] = {0, 0};
        FBN_HIP(hipMemcpy(bad, c->stats.p, 8, hipMemcpyDeviceToHost));
        if (bad[0])
            return SetError(FBN_ERR_ARG, "column store: variable %d holds a code >= its state count %d", bad[1] - 1,
                            dims[bad[1] - 1]);
    }
    for (auto &sl : c->slot) {
        FBN_HIP(hipEventCreate(&sl.ev0));
        FBN_HIP(hipEventCreate(&sl.ev1));
        FBN_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
    FBN_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if ((rc = CiResetMargin(c.get()))) return rc;
    *out = c.release();
    return FBN_OK;
}
int fbn_ci_set_kernel_timing(fbn_ci_ctx *c, int enable) {
    if (!c) return SetError(FBN_ERR_ARG, "null pointer");
    c->timing = enable != 0;
    return FBN_OK;
}
int fbn_ci_dataset_upload(const uint8_t *cols, int nvars, int64_t nsamples, const int32_t *dims, int device,
                          fbn_ci_ctx **out) {
    return CiCreate(cols, false, nvars, nsamples, dims, device, out);
}
int fbn_ci_dataset_from_device(const uint8_t *d_cols, int nvars, int64_t nsamples, const int32_t *dims, int device,
                               fbn_ci_ctx **out) {
    return CiCreate(d_cols, true, nvars, nsamples, dims, device, out);
}

// Tasks of the register-blocked level-0 kernel for the pairs [t0, t1) of the complete graph (pair
// index = lexicographic (u < v) order): x-side variables = the range's rows u, y-side = all variables,
// both cut into sorted blocks per state-count class (fbn_ci_pair_block); a task is kept if it holds
// a pair (x < y) of the range, so every pair of the range is in exactly one task (x-side = its u).
// Cached per range (a PC run's level 0 repeats it).
static int CiPairTasks(fbn_ci_ctx *c, int64_t t0, int64_t t1, hipStream_t s) {
    if (c->ptask_t0 == t0 && c->ptask_t1 == t1) return FBN_OK;
    const int nv = c->nvars;
    const int64_t P = (int64_t)nv * (nv - 1) / 2;
    auto row_of = [&](int64_t t) {  // u of pair t
        int64_t lo = 0, hi = nv - 2;
        while (lo < hi) {
            const int64_t m = (lo + hi + 1) / 2;
            if (m * nv - m * (m + 1) / 2 <= t) lo = m;
            else hi = m - 1;
        }
        return (int)lo;
    };
    auto idx = [&](int64_t u, int64_t v) { return u * nv - u * (u + 1) / 2 + (v - u - 1); };
    const int u0 = t1 > t0 ? row_of(t0) : 0, u1 = t1 > t0 ? row_of(t1 - 1) : -1;
    const bool full = t0 == 0 && t1 == P;
    std::vector<int> cls[5], ucls[5];
    for (int v = 0; v < nv; ++v) {
        const int d = c->dims[v];
        if (d < 1 || d > 4) return SetError(FBN_ERR_ARG, "blocked pairs: variable %d has %d states", v, d);
        cls[d].push_back(v);
        if (v >= u0 && v <= u1) ucls[d].push_back(v);
    }
    std::vector<int32_t> tasks;
    for (int dx = 1; dx <= 4; ++dx)
        for (int dy = 1; dy <= 4; ++dy) {
            const int bx = fbn_ci_pair_block(dx), by = fbn_ci_pair_block(dy);
            const std::vector<int> &X = ucls[dx], &Y = cls[dy];
            for (size_t i = 0; i < X.size(); i += bx) {
                const int nxs = (int)std::min<size_t>(bx, X.size() - i);
                for (size_t j = 0; j < Y.size(); j += by) {
                    const int nys = (int)std::min<size_t>(by, Y.size() - j);
                    if (Y[j + nys - 1] <= X[i]) continue;  // no y above any x
                    bool any = full;
                    for (int a = 0; a < nxs && !any; ++a)
                        for (int b = 0; b < nys && !any; ++b) {
                            const int x = X[i + a], y = Y[j + b];
                            if (x < y) {
                                const int64_t t = idx(x, y);
                                any = t >= t0 && t < t1;
                            }
                        }
                    if (!any) continue;
                    const size_t o = tasks.size();
                    tasks.resize(o + 12, -1);
                    tasks[o] = dx, tasks[o + 1] = dy, tasks[o + 2] = nxs, tasks[o + 3] = nys;
                    for (int a = 0; a < nxs; ++a) tasks[o + 4 + a] = X[i + a];
                    for (int b = 0; b < nys; ++b) tasks[o + 8 + b] = Y[j + b];
                }
            }
        }
    int rc;
    if ((rc = c->ptasks.ensure(std::max<size_t>(tasks.size(), 1) * 4))) return rc;
    if (!tasks.empty()) FBN_HIP(hipMemcpyAsync(c->ptasks.p, tasks.data(), tasks.size() * 4, hipMemcpyHostToDevice, s));
    FBN_HIP(hipStreamSynchronize(s));  // the host vector goes out of scope
    c->ptask_t0 = t0, c->ptask_t1 = t1, c->ptask_n = (int64_t)tasks.size() / 12;
    return FBN_OK;
}

// the leading rows of the bit-sliced store (once per ctx, after the bits build)
static int CiLeadEnsure(fbn_ci_ctx *c, hipStream_t s) {
    if (c->lead_ready) return FBN_OK;
    const int nv = c->nvars;
    c->lead0_host.assign(nv, 0);
    c->leadrows_host.clear();
    for (int v = 0; v < nv; ++v) {
        c->lead0_host[v] = (int32_t)c->leadrows_host.size();
        for (int a = 0; a + 1 < c->dims[v]; ++a) c->leadrows_host.push_back(c->row0_host[v] + a);
    }
    int rc;
    if ((rc = c->lead0.ensure((size_t)nv * 4))) return rc;
    if ((rc = c->leadrows.ensure(std::max<size_t>(c->leadrows_host.size(), 1) * 4))) return rc;
    FBN_HIP(hipMemcpyAsync(c->lead0.p, c->lead0_host.data(), (size_t)nv * 4, hipMemcpyHostToDevice, s));
    if (!c->leadrows_host.empty())
        FBN_HIP(hipMemcpyAsync(c->leadrows.p, c->leadrows_host.data(), c->leadrows_host.size() * 4,
                               hipMemcpyHostToDevice, s));
    c->lead_ready = true;
    return FBN_OK;
}

// level 0 through the Gram when its ld x ld int32 matrix fits this budget (else the tiled kernel)
constexpr int64_t kGram0MaxBytes = (int64_t)1 << 30;
static bool CiGram0Eligible(const fbn_ci_ctx *c) {
    int64_t R = 0;
    for (int v = 0; v < c->nvars; ++v) R += c->dims[v] - 1;
    return R > 0 && R * R * 4 <= kGram0MaxBytes && !getenv("FBN_CI_NO_GRAM");
}

// 8 x 8 tiles (i-block <= j-block) of the leading-row Gram holding a pair (x < y) of [t0, t1): row
// i of x's leading rows, column j of y's (x < y puts every needed entry in an upper tile).  Cached
// per range.
static int CiGram0Tasks(fbn_ci_ctx *c, int64_t t0, int64_t t1, hipStream_t s) {
    if (c->g0_t0 == t0 && c->g0_t1 == t1) return FBN_OK;
    const int nv = c->nvars;
    const int64_t R = (int64_t)c->leadrows_host.size(), nb = (R + 7) / 8;
    std::vector<int32_t> var_of(R);
    for (int v = 0; v < nv; ++v)
        for (int a = 0; a + 1 < c->dims[v]; ++a) var_of[c->lead0_host[v] + a] = v;
    auto idx = [&](int64_t u, int64_t v) { return u * nv - u * (u + 1) / 2 + (v - u - 1); };
    const int TI = fbn_ci_gram_task_ints();
    std::vector<int32_t> tasks;
    // tiles in 16 x 16-tile super-blocks (128 + 128 rows = 3.2 MB at 100k samples: one XCD's L2),
    // consecutive in the task list, which the kernel splits XCD-contiguously
    constexpr int64_t SB = 16;
    for (int64_t si = 0; si < nb; si += SB)
    for (int64_t sj = si; sj < nb; sj += SB)
    for (int64_t bi = si; bi < std::min(nb, si + SB); ++bi) {
        const int64_t r0 = 8 * bi, r1 = std::min(R, r0 + 8);
        const int vi0 = var_of[r0], vi1 = var_of[r1 - 1];
        for (int64_t bj = std::max(bi, sj); bj < std::min(nb, sj + SB); ++bj) {
            const int64_t c0 = 8 * bj, c1 = std::min(R, c0 + 8);
            const int vj0 = var_of[c0], vj1 = var_of[c1 - 1];
            if (vi0 >= vj1) continue;  // no x < y in the tile
            const int64_t tmin = idx(vi0, std::max(vj0, vi0 + 1)), tmax = idx(std::min(vi1, vj1 - 1), vj1);
            if (tmax < t0 || tmin >= t1) continue;
            const int64_t off = r0 * R + c0;
            const int32_t t[8] = {-1, (int32_t)r0, (int32_t)(r1 - r0), (int32_t)c0, (int32_t)(c1 - c0),
                                  (int32_t)(uint32_t)(off & 0xffffffff), (int32_t)(off >> 32), (int32_t)R};
            tasks.insert(tasks.end(), t, t + TI);
        }
    }
    int rc;
    if ((rc = c->g0tasks.ensure(std::max<size_t>(tasks.size(), 1) * 4))) return rc;
    if (!tasks.empty()) FBN_HIP(hipMemcpyAsync(c->g0tasks.p, tasks.data(), tasks.size() * 4, hipMemcpyHostToDevice, s));
    FBN_HIP(hipStreamSynchronize(s));  // the host vector goes out of scope
    c->g0_t0 = t0, c->g0_t1 = t1, c->g0_ntasks = (int64_t)tasks.size() / TI;
    return FBN_OK;
}

// x-variable row range [r0, r1) of the leading rows that the pairs [t0, t0 + n) read as rows of G
static void CiPairRowRange(const fbn_ci_ctx *c, int64_t t0, int64_t n, int64_t *r0, int64_t *r1) {
    const int nv = c->nvars;
    auto row_of = [&](int64_t t) {
        int64_t lo = 0, hi = nv - 2;
        while (lo < hi) {
            const int64_t m = (lo + hi + 1) / 2;
            if (m * nv - m * (m + 1) / 2 <= t) lo = m;
            else hi = m - 1;
        }
        return (int)lo;
    };
    const int u0 = row_of(t0), u1 = row_of(t0 + n - 1);
    *r0 = c->lead0_host[u0];
    *r1 = u1 + 1 < nv ? c->lead0_host[u1 + 1] : (int64_t)c->leadrows_host.size();
}

// The level-0 Gram on the matrix cores, hand-written (ci_gram_mfma.hip): FP4 one-hot store built
// once per ctx, the 256 x 256 tiles (I, J >= I) covering rows [r0, r1) x all columns, split-K so the
// launch fills the CUs, uint16 partial slabs summed into gram0 (entries i < j).  *done = false: not
// used (small Gram -- ALARM's 60 rows x 5k samples stay on the popcount kernel --, over the byte
// budget, or FBN_CI_GRAM_NO_MFMA).
constexpr int64_t kOnehot4MaxBytes = (int64_t)4 << 30;
static int CiGram0Mfma(fbn_ci_ctx *c, int64_t t0, int64_t n, hipStream_t s, bool *done) {
    *done = false;
    const int64_t R = (int64_t)c->leadrows_host.size(), T = fbn_ci_gram4_tile(), KT = fbn_ci_gram4_stage();
    const int64_t Rp = (R + T - 1) / T * T, KS = (c->N + KT - 1) / KT, Kb = KS * KT / 2;
    if (getenv("FBN_CI_GRAM_NO_MFMA") || (double)R * R * c->N < 1e10 || Rp * Kb > kOnehot4MaxBytes || KS > INT32_MAX)
        return FBN_OK;
    int rc;
    if (!c->onehot4_ready) {
        if ((rc = c->onehot4.ensure((size_t)(Rp * Kb)))) return rc;
        FBN_HIP(hipMemsetAsync(c->onehot4.p, 0, (size_t)(Rp * Kb), s));  // pad rows R..Rp-1
        hipError_t e = fbn_ci_onehot4_build(c->cols.as<uint8_t>(), c->ddims.as<int32_t>(), c->lead0.as<int32_t>(), c->N,
                                            KS, Rp, c->nvars, c->onehot4.as<uint8_t>(), s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "fp4 one-hot build: %s", hipGetErrorString(e));
        c->onehot4_ready = true;
    }
    int64_t r0, r1;
    CiPairRowRange(c, t0, n, &r0, &r1);
    if (r1 <= r0) {
        *done = true;
        return FBN_OK;
    }
    if (c->g4_r0 != r0 || c->g4_r1 != r1) {
        std::vector<int32_t> tasks;
        const int64_t nb = Rp / T;
        for (int64_t I = r0 / T; I <= (r1 - 1) / T; ++I)
            for (int64_t J = I; J < nb; ++J) tasks.push_back((int32_t)I), tasks.push_back((int32_t)J);
        if ((rc = c->g4tasks.ensure(tasks.size() * 4))) return rc;
        FBN_HIP(hipMemcpyAsync(c->g4tasks.p, tasks.data(), tasks.size() * 4, hipMemcpyHostToDevice, s));
        FBN_HIP(hipStreamSynchronize(s));  // the host vector goes out of scope
        c->g4_nt = (int)(tasks.size() / 2), c->g4_r0 = r0, c->g4_r1 = r1;
    }
    // split-K: about one block per CU; uint16 partials need every slice <= 65535 samples
    const int nt = c->g4_nt;
    int64_t S = std::max<int64_t>(1, EnvOr0("FBN_CI_GRAM4_SPLITS", c->num_cu / nt));
    S = std::max<int64_t>(S, (KS + 510) / 511);  // slices of <= 511 stages x 128 samples
    S = std::min<int64_t>(S, KS);
    if ((rc = c->g4slab.ensure((size_t)(nt * S * T * T * 2)))) return rc;
    hipError_t e = fbn_ci_gram4(c->onehot4.as<uint8_t>(), Rp, c->g4tasks.as<int2>(), nt, (int)S, (int)KS,
                                c->g4slab.as<uint16_t>(), (int)R, R, c->gram0.as<int32_t>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "mfma gram: %s", hipGetErrorString(e));
    *done = true;
    return FBN_OK;
}

// The level-0 Gram as an int8 GEMM on the matrix cores (rocBLAS gemm_ex, int32 accumulation: the
// counts are exact): O = one byte per (leading row, sample), built once per ctx; for the pairs
// [t0, t0 + n) only the columns of their x-variables' leading rows are computed (C[:, r0:r1] = O^T
// O[:, r0:r1], column-major, ld = R).  *done = false: not used (no library, over the byte budget,
// FBN_CI_GRAM_NO_BLAS, or a failed call) -- the popcount Gram kernel runs instead.
constexpr int64_t kOnehotMaxBytes = (int64_t)4 << 30;
static int CiGram0Blas(fbn_ci_ctx *c, int64_t t0, int64_t n, hipStream_t s, bool *done) {
    *done = false;
    const int64_t R = (int64_t)c->leadrows_host.size(), Npad = (c->N + 511) & ~(int64_t)511;
    // small Grams (ALARM: 60 rows x 5k samples) stay on the popcount kernel: a library call and the
    // one-hot store cost more than they save there
    if (c->blas_failed || !getenv("FBN_CI_GRAM_ROCBLAS") || getenv("FBN_CI_GRAM_NO_BLAS") || R * Npad > kOnehotMaxBytes || Npad > INT32_MAX ||
        (double)R * R * Npad < 1e10 || !Blas().ok)
        return FBN_OK;
    int rc;
    if (!c->onehot_ready) {
        if ((rc = c->onehot.ensure((size_t)(R * Npad)))) return rc;
        hipError_t e = fbn_ci_onehot_build(c->cols.as<uint8_t>(), c->ddims.as<int32_t>(), c->lead0.as<int32_t>(), c->N,
                                           Npad, c->nvars, c->onehot.as<int8_t>(), s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "one-hot build: %s", hipGetErrorString(e));
        c->onehot_Npad = Npad;
        c->onehot_ready = true;
    }
    if (!c->blas) {
        rocblas_handle h = nullptr;
        if (Blas().create(&h) != rocblas_status_success) {
            c->blas_failed = true;
            return FBN_OK;
        }
        c->blas = h;
    }
    rocblas_handle h = (rocblas_handle)c->blas;
    if (Blas().set_stream(h, s) != rocblas_status_success) return FBN_OK;
    // x-variables of the range: pair rows u0 .. u1
    const int nv = c->nvars;
    auto row_of = [&](int64_t t) {
        int64_t lo = 0, hi = nv - 2;
        while (lo < hi) {
            const int64_t m = (lo + hi + 1) / 2;
            if (m * nv - m * (m + 1) / 2 <= t) lo = m;
            else hi = m - 1;
        }
        return (int)lo;
    };
    const int u0 = row_of(t0), u1 = row_of(t0 + n - 1);
    const int64_t r0 = c->lead0_host[u0], r1 = u1 + 1 < nv ? c->lead0_host[u1 + 1] : R;
    if (r1 <= r0) {
        *done = true;
        return FBN_OK;
    }
    const int32_t one = 1, zero = 0;
    const int8_t *O = c->onehot.as<int8_t>();
    // split-K: the 2000 x 2000 output is only 256 tiles of rocBLAS's 128 x 128 for 256 CUs; KS
    // batches over K slices (strided views of the same operand) into separate int32 planes, then one
    // summing pass (integers: exact in any order)
    const int KS = (int)std::max<int64_t>(1, EnvOr0("FBN_CI_GRAM_SPLITK", 4));
    if (KS > 1 && Blas().gemm_sb_ex && Npad % (64 * KS) == 0) {
        const int64_t Kc = Npad / KS, m = r1 - r0;
        int rc2;
        if ((rc2 = c->gram0split.ensure((size_t)(KS * R * m * 4)))) return rc2;
        rocblas_status st = Blas().gemm_sb_ex(
            h, rocblas_operation_transpose, rocblas_operation_none, (rocblas_int)R, (rocblas_int)m, (rocblas_int)Kc,
            &one, O, rocblas_datatype_i8_r, (rocblas_int)Npad, (rocblas_stride)Kc, O + r0 * Npad,
            rocblas_datatype_i8_r, (rocblas_int)Npad, (rocblas_stride)Kc, &zero, c->gram0split.as<int32_t>(),
            rocblas_datatype_i32_r, (rocblas_int)R, (rocblas_stride)(R * m), c->gram0split.as<int32_t>(),
            rocblas_datatype_i32_r, (rocblas_int)R, (rocblas_stride)(R * m), KS, rocblas_datatype_i32_r,
            rocblas_gemm_algo_standard, 0, 0);
        if (st == rocblas_status_success) {
            hipError_t e = fbn_ci_sum_planes(c->gram0split.as<int32_t>(), KS, R * m, c->gram0.as<int32_t>() + r0 * R, s);
            if (e != hipSuccess) return SetError(FBN_ERR_HIP, "gram plane sum: %s", hipGetErrorString(e));
            *done = true;
            return FBN_OK;
        }
    }
    rocblas_status st = Blas().gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, (rocblas_int)R,
                                       (rocblas_int)(r1 - r0), (rocblas_int)Npad, &one, O, rocblas_datatype_i8_r,
                                       (rocblas_int)Npad, O + r0 * Npad, rocblas_datatype_i8_r, (rocblas_int)Npad,
                                       &zero, c->gram0.as<int32_t>() + r0 * R, rocblas_datatype_i32_r, (rocblas_int)R,
                                       c->gram0.as<int32_t>() + r0 * R, rocblas_datatype_i32_r, (rocblas_int)R,
                                       rocblas_datatype_i32_r, rocblas_gemm_algo_standard, 0, 0);
    if (st != rocblas_status_success) {
        c->blas_failed = true;
        return FBN_OK;
    }
    *done = true;
    return FBN_OK;
}

// items: host copy (validated here).  zc_items / zc_indep / zc_df: optional device-visible
// (pinned, mapped) host buffers the kernels read the items from and write the decisions to
// directly -- no staging copies for the small batches of a latency-bound driver round.
// the bit-sliced store (one mask row per value, W words per row padded to a multiple of 4 for
// 16-byte loads) and the per-row sample counts, built once per ctx on stream s
static int CiBitsEnsure(fbn_ci_ctx *c, hipStream_t s) {
    if (c->bits_ready) return FBN_OK;
    int rc;
    const int64_t W = ((c->N + 31) / 32 + 3) & ~(int64_t)3;
    std::vector<int32_t> row0(c->nvars);
    int64_t rows = 0;
    for (int v = 0; v < c->nvars; ++v) row0[v] = (int32_t)rows, rows += std::min(c->dims[v], 8);
    c->row0_host = row0;
    if ((rc = c->bits.ensure((size_t)std::max<int64_t>(rows * W, 1) * 4))) return rc;
    if ((rc = c->brow.ensure((size_t)c->nvars * 4))) return rc;
    FBN_HIP(hipMemcpyAsync(c->brow.p, c->row0_host.data(), (size_t)c->nvars * 4, hipMemcpyHostToDevice, s));
    hipError_t e = fbn_ci_bits_build(c->cols.as<uint8_t>(), c->ddims.as<int32_t>(), c->brow.as<int32_t>(), c->N, W,
                                     c->nvars, c->bits.as<uint32_t>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci bits build: %s", hipGetErrorString(e));
    if ((rc = c->browcnt.ensure((size_t)std::max<int64_t>(rows, 1) * 4))) return rc;
    e = fbn_ci_bits_rowcount(c->bits.as<uint32_t>(), rows, W, c->browcnt.as<int32_t>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci bits row counts: %s", hipGetErrorString(e));
    c->bits_W = W;
    c->bits_ready = true;
    return FBN_OK;
}

// the 2-bit packed columns (every state count <= 4): PW words per variable, built once per ctx
static int CiPack2Ensure(fbn_ci_ctx *c, hipStream_t s) {
    if (c->pack2_ready) return FBN_OK;
    int rc;
    const int64_t PW = (c->N + 15) / 16;
    if ((rc = c->pack2.ensure((size_t)std::max<int64_t>(PW * c->nvars, 1) * 4))) return rc;
    hipError_t e = fbn_ci_pack2_build(c->cols.as<uint8_t>(), c->nvars, c->N, PW, c->pack2.as<uint32_t>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci pack2 build: %s", hipGetErrorString(e));
    c->pack2_W = PW;
    c->pack2_ready = true;
    return FBN_OK;
}

static int CiLaunchDevice(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, bool want_g2p,
                          int32_t *counts_dev, hipStream_t s, int k = 0, const int32_t *zc_items = nullptr,
                          uint8_t *zc_indep = nullptr, int32_t *zc_df = nullptr, const fbn::CiBatchStats *pre = nullptr,
                          bool all_pairs = false, int64_t pair0 = 0) {
    CiSlot &S = c->slot[k];
    if (d < 0 || d > 8) return SetError(FBN_ERR_LIMIT, "conditioning set size %d (supported 0..8)", d);
    const int w = 2 + d;
    // one validation pass: variable ranges and the largest state count (bit-sliced eligibility)
    // (skipped for batches generated by the driver from the skeleton, which pass the same figures)
    int maxdim = 0;
    int64_t dim_rows = 0;  // sum of the items' state counts (bit-sliced input bytes)
    const int *dims = c->dims.data();
    if (pre) {
        maxdim = pre->maxdim, dim_rows = pre->dim_rows;
    } else {
        for (int64_t i = 0; i < n * w; ++i) {
            const int v = items[i];
            if ((unsigned)v >= (unsigned)c->nvars)
                return SetError(FBN_ERR_ARG, "test %lld: variable %d out of range", (long long)(i / w), v);
            maxdim = std::max(maxdim, dims[v]);
            dim_rows += dims[v];
        }
    }
    int rc;
    // tests with <= 1 conditioning variable over variables with <= 4 states: popcounts of
    // bit-sliced columns (ci_bits.hip).  From 4096 samples up (ALARM-5000 included: 0.46 -> 0.40 ms
    // per PC run with the pair-table level 1); below, the byte-column kernel (untuned regime).
    const int64_t kBitsMinSamples = 4096;
    const bool bits_path = d <= 1 && maxdim <= 4 && !getenv("FBN_CI_NO_BITS") &&
                           (c->N >= kBitsMinSamples || getenv("FBN_CI_FORCE_BITS"));
    if (bits_path) {
        if ((rc = CiBitsEnsure(c, s))) return rc;
        if (!all_pairs && (rc = S.items.ensure((size_t)n * w * 4))) return rc;
        if ((rc = S.indep.ensure((size_t)n))) return rc;
        if ((rc = S.df.ensure((size_t)n * 4))) return rc;
        if ((rc = S.bcounts.ensure((size_t)n * 64 * 4))) return rc;
        if (want_g2p) {
            if ((rc = c->g2.ensure((size_t)n * 8))) return rc;
            if ((rc = c->p.ensure((size_t)n * 8))) return rc;
        }
        if (!zc_items && !all_pairs)
            FBN_HIP(hipMemcpyAsync(S.items.p, items, (size_t)n * w * 4, hipMemcpyHostToDevice, s));
        // all pairs of the complete graph: the kernels decode test t into its pair (no item array)
        const int32_t *ditems = all_pairs ? nullptr : zc_items ? zc_items : S.items.as<int32_t>();
        int pmode = 0;
        double *g2rec = nullptr;  // level 0's G^2 per pair, kept for the level-1 screen
        if (c->pair_mode == 1 && d == 0) {
            const size_t np = (size_t)c->nvars * (c->nvars - 1) / 2;
            if ((rc = c->pairtab.ensure(std::max<size_t>(np, 1) * 16 * 4))) return rc;
            pmode = 1;
            c->pairs_recorded = true;
            if (all_pairs && !want_g2p && pair0 == c->l1mi_covered) {
                if ((rc = c->l1mi.ensure(std::max<size_t>(np, 1) * 8))) return rc;
                g2rec = c->l1mi.as<double>() + pair0;
                c->l1mi_covered = pair0 + n;
            }
        } else if (c->pair_mode == 2 && d == 1 && c->pairs_recorded) {
            pmode = 2;
        }
        // mask rows the count kernel reads: the last value of x and y (and z with pair tables)
        // is derived, not read (ci_bits.hip)
        const int64_t skipped = d == 0 ? 2 : (pmode == 2 ? 3 : 0);
        S.last_bytes = (dim_rows - skipped * n) * c->bits_W * 4;
        const double *band = nullptr;  // decisions only: p evaluated inside the band
        int nband = 0;
        if (!want_g2p && (rc = CiBand(c, alpha, s, &band, &nband))) return rc;
        if (c->timing) FBN_HIP(hipEventRecord(S.ev0, s));
        // all pairs of a range: register-blocked count kernel (ci_bits_pairs_tiled), then phase 2
        const bool gram0 = all_pairs && d == 0 && CiGram0Eligible(c);
        const bool tiled = all_pairs && d == 0 && !gram0 && !getenv("FBN_CI_NO_TILED");
        if (tiled && (rc = CiPairTasks(c, pair0, pair0 + n, s))) return rc;
        hipError_t e = hipSuccess;
        if (gram0) {  // Gram of the leading rows, then every pair's table from it
            if ((rc = CiLeadEnsure(c, s))) return rc;
            const int64_t R = (int64_t)c->leadrows_host.size();
            if ((rc = c->gram0.ensure((size_t)(R * R * 4)))) return rc;
            bool done = false;
            if (!getenv("FBN_CI_GRAM_NO_BLAS") && (rc = CiGram0Mfma(c, pair0, n, s, &done))) return rc;
            if (!done && (rc = CiGram0Blas(c, pair0, n, s, &done))) return rc;
            if (!done) {
                if ((rc = CiGram0Tasks(c, pair0, pair0 + n, s))) return rc;
                e = fbn_ci_gram(c->bits.as<uint32_t>(), c->bits_W, c->leadrows.as<int32_t>(),
                                c->g0tasks.as<int32_t>(), c->g0_ntasks, 0, c->gram0.as<int32_t>(), c->num_cu, s);
            }
            if (e == hipSuccess)
                e = fbn_ci_gram_pairs(c->gram0.as<int32_t>(), R, c->lead0.as<int32_t>(), c->ddims.as<int32_t>(),
                                      c->brow.as<int32_t>(), c->browcnt.as<int32_t>(), pair0, n, c->nvars,
                                      S.bcounts.as<int32_t>(), pmode == 1 ? c->pairtab.as<int32_t>() : nullptr,
                                      c->num_cu, s);
            if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci gram level 0: %s", hipGetErrorString(e));
        }
        // level 1 with the per-variable Grams prepared (CiTriplePrepare): tables gathered from them
        const bool gram1 = d == 1 && pmode == 2 && c->triples_ready && pre;  // driver batches only
        if (gram1) {
            e = fbn_ci_gram_triples(c->g1.as<int32_t>(), c->g1goff.as<long long>(), c->g1R.as<int32_t>(),
                                    c->g1adj.as<int32_t>(), c->g1adjoff.as<int32_t>(), c->g1loff.as<int32_t>(),
                                    c->ddims.as<int32_t>(), ditems, n, S.bcounts.as<int32_t>(),
                                    c->pairtab.as<int32_t>(), c->nvars, c->num_cu, s);
            if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci gram level 1: %s", hipGetErrorString(e));
        }
        if (tiled) {
            e = fbn_ci_bits_pairs_tiled(c->bits.as<uint32_t>(), c->brow.as<int32_t>(), c->browcnt.as<int32_t>(),
                                        c->bits_W, c->ptasks.as<int32_t>(), c->ptask_n, c->nvars, pair0, pair0 + n,
                                        S.bcounts.as<int32_t>(), pmode == 1 ? c->pairtab.as<int32_t>() : nullptr,
                                        c->num_cu, s);
            if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci tiled pairs launch: %s", hipGetErrorString(e));
        }
        e = fbn_ci_bits_launch(c->bits.as<uint32_t>(), c->ddims.as<int32_t>(), c->brow.as<int32_t>(),
                                          ditems, c->bits_W, n, d, alpha,
                                          want_g2p ? c->g2.as<double>() : g2rec, zc_df ? zc_df : S.df.as<int32_t>(),
                                          want_g2p ? c->p.as<double>() : nullptr,
                                          zc_indep ? zc_indep : S.indep.as<uint8_t>(),
                                          S.bcounts.as<int32_t>(), counts_dev, c->stats.as<unsigned long long>(),
                                          c->browcnt.as<int32_t>(), c->pairtab.as<int32_t>(), pmode, c->nvars,
                                          c->num_cu, (long long)pair0, (tiled || gram0 || gram1) ? 1 : 0, band,
                                          nband, s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci bits kernel launch: %s", hipGetErrorString(e));
        if (c->timing) FBN_HIP(hipEventRecord(S.ev1, s));
        return FBN_OK;
    }
    if (all_pairs) return SetError(FBN_ERR_ARG, "implicit pair batches need the bit-sliced path");
    size_t lds = 0;
    int64_t mask_rows = 0;  // bit-sliced counting: dimz * (dx + dy + d) mask rows per test
    for (int64_t i = 0; i < n; ++i) {
        const int32_t *it = items + i * w;
        int64_t dimz = 1;
        for (int j = 0; j < d; ++j) dimz *= c->dims[it[2 + j]];
        if (dimz > (1 << 24)) return SetError(FBN_ERR_LIMIT, "test %lld: conditioning table too large", (long long)i);
        lds = std::max(lds, fbn_ci_lds_bytes((int)dimz, c->dims[it[0]], c->dims[it[1]]));
        mask_rows += dimz * (c->dims[it[0]] + c->dims[it[1]] + d);
    }
    // tables beyond the LDS budget: the same layout in a per-workgroup global scratch region
    const bool global_tables = lds > 160 * 1024;
    if ((rc = S.items.ensure((size_t)n * w * 4))) return rc;
    if ((rc = S.indep.ensure((size_t)n))) return rc;
    if ((rc = S.df.ensure((size_t)n * 4))) return rc;
    if (want_g2p) {
        if ((rc = c->g2.ensure((size_t)n * 8))) return rc;
        if ((rc = c->p.ensure((size_t)n * 8))) return rc;
    }
    if (!zc_items) FBN_HIP(hipMemcpyAsync(S.items.p, items, (size_t)n * w * 4, hipMemcpyHostToDevice, s));
    int grid = (int)std::min<int64_t>(n, (int64_t)c->num_cu * 8);
    int32_t *gscratch = nullptr;
    if (global_tables) {
        // one table region per workgroup, at most 4 GiB of scratch in total (fewer, longer-lived
        // workgroups for very large tables; each loops over its tests)
        const size_t stride = ((lds / 4 + 1) & ~(size_t)1) * 4;
        grid = (int)std::max<size_t>(1, std::min<size_t>((size_t)grid, ((size_t)4 << 30) / stride));
        if ((rc = S.scratch.ensure((size_t)grid * stride))) return rc;
        gscratch = S.scratch.as<int32_t>();
    }
    // FBN_CI_BITSN = 1: d >= 2 tests with every state count <= 4 count from the bit-sliced store
    // (ci_kernels.hip) when it is built.  Opt-in: every z-configuration re-reads the x / y value rows,
    // so config 5 level 2 moves more bytes than the byte columns (0.79 vs 0.76 ms) and levels 3-5
    // are several times slower (up to 4^5 configurations per test)
    const bool bitsn0 = d >= 2 && c->bits_ready && maxdim <= 4 && getenv("FBN_CI_BITSN");
    // d = 2 within a PC run (level-0 pair tables recorded), every state count <= 4, the bit-sliced
    // store built: derived counting of the leading cells (ci_kernels.hip MODE 3; FBN_CI_NO_DER2 = 1
    // takes the 2-bit packed histogram kernel instead)
    const bool der2 = d == 2 && c->bits_ready && maxdim <= 4 && c->pair_mode == 2 && c->pairs_recorded &&
                      !global_tables && !getenv("FBN_CI_NO_DER2");
    const bool bitsn = bitsn0 || der2;
    // decisions only: the decision band up to this batch's largest df ((maxdim-1)^2 maxdim^d)
    const double *hband = nullptr;
    int hnband = 0;
    if (!want_g2p) {
        double dfmax = (double)(maxdim - 1) * (maxdim - 1);
        for (int j = 0; j < d; ++j) dfmax *= maxdim;
        if ((rc = CiBand(c, alpha, s, &hband, &hnband, (int)std::min<double>(dfmax, kBandDfMax)))) return rc;
    }
    // every variable of the batch with <= 4 states and >= 64k samples: the histogram kernel reads
    // the columns packed 2 bits per sample (a quarter of the byte columns' bytes; built once per
    // context, 25 MB for config 5).  Config-5 level 2: 0.614 -> 0.589 ms (the kernel's binning, not
    // its column reads, bounds it); below 64k samples (ALARM-5000) the byte columns measured faster.
    // FBN_CI_PACK2 = 1 forces it at any size, FBN_CI_NO_PACK2 = 1 disables it.
    const bool pk = !bitsn && maxdim <= 4 && !getenv("FBN_CI_NO_PACK2") &&
                    (c->N >= 65536 || getenv("FBN_CI_PACK2"));
    if (pk && (rc = CiPack2Ensure(c, s))) return rc;
    S.last_bytes = bitsn ? mask_rows * c->bits_W * 4  // the mask rows each z-configuration reads
                   : pk  ? n * c->pack2_W * 4 * (2 + d)  // the 2-bit columns x, y, z_1..z_d
                         : n * c->N * (2 + d);  // uint8 columns x, y, z_1..z_d streamed once
    // small batches on the packed columns (config 5 levels 3-5: 1056 / 260 / 30 tests of 100k
    // samples): each test's words split over several workgroups so the batch fills the chip, the
    // partial histograms added into a global table per test, then one workgroup per test decides
    int split = 1, split_grid = 0;
    int64_t tstride = 0;
    int32_t *tab = nullptr;
    static const int split_env = getenv("FBN_CI_SPLIT") ? atoi(getenv("FBN_CI_SPLIT")) : -1;  // (tuning knob)
    if (pk && !bitsn && !global_tables) {
        const int64_t want = 4 * (int64_t)c->num_cu;  // counting workgroups to aim for
        split = split_env >= 0 ? std::max(1, split_env) : (int)std::min<int64_t>(16, want / std::max<int64_t>(n, 1));
        if (split > 1) {
            int64_t cmax = 1;
            for (int64_t i = 0; i < n; ++i) {
                const int32_t *it = items + i * w;
                int64_t cells = (int64_t)c->dims[it[0]] * c->dims[it[1]];
                for (int j = 0; j < d; ++j) cells *= c->dims[it[2 + j]];
                cmax = std::max(cmax, cells);
            }
            tstride = (cmax + 63) & ~(int64_t)63;
            if ((rc = S.scratch.ensure((size_t)n * tstride * 4))) return rc;
            tab = S.scratch.as<int32_t>();
            split_grid = (int)std::min<int64_t>(n * split, (int64_t)c->num_cu * 8);
        }
    }
    if (c->timing) FBN_HIP(hipEventRecord(S.ev0, s));
    hipError_t e = fbn_ci_launch(c->cols.as<uint8_t>(), c->ddims.as<int32_t>(),
                                 zc_items ? zc_items : S.items.as<int32_t>(), c->N, n, d, alpha,
                                 want_g2p ? c->g2.as<double>() : nullptr, zc_df ? zc_df : S.df.as<int32_t>(),
                                 want_g2p ? c->p.as<double>() : nullptr, zc_indep ? zc_indep : S.indep.as<uint8_t>(),
                                 counts_dev, lds, grid, gscratch, c->stats.as<unsigned long long>(),
                                 bitsn ? c->bits.as<uint32_t>() : nullptr, c->brow.as<int32_t>(), c->bits_W, hband,
                                 hnband, pk ? c->pack2.as<uint32_t>() : nullptr, c->pack2_W, c->counts_stride, tab,
                                 tstride, split, split_grid, der2 ? c->pairtab.as<int32_t>() : nullptr, c->nvars, s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci kernel launch: %s", hipGetErrorString(e));
    if (c->timing) FBN_HIP(hipEventRecord(S.ev1, s));
    return FBN_OK;
}

int fbn_ci_run(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, double *g2, int32_t *df, double *p,
               uint8_t *indep, void *hip_stream) {
    if (!c || (!items && n > 0) || n < 0) return SetError(FBN_ERR_ARG, "bad argument");
    if (n == 0) return FBN_OK;
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (std::find(c->streams_used.begin(), c->streams_used.end(), s) == c->streams_used.end())
        c->streams_used.push_back(s);
    int rc = CiLaunchDevice(c, items, n, d, alpha, g2 || p, nullptr, s);
    if (rc) return rc;
    if (g2) FBN_HIP(hipMemcpyAsync(g2, c->g2.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    if (p) FBN_HIP(hipMemcpyAsync(p, c->p.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
    if (df) FBN_HIP(hipMemcpyAsync(df, c->slot[0].df.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (indep) FBN_HIP(hipMemcpyAsync(indep, c->slot[0].indep.p, (size_t)n, hipMemcpyDeviceToHost, s));
    FBN_HIP(hipStreamSynchronize(s));
    c->last_ms = 0.f;
    if (c->timing) FBN_HIP(hipEventElapsedTime(&c->last_ms, c->slot[0].ev0, c->slot[0].ev1));
    return FBN_OK;
}

int fbn_ci_counts(fbn_ci_ctx *c, int x, int y, const int32_t *z, int d, int32_t *counts, int64_t cap, int64_t *cells) {
    if (!c || (!z && d > 0) || d < 0 || d > 8) return SetError(FBN_ERR_ARG, "bad argument");
    std::vector<int32_t> item{x, y};
    for (int j = 0; j < d; ++j) item.push_back(z[j]);
    for (int32_t v : item)
        if (v < 0 || v >= c->nvars) return SetError(FBN_ERR_ARG, "variable out of range");
    int64_t nc = (int64_t)c->dims[x] * c->dims[y];
    for (int j = 0; j < d; ++j) nc *= c->dims[z[j]];
    if (cells) *cells = nc;
    FBN_HIP(hipSetDevice(c->device));
    int rc;
    if ((rc = c->counts.ensure((size_t)nc * 4))) return rc;
    rc = CiLaunchDevice(c, item.data(), 1, d, 0.05, false, c->counts.as<int32_t>(), nullptr);
    if (rc) return rc;
    if (counts) FBN_HIP(hipMemcpy(counts, c->counts.p, (size_t)std::min(nc, cap) * 4, hipMemcpyDeviceToHost));
    FBN_HIP(hipDeviceSynchronize());
    return FBN_OK;
}

// Counts of n tests through the kernels a PC run uses at level d (parity pinning of the production
// paths): d = 0 the complete-graph level-0 batch (the Gram of the leading mask rows, then every
// pair's table, recorded for level 1), d = 1 the derived counting from those recorded pair tables
// (the level-0 batch runs first if none are recorded), d >= 2 the histogram kernel over one batch.
// counts [n][cap]: test t's table in Counts3D order, cells beyond it untouched.
int fbn_ci_debug_counts(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, int32_t *counts, int64_t cap) {
    if (!c || (!items && n > 0) || n < 0 || d < 0 || d > 8 || (!counts && n > 0) || cap < 1)
        return SetError(FBN_ERR_ARG, "bad argument");
    if (n == 0) return FBN_OK;
    const int w = 2 + d;
    for (int64_t i = 0; i < n * w; ++i)
        if ((unsigned)items[i] >= (unsigned)c->nvars) return SetError(FBN_ERR_ARG, "variable out of range");
    FBN_HIP(hipSetDevice(c->device));
    int rc;
    const int nv = c->nvars;
    fbn::PCResultHost scratch;
    // a debug call must not change which path later batches on this ctx take: the pair mode (and
    // with it the derived level-1 / level-2 counting) is restored on every exit
    struct PairModeGuard {
        fbn_ci_ctx *c;
        int mode;
        bool recorded, triples;
        ~PairModeGuard() { c->pair_mode = mode, c->pairs_recorded = recorded, c->triples_ready = triples; }
    } guard{c, c->pair_mode, c->pairs_recorded, c->triples_ready};
    auto level0 = [&]() -> int {  // the PC run's level 0, pair tables recorded
        fbn::CiBatchStats st{0, 0};
        for (int v = 0; v < nv; ++v) st.dim_rows += (int64_t)(nv - 1) * c->dims[v], st.maxdim = std::max(st.maxdim, (int)c->dims[v]);
        if (!fbn::CiAllPairsEligible(c, st))
            return SetError(FBN_ERR_ARG, "dataset not eligible for the bit-sliced level-0 path");
        const int64_t P = (int64_t)nv * (nv - 1) / 2;
        fbn::CiSetPairMode(c, 1);
        int r = fbn::CiBatchLaunchAllPairs(c, 0.05, &st, 0, P);
        std::vector<uint8_t> flags((size_t)P);
        if (!r) r = fbn::CiBatchWait(c, 0, flags.data(), nullptr, scratch);
        if (!r) fbn::CiSetPairMode(c, 2);
        return r;
    };
    std::vector<int32_t> rec((size_t)n * 64);
    if (d == 0) {
        if ((rc = level0())) return rc;
        FBN_HIP(hipStreamSynchronize(c->stream));
        for (int64_t t = 0; t < n; ++t) {
            const int x = items[2 * t], y = items[2 * t + 1];
            if (x >= y) return SetError(FBN_ERR_ARG, "level-0 tests are pairs x < y");
            const int64_t pi = (int64_t)x * nv - (int64_t)x * (x + 1) / 2 + (y - x - 1);
            FBN_HIP(hipMemcpy(rec.data() + t * 64, c->slot[0].bcounts.as<int32_t>() + pi * 64, 64 * 4,
                              hipMemcpyDeviceToHost));
        }
    } else if (d == 1) {
        if (!c->pairs_recorded && (rc = level0())) return rc;
        fbn::CiSetPairMode(c, 2);
        std::vector<uint8_t> ind((size_t)n);
        if ((rc = fbn::CiBatchLaunch(c, 0, items, n, 1, 0.05, false)) || (rc = fbn::CiBatchWait(c, 0, ind.data(), nullptr, scratch)))
            return rc;
        FBN_HIP(hipMemcpy(rec.data(), c->slot[0].bcounts.p, (size_t)n * 64 * 4, hipMemcpyDeviceToHost));
    }
    if (d <= 1) {
        for (int64_t t = 0; t < n; ++t) {
            int64_t cells = (int64_t)c->dims[items[w * t]] * c->dims[items[w * t + 1]];
            if (d == 1) cells *= c->dims[items[w * t + 2]];
            std::copy(rec.begin() + t * 64, rec.begin() + t * 64 + std::min<int64_t>(cells, cap), counts + t * cap);
        }
        return FBN_OK;
    }
    if (d == 2) {  // a PC run's level 2 has its level-0 pair tables (derived counting, ci_kernels.hip MODE 3)
        fbn::CiBatchStats st{0, 0};
        for (int v = 0; v < nv; ++v) st.maxdim = std::max(st.maxdim, (int)c->dims[v]);
        if (!c->pairs_recorded && st.maxdim <= 4 && c->N >= 4096 && (rc = level0())) return rc;
        if (c->pairs_recorded) fbn::CiSetPairMode(c, 2);
    }
    if ((rc = c->counts.ensure((size_t)n * cap * 4))) return rc;
    FBN_HIP(hipMemsetAsync(c->counts.p, 0, (size_t)n * cap * 4, c->stream));  // cells beyond a table: 0
    c->counts_stride = cap;
    rc = CiLaunchDevice(c, items, n, d, 0.05, false, c->counts.as<int32_t>(), c->stream);
    c->counts_stride = 0;
    if (rc) return rc;
    FBN_HIP(hipStreamSynchronize(c->stream));
    FBN_HIP(hipMemcpy(counts, c->counts.p, (size_t)n * cap * 4, hipMemcpyDeviceToHost));
    return FBN_OK;
}

int fbn_ci_decision_margin(fbn_ci_ctx *c, double *min_margin, int64_t *near_alpha, int reset) {
    if (!c) return SetError(FBN_ERR_ARG, "null pointer");
    FBN_HIP(hipSetDevice(c->device));
    int rc = CiReadMargin(c, min_margin, near_alpha);
    if (rc == FBN_OK && reset) rc = CiResetMargin(c);
    return rc;
}

int fbn_pc_decision_margin(const fbn_pc_result *r, double *min_margin, int64_t *near_alpha) {
    if (!r) return SetError(FBN_ERR_ARG, "null pointer");
    if (min_margin) *min_margin = r->r.min_margin;
    if (near_alpha) *near_alpha = r->r.near_alpha;
    return FBN_OK;
}

int fbn_ci_last_kernel_ms(const fbn_ci_ctx *c, float *ms) {
    if (!c || !ms) return SetError(FBN_ERR_ARG, "null pointer");
    *ms = c->last_ms;
    return FBN_OK;
}

int fbn_ci_ctx_destroy(fbn_ci_ctx *c) {
    if (!c) return FBN_OK;
    // nothing of this ctx may still run when its buffers, pinned records and stream go: the device-
    // resident search returns on its completion word, and batches may be queued on caller streams
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipStream_t s : c->streams_used) (void)hipStreamSynchronize(s);
    delete c;
    return FBN_OK;
}

// ------------------------------------------------------------------ PC-stable
int fbn_pc_stable(fbn_ci_ctx *c, double alpha, int depth, int group_size, fbn_pc_result **out) {
    if (!c || !out || depth < 1 || !(alpha >= 0.0 && alpha <= 1.0)) return SetError(FBN_ERR_ARG, "bad argument");
    auto r = std::unique_ptr<fbn_pc_result>(new (std::nothrow) fbn_pc_result());
    if (!r) return SetError(FBN_ERR_NOMEM, "out of memory");
    FBN_HIP(hipSetDevice(c->device));
    static const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    auto t0 = std::chrono::steady_clock::now();
    int rc;
    // the device-resident search (small graphs) sets the ctx's margin log itself (and resets it when
    // it falls back to the host levels)
    if (!fbn::CiPCSmallEligible(c, group_size) && (rc = CiResetMargin(c))) return rc;
    auto t1 = std::chrono::steady_clock::now();
    if ((rc = fbn::RunPCStable(c, alpha, depth, group_size, r->r))) return rc;
    auto t2 = std::chrono::steady_clock::now();
    // the run's work is all on the ctx stream
    if (!r->r.margin_done && (rc = CiReadMargin(c, &r->r.min_margin, &r->r.near_alpha, true))) return rc;
    auto t3 = std::chrono::steady_clock::now();
    if ((rc = fbn::OrientPC(c->nvars, r->r))) return rc;  // StructLearnByPCStable steps 2-3
    if (timing) {
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        fprintf(stderr, "pc_stable: margin reset %.2f ms, skeleton %.2f ms, margin read %.2f ms, orientation %.2f ms\n",
                ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, std::chrono::steady_clock::now()));
    }
    *out = r.release();
    return FBN_OK;
}
int fbn_pc_num_levels(const fbn_pc_result *r, int *n) {
    if (!r || !n) return SetError(FBN_ERR_ARG, "null pointer");
    *n = (int)r->r.tests_per_level.size();
    return FBN_OK;
}
int fbn_pc_level_tests(const fbn_pc_result *r, int64_t *tests) {
    if (!r || !tests) return SetError(FBN_ERR_ARG, "null pointer");
    std::copy(r->r.tests_per_level.begin(), r->r.tests_per_level.end(), tests);
    return FBN_OK;
}
int fbn_pc_level_launched(const fbn_pc_result *r, int64_t *tests) {
    if (!r || !tests) return SetError(FBN_ERR_ARG, "null pointer");
    std::copy(r->r.launched_per_level.begin(), r->r.launched_per_level.end(), tests);
    return FBN_OK;
}
int fbn_pc_num_edges(const fbn_pc_result *r, int *n) {
    if (!r || !n) return SetError(FBN_ERR_ARG, "null pointer");
    *n = (int)r->r.edges.size();
    return FBN_OK;
}
int fbn_pc_edges(const fbn_pc_result *r, int32_t *pairs) {
    if (!r || !pairs) return SetError(FBN_ERR_ARG, "null pointer");
    for (size_t i = 0; i < r->r.edges.size(); ++i) pairs[2 * i] = r->r.edges[i].first, pairs[2 * i + 1] = r->r.edges[i].second;
    return FBN_OK;
}
static constexpr int32_t kPcRecordMagic = 0x52504246;  // 'FBPR': fbn_pc_result_record layout version 1
int fbn_pc_sepsets(const fbn_pc_result *r, int32_t *buf, int64_t cap, int64_t *len) {
    if (!r) return SetError(FBN_ERR_ARG, "null pointer");
    int64_t k = 0;
    auto put = [&](int32_t v) {
        if (buf && k < cap) buf[k] = v;
        ++k;
    };
    const auto &sm = r->r.sepset;
    for (size_t i = 0, n = sm.sorted_size(); i < n; ++i) {
        const auto key = sm.key(i);
        const auto z = sm.value(i);
        put(key.first);
        put(key.second);
        put((int32_t)z.size());
        for (int v : z) put(v);
    }
    if (len) *len = k;
    return FBN_OK;
}
int fbn_pc_result_record(const fbn_pc_result *r, int32_t *buf, int64_t cap, int64_t *len) {
    if (!r) return SetError(FBN_ERR_ARG, "null pointer");
    int64_t k = 0;
    auto put = [&](int32_t v) {
        if (buf && k < cap) buf[k] = v;
        ++k;
    };
    const auto &R = r->r;
    put(kPcRecordMagic);
    put((int32_t)R.tests_per_level.size());
    for (int64_t t : R.tests_per_level) put((int32_t)(uint32_t)(uint64_t)t), put((int32_t)((uint64_t)t >> 32));
    put((int32_t)R.edges.size());
    for (auto &e : R.edges) put(e.first), put(e.second);
    int64_t slen = 0;
    fbn_pc_sepsets(r, nullptr, 0, &slen);
    put((int32_t)slen);
    if (buf && k + slen <= cap) fbn_pc_sepsets(r, buf + k, slen, nullptr);
    k += slen;
    if (len) *len = k;
    if (buf && k > cap) return SetError(FBN_ERR_LIMIT, "record needs %lld ints (cap %lld)", (long long)k, (long long)cap);
    return FBN_OK;
}
int fbn_pc_small_eligible(const fbn_ci_ctx *c, int group_size, int *eligible) {
    if (!c || !eligible) return SetError(FBN_ERR_ARG, "null pointer");
    *eligible = fbn::CiPCSmallEligible(c, group_size) ? 1 : 0;
    return FBN_OK;
}
int fbn_pc_small_eligible_shape(int nvars, int64_t nsamples, const int32_t *dims, int group_size, int *eligible) {
    if (!eligible || (nvars > 0 && !dims)) return SetError(FBN_ERR_ARG, "null pointer");
    *eligible = fbn::PCSmallShape(nvars, nsamples, dims, group_size) ? 1 : 0;
    return FBN_OK;
}
int fbn_pc_level(fbn_ci_ctx *c, double alpha, int d, int group_size, const int32_t *edges, int64_t nedges,
                 int64_t e_begin, int64_t e_end, uint8_t *removed, int32_t *sepsets, int64_t *counted,
                 int64_t *launched) {
    if (!c || d < 0 || d > 8 || group_size < 1 || group_size > 8 || nedges < 0 || (nedges && !edges) ||
        e_begin < 0 || e_end < e_begin || e_end > nedges || (e_end > e_begin && !removed))
        return SetError(FBN_ERR_ARG, "bad argument");
    std::vector<std::pair<int, int>> ev((size_t)nedges);
    std::vector<std::vector<int>> adj(c->nvars);
    for (int64_t i = 0; i < nedges; ++i) {
        const int a = edges[2 * i], b = edges[2 * i + 1];
        if (a < 0 || b <= a || b >= c->nvars) return SetError(FBN_ERR_ARG, "edge %lld must be (x < y) in range", (long long)i);
        if (i && !(ev[i - 1] < std::make_pair(a, b))) return SetError(FBN_ERR_ARG, "edges must be in (x, y) lexicographic order");
        ev[i] = {a, b};
        adj[a].push_back(b);  // lexicographic edges: every list comes out sorted (no sort pass)
        adj[b].push_back(a);
    }
    FBN_HIP(hipSetDevice(c->device));
    fbn::PCResultHost scratch;
    fbn::LevelOut out;
    int rc = fbn::RunLevel(c, alpha, d, group_size, adj, ev, (size_t)e_begin, (size_t)e_end, out, scratch);
    if (rc) return rc;
    for (int64_t e = 0; e < e_end - e_begin; ++e) {
        removed[e] = out.removed[e] ? 1 : 0;
        if (sepsets)
            for (int j = 0; j < d; ++j) sepsets[e * d + j] = out.removed[e] ? out.sep[(size_t)e * d + j] : -1;
    }
    if (counted) *counted = out.counted;
    if (launched) *launched = out.launched;
    return FBN_OK;
}
int fbn_pc_orient_skeleton(int nvars, const int32_t *pairs, int nedges, const int32_t *sepsets, int64_t len,
                           fbn_pc_result **out) {
    if (nvars <= 0 || nedges < 0 || (nedges && !pairs) || (len && !sepsets) || !out)
        return SetError(FBN_ERR_ARG, "bad argument");
    auto r = std::unique_ptr<fbn_pc_result>(new (std::nothrow) fbn_pc_result());
    if (!r) return SetError(FBN_ERR_NOMEM, "out of memory");
    for (int i = 0; i < nedges; ++i) {
        const int a = pairs[2 * i], b = pairs[2 * i + 1];
        if (a < 0 || b < 0 || a >= nvars || b >= nvars || a == b) return SetError(FBN_ERR_ARG, "bad edge %d", i);
        r->r.edges.push_back({std::min(a, b), std::max(a, b)});
    }
    for (int64_t k = 0; k < len;) {  // (x, y, m, z_0..z_{m-1}) records, as fbn_pc_sepsets writes them
        if (k + 3 > len || k + 3 + sepsets[k + 2] > len || sepsets[k + 2] < 0) return SetError(FBN_ERR_ARG, "bad sepset list");
        const int x = sepsets[k], y = sepsets[k + 1], m = sepsets[k + 2];
        r->r.sepset.set({std::min(x, y), std::max(x, y)}, sepsets + k + 3, m);
        k += 3 + m;
    }
    int rc = fbn::OrientPC(nvars, r->r);
    if (rc) return rc;
    *out = r.release();
    return FBN_OK;
}
int fbn_pc_num_oriented_edges(const fbn_pc_result *r, int *n) {
    if (!r || !n) return SetError(FBN_ERR_ARG, "null pointer");
    *n = (int)r->r.oriented.size();
    return FBN_OK;
}
int fbn_pc_oriented_edges(const fbn_pc_result *r, int32_t *triples) {
    if (!r || !triples) return SetError(FBN_ERR_ARG, "null pointer");
    for (size_t i = 0; i < r->r.oriented.size(); ++i)
        for (int k = 0; k < 3; ++k) triples[3 * i + k] = r->r.oriented[i][k];
    return FBN_OK;
}
int fbn_shd_bif(const char *bif_path, int nvars, const int32_t *triples, int n, int *shd) {
    if (!bif_path || !shd || n < 0 || (n && !triples)) return SetError(FBN_ERR_ARG, "bad argument");
    std::vector<std::string> names;
    std::vector<std::pair<int, int>> arcs;
    int rc = fbn::LoadBifGraph(bif_path, names, arcs);
    if (rc) return rc;
    if ((int)names.size() != nvars)
        return SetError(FBN_ERR_ARG, "%s has %zu variables, the learned graph %d", bif_path, names.size(), nvars);
    std::vector<std::array<int, 3>> learned(n);
    for (int i = 0; i < n; ++i) {
        learned[i] = {triples[3 * i], triples[3 * i + 1], triples[3 * i + 2] ? 1 : 0};
        if (learned[i][0] < 0 || learned[i][0] >= nvars || learned[i][1] < 0 || learned[i][1] >= nvars)
            return SetError(FBN_ERR_ARG, "edge %d out of range", i);
    }
    int unl = 0;
    return fbn::ComputeSHD(nvars, arcs, learned, shd, &unl);
}
int fbn_pc_shd_bif(const fbn_pc_result *r, const char *bif_path, int *shd) {
    if (!r || !bif_path || !shd) return SetError(FBN_ERR_ARG, "null pointer");
    std::vector<int32_t> t(3 * r->r.oriented.size() + 3);
    for (size_t i = 0; i < r->r.oriented.size(); ++i)
        for (int k = 0; k < 3; ++k) t[3 * i + k] = r->r.oriented[i][k];
    return fbn_shd_bif(bif_path, r->r.num_nodes, t.data(), (int)r->r.oriented.size(), shd);
}
int fbn_pc_device_bytes(const fbn_pc_result *r, int64_t *bytes) {
    if (!r || !bytes) return SetError(FBN_ERR_ARG, "null pointer");
    *bytes = r->r.device_bytes;
    return FBN_OK;
}
int fbn_pc_path(const fbn_pc_result *r, int *path) {
    if (!r || !path) return SetError(FBN_ERR_ARG, "null pointer");
    *path = r->r.path;
    return FBN_OK;
}
int fbn_pc_timing(const fbn_pc_result *r, double *total_s, double *kernel_s) {
    if (!r) return SetError(FBN_ERR_ARG, "null pointer");
    if (total_s) *total_s = r->r.total_s;
    if (kernel_s) *kernel_s = r->r.kernel_s;
    return FBN_OK;
}
int fbn_pc_result_destroy(fbn_pc_result *r) {
    delete r;
    return FBN_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ driver seam
namespace fbn {
void CiCtxShape(const fbn_ci_ctx *c, int *nvars, int64_t *nsamples) {
    *nvars = c->nvars;
    *nsamples = c->N;
}
// batches up to this many item bytes take the zero-copy path of CiBatchLaunch
constexpr size_t kZeroCopyBytes = 256 << 10;
const int32_t *CiCtxDims(const fbn_ci_ctx *c) { return c->dims.data(); }
void CiSetPairMode(fbn_ci_ctx *c, int mode) {
    c->pair_mode = mode;
    if (mode == 1) c->l1mi_covered = 0;  // a new level 0 records from pair 0
    c->triples_ready = false;
    if (mode != 2) c->pairs_recorded = false;
}
int CiBatchLaunch(fbn_ci_ctx *c, int k, const int32_t *items, int64_t n, int d, double alpha, bool want_df,
                  const CiBatchStats *pre) {
    CiSlot &S = c->slot[k];
    S.n = n;
    S.want_df = want_df;
    if (n == 0) return FBN_OK;
    // pinned staging: the copies are true DMA on the ctx stream, one host sync per round
    const size_t ib = (size_t)n * (2 + d) * 4, rb = (size_t)n * 5 + 8;
    int rc;
    if ((rc = PinnedEnsure(S.h_items, S.h_items_bytes, ib))) return rc;
    if ((rc = PinnedEnsure(S.h_res, S.h_res_bytes, rb))) return rc;
    memcpy(S.h_items, items, ib);
    uint8_t *h_ind = static_cast<uint8_t *>(S.h_res);
    int32_t *h_df = reinterpret_cast<int32_t *>(h_ind + (((size_t)n + 3) & ~(size_t)3));
    const int32_t *hi = static_cast<const int32_t *>(S.h_items);
    // small rounds (the latency-bound ones): the kernel reads the items from and writes the
    // decisions to the pinned buffers directly (one launch + one sync per round); large rounds
    // stage through device memory with DMA copies
    S.zc = ib <= kZeroCopyBytes && !getenv("FBN_CI_NO_ZEROCOPY");
    if (S.zc) {
        rc = CiLaunchDevice(c, hi, n, d, alpha, false, nullptr, c->stream, k, hi, h_ind, want_df ? h_df : nullptr, pre);
        if (rc) return rc;
    } else {
        rc = CiLaunchDevice(c, hi, n, d, alpha, false, nullptr, c->stream, k, nullptr, nullptr, nullptr, pre);
        if (rc) return rc;
        FBN_HIP(hipMemcpyAsync(h_ind, S.indep.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
        if (want_df) FBN_HIP(hipMemcpyAsync(h_df, S.df.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    FBN_HIP(hipEventRecord(S.done, c->stream));
    return FBN_OK;
}
bool CiAllPairsEligible(const fbn_ci_ctx *c, const CiBatchStats &st) {
    return st.maxdim <= 4 && !getenv("FBN_CI_NO_BITS") && (c->N >= 4096 || getenv("FBN_CI_FORCE_BITS"));
}
int CiBatchLaunchAllPairs(fbn_ci_ctx *c, double alpha, const CiBatchStats *pre, int64_t t0, int64_t n,
                          bool copy_flags) {
    CiSlot &S = c->slot[0];
    S.n = n;
    S.want_df = false;
    S.zc = false;
    if (n == 0) return FBN_OK;
    int rc;
    if ((rc = PinnedEnsure(S.h_res, S.h_res_bytes, (size_t)n * 5 + 8))) return rc;
    rc = CiLaunchDevice(c, nullptr, n, 0, alpha, false, nullptr, c->stream, 0, nullptr, nullptr, nullptr, pre, true,
                        t0);
    if (rc) return rc;
    if (copy_flags) FBN_HIP(hipMemcpyAsync(S.h_res, S.indep.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    FBN_HIP(hipEventRecord(S.done, c->stream));
    return FBN_OK;
}

bool CiPairsReady(const fbn_ci_ctx *c) { return c->pair_mode == 2 && c->pairs_recorded; }

// Decided before the level-0 launch, so the bit-sliced store the device hand-off reads is built
// here when the dataset qualifies for it (the same test as CiLaunchDevice's bits path): a fresh ctx
// -- every one-shot CLI run -- takes the device path from its first PC run on.
bool CiL0L1DeviceEligible(fbn_ci_ctx *c, int group_size) {
    if (group_size != 1 || getenv("FBN_PC_HOST_L1") || getenv("FBN_PC_HOST_L0L1") || c->nvars < 2) return false;
    for (int v = 0; v < c->nvars; ++v)
        if (c->dims[v] > 4) return false;
    if (!c->bits_ready) {
        const bool bits_path = !getenv("FBN_CI_NO_BITS") && (c->N >= 4096 || getenv("FBN_CI_FORCE_BITS"));
        if (!bits_path || CiBitsEnsure(c, c->stream) != FBN_OK) return false;
    }
    return true;
}

int CiL0L1Device(fbn_ci_ctx *c, int64_t P, int *E, int64_t *cands, PCResultHost &res) {
    const int n = c->nvars;
    if (P != (int64_t)n * (n - 1) / 2 || P > INT32_MAX / 2) return SetError(FBN_ERR_ARG, "level 0 -> 1 on the device: one complete-graph batch");
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    CiSlot &S = c->slot[0];
    int rc;
    if ((rc = c->kcnt.ensure((size_t)n * 8)) || (rc = c->kscal.ensure(16)) || (rc = c->l1adjoff.ensure((size_t)(n + 1) * 4)) ||
        (rc = c->l1adj.ensure((size_t)std::max<int64_t>(2 * P, 1) * 4)) || (rc = c->l1pairs.ensure((size_t)std::max<int64_t>(P, 1) * 8)) ||
        (rc = c->kupoff.ensure((size_t)n * 4)))
        return rc;
    if (!c->h_kept) {
        hipError_t e = hipHostMalloc((void **)&c->h_kept, 16, hipHostMallocDefault);
        if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc: %s", hipGetErrorString(e));
    }
    if (!c->side) {
        FBN_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        FBN_HIP(hipEventCreateWithFlags(&c->side_ev, hipEventDisableTiming));
        FBN_HIP(hipEventCreateWithFlags(&c->main_ev, hipEventDisableTiming));
    }
    // the decision flags to the host on the side stream, behind the level-0 kernels
    FBN_HIP(hipStreamWaitEvent(c->side, S.done, 0));
    FBN_HIP(hipMemcpyAsync(S.h_res, S.indep.p, (size_t)P, hipMemcpyDeviceToHost, c->side));
    int32_t *cnt = c->kcnt.as<int32_t>();
    hipError_t e = fbn_ci_kept_csr(S.indep.as<uint8_t>(), n, cnt, cnt + n, c->l1adjoff.as<int32_t>(), c->kupoff.as<int32_t>(),
                                   c->l1adj.as<int32_t>(), c->l1pairs.as<int32_t>(), c->kscal.as<long long>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "kept-pair CSR: %s", hipGetErrorString(e));
    long long *hk = reinterpret_cast<long long *>(c->h_kept);
    FBN_HIP(hipMemcpyAsync(hk, c->kscal.p, 16, hipMemcpyDeviceToHost, s));
    FBN_HIP(hipEventRecord(c->main_ev, s));
    FBN_HIP(EventWaitSpin(c->main_ev));
    *E = (int)hk[0];
    *cands = hk[1];
    // the edge list to the host on the side stream (the CSR kernels are done: main_ev)
    if ((rc = PinnedEnsure(c->h_pairs, c->h_pairs_bytes, (size_t)std::max(*E, 1) * 8))) return rc;
    FBN_HIP(hipStreamWaitEvent(c->side, c->main_ev, 0));
    if (*E) FBN_HIP(hipMemcpyAsync(c->h_pairs, c->l1pairs.p, (size_t)*E * 8, hipMemcpyDeviceToHost, c->side));
    FBN_HIP(hipEventRecord(c->side_ev, c->side));
    // the level-0 batch in the run's accounting (as CiBatchWait)
    float ms = 0.f;
    if (c->timing) FBN_HIP(hipEventElapsedTime(&ms, S.ev0, S.ev1));
    res.kernel_s += ms * 1e-3;
    res.device_bytes += S.last_bytes;
    S.n = 0;
    return FBN_OK;
}

int CiL0L1Host(fbn_ci_ctx *c, int64_t P, int E, std::vector<char> &removed, std::vector<std::pair<int, int>> &edges,
               std::vector<std::vector<int>> &adj) {
    FBN_HIP(EventWaitSpin(c->side_ev));
    removed.resize((size_t)P);
    memcpy(removed.data(), c->slot[0].h_res, (size_t)P);
    static_assert(sizeof(std::pair<int, int>) == 8, "pair layout");
    edges.resize((size_t)E);
    if (E) memcpy(static_cast<void *>(edges.data()), c->h_pairs, (size_t)E * 8);
    const int n = c->nvars;
    {
        std::vector<int> deg(n, 0);
        for (auto &e : edges) ++deg[e.first], ++deg[e.second];
        for (int v = 0; v < n; ++v) adj[v].reserve(deg[v]);
    }
    for (auto &e : edges) adj[e.first].push_back(e.second), adj[e.second].push_back(e.first);
    return FBN_OK;
}
int CiPairTablesCopy(fbn_ci_ctx *c, int64_t p0, int64_t np, void *buf, bool buf_on_device, bool to_ctx) {
    if (np < 0 || p0 < 0) return SetError(FBN_ERR_ARG, "bad pair range");
    const int64_t P = (int64_t)c->nvars * (c->nvars - 1) / 2;
    if (p0 + np > P) return SetError(FBN_ERR_ARG, "pair range [%lld, %lld) beyond %lld pairs", (long long)p0,
                                     (long long)(p0 + np), (long long)P);
    FBN_HIP(hipSetDevice(c->device));
    int rc;
    if ((rc = c->pairtab.ensure(std::max<size_t>((size_t)P, 1) * 16 * 4))) return rc;
    if (!to_ctx && !c->pairs_recorded) return SetError(FBN_ERR_ARG, "no pair tables recorded on this context");
    char *ctx_ptr = c->pairtab.as<char>() + (size_t)p0 * 64;
    const size_t bytes = (size_t)np * 64;
    const hipMemcpyKind kind = to_ctx ? (buf_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                                      : (buf_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost);
    FBN_HIP(hipStreamSynchronize(c->stream));
    if (bytes) FBN_HIP(hipMemcpy(to_ctx ? (void *)ctx_ptr : buf, to_ctx ? (const void *)buf : ctx_ptr, bytes, kind));
    return FBN_OK;
}
int CiMarginReset(fbn_ci_ctx *c) {
    FBN_HIP(hipSetDevice(c->device));
    return CiResetMargin(c);
}
int CiMarginRead(fbn_ci_ctx *c, double *min_margin, int64_t *near_alpha) {
    FBN_HIP(hipSetDevice(c->device));
    return CiReadMargin(c, min_margin, near_alpha);
}
bool CiPairsRecorded(const fbn_ci_ctx *c) { return c->pairs_recorded; }
void CiSetPairsRecorded(fbn_ci_ctx *c) {
    c->pair_mode = 2;
    c->pairs_recorded = true;
}
// A PC run's level 1 (group size 1) entirely on the device: ci_bits.hip's ci_l1_* kernels keep every
// edge's search state in device memory, generate each round's tests from the adjacency, count them
// from the bit-sliced store + pair tables, decide and resolve each edge's prefix in order; the host
// enqueues rounds (next chunk x4, FBN_PC_ROUND0 / FBN_PC_GROWTH as the host driver) and reads one
// open-edge count per round, one round behind, to stop.  Results equal the host driver's: the same
// tests in the same per-edge order and the same first-independent rule.  *done = false when not
// eligible (the host driver runs the level).
// Rounds are unbounded: the per-round open count lives in a two-entry ring (round r writes entry
// r & 1, the host reads round r - 1's entry while round r runs).  The per-edge chunk is clamped so
// a round's exclusive scan of the lengths (int32 offsets, hipcub) cannot overflow: E * chunk < 2^31.
constexpr int kL1Ring = 2;
int CiLevel1Device(fbn_ci_ctx *c, double alpha, const std::vector<std::vector<int>> &adj,
                   const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, LevelOut &out,
                   PCResultHost &res, bool *done) {
    *done = false;
    if (c->pair_mode != 2 || !c->pairs_recorded || !c->bits_ready || getenv("FBN_PC_HOST_L1")) return FBN_OK;
    const int nv = c->nvars;
    for (int v = 0; v < nv; ++v)
        if (c->dims[v] > 4) return FBN_OK;
    const int E = (int)(e_end - e_begin);
    int64_t cands = 0;  // every candidate set of the range: the most one round could hold
    for (size_t e = e_begin; e < e_end; ++e) cands += adj[edges[e].first].size() + adj[edges[e].second].size() - 2;
    // a level the host driver takes in one round (full speculation, ALARM-size) stays there: one
    // launch instead of a round's seven
    if (cands <= EnvOr0("FBN_PC_FULLSPEC", 16384)) return FBN_OK;
    if (E == 0) {
        out.removed.clear(), out.sep.clear(), out.d = 1, out.counted = out.launched = 0;
        *done = true;
        return FBN_OK;
    }
    static const bool ptiming = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    auto tq0 = std::chrono::steady_clock::now();
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    static thread_local std::vector<int32_t> adjf, adj_off;  // (capacity kept across runs)
    adjf.clear();
    adj_off.assign(nv + 1, 0);
    for (int u = 0; u < nv; ++u) {
        adj_off[u] = (int32_t)adjf.size();
        adjf.insert(adjf.end(), adj[u].begin(), adj[u].end());
    }
    adj_off[nv] = (int32_t)adjf.size();
    if ((rc = c->l1pairs.ensure((size_t)E * 8)) || (rc = c->l1adj.ensure(std::max<size_t>(adjf.size(), 1) * 4)) ||
        (rc = c->l1adjoff.ensure((size_t)(nv + 1) * 4)))
        return rc;
    static_assert(sizeof(std::pair<int, int>) == 8, "pair layout");
    FBN_HIP(hipMemcpyAsync(c->l1pairs.p, edges.data() + e_begin, (size_t)E * 8, hipMemcpyHostToDevice, s));
    if (!adjf.empty()) FBN_HIP(hipMemcpyAsync(c->l1adj.p, adjf.data(), adjf.size() * 4, hipMemcpyHostToDevice, s));
    FBN_HIP(hipMemcpyAsync(c->l1adjoff.p, adj_off.data(), (size_t)(nv + 1) * 4, hipMemcpyHostToDevice, s));
    if (ptiming)
        fprintf(stderr, "  level 1 device setup (host): %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
    *done = true;
    return CiLevel1Run(c, alpha, E, cands, out, res, nullptr);
}

// The level-1 rounds over the edge list / adjacency already in c->l1pairs / l1adj / l1adjoff (E
// edges, `cands` candidate sets in all); host_work (optional) runs once, after the first round is
// enqueued, while the device works.
int CiLevel1Run(fbn_ci_ctx *c, double alpha, int E, int64_t cands, LevelOut &out, PCResultHost &res,
                const std::function<int()> &host_work) {
    const int nv = c->nvars;
    out.removed.assign(E, 0);
    out.d = 1;
    out.sep.assign(E, -1);
    out.counted = out.launched = 0;
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(cands, EnvOr0("FBN_PC_L1CAP", 1 << 19)));
    if ((rc = c->l1ed.ensure((size_t)E * fbn_ci_l1_edge_bytes())) ||
        (rc = c->l1pos.ensure((size_t)E * 4)) || (rc = c->l1st.ensure((size_t)E)) ||
        (rc = c->l1sep.ensure((size_t)E * 4)) || (rc = c->l1cnt.ensure((size_t)E * 8)) ||
        (rc = c->l1len.ensure((size_t)E * 4)) || (rc = c->l1off.ensure((size_t)E * 4)) ||
        (rc = c->l1scal.ensure(96)) || (rc = c->l1open.ensure(kL1Ring * 4)) ||
        (rc = c->l1sstat.ensure((size_t)((E + 255) / 256) * 8)) ||
        (rc = c->l1items.ensure((size_t)cap * 12)) || (rc = c->l1counts.ensure((size_t)cap * 256)) ||
        (rc = c->l1df.ensure((size_t)cap * 4)) || (rc = c->l1indep.ensure((size_t)cap)))
        return rc;
    if (!c->h_open) {
        hipError_t e = hipHostMalloc((void **)&c->h_open, kL1Ring * 4, hipHostMallocDefault);
        if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc: %s", hipGetErrorString(e));
        for (auto &ev : c->l1ev) FBN_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    const double *band = nullptr;
    int nband = 0;
    if ((rc = CiBand(c, alpha, s, &band, &nband))) return rc;
    // scalars (total, launched, rows read, scan flag, tickets; the screen's scan at + 8) and the tile
    // scan's status words (epoch 0)
    FBN_HIP(hipMemsetAsync(c->l1scal.p, 0, 96, s));
    FBN_HIP(hipMemsetAsync(c->l1sstat.p, 0, (size_t)((E + 255) / 256) * 8, s));
    // the information screen (exact; FBN_PC_NO_MISCREEN=1: every candidate runs): needs the band (a
    // decision threshold per df) and the level-0 pair tables of the complete graph
    double *mi = nullptr;
    const bool mi_from_tables = c->l1mi_covered != (int64_t)nv * (nv - 1) / 2;
    if (band && !getenv("FBN_PC_NO_MISCREEN")) {
        const long long P = (long long)nv * (nv - 1) / 2;
        if ((rc = c->l1mi.ensure((size_t)std::max<long long>(P, 1) * 8)) ||
            (rc = c->l1plist.ensure((size_t)std::max<int64_t>(cands, 1) * 4)) ||
            (rc = c->l1pcnt.ensure((size_t)E * 4)) || (rc = c->l1sstat2.ensure((size_t)((E + 255) / 256) * 8)))
            return rc;
        FBN_HIP(hipMemsetAsync(c->l1sstat2.p, 0, (size_t)((E + 255) / 256) * 8, s));
        mi = c->l1mi.as<double>();
    }
    CiSlot &S = c->slot[0];
    if (c->timing) FBN_HIP(hipEventRecord(S.ev0, s));
    long long *scal = c->l1scal.as<long long>();  // total, launched, rows read, scan flag, tickets
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(32, EnvOr0("FBN_PC_ROUND0", 8192) / E));
    // chunk x2 per round: rounds here cost a few launches, speculation costs counted tests (config 5:
    // x4 launches 430k tests for 294k counted, x2 345k)
    const int64_t growth = std::max<int64_t>(2, EnvOr0("FBN_PC_GROWTH", 2));
    // (FBN_PC_L1_MAXCHUNK: tuning -- a cap on the per-edge chunk trades speculative tests for rounds)
    const int64_t max_chunk = std::max<int64_t>(
        1, std::min<int64_t>(std::min<int64_t>(1 << 16, EnvOr0("FBN_PC_L1_MAXCHUNK", 1 << 16)), (int64_t)INT32_MAX / E));
    chunk = std::min(chunk, max_chunk);
    // the setup writes round 0's lengths and zeroes the open-count ring; each round's resolve writes
    // the next round's lengths and zeroes the other ring slot (no length kernel or memset per round)
    unsigned long long *sstat = c->l1sstat.as<unsigned long long>();
    hipError_t e = fbn_ci_l1_setup(c->l1pairs.as<int32_t>(), E, c->l1adj.as<int32_t>(), c->l1adjoff.as<int32_t>(),
                                   c->l1ed.p, c->l1pos.as<int32_t>(), c->l1st.as<uint8_t>(), c->l1sep.as<int32_t>(),
                                   c->l1cnt.as<long long>(), (int)chunk, c->l1len.as<int32_t>(),
                                   c->l1off.as<int32_t>(), c->l1open.as<unsigned>(), sstat, cap, scal, c->num_cu,
                                   c->pairtab.as<int32_t>(), mi, mi_from_tables ? 1 : 0, c->ddims.as<int32_t>(), band, nband, nv,
                                   2.0 * (double)c->N, c->l1pcnt.as<int32_t>(), c->l1plist.as<int32_t>(),
                                   c->l1sstat2.as<unsigned long long>(), scal + 8, s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci level-1 setup: %s", hipGetErrorString(e));
    static const bool l1timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    const auto tl0 = std::chrono::steady_clock::now();
    int rounds = 0;
    for (int r = 0;; ++r) {
        rounds = r + 1;
        unsigned *open_r = c->l1open.as<unsigned>() + (r & 1);
        const int64_t next_chunk = std::min<int64_t>(chunk * growth, max_chunk);
        e = fbn_ci_l1_round(c->bits.as<uint32_t>(), c->ddims.as<int32_t>(), c->brow.as<int32_t>(), c->bits_W,
                            c->l1adj.as<int32_t>(), c->pairtab.as<int32_t>(), nv, c->l1ed.p, c->l1pos.as<int32_t>(),
                            c->l1st.as<uint8_t>(), c->l1sep.as<int32_t>(), c->l1cnt.as<long long>(),
                            c->l1len.as<int32_t>(), c->l1off.as<int32_t>(), E, cap, scal, c->l1items.as<int32_t>(),
                            c->l1counts.as<int32_t>(), c->l1df.as<int32_t>(), c->l1indep.as<uint8_t>(), alpha,
                            c->stats.as<unsigned long long>(), band, nband, open_r, c->num_cu,
                            c->l1open.as<unsigned>() + ((r + 1) & 1), (int)next_chunk, sstat, (unsigned)(r + 2),
                            mi ? c->l1plist.as<int32_t>() : nullptr, s);
        if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci level-1 round: %s", hipGetErrorString(e));
        FBN_HIP(hipMemcpyAsync(c->h_open + (r & 1), open_r, 4, hipMemcpyDeviceToHost, s));
        FBN_HIP(hipEventRecord(c->l1ev[r & 1], s));
        if (r == 0 && host_work)  // (while the first round runs)
            if ((rc = host_work())) return rc;
        if (r >= 1) {  // round r - 1's open count, while round r runs
            FBN_HIP(EventWaitSpin(c->l1ev[(r - 1) & 1]));
            if (c->h_open[(r - 1) & 1] == 0) break;  // round r found nothing to do
        }
        chunk = next_chunk;
    }
    if (c->timing) FBN_HIP(hipEventRecord(S.ev1, s));
    const auto tl1 = std::chrono::steady_clock::now();
    // results straight into one pinned buffer by a kernel (zero-copy writes; no DMA copies):
    // [scalars 32 | sepsets 4E | removal flags E]
    if ((rc = PinnedEnsure(c->h_xfer, c->h_xfer_bytes, (size_t)E * 5 + 40))) return rc;
    if ((rc = c->l1part.ensure(256 * 8))) return rc;
    char *hx = static_cast<char *>(c->h_xfer);
    long long *sc = reinterpret_cast<long long *>(hx);
    int32_t *hsep = reinterpret_cast<int32_t *>(hx + 32);
    char *hrm = hx + 32 + (size_t)E * 4;
    e = fbn_ci_l1_results(c->l1st.as<uint8_t>(), c->l1sep.as<int32_t>(), c->l1cnt.as<long long>(), E, scal, hrm, hsep, sc,
                          c->l1part.as<long long>(), s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci level-1 results: %s", hipGetErrorString(e));
    FBN_HIP(hipStreamSynchronize(s));
    if (sc[3]) return SetError(FBN_ERR_HIP, "level-1 offset scan: look-back timed out");
    std::memcpy(out.sep.data(), hsep, (size_t)E * 4);
    std::memcpy(out.removed.data(), hrm, (size_t)E);
    out.counted = sc[0];
    out.launched = sc[1];
    if (l1timing)
        fprintf(stderr, "  level 1 device rounds: %d, loop %.3f ms, read-back + results %.3f ms\n", rounds,
                std::chrono::duration<double, std::milli>(tl1 - tl0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl1).count());
    if (c->timing) {
        float ms = 0.f;
        FBN_HIP(hipEventElapsedTime(&ms, S.ev0, S.ev1));
        res.kernel_s += ms * 1e-3;
    }
    res.device_bytes += sc[2] * c->bits_W * 4;
    return FBN_OK;
}

// per-variable masked Grams of a PC run's level 1: for every endpoint u of the edges [e_begin,
// e_end), G_u[a] = popcount(u_a & r_i & r_j) over u's neighbours' leading rows (upper 8 x 8 tiles),
// enqueued on the ctx stream ahead of the level's batches; their tests then gather the leading
// cells instead of counting (ci_bits_gram_triples).  Only with recorded pair tables (the rest of
// each table is derived from them) and the bit-sliced store; skipped when the Grams exceed the
// budget.
constexpr int64_t kGram1MaxBytes = (int64_t)1 << 30;
int CiTriplePrepare(fbn_ci_ctx *c, const std::vector<std::vector<int>> &adj,
                    const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, bool *ready) {
    *ready = c->triples_ready = false;
    if (c->pair_mode != 2 || !c->pairs_recorded || !c->bits_ready || getenv("FBN_CI_NO_GRAM")) return FBN_OK;
    const int nv = c->nvars;
    for (int v = 0; v < nv; ++v)
        if (c->dims[v] > 4) return FBN_OK;
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = CiLeadEnsure(c, s))) return rc;
    std::vector<char> need(nv, 0);
    for (size_t e = e_begin; e < e_end; ++e) need[edges[e].first] = need[edges[e].second] = 1;
    std::vector<int32_t> adjf, adj_off(nv + 1, 0), loff, R(nv, 0), rl;
    std::vector<long long> goff(nv, 0);
    long long gtot = 0;
    for (int u = 0; u < nv; ++u) {
        adj_off[u] = (int32_t)adjf.size();
        int r = 0;
        for (int v : adj[u]) adjf.push_back(v), loff.push_back(r), r += c->dims[v] - 1;
        R[u] = r;
        goff[u] = gtot;
        if (need[u] && adj[u].size() >= 2) gtot += (long long)(c->dims[u] - 1) * r * r;
    }
    adj_off[nv] = (int32_t)adjf.size();
    if (gtot * 4 > kGram1MaxBytes) return FBN_OK;
    const int TI = fbn_ci_gram_task_ints();
    std::vector<int32_t> tasks;
    for (int u = 0; u < nv; ++u) {
        if (!need[u] || adj[u].size() < 2 || c->dims[u] < 2 || R[u] == 0) continue;
        const int64_t base = (int64_t)rl.size(), Ru = R[u], nb = (Ru + 7) / 8;
        for (int v : adj[u])
            for (int a = 0; a + 1 < c->dims[v]; ++a) rl.push_back(c->row0_host[v] + a);
        for (int a = 0; a + 1 < c->dims[u]; ++a)
            for (int64_t bi = 0; bi < nb; ++bi)
                for (int64_t bj = bi; bj < nb; ++bj) {
                    const int64_t off = goff[u] + (a * Ru + 8 * bi) * Ru + 8 * bj;
                    const int32_t t[8] = {c->row0_host[u] + a, (int32_t)(base + 8 * bi),
                                          (int32_t)std::min<int64_t>(8, Ru - 8 * bi), (int32_t)(base + 8 * bj),
                                          (int32_t)std::min<int64_t>(8, Ru - 8 * bj),
                                          (int32_t)(uint32_t)(off & 0xffffffff), (int32_t)(off >> 32), (int32_t)Ru};
                    tasks.insert(tasks.end(), t, t + TI);
                }
    }
    if ((rc = c->g1.ensure(std::max<size_t>((size_t)gtot, 1) * 4))) return rc;
    if ((rc = c->g1tasks.ensure(std::max<size_t>(tasks.size(), 1) * 4))) return rc;
    if ((rc = c->g1rl.ensure(std::max<size_t>(rl.size(), 1) * 4))) return rc;
    if ((rc = c->g1goff.ensure((size_t)nv * 8))) return rc;
    if ((rc = c->g1R.ensure((size_t)nv * 4))) return rc;
    if ((rc = c->g1adj.ensure(std::max<size_t>(adjf.size(), 1) * 4))) return rc;
    if ((rc = c->g1adjoff.ensure((size_t)(nv + 1) * 4))) return rc;
    if ((rc = c->g1loff.ensure(std::max<size_t>(loff.size(), 1) * 4))) return rc;
    auto up = [&](DevBuf &b, const void *h, size_t bytes) -> int {
        if (bytes) FBN_HIP(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, s));
        return FBN_OK;
    };
    if ((rc = up(c->g1tasks, tasks.data(), tasks.size() * 4)) || (rc = up(c->g1rl, rl.data(), rl.size() * 4)) ||
        (rc = up(c->g1goff, goff.data(), (size_t)nv * 8)) || (rc = up(c->g1R, R.data(), (size_t)nv * 4)) ||
        (rc = up(c->g1adj, adjf.data(), adjf.size() * 4)) ||
        (rc = up(c->g1adjoff, adj_off.data(), (size_t)(nv + 1) * 4)) ||
        (rc = up(c->g1loff, loff.data(), loff.size() * 4)))
        return rc;
    hipError_t e = fbn_ci_gram(c->bits.as<uint32_t>(), c->bits_W, c->g1rl.as<int32_t>(), c->g1tasks.as<int32_t>(),
                               (long long)(tasks.size() / TI), 1, c->g1.as<int32_t>(), c->num_cu, s);
    if (e != hipSuccess) return SetError(FBN_ERR_HIP, "ci gram level 1: %s", hipGetErrorString(e));
    FBN_HIP(hipStreamSynchronize(s));  // the host vectors go out of scope
    *ready = c->triples_ready = true;
    return FBN_OK;
}
struct FlagIsZero {
    __host__ __device__ bool operator()(uint8_t f) const { return f == 0; }
};
// the pairs (i < j) of the complete graph kept (decision 0) by the last all-pairs batch (slot 0:
// pairs [t0, t0 + P)), appended to `kept` in pair order: compacted on the device, only the kept
// indices cross PCIe
int CiAllPairsKept(fbn_ci_ctx *c, int64_t t0, int64_t P, std::vector<std::pair<int, int>> &kept) {
    if (P <= 0) return FBN_OK;
    if (P > INT32_MAX) return SetError(FBN_ERR_LIMIT, "too many pairs for the kept-pair compaction");
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    CiSlot &S = c->slot[0];
    hipcub::CountingInputIterator<int32_t> in(0);
    hipcub::TransformInputIterator<bool, FlagIsZero, const uint8_t *> flags(S.indep.as<uint8_t>(), FlagIsZero());
    size_t tmp = 0;
    FBN_HIP(hipcub::DeviceSelect::Flagged(nullptr, tmp, in, flags, (int32_t *)nullptr, (int *)nullptr, (int)P, s));
    int rc;
    if ((rc = c->kepttmp.ensure(std::max<size_t>(tmp, 16) + 16)) || (rc = c->keptidx.ensure((size_t)P * 4))) return rc;
    if (!c->h_kept) {
        hipError_t e = hipHostMalloc((void **)&c->h_kept, 16, hipHostMallocDefault);
        if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc: %s", hipGetErrorString(e));
    }
    int *d_num = reinterpret_cast<int *>(c->kepttmp.as<char>() + std::max<size_t>(tmp, 16));
    FBN_HIP(hipcub::DeviceSelect::Flagged(c->kepttmp.p, tmp, in, flags, c->keptidx.as<int32_t>(), d_num, (int)P, s));
    FBN_HIP(hipMemcpyAsync(c->h_kept, d_num, 4, hipMemcpyDeviceToHost, s));
    FBN_HIP(hipStreamSynchronize(s));
    const int nk = c->h_kept[0];
    if ((rc = PinnedEnsure(c->h_xfer, c->h_xfer_bytes, (size_t)std::max(nk, 1) * 4))) return rc;
    const int32_t *idx = static_cast<const int32_t *>(c->h_xfer);
    if (nk) {
        FBN_HIP(hipMemcpyAsync(c->h_xfer, c->keptidx.p, (size_t)nk * 4, hipMemcpyDeviceToHost, s));
        FBN_HIP(hipStreamSynchronize(s));
    }
    const size_t base = kept.size();
    kept.resize(base + (size_t)nk);
    const int n = c->nvars;
    int i = 0;
    int64_t row0 = 0, row1 = n - 1;  // pair indices of row i: [row0, row1)
    for (int t = 0; t < nk; ++t) {
        const int64_t q = t0 + idx[t];
        while (q >= row1) ++i, row0 = row1, row1 += n - 1 - i;
        kept[base + t] = {i, i + 1 + (int)(q - row0)};
    }
    return FBN_OK;
}
int CiBatchWait(fbn_ci_ctx *c, int k, uint8_t *indep, int32_t *df, PCResultHost &res) {
    CiSlot &S = c->slot[k];
    const int64_t n = S.n;
    if (n == 0) return FBN_OK;
    static const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    auto t1 = std::chrono::steady_clock::now();
    FBN_HIP(EventWaitSpin(S.done));
    auto t2 = std::chrono::steady_clock::now();
    const uint8_t *h_ind = static_cast<const uint8_t *>(S.h_res);
    memcpy(indep, h_ind, (size_t)n);
    if (df && S.want_df) memcpy(df, h_ind + (((size_t)n + 3) & ~(size_t)3), (size_t)n * 4);
    if (timing)
        fprintf(stderr, "  ci batch slot %d n=%lld: wait %.1f us\n", k, (long long)n,
                std::chrono::duration<double, std::micro>(t2 - t1).count());
    float ms = 0.f;
    if (c->timing) FBN_HIP(hipEventElapsedTime(&ms, S.ev0, S.ev1));
    res.kernel_s += ms * 1e-3;
    res.device_bytes += S.last_bytes;
    S.n = 0;
    return FBN_OK;
}
int CiRunBatch(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, uint8_t *indep, int32_t *df,
               PCResultHost &res) {
    int rc = CiBatchLaunch(c, 0, items, n, d, alpha, df != nullptr);
    if (rc) return rc;
    return CiBatchWait(c, 0, indep, df, res);
}

// the device-resident search's domain: <= 64 variables of <= 4 states, group size 1.  N cap: one
// test's samples bound the workgroups' skew at a grid barrier (its spin limit is 2 s)
bool PCSmallShape(int nvars, int64_t N, const int32_t *dims, int group_size) {
    if (group_size != 1 || nvars < 2 || nvars > kSmallMaxVars || N < 1 || N > (1ll << 24) || getenv("FBN_PC_NO_SMALL"))
        return false;
    for (int v = 0; v < nvars; ++v)
        if (dims[v] < 1 || dims[v] > 4) return false;
    return true;
}
bool CiPCSmallEligible(const fbn_ci_ctx *c, int group_size) {
    return PCSmallShape(c->nvars, c->N, c->dims.data(), group_size);
}

int CiPCSmall(fbn_ci_ctx *c, double alpha, int depth, PCResultHost &res, std::vector<std::pair<int, int>> &edges,
              std::vector<std::vector<int>> &adj, int *levels, bool *handoff, bool *fellback) {
    *levels = 0;
    *handoff = false;
    *fellback = false;
    static const bool htime = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic: host phases of the call
    const auto h0 = std::chrono::steady_clock::now();
    FBN_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = CiBitsEnsure(c, s)) || (rc = CiPack2Ensure(c, s))) return rc;
    const double *band = nullptr;
    int nband = 0;
    if ((rc = CiBand(c, alpha, s, &band, &nband, kBandDfMax))) return rc;
    // the host-driven levels instead (same answer): the barrier words may be mid-phase, so they are
    // zeroed again before the next launch, and the margin log starts over for the host levels
    auto fall_back = [&](const char *why) {
        c->small_zeroed = nullptr;
        const bool quiet = getenv("FBN_PC_SMALL_FAIL") != nullptr;  // (the test knob expects it)
        if (!quiet) fprintf(stderr, "fastbn: device-resident PC search %s; host-driven levels instead\n", why);
        *fellback = true;
        return CiResetMargin(c);
    };
    static const int per_cu = [] {  // (a property of the kernel: queried once, thread-safe)
        int v = 0;
        return fbn_pc_small_occupancy(&v) == hipSuccess ? v : 0;
    }();
    if (per_cu < 1) return fall_back("has no workgroup that fits a CU");
    const int grid = c->num_cu;  // one workgroup per CU: every workgroup resident (grid barrier)
    // scratch: [zeroed: barrier words | first-independent words] [statistics slots] [pair tables]
    const size_t acc_off = (kSmallZeroBytes + 255) & ~(size_t)255;
    const size_t pt_off = acc_off + (size_t)grid * 64;
    const size_t pg_off = (pt_off + (size_t)kSmallMaxEdges * 16 * 4 + 255) & ~(size_t)255;
    const size_t dout_off = (pg_off + (size_t)kSmallMaxEdges * 8 + 255) & ~(size_t)255;
    const size_t bytes = dout_off + sizeof(PcSmallOut);
    if ((rc = c->small_scr.ensure(bytes))) return rc;
    if (!c->h_small) {  // coherent: the host polls its completion word while the kernel runs
        hipError_t e = hipHostMalloc((void **)&c->h_small, sizeof(PcSmallOut), hipHostMallocCoherent);
        if (e != hipSuccess) return SetError(FBN_ERR_NOMEM, "hipHostMalloc: %s", hipGetErrorString(e));
        c->h_small->done = 0;
    }
    PcSmallOut *out = c->h_small;
    out->status = -1;
    char *scr = c->small_scr.as<char>();
    if (c->small_zeroed != c->small_scr.p || c->small_zeroed_bytes != c->small_scr.bytes) {
        FBN_HIP(hipMemsetAsync(scr, 0, kSmallZeroBytes, s));  // barrier counters and first[] words: once
        c->small_zeroed = c->small_scr.p;
        c->small_zeroed_bytes = c->small_scr.bytes;
        c->small_phase = 0;
    }
    if (++c->small_epoch == 0) ++c->small_epoch;  // (wrapped: skip 0 -- the zeroed words' epoch)
    PcSmallArgs a{};
    a.bits = c->bits.as<uint32_t>();
    a.row0 = c->brow.as<int32_t>();
    a.rowcnt = c->browcnt.as<int32_t>();
    a.nrows = c->row0_host.back() + std::min(c->dims[c->nvars - 1], 8);
    a.W = c->bits_W;
    a.pk = c->pack2.as<uint32_t>();
    a.PW = c->pack2_W;
    a.dims = c->ddims.as<int32_t>();
    a.nvars = c->nvars;
    a.N = c->N;
    a.alpha = alpha;
    a.band = band;
    a.nband = nband;
    a.depth = depth;
    static const int spec_a = getenv("FBN_PC_SPEC_A") ? std::max(1, atoi(getenv("FBN_PC_SPEC_A"))) : 8;  // (tuning)
    a.spec_a = spec_a;
    a.bar = reinterpret_cast<unsigned *>(scr);
    a.first = reinterpret_cast<unsigned long long *>(scr + (size_t)kSmallBarWords * 4);
    a.epoch = c->small_epoch;
    a.phase_base = c->small_phase;
    a.acc = reinterpret_cast<unsigned long long *>(scr + acc_off);
    a.pairtab = reinterpret_cast<int32_t *>(scr + pt_off);
    // the level-1 information screen (exact, see ci_bits.hip; FBN_PC_NO_MISCREEN=1: off)
    a.pg2 = band && !getenv("FBN_PC_NO_MISCREEN") ? reinterpret_cast<unsigned long long *>(scr + pg_off) : nullptr;
    a.ctx_stats = c->stats.as<unsigned long long>();
    a.dout = reinterpret_cast<PcSmallOut *>(scr + dout_off);
    a.out = out;
    static const bool trace = getenv("FBN_PC_SMALL_TRACE") != nullptr;  // diagnostic
    std::vector<unsigned long long> trace_host;
    unsigned long long *h_trace = nullptr;
    DevBuf trace_dev;
    if (trace) {
        const size_t tb = (64 + 10 * 1024) * 8;
        if ((rc = trace_dev.ensure(tb))) return rc;
        FBN_HIP(hipMemsetAsync(trace_dev.p, 0, tb, s));
        a.trace = trace_dev.as<unsigned long long>();
        trace_host.assign(tb / 8, 0);
    }
    CiSlot &S = c->slot[0];
    const auto h1 = std::chrono::steady_clock::now();
    if (c->timing) FBN_HIP(hipEventRecord(S.ev0, s));
    // FBN_PC_SMALL_FAIL (test knob): "launch" = treat the launch as refused, "timeout" = a barrier
    // limit of one tick, so the first level's barrier times out in the kernel itself
    const char *force = getenv("FBN_PC_SMALL_FAIL");  // (read per call: tests set it)
    // launch: plain by default -- the grid (one workgroup per CU, occupancy checked above) is resident
    // unless other work holds CUs, and then a barrier times out (bounded spin) and the host driver
    // takes over; hipLaunchCooperativeKernel (FBN_PC_SMALL_COOP=1, read per call) refuses such a grid
    // up front but measured 12-15 us more kernel time per call (0.140 vs 0.126 ms on ALARM-5000)
    const char *coop_env = getenv("FBN_PC_SMALL_COOP");
    const bool plain = !(coop_env && atoi(coop_env) != 0);
    const bool force_launch = force && !strcmp(force, "launch");
    const long long spin = (force && !strcmp(force, "timeout")) ? 1 : 0;
    {
        const hipError_t le = force_launch ? hipErrorCooperativeLaunchTooLarge
                                           : fbn_pc_small_launch(&a, grid, spin, plain ? 0 : 1, s);
        if (le != hipSuccess) {
            (void)hipGetLastError();  // (clear the sticky launch error)
            return fall_back(hipGetErrorString(le));
        }
    }
    if (c->timing) FBN_HIP(hipEventRecord(S.ev1, s));
    const auto h2 = std::chrono::steady_clock::now();
    // wait for the kernel's completion word (written after the record) instead of a stream sync;
    // a stream sync only for the events / trace, or when the word does not come (fault, hang)
    {
        const auto t0 = std::chrono::steady_clock::now();
        bool got = false;
        for (unsigned spin = 0;; ++spin) {
            if (__atomic_load_n(&out->done, __ATOMIC_ACQUIRE) == c->small_epoch) {
                got = true;
                break;
            }
            if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) break;
        }
        if (!got || c->timing || trace) FBN_HIP(hipStreamSynchronize(s));
    }
    const auto h3 = std::chrono::steady_clock::now();
    if (trace) {
        FBN_HIP(hipMemcpy(trace_host.data(), trace_dev.p, trace_host.size() * 8, hipMemcpyDeviceToHost));
        h_trace = trace_host.data();
    }
    if (h_trace) {
        const unsigned long long t0 = h_trace[63];
        for (int d = 0; d < out->levels; ++d) {
            unsigned long long mx = 0, mn = ~0ull, smx = 0, smn = ~0ull;
            double dur = 0, dmax = 0;
            for (int b = 0; b < grid; ++b) {
                const unsigned long long v = h_trace[64 + d * 1024 + b], u = h_trace[64 + 5 * 1024 + d * 1024 + b];
                if (v) mx = std::max(mx, v), mn = std::min(mn, v);
                if (u) smx = std::max(smx, u), smn = std::min(smn, u);
                if (u && v) dur += (v - u) * 0.01, dmax = std::max(dmax, (v - u) * 0.01);
            }
            fprintf(stderr, "pc small level %d: workgroups start %.2f..%.2f us, done %.2f..%.2f us (test phase mean "
                    "%.2f max %.2f us), barrier passed %.2f us, applied %.2f us\n", d, (smn - t0) * 0.01,
                    (smx - t0) * 0.01, (mn - t0) * 0.01, (mx - t0) * 0.01, dur / grid, dmax,
                    (h_trace[8 * d + 2] - t0) * 0.01, (h_trace[8 * d + 3] - t0) * 0.01);
            const double nt = (double)std::max<unsigned long long>(1, h_trace[8 * d + 7]);
            fprintf(stderr, "    one-wave tests: %.0f, cycles per test: count %.0f, complete/margins %.0f, G2/decision %.0f\n",
                    nt, h_trace[8 * d + 4] / nt, h_trace[8 * d + 5] / nt, h_trace[8 * d + 6] / nt);
        }
    }
    if (out->status != 0) {
        // a grid barrier timed out (or no record): wait for the kernel's last workgroups, so none
        // writes into the next launch's record, then run the host levels
        FBN_HIP(hipStreamSynchronize(s));
        if (out->status != 1) return SetError(FBN_ERR_HIP, "pc small kernel: no result (status %d)", out->status);
        return fall_back("timed out at a grid barrier");
    }
    c->small_phase += (unsigned)out->levels;  // one grid barrier per completed level
    if (c->timing) {
        float ms = 0.f;
        FBN_HIP(hipEventElapsedTime(&ms, S.ev0, S.ev1));
        res.kernel_s += ms * 1e-3;
    }
    // the levels the device completed -> counts, sepsets, skeleton (edges in vec_edges order =
    // lexicographic pairs of each snapshot)
    const int n = c->nvars;
    const int L = out->levels;
    std::vector<uint64_t> prev(n);
    for (int v = 0; v < n; ++v) prev[v] = (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) & ~(1ull << v);
    std::vector<std::pair<int, int>> ledges;
    std::vector<char> rm;
    std::vector<int> sep;
    for (int d = 0; d < L; ++d) {
        ledges.clear();
        rm.clear();
        for (int x = 0; x < n; ++x)
            for (int y = x + 1; y < n; ++y)
                if ((prev[x] >> y) & 1ull) {
                    ledges.push_back({x, y});
                    rm.push_back(((out->adj[d][x] >> y) & 1ull) ? 0 : 1);
                }
        if (d == 0) {
            res.sepset.set_level0(n, rm.data());  // level 0 = the complete graph
        } else {
            sep.assign(ledges.size() * (size_t)d, -1);
            const int32_t *pool = out->pool + out->sep_off[d];
            size_t r = 0;
            for (size_t e = 0; e < ledges.size(); ++e)
                if (rm[e]) {
                    for (int j = 0; j < d; ++j) sep[e * d + j] = pool[r * d + j];
                    ++r;
                }
            if ((int64_t)r * d != (int64_t)(out->sep_off[d + 1] - out->sep_off[d]))
                return SetError(FBN_ERR_HIP, "pc small kernel: level %d sepset count mismatch", d);
            res.sepset.append_level(ledges.data(), rm.data(), sep.data(), ledges.size(), d);
        }
        res.tests_per_level.push_back(out->counted[d]);
        res.launched_per_level.push_back(out->launched[d]);
        // bytes of the 2-bit packed columns / bit-sliced rows the tests touched: (d + 2) columns of
        // N / 4 bytes per launched test (roofline accounting)
        res.device_bytes += out->launched[d] * (int64_t)(d + 2) * ((c->N + 3) / 4);
        for (int v = 0; v < n; ++v) prev[v] = out->adj[d][v];
    }
    edges.clear();
    for (int x = 0; x < n; ++x)
        for (int y = x + 1; y < n; ++y)
            if ((prev[x] >> y) & 1ull) edges.push_back({x, y});
    adj.assign(n, {});
    for (auto &e : edges) adj[e.first].push_back(e.second), adj[e.second].push_back(e.first);
    for (auto &l : adj) std::sort(l.begin(), l.end());
    *levels = L;
    *handoff = out->handoff != 0;
    if (!*handoff) {
        double m;
        memcpy(&m, &out->margin_bits, 8);
        res.min_margin = m;
        res.near_alpha = (int64_t)out->near;
        res.margin_done = true;
    }
    if (htime) {
        const auto h4 = std::chrono::steady_clock::now();
        auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::micro>(b - a).count();
        };
        fprintf(stderr, "pc small host: set-up %.1f us, launch %.1f us, wait %.1f us, record -> result %.1f us\n",
                us(h0, h1), us(h1, h2), us(h2, h3), us(h3, h4));
    }
    return FBN_OK;
}
}  // namespace fbn
