// pc_dist.cpp -- the multi-GPU PC-stable skeleton: one session per rank (one process per GPU),
// the level bookkeeping native, one exchange step per level.
//
// Every rank holds the same skeleton (edges in vec_edges order + sorted adjacency lists) and the
// same sepset store.  Per level d:
//   fbn_pc_dist_level   the level's edges are cut into `world` contiguous ranges -- level 0 into
//                       equal chunks of the complete graph (pair index = edge index), level d >= 1
//                       by candidate-set cost C(|adj(x)|-1, d) + C(|adj(y)|-1, d) + 1 -- the same
//                       cut on every rank (deterministic, no communication);
//   fbn_pc_dist_run     this rank's range through the single-GPU level driver (RunLevel: an edge's
//                       sequential first-independent-set search stays on one rank), packed into a
//                       fixed-size int32 record;
//   (caller)            one all-gather of the records over the ranks (RCCL / gloo), and at level 0
//                       one all-gather of the pair tables so every rank keeps the derived level-1
//                       counting (fbn_pc_dist_pairs_export / _import);
//   fbn_pc_dist_apply   every rank applies all records in rank order = vec_edges order: sepsets,
//                       test counts, removals (src/PCStable.cpp:131-147, 310-326), FreeDegree stop.
// Nothing per edge crosses the C-ABI except inside the records; no Python loops per edge.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>

#include "fbn_internal.h"
#include "pc_internal.h"

using fbn::SetError;

struct fbn_pc_dist {
    int nvars = 0;
    double alpha = 0.05;
    int depth = 1000, group_size = 1;
    int d = 0;
    bool done = false;
    // level 0 works on the implicit complete graph (pair index = edge index): edges / adj are built
    // from the kept pairs after it (or materialized on demand: Complete())
    bool implicit0 = true;
    std::vector<std::pair<int, int>> edges;
    std::vector<std::vector<int>> adj;
    fbn::PCResultHost res;
    // the current level's partition (valid after fbn_pc_dist_level)
    int world = 0, rank = 0;
    std::vector<int64_t> cuts;  // world + 1
    int64_t rec_len = 0;
    bool ran = false;           // this rank's range of the current level was run / packed
    bool pairs = true;          // level 0 records pair tables (derived level-1 counting)
    bool pairs_imported = false;
    fbn_ci_ctx *ctx = nullptr;  // last context run on (pair mode / margin bookkeeping); released by
                                // the last fbn_pc_dist_apply, which snapshots its margin log
    // the last applied level's sepsets (d >= 1), appended to the store while the next level's first
    // batches run (RunLevel's deferred hook) instead of on the exchange's critical path
    bool pending = false;
    int pend_d = 0;
    std::vector<std::pair<int, int>> pend_keys;  // the level's edges before its removals
    std::vector<char> pend_rm;
    std::vector<int> pend_sep;
    double wall_s = 0.0;
    bool margin_taken = false;
    double min_margin = 0.0;
    int64_t near_alpha = 0;
};

namespace {

constexpr int kHdr = 8;  // record header: d, n, counted (2), launched (2), kernel us (2)

int64_t Binom(int64_t m, int k) {
    if (k < 0 || m < k) return 0;
    int64_t r = 1;
    for (int i = 1; i <= k; ++i) {
        r = r * (m - k + i) / i;
        if (r > (int64_t)1 << 40) return (int64_t)1 << 40;
    }
    return r;
}

void Put64(int32_t *p, int64_t v) { memcpy(p, &v, 8); }

// 8 flag bytes (any nonzero = set) -> 8 bits, byte k -> bit k: fold each byte onto its bit 0, then
// one multiply gathers the eight bit-0s into the top byte (terms land on distinct bits, no carries)
inline uint32_t PackFlags8(const uint8_t *p) {
    uint64_t x;
    memcpy(&x, p, 8);
    x |= x >> 4;
    x |= x >> 2;
    x |= x >> 1;
    x &= 0x0101010101010101ull;
    return (uint32_t)((x * 0x0102040810204080ull) >> 56);
}

// the inverse: bit k of a byte -> flag byte k (0 / 1), one table row per byte value
struct FlagSpread {
    uint64_t t[256];
    FlagSpread() {
        for (int b = 0; b < 256; ++b) {
            uint64_t v = 0;
            for (int k = 0; k < 8; ++k) v |= (uint64_t)((b >> k) & 1) << (8 * k);
            t[b] = v;
        }
    }
};
const FlagSpread kSpread;
int64_t Get64(const int32_t *p) {
    int64_t v;
    memcpy(&v, p, 8);
    return v;
}

// the complete graph's edge list and adjacency (GenerateUndirectedCompleteGraph order,
// src/Network.cpp:346-358), only when a level-0 path needs them explicitly
void Complete(fbn_pc_dist *s) {
    if (!s->implicit0) return;
    const int n = s->nvars;
    s->edges.clear();
    s->edges.reserve((size_t)n * (n - 1) / 2);
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) s->edges.push_back({i, j});
    s->adj.assign(n, {});
    for (int i = 0; i < n; ++i) {
        s->adj[i].reserve(n - 1);
        for (int j = 0; j < n; ++j)
            if (i != j) s->adj[i].push_back(j);
    }
    s->implicit0 = false;
}
void FlushSepsets(fbn_pc_dist *s) {
    if (!s->pending) return;
    s->res.sepset.append_level(s->pend_keys.data(), s->pend_rm.data(), s->pend_sep.data(), s->pend_keys.size(),
                               s->pend_d);
    s->pending = false;
}

int64_t NumEdges(const fbn_pc_dist *s) {
    return s->d == 0 && s->implicit0 ? (int64_t)s->nvars * (s->nvars - 1) / 2 : (int64_t)s->edges.size();
}

int Partition(fbn_pc_dist *s, int world) {
    const int64_t E = NumEdges(s);
    s->cuts.assign(world + 1, E);
    s->cuts[0] = 0;
    if (world == 1) {
        // one range: no cost cut
    } else if (s->d == 0) {
        const int64_t chunk = (E + world - 1) / world;
        for (int r = 1; r < world; ++r) s->cuts[r] = std::min<int64_t>(E, r * chunk);
    } else {
        std::vector<double> cum((size_t)E + 1, 0.0);
        for (int64_t e = 0; e < E; ++e) {
            const auto &ed = s->edges[(size_t)e];
            cum[e + 1] = cum[e] + (double)Binom((int64_t)s->adj[ed.first].size() - 1, s->d) +
                         (double)Binom((int64_t)s->adj[ed.second].size() - 1, s->d) + 1.0;
        }
        for (int r = 1; r < world; ++r) {
            const double target = cum[E] * r / world;
            s->cuts[r] = std::lower_bound(cum.begin(), cum.end(), target) - cum.begin();
        }
        for (int r = 1; r <= world; ++r) s->cuts[r] = std::max(s->cuts[r], s->cuts[r - 1]);
        s->cuts[world] = E;
    }
    int64_t maxe = 0;
    for (int r = 0; r < world; ++r) maxe = std::max(maxe, s->cuts[r + 1] - s->cuts[r]);
    // level 0: one removal bit per pair (32 per int); level d: removal flag + sepset per edge
    s->rec_len = kHdr + (s->d == 0 ? (maxe + 31) / 32 : maxe * (1 + s->d));
    return FBN_OK;
}

int Pack(fbn_pc_dist *s, const uint8_t *removed, const int32_t *sep, int64_t counted, int64_t launched,
         double kernel_s, int32_t *rec) {
    const int64_t b = s->cuts[s->rank], n = s->cuts[s->rank + 1] - b;
    const int d = s->d;
    memset(rec, 0xFF, (size_t)s->rec_len * 4);
    rec[0] = d;
    rec[1] = (int32_t)n;
    Put64(rec + 2, counted);
    Put64(rec + 4, launched);
    Put64(rec + 6, (int64_t)std::llround(kernel_s * 1e9));  // ns
    int32_t *p = rec + kHdr;
    if (d == 0) {
        const int64_t full = n / 32;
        for (int64_t w = 0; w < full; ++w) {
            const uint8_t *q = removed + 32 * w;
            p[w] = (int32_t)(PackFlags8(q) | PackFlags8(q + 8) << 8 | PackFlags8(q + 16) << 16 | PackFlags8(q + 24) << 24);
        }
        if (n % 32) {
            uint32_t bits = 0;
            for (int64_t k = 0; 32 * full + k < n; ++k) bits |= (uint32_t)(removed[32 * full + k] != 0) << k;
            p[full] = (int32_t)bits;
        }
    } else {
        for (int64_t e = 0; e < n; ++e) {
            const bool rm = removed[e] != 0;
            *p++ = rm ? 1 : 0;
            for (int j = 0; j < d; ++j) *p++ = rm && sep ? sep[e * d + j] : -1;
        }
    }
    s->ran = true;
    return FBN_OK;
}

}  // namespace

extern "C" {

int fbn_pc_dist_create(int nvars, double alpha, int depth, int group_size, fbn_pc_dist **out) {
    if (!out || nvars < 2 || depth < 1 || group_size < 1 || group_size > 8 || !(alpha >= 0.0 && alpha <= 1.0))
        return SetError(FBN_ERR_ARG, "bad argument");
    auto s = std::unique_ptr<fbn_pc_dist>(new (std::nothrow) fbn_pc_dist());
    if (!s) return SetError(FBN_ERR_NOMEM, "out of memory");
    s->nvars = nvars;
    s->alpha = alpha;
    s->depth = depth;
    s->group_size = group_size;
    s->pairs = !getenv("FBN_CI_NO_PAIRS");
    s->adj.assign(nvars, {});
    *out = s.release();
    return FBN_OK;
}

int fbn_pc_dist_level(fbn_pc_dist *s, int world, int rank, int *d, int64_t *e_begin, int64_t *e_end,
                      int64_t *record_len) {
    if (!s || world < 1 || rank < 0 || rank >= world) return SetError(FBN_ERR_ARG, "bad argument");
    if (s->done) {
        if (d) *d = -1;
        return FBN_OK;
    }
    s->world = world;
    s->rank = rank;
    s->ran = false;
    int rc = Partition(s, world);
    if (rc) return rc;
    if (d) *d = s->d;
    if (e_begin) *e_begin = s->cuts[rank];
    if (e_end) *e_end = s->cuts[rank + 1];
    if (record_len) *record_len = s->rec_len;
    return FBN_OK;
}

int fbn_pc_dist_num_edges(const fbn_pc_dist *s, int64_t *n) {
    if (!s || !n) return SetError(FBN_ERR_ARG, "null pointer");
    *n = NumEdges(s);
    return FBN_OK;
}

int fbn_pc_dist_edges(const fbn_pc_dist *s, int32_t *pairs, int64_t cap) {
    if (!s || (!pairs && cap > 0)) return SetError(FBN_ERR_ARG, "null pointer");
    const int64_t n = std::min<int64_t>(cap, NumEdges(s));
    if (s->d == 0 && s->implicit0) {  // the complete graph, decoded
        int64_t k = 0;
        for (int i = 0; i < s->nvars && k < n; ++i)
            for (int j = i + 1; j < s->nvars && k < n; ++j, ++k) pairs[2 * k] = i, pairs[2 * k + 1] = j;
        return FBN_OK;
    }
    for (int64_t i = 0; i < n; ++i) pairs[2 * i] = s->edges[i].first, pairs[2 * i + 1] = s->edges[i].second;
    return FBN_OK;
}

int fbn_pc_dist_run(fbn_pc_dist *s, fbn_ci_ctx *c, int32_t *record) {
    if (!s || !c || !record) return SetError(FBN_ERR_ARG, "null pointer");
    if (s->done || s->world == 0) return SetError(FBN_ERR_ARG, "no level in progress (fbn_pc_dist_level)");
    int nv = 0;
    int64_t ns = 0;
    fbn::CiCtxShape(c, &nv, &ns);
    if (nv != s->nvars) return SetError(FBN_ERR_ARG, "context has %d variables, the session %d", nv, s->nvars);
    auto t0 = std::chrono::steady_clock::now();
    int rc;
    if (s->d == 0) {
        if ((rc = fbn::CiMarginReset(c))) return rc;
        fbn::CiSetPairMode(c, s->pairs ? 1 : 0);
    }
    s->ctx = c;
    fbn::LevelOut out;
    fbn::PCResultHost scratch;
    const size_t b = (size_t)s->cuts[s->rank], e = (size_t)s->cuts[s->rank + 1];
    if (s->d == 0 && s->implicit0) {
        // the range of the implicit complete graph: all-pairs batches straight into the flags
        const int32_t *dims = fbn::CiCtxDims(c);
        fbn::CiBatchStats st{0, 0};
        for (int v = 0; v < nv; ++v) st.dim_rows += (int64_t)(nv - 1) * dims[v], st.maxdim = std::max(st.maxdim, (int)dims[v]);
        if (fbn::CiAllPairsEligible(c, st) && !getenv("FBN_CI_NO_IMPLICIT")) {
            std::vector<uint8_t> rm(e - b);
            const int64_t chunk = getenv("FBN_PC_L0CHUNK") ? std::max(1ll, atoll(getenv("FBN_PC_L0CHUNK"))) : (1ll << 22);
            for (int64_t t0 = (int64_t)b; t0 < (int64_t)e; t0 += chunk) {
                const int64_t m = std::min<int64_t>(chunk, (int64_t)e - t0);
                if ((rc = fbn::CiBatchLaunchAllPairs(c, s->alpha, &st, t0, m))) return rc;
                if ((rc = fbn::CiBatchWait(c, 0, rm.data() + (t0 - (int64_t)b), nullptr, scratch))) return rc;
            }
            s->res.kernel_s += scratch.kernel_s;
            s->res.device_bytes += scratch.device_bytes;
            rc = Pack(s, rm.data(), nullptr, (int64_t)(e - b), (int64_t)(e - b), scratch.kernel_s, record);
            s->wall_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            return rc;
        }
        Complete(s);
    }
    std::function<void()> deferred;
    if (s->pending) deferred = [s]() { FlushSepsets(s); };
    rc = fbn::RunLevel(c, s->alpha, s->d, s->group_size, s->adj, s->edges, b, e, out, scratch, &deferred);
    FlushSepsets(s);
    if (rc) return rc;
    s->res.kernel_s += scratch.kernel_s;
    s->res.device_bytes += scratch.device_bytes;
    std::vector<uint8_t> rm(out.removed.begin(), out.removed.end());
    rc = Pack(s, rm.data(), out.sep.data(), out.counted, out.launched, scratch.kernel_s, record);
    s->wall_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int fbn_pc_dist_pack(fbn_pc_dist *s, const uint8_t *removed, const int32_t *sepsets, int64_t counted,
                     int64_t launched, int32_t *record) {
    if (!s || !record) return SetError(FBN_ERR_ARG, "null pointer");
    if (s->done || s->world == 0) return SetError(FBN_ERR_ARG, "no level in progress (fbn_pc_dist_level)");
    const int64_t n = s->cuts[s->rank + 1] - s->cuts[s->rank];
    if (n > 0 && (!removed || (s->d > 0 && !sepsets))) return SetError(FBN_ERR_ARG, "null pointer");
    FlushSepsets(s);
    return Pack(s, removed, sepsets, counted, launched, 0.0, record);
}

int fbn_pc_dist_pairs_chunk(const fbn_pc_dist *s, int64_t *pairs_per_rank) {
    if (!s || !pairs_per_rank) return SetError(FBN_ERR_ARG, "null pointer");
    if (s->world == 0) return SetError(FBN_ERR_ARG, "no level in progress (fbn_pc_dist_level)");
    // 0 = nothing to exchange: this rank's level 0 recorded no pair tables (the bit-sliced path was
    // not eligible -- > 4 states, < 4096 samples, FBN_CI_NO_BITS -- or FBN_CI_NO_PAIRS); that depends
    // only on the dataset and the environment, so every rank of a run agrees
    if (!s->pairs || s->d != 0 || !s->ran || !s->ctx || !fbn::CiPairsRecorded(s->ctx)) {
        *pairs_per_rank = 0;
        return FBN_OK;
    }
    const int64_t P = (int64_t)s->nvars * (s->nvars - 1) / 2;
    *pairs_per_rank = (P + s->world - 1) / s->world;
    return FBN_OK;
}

int fbn_pc_dist_pairs_export(fbn_pc_dist *s, void *buf, int buf_on_device) {
    if (!s || !buf) return SetError(FBN_ERR_ARG, "null pointer");
    if (s->d != 0 || !s->ran || !s->ctx || !s->pairs || !fbn::CiPairsRecorded(s->ctx))
        return SetError(FBN_ERR_ARG, "pair tables exist after this rank's level-0 run only (fbn_pc_dist_pairs_chunk = 0)");
    const int64_t b = s->cuts[s->rank], n = s->cuts[s->rank + 1] - b;
    return fbn::CiPairTablesCopy(s->ctx, b, n, buf, buf_on_device != 0, false);
}

int fbn_pc_dist_pairs_import(fbn_pc_dist *s, fbn_ci_ctx *c, const void *buf, int buf_on_device) {
    if (!s || !c || !buf) return SetError(FBN_ERR_ARG, "null pointer");
    const int64_t P = (int64_t)s->nvars * (s->nvars - 1) / 2;
    int rc = fbn::CiPairTablesCopy(c, 0, P, const_cast<void *>(buf), buf_on_device != 0, true);
    if (rc) return rc;
    fbn::CiSetPairsRecorded(c);
    s->pairs_imported = true;
    s->ctx = c;
    return FBN_OK;
}

int fbn_pc_dist_apply(fbn_pc_dist *s, const int32_t *records, int *more) {
    if (!s || !records) return SetError(FBN_ERR_ARG, "null pointer");
    if (s->done || s->world == 0) return SetError(FBN_ERR_ARG, "no level in progress (fbn_pc_dist_level)");
    auto t0 = std::chrono::steady_clock::now();
    const int d = s->d, world = s->world;
    const size_t E = (size_t)NumEdges(s);
    std::vector<char> rm(E, 0);
    std::vector<int> sep(d > 0 ? E * (size_t)d : 0, -1);
    int64_t counted = 0, launched = 0;
    std::vector<int64_t> kept;  // level 0: kept pair indices, ascending
    if (d == 0) kept.reserve(E / 8 + 64);
    for (int r = 0; r < world; ++r) {
        const int32_t *rec = records + (size_t)r * s->rec_len;
        const int64_t b = s->cuts[r], n = s->cuts[r + 1] - b;
        if (rec[0] != d || rec[1] != n)
            return SetError(FBN_ERR_ARG, "record of rank %d is for level %d / %d edges, expected %d / %lld", r, rec[0],
                            rec[1], d, (long long)n);
        counted += Get64(rec + 2);
        launched += Get64(rec + 4);
        const int32_t *p = rec + kHdr;
        if (d == 0) {  // removal bits -> flags; kept pair indices collected from the zero bits
            for (int64_t w = 0; w < (n + 31) / 32; ++w) {
                const uint32_t bits = (uint32_t)p[w];
                const int cnt = (int)std::min<int64_t>(32, n - 32 * w);
                if (cnt == 32)
                    for (int q = 0; q < 4; ++q) memcpy(&rm[b + 32 * w + 8 * q], &kSpread.t[(bits >> (8 * q)) & 0xFFu], 8);
                else
                    for (int k = 0; k < cnt; ++k) rm[b + 32 * w + k] = (char)((bits >> k) & 1u);
                uint32_t m = ~bits & (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u));
                // kept pairs are sparse (~6 % on config 5): up to four per word written without a
                // data-dependent branch (a while-per-bit loop mispredicted ~2 branches per word:
                // 0.25-0.4 ms per 499,500 pairs), more by the loop
                const int c = __builtin_popcount(m);
                const int64_t base = b + 32 * w;
                if (c <= 4) {
                    const size_t at = kept.size();
                    kept.resize(at + 4);
                    int64_t *o = kept.data() + at;
#pragma GCC unroll 4
                    for (int j = 0; j < 4; ++j) {
                        o[j] = base + __builtin_ctz(m | 0x80000000u);
                        m &= m - 1;
                    }
                    kept.resize(at + c);
                } else {
                    while (m) {
                        kept.push_back(base + __builtin_ctz(m));
                        m &= m - 1;
                    }
                }
            }
            continue;
        }
        for (int64_t e = 0; e < n; ++e) {
            rm[b + e] = p[0] != 0;
            if (p[0])
                for (int j = 0; j < d; ++j) sep[(b + e) * d + j] = p[1 + j];
            p += 1 + d;
        }
    }
    static const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    auto ta = std::chrono::steady_clock::now();
    FlushSepsets(s);
    if (d == 0) s->res.sepset.set_level0(s->nvars, std::move(rm));  // edges = the complete graph (flags taken over)
    else s->pend_keys.assign(s->edges.begin(), s->edges.end());  // sepsets: FlushSepsets, below or next run
    s->res.tests_per_level.push_back(counted);
    s->res.launched_per_level.push_back(launched);
    if (d == 0) {  // the kept pairs of the complete graph, in pair order, become the skeleton
        const int n = s->nvars;
        s->edges.resize(kept.size());
        int i = 0;
        int64_t row0 = 0, row1 = n - 1;  // pair indices of row i: [row0, row1)
        for (size_t t = 0; t < kept.size(); ++t) {
            while (kept[t] >= row1) ++i, row0 = row1, row1 += n - 1 - i;
            s->edges[t] = {i, i + 1 + (int)(kept[t] - row0)};
        }
        // adjacency sized from the degrees first: one allocation per list instead of a doubling
        // chain of them (~0.2 ms for the ~30k kept pairs of a 1000-variable run)
        std::vector<int> deg(n, 0);
        for (auto &ed : s->edges) ++deg[ed.first], ++deg[ed.second];
        s->adj.resize(n);
        for (int v = 0; v < n; ++v) s->adj[v].clear(), s->adj[v].reserve(deg[v]);
        for (auto &ed : s->edges) s->adj[ed.first].push_back(ed.second), s->adj[ed.second].push_back(ed.first);
        s->implicit0 = false;
        if (timing)
            fprintf(stderr, "pc dist apply level 0: records %.3f ms, skeleton %.3f ms\n",
                    std::chrono::duration<double, std::milli>(ta - t0).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count());
    } else {
        fbn::ApplyRemovals(rm, s->edges, s->adj);
        s->pend_rm = std::move(rm);
        s->pend_sep = std::move(sep);
        s->pend_d = d;
        s->pending = true;
    }
    if (d == 0 && s->ctx) {
        // level 1 derives from pair tables only if every pair's table is in the ctx
        if (world == 1 && s->pairs) fbn::CiSetPairMode(s->ctx, 2);
        else if (!s->pairs_imported) fbn::CiSetPairMode(s->ctx, 0);
    }
    const bool cont = d + 1 < s->depth && (d == 0 || fbn::ContinueAfter(s->adj, d));
    if (cont) ++s->d;
    else s->done = true, FlushSepsets(s);
    if (!cont && s->ctx) {
        // the search is over: this rank's margin log is read and the pair tables dropped now, while
        // the ctx is certainly alive (the caller's level loop), so fbn_pc_dist_result never touches a
        // ctx the caller may already have destroyed
        int rc = fbn::CiMarginRead(s->ctx, &s->min_margin, &s->near_alpha);
        if (rc) return rc;
        fbn::CiSetPairMode(s->ctx, 0);
        s->margin_taken = true;
        s->ctx = nullptr;
    }
    s->world = 0;
    s->ran = false;
    if (more) *more = cont ? 1 : 0;
    s->wall_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return FBN_OK;
}

int fbn_pc_dist_result(fbn_pc_dist *s, fbn_pc_result **out) {
    if (!s || !out) return SetError(FBN_ERR_ARG, "null pointer");
    if (!s->done) return SetError(FBN_ERR_ARG, "the skeleton search has not finished");
    FlushSepsets(s);
    auto r = std::unique_ptr<fbn_pc_result>(new (std::nothrow) fbn_pc_result());
    if (!r) return SetError(FBN_ERR_NOMEM, "out of memory");
    r->r = s->res;
    r->r.edges = s->edges;
    r->r.total_s = s->wall_s;
    if (s->margin_taken) r->r.min_margin = s->min_margin, r->r.near_alpha = s->near_alpha;  // this rank's tests
    int rc = fbn::OrientPC(s->nvars, r->r);
    if (rc) return rc;
    *out = r.release();
    return FBN_OK;
}

int fbn_pc_dist_destroy(fbn_pc_dist *s) {
    delete s;
    return FBN_OK;
}

}  // extern "C"
