// pc_driver.cpp -- PC-stable skeleton search driven from the host, CI tests on the device.
//
// Semantics are the reference's sequential (t = 1) ones (src/PCStable.cpp:49-563):
//   * level 0 tests every edge of the complete graph marginally;
//   * level d >= 1 works on a snapshot of the adjacencies; for edge (x, y) (x < y) the candidate
//     conditioning sets are the size-d subsets of adj(x)\{y} in ChoiceGenerator order, then those
//     of adj(y)\{x}; the first independent one removes the edge and becomes its sepset;
//   * with -g gs > 1, sets are evaluated in groups of gs per side (NextN), the whole group counts,
//     and a df == 0 result inside a group of size > 1 is a dependence (src/IndependenceTest.cpp:262-271);
//   * removals are applied after the level in vec_edges order; the search continues while
//     FreeDegree > d.
// Instead of the reference's 128-edge work pool, every unresolved edge contributes its next
// chunk of candidate sets to one device batch per round (first chunk sized so one round holds
// ~8k tests, at most 32 per edge; then x4 per round), and the host resolves each edge's prefix in
// order.  Tests beyond an edge's first independent set are
// speculative: they are run but not counted, so the reported counts equal the reference's.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>

#include "fbn_internal.h"
#include "pc_internal.h"

namespace fbn {

namespace {

constexpr int kMaxD = 8;  // CI tests take at most 8 conditioning variables (capi.hip)

// one edge's search state: the current side's candidate list is adj(a) \ {b}, read in place
// (element i = base[i + (i >= skip)]), the next combination as positions into it
struct EdgeState {
    int x, y;
    int side = 0;                // 0: adj(x)\{y}, 1: adj(y)\{x}, 2: exhausted
    const int *base = nullptr;   // adj(a), sorted
    int m = 0;                   // |adj(a) \ {b}|
    int skip = 0;                // position of b in adj(a) (m + 1 if absent)
    int ch[kMaxD];               // next combination (positions in the candidate list)
    bool has_next = false;
    int64_t pos_in_side = 0;     // index of the next combination within the side
    bool resolved = false, removed = false;
    int A(int i) const { return base[i + (i >= skip)]; }
};

void StartSide(EdgeState &e, const std::vector<std::vector<int>> &adj, int d) {
    while (e.side < 2) {
        const int a = e.side ? e.y : e.x, b = e.side ? e.x : e.y;
        const std::vector<int> &L = adj[a];
        const int pos = (int)(std::lower_bound(L.begin(), L.end(), b) - L.begin());
        const bool has_b = pos < (int)L.size() && L[pos] == b;
        e.base = L.data();
        e.m = (int)L.size() - (has_b ? 1 : 0);
        e.skip = has_b ? pos : (int)L.size() + 1;
        if (e.m >= d) {
            for (int i = 0; i < d; ++i) e.ch[i] = i;
            e.has_next = true;
            e.pos_in_side = 0;
            return;
        }
        ++e.side;
    }
    e.has_next = false;
}

void Advance(EdgeState &e, int d) {  // ChoiceGenerator::Next (src/ChoiceGenerator.cpp:55-85)
    const int m = e.m;
    int i = d - 1;
    while (i >= 0 && e.ch[i] == m - d + i) --i;
    if (i < 0) {
        e.has_next = false;
        return;
    }
    ++e.ch[i];
    for (int k = i + 1; k < d; ++k) e.ch[k] = e.ch[k - 1] + 1;
    ++e.pos_in_side;
}

// levels whose candidate sets number at most this many run in a single round; levels with fewer
// open edges than kPipelineEdges run as one half (FBN_PC_FULLSPEC / FBN_PC_PIPELINE_EDGES: test and
// diagnostic overrides, read per level)
int64_t EnvOr(const char *name, int64_t dflt) {
    const char *v = getenv(name);
    return v ? atoll(v) : dflt;
}
int64_t FullSpeculation() { return EnvOr("FBN_PC_FULLSPEC", 16384); }
constexpr int64_t kPipelineEdges = 2048;

int64_t binom(int64_t m, int k) {  // C(m, k), saturating at 2^40
    if (k < 0 || m < k) return 0;
    int64_t r = 1;
    for (int i = 1; i <= k; ++i) {
        r = r * (m - k + i) / i;
        if (r > (int64_t)1 << 40) return (int64_t)1 << 40;
    }
    return r;
}

struct Pending {  // one generated test
    int edge;
    int side;
    int64_t group_end;  // first position after this test's group (within the side)
};

}  // namespace

// One level of the skeleton search for the edges [e_begin, e_end) of `edges` (vec_edges order),
// against the adjacency snapshot `adj` (sorted lists).  Level 0: one marginal test per edge
// (src/PCStable.cpp:73-157); level d >= 1: SearchAtDepth / CheckEdge semantics (see file header).
// Outputs per edge of the range: removed flag and, if removed, its sepset (sorted).
int RunLevel(fbn_ci_ctx *ctx, double alpha, int d, int group_size, const std::vector<std::vector<int>> &adj,
             const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, LevelOut &out,
             PCResultHost &res, std::function<void()> *deferred) {
    const size_t E = e_end - e_begin;
    out.removed.assign(E, 0);
    out.d = d;
    out.sep.assign(E * (size_t)d, -1);
    out.counted = out.launched = 0;
    std::vector<int32_t> items;
    std::vector<uint8_t> indep;
    std::vector<int32_t> dfv;
    if (d == 0) {
        // the (x, y) pairs of the edge range are the items, in place (pair<int, int> = two ints)
        static_assert(sizeof(std::pair<int, int>) == 2 * sizeof(int32_t), "pair layout");
        const int32_t *pairs = reinterpret_cast<const int32_t *>(edges.data() + e_begin);
        // statistics of the pairs without the validation pass (they come from the skeleton); for
        // the whole complete graph in closed form: every variable is in nv - 1 pairs
        const int32_t *dims = CiCtxDims(ctx);
        int nv = 0;
        int64_t ns = 0;
        CiCtxShape(ctx, &nv, &ns);
        CiBatchStats st0{0, 0};
        if (e_begin == 0 && (int64_t)E == (int64_t)nv * (nv - 1) / 2 && edges.size() == E) {
            for (int v = 0; v < nv; ++v) st0.dim_rows += (int64_t)(nv - 1) * dims[v], st0.maxdim = std::max(st0.maxdim, (int)dims[v]);
        } else {
            for (size_t e = e_begin; e < e_end; ++e) {
                const int a = dims[edges[e].first], b = dims[edges[e].second];
                st0.dim_rows += a + b, st0.maxdim = std::max(st0.maxdim, std::max(a, b));
            }
        }
        // the complete graph (a PC run's level 0): edge index = pair index, the kernels decode the
        // pairs of the range themselves
        const bool all_pairs = (int64_t)edges.size() == (int64_t)nv * (nv - 1) / 2 &&
                               CiAllPairsEligible(ctx, st0) && !getenv("FBN_CI_NO_IMPLICIT");
        int rc = all_pairs ? CiBatchLaunchAllPairs(ctx, alpha, &st0, (int64_t)e_begin, (int64_t)E)
                           : CiBatchLaunch(ctx, 0, pairs, (int64_t)E, 0, alpha, false, &st0);
        if (rc) return rc;
        // the device's 0/1 decisions land in the removal flags directly
        static_assert(sizeof(char) == sizeof(uint8_t), "flag layout");
        rc = CiBatchWait(ctx, 0, reinterpret_cast<uint8_t *>(out.removed.data()), nullptr, res);
        if (rc) return rc;
        out.counted = out.launched = (int64_t)E;
        return FBN_OK;
    }
    if (d > kMaxD) return SetError(FBN_ERR_LIMIT, "conditioning set size %d (supported 0..%d)", d, kMaxD);
    if (d == 1 && group_size == 1) {  // the whole level on the device when eligible
        bool done = false;
        if (int rc = CiLevel1Device(ctx, alpha, adj, edges, e_begin, e_end, out, res, &done)) return rc;
        if (done) return FBN_OK;
    }
    // level 1 on the bit-sliced store, FBN_CI_GRAM1 = 1: per-variable Grams make every candidate
    // set's table a gather (a test then costs about its G^2 pass; FBN_PC_FULLSPEC1 = speculation
    // cap).  Off by default: config 5's Grams cover all 3.46M candidate sets (45.9 G popcount words,
    // 4.6 ms) where the rounds launch 0.39M sets (1.9 ms of derived counting).
    bool gram = false;
    if (d == 1 && getenv("FBN_CI_GRAM1") && !getenv("FBN_CI_NO_GRAM"))
        if (int rc = CiTriplePrepare(ctx, adj, edges, e_begin, e_end, &gram)) return rc;
    std::vector<EdgeState> st(E);
    for (size_t e = 0; e < E; ++e) {
        st[e].x = edges[e_begin + e].first;
        st[e].y = edges[e_begin + e].second;
        StartSide(st[e], adj, d);
        if (!st[e].has_next) st[e].resolved = true;  // both sides too small: kept
    }
    // first round: enough tests to fill the device (~8k) without speculating deep into edges
    // that usually resolve early; later rounds grow 4x per round
    int64_t open_edges = 0;
    for (auto &s : st) open_edges += !s.resolved;
    int64_t chunk = std::max<int64_t>(
        1, std::min<int64_t>(32, EnvOr("FBN_PC_ROUND0", 8192) / std::max<int64_t>(1, open_edges)));
    const int64_t growth = std::max<int64_t>(2, EnvOr("FBN_PC_GROWTH", 4));  // chunk factor per round
    bool full = false;
    // small levels: every candidate set of every edge in one round (one host round trip per level;
    // the extra speculative tests cost less than the round trips they save)
    {
        const int64_t cap = gram ? EnvOr("FBN_PC_FULLSPEC1", 16384) : FullSpeculation();
        int64_t all = 0;
        for (auto &s : st) {
            if (s.resolved) continue;
            all += binom((int64_t)adj[s.x].size() - 1, d) + binom((int64_t)adj[s.y].size() - 1, d);
            if (all > cap) break;
        }
        if (all <= cap) chunk = all, full = true;
    }
    static const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    // Two halves of the edge range, each with its own rounds, alternate on the device: while one
    // half's batch runs, the host resolves the other's results and generates its next round (the
    // device stays busy through the host work).  One half when a single round covers the level or
    // the level is small.
    struct Half {
        size_t e0, e1;
        int64_t chunk;
        std::vector<int32_t> items;
        std::vector<Pending> pend;
        std::vector<uint8_t> indep;
        std::vector<int32_t> dfv;
        CiBatchStats stats;
    };
    // (a single-round level of many candidate sets -- config-5 level 2, 8.7k -- also splits in two:
    // the second half is generated on the host while the first half's batch runs)
    const int nh = full ? (chunk >= EnvOr("FBN_PC_PIPELINE_FULL", (int64_t)4096) ? 2 : 1)
                        : (open_edges < EnvOr("FBN_PC_PIPELINE_EDGES", kPipelineEdges) ? 1 : 2);
    Half H[2];
    for (int h = 0; h < nh; ++h) H[h].e0 = E * h / nh, H[h].e1 = E * (h + 1) / nh, H[h].chunk = chunk;
    if (nh == 2) {  // cut where the candidate-set counts of the open edges reach a fraction (the
                    // first half's generation is on the critical path, the second's is not)
        std::vector<double> cost(E, 0.0);
        double tot = 0.0;
        for (size_t e = 0; e < E; ++e)
            if (!st[e].resolved)
                tot += cost[e] = (double)binom((int64_t)adj[st[e].x].size() - 1, d) +
                                 (double)binom((int64_t)adj[st[e].y].size() - 1, d);
        double acc = 0.0;
        size_t cut = 0;
        // (config 5 level 2, driver median: 50 % 3.55 ms, 25 % 3.51, 15 % 3.51, 10 % 3.49)
        static const double first = EnvOr("FBN_PC_SPLIT_PCT", 20) / 100.0;  // (tuning)
        while (cut < E && acc + cost[cut] <= tot * first) acc += cost[cut++];
        H[0].e1 = H[1].e0 = std::max<size_t>(1, std::min(cut, E - 1));
    }
    const int32_t *dims = CiCtxDims(ctx);
    auto generate = [&](Half &hf) {
        hf.items.clear();
        hf.pend.clear();
        hf.stats = CiBatchStats{0, 0};
        if (d == 1 && group_size == 1 && !getenv("FBN_PC_GEN_GENERAL")) {
            // one conditioning variable, no groups: an edge's next chunk is a contiguous slice of
            // its candidate list (with full speculation: both sides whole) -- written into arrays
            // sized up front, without per-test bookkeeping (the same tests and state transitions
            // as the general loop below)
            size_t cap = 0;
            for (size_t e = hf.e0; e < hf.e1; ++e) {
                const EdgeState &s = st[e];
                if (!s.resolved && s.has_next)
                    cap += full ? adj[s.x].size() + adj[s.y].size()
                                : (size_t)std::min<int64_t>(hf.chunk, s.m - s.ch[0]);
            }
            hf.items.resize(3 * cap);
            hf.pend.resize(cap);
            int32_t *it = hf.items.data();
            Pending *pp = hf.pend.data();
            int64_t rows = 0;
            int mx = 0;
            for (size_t e = hf.e0; e < hf.e1; ++e) {
                EdgeState &s = st[e];
                if (s.resolved) continue;
                const int dx = dims[s.x], dy = dims[s.y];
                while (s.has_next) {
                    const int cnt = (int)std::min<int64_t>(hf.chunk, s.m - s.ch[0]);
                    mx = std::max(mx, std::max(dx, dy));
                    for (int i = 0; i < cnt; ++i) {
                        const int z = s.A(s.ch[0] + i);
                        it[0] = s.x, it[1] = s.y, it[2] = z, it += 3;
                        rows += dx + dy + dims[z], mx = std::max(mx, dims[z]);
                        *pp++ = Pending{(int)e, s.side, s.pos_in_side + i + 1};
                    }
                    if (s.ch[0] + cnt == s.m) {  // side exhausted: the next side starts fresh
                        if (s.side == 0) {
                            s.side = 1;
                            StartSide(s, adj, d);
                            if (full) continue;  // one round takes every candidate set
                        } else {
                            s.side = 2;
                            s.has_next = false;
                        }
                    } else {
                        s.ch[0] += cnt;
                        s.pos_in_side += cnt;
                    }
                    break;
                }
            }
            const size_t total = (size_t)(pp - hf.pend.data());
            hf.items.resize(3 * total);
            hf.pend.resize(total);
            hf.stats = CiBatchStats{mx, rows};
            hf.chunk = std::min<int64_t>(hf.chunk * growth, 1 << 16);
            return;
        }
        if (full) {  // one round takes all `chunk` candidate sets of the level
            hf.items.reserve((size_t)chunk * (2 + d));
            hf.pend.reserve((size_t)chunk);
        }
        for (size_t e = hf.e0; e < hf.e1; ++e) {
            EdgeState &s = st[e];
            if (s.resolved) continue;
            // next chunk: whole groups only, never across a side boundary
            int64_t want = ((hf.chunk + group_size - 1) / group_size) * group_size;
            while (want > 0 && s.has_next) {
                const int64_t gstart = (s.pos_in_side / group_size) * group_size;
                hf.pend.push_back(Pending{(int)e, s.side, gstart + group_size});
                hf.items.push_back(s.x);
                hf.items.push_back(s.y);
                int r = dims[s.x] + dims[s.y], mx = std::max(dims[s.x], dims[s.y]);
                for (int i = 0; i < d; ++i) {
                    const int z = s.A(s.ch[i]);
                    hf.items.push_back(z);
                    r += dims[z], mx = std::max(mx, dims[z]);
                }
                hf.stats.dim_rows += r, hf.stats.maxdim = std::max(hf.stats.maxdim, mx);
                --want;
                Advance(s, d);
                if (!s.has_next) {
                    // side exhausted: next side starts fresh (its groups restart at 0)
                    if (s.side == 0) {
                        s.side = 1;
                        StartSide(s, adj, d);
                    } else {
                        s.side = 2;
                    }
                    // keep groups aligned: a partial chunk ends at the side boundary (not needed
                    // when the round takes every candidate set: no group is ever split)
                    if (!full) break;
                }
            }
        }
        hf.chunk = std::min<int64_t>(hf.chunk * growth, 1 << 16);
    };
    auto resolve = [&](Half &hf) {  // in order per edge
        const auto &pend = hf.pend;
        size_t i = 0;
        while (i < pend.size()) {
            const int e = pend[i].edge;
            size_t j = i;
            while (j < pend.size() && pend[j].edge == e) ++j;  // tests of this edge: [i, j)
            EdgeState &s = st[e];
            size_t k = i;
            while (k < j && !s.removed) {
                // one group: tests with the same side and group_end
                size_t g = k;
                while (g < j && pend[g].side == pend[k].side && pend[g].group_end == pend[k].group_end) ++g;
                const int gsz = (int)(g - k);
                out.counted += gsz;
                for (size_t t = k; t < g; ++t) {
                    bool ind = hf.indep[t] != 0;
                    if (gsz > 1 && hf.dfv[t] == 0) ind = false;  // group quirk (see file header)
                    if (ind) {
                        s.removed = true;
                        s.resolved = true;
                        int *z = out.sep.data() + (size_t)e * d;
                        std::copy(hf.items.begin() + (2 + d) * t + 2, hf.items.begin() + (2 + d) * (t + 1), z);
                        std::sort(z, z + d);
                        break;
                    }
                }
                k = g;
            }
            if (!s.removed && !s.has_next) s.resolved = true;  // exhausted: dependent, kept
            i = j;
        }
    };
    auto launch = [&](int h) -> int {  // generate + launch half h's next round; 0 tests = done
        auto t0 = std::chrono::steady_clock::now();
        generate(H[h]);
        const int64_t nt = (int64_t)H[h].pend.size();
        if (nt == 0) return FBN_OK;
        H[h].indep.resize(nt);
        H[h].dfv.resize(nt);
        int rc = CiBatchLaunch(ctx, h, H[h].items.data(), nt, d, alpha, true, &H[h].stats);
        if (rc) return rc;
        out.launched += nt;
        if (timing)
            fprintf(stderr, "   half %d d=%d: %lld tests, generate + launch %.2f ms\n", h, d, (long long)nt,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        return FBN_OK;
    };
    for (int h = 0; h < nh; ++h)
        if (int rc = launch(h)) return rc;
    if (deferred && *deferred) {  // (while the first batches run)
        (*deferred)();
        *deferred = nullptr;
    }
    while (true) {
        bool any = false;
        for (int h = 0; h < nh; ++h) {
            if (H[h].pend.empty()) continue;
            any = true;
            if (int rc = CiBatchWait(ctx, h, H[h].indep.data(), H[h].dfv.data(), res)) return rc;
            resolve(H[h]);
            if (int rc = launch(h)) return rc;
        }
        if (!any) break;
    }
    for (size_t e = 0; e < E; ++e)
        if (st[e].removed) out.removed[e] = 1;
    return FBN_OK;
}

void ApplyRemovals(const std::vector<char> &rm, std::vector<std::pair<int, int>> &edges,
                   std::vector<std::vector<int>> &adj) {
    // removals after a level, in vec_edges order (src/PCStable.cpp:310-326); the adjacency lists
    // are rebuilt from the kept edges in O(E) (edges stay in (i < j) lexicographic order, so every
    // list comes out sorted) instead of erasing element by element (the reference's O(E^2) hot spot)
    size_t w = 0;  // compacted in place (no second edge array)
    for (size_t e = 0; e < edges.size(); ++e)
        if (!rm[e]) edges[w++] = edges[e];
    edges.resize(w);
    for (auto &a : adj) a.clear();
    for (auto &e : edges) adj[e.first].push_back(e.second), adj[e.second].push_back(e.first);
}

bool ContinueAfter(const std::vector<std::vector<int>> &adj, int d) {  // FreeDegree (:557-563)
    size_t maxdeg = 0;
    for (auto &a : adj) maxdeg = std::max(maxdeg, a.size());
    return (int64_t)maxdeg - 1 > d;
}

int RunPCStable(fbn_ci_ctx *ctx, double alpha, int depth, int group_size, PCResultHost &res) {
    if (group_size < 1 || group_size > 8) return SetError(FBN_ERR_ARG, "group_size must be 1..8 (reference cap, src/IndependenceTest.cpp:170)");
    auto t0 = std::chrono::steady_clock::now();
    res = PCResultHost();
    int nvars = 0;
    int64_t nsamples = 0;
    CiCtxShape(ctx, &nvars, &nsamples);
    const int n = nvars;
    const int64_t P = (int64_t)n * (n - 1) / 2;
    // the edge list and adjacency lists keep their capacity from the previous run on this thread
    // (a run of config 5 otherwise allocates ~1,000 adjacency vectors before level 1: ~0.05 ms)
    static thread_local std::vector<std::pair<int, int>> edges_tls;
    static thread_local std::vector<std::vector<int>> adj_tls;
    std::vector<std::pair<int, int>> &edges = edges_tls;
    std::vector<std::vector<int>> &adj = adj_tls;
    edges.clear();
    if ((int)adj.size() > n) adj.resize(n);
    for (auto &a : adj) a.clear();
    adj.resize(n);
    std::function<void()> deferred;  // host work that waits for the next level's first batches
    const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic: host phase times per level
    // level 0 tests every pair: its tables are recorded for the level-1 kernel (derived counting)
    // and dropped when this run ends, however it ends
    struct PairModeGuard {
        fbn_ci_ctx *c;
        ~PairModeGuard() { CiSetPairMode(c, 0); }
    } pair_guard{ctx};
    const bool pairs = !getenv("FBN_CI_NO_PAIRS");
    CiSetPairMode(ctx, pairs ? 1 : 0);
    // level 0 over the implicit complete graph (the kernels decode pair indices): no edge list or
    // adjacency of the complete graph is built; the kept pairs become the skeleton directly
    const int32_t *dims = CiCtxDims(ctx);
    CiBatchStats st_all{0, 0};
    for (int v = 0; v < n; ++v) st_all.dim_rows += (int64_t)(n - 1) * dims[v], st_all.maxdim = std::max(st_all.maxdim, (int)dims[v]);
    int d0 = 0;
    bool small_done = false;  // the device-resident search ran (all levels, or the first ones)
    int small_levels = 0;
    bool small_handoff = false;
    auto ta_small = std::chrono::steady_clock::now();
    if (CiPCSmallEligible(ctx, group_size)) {
        // small graph: the whole search (or its first levels) in one device launch; refused at launch
        // or timed out at a grid barrier: the host-driven levels below (same answer)
        bool fellback = false;
        if (int rc = CiPCSmall(ctx, alpha, depth, res, edges, adj, &small_levels, &small_handoff, &fellback))
            return rc;
        res.path = fellback ? 2 : 1;
        small_done = !fellback;
    }
    if (small_done) {
        if (timing)
            fprintf(stderr, "pc device-resident levels 0-%d: %.3f ms%s\n", small_levels - 1,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta_small).count(),
                    small_handoff ? " (host continues)" : "");
        if (!small_handoff) {
            res.edges = edges;
            res.total_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            return FBN_OK;
        }
        CiSetPairMode(ctx, 0);  // the ctx recorded no pair tables: the host levels count in full
        d0 = small_levels;
    } else if (n >= 2 && CiAllPairsEligible(ctx, st_all) && !getenv("FBN_CI_NO_IMPLICIT")) {
        auto ta = std::chrono::steady_clock::now();
        const double k0 = res.kernel_s;
        std::vector<char> removed;  // (sized below on the host path only)
        static_assert(sizeof(char) == sizeof(uint8_t), "flag layout");
        // batches of at most FBN_PC_L0CHUNK pairs (per-test count records: 256 B each; a
        // 10k-variable graph has 5e7 pairs), kept pairs compacted per batch
        const int64_t chunk = std::max<int64_t>(1, EnvOr("FBN_PC_L0CHUNK", (int64_t)1 << 22));
        int rc = FBN_OK;
        double t_wait = 0, t_kept = 0;
        bool P_done = false;
        // level 0 -> level 1 without a host round trip: one complete-graph batch, whose kept pairs
        // become the level-1 edge list / adjacency on the device; the host reads back only (E, the
        // level's candidate sets) and builds its own copies (flags, edges, adjacency) while the first
        // level-1 round runs (FBN_PC_HOST_L0L1: the host path)
        if (pairs && P <= chunk && depth > 1 && CiL0L1DeviceEligible(ctx, group_size)) {
            if ((rc = CiBatchLaunchAllPairs(ctx, alpha, &st_all, 0, P, false))) return rc;
            int E = 0;
            int64_t cands = 0;
            if ((rc = CiL0L1Device(ctx, P, &E, &cands, res))) return rc;
            res.tests_per_level.push_back(P);
            res.launched_per_level.push_back(P);
            if (res.path == 0) res.path = 3;  // (2 -- a refused device-resident search -- stays)
            CiSetPairMode(ctx, 2);
            bool host_done = false;
            auto host_side = [&]() -> int {
                std::vector<char> removed;
                if (int r = CiL0L1Host(ctx, P, E, removed, edges, adj)) return r;
                res.sepset.set_level0(n, std::move(removed));
                host_done = true;
                return FBN_OK;
            };
            auto tb = std::chrono::steady_clock::now();
            if (E > 0 && CiPairsReady(ctx) && cands > EnvOr("FBN_PC_FULLSPEC", 16384)) {
                LevelOut out;
                const double k1 = res.kernel_s;
                if ((rc = CiLevel1Run(ctx, alpha, E, cands, out, res, host_side))) return rc;
                if (!host_done && (rc = host_side())) return rc;
                auto tr = std::chrono::steady_clock::now();
                res.tests_per_level.push_back(out.counted);
                res.launched_per_level.push_back(out.launched);
                // the level-1 sepsets are recorded while level 2 runs (only the orientation reads
                // them): the level-1 edge list moves aside, the kept edges (few) become `edges`
                static thread_local std::vector<std::pair<int, int>> e1_tls;
                static thread_local LevelOut l1_tls;
                e1_tls.swap(edges);
                edges.clear();
                for (size_t i = 0; i < e1_tls.size(); ++i)
                    if (!out.removed[i]) edges.push_back(e1_tls[i]);
                for (auto &a : adj) a.clear();
                for (auto &e : edges) adj[e.first].push_back(e.second), adj[e.second].push_back(e.first);
                std::swap(l1_tls, out);
                deferred = [&res]() {
                    res.sepset.append_level(e1_tls.data(), l1_tls.removed.data(), l1_tls.sep.data(), e1_tls.size(), 1);
                };
                if (timing)
                    fprintf(stderr, "  level 1 removals %.3f ms\n",
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count());
                if (timing)
                    fprintf(stderr, "pc levels 0-1 on the device: level 0 %.2f ms, level 1 %.2f ms (kernels %.2f)\n",
                            std::chrono::duration<double, std::milli>(tb - ta).count(),
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count(),
                            (res.kernel_s - k1) * 1e3);
                d0 = ContinueAfter(adj, 1) ? 2 : std::max(depth, 1);
            } else {  // level 1 (if any) on the host path
                if ((rc = host_side())) return rc;
                d0 = 1;
            }
            P_done = true;
        }
        if (!P_done) removed.resize((size_t)P);
        for (int64_t t0 = 0; t0 < P && !rc && !P_done; t0 += chunk) {
            const int64_t m = std::min(chunk, P - t0);
            auto q0 = std::chrono::steady_clock::now();
            rc = CiBatchLaunchAllPairs(ctx, alpha, &st_all, t0, m);
            if (!rc) rc = CiBatchWait(ctx, 0, reinterpret_cast<uint8_t *>(removed.data() + t0), nullptr, res);
            auto q1 = std::chrono::steady_clock::now();
            if (!rc && P > (1 << 16)) rc = CiAllPairsKept(ctx, t0, m, edges);  // compacted on the device
            auto q2 = std::chrono::steady_clock::now();
            t_wait += std::chrono::duration<double, std::milli>(q1 - q0).count();
            t_kept += std::chrono::duration<double, std::milli>(q2 - q1).count();
        }
        if (rc) return rc;
        if (!P_done) {
        auto tb = std::chrono::steady_clock::now();
        if (timing) fprintf(stderr, "pc level 0: launch + wait %.3f ms, kept pairs %.3f ms\n", t_wait, t_kept);
        res.tests_per_level.push_back(P);
        res.launched_per_level.push_back(P);
        if (P <= (1 << 16)) {  // small graphs: a host pass over the flags costs less than the round trip
            int64_t k = 0;
            for (int i = 0; i < n; ++i)
                for (int j = i + 1; j < n; ++j, ++k)
                    if (!removed[k]) edges.push_back({i, j});
        }
        res.sepset.set_level0(n, std::move(removed));
        {  // adjacency lists sized first (one allocation per variable)
            std::vector<int> deg(n, 0);
            for (auto &e : edges) ++deg[e.first], ++deg[e.second];
            for (int v = 0; v < n; ++v) adj[v].reserve(deg[v]);
        }
        for (auto &e : edges) adj[e.first].push_back(e.second), adj[e.second].push_back(e.first);
        if (pairs) CiSetPairMode(ctx, 2);
        if (timing)
            fprintf(stderr, "pc level 0 (implicit): run %.2f ms (kernels %.2f), skeleton %.2f ms\n",
                    std::chrono::duration<double, std::milli>(tb - ta).count(), (res.kernel_s - k0) * 1e3,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
        d0 = 1;
        }
    } else {
        edges.reserve((size_t)P);
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) edges.push_back({i, j});
        for (int i = 0; i < n; ++i) {
            adj[i].reserve(n - 1);
            for (int j = 0; j < n; ++j)
                if (i != j) adj[i].push_back(j);
        }
    }
    for (int d = d0; d < std::max(depth, 1); ++d) {
        LevelOut out;
        auto ta = std::chrono::steady_clock::now();
        const double k0 = res.kernel_s;
        int rc = RunLevel(ctx, alpha, d, group_size, adj, edges, 0, edges.size(), out, res, &deferred);
        if (rc) return rc;
        if (deferred) deferred(), deferred = nullptr;
        auto tb = std::chrono::steady_clock::now();
        // (recording a level's sepsets on a worker thread while the next level runs measured slower:
        // config 5 4.3 -> 4.5 ms of driver time, the orientation then reads a map built on another core)
        if (d == 0) res.sepset.set_level0(n, out.removed.data());  // edges = the complete graph
        else res.sepset.append_level(edges.data(), out.removed.data(), out.sep.data(), edges.size(), d);
        res.tests_per_level.push_back(out.counted);
        res.launched_per_level.push_back(out.launched);
        ApplyRemovals(out.removed, edges, adj);
        auto tc = std::chrono::steady_clock::now();
        if (d == 0 && pairs) CiSetPairMode(ctx, 2);
        auto td = std::chrono::steady_clock::now();
        if (timing)
            fprintf(stderr, "pc level %d: run %.2f ms (kernels %.2f), sepsets + removals %.2f ms, %.2f ms\n", d,
                    std::chrono::duration<double, std::milli>(tb - ta).count(), (res.kernel_s - k0) * 1e3,
                    std::chrono::duration<double, std::milli>(tc - tb).count(),
                    std::chrono::duration<double, std::milli>(td - tc).count());
        if (d >= 1 && !ContinueAfter(adj, d)) break;
    }
    if (deferred) deferred(), deferred = nullptr;
    res.edges = edges;
    res.total_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return FBN_OK;
}

}  // namespace fbn
