// pc_internal.h -- host <-> device seam of the PC-stable driver (internal to libfastbn).
#ifndef FBN_PC_INTERNAL_H
#define FBN_PC_INTERNAL_H

#include <algorithm>
#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fastbn.h"

namespace fbn {

// sepsets keyed by (min, max), flat: keys, (offset, length) into one int pool.  Appended per level,
// sorted once on first lookup / iteration (a node-based map cost ~40 ms, a vector of vectors ~3 ms,
// of host time for the ~500k marginal removals of a 1000-variable run)
class SepsetMap {
  public:
    struct View {  // the sorted sepset of one key
        const int *p;
        int n;
        const int *begin() const { return p; }
        const int *end() const { return p + n; }
        size_t size() const { return (size_t)n; }
    };
    void set(std::pair<int, int> key, const int *z, int n) {
        if (!e_.empty() && !(e_.back().key < key)) sorted_ = false, runs_.push_back(e_.size());
        e_.push_back(Ent{key, (int64_t)pool_.size(), n});
        pool_.insert(pool_.end(), z, z + n);
    }
    void set(std::pair<int, int> key, const std::vector<int> &z) { set(key, z.data(), (int)z.size()); }
    // one level's removals in one go: keys[i] for every i with removed[i], sepset sep[i*d .. +d)
    void append_level(const std::pair<int, int> *keys, const char *removed, const int *sep, size_t n, int d) {
        size_t cnt = 0;
        for (size_t i = 0; i < n; ++i) cnt += removed[i] != 0;
        size_t o = e_.size();
        e_.resize(o + cnt);
        const int64_t p0 = (int64_t)pool_.size();
        pool_.resize(pool_.size() + cnt * (size_t)d);
        int64_t q = p0;
        for (size_t i = 0; i < n; ++i) {
            if (!removed[i]) continue;
            if (o > 0 && !(e_[o - 1].key < keys[i])) sorted_ = false, runs_.push_back(o);
            e_[o++] = Ent{keys[i], q, d};
            for (int j = 0; j < d; ++j) pool_[(size_t)q + j] = sep[i * (size_t)d + j];
            q += d;
        }
    }
    // level 0 of a run over n variables: removed[k] for the k-th pair (i < j) of the complete graph
    // in lexicographic order, all with empty sepsets (a flag per pair instead of ~500k entries)
    void set_level0(int n, const char *removed) {
        n0_ = n;
        l0_.assign(removed, removed + (size_t)n * (n - 1) / 2);
    }
    void set_level0(int n, std::vector<char> &&removed) {  // takes the flags over (no copy)
        n0_ = n;
        l0_ = std::move(removed);
        l0_.resize((size_t)n * (n - 1) / 2);
    }
    // lookups need no sort: the entries are a few ascending runs (one per level), searched from the
    // last run back (a key set twice keeps its last value)
    bool find(std::pair<int, int> key, View *v) const {
        // a pair removed at level 0 is never tested again, so its flag is its only entry: checked
        // first (most absent skeleton pairs of a PC run were removed at level 0)
        if (l0_hit(key)) {
            *v = View{pool_.data(), 0};
            return true;
        }
        size_t end = e_.size();
        for (size_t r = runs_.size() + 1; r-- > 0;) {
            const size_t begin = r ? runs_[r - 1] : 0;
            auto it = std::lower_bound(e_.begin() + begin, e_.begin() + end, key,
                                       [](const Ent &a, const std::pair<int, int> &k) { return a.key < k; });
            if (it != e_.begin() + end && it->key == key) {
                *v = View{pool_.data() + it->off, it->len};
                return true;
            }
            end = begin;
        }
        return false;
    }
    // n lookups at once, answers as find() (found[i] = 0/1, v[i]): the keys are sorted and resolved
    // run by run, each search galloping forward from where the previous one ended, so it touches
    // the entries near the last hit instead of a cold binary search over the whole run
    // (orientation's v-structure pass: ~1.7k lookups on a 1000-variable run)
    void find_many(const std::pair<int, int> *keys, size_t n, View *v, char *found) const {
        // the level-0 flags first (most keys of a PC run end there), then only the rest sorted
        std::vector<uint32_t> open;
        open.reserve(n);
        for (size_t q = 0; q < n; ++q) {
            found[q] = l0_hit(keys[q]);
            if (found[q]) v[q] = View{pool_.data(), 0};
            else open.push_back((uint32_t)q);
        }
        std::sort(open.begin(), open.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
        size_t k;
        size_t end = e_.size();
        for (size_t r = runs_.size() + 1; r-- > 0 && !open.empty();) {  // last run first, as find()
            const size_t begin = r ? runs_[r - 1] : 0;
            size_t p = begin;
            k = 0;
            for (uint32_t q : open) {
                // gallop from the previous position, then binary search the last step's interval
                size_t lo = p, step = 1;
                while (lo + step < end && e_[lo + step].key < keys[q]) lo += step, step <<= 1;
                const size_t hi = std::min(end, lo + step + 1);
                auto it = std::lower_bound(e_.begin() + lo, e_.begin() + hi, keys[q],
                                           [](const Ent &a, const std::pair<int, int> &key) { return a.key < key; });
                p = (size_t)(it - e_.begin());
                if (it != e_.begin() + end && it->key == keys[q]) {
                    v[q] = View{pool_.data() + it->off, it->len};
                    found[q] = 1;
                } else {
                    open[k++] = q;
                }
            }
            open.resize(k);
            end = begin;
        }
    }
    // iteration in ascending key order: n = sorted_size(), then key(i) / value(i) for i < n (folds
    // the level-0 flags into explicit entries first)
    size_t sorted_size() const {
        if (!l0_.empty()) {
            size_t k = 0;
            for (int i = 0; i < n0_; ++i)
                for (int j = i + 1; j < n0_; ++j, ++k)
                    if (l0_[k]) {
                        if (!e_.empty() && !(e_.back().key < std::make_pair(i, j))) sorted_ = false;
                        e_.push_back(Ent{{i, j}, 0, 0});
                    }
            l0_.clear();
        }
        sort();
        return e_.size();
    }
    std::pair<int, int> key(size_t i) const { return e_[i].key; }
    View value(size_t i) const { return View{pool_.data() + e_[i].off, e_[i].len}; }

  private:
    struct Ent {
        std::pair<int, int> key;
        int64_t off;
        int len;
    };
    bool l0_hit(std::pair<int, int> key) const {
        const int i = key.first, j = key.second;
        return !l0_.empty() && 0 <= i && i < j && j < n0_ &&
               l0_[(size_t)i * n0_ - (size_t)i * (i + 1) / 2 + (size_t)(j - i - 1)];
    }
    void sort() const {
        if (sorted_) return;
        // a key set twice keeps its last value (std::map assignment semantics)
        std::stable_sort(e_.begin(), e_.end(), [](const Ent &a, const Ent &b) { return a.key < b.key; });
        size_t o = 0;
        for (size_t i = 0; i < e_.size(); ++i) {
            if (o > 0 && e_[o - 1].key == e_[i].key) e_[o - 1] = e_[i];
            else e_[o++] = e_[i];
        }
        e_.resize(o);
        sorted_ = true;
        runs_.clear();
    }
    mutable std::vector<Ent> e_;
    mutable std::vector<size_t> runs_;  // start of every ascending run after the first
    std::vector<int> pool_;
    mutable std::vector<char> l0_;
    int n0_ = 0;
    mutable bool sorted_ = true;
};

struct PCResultHost {
    std::vector<std::pair<int, int>> edges;
    SepsetMap sepset;
    std::vector<int64_t> tests_per_level;     // reference (t = 1) counts
    std::vector<int64_t> launched_per_level;  // device tests incl. speculation
    double total_s = 0.0, kernel_s = 0.0;
    int64_t device_bytes = 0;  // input bytes the CI kernels had to read, in their own column format
    // after orientation: (from, to, 1) arcs and (min, max, 0) undirected edges, vec_edges order
    std::vector<std::array<int, 3>> oriented;
    int num_nodes = 0;
    // SURVEY §8(c) decision-margin log over every test evaluated (speculative ones included)
    double min_margin = 0.0;
    int64_t near_alpha = 0;
    bool margin_done = false;  // min_margin / near_alpha already hold the run's log (device-resident run)
    // skeleton path: 0 host-driven levels, 1 device-resident search (pc_small), 2 device-resident
    // search refused at launch or timed out at a grid barrier -> host-driven levels (same answer)
    int path = 0;
};

void CiCtxShape(const fbn_ci_ctx *c, int *nvars, int64_t *nsamples);
// run n tests of size d on the device; indep[n] (and df[n] if non-null) come back to the host;
// accumulates kernel time into res.kernel_s
int CiRunBatch(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, uint8_t *indep, int32_t *df,
               PCResultHost &res);
// the same as two halves: launch a batch into slot k (0 or 1) on the ctx stream, wait for it later
// (each slot holds one batch in flight; a slot's batch must be waited for before its next launch)
// pre: the batch's largest state count and sum of state counts over all item variables, when the
// caller generated the items from valid variables (skips the validation pass); nullptr: validate
struct CiBatchStats {
    int maxdim;
    int64_t dim_rows;
};
int CiBatchLaunch(fbn_ci_ctx *c, int k, const int32_t *items, int64_t n, int d, double alpha, bool want_df,
                  const CiBatchStats *pre = nullptr);
const int32_t *CiCtxDims(const fbn_ci_ctx *c);  // state count per variable
// all nvars(nvars-1)/2 marginal tests of the complete graph (lexicographic pairs) as one batch in
// slot 0 with no item array (the kernels decode the pair); only when eligible for the bit-sliced
// path (st = the batch's statistics)
bool CiAllPairsEligible(const fbn_ci_ctx *c, const CiBatchStats &st);
// pairs [t0, t0 + n) of that order (one rank's range of a distributed level 0)
int CiBatchLaunchAllPairs(fbn_ci_ctx *c, double alpha, const CiBatchStats *pre, int64_t t0, int64_t n,
                          bool copy_flags = true);
// copy the pair tables of pairs [p0, p0 + np) (16 int32 each) out of the ctx (to_ctx = false; they
// must have been recorded) or into it (to_ctx = true); buf in device or host memory
int CiPairTablesCopy(fbn_ci_ctx *c, int64_t p0, int64_t np, void *buf, bool buf_on_device, bool to_ctx);
// every pair's table is now in the ctx (imported from all ranks): level-1 batches derive from them
void CiSetPairsRecorded(fbn_ci_ctx *c);
// whether the ctx holds pair tables of the current run (recorded by its level 0, or imported)
bool CiPairsRecorded(const fbn_ci_ctx *c);
// pair tables of the bit-sliced path: 1 = the next marginal batch records every pair's table (it
// must test all pairs i < j: a PC run's level 0), 2 = one-conditioning-variable batches derive the
// last value of x, y and z from them, 0 = off (also drops what was recorded)
void CiSetPairMode(fbn_ci_ctx *c, int mode);
// level 1 of a PC run: per-variable masked Grams for the endpoints of edges [e_begin, e_end)
// (capi.hip); a no-op when not eligible
int CiTriplePrepare(fbn_ci_ctx *c, const std::vector<std::vector<int>> &adj,
                    const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, bool *ready);
int CiBatchWait(fbn_ci_ctx *c, int k, uint8_t *indep, int32_t *df, PCResultHost &res);
int RunPCStable(fbn_ci_ctx *ctx, double alpha, int depth, int group_size, PCResultHost &res);
// The skeleton search of a small graph (<= 64 variables, every state count <= 4, group size 1) in
// ONE device launch (pc_small.hip).  Levels [0, *levels) land in res (tests and launched per level,
// sepsets) and edges / adj hold the skeleton after them; *handoff: a level the kernel does not take
// (d > 4 or > 2^22 candidate sets) follows, and the host driver continues at level *levels.  When
// the search ended on the device res.min_margin / near_alpha hold its decision-margin log.
bool CiPCSmallEligible(const fbn_ci_ctx *c, int group_size);
bool PCSmallShape(int nvars, int64_t N, const int32_t *dims, int group_size);  // (the same rule, from the shape)
// *fellback: the launch was refused or a grid barrier timed out; res / edges / adj untouched and the
// ctx's margin log reset, the caller runs the host-driven levels from level 0
int CiPCSmall(fbn_ci_ctx *c, double alpha, int depth, PCResultHost &res, std::vector<std::pair<int, int>> &edges,
              std::vector<std::vector<int>> &adj, int *levels, bool *handoff, bool *fellback);
// one level for an edge range (the unit a multi-GPU driver partitions), see pc_driver.cpp
struct LevelOut {
    std::vector<char> removed;
    int d = 0;
    std::vector<int> sep;  // [edge][d]: the sorted sepset of each removed edge of the range
    int64_t counted = 0, launched = 0;
};
// the kept pairs of the last complete-graph level-0 batch (pairs [t0, t0 + P)), appended in pair
// order, compacted on the device (capi.hip)
int CiAllPairsKept(fbn_ci_ctx *c, int64_t t0, int64_t P, std::vector<std::pair<int, int>> &kept);
// a PC run's level 1 (group size 1) on the device (capi.hip); *done = false: not eligible
int CiLevel1Device(fbn_ci_ctx *c, double alpha, const std::vector<std::vector<int>> &adj,
                   const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, LevelOut &out,
                   PCResultHost &res, bool *done);
// the level-1 rounds over an edge list / adjacency already on the device (capi.hip); host_work runs
// once while the first round is on the device
int CiLevel1Run(fbn_ci_ctx *c, double alpha, int E, int64_t cands, LevelOut &out, PCResultHost &res,
                const std::function<int()> &host_work);
// Level 0 -> level 1 without a host round trip (capi.hip): whether the ctx qualifies (level 1 would
// run on the device: pair tables recorded, bit-sliced store, every variable <= 4 states, group 1)
bool CiL0L1DeviceEligible(fbn_ci_ctx *c, int group_size);
// level 0 recorded its pair tables and the ctx uses them (pair mode 2): level 1 can run on the device
bool CiPairsReady(const fbn_ci_ctx *c);
// after CiBatchLaunchAllPairs(copy_flags = false) of the whole complete graph (P pairs): the kept
// pairs become the level-1 edge list and CSR adjacency on the device; one small read-back gives
// *E and *cands (the level's candidate sets); the decision flags and the edge list are copied to
// pinned host memory on a side stream (CiL0L1Host waits for them); accounts the level-0 batch in res
int CiL0L1Device(fbn_ci_ctx *c, int64_t P, int *E, int64_t *cands, PCResultHost &res);
// the host's copies: removed[P] (level-0 decisions), edges (lexicographic) and adj
int CiL0L1Host(fbn_ci_ctx *c, int64_t P, int E, std::vector<char> &removed, std::vector<std::pair<int, int>> &edges,
               std::vector<std::vector<int>> &adj);
// deferred (optional): host work run once while the level's first batches are on the device
int RunLevel(fbn_ci_ctx *ctx, double alpha, int d, int group_size, const std::vector<std::vector<int>> &adj,
             const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, LevelOut &out,
             PCResultHost &res, std::function<void()> *deferred = nullptr);
// removals after a level in vec_edges order + adjacency rebuild; FreeDegree > d (pc_driver.cpp)
void ApplyRemovals(const std::vector<char> &rm, std::vector<std::pair<int, int>> &edges,
                   std::vector<std::vector<int>> &adj);
bool ContinueAfter(const std::vector<std::vector<int>> &adj, int d);
// decision-margin log of a ctx (capi.hip): reset / read
int CiMarginReset(fbn_ci_ctx *c);
int CiMarginRead(fbn_ci_ctx *c, double *min_margin, int64_t *near_alpha);
// orientation (pc_orient.cpp): v-structures + Meek rules 1-3 on res.edges / res.sepset
int OrientPC(int nvars, PCResultHost &res);
int LoadBifGraph(const std::string &path, std::vector<std::string> &names, std::vector<std::pair<int, int>> &arcs);
int ComputeSHD(int n, const std::vector<std::pair<int, int>> &arcs, const std::vector<std::array<int, 3>> &learned,
               int *shd, int *unlabelled);

}  // namespace fbn

struct fbn_pc_result {
    fbn::PCResultHost r;
};

#endif
