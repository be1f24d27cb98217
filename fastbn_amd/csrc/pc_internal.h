// pc_internal.h -- host <-> device seam of the PC-stable driver (internal to libfastbn).
#ifndef FBN_PC_INTERNAL_H
#define FBN_PC_INTERNAL_H

#include <algorithm>
#include <array>
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/fastbn.h"

namespace fbn {

// sepsets keyed by (min, max): appended per level, sorted once on first lookup / iteration (a
// node-based map cost ~40 ms of host time for the ~500k marginal removals of a 1000-variable run)
class SepsetMap {
  public:
    typedef std::pair<std::pair<int, int>, std::vector<int>> Entry;
    void set(std::pair<int, int> key, std::vector<int> z) {
        sorted_ = sorted_ && (v_.empty() || v_.back().first < key);
        v_.emplace_back(key, std::move(z));
    }
    const std::vector<int> *find(std::pair<int, int> key) const {
        sort();
        auto it = std::lower_bound(v_.begin(), v_.end(), key,
                                   [](const Entry &e, const std::pair<int, int> &k) { return e.first < k; });
        return (it != v_.end() && it->first == key) ? &it->second : nullptr;
    }
    const std::vector<Entry> &entries() const {  // ascending keys
        sort();
        return v_;
    }
    size_t size() const { return v_.size(); }
    void reserve(size_t n) { v_.reserve(n); }

  private:
    void sort() const {
        if (sorted_) return;
        // a key set twice keeps its last value (std::map assignment semantics)
        std::stable_sort(v_.begin(), v_.end(), [](const Entry &a, const Entry &b) { return a.first < b.first; });
        size_t o = 0;
        for (size_t i = 0; i < v_.size(); ++i) {
            if (o > 0 && v_[o - 1].first == v_[i].first) v_[o - 1] = std::move(v_[i]);
            else if (o != i) v_[o++] = std::move(v_[i]);
            else ++o;
        }
        v_.resize(o);
        sorted_ = true;
    }
    mutable std::vector<Entry> v_;
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
};

void CiCtxShape(const fbn_ci_ctx *c, int *nvars, int64_t *nsamples);
// run n tests of size d on the device; indep[n] (and df[n] if non-null) come back to the host;
// accumulates kernel time into res.kernel_s
int CiRunBatch(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, uint8_t *indep, int32_t *df,
               PCResultHost &res);
int RunPCStable(fbn_ci_ctx *ctx, double alpha, int depth, int group_size, PCResultHost &res);
// one level for an edge range (the unit a multi-GPU driver partitions), see pc_driver.cpp
struct LevelOut {
    std::vector<char> removed;
    std::vector<std::vector<int>> sep;
    int64_t counted = 0, launched = 0;
};
int RunLevel(fbn_ci_ctx *ctx, double alpha, int d, int group_size, const std::vector<std::vector<int>> &adj,
             const std::vector<std::pair<int, int>> &edges, size_t e_begin, size_t e_end, LevelOut &out,
             PCResultHost &res);
// orientation (pc_orient.cpp): v-structures + Meek rules 1-3 on res.edges / res.sepset
int OrientPC(int nvars, PCResultHost &res);
int LoadBifGraph(const std::string &path, std::vector<std::string> &names, std::vector<std::pair<int, int>> &arcs);
int ComputeSHD(int n, const std::vector<std::pair<int, int>> &arcs, const std::vector<std::array<int, 3>> &learned,
               int *shd, int *unlabelled);

}  // namespace fbn

#endif
