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
        sorted_ = sorted_ && (keys_.empty() || keys_.back() < key);
        keys_.push_back(key);
        off_.push_back((int64_t)pool_.size());
        len_.push_back(n);
        pool_.insert(pool_.end(), z, z + n);
    }
    void set(std::pair<int, int> key, const std::vector<int> &z) { set(key, z.data(), (int)z.size()); }
    bool find(std::pair<int, int> key, View *v) const {
        sort();
        auto it = std::lower_bound(keys_.begin(), keys_.end(), key);
        if (it == keys_.end() || *it != key) return false;
        const size_t i = (size_t)(it - keys_.begin());
        *v = View{pool_.data() + off_[i], len_[i]};
        return true;
    }
    size_t size() const { return keys_.size(); }  // entries appended (no sort)
    // iteration in ascending key order: n = sorted_size(), then key(i) / value(i) for i < n
    size_t sorted_size() const {
        sort();
        return keys_.size();
    }
    std::pair<int, int> key(size_t i) const { return keys_[i]; }
    View value(size_t i) const { return View{pool_.data() + off_[i], len_[i]}; }
    void reserve(size_t n) {
        keys_.reserve(n);
        off_.reserve(n);
        len_.reserve(n);
    }

  private:
    void sort() const {
        if (sorted_) return;
        // a key set twice keeps its last value (std::map assignment semantics)
        std::vector<int64_t> idx(keys_.size());
        for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int64_t)i;
        std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return keys_[a] < keys_[b]; });
        std::vector<std::pair<int, int>> k;
        std::vector<int64_t> o;
        std::vector<int> l;
        k.reserve(idx.size()), o.reserve(idx.size()), l.reserve(idx.size());
        for (int64_t i : idx) {
            if (!k.empty() && k.back() == keys_[i]) {
                o.back() = off_[i], l.back() = len_[i];
            } else {
                k.push_back(keys_[i]), o.push_back(off_[i]), l.push_back(len_[i]);
            }
        }
        keys_.swap(k), off_.swap(o), len_.swap(l);
        sorted_ = true;
    }
    mutable std::vector<std::pair<int, int>> keys_;
    mutable std::vector<int64_t> off_;
    mutable std::vector<int> len_;
    std::vector<int> pool_;
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
    int d = 0;
    std::vector<int> sep;  // [edge][d]: the sorted sepset of each removed edge of the range
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
