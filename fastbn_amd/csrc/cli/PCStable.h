// PCStable.h -- host-side mirror of the reference's PC-stable API (include/PCStable.h:23-59,
// include/StructureLearning.h:13-25) on top of the C-ABI: PCStable(alpha, depth) +
// StructLearnCompData(dataset, group_size, num_threads, print_struct, verbose).  The skeleton
// (level-k CI sweep) runs on the GPU; results are exposed in the reference's shapes.
#ifndef FBN_CLI_PCSTABLE_H
#define FBN_CLI_PCSTABLE_H

#include <array>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "fastbn.h"

class PCStable {
public:
    // gpus > 1: the skeleton search runs on devices device .. device + gpus - 1 (RCCL, MultiGpu.h)
    PCStable(double alpha, int depth = 1000, int device = 0, int gpus = 1)
        : alpha(alpha), depth(depth), device_(device), gpus_(gpus) {}
    void StructLearnCompData(fbn_dataset *dts, int group_size, int num_threads, bool print_struct, bool verbose);

    double alpha;
    int depth;
    int64_t num_ci_test = 0;
    int64_t num_dependence_judgement = 0;
    std::vector<std::pair<int, int>> edges;         // skeleton, vec_edges order
    std::map<std::pair<int, int>, std::set<int>> sepset;
    std::vector<int64_t> tests_per_level;
    double min_margin = 0.0;  // min |p - alpha| over the run's tests
    int64_t near_alpha = 0;   // tests with |p - alpha| < 1e-9
    std::vector<std::array<int, 3>> oriented;  // after steps 2-3: (from, to, 1) / (a, b, 0)
    // BNSLComparison(ref_net, network).GetSHD() with ref_net loaded from a BIF file (src/main.cpp:39-44)
    int GetSHD(const std::string &bif_path) const;

private:
    int device_;
    int gpus_;
    int nvars_ = 0;
};

#endif
