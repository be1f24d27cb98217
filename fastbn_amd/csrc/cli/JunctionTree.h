// JunctionTree.h -- host-side mirror of the reference's JT inference API (include/JunctionTree.h:19-94,
// include/Inference.h:23-49) on top of the C-ABI.  Same constructor arguments and the same
// EvaluateAccuracy(path, num_threads) contract; the per-case loop runs on the GPU.
#ifndef FBN_CLI_JUNCTIONTREE_H
#define FBN_CLI_JUNCTIONTREE_H

#include <string>
#include <vector>

#include "fastbn.h"

struct TestSet {  // what Dataset::LoadLIBSVMDataKnownNetwork + Inference ctor extract
    int num_nodes = 0;
    std::vector<int8_t> evidence;    // [ncases][num_nodes], -1 unobserved
    std::vector<int32_t> ground_truths;
    int64_t num_instances() const { return (int64_t)ground_truths.size(); }
    int Load(const std::string &path, int num_nodes);
};

class JunctionTree {
public:
    // gpus > 1: the cases are sharded over devices device .. device + gpus - 1 (RCCL, MultiGpu.h)
    JunctionTree(fbn_network *net, TestSet *tester, int device = 0, int gpus = 1);
    ~JunctionTree();
    // LoadGroundTruthProbabilityTable + PredictUseJTInfer over all cases + Accuracy
    // (src/JunctionTree.cpp:57-129, 1508-1534).  num_threads is accepted for CLI compatibility.
    double EvaluateAccuracy(const std::string &pt_path, int num_threads);

    std::vector<int32_t> predictions;
    std::vector<double> marginals;  // [ncases][sum_dom] (one GPU; empty when sharded: they stay per rank)
    double mse = 0, hd = 0;

private:
    fbn_network *net_;
    TestSet *tester_;
    fbn_jt_plan *plan_ = nullptr;
    fbn_jt_plan_info info_{};
    int device_ = 0, gpus_ = 1;
    // PredictUseJTInfer over all cases on gpus_ devices -> predictions, sums = {MSE, HD, #correct}
    // over all cases (each rank scores its shard against `golden`); "" or an error
    std::string RunSharded(const std::vector<double> &golden, float *kernel_ms, double *sums);
};

#endif
