// jt_oracle.h -- TEST INFRASTRUCTURE: CPU restatement of the reference junction-tree path, used
// only as the parity checker (tests/, __graft_entry__.smoke()) and as bench.py's cpu_baseline
// "port".  It follows the reference operation by operation on *reduced* tables (the reference's
// own formulation), so it is an independent check of the product's masked-evidence GPU kernels.
// Parity of this restatement is pinned against the unmodified reference compiled by
// oracle/Makefile (tests/golden/alarm_*.plan/.init/.marg) and the shipped alarm_1k_pt.
#ifndef FBN_ORACLE_JT_H
#define FBN_ORACLE_JT_H

#include <cstdint>
#include <string>
#include <vector>

#include "bn_model.h"

namespace oracle {

struct PTable {  // PotentialTableBase (include/PotentialTableBase.h:21-38)
    std::vector<int> vars, dims, cum;
    std::vector<double> pot;
    int size() const { return (int)pot.size(); }
    void Rebuild();  // cum_levels + size, src/PotentialTableBase.cpp:599-607
};

struct JTree {
    BayesNet bn;
    // container order (vector_clique_ptr_container / vector_separator_ptr_container)
    std::vector<PTable> clique_init, sep_init;  // after ReorganizeTableStorage
    std::vector<int> clique_up;                 // upstream separator (-1 root)
    std::vector<std::vector<int>> clique_down;  // downstream separators, MarkLevel order
    std::vector<int> sep_up, sep_down;          // parent / child clique
    int root = -1;
    std::vector<std::vector<int>> levels;       // nodes_by_level (even: cliques, odd: seps)

    void Build(const BayesNet &net);  // JunctionTree ctor, src/JunctionTree.cpp:3-46
    void DumpPlan(const std::string &plan_path, const std::string &init_path) const;

    // one case: PredictUseJTInfer(E, ...) src/JunctionTree.cpp:1473-1502.
    // ev[v] = observed value or -1.  marg gets sum(dom) doubles (evidence nodes = 0).
    int Infer(const int8_t *ev, double *marg) const;
};

double Round7(double x);  // Round(x, 7), src/Inference.cpp:195-206

}  // namespace oracle

#endif
