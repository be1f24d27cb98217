// pc_oracle.h -- TEST INFRASTRUCTURE: CPU restatement of the reference PC-stable skeleton search
// (src/PCStable.cpp:49-563) and its G^2 conditional-independence test (src/IndependenceTest.cpp,
// src/CellTable.cpp).  Used only as the parity checker and as bench.py's cpu_baseline "port".
//
// The p-value goes through stats::pchisq (third-party submodule lib/stats + lib/gcem, pinned
// commit unknown and absent from the snapshot, `.gitmodules:10-15`).  It is restated here as
// p = 1 - P(df/2, G^2/2), P the regularized lower incomplete gamma (series / Lentz continued
// fraction), formed as the reference forms it (1.0 - pchisq).  No
// reference test pins values at this boundary: p-values are "parity unpinned"; the counts are
// pinned by the reference's own Counts2D/Counts3D (tests/golden/alarm_s5000.ci).
#ifndef FBN_ORACLE_PC_H
#define FBN_ORACLE_PC_H

#include <cstdint>
#include <map>
#include <set>
#include <vector>

#include "bn_model.h"

namespace oracle {

struct CIResult {
    double g2 = 0;
    int df = 0;
    double p = 1;
    bool indep = true;
};

double ChiSquarePValue(double g2, int df);  // 1 - pchisq(g2, df)

// ComputeGSquareXY / ComputeGSquareXYZ (src/IndependenceTest.cpp:65-155, 295-364)
CIResult CITest(const CodedDataset &ds, int x, int y, const int *z, int d, double alpha,
                std::vector<int> *counts_out = nullptr);

struct CILogEntry {
    int level, x, y;
    std::vector<int> z;
    CIResult r;
};

struct PCResult {
    std::vector<std::pair<int, int>> edges;             // remaining skeleton edges, vec_edges order
    std::map<std::pair<int, int>, std::set<int>> sepset;  // key (min, max)
    std::vector<long long> tests_per_level;              // t=1 semantic CI-test counts
    std::vector<CILogEntry> log;                          // every executed test, in reference order
    long long num_ci_test = 0;
};

// skeleton phase of StructLearnByPCStable; group_size as `-g`
PCResult PCStableSkeleton(const CodedDataset &ds, double alpha, int depth, int group_size, bool keep_log);

}  // namespace oracle

#endif
