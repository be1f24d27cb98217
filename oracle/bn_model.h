// bn_model.h -- TEST INFRASTRUCTURE: CPU oracle model + loaders.  Restates the reference's input
// side so the oracle does not depend on the product library:
//   * XMLBIF -> discrete nodes, parents, CPT counts   (src/XMLBIFParser.cpp:33-179)
//   * CPT value (count+1)/(total+|dom|)               (src/DiscreteNode.cpp:139-161)
//   * CSV with first-appearance value coding          (src/Dataset.cpp:267-414, 549-580)
//   * LIBSVM test set -> evidence rows                (src/Dataset.cpp:162-262, src/Inference.cpp:13-42)
#ifndef FBN_ORACLE_BN_MODEL_H
#define FBN_ORACLE_BN_MODEL_H

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace oracle {

struct BayesNet {
    int n = 0;
    std::vector<std::string> names;
    std::vector<int> dom;
    std::vector<std::vector<int>> given;       // parents in <GIVEN> order
    std::vector<std::vector<int>> parents_asc;  // parents in ascending index order
    // counts[v][q * npc + pc] with pc = mixed radix over parents_asc (last fastest)
    std::vector<std::vector<long long>> counts;
    std::vector<std::vector<long long>> totals;  // totals[v][pc]

    // P(v = q | parents_asc values) exactly as DiscreteNode::GetProbability computes it
    double Prob(int v, int q, const std::vector<int> &parent_vals_asc) const;
};

// XMLBIF reader; exits the process on malformed input (the reference does the same)
BayesNet LoadXmlbif(const std::string &path);

struct CodedDataset {
    int num_vars = 0;
    int64_t num_samples = 0;
    std::vector<std::string> var_names;
    std::vector<int> dims;                 // #distinct values seen per column
    std::vector<std::vector<uint8_t>> col; // col[v][k], codes in first-appearance order
};

// LoadCSVData(path, header=true, str_val=true) semantics
CodedDataset LoadCsv(const std::string &path);

// LoadLIBSVMDataKnownNetwork + Inference ctor: evidence rows (-1 = unobserved) and labels.
// Returns ncases; ev is [ncases][num_nodes] int8.
int64_t LoadLibsvmEvidence(const std::string &path, int num_nodes, std::vector<int8_t> &ev,
                           std::vector<int> &labels);

}  // namespace oracle

#endif
