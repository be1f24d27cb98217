// JunctionTree.cpp -- see JunctionTree.h
#include "JunctionTree.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>

static void Die(const char *what) {
    fprintf(stderr, "Error in %s: %s\n", what, fbn_last_error());
    exit(1);  // the reference exits on every load/compute error
}

int TestSet::Load(const std::string &path, int n) {
    num_nodes = n;
    int64_t nc = 0;
    if (fbn_evidence_load_libsvm(path.c_str(), n, nullptr, nullptr, 0, &nc)) return -1;
    evidence.resize((size_t)nc * n);
    ground_truths.resize(nc);
    if (fbn_evidence_load_libsvm(path.c_str(), n, evidence.data(), ground_truths.data(), nc, &nc)) return -1;
    std::cout << "Finish loading data. Number of instances: " << nc << ". Number of features: " << n << ". "
              << std::endl;
    return 0;
}

JunctionTree::JunctionTree(fbn_network *net, TestSet *tester, int device) : net_(net), tester_(tester) {
    auto t0 = std::chrono::steady_clock::now();
    if (fbn_jt_plan_create(net, device, &plan_)) Die("JunctionTree");
    fbn_jt_plan_info_get(plan_, &info_);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "Finish FormJunctionTree, number of cliques = " << info_.num_cliques
              << ", number of separators = " << info_.num_separators << std::endl;
    std::cout << "Finish MarkLevel, maximum level of the junction tree = " << info_.num_levels << std::endl;
    std::cout << "==================================================" << std::endl
              << "construct jt: " << s << " s " << std::endl;
}

JunctionTree::~JunctionTree() { fbn_jt_plan_destroy(plan_); }

double JunctionTree::EvaluateAccuracy(const std::string &pt_path, int /*num_threads*/) {
    const int64_t n = tester_->num_instances();
    const int V = info_.num_nodes, SD = info_.sum_dom;
    std::vector<int32_t> dims(V);
    fbn_network_dims(net_, dims.data());
    // LoadGroundTruthProbabilityTable (src/Inference.cpp:108-146): one line per (case, node),
    // empty line = evidence node (first entry marked -1)
    std::vector<double> golden((size_t)n * SD, 0.0);
    std::ifstream in(pt_path);
    if (!in.is_open()) {
        fprintf(stderr, "Error in function LoadGroundTruthProbabilityTable!Unable to open file %s!", pt_path.c_str());
        exit(1);
    }
    std::cout << "Data file opened. Begin to load ground truth probability tables computed by JT. " << std::endl;
    std::string line;
    for (int64_t c = 0; c < n; ++c) {
        int off = 0;
        for (int v = 0; v < V; ++v) {
            std::getline(in, line);
            size_t e = line.size();
            while (e > 0 && (unsigned char)line[e - 1] < 33) --e;
            line.resize(e);
            if (line.empty()) {
                golden[c * SD + off] = -1;
            } else {
                const char *p = line.c_str();
                for (int k = 0; k < dims[v]; ++k) {
                    char *endp;
                    golden[c * SD + off + k] = strtod(p, &endp);
                    p = endp;
                }
            }
            off += dims[v];
        }
    }
    std::cout << "==================================================" << '\n'
              << "Begin testing the trained network." << std::endl;
    auto t0 = std::chrono::steady_clock::now();
    predictions.assign(n, 0);
    marginals.assign((size_t)n * SD, 0.0);
    if (fbn_jt_run(plan_, tester_->evidence.data(), n, predictions.data(), marginals.data(), nullptr))
        Die("PredictUseJTInfer");
    if (fbn_jt_score(plan_, marginals.data(), golden.data(), n, &mse, &hd)) Die("CalculateMSE");
    std::cout << "average MSE = " << mse / n << std::endl;
    std::cout << "average HD = " << hd / n << std::endl;
    int64_t correct = 0;  // Accuracy (src/Inference.cpp:46-61)
    for (int64_t c = 0; c < n; ++c) correct += predictions[c] == tester_->ground_truths[c];
    double acc = correct / (double)n;
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    float kms = 0.f;
    fbn_jt_last_kernel_ms(plan_, &kms);
    std::cout << "==================================================" << std::endl
              << "jt: " << s << " s (device kernel " << kms * 1e-3 << " s, " << n / (kms * 1e-3)
              << " cases/s)" << std::endl;
    return acc;
}
