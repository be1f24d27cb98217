// JunctionTree.cpp -- see JunctionTree.h
#include "JunctionTree.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>

#include "MultiGpu.h"

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

JunctionTree::JunctionTree(fbn_network *net, TestSet *tester, int device, int gpus)
    : net_(net), tester_(tester), device_(device), gpus_(gpus) {
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
    float kms = 0.f;
    int64_t correct = 0;  // Accuracy (src/Inference.cpp:46-61)
    if (gpus_ > 1 || ForceExchange()) {
        // marginals stay on the devices: every rank scores its own shard
        marginals.clear();
        double sums[3] = {0, 0, 0};
        std::string e = RunSharded(golden, &kms, sums);
        if (!e.empty()) {
            fprintf(stderr, "Error in PredictUseJTInfer: %s\n", e.c_str());
            exit(1);
        }
        mse = sums[0], hd = sums[1], correct = (int64_t)sums[2];
    } else {
        marginals.assign((size_t)n * SD, 0.0);
        if (fbn_jt_run(plan_, tester_->evidence.data(), n, predictions.data(), marginals.data(), nullptr))
            Die("PredictUseJTInfer");
        fbn_jt_last_kernel_ms(plan_, &kms);
        if (fbn_jt_score(plan_, marginals.data(), golden.data(), n, &mse, &hd)) Die("CalculateMSE");
        for (int64_t c = 0; c < n; ++c) correct += predictions[c] == tester_->ground_truths[c];
    }
    std::cout << "average MSE = " << mse / n << std::endl;
    std::cout << "average HD = " << hd / n << std::endl;
    double acc = correct / (double)n;
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "==================================================" << std::endl
              << "jt: " << s << " s (device kernel " << kms * 1e-3 << " s, " << n / (kms * 1e-3)
              << " cases/s)" << std::endl;
    return acc;
}

// Cases sharded over the GPUs: rank r takes cases [r * chunk, (r + 1) * chunk), builds
// its plan on its device from the parsed network (rank 0 reuses the constructor's), runs its shard
// from device memory and scores it there: its slice of the golden table is uploaded once and
// fbn_jt_score_terms_device forms every case's (MSE, HD) terms (CalculateMSE / HD,
// src/Inference.cpp:153-206) from the marginals in place -- no [n][sum_dom] buffer leaves a device.
// One ncclAllGather of the labels (the final gather), one of the 16-byte per-case terms and one
// ncclAllReduce (max) of the kernel times; rank 0 then adds the terms and counts the correct labels
// in case order, so MSE / HD / accuracy equal the one-GPU run bit for bit.
std::string JunctionTree::RunSharded(const std::vector<double> &golden, float *kernel_ms, double *sums) {
    const int64_t n = tester_->num_instances();
    const int V = info_.num_nodes, SD = info_.sum_dom;
    GpuGroup g(gpus_, device_);
    if (!g.ok()) return g.error();
    const int world = g.size();
    const int64_t chunk = std::max<int64_t>(1, (n + world - 1) / world);
    float kmax = 0.f;
    std::vector<int32_t> all_labels((size_t)chunk * world, -1);
    std::vector<double> all_terms((size_t)chunk * world * 2, 0.0);
    std::string err = g.Run([&](int r) -> std::string {
        hipStream_t s = g.stream(r);
        ncclComm_t comm = g.comm(r);
        std::string e;
        fbn_jt_plan *plan = plan_;
        if (r > 0 && fbn_jt_plan_create(net_, g.device(r), &plan)) return std::string("fbn_jt_plan_create: ") + fbn_last_error();
        const int64_t c0 = std::min<int64_t>(n, r * chunk), nr = std::min<int64_t>(n, c0 + chunk) - c0;
        void *d_ev = nullptr, *d_lab = nullptr, *d_all = nullptr, *d_marg = nullptr, *d_k = nullptr, *d_gold = nullptr,
             *d_terms = nullptr, *d_tall = nullptr;
        auto cleanup = [&] {
            for (void *p : {d_ev, d_lab, d_all, d_marg, d_k, d_gold, d_terms, d_tall})
                if (p) (void)hipFree(p);
            if (r > 0) fbn_jt_plan_destroy(plan);
        };
        if ((e = HipErr(hipMalloc(&d_ev, (size_t)chunk * V), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_lab, (size_t)chunk * 4), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_all, (size_t)chunk * 4 * world), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_marg, (size_t)chunk * SD * 8), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_gold, (size_t)chunk * SD * 8), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_terms, (size_t)chunk * 2 * 8), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_tall, (size_t)chunk * 2 * 8 * world), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_k, 4), "hipMalloc")).size()) {
            cleanup();
            return e;
        }
        (void)hipMemsetAsync(d_lab, 0xFF, (size_t)chunk * 4, s);  // labels past n: -1
        (void)hipMemsetAsync(d_terms, 0, (size_t)chunk * 2 * 8, s);
        float ms = 0.f;
        if (nr > 0) {
            (void)hipMemcpyAsync(d_ev, tester_->evidence.data() + (size_t)c0 * V, (size_t)nr * V, hipMemcpyHostToDevice, s);
            (void)hipMemcpyAsync(d_gold, golden.data() + (size_t)c0 * SD, (size_t)nr * SD * 8, hipMemcpyHostToDevice, s);
            if (fbn_jt_run_device(plan, static_cast<const int8_t *>(d_ev), nr, static_cast<int32_t *>(d_lab),
                                  static_cast<double *>(d_marg), s) ||
                fbn_jt_score_terms_device(plan, static_cast<const double *>(d_marg), static_cast<const double *>(d_gold),
                                          nr, static_cast<double *>(d_terms), s)) {
                e = std::string("fbn_jt_run_device / fbn_jt_score_terms_device: ") + fbn_last_error();
                cleanup();
                return e;
            }
            fbn_jt_last_kernel_ms(plan, &ms);
        }
        (void)hipMemcpyAsync(d_k, &ms, 4, hipMemcpyHostToDevice, s);
        ncclGroupStart();
        ncclAllGather(d_lab, d_all, (size_t)chunk, ncclInt32, comm, s);
        ncclAllGather(d_terms, d_tall, (size_t)chunk * 2, ncclFloat64, comm, s);
        ncclAllReduce(d_k, d_k, 1, ncclFloat32, ncclMax, comm, s);
        if ((e = NcclErr(ncclGroupEnd(), "ncclGroupEnd (gathers)")).size()) {
            cleanup();
            return e;
        }
        if (r == 0) {
            (void)hipMemcpyAsync(all_labels.data(), d_all, all_labels.size() * 4, hipMemcpyDeviceToHost, s);
            (void)hipMemcpyAsync(all_terms.data(), d_tall, all_terms.size() * 8, hipMemcpyDeviceToHost, s);
            (void)hipMemcpyAsync(&kmax, d_k, 4, hipMemcpyDeviceToHost, s);
        }
        e = HipErr(hipStreamSynchronize(s), "gather");
        cleanup();
        return e;
    });
    if (err.empty()) {  // case order, as fbn_jt_score and the reference's EvaluateAccuracy loop
        double mse = 0.0, hd = 0.0, correct = 0.0;
        for (int64_t c = 0; c < n; ++c) {
            mse += all_terms[2 * c];
            hd += all_terms[2 * c + 1];
            correct += all_labels[c] == tester_->ground_truths[c];
        }
        sums[0] = mse, sums[1] = hd, sums[2] = correct;
    }
    if (!err.empty()) return err;
    std::copy(all_labels.begin(), all_labels.begin() + n, predictions.begin());
    *kernel_ms = kmax;
    std::cout << "junction tree on " << world << " GPU(s) (RCCL), " << chunk << " cases per GPU" << std::endl;
    return std::string();
}
