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
    marginals.assign((size_t)n * SD, 0.0);
    float kms = 0.f;
    if (gpus_ > 1 || ForceExchange()) {
        std::string e = RunSharded(&kms);
        if (!e.empty()) {
            fprintf(stderr, "Error in PredictUseJTInfer: %s\n", e.c_str());
            exit(1);
        }
    } else {
        if (fbn_jt_run(plan_, tester_->evidence.data(), n, predictions.data(), marginals.data(), nullptr))
            Die("PredictUseJTInfer");
        fbn_jt_last_kernel_ms(plan_, &kms);
    }
    if (fbn_jt_score(plan_, marginals.data(), golden.data(), n, &mse, &hd)) Die("CalculateMSE");
    std::cout << "average MSE = " << mse / n << std::endl;
    std::cout << "average HD = " << hd / n << std::endl;
    int64_t correct = 0;  // Accuracy (src/Inference.cpp:46-61)
    for (int64_t c = 0; c < n; ++c) correct += predictions[c] == tester_->ground_truths[c];
    double acc = correct / (double)n;
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "==================================================" << std::endl
              << "jt: " << s << " s (device kernel " << kms * 1e-3 << " s, " << n / (kms * 1e-3)
              << " cases/s)" << std::endl;
    return acc;
}

// Cases sharded over the GPUs: rank r takes cases [r * chunk, (r + 1) * chunk), builds
// its plan on its device from the parsed network (rank 0 reuses the constructor's), runs its shard
// from device memory, and the final gather brings every shard's labels and marginals to rank 0
// (ncclSend / ncclRecv in one group); one ncclAllReduce (max) of the kernel times.  Rank 0 then
// scores in the reference's case order, so MSE / HD / accuracy equal the one-GPU run exactly.
std::string JunctionTree::RunSharded(float *kernel_ms) {
    const int64_t n = tester_->num_instances();
    const int V = info_.num_nodes, SD = info_.sum_dom;
    GpuGroup g(gpus_, device_);
    if (!g.ok()) return g.error();
    const int world = g.size();
    const int64_t chunk = std::max<int64_t>(1, (n + world - 1) / world);
    float kmax = 0.f;
    std::string err = g.Run([&](int r) -> std::string {
        hipStream_t s = g.stream(r);
        ncclComm_t comm = g.comm(r);
        std::string e;
        fbn_jt_plan *plan = plan_;
        if (r > 0 && fbn_jt_plan_create(net_, g.device(r), &plan)) return std::string("fbn_jt_plan_create: ") + fbn_last_error();
        const int64_t c0 = std::min<int64_t>(n, r * chunk), nr = std::min<int64_t>(n, c0 + chunk) - c0;
        void *d_ev = nullptr, *d_lab = nullptr, *d_marg = nullptr, *d_k = nullptr;
        auto cleanup = [&] {
            for (void *p : {d_ev, d_lab, d_marg, d_k})
                if (p) (void)hipFree(p);
            if (r > 0) fbn_jt_plan_destroy(plan);
        };
        const size_t gathered = r == 0 ? (size_t)world : 1;  // rank 0 receives every shard
        if ((e = HipErr(hipMalloc(&d_ev, (size_t)chunk * V), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_lab, (size_t)chunk * 4 * gathered), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_marg, (size_t)chunk * SD * 8 * gathered), "hipMalloc")).size() ||
            (e = HipErr(hipMalloc(&d_k, 4), "hipMalloc")).size()) {
            cleanup();
            return e;
        }
        float ms = 0.f;
        if (nr > 0) {
            (void)hipMemcpyAsync(d_ev, tester_->evidence.data() + (size_t)c0 * V, (size_t)nr * V, hipMemcpyHostToDevice, s);
            if (fbn_jt_run_device(plan, static_cast<const int8_t *>(d_ev), nr, static_cast<int32_t *>(d_lab),
                                  static_cast<double *>(d_marg), s)) {
                e = std::string("fbn_jt_run_device: ") + fbn_last_error();
                cleanup();
                return e;
            }
            fbn_jt_last_kernel_ms(plan, &ms);
        }
        // final gather at rank 0: shard q lands at offset q * chunk
        ncclGroupStart();
        if (r == 0) {
            for (int q = 1; q < world; ++q) {
                ncclRecv(static_cast<int32_t *>(d_lab) + (size_t)q * chunk, (size_t)chunk, ncclInt32, q, comm, s);
                ncclRecv(static_cast<double *>(d_marg) + (size_t)q * chunk * SD, (size_t)chunk * SD, ncclFloat64, q,
                         comm, s);
            }
        } else {
            ncclSend(d_lab, (size_t)chunk, ncclInt32, 0, comm, s);
            ncclSend(d_marg, (size_t)chunk * SD, ncclFloat64, 0, comm, s);
        }
        if ((e = NcclErr(ncclGroupEnd(), "ncclGroupEnd (gather)")).size()) {
            cleanup();
            return e;
        }
        (void)hipMemcpyAsync(d_k, &ms, 4, hipMemcpyHostToDevice, s);
        if ((e = NcclErr(ncclAllReduce(d_k, d_k, 1, ncclFloat32, ncclMax, comm, s), "ncclAllReduce")).size()) {
            cleanup();
            return e;
        }
        if (r == 0) {
            (void)hipMemcpyAsync(predictions.data(), d_lab, (size_t)n * 4, hipMemcpyDeviceToHost, s);
            (void)hipMemcpyAsync(marginals.data(), d_marg, (size_t)n * SD * 8, hipMemcpyDeviceToHost, s);
            (void)hipMemcpyAsync(&kmax, d_k, 4, hipMemcpyDeviceToHost, s);
        }
        e = HipErr(hipStreamSynchronize(s), "gather");
        cleanup();
        return e;
    });
    if (!err.empty()) return err;
    *kernel_ms = kmax;
    std::cout << "junction tree on " << world << " GPU(s) (RCCL), " << chunk << " cases per GPU" << std::endl;
    return std::string();
}
