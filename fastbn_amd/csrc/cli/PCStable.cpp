// PCStable.cpp -- see PCStable.h
#include "PCStable.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "MultiGpu.h"

namespace {

struct DevMem {  // one device allocation on the calling thread's device
    void *p = nullptr;
    std::string alloc(size_t bytes) { return HipErr(hipMalloc(&p, bytes ? bytes : 1), "hipMalloc"); }
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
};

std::string FbnErr(int rc, const char *what) {
    if (rc == 0) return std::string();
    return std::string(what) + ": " + fbn_last_error();
}

// Rank 0's column store to rank r's device by ONE ncclBroadcast, adopted as rank r's CI context.
std::string BroadcastCtx(const std::vector<uint8_t> &cols, const std::vector<int32_t> &dims, int nvars,
                         int64_t nsamples, GpuGroup &g, int r, fbn_ci_ctx **ctx) {
    hipStream_t s = g.stream(r);
    std::string e;
    const size_t bytes = (size_t)nvars * nsamples;
    DevMem d_cols;
    if ((e = d_cols.alloc(bytes)).size()) return e;
    if (r == 0 && (e = HipErr(hipMemcpyAsync(d_cols.p, cols.data(), bytes, hipMemcpyHostToDevice, s),
                              "hipMemcpyAsync")).size())
        return e;
    if ((e = NcclErr(ncclBroadcast(d_cols.p, d_cols.p, bytes, ncclUint8, 0, g.comm(r), s), "ncclBroadcast")).size())
        return e;
    if ((e = HipErr(hipStreamSynchronize(s), "broadcast")).size()) return e;
    return FbnErr(fbn_ci_dataset_from_device(static_cast<const uint8_t *>(d_cols.p), nvars, nsamples, dims.data(),
                                             g.device(r), ctx),
                  "fbn_ci_dataset_from_device");
}

// Small graphs (fbn_pc_small_eligible: the one-launch device-resident search) on g.size() GPUs:
// REPLICAS -- every rank runs the whole search on its own copy of the broadcast column store, then
// ncclBroadcasts of rank 0's result record (fbn_pc_result_record: its length, then the record) and every
// rank checks its own result against it.  Five dependent levels in one 0.14 ms launch do not
// shard: cutting them over ranks would add an all-gather per level.
std::string PcReplicas(const std::vector<uint8_t> &cols, const std::vector<int32_t> &dims, int nvars,
                       int64_t nsamples, double alpha, int depth, GpuGroup &g, fbn_pc_result **out) {
    const int world = g.size();
    std::vector<fbn_pc_result *> res(world, nullptr);
    std::string err = g.Run([&](int r) -> std::string {
        hipStream_t s = g.stream(r);
        fbn_ci_ctx *ctx = nullptr;
        std::string e = BroadcastCtx(cols, dims, nvars, nsamples, g, r, &ctx);
        if (e.empty()) e = FbnErr(fbn_pc_stable(ctx, alpha, depth, 1, &res[r]), "fbn_pc_stable");
        // the record is sized by the result: rank 0's length goes out first (one int64), then the
        // record at that length.  (Every rank reaches both broadcasts, even after an error, so no
        // rank waits forever; a rank with an error sends / receives zeros and reports its own error.)
        int64_t len = 0;
        if (e.empty()) e = FbnErr(fbn_pc_result_record(res[r], nullptr, 0, &len), "fbn_pc_result_record");
        DevMem d_len;
        std::string e2 = d_len.alloc(8);
        if (e2.empty()) e2 = HipErr(hipMemcpyAsync(d_len.p, &len, 8, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        const std::string e3 = NcclErr(ncclBroadcast(d_len.p, d_len.p, 1, ncclInt64, 0, g.comm(r), s), "ncclBroadcast");
        if (e2.empty()) e2 = e3;
        int64_t len0 = 0;
        if (e2.empty()) e2 = HipErr(hipMemcpyAsync(&len0, d_len.p, 8, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
        if (e2.empty()) e2 = HipErr(hipStreamSynchronize(s), "record length");
        if (e.empty()) e = e2;
        const int64_t cap = std::max<int64_t>(len0, 1);
        std::vector<int32_t> mine((size_t)std::max(cap, len), 0), got((size_t)cap, 0);
        if (e.empty()) e = FbnErr(fbn_pc_result_record(res[r], mine.data(), (int64_t)mine.size(), nullptr),
                                  "fbn_pc_result_record");
        DevMem d_rec;
        e2 = d_rec.alloc((size_t)cap * 4);
        if (e2.empty())
            e2 = HipErr(hipMemcpyAsync(d_rec.p, mine.data(), (size_t)cap * 4, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        const std::string e4 = NcclErr(ncclBroadcast(d_rec.p, d_rec.p, (size_t)cap, ncclInt32, 0, g.comm(r), s), "ncclBroadcast");
        if (e2.empty()) e2 = e4;
        if (e.empty()) e = e2;
        if (e.empty()) e = HipErr(hipMemcpyAsync(got.data(), d_rec.p, (size_t)cap * 4, hipMemcpyDeviceToHost, s),
                                  "hipMemcpyAsync");
        if (e.empty()) e = HipErr(hipStreamSynchronize(s), "record");
        if (e.empty() && len != len0) e = "PC replicas disagree with rank 0's result record (length)";
        mine.resize((size_t)cap);
        if (e.empty() && got != mine) e = "PC replicas disagree with rank 0's result record";
        if (ctx) fbn_ci_ctx_destroy(ctx);
        return e;
    });
    for (int r = 1; r < world; ++r)
        if (res[r]) fbn_pc_result_destroy(res[r]);
    if (!err.empty()) {
        if (res[0]) fbn_pc_result_destroy(res[0]);
        return err;
    }
    *out = res[0];
    return std::string();
}

// The skeleton search on g.size() GPUs (INTEGRATION.md "Multi-GPU"): rank 0's column
// store reaches every device by ONE ncclBroadcast; each rank runs its edge range of every level
// through the native session; per level ONE ncclAllGather of the fixed-size records (level 0 also
// of the pair tables, device to device, after the ranks agree on their size with an ncclAllReduce).
// Every rank ends with the same skeleton; rank 0's result is returned.
std::string PcDistributed(const std::vector<uint8_t> &cols, const std::vector<int32_t> &dims, int nvars,
                          int64_t nsamples, double alpha, int depth, int group_size, GpuGroup &g,
                          fbn_pc_result **out) {
    const int world = g.size();
    std::vector<fbn_pc_result *> res(world, nullptr);
    std::string err = g.Run([&](int r) -> std::string {
        hipStream_t s = g.stream(r);
        ncclComm_t comm = g.comm(r);
        std::string e;
        fbn_ci_ctx *ctx = nullptr;
        if ((e = BroadcastCtx(cols, dims, nvars, nsamples, g, r, &ctx)).size()) return e;
        fbn_pc_dist *sess = nullptr;
        if ((e = FbnErr(fbn_pc_dist_create(nvars, alpha, depth, group_size, &sess), "fbn_pc_dist_create")).size()) {
            fbn_ci_ctx_destroy(ctx);
            return e;
        }
        auto body = [&]() -> std::string {
            std::string e2;
            for (;;) {
                int d = 0;
                int64_t b = 0, en = 0, L = 0;
                if ((e2 = FbnErr(fbn_pc_dist_level(sess, world, r, &d, &b, &en, &L), "fbn_pc_dist_level")).size())
                    return e2;
                if (d < 0) break;
                std::vector<int32_t> rec((size_t)L), all((size_t)L * world);
                if ((e2 = FbnErr(fbn_pc_dist_run(sess, ctx, rec.data()), "fbn_pc_dist_run")).size()) return e2;
                if (d == 0) {  // level-0 pair tables to every rank (derived level-1 counting)
                    int64_t chunk = 0;
                    if ((e2 = FbnErr(fbn_pc_dist_pairs_chunk(sess, &chunk), "fbn_pc_dist_pairs_chunk")).size())
                        return e2;
                    DevMem d_c;
                    if ((e2 = d_c.alloc(8)).size()) return e2;
                    (void)hipMemcpyAsync(d_c.p, &chunk, 8, hipMemcpyHostToDevice, s);
                    if ((e2 = NcclErr(ncclAllReduce(d_c.p, d_c.p, 1, ncclInt64, ncclMin, comm, s), "ncclAllReduce")).size())
                        return e2;
                    (void)hipMemcpyAsync(&chunk, d_c.p, 8, hipMemcpyDeviceToHost, s);
                    if ((e2 = HipErr(hipStreamSynchronize(s), "pair chunk")).size()) return e2;
                    if (chunk > 0) {
                        DevMem mine, gathered;
                        if ((e2 = mine.alloc((size_t)chunk * 64)).size() ||
                            (e2 = gathered.alloc((size_t)chunk * 64 * world)).size())
                            return e2;
                        (void)hipMemsetAsync(mine.p, 0, (size_t)chunk * 64, s);
                        if ((e2 = HipErr(hipStreamSynchronize(s), "memset")).size()) return e2;
                        if ((e2 = FbnErr(fbn_pc_dist_pairs_export(sess, mine.p, 1), "fbn_pc_dist_pairs_export")).size())
                            return e2;
                        if ((e2 = NcclErr(ncclAllGather(mine.p, gathered.p, (size_t)chunk * 16, ncclInt32, comm, s),
                                          "ncclAllGather")).size())
                            return e2;
                        if ((e2 = HipErr(hipStreamSynchronize(s), "pair tables")).size()) return e2;
                        if ((e2 = FbnErr(fbn_pc_dist_pairs_import(sess, ctx, gathered.p, 1), "fbn_pc_dist_pairs_import")).size())
                            return e2;
                    }
                }
                DevMem d_rec, d_all;
                if ((e2 = d_rec.alloc((size_t)L * 4)).size() || (e2 = d_all.alloc((size_t)L * 4 * world)).size()) return e2;
                (void)hipMemcpyAsync(d_rec.p, rec.data(), (size_t)L * 4, hipMemcpyHostToDevice, s);
                if ((e2 = NcclErr(ncclAllGather(d_rec.p, d_all.p, (size_t)L, ncclInt32, comm, s), "ncclAllGather")).size())
                    return e2;
                (void)hipMemcpyAsync(all.data(), d_all.p, (size_t)L * 4 * world, hipMemcpyDeviceToHost, s);
                if ((e2 = HipErr(hipStreamSynchronize(s), "records")).size()) return e2;
                int more = 0;
                if ((e2 = FbnErr(fbn_pc_dist_apply(sess, all.data(), &more), "fbn_pc_dist_apply")).size()) return e2;
                if (!more) break;
            }
            return FbnErr(fbn_pc_dist_result(sess, &res[r]), "fbn_pc_dist_result");
        };
        e = body();
        fbn_pc_dist_destroy(sess);
        fbn_ci_ctx_destroy(ctx);
        return e;
    });
    for (int r = 1; r < world; ++r)
        if (res[r]) fbn_pc_result_destroy(res[r]);
    if (!err.empty()) {
        if (res[0]) fbn_pc_result_destroy(res[0]);
        return err;
    }
    *out = res[0];
    return std::string();
}

}  // namespace

void PCStable::StructLearnCompData(fbn_dataset *dts, int group_size, int /*num_threads*/, bool print_struct,
                                   bool /*verbose*/) {
    std::cout << "==================================================" << '\n'
              << "Begin structural learning with PC-stable" << std::endl;
    auto t0 = std::chrono::steady_clock::now();
    int nvars = 0;
    int64_t nsamples = 0;
    fbn_dataset_shape(dts, &nvars, &nsamples);
    nvars_ = nvars;
    std::vector<int32_t> dims(nvars);
    std::vector<uint8_t> cols((size_t)nvars * nsamples);
    fbn_dataset_dims(dts, dims.data());
    fbn_dataset_columns(dts, cols.data());
    fbn_ci_ctx *ctx = nullptr;
    fbn_pc_result *res = nullptr;
    if (gpus_ > 1 || ForceExchange()) {  // RCCL over the node's GPUs (MultiGpu.h)
        GpuGroup g(gpus_, device_);
        // a small graph runs the one-launch device-resident search on every rank (replicas); a
        // larger one is cut by edges per level (the eligibility is a property of the dataset)
        int small = 0;
        fbn_pc_small_eligible_shape(nvars, nsamples, dims.data(), group_size, &small);
        std::string e = !g.ok() ? g.error()
                        : small ? PcReplicas(cols, dims, nvars, nsamples, alpha, depth, g, &res)
                                : PcDistributed(cols, dims, nvars, nsamples, alpha, depth, group_size, g, &res);
        if (!e.empty()) {
            fprintf(stderr, "Error in StructLearnCompData: %s\n", e.c_str());
            exit(1);
        }
        std::cout << "PC-stable skeleton on " << g.size() << " GPU(s) (RCCL, "
                  << (small ? "replicas + result broadcast" : "edges split per level") << ")" << std::endl;
    } else if (fbn_ci_dataset_upload(cols.data(), nvars, nsamples, dims.data(), device_, &ctx) ||
               fbn_pc_stable(ctx, alpha, depth, group_size, &res)) {
        fprintf(stderr, "Error in StructLearnCompData: %s\n", fbn_last_error());
        exit(1);
    }
    int nl = 0, ne = 0;
    fbn_pc_num_levels(res, &nl);
    tests_per_level.resize(nl);
    fbn_pc_level_tests(res, tests_per_level.data());
    fbn_pc_num_edges(res, &ne);
    std::vector<int32_t> pairs(2 * (size_t)ne);
    fbn_pc_edges(res, pairs.data());
    edges.clear();
    for (int i = 0; i < ne; ++i) edges.push_back({pairs[2 * i], pairs[2 * i + 1]});
    int64_t len = 0;
    fbn_pc_sepsets(res, nullptr, 0, &len);
    std::vector<int32_t> buf(len);
    fbn_pc_sepsets(res, buf.data(), len, &len);
    sepset.clear();
    for (int64_t k = 0; k < len;) {
        int x = buf[k], y = buf[k + 1], m = buf[k + 2];
        sepset[{x, y}] = std::set<int>(buf.begin() + k + 3, buf.begin() + k + 3 + m);
        k += 3 + m;
    }
    num_ci_test = 0;
    for (int l = 0; l < nl; ++l) {
        num_ci_test += tests_per_level[l];
        std::cout << "Level " << l << "... # of CI-tests is " << num_ci_test << std::endl;
    }
    // level-0 dependence judgements (src/PCStable.cpp:113-115): edges surviving level 0
    int64_t removed0 = 0;
    for (auto &kv : sepset) removed0 += kv.second.empty();
    num_dependence_judgement = (int64_t)nvars * (nvars - 1) / 2 - removed0;
    double total_s = 0, kernel_s = 0;
    fbn_pc_timing(res, &total_s, &kernel_s);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "==================================================" << std::endl;
    std::cout << "# of CI-tests is " << num_ci_test << ", # of dependence judgements is " << num_dependence_judgement
              << std::endl;
    std::cout << "# remaining edges = " << edges.size() << std::endl;
    std::cout << "pc-stable: " << s << " s pc-stable step 1: " << total_s << " s (device kernels " << kernel_s
              << " s)" << std::endl;
    // decision-margin log (p-values are parity-unpinned)
    fbn_pc_decision_margin(res, &min_margin, &near_alpha);
    std::cout << "min |p - alpha| = " << min_margin << " (" << near_alpha << " decisions within 1e-9)" << std::endl;
    int no = 0;
    fbn_pc_num_oriented_edges(res, &no);
    std::vector<int32_t> tri(3 * (size_t)no + 3);
    fbn_pc_oriented_edges(res, tri.data());
    oriented.clear();
    for (int i = 0; i < no; ++i) oriented.push_back({tri[3 * i], tri[3 * i + 1], tri[3 * i + 2]});
    if (print_struct) {  // Network::PrintEachEdgeWithName
        char a[256], b[256];
        for (auto &e : oriented) {
            fbn_dataset_var_name(dts, e[0], a, sizeof a);
            fbn_dataset_var_name(dts, e[1], b, sizeof b);
            std::cout << a << (e[2] ? " -> " : " -- ") << b << std::endl;
        }
    }
    fbn_pc_result_destroy(res);
    if (ctx) fbn_ci_ctx_destroy(ctx);
}

int PCStable::GetSHD(const std::string &bif_path) const {
    std::vector<int32_t> tri;
    for (auto &e : oriented) tri.insert(tri.end(), e.begin(), e.end());
    tri.resize(tri.size() + 3);
    int shd = -1, nvars = 0;
    for (auto &e : oriented) nvars = std::max(nvars, std::max(e[0], e[1]) + 1);
    if (fbn_shd_bif(bif_path.c_str(), nvars_ > 0 ? nvars_ : nvars, tri.data(), (int)oriented.size(), &shd)) {
        fprintf(stderr, "Error in GetSHD: %s\n", fbn_last_error());
        exit(1);
    }
    return shd;
}
