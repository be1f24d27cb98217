// PCStable.cpp -- see PCStable.h
#include "PCStable.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

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
    if (fbn_ci_dataset_upload(cols.data(), nvars, nsamples, dims.data(), device_, &ctx) ||
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
    fbn_ci_ctx_destroy(ctx);
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
