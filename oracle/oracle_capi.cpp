// oracle_capi.cpp -- TEST INFRASTRUCTURE.  extern "C" surface of the CPU oracle for ctypes
// (tests/, bench.py cpu_baseline, __graft_entry__.smoke()).  Not part of the product.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "bn_model.h"
#include "jt_oracle.h"
#include "pc_oracle.h"

using namespace oracle;

extern "C" {

// ------------------------------------------------------------------ junction tree
void *or_jt_load(const char *xml_path) {
    auto *t = new JTree();
    t->Build(LoadXmlbif(xml_path));
    return t;
}
void or_jt_destroy(void *h) { delete static_cast<JTree *>(h); }
int or_jt_nvars(void *h) { return static_cast<JTree *>(h)->bn.n; }
int or_jt_dims(void *h, int *out) {
    auto *t = static_cast<JTree *>(h);
    for (int i = 0; i < t->bn.n; ++i) out[i] = t->bn.dom[i];
    return t->bn.n;
}
int or_jt_dump_plan(void *h, const char *plan, const char *init) {
    static_cast<JTree *>(h)->DumpPlan(plan, init);
    return 0;
}
// ev: [ncases][nvars] int8 (-1 unobserved); marg: [ncases][sum dom] (may be NULL)
int or_jt_infer(void *h, const int8_t *ev, int64_t ncases, double *marg, int32_t *labels) {
    auto *t = static_cast<JTree *>(h);
    int sd = 0;
    for (int d : t->bn.dom) sd += d;
    std::vector<double> tmp(sd);
    for (int64_t c = 0; c < ncases; ++c) {
        double *m = marg ? marg + c * sd : tmp.data();
        labels[c] = t->Infer(ev + c * t->bn.n, m);
    }
    return 0;
}
double or_round7(double x) { return Round7(x); }

int64_t or_libsvm_load(const char *path, int nnodes, int8_t *ev, int32_t *labels, int64_t cap) {
    std::vector<int8_t> e;
    std::vector<int> l;
    int64_t n = LoadLibsvmEvidence(path, nnodes, e, l);
    if (ev && labels) {
        int64_t m = n < cap ? n : cap;
        memcpy(ev, e.data(), (size_t)m * nnodes);
        for (int64_t i = 0; i < m; ++i) labels[i] = l[i];
    }
    return n;
}

// ------------------------------------------------------------------ datasets / CI tests
void *or_csv_load(const char *path) { return new CodedDataset(LoadCsv(path)); }
void *or_ds_from_columns(const uint8_t *cols, int nvars, int64_t nsamples, const int32_t *dims) {
    auto *ds = new CodedDataset();
    ds->num_vars = nvars;
    ds->num_samples = nsamples;
    ds->col.resize(nvars);
    for (int v = 0; v < nvars; ++v) {
        ds->col[v].assign(cols + (size_t)v * nsamples, cols + (size_t)(v + 1) * nsamples);
        ds->dims.push_back(dims[v]);
    }
    return ds;
}
void or_ds_destroy(void *h) { delete static_cast<CodedDataset *>(h); }
int or_ds_shape(void *h, int *nvars, int64_t *nsamples) {
    auto *ds = static_cast<CodedDataset *>(h);
    *nvars = ds->num_vars;
    *nsamples = ds->num_samples;
    return 0;
}
int or_ds_dims(void *h, int32_t *out) {
    auto *ds = static_cast<CodedDataset *>(h);
    for (int v = 0; v < ds->num_vars; ++v) out[v] = ds->dims[v];
    return 0;
}
int or_ds_columns(void *h, uint8_t *out) {
    auto *ds = static_cast<CodedDataset *>(h);
    for (int v = 0; v < ds->num_vars; ++v)
        memcpy(out + (size_t)v * ds->num_samples, ds->col[v].data(), ds->num_samples);
    return 0;
}
double or_chisq_pvalue(double g2, int df) { return ChiSquarePValue(g2, df); }

int or_ci_test(void *h, int x, int y, const int32_t *z, int d, double alpha, double *g2, int32_t *df,
               double *p, int32_t *indep, int32_t *counts, int64_t counts_cap) {
    auto *ds = static_cast<CodedDataset *>(h);
    std::vector<int> zz(z, z + d), cnt;
    CIResult r = CITest(*ds, x, y, zz.data(), d, alpha, counts ? &cnt : nullptr);
    *g2 = r.g2;
    *df = r.df;
    *p = r.p;
    *indep = r.indep;
    if (counts) {
        int64_t m = (int64_t)cnt.size() < counts_cap ? (int64_t)cnt.size() : counts_cap;
        for (int64_t i = 0; i < m; ++i) counts[i] = cnt[i];
        return (int)cnt.size();
    }
    return 0;
}

// ------------------------------------------------------------------ PC-stable skeleton
void *or_pc_run(void *h, double alpha, int depth, int group_size, int keep_log) {
    auto *ds = static_cast<CodedDataset *>(h);
    return new PCResult(PCStableSkeleton(*ds, alpha, depth, group_size, keep_log != 0));
}
void or_pc_destroy(void *r) { delete static_cast<PCResult *>(r); }
int64_t or_pc_num_ci(void *r) { return static_cast<PCResult *>(r)->num_ci_test; }
int or_pc_levels(void *r, int64_t *out, int cap) {
    auto *R = static_cast<PCResult *>(r);
    int n = (int)R->tests_per_level.size();
    for (int i = 0; i < n && i < cap; ++i) out[i] = R->tests_per_level[i];
    return n;
}
int or_pc_edges(void *r, int32_t *out, int cap) {  // out: pairs
    auto *R = static_cast<PCResult *>(r);
    int n = (int)R->edges.size();
    for (int i = 0; i < n && i < cap; ++i) {
        out[2 * i] = R->edges[i].first;
        out[2 * i + 1] = R->edges[i].second;
    }
    return n;
}
// sepsets flattened: for each entry x, y, size, members...; returns int count needed
int64_t or_pc_sepsets(void *r, int32_t *out, int64_t cap) {
    auto *R = static_cast<PCResult *>(r);
    int64_t k = 0;
    for (auto &kv : R->sepset) {
        int32_t vals[3] = {kv.first.first, kv.first.second, (int32_t)kv.second.size()};
        for (int i = 0; i < 3; ++i, ++k)
            if (out && k < cap) out[k] = vals[i];
        for (int m : kv.second) {
            if (out && k < cap) out[k] = m;
            ++k;
        }
    }
    return k;
}
int64_t or_pc_log_size(void *r) { return (int64_t)static_cast<PCResult *>(r)->log.size(); }
// one log entry: level, x, y, d, z[0..d-1] (zcap slots), g2, df, p, indep
int or_pc_log_entry(void *r, int64_t i, int32_t *ints /*4 + zcap*/, int zcap, double *g2, int32_t *df,
                    double *p, int32_t *indep) {
    auto &e = static_cast<PCResult *>(r)->log[i];
    ints[0] = e.level;
    ints[1] = e.x;
    ints[2] = e.y;
    ints[3] = (int32_t)e.z.size();
    for (int j = 0; j < (int)e.z.size() && j < zcap; ++j) ints[4 + j] = e.z[j];
    *g2 = e.r.g2;
    *df = e.r.df;
    *p = e.r.p;
    *indep = e.r.indep;
    return 0;
}

}  // extern "C"
