// fbn_internal.h -- internal types of libfastbn (host side).  Not part of the ABI.
#ifndef FBN_INTERNAL_H
#define FBN_INTERNAL_H

#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/fastbn.h"
#include "jt_program.h"

namespace fbn {

// thread-local error channel behind fbn_last_error()
int SetError(int code, const char *fmt, ...);

// ---------------------------------------------------------------------------------------------
// discrete Bayesian network (CustomNetwork + DiscreteNode state the hot paths read)
struct Network {
    std::vector<std::string> names;
    std::vector<int> dom;
    std::vector<std::vector<int>> given;        // parents in <GIVEN> order
    std::vector<std::vector<int>> parents_asc;  // parents in ascending index order
    std::vector<std::vector<int64_t>> counts;   // [v][q * npc + pc]
    std::vector<std::vector<int64_t>> totals;   // [v][pc], pc over parents_asc, last fastest
    int n() const { return (int)dom.size(); }
    double Prob(int v, int q, const int *parent_vals_asc) const;
};
int LoadXmlbif(const std::string &path, Network &net);
int BuildNetwork(int n, const int32_t *dims, const int32_t *parent_off, const int32_t *parents, const int64_t *counts,
                 const char *const *names, Network &net);
int NodeCounts(const Network &net, int v, int32_t *parents_asc, int64_t *counts, int *nparents, int64_t *ncounts);

struct Dataset {
    int nvars = 0;
    int64_t nsamples = 0;
    std::vector<std::string> names;
    std::vector<int32_t> dims;
    std::vector<uint8_t> cols;  // [var][sample]
};
int LoadCsv(const std::string &path, Dataset &ds);
// ev == nullptr: only *nrows; otherwise the first min(rows, cap) rows into ev [row][num_nodes] / labels
int LoadLibsvm(const std::string &path, int num_nodes, int8_t *ev, int32_t *labels, int64_t cap, int64_t *nrows);

// seeded generators (synth.cpp): numpy-PCG64-identical forward sampling and evidence cases, and
// writers of the reference's text formats
int ForwardSample(const Network &net, int64_t n, uint64_t seed, uint8_t *cols);
int EvidenceCases(const Network &net, int64_t n, int k, uint64_t seed, int query, int8_t *ev);
int WriteCsv(const std::string &path, const uint8_t *cols, int nvars, int64_t n, const std::vector<std::string> &names,
             const std::vector<std::vector<std::string>> &values);
int WriteLibsvm(const std::string &path, const int8_t *ev, int64_t n, int V, const int32_t *labels);

// ---------------------------------------------------------------------------------------------
// junction-tree static plan (host), container order as in JunctionTreeStructure
struct Table {
    std::vector<int> vars, dims, cum;  // row-major, left-most var most significant
    std::vector<double> pot;
    int64_t size() const { return (int64_t)pot.size(); }
    void Rebuild();
};

struct JTPlanHost {
    int num_nodes = 0;
    std::vector<int> dom;
    std::vector<Table> cliques, seps;  // initial potentials after ReorganizeTableStorage
    std::vector<int> clique_up;                 // upstream separator, -1 for the root
    std::vector<std::vector<int>> clique_down;  // downstream separators (MarkLevel order)
    std::vector<int> sep_up, sep_down;          // parent clique, child clique
    int root = -1;
    std::vector<std::vector<int>> levels;       // even levels: cliques, odd levels: separators
};
int BuildJTPlan(const Network &net, JTPlanHost &plan);

// device program (see jt_program.h) compiled from the host plan
struct JTProgram {
    std::vector<JtOp> ops;
    std::vector<int32_t> aux;
    std::vector<double> initv;
    std::vector<uint64_t> dig;
    int64_t state_entries = 0;  // NE: table entries + one pending denominator per clique
    int num_cliques = 0;
    int sum_dom = 0;
    int max_vars = 0;
};
int CompileJTProgram(const JTPlanHost &plan, JTProgram &prog);

// LDS-resident variant: per-wave global regions (entries of 64 lanes x fp64)
struct JTProgramLDS {
    std::vector<JtOp> ops;
    std::vector<int32_t> aux;
    std::vector<double> initv;
    std::vector<uint64_t> dig;
    int64_t store_entries = 0;  // parked collect tables (all cliques but the root)
    int64_t sep_entries = 0;    // separator messages
    int64_t max_table = 0;      // largest clique table (LDS rows needed for no spill)
    int num_cliques = 0;
    int sum_dom = 0;
};
int CompileJTProgramLDS(const JTPlanHost &plan, JTProgramLDS &prog);

// streamed ("virtual table") variant, see jt_program.h
struct JTProgramV {
    std::vector<JtVClique> cl;
    std::vector<int32_t> aux;
    std::vector<double> initv;
    std::vector<uint64_t> dig;
    std::vector<int32_t> order;  // clique ids of the schedule segments (see sched)
    std::vector<int32_t> sched;  // 2 * JT_V_WAVES + 3 segment offsets into order: Collect per wave,
                                 // Collect top, Distribute top, Distribute per wave, end
    double split_efficiency = 1.0;  // modelled parallel efficiency of the waves' tree split
    std::vector<int32_t> vsel;   // per variable {cand_off, ncand, out_off, dim} (candidates in aux)
    int64_t store_rows = 0;      // per-wave fp64 rows: Collect messages, Distribute messages, denominators,
    int64_t scratch_row = 0;     // then one scratch table per wave of the block
    int64_t scratch_rows = 0;    // rows per scratch table
    int num_cliques = 0;
    int sum_dom = 0;
};
// FBN_ERR_LIMIT when the plan does not fit the variant (a clique with > JT_V_MAX_CHILDREN children,
// more than 8 * JT_MAX_DIG_WORDS variables, or tables beyond int32 indexing)
int CompileJTProgramV(const JTPlanHost &plan, JTProgramV &prog);

// tiled variant (jt_tile.hip), see jt_program.h
struct JTProgramT {
    std::vector<JtTPass> passes;  // Collect (post-order), then Distribute (pre-order)
    std::vector<int32_t> tab;     // G / R / outer / bin-digit / marginal / variable / staging records
    std::vector<double> initv;
    int64_t scr_row = 0;          // wave store rows (JT_T_C fp64 each): messages, then partial bins,
    int64_t red_row = 0;          // then reduced bins
    int64_t store_rows = 0;
    int64_t lds_bytes = 0;        // per wave: the largest set of factors staged at once
    int64_t entry_visits = 0;     // clique entries summed over all passes (one case)
    int num_cliques = 0, sum_dom = 0;
    int waves = 1;                // waves per workgroup (one case group each) the passes' splits assume
};
// FBN_ERR_LIMIT when the plan does not fit (a domain > JT_T_MAXDIM states, > JT_T_MAXF - 1 children,
// > 32 digit bits in a clique, tables beyond int32 indexing).  lds_budget: bytes of factors per wave.
int CompileJTProgramT(const JTPlanHost &plan, JTProgramT &prog, int lds_budget);

// plan-specialized kernel source (jt_codegen.cpp): eligibility and generation.  The generated
// kernel's per-wave workspace holds wave_entries rows of 64 fp64 lanes; initv is its constant input.
bool JTCodegenEligible(const JTPlanHost &plan, int64_t *entry_ops);
// fast: the fast arithmetic order (normalizations that cancel are left out; results within 1e-12 of
// the exact order, which repeats the reference's every multiply + Normalize); var_major: marginals
// stored variable-major [sum_dom][ncases] instead of case-major [ncases][sum_dom]
int GenerateJTKernel(const JTPlanHost &plan, std::string &src, int64_t *wave_entries, std::vector<double> &initv,
                     int64_t *lds_bytes = nullptr, bool fast = false, bool var_major = false);

}  // namespace fbn

// C-ABI handles over the host model (capi.hip, synth.cpp)
struct fbn_network {
    fbn::Network net;
};
struct fbn_dataset {
    fbn::Dataset ds;
};

#endif
