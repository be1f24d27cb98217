/* fastbn.h -- C-ABI of the MI355X-native FastBN hot paths (libfastbn.so).
 *
 * Drop-in boundary for the two data-parallel paths of the reference:
 *   * JT: batched junction-tree sum-product.  Replaces the per-case loop of
 *         JunctionTree::PredictUseJTInfer (src/JunctionTree.cpp:1473-1534) behind
 *         Inference::EvaluateAccuracy (include/Inference.h:44).
 *   * PC: the PC-stable skeleton CI sweep.  Replaces IndependenceTest::IndependenceResult
 *         (include/IndependenceTest.h:56, src/IndependenceTest.cpp:35-364) and the level loop of
 *         PCStable::StructLearnByPCStable / SearchAtDepth (src/PCStable.cpp:49-563) behind
 *         StructureLearning::StructLearnCompData (include/StructureLearning.h:22).
 *
 * Conventions: every function returns 0 (FBN_OK) or a negative fbn_err_t; fbn_last_error()
 * gives the message of the last failure on the calling thread.  No exceptions cross the ABI.
 * Plain pointers and sizes only.  Host arrays are caller-owned and only touched during the call;
 * device buffers are owned by the handle.  A handle is bound to one device and is not
 * thread-safe; multi-GPU = one handle per device (one process per GPU).
 */
#ifndef FASTBN_H
#define FASTBN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    FBN_OK = 0,
    FBN_ERR_ARG = -1,     /* bad argument / shape */
    FBN_ERR_IO = -2,      /* file missing or malformed (the reference exit(1)s here) */
    FBN_ERR_HIP = -3,     /* HIP runtime / kernel failure */
    FBN_ERR_NOMEM = -4,   /* host or device allocation failed */
    FBN_ERR_NODEV = -5,   /* no usable gfx950 device */
    FBN_ERR_LIMIT = -6    /* plan exceeds a kernel limit (e.g. variables per clique) */
} fbn_err_t;

const char *fbn_last_error(void);
int fbn_version(int *major, int *minor);
int fbn_device_count(int *n);

/* ------------------------------------------------------------------ networks & data (host) */
typedef struct fbn_network fbn_network;

/* XMLBIF -> discrete network with the reference's CPT convention ((int(p*1e4)+1)/(sum+|dom|),
 * node-major TABLE).  Replaces CustomNetwork::GetNetFromXMLBIFFile (src/CustomNetwork.cpp:20-41)
 * + XMLBIFParser (src/XMLBIFParser.cpp:3-218). */
int fbn_network_load_xmlbif(const char *path, fbn_network **out);
/* A network built in memory -- learned, or constructed by the caller -- with no file in between.
 * Mirrors what the reference's Network of DiscreteNodes holds after InitializeCPT + AddCount
 * (src/DiscreteNode.cpp:114-147): node v has dims[v] states, parents parents[parent_off[v] ..
 * parent_off[v+1]) (any order: the node's own parent order) and the count map
 * map_cond_prob_table_statistics as int64 counts[value][parent config] (parent configurations over
 * the parents in ASCENDING index order, last fastest -- a DiscreteConfig is an ordered set), node
 * after node in one array; totals are the sums over the values (as AddCount keeps
 * map_total_count_under_parents_config), probabilities (count + 1) / (total + dims[v]) as
 * GetProbability (:154-164).  names may be NULL ("X<v>").  The parent lists must form a DAG.
 * The JunctionTree(Network*, ...) constructor of the reference (src/JunctionTree.cpp:3-9) binds to
 * this + fbn_jt_plan_create. */
int fbn_network_create(int nvars, const int32_t *dims, const int32_t *parent_off /* [nvars+1] */,
                       const int32_t *parents, const int64_t *counts, const char *const *names,
                       fbn_network **out);
/* Node v's parents (ascending) and count map in fbn_network_create's layout; NULL buffers: sizes only. */
int fbn_network_node_counts(const fbn_network *net, int node, int32_t *parents, int64_t *counts, int *nparents,
                            int64_t *ncounts);
int fbn_network_num_nodes(const fbn_network *net, int *n);
int fbn_network_dims(const fbn_network *net, int32_t *dims /* [n] */);
int fbn_network_name(const fbn_network *net, int node, char *buf, int cap);
int fbn_network_destroy(fbn_network *net);

/* LIBSVM test set -> evidence rows.  Replaces Dataset::LoadLIBSVMDataKnownNetwork
 * (src/Dataset.cpp:162-262) + the evidence extraction of Inference::Inference
 * (src/Inference.cpp:13-42).  evidence: [ncases][num_nodes] int8, -1 = unobserved.
 * Call with evidence == NULL to get the case count. */
int fbn_evidence_load_libsvm(const char *path, int num_nodes, int8_t *evidence, int32_t *labels,
                             int64_t cap, int64_t *ncases);

/* Seeded workload generators (the reference's SampleSetGenerator is wall-clock seeded
 * and unreachable): forward sampling of n complete cases (cols [V][n] uint8, the reference's CPT
 * convention) and n evidence cases observing k variables each, never `query`, -1 elsewhere
 * (evidence [n][V] int8).  Bit-identical to fastbn_amd/synth.py's numpy PCG64(seed) generators. */
int fbn_synth_forward_sample(const fbn_network *net, int64_t n, uint64_t seed, uint8_t *cols);
int fbn_synth_evidence(const fbn_network *net, int64_t n, int k, uint64_t seed, int query, int8_t *evidence);
/* Writers of the reference's input formats (multi-threaded): CSV with header (network names or
 * X<v>) and values "s<code>"; LIBSVM rows "label v:x ..." of the observed variables. */
int fbn_write_csv(const char *path, const uint8_t *cols, int nvars, int64_t n, const fbn_network *net);
int fbn_write_libsvm(const char *path, const int8_t *evidence, int64_t n, int num_nodes, const int32_t *labels);

typedef struct fbn_dataset fbn_dataset;
/* CSV with header and string values coded by first appearance; column store uint8 [var][sample].
 * Replaces Dataset::LoadCSVData + RowMajor2ColumnMajor (src/Dataset.cpp:267-414,568-580). */
int fbn_dataset_load_csv(const char *path, fbn_dataset **out);
int fbn_dataset_shape(const fbn_dataset *ds, int *nvars, int64_t *nsamples);
int fbn_dataset_dims(const fbn_dataset *ds, int32_t *dims);
int fbn_dataset_columns(const fbn_dataset *ds, uint8_t *cols /* [nvars][nsamples] */);
int fbn_dataset_var_name(const fbn_dataset *ds, int v, char *buf, int cap);
int fbn_dataset_destroy(fbn_dataset *ds);

/* ------------------------------------------------------------------ junction tree */
typedef struct fbn_jt_plan fbn_jt_plan;

typedef struct {
    int32_t num_nodes, num_cliques, num_separators, num_levels;
    int32_t root, sum_dom;
    int64_t clique_entries;     /* sum of clique table sizes */
    int64_t separator_entries;  /* sum of separator table sizes */
    int64_t algorithmic_bytes_per_case; /* 16*(clique+sep entries) + 8*sum_dom + num_nodes */
    int32_t num_ops;            /* device program length */
    int32_t max_vars_per_table;
    int32_t specialized_eligible; /* cliques small enough for the plan-specialized kernel */
    int32_t variant;              /* kernel variant runs use (-1 auto before the first run) */
    int32_t streamed_eligible;    /* the streamed kernel (variant 4) can take the plan */
    int32_t streamed_waves;       /* waves sharing one 64-case block in variant 4 */
    double streamed_split_efficiency; /* modelled parallel efficiency of their subtree split */
    int32_t tiled_eligible;       /* the tiled kernel (variant 5, fast order) can take the plan */
    int32_t tiled_passes;         /* its clique passes per case group */
    int64_t tiled_entry_visits;   /* clique entries summed over those passes (one case) */
    int64_t tiled_lds_bytes;      /* LDS per wave for staged factors */
    int64_t tiled_table_bytes;    /* its index tables (G / R records, ...) */
} fbn_jt_plan_info;

/* Build the case-independent schedule (JunctionTree ctor, src/JunctionTree.cpp:3-46:
 * JunctionTreeStructure src/JunctionTreeStructure.cpp:12-348, root/levels/reorganization
 * :137-281), compile it to a device program and upload it to `device`.  device < 0 builds a
 * host-only plan (info / dump; runs return FBN_ERR_NODEV). */
int fbn_jt_plan_create(const fbn_network *net, int device, fbn_jt_plan **out);
int fbn_jt_plan_info_get(const fbn_jt_plan *p, fbn_jt_plan_info *info);
/* Text dump in the same format as the reference harness (tests/golden/alarm_1k.plan/.init). */
int fbn_jt_plan_dump(const fbn_jt_plan *p, const char *plan_path, const char *init_path);
/* Diagnostics: the streamed kernel's clique schedule.  order[n_order] = clique ids of the segments
 * sched[0..n_sched-1] delimits (waves W = streamed_waves): Collect per wave (W), Collect top,
 * Distribute top, Distribute per wave (W), end.  Pass NULL buffers to query the sizes. */
int fbn_jt_stream_schedule(const fbn_jt_plan *p, int32_t *order, int64_t order_cap, int32_t *sched,
                           int64_t sched_cap, int64_t *n_order, int64_t *n_sched);
/* Evidence cases on the host: evidence [ncases][num_nodes] int8; labels_out [ncases] (arg-max
 * of the query variable 0, InferenceUsingJT src/JunctionTree.cpp:1459-1467); marginals_out
 * [ncases][sum_dom] fp64 or NULL (GetProbabilitiesAllNodes :1385-1454, evidence nodes = 0).
 * Copies in/out over PCIe; synchronous. */
int fbn_jt_run(fbn_jt_plan *p, const int8_t *evidence, int64_t ncases, int32_t *labels_out,
               double *marginals_out, void *hip_stream);
/* Same with device-resident buffers (inputs already in HBM); asynchronous on hip_stream.  Every
 * evidence code must be -1 or < the node's state count: by default the call checks that on the
 * device first (one stream sync) and returns FBN_ERR_ARG naming the first bad case/node; see
 * fbn_jt_set_evidence_check. */
int fbn_jt_run_device(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, int32_t *d_labels,
                      double *d_marginals, void *hip_stream);
/* The device-side evidence check alone (synchronous on hip_stream): FBN_ERR_ARG on the first
 * out-of-domain code.  For callers that validate a buffer once and run it many times. */
int fbn_jt_evidence_validate(fbn_jt_plan *p, const int8_t *d_evidence, int64_t ncases, void *hip_stream);
/* enable = 0: fbn_jt_run_device skips its check (fully asynchronous); the caller guarantees valid
 * evidence (e.g. fbn_jt_evidence_validate once per buffer).  An unchecked out-of-domain code gives
 * unspecified marginals and labels for its case (never an out-of-bounds access).  Default 1.
 * fbn_jt_run always checks. */
int fbn_jt_set_evidence_check(fbn_jt_plan *p, int enable);
/* Per-case MSE and Hellinger distance vs a golden table (CalculateMSE / CalculateHellingerDistance
 * with Round(.,7), src/Inference.cpp:153-206); golden [ncases][sum_dom], evidence nodes marked by
 * golden[.][first state] <= 0.  Host arrays; sums accumulated in case order. */
int fbn_jt_score(const fbn_jt_plan *p, const double *marginals, const double *golden, int64_t ncases,
                 double *mse_sum, double *hd_sum);
/* Layout of the d_marginals buffer of fbn_jt_run_device: 0 = case-major [ncases][sum_dom] (default,
 * the reference's per-case vectors, GetProbabilitiesAllNodes src/JunctionTree.cpp:1385-1454),
 * 1 = variable-major [sum_dom][ncases] (value k of every case contiguous: a kernel store covers 64
 * consecutive cases, written once per cache line).  Same values either way; fbn_jt_run (host
 * buffers) always returns case-major. */
int fbn_jt_set_output_layout(fbn_jt_plan *p, int layout);
/* The per-case terms of fbn_jt_score on the device: d_terms[2 * c] = sqrt(e1 / num) (MSE) and
 * d_terms[2 * c + 1] = sqrt(e2 / num) (HD) of case c, computed exactly as fbn_jt_score computes
 * them (same operations, no contraction), from d_marginals in the plan's output layout and
 * d_golden [ncases][sum_dom] (case-major, as read from the golden file).  Summing the terms in case
 * order reproduces fbn_jt_score's sums bit for bit; asynchronous on hip_stream.  Replaces
 * Inference::CalculateMSE / CalculateHellingerDistance (src/Inference.cpp:153-206) for marginals
 * that stay on the device (the multi-GPU CLI: 16 bytes per case leave a rank instead of sum_dom * 8). */
int fbn_jt_score_terms_device(fbn_jt_plan *p, const double *d_marginals, const double *d_golden, int64_t ncases,
                              double *d_terms, void *hip_stream);
/* Device kernel time (ms, hipEvent) of the last fbn_jt_run*; launches of the main kernel. */
int fbn_jt_last_kernel_ms(const fbn_jt_plan *p, float *ms);
/* enable = 0: fbn_jt_run* records no timing events (two fewer stream markers per call; callers that
 * time with their own events); fbn_jt_last_kernel_ms then fails.  Default 1. */
int fbn_jt_set_kernel_timing(fbn_jt_plan *p, int enable);
/* Tuning: persistent waves per CU (0 = default: as many as keep the largest clique in LDS). */
int fbn_jt_set_waves_per_cu(fbn_jt_plan *p, int waves);
/* Kernel variant: -1 = auto (default: 3 when eligible and its code object loads, else 5 in the fast
 * order, else 4, else 0/1), 0 = clique-in-LDS interpreter, 1 = whole case state in a global
 * workspace interpreter, 2 = variant 0 with the IEEE division sequence forced (ablation / testing),
 * 3 = plan-specialized kernel (jt_codegen.cpp; hiprtc or the on-disk code-object cache) followed
 *     by an exact-path fixup of the blocks it flags.  Selecting 3 fails if the plan is not eligible.
 * 4 = streamed ("virtual table") kernel for large trees (jt_virt.hip): tables recomputed per pass
 *     from initial potentials + received messages, only messages stored; exact-path fixup as 3.
 *     Selecting 4 fails for plans it cannot take (a clique with more than 6 children, ...).
 * 5 = tiled kernel (jt_tile.hip, the Munin-class default): 16 evidence cases x 4 entry slots per
 *     wave, every clique entry recomputed per pass from its initial potential and the messages,
 *     fast arithmetic order only (the exact setting does not apply); exact-path fixup as 3.  Fails
 *     for plans with > 6 children per clique, > 32 digit bits per clique or a domain > 8 states. */
int fbn_jt_set_variant(fbn_jt_plan *p, int variant);
/* Arithmetic order of the specialized (3) and streamed (4) kernels: 1 = exact (the reference's
 * sequential Normalize after every multiply: bit-identical marginals), 0 = fast (a clique's table is
 * its initial potential times its messages, normalized once where a result is formed -- the
 * reference's intermediate normalizations cancel: labels equal, marginals within 1e-12 relative,
 * inside north_star's 1e-6), -1 = auto (default: fast).  This is a parity-relevant default: a
 * caller that needs the reference's bits selects 1.  Replaces no reference interface (the reference
 * has one arithmetic order, src/JunctionTree.cpp:829-941). */
int fbn_jt_set_exact(fbn_jt_plan *p, int exact);
/* Diagnostics (LDS variant): enable per-op-type s_memtime accounting for subsequent runs and/or
 * read the totals of the last run (cycles[10], op types JT_L_INIT..JT_L_EVZERO, summed over waves). */
int fbn_jt_debug_op_cycles(fbn_jt_plan *p, int enable, unsigned long long *cycles);
/* Source of the plan-specialized kernel (variant 3); *len = bytes incl. NUL.  FBN_ERR_ARG if the
 * plan is not eligible (cliques too large for the register-resident form). */
int fbn_jt_kernel_source(const fbn_jt_plan *p, char *buf, int64_t cap, int64_t *len);
/* Testing: variant 3 marks every block for the exact fixup pass (exercises the fixup path). */
int fbn_jt_debug_force_fixup(fbn_jt_plan *p, int enable);
/* Testing: number of 64-case blocks the last run of variant 3 / 4 / 5 flagged for the exact fixup
 * (0 for other variants); synchronizes the device. */
int fbn_jt_debug_flagged_blocks(fbn_jt_plan *p, int64_t *count);
/* Path of the specialized kernel's code object in the on-disk cache (whether or not it exists);
 * a build step may compile fbn_jt_kernel_source() there with the options of fbn_jt_kernel_options. */
int fbn_jt_kernel_cache_path(const fbn_jt_plan *p, char *buf, int64_t cap);
/* Compile the specialized kernel into the on-disk cache now (no device needed); FBN_OK if cached. */
int fbn_jt_kernel_build(const fbn_jt_plan *p);
/* Compile options of the specialized kernel, '\n'-separated. */
int fbn_jt_kernel_options(char *buf, int64_t cap);
/* The tiled kernel's program (variant 5, jt_program.h JtTPass): passes [n_passes] (33 int32 each),
 * index tables [n_tab], initial potentials [n_init]; geometry = {n_passes, n_tab, n_init,
 * partial-bin row, reduced-bin row, store rows, cases per wave, slots per case}.  Buffers may be
 * NULL (sizes only).  For tests that execute the tables on the host (tests/tile_emulator.py). */
int fbn_jt_tile_program(const fbn_jt_plan *p, int32_t *passes, int32_t *tab, double *initv, int64_t *geometry);
int fbn_jt_plan_destroy(fbn_jt_plan *p);

/* ------------------------------------------------------------------ CI tests (G^2) */
typedef struct fbn_ci_ctx fbn_ci_ctx;

/* Upload the column store (uint8 [nvars][nsamples], codes < dims[v] <= 255) to `device`. */
int fbn_ci_dataset_upload(const uint8_t *cols, int nvars, int64_t nsamples, const int32_t *dims,
                          int device, fbn_ci_ctx **out);
/* The same from a column store already in `device`'s memory (uint8 [nvars][nsamples]), e.g. filled
 * by one RCCL broadcast from the rank that loaded the file; copied into the handle.
 * Replaces every rank's own Dataset::LoadCSVData (src/Dataset.cpp:267-414) in a multi-GPU run.
 * Both entry points reject a code >= dims[v] (FBN_ERR_ARG). */
int fbn_ci_dataset_from_device(const uint8_t *d_cols, int nvars, int64_t nsamples, const int32_t *dims,
                               int device, fbn_ci_ctx **out);
/* Kernel-time accounting of a context (default on): HIP events around every CI kernel, summed into
 * fbn_ci_last_kernel_ms / fbn_pc_timing's kernel time.  Off: no events (≈30 µs less per ALARM-5000
 * PC-stable run; the reference's Timer measures wall time only), kernel times read 0. */
int fbn_ci_set_kernel_timing(fbn_ci_ctx *c, int enable);
/* n tests of one conditioning size d: items [n][2+d] = (x, y, z_0..z_{d-1}).  Outputs per test
 * (any may be NULL): G^2, adjusted df, p = 1 - pchisq(G^2, df), indep = (df == 0 || p > alpha).
 * ComputeGSquareXY / ComputeGSquareXYZ semantics (src/IndependenceTest.cpp:65-155,295-364).
 * Host arrays, synchronous. */
int fbn_ci_run(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, double alpha, double *g2,
               int32_t *df, double *p, uint8_t *indep, void *hip_stream);
/* Debug/parity: the contingency table N[z][x][y] of one test (int32, cells = dimz*dx*dy). */
int fbn_ci_counts(fbn_ci_ctx *c, int x, int y, const int32_t *z, int d, int32_t *counts, int64_t cap,
                  int64_t *cells);
int fbn_ci_last_kernel_ms(const fbn_ci_ctx *c, float *ms);
/* Parity pinning of the production paths: counts of n tests (items [n][2+d], level-0 pairs x < y)
 * through the kernels a PC run uses at level d -- d = 0 the complete-graph level-0 batch (Gram of
 * the leading bit-sliced rows, every pair's table recorded), d = 1 the derived counting from those
 * recorded pair tables, d >= 2 the histogram kernel (2-bit packed columns at >= 64k samples) over
 * one batch.  counts [n][cap], Counts3D cell order (src/CellTable.cpp:277-281). */
int fbn_ci_debug_counts(fbn_ci_ctx *c, const int32_t *items, int64_t n, int d, int32_t *counts, int64_t cap);
/* Decision-margin log: the p-value CDF (stats::pchisq, src/IndependenceTest.cpp:146,
 * 268,355) is not pinned by any reference fixture, so every test records min |p - alpha| and counts
 * tests with |p - alpha| < 1e-9 (a decision a different-but-accurate CDF could flip).  Covers every
 * test run on `c` since the last reset (creation resets; `reset` != 0 resets after reading). */
int fbn_ci_decision_margin(fbn_ci_ctx *c, double *min_margin, int64_t *near_alpha, int reset);
int fbn_ci_ctx_destroy(fbn_ci_ctx *c);

/* ------------------------------------------------------------------ PC-stable skeleton */
typedef struct fbn_pc_result fbn_pc_result;

/* Skeleton phase of PC-stable (levels 0 .. depth-1, stop when FreeDegree <= level) with the
 * reference's sequential semantics: per edge the conditioning sets of adj(x)\{y} then adj(y)\{x}
 * in ChoiceGenerator order, first independent set wins, removals applied after each level.
 * group_size as the reference's -g.  CI tests run on the device in speculative batches; the
 * reported counts are the reference's (t = 1) counts. */
int fbn_pc_stable(fbn_ci_ctx *c, double alpha, int depth, int group_size, fbn_pc_result **out);
int fbn_pc_num_levels(const fbn_pc_result *r, int *n);
/* The run's decision-margin log (see fbn_ci_decision_margin): over every test of the skeleton phase. */
int fbn_pc_decision_margin(const fbn_pc_result *r, double *min_margin, int64_t *near_alpha);
int fbn_pc_level_tests(const fbn_pc_result *r, int64_t *tests /* [n_levels] */);
int fbn_pc_level_launched(const fbn_pc_result *r, int64_t *tests /* device tests incl. speculation */);
int fbn_pc_num_edges(const fbn_pc_result *r, int *n);
int fbn_pc_edges(const fbn_pc_result *r, int32_t *pairs /* [n][2], vec_edges order */);
/* sepsets flattened as (x, y, k, z_0..z_{k-1})*, key x < y; returns total int count in *len */
int fbn_pc_sepsets(const fbn_pc_result *r, int32_t *buf, int64_t cap, int64_t *len);
/* One skeleton level for the edge range [e_begin, e_end) of the current skeleton `edges`
 * ([nedges][2], x < y, lexicographic = the reference's vec_edges order): level 0 = one marginal test
 * per edge (src/PCStable.cpp:73-157), level d >= 1 = SearchAtDepth/CheckEdge over the adjacency
 * snapshot implied by `edges` (:209-551).  removed[e - e_begin] = 1 if the edge goes; sepsets
 * [(e_end - e_begin)][d] (or NULL) holds the removing set (sorted, -1 if kept); counted = tests the
 * reference would run, launched = device tests incl. speculation.  The unit a multi-GPU driver
 * partitions (fastbn_amd/pc_dist.py): ranges are independent within a level. */
int fbn_pc_level(fbn_ci_ctx *c, double alpha, int d, int group_size, const int32_t *edges, int64_t nedges,
                 int64_t e_begin, int64_t e_end, uint8_t *removed, int32_t *sepsets, int64_t *counted,
                 int64_t *launched);
/* Host-only: orient a given skeleton (pairs [nedges][2] in vec_edges order) with its sepsets
 * (records (x, y, m, z_0..z_{m-1}) as fbn_pc_sepsets writes them) into a new result. */
int fbn_pc_orient_skeleton(int nvars, const int32_t *pairs, int nedges, const int32_t *sepsets, int64_t len,
                           fbn_pc_result **out);
/* After the skeleton, fbn_pc_stable orients like StructLearnByPCStable steps 2-3
 * (OrientVStructure / OrientImplied, src/PCStable.cpp:576-843): triples [n][3] =
 * (from, to, 1) for arcs, (min, max, 0) for undirected edges, in the reference's vec_edges order. */
int fbn_pc_num_oriented_edges(const fbn_pc_result *r, int *n);
int fbn_pc_oriented_edges(const fbn_pc_result *r, int32_t *triples);
/* SHD against the CPDAG of the DAG in a BIF file (BNSLComparison::GetSHD, src/BNSLComparison.cpp:12-121,
 * true graph via CustomNetwork::LoadBIFFile, src/CustomNetwork.cpp:49-160). */
int fbn_pc_shd_bif(const fbn_pc_result *r, const char *bif_path, int *shd);
/* Same for any learned graph given as triples [n][3] (from, to, 1) / (a, b, 0). */
int fbn_shd_bif(const char *bif_path, int nvars, const int32_t *triples, int n, int *shd);
int fbn_pc_timing(const fbn_pc_result *r, double *total_s, double *kernel_s);
/* Which skeleton path ran: 0 host-driven levels, 1 the device-resident search (small graphs, one
 * launch: plain by default after an occupancy check, cooperative with FBN_PC_SMALL_COOP=1), 2 the
 * device-resident search was refused at launch or timed out at a grid
 * barrier and the host-driven levels ran instead (same answer), 3 host-driven levels whose level 0
 * -> level 1 hand-off ran on the device (the kept pairs became the level-1 edge list / adjacency
 * there; FBN_PC_HOST_L0L1=1 forces 0). */
int fbn_pc_path(const fbn_pc_result *r, int *path);
/* The result as one flat int32 record (for moving it between ranks): magic 0x52504246, n_levels,
 * n_levels (lo, hi) halves of the per-level test counts, n_edges, pairs [n_edges][2], then the
 * fbn_pc_sepsets ints preceded by their count.  *len = ints needed; FBN_ERR_LIMIT if cap is short. */
int fbn_pc_result_record(const fbn_pc_result *r, int32_t *buf, int64_t cap, int64_t *len);
/* 1 if fbn_pc_stable on this context runs the device-resident search (small graphs: <= 64 variables
 * of <= 4 states, group size 1): multi-GPU drivers run such graphs as replicas, not partitioned. */
int fbn_pc_small_eligible(const fbn_ci_ctx *c, int group_size, int *eligible);
/* The same rule from the dataset's shape (no context needed). */
int fbn_pc_small_eligible_shape(int nvars, int64_t nsamples, const int32_t *dims, int group_size, int *eligible);

/* ------------------------------------------------------------------ multi-GPU PC-stable session
 * One session per rank (one process per GPU); the per-level exchange is the caller's collective
 * (RCCL all-gather), everything per edge stays native (fastbn_amd/csrc/pc_dist.cpp).  Replaces the
 * level loop of PCStable::StructLearnByPCStable (src/PCStable.cpp:49-200) for a partitioned run:
 *   create -> { level(world, rank) -> run (or pack) -> [level 0: pairs_export / all-gather /
 *   pairs_import] -> all-gather the records -> apply } until apply reports no further level ->
 *   result (orientation included).  Every rank must apply the same records in rank order. */
typedef struct fbn_pc_dist fbn_pc_dist;
int fbn_pc_dist_create(int nvars, double alpha, int depth, int group_size, fbn_pc_dist **out);
/* Partition of the current level: d (-1 when finished), this rank's edge range [e_begin, e_end) of
 * the current skeleton (vec_edges order) and the int32 length of every rank's record. */
int fbn_pc_dist_level(fbn_pc_dist *s, int world, int rank, int *d, int64_t *e_begin, int64_t *e_end,
                      int64_t *record_len);
int fbn_pc_dist_num_edges(const fbn_pc_dist *s, int64_t *n);
int fbn_pc_dist_edges(const fbn_pc_dist *s, int32_t *pairs /* [n][2] */, int64_t cap);
/* This rank's range on the device of `c` (column store resident there) -> record [record_len]. */
int fbn_pc_dist_run(fbn_pc_dist *s, fbn_ci_ctx *c, int32_t *record);
/* A record from results computed elsewhere: removed [n], sepsets [n][d] (sorted; ignored where
 * not removed), counted / launched tests.  For engines other than the device (testing). */
int fbn_pc_dist_pack(fbn_pc_dist *s, const uint8_t *removed, const int32_t *sepsets, int64_t counted,
                     int64_t launched, int32_t *record);
/* Level 0 pair tables (16 int32 per pair) for the derived level-1 counting: after this rank's
 * level-0 run, export writes its chunk (pairs_chunk pairs, the tail zero-padded by the caller) to
 * buf; the caller all-gathers the chunks in rank order (pair index = offset / 16) and imports the
 * gathered buffer into its context.  buf in device (buf_on_device = 1) or host memory.
 * pairs_chunk = 0: this rank's level 0 recorded no pair tables (the bit-sliced path was not eligible
 * for the dataset, or FBN_CI_NO_PAIRS); the exchange is then skipped on every rank (eligibility
 * depends on the dataset only) and level 1 counts without them. */
int fbn_pc_dist_pairs_chunk(const fbn_pc_dist *s, int64_t *pairs_per_rank);
int fbn_pc_dist_pairs_export(fbn_pc_dist *s, void *buf, int buf_on_device);
int fbn_pc_dist_pairs_import(fbn_pc_dist *s, fbn_ci_ctx *c, const void *buf, int buf_on_device);
/* All ranks' records [world][record_len], rank order: sepsets, counts, removals; *more = 1 if
 * another level follows (depth and FreeDegree, src/PCStable.cpp:159-178). */
int fbn_pc_dist_apply(fbn_pc_dist *s, const int32_t *records, int *more);
/* After the last level: skeleton, sepsets, per-level counts (all ranks), this rank's kernel time /
 * decision margin, orientation (as fbn_pc_stable).  Lifetime: the fbn_ci_ctx passed to
 * fbn_pc_dist_run / _pairs_import must stay alive until the last fbn_pc_dist_apply (the one that
 * reports no further level), which snapshots its margin log and drops its pair tables; result never
 * touches it, so the ctx may be destroyed before this call. */
int fbn_pc_dist_result(fbn_pc_dist *s, fbn_pc_result **out);
int fbn_pc_dist_destroy(fbn_pc_dist *s);
/* Roofline accounting: bytes of column data the CI kernels had to read for every launched test,
 * in the format they read (uint8 columns: N per variable; bit-sliced masks: N/8 per value). */
int fbn_pc_device_bytes(const fbn_pc_result *r, int64_t *bytes);
int fbn_pc_result_destroy(fbn_pc_result *r);

#ifdef __cplusplus
}
#endif

#endif /* FASTBN_H */
