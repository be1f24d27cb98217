// jt_program.h -- the junction-tree "device program": a case-independent op list compiled on the
// host from the static plan and interpreted by every lane of jt_kernels.hip for its own evidence
// case.  Shared by host (plan compiler) and device (interpreter); plain C layout.
//
// State of one case: NE fp64 entries -- all clique tables, then all separator tables (offsets in
// the ops), then one "pending denominator" per clique.  A clique table is stored *un-divided*
// together with the sum that Normalize() (src/PotentialTableBase.cpp:433-445) would divide it by;
// every consumer reads value / den, which is the exact IEEE result the reference stores, so the
// lazy form is bit-identical while saving one read+write pass per normalization.
//
// Evidence is applied by masking (entries inconsistent with the case's evidence are zero) instead
// of the reference's table reduction (src/PotentialTable.cpp:309-396): the consistent entries keep
// their relative order, zeros add exactly, and every division is zero-guarded, so all sums and
// products equal the reduced-table ones bit for bit; the index maps become case-independent.
#ifndef FBN_JT_PROGRAM_H
#define FBN_JT_PROGRAM_H

#include <stdint.h>

enum JtOpType : int32_t {
    // a=table off, b=T, c=aux off of var list, d=nv, e=dig word off, f=den idx (-1 sep),
    // g=clique id (-1 sep), h=initv off
    JT_OP_INIT = 1,
    // a=sep off, b=Ts, c=child off, d=Tc, e=child den idx   (SeparatorLevelCollectionOptimized)
    JT_OP_SEPCOL = 2,
    // a=parent off, b=Tp, c=parent den idx, d=sep off, e=aux off of map[Tp]  (CliqueLevelCollection)
    JT_OP_CLQMUL = 3,
    // a=sep off, b=Ts, c=parent off, d=parent den idx, e=aux off of lists[Ts][f], f=Tp/Ts
    //                                                                      (SeparatorLevelDistribution)
    JT_OP_SEPDIS = 4,
    // a=child off, b=Tc, c=child den idx, d=sep off, e=Ts   (CliqueLevelDistributionOptimized)
    JT_OP_CLQDIS = 5,
    // a=output offset of the var in the case row, b=dim, c=aux off of candidates, d=#candidates,
    // e=var, f=1 if the query var (label)                    (GetProbabilitiesOneNode / ArgMax)
    // candidate record (6 int32): clique id, table off, den idx, nv, cum of var, T
    JT_OP_MARG = 6
};

// ---- LDS-resident variant (jt_lds_kernel): the clique being worked on lives in LDS (lane = case,
// [entry][64] layout), its pending normalization denominator in a register; finished collect
// tables are parked in a per-wave global store and read back once in Distribute, separator
// messages live in a per-wave global store.  Cliques are processed one at a time, children before
// parents in Collect and parents before children in Distribute (the reference's level order).
enum JtLOpType : int32_t {
    JT_L_INIT = 11,    // b=T, c=aux off of var list, d=nv, e=dig word off, g=clique id, h=initv off
    JT_L_MUL = 12,     // b=T, c=Ts, d=sep store off, e=aux off of lists[Ts][T/Ts] (CliqueLevelCollection)
    JT_L_SEPCOL = 13,  // a=sep store off, b=Ts, c=T                          (SeparatorLevelCollection)
    JT_L_STORE = 14,   // a=store off, b=T, c=clique id (den slot)
    JT_L_LOAD = 15,    // a=store off, b=T, c=clique id
    JT_L_DMUL = 16,    // b=T, d=sep store off, e=Ts                          (CliqueLevelDistribution)
    JT_L_SEPDIS = 17,  // a=sep store off, b=Ts, e=aux off of lists[Ts][f], f=T/Ts (SeparatorLevelDistribution)
    JT_L_MARG = 18,    // a=out off, b=dim, c=aux off of candidate clique ids, d=#candidates, e=var,
                       // f=is query, g=this clique id, h=cum of var in this clique, pad=T
    JT_L_EVZERO = 19   // a=out off, b=dim, e=var
};

struct JtOp {
    int32_t type, a, b, c, d, e, f, g, h, pad;
};

#define JT_MAX_DIG_WORDS 4  // 8 variables per 64-bit word -> at most 32 variables per table

// ---- streamed ("virtual table") variant, jt_virt.hip: clique tables are never stored.  Every
// pass over a clique recomputes each entry from its initial potential, the case's evidence mask,
// the messages already received and the normalization denominators of the earlier steps:
//     c_0(e) = mask(e) ? init(e) : 0,   c_j(e) = (c_{j-1}(e) / D_{j-1}) * M_j(e),   D_j = sum_e c_j(e)
// (M_1..M_k = child Collect messages in multiplication order, M_{k+1} = the parent's Distribute
// message), i.e. exactly the values the reference stores after each multiply + Normalize.  Only
// separator messages (and the per-step denominators) live in the per-wave global store.
struct JtVClique {
    int32_t T, nv, k, root;         // entries, variables, children, is the root
    int32_t iv_off, dig_off, nw;    // initial potentials; entry digits: nw = 0 -> one packed 32-bit
                                    // word per entry (uint32 index 2 * dig_off + e), else 8-bit
                                    // digits in nw uint64 words per entry
    int32_t vars_off;               // aux: per variable {id, digit shift, digit field mask}
    int32_t map_off;                // aux: for each message j < k (+1 for the parent message unless
                                    //      root) T int32 byte offsets (store row * 512) of M_j(e)
    int32_t den_row;                // store rows den_row + j hold D_j (j = 0 .. k+1)
    int32_t up_Ts, up_col_row;      // upstream separator size, its Collect message rows
    int32_t child_off;              // aux: k records {Ts, per, list_off, col_row, dis_row}
    int32_t marg_off, nmarg;        // aux: nmarg records {out_off, dim, var, cum}
    int32_t id;
    int32_t mat;                    // Distribute: the final table is written to the per-wave scratch
                                    // rows once (fused into its normalization pass) and the separator
                                    // and marginal passes read it instead of recomputing the chain
    int32_t cmat;                   // Collect: the last normalization pass writes the table to the
                                    // scratch rows for SEPCOL (else SEPCOL recomputes the chain)
};
#define JT_V_MAX_CHILDREN 6
#define JT_V_WAVES 2  // waves sharing one 64-case block (disjoint subtrees in parallel)

// ---- tiled variant, jt_tile.hip (fast arithmetic order; the Munin-class default): one wave = JT_T_C
// evidence cases x JT_T_L entry slots; JT_T_W waves work on the same case group.  A pass over a clique splits the clique's variables into G
// (lane variables: slot s of a round takes G-configuration round * JT_T_L + s) and R (a stream of
// configurations every lane walks in the same order: outer R-configurations over the output's
// remaining variables, inner ones over the rest).  Entry e = G-part + R-part, so every index map is
// one per-lane constant plus one wave-uniform offset (scalar loads of the R table); an entry is
//     init(e) * M_1(s_1(e)) * ... * M_F(s_F(e))   (0 if it contradicts the case's evidence)
// with the factors = the child Collect messages [+ the parent's Distribute message].  A lane sums
// its entries over the inner stream in a register and stores the sum once per outer configuration
// into the output's bin (distinct per lane: G holds output variables, or extra variables E whose
// partial bins the post sweep adds up), so no atomics and a fixed summation order.  Messages are
// rows [separator entry][JT_T_C cases]: the factors of a clique fit LDS, the per-case
// normalizations of the reference cancel in the normalized results (fast order, within 1e-12).
#define JT_T_C 16           // cases per wave: a message row is JT_T_C fp64 = 128 B, one cache line
#define JT_T_L 4            // entry slots per case (JT_T_C * JT_T_L = 64 lanes)
#define JT_T_MAXF 7         // factors per pass: <= 6 child messages + the parent message
#define JT_T_MAXDIM 128     // state counts of the variables (int8 evidence codes; marginal sweep in
                            // groups of 8 values, value d in slot d % JT_T_L)
#define JT_T_LDS_BIN_ROWS 16  // a pass's partial bins live in LDS when they are at most this many rows
#define JT_T_W 4            // most waves per workgroup: they share one case group, its message store and
                            // its LDS factor stage, and split every pass (rounds or outer configurations);
                            // the plan's choice (FBN_JT_TW, default 1: measured fastest)
enum JtTKind : int32_t { JT_T_COL = 0, JT_T_DIS = 1, JT_T_MARG = 2 };
struct JtTPass {
    int32_t kind, clique, nf, nl;    // factors; factors 0 .. nl-1 are staged in LDS, the rest are read
                                     // from the wave store
    int32_t nG, rounds, nRo, nRi;    // G-configurations, rounds of JT_T_L, outer / inner R stream
    int32_t g_off, o_off, i_off;     // tab: G records and outer R records (4 + nf ints each: entry, digit
                                     // word, bin, pad, factor byte offsets), inner R records (2 + nf
                                     // ints: entry byte offset, digit word, factor byte offsets)
    int32_t nE, nbins;               // partial bins per output bin (E configurations), output bins
    int32_t dest_row, col_row;       // output message rows (-1: MARG), the child's Collect message (DIS)
    int32_t bdig_off;                // tab: packed digits of every output bin (marginal sweep)
    int32_t nmv, mv_off;             // marginals taken from this pass's bins: {var, out_off, dim, shift, mask}
    int32_t iv_off;                  // initial potentials (fp64 index)
    int32_t nv, vars_off;            // clique variables {var, shift, mask} (evidence digit fields)
    uint32_t gfields, ofields;       // digit fields of the G / outer R variables
    int32_t first;                   // first pass of a clique phase: the lanes' evidence words, then the
    int32_t nstage, stage_off;       // factors staged into LDS ({src row, rows, lds byte offset} records)
    int32_t et_off;                  // tab: the R part of the entry (bytes) of every flattened R step
    int32_t st_off;                  // tab: step records {factor soffsets [nf] (bit 0: the same row as the
                                     //      step before), digit word, bin offset of the inner run ending
                                     //      at the step or -1}
    // messages are stored un-normalized with a per-case scale row (normalized = values / scale):
    int32_t fsc_off;                 // tab: the nf factors' scale rows
    int32_t dest_sc, col_sc;         // scale rows of the output message and of the child's Collect message (DIS)
    int32_t split;                   // work of the JT_T_W waves: 0 = rounds (round r -> wave r % JT_T_W),
                                     // 1 = outer configurations (contiguous blocks, every round)
    int32_t chunk;                   // inner steps per run: nRi, or (loop-tiled R stream) fewer -- the
                                     // stream is then chunk-major (for each chunk of the inner range, every
                                     // outer configuration), a run's sum writes its bin in the first chunk
                                     // and adds into it after (step record bin field -(bin + 2))
};

#endif
