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

struct JtOp {
    int32_t type, a, b, c, d, e, f, g, h, pad;
};

#define JT_MAX_DIG_WORDS 4  // 8 variables per 64-bit word -> at most 32 variables per table

#endif
