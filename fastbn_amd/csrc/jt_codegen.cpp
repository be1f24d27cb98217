// jt_codegen.cpp -- plan-specialized junction-tree kernel (HIP source, compiled with hiprtc for gfx950).
//
// For trees whose cliques are small (ALARM-class), the case-independent schedule is emitted as
// straight-line code: every table entry of the clique in flight is a named fp64 register value
// (lane = evidence case), every index map / digit / stride and every initial potential is a
// compile-time constant; the initial potentials are read with wave-uniform scalar loads from a
// constant buffer (or, FBN_JT_IV_LDS=1, from an LDS copy per wave).  No op dispatch, no index arrays;
// LDS holds the entries of a large clique past the register-resident ones and a pool of message
// rows (PlaceMessages).
//
// Schedule (values identical to the reference's level order -- a clique's Collect result depends
// only on its subtree and the fixed order of its child messages, its Distribute result only on its
// parent's -- so any children-first / parent-first traversal gives the same bits):
//  * Collect in DFS post-order: the last child's message stays in registers for its parent; other
//    messages are stored (they are needed again anyway as the "old" separator of Distribute) --
//    in LDS pool rows when their live interval fits, else in the per-wave rows in global memory.
//  * Distribute in DFS pre-order: a clique's Collect table is not parked and reloaded but
//    recomputed from its initial potential and its children's stored messages (which Distribute
//    loads anyway) -- ALU is cheap here, HBM round trips are not.  The message to the first child
//    stays in registers; the others go to LDS pool rows or overwrite their (now dead) Collect
//    message's global rows.
//  * Loads for the next clique are issued at the start of the current one (register budget
//    permitting) so their latency hides behind its arithmetic.
// Operation order per entry is exactly the interpreter's (= the reference's), so results are
// bit-identical; a lane whose normalization denominator leaves [2^-600, 2^600] flags its block,
// which the exact interpreter then recomputes (see capi.hip).
#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <sstream>
#include <string>

#include "fbn_internal.h"

namespace fbn {

namespace {

int LocOfT(const Table &t, int v) {
    for (size_t i = 0; i < t.vars.size(); ++i)
        if (t.vars[i] == v) return (int)i;
    return -1;
}

std::string Lit(double x) {  // exact decimal literal (%.17g round-trips)
    char b[64];
    snprintf(b, sizeof b, "%.17g", x);
    std::string s = b;
    if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
    return s;
}

}  // namespace

bool JTCodegenEligible(const JTPlanHost &plan, int64_t *entry_ops) {
    int64_t tmax = 0, ops = 0;
    for (const auto &t : plan.cliques) {
        tmax = std::max<int64_t>(tmax, t.size());
        ops += t.size() * (4 + (int64_t)t.vars.size());
    }
    if (entry_ops) *entry_ops = ops;
    for (int d : plan.dom)
        if (d > 32) return false;  // evidence bit packing
    return tmax <= 256 && ops <= 40000;  // tails beyond 96 entries in LDS: <= 80 KB per wave
}

namespace {

constexpr int kDefaultMerge = 1;  // FBN_JT_MERGE default (fast order; round 5 sweep: -1..3 %)

class JTGen {
  public:
    JTGen(const JTPlanHost &p, bool fast_order, bool var_major) : plan(p), fast(fast_order), vmajor(var_major) {}
    int Run(std::string &src, int64_t *wave_entries, std::vector<double> &initv);
    int64_t lds_rows = 0;  // LDS rows (64 lanes x fp64) per wave: the clique tail
    int64_t pool_rows = 0;  // + LDS rows of the message pool (after the tail, before the initial potentials)
    // initial potentials: scalar loads from the constant buffer (round 5 default; 1 = an LDS copy per
    // wave, which takes LDS from the message pool: ALARM 0.163 vs 0.141 ms)
    bool iv_lds = false;

  private:
    const JTPlanHost &plan;
    // fast arithmetic order: a clique's table is init * (product of its messages), never normalized
    // in between (the reference's per-step normalizations cancel in every normalized result);
    // messages are normalized once, marginals from a statically chosen clique
    const bool fast;
    const bool vmajor;  // marginals variable-major [SD][ncases] (fbn_jt_set_output_layout)
    std::ostringstream o;
    std::vector<int> okw_word, okw_pos, out_off;
    std::vector<int64_t> sep_row, init_off;
    std::vector<std::vector<int>> cand;
    // fast order: the one clique each variable's evidence is entered in (its smallest holder): the
    // indicator of an observed value multiplies the joint once, so every calibrated clique still
    // holds P(clique, evidence) -- the other holders receive the zeros through their messages
    // (running intersection: the path to the home clique carries the variable)
    std::vector<int> home;
    // fast order: the separator a variable's marginal is summed from (its smallest holder when that
    // is smaller than its smallest clique; -1: the clique): the calibrated separator belief is the
    // parent's bin sums of its SepDis, P(separator, evidence) up to a per-case constant
    std::vector<int> msep;
    // fast order: the clique a variable's marginal is summed in when msep[v] < 0 (default: home[v])
    std::vector<int> mclq;
    // FBN_JT_MARG_SRC (tuning): 0 = the smallest holder (default), 1 = the holder whose Distribute
    // op comes last, 2 = first -- the marginal stores of neighbouring output offsets then land
    // closer together in time (fewer partial write-backs of the case-major output lines).  ALARM:
    // 0.128 / 0.155 / 0.144 ms for 0 / 1 / 2 (gpurun_out/r05an): larger holders cost more terms
    void ChooseMarginalSources(const std::vector<int> &pre);
    // fast order: a marginal (and the label of variable 0) from the terms of each value
    void MargTerms(int v, const std::vector<std::vector<std::string>> &terms);
    int nobs = 0;
    // op boundary (+ diagnostic cycle stamp of op category k when FBN_JT_PROFILE is set)
    bool profile = false;
    // fast order, op regions merged (FBN_JT_MERGE bits): 1 = a clique's SepDis ops and marginals in
    // one region (independent of each other: their latencies overlap), 2 = a Collect message's
    // sums in one region with the next clique's product (small cliques)
    int merge = 0;
    int64_t init_batch = 16;  // fast order: entries per software-pipelined batch of the fused product
    bool in_merged = false;  // the current op's closing boundary is left out
    int min_waves = 1;
    // fast order: unbranched marginals with observed lanes stored as 0.0 (FBN_JT_MARG_V2, default 1)
    // and 16-byte stores of adjacent values (FBN_JT_MARG_PAIR, default 1)
    bool marg_v2 = true, marg_pair = true;
    // where each stored message lives, per separator entry: "W(row)" (the per-wave workspace in
    // global memory) or "LP(row)" (the LDS message pool); the Collect message (child -> parent) and
    // the Distribute message (parent -> child) of a separator are placed separately
    std::vector<std::vector<std::string>> col_loc, dis_loc;
    std::vector<bool> md_reg;  // Distribute messages kept in registers (first child, if it fits)
    // fast order, opt-in (FBN_JT_LEAF_RC=1): Collect messages of small leaf cliques recomputed in the
    // parent's Distribute (initial potential x home indicators, bin sums: the same expression as in
    // Collect) instead of being parked from Collect to Distribute, stored only while the parent's
    // Collect needs them.  ALARM: 195 -> 151 global rows, but 0.137 -> 0.155 ms -- the recomputation
    // sits on the parent's critical path (gpurun_out/r05o), so it is off by default
    std::vector<bool> leaf_rc, col_store;
    void LoadCol(const std::string &name, int s) {
        if (!leaf_rc[s]) return Load(name, s);
        const int c = plan.sep_down[s];
        const int64_t Ts = plan.seps[s].size(), Q = plan.cliques[c].size() / Ts;
        for (int64_t j = 0; j < Ts; ++j) o << "        double " << name << s << "_" << j << ";\n";
        o << "        { // recompute the Collect message of leaf clique " << c << "\n";
        const std::string P = "r" + name;
        InitProd(P, c, {}, -1, "");
        for (int64_t j = 0; j < Ts; ++j) {
            std::vector<std::string> terms;
            for (int64_t q = 0; q < Q; ++q) terms.push_back(N(P, c, q * Ts + j));
            o << "        " << name << s << "_" << j << " = " << TreeSum(terms) << ";\n";
        }
        o << "        }\n";
    }
    void PlaceMessages(const std::vector<int> &post, const std::vector<int> &pre, int64_t budget);
    std::string B(int k) const {
        return profile ? "        FBN_OP_BOUNDARY(); FBN_STAMP(" + std::to_string(k) + ");\n" : "        FBN_OP_BOUNDARY();\n";
    }

    std::string R(int c) const {  // number of unobserved variables of clique c
        std::vector<unsigned> m(nobs, 0u);
        for (int v : plan.cliques[c].vars) m[v / 32] |= 1u << (v % 32);
        std::ostringstream t;
        t << "(" << plan.cliques[c].vars.size();
        for (int k = 0; k < nobs; ++k)
            if (m[k]) t << " - __builtin_popcount(obs" << k << " & " << m[k] << "u)";
        t << ")";
        return t.str();
    }
    std::string observed(int v) const {
        std::ostringstream t;
        t << "((obs" << v / 32 << " >> " << v % 32 << ") & 1u)";
        return t.str();
    }
    int child(int s) const { return plan.sep_down[s]; }
    // separator index of clique entry e (the clique's digits of the separator's variables)
    int64_t SepIndex(const Table &t, const Table &sp, int64_t e) const {
        int64_t r = e, idx = 0;
        for (size_t j = 0; j < t.vars.size(); ++j) {
            const int64_t dgt = r / t.cum[j];
            r %= t.cum[j];
            const int l = LocOfT(sp, t.vars[j]);
            if (l >= 0) idx += dgt * sp.cum[l];
        }
        return idx;
    }
    void Init(const std::string &P, int c);
    // fast order: Init and every multiplication of the clique fused into one op (per entry the
    // initial potential x the home-evidence indicators x each message), ILP over all entries
    void InitProd(const std::string &P, int c, const std::vector<std::pair<int, std::string>> &kids, int up,
                  const std::string &upM);
    void Mul(const std::string &P, int c, int s, const std::string &M);
    void SepCol(const std::string &P, int c, int s, bool store);
    void DMul(const std::string &P, int c, int s, const std::string &M);
    void SepDis(const std::string &P, int c, int s, const std::string &old, bool store);
    void Marg(const std::string &P, int c);
    void Load(const std::string &name, int s) {  // "ld": the Distribute message, else the Collect one
        const auto &loc = name == "ld" ? dis_loc[s] : col_loc[s];
        for (int64_t j = 0; j < plan.seps[s].size(); ++j)
            o << "        const double " << name << s << "_" << j << " = " << loc[j] << ";\n";
    }
    // entry e of clique c's table: a register value, or (entries >= kRegEntries of a large table)
    // an LDS row [row][64 lanes] -- only one clique is in flight, so every table starts at row 0
    // (round 5: 144 -- with the initial potentials as scalar loads, the LDS this frees holds the
    // message pool: ALARM 0.165 -> 0.138 ms per 100k cases; 96 / 112 / 128 / 136 / 144 measured
    // 0.151 / 0.142 / 0.141 / 0.140 / 0.138 ms, gpurun_out/r05l, r05m)
    int64_t kRegEntries = 144;
    std::string N(const std::string &P, int c, int64_t e) const {
        if (e >= kRegEntries) return "L(" + std::to_string(e - kRegEntries) + ")";
        return P + std::to_string(c) + "_" + std::to_string(e);
    }
    // value of entry e as the reference holds it: divided by the pending denominator unless the
    // table has been normalized eagerly (Normalize) since its last update
    bool normed = false;
    std::string Val(const std::string &P, int c, int64_t e) const {
        return (normed || fast) ? N(P, c, e) : "dv(" + N(P, c, e) + ", den, y)";
    }
    // fast order: a sum as a balanced tree of adds (depth log2 n instead of an n-long dependency
    // chain: a dependent fp64 add costs ~45 cycles at one wave per SIMD, an independent one ~5,
    // tools/micro/fp64_ilp.hip); the reference's left-to-right order is kept in the exact order
    static std::string TreeSum(const std::vector<std::string> &t, size_t b, size_t e) {
        if (e - b == 1) return t[b];
        const size_t m = b + (e - b) / 2;
        return "(" + TreeSum(t, b, m) + " + " + TreeSum(t, m, e) + ")";
    }
    static std::string TreeSum(const std::vector<std::string> &t) { return TreeSum(t, 0, t.size()); }
    void Normalize(const std::string &P, int c) {
        const Table &t = plan.cliques[c];
        for (int64_t e = 0; e < t.size(); ++e) o << (e % 8 ? " " : (e ? "\n        " : "        ")) << N(P, c, e) << " = dv(" << N(P, c, e) << ", den, y);";
        o << "\n" << B(6);
        normed = true;
    }
};

// masked initial potential + Normalize (lazy: values raw, den/y pending)
void JTGen::Init(const std::string &P, int c) {
    const Table &t = plan.cliques[c];
    const int nv = (int)t.vars.size();
    // per (variable, value) "allowed by the evidence" lane masks, then one AND chain per entry
    std::vector<bool> ev_here(nv, true);  // variables whose evidence this table carries
    for (int j = 0; j < nv; ++j) ev_here[j] = !fast || home[t.vars[j]] == c;
    for (int j = 0; j < nv; ++j) {
        const int v = t.vars[j];
        if (!ev_here[j]) continue;
        for (int d = 0; d < plan.dom[v]; ++d)
            o << (d ? " " : "        ") << "const bool k" << P << c << "_" << j << "_" << d << " = (okw" << okw_word[v] << " >> "
              << okw_pos[v] + d << ") & 1u;";
        o << "\n";
    }
    if (!fast) o << "        double s_" << P << c << " = 0.0;\n";
    // software-pipelined in batches: the LDS reads of batch b+1 are issued before batch b computes
    const int64_t kB = 16, T = t.size();
    auto loads = [&](int64_t b0) {
        if (b0 >= T) return;
        o << "       ";
        for (int64_t e = b0; e < std::min(T, b0 + kB); ++e)
            o << " const double w" << P << c << "_" << e << " = IV(" << init_off[c] + e << ");";
        o << "\n        __builtin_amdgcn_sched_barrier(0);\n";
    };
    loads(0);
    for (int64_t b0 = 0; b0 < T; b0 += kB) {
        loads(b0 + kB);
        for (int64_t e = b0; e < std::min(T, b0 + kB); ++e) {
            std::ostringstream cond;
            int64_t r = e;
            bool any = false;
            for (int j = 0; j < nv; ++j) {
                const int64_t dgt = r / t.cum[j];
                r %= t.cum[j];
                if (!ev_here[j]) continue;
                cond << (any ? " && " : "") << "k" << P << c << "_" << j << "_" << dgt;
                any = true;
            }
            o << "        " << (e < kRegEntries ? "double " : "") << N(P, c, e) << " = ";
            if (any) o << "sel(" << cond.str() << ", w" << P << c << "_" << e << ");";
            else o << "w" << P << c << "_" << e << ";";
            if (!fast) o << " s_" << P << c << " += " << N(P, c, e) << ";";
            o << "\n";
        }
        o << "        __builtin_amdgcn_sched_barrier(0);\n";
    }
    if (!fast) o << "        den = s_" << P << c << "; y = 1.0 / den; bad |= den_bad(den);\n";
    o << B(2);
    normed = false;
}

void JTGen::InitProd(const std::string &P, int c, const std::vector<std::pair<int, std::string>> &kids, int up,
                     const std::string &upM) {
    const Table &t = plan.cliques[c];
    const int nv = (int)t.vars.size();
    // 0.0 / 1.0 indicators of the home variables' allowed values (x * 1.0 == x, x * 0.0 == 0 for the
    // finite potentials: the masking of the reference's reduction, one multiply instead of a select)
    std::vector<bool> ev_here(nv, false);
    for (int j = 0; j < nv; ++j) ev_here[j] = home[t.vars[j]] == c;
    for (int j = 0; j < nv; ++j) {
        if (!ev_here[j]) continue;
        const int v = t.vars[j];
        for (int d = 0; d < plan.dom[v]; ++d)
            o << (d ? " " : "        ") << "const double i" << P << c << "_" << j << "_" << d << " = (double)((okw"
              << okw_word[v] << " >> " << okw_pos[v] + d << ") & 1u);";
        o << "\n";
    }
    std::vector<std::vector<int64_t>> kidx(kids.size());
    for (size_t i = 0; i < kids.size(); ++i) {
        const Table &sp = plan.seps[kids[i].first];
        for (int64_t e = 0; e < t.size(); ++e) kidx[i].push_back(SepIndex(t, sp, e));
    }
    const int64_t Tup = up >= 0 ? plan.seps[up].size() : 0;
    const int64_t kB = init_batch, T = t.size();  // (FBN_JT_INIT_BATCH: tuning)
    auto loads = [&](int64_t b0) {
        if (b0 >= T) return;
        o << "       ";
        for (int64_t e = b0; e < std::min(T, b0 + kB); ++e)
            o << " const double w" << P << c << "_" << e << " = IV(" << init_off[c] + e << ");";
        o << "\n        __builtin_amdgcn_sched_barrier(0);\n";
    };
    loads(0);
    for (int64_t b0 = 0; b0 < T; b0 += kB) {
        loads(b0 + kB);
        for (int64_t e = b0; e < std::min(T, b0 + kB); ++e) {
            std::vector<std::string> f{"w" + P + std::to_string(c) + "_" + std::to_string(e)};
            int64_t r = e;
            for (int j = 0; j < nv; ++j) {
                const int64_t dgt = r / t.cum[j];
                r %= t.cum[j];
                if (ev_here[j]) f.push_back("i" + P + std::to_string(c) + "_" + std::to_string(j) + "_" + std::to_string(dgt));
            }
            for (size_t i = 0; i < kids.size(); ++i)
                f.push_back(kids[i].second + std::to_string(kids[i].first) + "_" + std::to_string(kidx[i][e]));
            if (up >= 0) f.push_back(upM + std::to_string(up) + "_" + std::to_string(e % Tup));
            // a balanced product tree (depth log2 of the factor count)
            std::function<std::string(size_t, size_t)> prod = [&](size_t lo, size_t hi) -> std::string {
                if (hi - lo == 1) return f[lo];
                const size_t m = lo + (hi - lo) / 2;
                return "(" + prod(lo, m) + " * " + prod(m, hi) + ")";
            };
            o << "        " << (e < kRegEntries ? "double " : "") << N(P, c, e) << " = " << prod(0, f.size()) << ";\n";
        }
        o << "        __builtin_amdgcn_sched_barrier(0);\n";
    }
    o << B(2);
    normed = false;
}

// CliqueLevelCollection: table *= extended child message (by separator entry), then Normalize
void JTGen::Mul(const std::string &P, int c, int s, const std::string &M) {
    const Table &t = plan.cliques[c], &sp = plan.seps[s];
    std::vector<std::vector<int64_t>> inv(sp.size());
    for (int64_t e = 0; e < t.size(); ++e) inv[SepIndex(t, sp, e)].push_back(e);
    for (int64_t j = 0; j < sp.size(); ++j) {
        o << "       ";
        for (int64_t e : inv[j]) o << " " << N(P, c, e) << " = " << Val(P, c, e) << " * " << M << s << "_" << j << ";";
        o << "\n";
    }
    if (!fast) {
        o << "        { double sm = 0.0;";
        for (int64_t e = 0; e < t.size(); ++e) o << " sm += " << N(P, c, e) << ";";
        o << " den = sm; y = 1.0 / den; bad |= den_bad(den); }\n";
    }
    o << B(3);
    normed = false;
}

// SeparatorLevelCollection: message[k % Ts] += table[k] / den  -> registers mc<s>_j (+ store)
void JTGen::SepCol(const std::string &P, int c, int s, bool store) {
    const Table &t = plan.cliques[c];
    const int64_t Ts = plan.seps[s].size(), Q = t.size() / Ts;
    if (fast) {
        // message = the raw bin sums (tree sums), never normalized: every later use is invariant to
        // a per-case scale of it (the Distribute ratio a / old, the normalized marginals), and its
        // values are likelihoods of the evidence below (<= 1); Marg range-checks the products
        for (int64_t j = 0; j < Ts; ++j) {
            std::vector<std::string> terms;
            for (int64_t q = 0; q < Q; ++q) terms.push_back(N(P, c, q * Ts + j));
            o << "        const double mc" << s << "_" << j << " = " << TreeSum(terms) << ";";
            if (store) o << " " << col_loc[s][j] << " = mc" << s << "_" << j << ";";
            o << "\n";
        }
        if (!in_merged) o << B(4);
        return;
    }
    for (int64_t j = 0; j < Ts; ++j) {
        o << "        const double mc" << s << "_" << j << " = " << Val(P, c, j);
        for (int64_t q = 1; q < Q; ++q) o << " + " << Val(P, c, q * Ts + j);
        o << ";";
        if (store) o << " " << col_loc[s][j] << " = mc" << s << "_" << j << ";";
        o << "\n";
    }
    o << B(4);
}

// CliqueLevelDistribution: table *= parent message broadcast over k % Ts, then Normalize
void JTGen::DMul(const std::string &P, int c, int s, const std::string &M) {
    const Table &t = plan.cliques[c];
    const int64_t Ts = plan.seps[s].size();
    for (int64_t j = 0; j < Ts; ++j) {
        o << "       ";
        for (int64_t e = j; e < t.size(); e += Ts)
            o << " " << N(P, c, e) << " = " << Val(P, c, e) << " * " << M << s << "_" << j << ";";
        o << "\n";
    }
    if (!fast) {
        o << "        { double sm = 0.0;";
        for (int64_t e = 0; e < t.size(); ++e) o << " sm += " << N(P, c, e) << ";";
        o << " den = sm; y = 1.0 / den; bad |= den_bad(den); }\n";
    }
    o << B(5);
    normed = false;
}

// SeparatorLevelDistribution: tmp[map(k)] += table[k] / den; message = tmp / old (zero-guarded)
void JTGen::SepDis(const std::string &P, int c, int s, const std::string &old, bool store) {
    const Table &t = plan.cliques[c], &sp = plan.seps[s];
    std::vector<std::vector<int64_t>> lists(sp.size());
    for (int64_t e = 0; e < t.size(); ++e) lists[SepIndex(t, sp, e)].push_back(e);
    if (fast) {
        // bin sums a(j) as trees; md(j) = a(j) / old(j), 0 where old(j) == 0, with branch-free
        // reciprocals (v_rcp_f64 + one Newton step) so the Ts quotients overlap; no normalization
        // (the child's marginals are normalized at the end; values stay likelihoods <= 1)
        for (int64_t j = 0; j < sp.size(); ++j) {
            std::vector<std::string> terms;
            for (int64_t e : lists[j]) terms.push_back(N(P, c, e));
            const std::string sa = "sa" + std::to_string(s) + "_" + std::to_string(j);
            o << "        const double " << sa << " = " << TreeSum(terms) << ";";
            o << " double md" << s << "_" << j << "; { const double od = " << old << s << "_" << j
              << "; const double q = " << sa << " * frcp(od); md" << s << "_" << j << " = (od == 0.0) ? 0.0 : q; }";
            if (store) o << " " << dis_loc[s][j] << " = md" << s << "_" << j << ";";
            o << "\n";
        }
        // the marginals summed from this separator's calibrated belief (its bin sums)
        for (size_t l = 0; l < sp.vars.size(); ++l) {
            const int v = sp.vars[l];
            if (msep[v] != s) continue;
            std::vector<std::vector<std::string>> terms(plan.dom[v]);
            for (int64_t j = 0; j < sp.size(); ++j)
                terms[(j / sp.cum[l]) % sp.dims[l]].push_back("sa" + std::to_string(s) + "_" + std::to_string(j));
            MargTerms(v, terms);
        }
        if (!in_merged) o << B(7);
        return;
    }
    for (int64_t j = 0; j < sp.size(); ++j) {
        o << "        double md" << s << "_" << j << ";";
        o << " { double a = " << Val(P, c, lists[j][0]) << ";";
        for (size_t q = 1; q < lists[j].size(); ++q) o << " a += " << Val(P, c, lists[j][q]) << ";";
        o << " const double od = " << old << s << "_" << j << "; md" << s << "_" << j << " = (od == 0.0) ? 0.0 : a / od; }";
        if (store) o << " " << dis_loc[s][j] << " = md" << s << "_" << j << ";";
        o << "\n";
    }
    o << B(7);
}

void JTGen::MargTerms(int v, const std::vector<std::vector<std::string>> &terms) {
    const int dim = plan.dom[v];
    if (marg_v2) {
        // unbranched: computed for every lane, observed lanes store 0.0 (the reference's marginal of
        // an observed variable) in the same stores -- no divergent branch, no second store pass
        // (ALARM 0.137 -> 0.130 ms); adjacent values go out as one 16-byte store per lane (neutral).
        // (Measured and dropped: staging groups of 8 / 16 output values in LDS pool rows and writing
        // them out coalesced, 0.205 / 0.223 ms -- gpurun_out/r05q.)
        o << "        { // marginal of var " << v << "\n          const bool ob = " << observed(v) << " != 0u;\n";
        std::vector<std::string> ps;
        for (int d = 0; d < dim; ++d) {
            o << "          const double p" << d << " = " << TreeSum(terms[d]) << ";\n";
            ps.push_back("p" + std::to_string(d));
        }
        o << "          const double tot = " << TreeSum(ps) << "; const double yt = frcp(tot); bad |= ob ? 0u : den_bad(tot);\n";
        if (v == 0) {
            o << "          if (ACT && !ob) { int lab = 0; double mp = 0.0, m2 = 0.0;";
            for (int d = 0; d < dim; ++d)
                o << " { const double q = dv(p" << d << ", tot, yt); if (q > mp) { m2 = mp; mp = q; lab = " << d
                  << "; } else if (q > m2) m2 = q; }";
            o << " labels[CS] = lab; bad |= (mp - m2 <= 1e-12 * mp) ? 1u : 0u; }\n";
        }
        for (int d = 0; d < dim; ++d) {
            const int64_t k = out_off[v] + d;
            if (marg_pair && d + 1 < dim) {
                o << "          if (ACT) OUTS2(" << k << ", ob ? 0.0 : dv(p" << d << ", tot, yt), ob ? 0.0 : dv(p" << d + 1 << ", tot, yt));\n";
                ++d;
            } else {
                o << "          if (ACT) OUTS(" << k << ", ob ? 0.0 : dv(p" << d << ", tot, yt));\n";
            }
        }
        o << "        }\n";
        return;
    }
    o << "        if (!" << observed(v) << ") { // marginal of var " << v << "\n";
    std::vector<std::string> ps;
    for (int d = 0; d < dim; ++d) {
        o << "          const double p" << d << " = " << TreeSum(terms[d]) << ";\n";
        ps.push_back("p" + std::to_string(d));
    }
    o << "          const double tot = " << TreeSum(ps) << "; const double yt = frcp(tot); bad |= den_bad(tot);\n";
    if (v == 0) {
        // a near-tie (top two within 1e-12 relative) may break differently from the reference's exact
        // values: the block is flagged for the exact pass
        o << "          if (ACT) { int lab = 0; double mp = 0.0, m2 = 0.0;";
        for (int d = 0; d < dim; ++d)
            o << " { const double q = dv(p" << d << ", tot, yt); if (q > mp) { m2 = mp; mp = q; lab = " << d
              << "; } else if (q > m2) m2 = q; }";
        o << " labels[CS] = lab; bad |= (mp - m2 <= 1e-12 * mp) ? 1u : 0u; }\n";
    }
    o << "          if (ACT) {";
    for (int d = 0; d < dim; ++d) o << " OUTS(" << out_off[v] + d << ", dv(p" << d << ", tot, yt));";
    o << " }\n        }\n";
}

// GetProbabilitiesOneNode for every variable whose selected clique (first with the fewest reduced
// variables) is c, and the label (ArgMax, strict '>' from 0; un-normalized if c reduces to one var)
void JTGen::Marg(const std::string &P, int c) {
    const Table &t = plan.cliques[c];
    for (size_t j = 0; j < t.vars.size(); ++j) {
        const int v = t.vars[j];
        const int dim = plan.dom[v];
        const int64_t cum = t.cum[j], bw = dim * cum, nhi = t.size() / bw;
        if (fast) {  // the smallest clique holding the variable (a calibrated tree: any gives the marginal)
            if (mclq[v] != c || msep[v] >= 0) continue;
            std::vector<std::vector<std::string>> terms(dim);
            for (int d = 0; d < dim; ++d)
                for (int64_t hi = 0; hi < nhi; ++hi)
                    for (int64_t l = 0; l < cum; ++l) terms[d].push_back(N(P, c, hi * bw + d * cum + l));
            MargTerms(v, terms);
            if (!in_merged) o << B(8);
            continue;
        } else {
            // selection: first candidate clique with the fewest reduced variables (recomputed here)
            o << "        { int b = " << R(cand[v][0]) << ", sl = " << cand[v][0] << ";";
            for (size_t k = 1; k < cand[v].size(); ++k)
                o << " { const int r = " << R(cand[v][k]) << "; if (r < b) { b = r; sl = " << cand[v][k] << "; } }";
            o << "\n        if (sl == " << c << " && !" << observed(v) << ") { // marginal of var " << v << "\n";
        }
        if (fast) {  // tree sums, branch-free reciprocal of the total
            std::vector<std::string> ps;
            for (int d = 0; d < dim; ++d) {
                std::vector<std::string> terms;
                for (int64_t hi = 0; hi < nhi; ++hi)
                    for (int64_t l = 0; l < cum; ++l) terms.push_back(N(P, c, hi * bw + d * cum + l));
                o << "          const double p" << d << " = " << TreeSum(terms) << ";\n";
                ps.push_back("p" + std::to_string(d));
            }
            o << "          const double tot = " << TreeSum(ps) << "; const double yt = frcp(tot); bad |= den_bad(tot);\n";
        } else {
            o << "          double tot = 0.0;";
            for (int d = 0; d < dim; ++d) o << " double p" << d << ";";
            o << "\n";
            for (int d = 0; d < dim; ++d) {
                bool first = true;
                o << "          { double a = ";
                for (int64_t hi = 0; hi < nhi; ++hi)
                    for (int64_t l = 0; l < cum; ++l) {
                        const int64_t e = hi * bw + d * cum + l;
                        o << (first ? "" : " a += ") << Val(P, c, e) << ";";
                        first = false;
                    }
                o << " p" << d << " = a; tot += a; }\n";
            }
            o << "          const double yt = 1.0 / tot; bad |= den_bad(tot);\n";
        }
        if (v == 0) {
            // (fast order: a near-tie, top two within 1e-12 relative, may break differently from the
            // reference's exact values -- the block is flagged for the exact pass)
            o << "          if (ACT) { int lab = 0; double mp = 0.0, m2 = 0.0;";
            for (int d = 0; d < dim; ++d)
                o << " { const double q = (b == 1) ? p" << d << " : dv(p" << d << ", tot, yt); if (q > mp) { m2 = mp; mp = q; lab = " << d
                  << "; } else if (q > m2) m2 = q; }";
            o << " labels[CS] = lab;" << (fast ? " bad |= (mp - m2 <= 1e-12 * mp) ? 1u : 0u;" : "") << " }\n";
        }
        o << "          if (ACT) {";
        for (int d = 0; d < dim; ++d) o << " OUTS(" << out_off[v] + d << ", dv(p" << d << ", tot, yt));";
        o << " }\n        } }\n" << (in_merged ? std::string() : B(8));
    }
}

void JTGen::ChooseMarginalSources(const std::vector<int> &pre) {
    const int mode = getenv("FBN_JT_MARG_SRC") ? atoi(getenv("FBN_JT_MARG_SRC")) : 0;
    if (mode == 0 || getenv("FBN_JT_NO_SEPMARG")) return;
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size(), V = (int)plan.dom.size();
    std::vector<int> pi(nc);
    for (int k = 0; k < nc; ++k) pi[pre[k]] = k;
    for (int v = 0; v < V; ++v) {
        // candidates: every clique holding v (its Marg, at its Distribute) and every separator
        // holding v (its parent's SepDis); time = the pre-order position of that op
        int best_t = -1, bc = -1, bs = -1;
        int64_t best_sz = 0;
        auto consider = [&](int t, int64_t sz, int c, int sp) {
            const bool better = best_t < 0 || (mode == 1 ? t > best_t : t < best_t) || (t == best_t && sz < best_sz);
            if (better) best_t = t, best_sz = sz, bc = c, bs = sp;
        };
        for (int c : cand[v]) consider(pi[c], plan.cliques[c].size(), c, -1);
        for (int sp = 0; sp < ns; ++sp)
            for (int u : plan.seps[sp].vars)
                if (u == v) consider(pi[plan.sep_up[sp]], plan.seps[sp].size(), -1, sp);
        if (bs >= 0) msep[v] = bs;
        else msep[v] = -1, mclq[v] = bc;
    }
}

// Message placement.  Every stored message has a live interval on the schedule's clock (Collect
// clique k of the post-order at time k, Distribute clique k of the pre-order at time nc + k): the
// Collect message of separator s from its child's Collect to its parent's Distribute, the
// Distribute message from the parent's Distribute to the child's.  The per-wave workspace of all
// of them (ALARM: 265 rows = 136 KB per wave, 139 MB for 1,024 waves) does not stay in L2, and each
// row written twice per block left L2 twice (PMC, round 5: 0.49 GB written per 100k cases, the
// kernel 20 % slower than with the workspace L2-resident).  So the LDS left over by the clique tail
// and the initial potentials (the budget of four waves per CU) holds a pool of rows, and messages
// get pool rows by interval: shortest intervals first while the pool has room at every time of
// the interval, rows then assigned in start order (an interval graph: the room suffices).  The
// rest keep global rows (Collect and Distribute message of a separator in the same rows, as
// before).  FBN_JT_LDS_POOL=n caps the pool at n rows (0: off).
void JTGen::PlaceMessages(const std::vector<int> &post, const std::vector<int> &pre, int64_t budget) {
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size();
    auto tsize = [&](int c) { return plan.cliques[c].size(); };
    std::vector<int> pi(nc), qi(nc);
    for (int k = 0; k < nc; ++k) qi[post[k]] = k, pi[pre[k]] = k;
    md_reg.assign(ns, false);
    for (int c : pre)
        if (!plan.clique_down[c].empty()) {
            // the child Distribute visits first (the next clique of the pre-order)
            const int q = pre[pi[c] + 1], s = plan.clique_up[q];
            int64_t mk = 0;
            for (int s2 : plan.clique_down[q]) mk = std::max<int64_t>(mk, plan.seps[s2].size());
            md_reg[s] = tsize(q) + plan.seps[s].size() + mk <= budget;
        }
    const bool no_leaf_rc = !getenv("FBN_JT_LEAF_RC") || atoi(getenv("FBN_JT_LEAF_RC")) == 0;  // (tuning)
    leaf_rc.assign(ns, false);
    col_store.assign(ns, true);
    for (int s = 0; s < ns; ++s) {
        const int c = plan.sep_down[s], p = plan.sep_up[s];
        if (!fast || no_leaf_rc || !plan.clique_down[c].empty() || tsize(c) > 64) continue;
        leaf_rc[s] = true;
        // the parent's Collect takes the last child's message from registers when that child ran
        // just before it (Run's collect_loads)
        col_store[s] = !(qi[p] > 0 && post[qi[p] - 1] == c);
    }
    struct Item {
        int s;
        bool dist;
        int a, b;  // live interval [a, b]
        int64_t n;
    };
    std::vector<Item> items;
    for (int s = 0; s < ns; ++s) {
        const int c = plan.sep_down[s], p = plan.sep_up[s];
        if (!leaf_rc[s]) items.push_back({s, false, qi[c], nc + pi[p], plan.seps[s].size()});
        else if (col_store[s]) items.push_back({s, false, qi[c], qi[p], plan.seps[s].size()});
        if (!md_reg[s]) items.push_back({s, true, nc + pi[p], nc + pi[c], plan.seps[s].size()});
    }
    // room: the LDS of four waves per CU (160 KB) less the clique tail and the initial potentials
    const int64_t per_wave = 160 * 1024 / 4 / 8;  // fp64 values
    int64_t ivn = 0;
    for (const auto &t : plan.cliques) ivn += t.size();
    int64_t cap = std::max<int64_t>(0, (per_wave - lds_rows * 64 - (iv_lds ? ivn : 0)) / 64);
    if (const char *e = getenv("FBN_JT_LDS_POOL")) cap = std::min<int64_t>(cap, std::max(0, atoi(e)));
    std::vector<int> order(items.size());
    for (size_t i = 0; i < items.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
        return items[x].b - items[x].a < items[y].b - items[y].a;
    });
    std::vector<int64_t> use(2 * nc + 1, 0);
    std::vector<bool> in_lds(items.size(), false);
    for (int i : order) {
        const Item &it = items[i];
        if (it.n > cap) continue;
        int64_t mx = 0;
        for (int t = it.a; t <= it.b; ++t) mx = std::max(mx, use[t]);
        if (mx + it.n > cap) continue;
        for (int t = it.a; t <= it.b; ++t) use[t] += it.n;
        in_lds[i] = true;
    }
    // concrete pool rows, in start order
    std::vector<int> byst;
    for (size_t i = 0; i < items.size(); ++i)
        if (in_lds[i]) byst.push_back((int)i);
    std::stable_sort(byst.begin(), byst.end(), [&](int x, int y) { return items[x].a < items[y].a; });
    std::vector<std::vector<int64_t>> rows_of(items.size());
    std::vector<int64_t> free_rows;
    for (int64_t r = cap - 1; r >= 0; --r) free_rows.push_back(r);  // (pop_back takes the lowest)
    std::vector<int> active;
    pool_rows = 0;
    for (int i : byst) {
        const Item &it = items[i];
        for (size_t k = 0; k < active.size();) {  // release intervals that ended before this one
            if (items[active[k]].b < it.a) {
                for (int64_t r : rows_of[active[k]]) free_rows.push_back(r);
                std::sort(free_rows.rbegin(), free_rows.rend());
                active.erase(active.begin() + k);
            } else {
                ++k;
            }
        }
        for (int64_t j = 0; j < it.n; ++j) {
            rows_of[i].push_back(free_rows.back());
            pool_rows = std::max<int64_t>(pool_rows, free_rows.back() + 1);
            free_rows.pop_back();
        }
        active.push_back(i);
    }
    col_loc.assign(ns, {});
    dis_loc.assign(ns, {});
    sep_row.assign(ns, -1);
    int64_t grow = 0;
    for (size_t i = 0; i < items.size(); ++i) {
        const Item &it = items[i];
        auto &loc = it.dist ? dis_loc[it.s] : col_loc[it.s];
        loc.assign(it.n, std::string());
        if (in_lds[i]) {
            for (int64_t j = 0; j < it.n; ++j) loc[j] = "LP(" + std::to_string(rows_of[i][j]) + ")";
            continue;
        }
        if (sep_row[it.s] < 0) sep_row[it.s] = grow, grow += it.n;  // (shared by both messages)
        for (int64_t j = 0; j < it.n; ++j) loc[j] = "W(" + std::to_string(sep_row[it.s] + j) + "LL)";
    }
    for (int s = 0; s < ns; ++s) {
        if (sep_row[s] < 0) sep_row[s] = 0;
        if (dis_loc[s].empty()) dis_loc[s].assign(plan.seps[s].size(), "0.0");  // (in registers: never read)
        if (col_loc[s].empty()) col_loc[s].assign(plan.seps[s].size(), "0.0");  // (recomputed: never read)
    }
    if (getenv("FBN_JT_PLACE_DEBUG")) {  // diagnostic: the placement's summary
        int64_t lc = 0, ld = 0, gc = 0, gd = 0, leaf = 0;
        for (size_t i = 0; i < items.size(); ++i)
            (items[i].dist ? (in_lds[i] ? ld : gd) : (in_lds[i] ? lc : gc)) += items[i].n;
        for (int s = 0; s < ns; ++s)
            if (plan.clique_down[plan.sep_down[s]].empty()) leaf += plan.seps[s].size();
        fprintf(stderr, "placement: pool %lld of %lld rows; Collect rows LDS %lld global %lld; Distribute rows LDS %lld "
                        "global %lld (registers: the rest); global rows %lld; leaf-separator rows %lld\n",
                (long long)pool_rows, (long long)cap, (long long)lc, (long long)gc, (long long)ld, (long long)gd,
                (long long)grow, (long long)leaf);
        std::string u;
        for (int t = 0; t <= 2 * nc; ++t) u += std::to_string(use[t]) + (t == nc - 1 ? " | " : " ");
        fprintf(stderr, "pool rows in use by time (Collect | Distribute): %s\n", u.c_str());
        if (fast) {
            std::string m;
            for (int v = 0; v < (int)plan.dom.size(); ++v) {
                const int t = msep[v] >= 0 ? nc + pi[plan.sep_up[msep[v]]] : nc + pi[mclq[v]];
                m += std::to_string(v) + ":" + std::to_string(t) + " ";
            }
            fprintf(stderr, "marginal time per variable: %s\n", m.c_str());
        }
    }
}

int JTGen::Run(std::string &src, int64_t *wave_entries, std::vector<double> &initv) {
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size(), V = plan.num_nodes;
    if (const char *e = getenv("FBN_JT_REG_ENTRIES")) kRegEntries = std::max<int64_t>(1, atoll(e));  // tuning
    profile = getenv("FBN_JT_PROFILE") && atoi(getenv("FBN_JT_PROFILE")) != 0;  // diagnostic build
    merge = fast ? (getenv("FBN_JT_MERGE") ? atoi(getenv("FBN_JT_MERGE")) : kDefaultMerge) : 0;  // (tuning)
    init_batch = getenv("FBN_JT_INIT_BATCH") ? std::max<int64_t>(1, atoll(getenv("FBN_JT_INIT_BATCH"))) : 16;
    marg_v2 = fast && (!getenv("FBN_JT_MARG_V2") || atoi(getenv("FBN_JT_MARG_V2")) != 0);  // (tuning)
    marg_pair = marg_v2 && (!getenv("FBN_JT_MARG_PAIR") || atoi(getenv("FBN_JT_MARG_PAIR")) != 0);  // (tuning)
    // occupancy: waves per SIMD the register allocation must allow (1: up to 512 registers)
    min_waves = getenv("FBN_JT_MIN_WAVES") ? std::max(1, atoi(getenv("FBN_JT_MIN_WAVES"))) : min_waves;
    // initial potentials: LDS copy per wave (1) or scalar loads from the constant buffer (0)
    iv_lds = getenv("FBN_JT_IV_LDS") ? atoi(getenv("FBN_JT_IV_LDS")) != 0 : iv_lds;
    lds_rows = 0;
    for (const auto &t : plan.cliques) lds_rows = std::max<int64_t>(lds_rows, t.size() - kRegEntries);
    // initial potentials: one constant buffer, read with wave-uniform (scalar) loads
    initv.clear();
    init_off.assign(nc, 0);
    for (int c = 0; c < nc; ++c) {
        init_off[c] = (int64_t)initv.size();
        initv.insert(initv.end(), plan.cliques[c].pot.begin(), plan.cliques[c].pot.end());
    }
    int SD = 0;
    out_off.assign(V, 0);
    for (int v = 0; v < V; ++v) out_off[v] = SD, SD += plan.dom[v];
    cand.assign(V, {});
    for (int c = 0; c < nc; ++c)
        for (int v : plan.cliques[c].vars) cand[v].push_back(c);
    home.assign(V, -1);
    for (int v = 0; v < V; ++v)
        for (int q : cand[v])
            if (home[v] < 0 || plan.cliques[q].size() < plan.cliques[home[v]].size()) home[v] = q;
    msep.assign(V, -1);
    if (fast && !getenv("FBN_JT_NO_SEPMARG"))  // (diagnostic: marginals from cliques only)
        for (int sp = 0; sp < ns; ++sp)
            for (int v : plan.seps[sp].vars) {
                const int64_t have = msep[v] >= 0 ? plan.seps[msep[v]].size() : plan.cliques[home[v]].size();
                if (plan.seps[sp].size() < have) msep[v] = sp;
            }
    mclq = home;
    // traversal orders: Collect in post-order, Distribute in pre-order of a DFS.  Any child order
    // gives the same values (schedule freedom, section 4 of DESIGN.md); the fast order may pick one
    // per phase (FBN_JT_CHILD_ORDER bits, tuning): 1 = Collect visits children by ascending
    // separator size (a big message is produced last, so it is parked for less of the schedule),
    // 2 = Distribute visits them by descending size (a big message is consumed first).  ALARM: 1
    // changes nothing, 2 moves 85 message rows to registers and measured slower (0.127 -> 0.132 ms,
    // gpurun_out/r05y), so the default keeps the plan's order
    const int child_order = fast && getenv("FBN_JT_CHILD_ORDER") ? atoi(getenv("FBN_JT_CHILD_ORDER")) : 0;
    auto dfs = [&](bool collect, std::vector<int> &post_o, std::vector<int> &pre_o) {
        std::vector<std::vector<int>> kids(nc);
        for (int c = 0; c < nc; ++c) {
            kids[c] = plan.clique_down[c];
            const bool asc = collect && (child_order & 1), desc = !collect && (child_order & 2);
            if (asc || desc)
                std::stable_sort(kids[c].begin(), kids[c].end(), [&](int x, int y) {
                    return asc ? plan.seps[x].size() < plan.seps[y].size() : plan.seps[x].size() > plan.seps[y].size();
                });
        }
        std::vector<std::pair<int, size_t>> st{{plan.root, 0}};
        while (!st.empty()) {  // iterative DFS
            auto &top = st.back();
            const int c = top.first;
            if (top.second == 0) pre_o.push_back(c);
            if (top.second < kids[c].size()) {
                const int ch = child(kids[c][top.second++]);
                st.push_back({ch, 0});
            } else {
                post_o.push_back(c);
                st.pop_back();
            }
        }
    };
    std::vector<int> post, pre, unused;
    dfs(true, post, unused);
    unused.clear();
    dfs(false, unused, pre);
    if ((int)post.size() != nc) return SetError(FBN_ERR_LIMIT, "codegen: tree traversal covers %zu of %d cliques", post.size(), nc);
    // fp64 values per lane: table in flight + prefetched rows (FBN_JT_PREFETCH_BUDGET: tuning)
    // (fast order: 260 -- round 5 sweep 150 / 200 / 260 / 320: 0.171 / 0.169 / 0.165 / 0.166 ms)
    const int64_t kBudget = getenv("FBN_JT_PREFETCH_BUDGET") ? atoll(getenv("FBN_JT_PREFETCH_BUDGET")) : fast ? 260 : 200;
    if (fast) ChooseMarginalSources(pre);
    PlaceMessages(post, pre, kBudget);
    int64_t rows = 0;
    for (int s = 0; s < ns; ++s) rows = std::max<int64_t>(rows, sep_row[s] + plan.seps[s].size());
    *wave_entries = std::max<int64_t>(rows, 1);

    o << "// generated by libfastbn (jt_codegen.cpp): " << nc << " cliques, " << ns << " separators, "
      << (fast ? "fast" : "exact") << " arithmetic order\n";
    o << "#define FBN_V " << V << "\n#define FBN_SD " << SD << "\n#define FBN_WE " << *wave_entries << "LL\n";
    o << "#define FBN_LP_BASE " << lds_rows << "\n";
    o << "#define FBN_IV_BASE " << (lds_rows + pool_rows) * 64 << "\n#define FBN_NIV " << initv.size() << "\n";
    o << "#define FBN_IV_LDS " << (iv_lds ? 1 : 0) << "\n#define FBN_MIN_WAVES " << min_waves << "\n";
    // diagnostic only (FBN_JT_WS_FOLD=K, wrong results): K workspaces shared by all waves, so the
    // workspace stays in L2 -- times the kernel without its workspace's fabric traffic
    if (const char *e = getenv("FBN_JT_WS_FOLD")) o << "#define FBN_WS_FOLD " << atoi(e) << "\n";
    if (getenv("FBN_JT_NO_OUT") && atoi(getenv("FBN_JT_NO_OUT")) != 0) o << "#define FBN_NO_OUT 1\n";
    if (vmajor) o << "#define FBN_VMAJOR 1\n";
    o << R"FBN(typedef signed char i8;
__device__ __forceinline__ double dv(double x, double den, double y) {  // x / den (Markstein, see jt_kernels.hip)
    const double q = x * y;
    const double r = __builtin_fma(-den, q, x);
    return __builtin_fma(r, y, q);
}
// row r of the per-wave workspace, this lane: uniform row base (SGPRs) + lane byte offset (VGPR)
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) char gchar;
typedef __attribute__((address_space(4))) const double cdouble;
#define W(row) (*(gdouble *)((gchar *)(Wb + (row) * 64) + (unsigned long long)lo))
// LDS row of the clique in flight (entries beyond the register-resident part of large tables)
typedef __attribute__((address_space(3))) double ldouble;
extern __shared__ double fbn_lds[];
#define L(row) (ltail[(row) * 64])
// LDS message pool row (after the clique tail)
#define LP(row) (ltail[(FBN_LP_BASE + (row)) * 64])
// initial potentials: copied into LDS once per wave (wave-uniform address: broadcast reads), or
// read with scalar loads from the constant buffer
#if FBN_IV_LDS
#define IV(k) (ivl[k])
#else
#define IV(k) (ivc[k])
#endif
// unconditional (LDS broadcast) load + select: no branch per table entry
__device__ __forceinline__ double sel(bool c, double v) { return c ? v : 0.0; }
#define FBN_STAMP(k) do { unsigned long long t_; __asm__ volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); pacc[k] += t_ - tprev; tprev = t_; } while (0)
__device__ __forceinline__ unsigned den_bad(double d) { return (d >= 0x1p-600 && d <= 0x1p+600) ? 0u : 1u; }
// fast order: 1 / x as v_rcp_f64 + one Newton step (relative error <= 2.3e-15 over 2^-60..2^60,
// tools/micro/fp64_ilp.hip), branch-free, so independent reciprocals overlap; the operands are
// range-checked by den_bad (a block outside [2^-600, 2^600] goes to the exact pass)
__device__ __forceinline__ double frcp(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
}
// this lane's case / output row, recomputed per segment from the (laundered) block index
#define CS (blkl * 64 + lane)
#define ACT (CS < ncases)
#ifdef FBN_VMAJOR
// variable-major output [SD][ncases]: value k of every case is one column, so a store instruction
// writes 64 consecutive cases = 512 contiguous bytes (4 full lines) instead of one value into 64
// lines.  Through a buffer resource: voffset = the lane's case (bytes), soffset = column k (bytes,
// one scalar multiply) -- 64-bit column addresses measured 10 % more instructions and SGPR spills.
// (The host takes this kernel only when ncases * SD * 8 < 2^31.)
typedef unsigned fbn_u2v __attribute__((ext_vector_type(2)));
#ifdef FBN_NO_OUT
#define OUTS(k, v) do { if (ncases < 0) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(fbn_u2v, (double)(v)), mrs, (int)(CS * 8), (int)(k) * mcb, 0); } while (0)
#else
#define OUTS(k, v) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(fbn_u2v, (double)(v)), mrs, (int)(CS * 8), (int)(k) * mcb, 0)
#endif
#else
#define OUT(k) (marg[CS * FBN_SD + (k)])
#ifdef FBN_NO_OUT  // diagnostic only (FBN_JT_NO_OUT=1): marginals computed, never stored
#define OUTS(k, v) do { if (ncases < 0) OUT(k) = (v); } while (0)
#else
#define OUTS(k, v) (OUT(k) = (v))  // (non-temporal stores measured 2.1x slower: partial lines)
#endif
#endif
#ifdef FBN_VMAJOR
#define OUTS2(k, a, b) do { OUTS(k, a); OUTS((k) + 1, b); } while (0)
#else
// two adjacent output values in one 16-byte store (8-byte aligned: the rows are 8 * FBN_SD bytes)
typedef double fbn_d2u __attribute__((ext_vector_type(2), aligned(8)));
#ifdef FBN_NO_OUT
#define OUTS2(k, a, b) do { if (ncases < 0) *(fbn_d2u *)&OUT(k) = (fbn_d2u){(a), (b)}; } while (0)
#else
#define OUTS2(k, a, b) (*(fbn_d2u *)&OUT(k) = (fbn_d2u){(a), (b)})
#endif
#endif
extern "C" __global__ void __launch_bounds__(64, FBN_MIN_WAVES)
fbn_jt_gen(const i8 *__restrict__ evid, double *__restrict__ marg, int *__restrict__ labels,
           double *__restrict__ ws, int *__restrict__ flags, const double *ivp, long long ncases,
           unsigned long long *__restrict__ prof) {
    const int lane = threadIdx.x;
    // LDS bases are laundered at every op boundary (so addresses fold into ds_* offsets instead of
    // being hoisted as loop-invariant constants)
    ldouble *ltail = (ldouble *)fbn_lds + lane;
#if FBN_IV_LDS
    ldouble *ivl = (ldouble *)fbn_lds + FBN_IV_BASE;
    for (int k = lane; k < FBN_NIV; k += 64) IV(k) = ivp[k];
    __syncthreads();
#else
    const cdouble *ivc = (const cdouble *)ivp;
    ldouble *ivl = (ldouble *)fbn_lds;  // unused (laundered at op boundaries)
#endif
    unsigned long long pacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime();
#ifdef FBN_WS_FOLD
    gdouble *Wb = (gdouble *)ws + (unsigned long long)(blockIdx.x % FBN_WS_FOLD) * FBN_WE * 64;
#else
    gdouble *Wb = (gdouble *)ws + (unsigned long long)blockIdx.x * FBN_WE * 64;
#endif
    unsigned lo = (unsigned)lane * 8;
#ifdef FBN_VMAJOR
    const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(marg, 0, 0x7FFFFFFF, 0x00020000);
    const int mcb = (int)ncases * 8;  // column stride, bytes
#endif
    for (long long blk = blockIdx.x; blk * 64 < ncases; blk += gridDim.x) {
        long long blkl = blk;
        const long long cs = blk * 64 + lane;
        const long long csr = cs < ncases ? cs : ncases - 1;
        const i8 *__restrict__ ev = evid + csr * FBN_V;
        unsigned bad = 0u;  // laundered at op boundaries: checked where computed, never deferred
        double den, y;
)FBN";
    // evidence: allowed-value bits of every variable packed into 32-bit words (okw<k>), observed
    // flags (obs<k>); var v owns bits [pos, pos + dom) of its word
    okw_word.assign(V, 0);
    okw_pos.assign(V, 0);
    int nokw = 0;
    {
        int pos = 32;
        for (int v = 0; v < V; ++v) {
            if (pos + plan.dom[v] > 32) ++nokw, pos = 0;
            okw_word[v] = nokw - 1, okw_pos[v] = pos, pos += plan.dom[v];
        }
    }
    nobs = (V + 31) / 32;
    // op boundary: no store->load forwarding, no hoisting of addresses, no scheduling across it,
    // and the evidence words are opaque per segment, so a Distribute recomputation is not merged
    // with (and kept live from) its Collect twin
    {
        std::vector<std::string> regs;
        for (int k = 0; k < nokw; ++k) regs.push_back("okw" + std::to_string(k));
        for (int k = 0; k < nobs; ++k) regs.push_back("obs" + std::to_string(k));
        o << "#define FBN_OP_BOUNDARY() do { __asm__ volatile(\"\" : \"+s\"(Wb), \"+v\"(lo), \"+v\"(ltail), \"+v\"(ivl), \"+v\"(bad), \"+s\"(blkl) :: \"memory\");";
        for (size_t i = 0; i < regs.size(); i += 16) {
            o << " __asm__ volatile(\"\" :";
            for (size_t k = i; k < std::min(regs.size(), i + 16); ++k) o << (k > i ? ", " : " ") << "\"+v\"(" << regs[k] << ")";
            o << ");";
        }
        o << " __builtin_amdgcn_sched_barrier(0); } while (0)\n";
    }
    for (int k = 0; k < nokw; ++k) o << "        unsigned okw" << k << " = 0u;\n";
    for (int k = 0; k < nobs; ++k) o << "        unsigned obs" << k << " = 0u;\n";
    for (int v = 0; v < V; ++v) {
        const unsigned full = (plan.dom[v] >= 32) ? 0xFFFFFFFFu : ((1u << plan.dom[v]) - 1u);
        o << "        { const int x = ev[" << v << "]; okw" << okw_word[v] << " |= (x < 0 ? " << full << "u : (1u << x)) << "
          << okw_pos[v] << "; obs" << v / 32 << " |= (x >= 0 ? 1u : 0u) << " << v % 32 << "; }\n";
    }
    o << B(0);

    auto tsize = [&](int c) { return plan.cliques[c].size(); };
    // ---------------- Collect, DFS post-order
    // loads of clique post[k]: its children's messages except a last child that is post[k-1]
    auto collect_loads = [&](size_t k, std::vector<int> &ls) {
        ls.clear();
        const int c = post[k];
        const auto &down = plan.clique_down[c];
        for (size_t i = 0; i < down.size(); ++i)
            if (!(k > 0 && child(down[i]) == post[k - 1])) ls.push_back(down[i]);  // (the child just collected: registers)
    };
    auto rows_of = [&](const std::vector<int> &ls) {
        int64_t r = 0;
        for (int s : ls) r += plan.seps[s].size();
        return r;
    };
    std::vector<bool> loaded_a(ns, false);
    for (size_t k = 0; k < post.size(); ++k) {
        const int c = post[k];
        std::vector<int> mine, next;
        collect_loads(k, mine);
        o << "        // ---- collect clique " << c << " (" << tsize(c) << " entries)\n";
        for (int s : mine)
            if (!loaded_a[s]) Load("la", s), loaded_a[s] = true;
        if (k + 1 < post.size()) {  // prefetch for the next clique
            collect_loads(k + 1, next);
            int64_t pend = 0;
            for (int s : mine) pend += plan.seps[s].size();
            if (tsize(c) + pend + rows_of(next) <= kBudget)
                for (int s : next)
                    if (!loaded_a[s]) Load("la", s), loaded_a[s] = true;
        }
        if (!in_merged) o << B(1);
        in_merged = false;
        const auto &down = plan.clique_down[c];
        if (fast) {
            std::vector<std::pair<int, std::string>> kids;
            for (int s : down) kids.push_back({s, loaded_a[s] ? "la" : "mc"});
            InitProd("t", c, kids, -1, "");
        } else {
            Init("t", c);
            for (size_t i = 0; i < down.size(); ++i) {
                const int s = down[i];
                Mul("t", c, s, loaded_a[s] ? "la" : "mc");
            }
        }
        // merge the message's sums with the next clique's product when both are small
        in_merged = fast && (merge & 2) && c != plan.root && k + 1 < post.size() && tsize(c) + tsize(post[k + 1]) <= 96;
        if (c != plan.root) SepCol("t", c, plan.clique_up[c], col_store[plan.clique_up[c]]);
    }
    in_merged = false;
    // ---------------- Distribute, DFS pre-order (root continues from its Collect registers)
    // Register policy (kBudget fp64 values per lane):
    //  * the message to a first child stays in registers if that child's table, the message and
    //    its largest child message fit; otherwise it is stored and loaded ("ld") right before DMul
    //  * a clique's children's Collect messages ("lb") are loaded at its start (or prefetched by
    //    the previous clique) if they fit next to its table; otherwise each is loaded right before
    //    its Mul and loaded again ("lc") right before its SepDis
    auto kids_rows = [&](int c) {
        int64_t r = 0;
        for (int s : plan.clique_down[c]) r += plan.seps[s].size();
        return r;
    };
    auto early_lb = [&](int c) {
        const int up = plan.clique_up[c];
        const int64_t held = (c != plan.root) ? plan.seps[up].size() : 0;  // in registers at DMul either way
        return tsize(c) + kids_rows(c) + held <= kBudget;
    };
    std::vector<bool> loaded_b(ns, false), loaded_d(ns, false);
    for (size_t k = 0; k < pre.size(); ++k) {
        const int c = pre[k];
        const int up = plan.clique_up[c];
        const bool early = early_lb(c);
        o << "        // ---- distribute clique " << c << " (" << tsize(c) << " entries)\n";
        int64_t pend = 0;
        if (early)
            for (int s : plan.clique_down[c]) {
                if (!loaded_b[s]) LoadCol("lb", s), loaded_b[s] = true;
                pend += plan.seps[s].size();
            }
        if (c != plan.root && md_reg[up]) pend += plan.seps[up].size();
        if (k + 1 < pre.size()) {  // prefetch for the next clique (before this clique's stores)
            const int nx = pre[k + 1], nup = plan.clique_up[nx];
            // its parent message, unless still in registers or produced by this clique
            const bool ld_next = !md_reg[nup] && plan.sep_up[nup] != c;
            const int64_t nrows = (early_lb(nx) ? kids_rows(nx) : 0) + (ld_next ? plan.seps[nup].size() : 0);
            if (tsize(c) + pend + nrows <= kBudget) {
                if (early_lb(nx))
                    for (int s : plan.clique_down[nx])
                        if (!loaded_b[s] && !leaf_rc[s]) Load("lb", s), loaded_b[s] = true;
                if (ld_next && !loaded_d[nup]) Load("ld", nup), loaded_d[nup] = true;
            }
        }
        o << B(1);
        std::string P = "t";
        if (c != plan.root && fast && early) {  // all messages in registers: one fused op
            P = "u";
            if (!md_reg[up] && !loaded_d[up]) Load("ld", up), loaded_d[up] = true, o << B(1);
            std::vector<std::pair<int, std::string>> kids;
            for (int s : plan.clique_down[c]) kids.push_back({s, "lb"});
            InitProd(P, c, kids, up, md_reg[up] ? "md" : "ld");
        } else if (c != plan.root) {
            P = "u";  // recompute the Collect table (same ops, same order -> same bits)
            Init(P, c);
            for (int s : plan.clique_down[c]) {
                if (!early) LoadCol("lb", s), o << B(1);
                Mul(P, c, s, "lb");
            }
            if (!md_reg[up] && !loaded_d[up]) Load("ld", up), loaded_d[up] = true, o << B(1);
            DMul(P, c, up, md_reg[up] ? "md" : "ld");
        }
        const auto &down = plan.clique_down[c];
        // consumers of the normalized table: one SepDis per child, one marginal per variable
        // (fast order: each SepDis takes the clique total from its own bin sums)
        if (!fast && down.size() + plan.cliques[c].vars.size() >= 2) Normalize(P, c);
        in_merged = fast && (merge & 1) && early;
        for (size_t i = 0; i < down.size(); ++i) {
            if (!early) LoadCol("lc", down[i]), o << B(1);
            SepDis(P, c, down[i], early ? "lb" : "lc", !md_reg[down[i]]);
        }
        Marg(P, c);
        if (in_merged) o << B(8);
        in_merged = false;
    }
    for (int v = 0; v < V && !marg_v2; ++v) {  // (unbranched marginals store the zeros themselves)
        o << "        if (ACT && " << observed(v) << ") {";
        for (int d = 0; d < plan.dom[v]; ++d) o << " OUTS(" << out_off[v] + d << ", 0.0);";
        o << " }\n";
    }
    o << R"(        const bool any_bad = __builtin_amdgcn_ballot_w64(bad != 0u) != 0ull;
        if (lane == 0) flags[blk] = any_bad ? 1 : 0;  // every block writes its flag: no clearing pass
    }
    if (prof && lane == 0)
        for (int k = 0; k < 10; ++k) prof[(unsigned long long)blockIdx.x * 16 + k] = pacc[k];
}
)";
    src = o.str();
    return FBN_OK;
}

}  // namespace

int GenerateJTKernel(const JTPlanHost &plan, std::string &src, int64_t *wave_entries, std::vector<double> &initv,
                     int64_t *lds_bytes, bool fast, bool var_major) {
    JTGen g(plan, fast, var_major);
    int rc = g.Run(src, wave_entries, initv);
    if (lds_bytes) *lds_bytes = ((g.lds_rows + g.pool_rows) * 64 + (g.iv_lds ? (int64_t)initv.size() : 0)) * 8;
    return rc;
}

}  // namespace fbn
