// jt_tile_plan.cpp -- compiles the host plan into the passes of the tiled kernel (jt_tile.hip,
// descriptor JtTPass in jt_program.h).
//
// Per clique and direction (Collect in DFS post-order, Distribute in DFS pre-order, children in
// clique_down order = the reference's multiplication order, src/JunctionTree.cpp:1282-1302):
//   Collect      one pass, output = the upstream separator (SeparatorLevelCollectionOptimized,
//                src/JunctionTree.cpp:1056-1148), factors = the children's Collect messages;
//   Distribute   one pass per child, output = that child's separator (SeparatorLevelDistribution,
//                :700-816), factors = the children's Collect messages + the parent's Distribute
//                message; one more pass for the clique's private variables (in no separator) when
//                their marginals are needed.
// Marginals (GetProbabilitiesOneNode, :1392-1454): after Distribute every clique holding a variable
// has the same marginal of it (a calibrated tree), so each variable's marginal is summed from the
// bins of the smallest Distribute output that contains it -- no pass of its own unless private.
//
// G / R split of a pass: G = output variables whose state product fills the JT_T_L slots of a round
// best (plus extra variables E when the output has fewer than JT_T_L bins: their partial bins are
// added by the post sweep), R outer = the remaining output variables, R inner = the rest.  Every
// index map is linear in the digits (entry = sum d_v cum_v, separator index = sum d_v stride_v),
// so a G record and an R record hold the two halves of each map.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <functional>

#include "fbn_internal.h"

namespace fbn {

namespace {

int PosIn(const std::vector<int> &vars, int v) {
    for (size_t i = 0; i < vars.size(); ++i)
        if (vars[i] == v) return (int)i;
    return -1;
}

struct Factor {
    const Table *sep;
    int64_t row;   // first row of the message in the wave store
    int64_t srow;  // its scale row (the message is stored un-normalized: values / scale)
    int lds_off;   // byte offset in the wave's LDS, -1: read from the wave store
};

// Cartesian enumeration of the digits of `pos` (positions into the clique's variables), last fastest
void ForEachConfig(const Table &t, const std::vector<int> &pos, const std::function<void(const std::vector<int> &)> &fn) {
    std::vector<int> d(pos.size(), 0);
    while (true) {
        fn(d);
        int j = (int)pos.size() - 1;
        while (j >= 0 && ++d[j] == t.dims[pos[j]]) d[j--] = 0;
        if (j < 0) break;
    }
}

int64_t Prod(const Table &t, const std::vector<int> &pos) {
    int64_t p = 1;
    for (int i : pos) p *= t.dims[i];
    return p;
}

// slots used / slots occupied over the rounds of a G of `n` configurations
double SlotEfficiency(int64_t n) { return (double)n / (double)(JT_T_L * ((n + JT_T_L - 1) / JT_T_L)); }

// best subset of `cand` (positions) by slot efficiency, ties -> fewer configurations; `base` always in
std::vector<int> BestSubset(const Table &t, const std::vector<int> &base, const std::vector<int> &cand, bool need_full) {
    const int m = (int)cand.size();
    std::vector<int> best = base;
    double be = -1.0;
    int64_t bn = INT64_MAX;
    for (int mask = 0; mask < (1 << m); ++mask) {
        std::vector<int> g = base;
        for (int i = 0; i < m; ++i)
            if (mask >> i & 1) g.push_back(cand[i]);
        if (g.empty()) continue;
        const int64_t n = Prod(t, g);
        if (need_full && n < JT_T_L && mask != (1 << m) - 1) continue;  // fill a round when possible
        const double e = SlotEfficiency(n);
        if (e > be + 1e-9 || (e > be - 1e-9 && n < bn)) be = e, bn = n, best = g;
    }
    return best;
}

}  // namespace

int CompileJTProgramT(const JTPlanHost &plan, JTProgramT &prog, int lds_budget) {
    prog = JTProgramT();
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size(), V = plan.num_nodes;
    for (int d : plan.dom)
        if (d < 1 || d > JT_T_MAXDIM) return SetError(FBN_ERR_LIMIT, "a domain of %d states (tiled variant: 1..%d)", d, JT_T_MAXDIM);
    for (int c = 0; c < nc; ++c) {
        const Table &t = plan.cliques[c];
        if ((int)plan.clique_down[c].size() + 1 > JT_T_MAXF)
            return SetError(FBN_ERR_LIMIT, "clique %d has %zu children (tiled variant: max %d)", c,
                            plan.clique_down[c].size(), JT_T_MAXF - 1);
        int bits = 0;
        for (int d : t.dims) {
            int w = 1;
            while ((1 << w) < d) ++w;
            bits += w;
        }
        if (bits > 32) return SetError(FBN_ERR_LIMIT, "clique %d: %d digit bits (tiled variant: max 32)", c, bits);
        if (t.size() >= ((int64_t)1 << 26)) return SetError(FBN_ERR_LIMIT, "clique table of %lld entries", (long long)t.size());
    }
    prog.num_cliques = nc;
    std::vector<int64_t> out_off(V);
    for (int v = 0; v < V; ++v) out_off[v] = prog.sum_dom, prog.sum_dom += plan.dom[v];
    // wave store rows (JT_T_C doubles each): Collect messages, Distribute messages, partial bins of the
    // pass in flight, its reduced bins
    // messages are stored un-normalized, each with a scale row (per case: the normalized message =
    // row values / scale), so a pass writes its output bins once, straight from the entry sweep
    std::vector<int64_t> col(ns), dis(ns), col_sc(ns), dis_sc(ns);
    int64_t rows = 0;
    for (int s = 0; s < ns; ++s) col[s] = rows, rows += plan.seps[s].size();
    for (int s = 0; s < ns; ++s) dis[s] = rows, rows += plan.seps[s].size();
    for (int s = 0; s < ns; ++s) col_sc[s] = rows++, dis_sc[s] = rows++;
    prog.scr_row = rows;

    // clique digit fields (evidence masks), initial potentials
    std::vector<std::vector<int>> sh(nc), fm(nc);
    std::vector<int32_t> iv_off(nc), vars_off(nc);
    for (int c = 0; c < nc; ++c) {
        const Table &t = plan.cliques[c];
        int bits = 0;
        vars_off[c] = (int32_t)prog.tab.size();
        for (size_t j = 0; j < t.vars.size(); ++j) {
            int w = 1;
            while ((1 << w) < t.dims[j]) ++w;
            sh[c].push_back(bits), fm[c].push_back((1 << w) - 1);
            prog.tab.push_back(t.vars[j]);
            prog.tab.push_back(bits);
            prog.tab.push_back((1 << w) - 1);
            bits += w;
        }
        iv_off[c] = (int32_t)prog.initv.size();
        prog.initv.insert(prog.initv.end(), t.pot.begin(), t.pot.end());
    }
    if (prog.initv.size() > (size_t)INT32_MAX / 8) return SetError(FBN_ERR_LIMIT, "clique tables too large for the tiled variant");

    // DFS orders
    std::vector<int> post, pre;
    {
        std::vector<std::pair<int, size_t>> st{{plan.root, 0}};
        while (!st.empty()) {
            auto &top = st.back();
            const int c = top.first;
            if (top.second == 0) pre.push_back(c);
            if (top.second < plan.clique_down[c].size()) {
                const int ch = plan.sep_down[plan.clique_down[c][top.second++]];
                st.push_back({ch, 0});
            } else {
                post.push_back(c);
                st.pop_back();
            }
        }
        if ((int)pre.size() != nc) return SetError(FBN_ERR_LIMIT, "tree traversal covers %zu of %d cliques", pre.size(), nc);
    }

    // marginal sources: the smallest separator holding the variable (its SEPDIS pass), else the
    // private-variable pass of the only clique holding it
    std::vector<int> src_sep(V, -1);
    for (int s = 0; s < ns; ++s)
        for (int v : plan.seps[s].vars)
            if (src_sep[v] < 0 || plan.seps[s].size() < plan.seps[src_sep[v]].size()) src_sep[v] = s;
    std::vector<std::vector<int>> priv(nc);  // positions of private variables
    {
        std::vector<int> holder(V, -1), count(V, 0);
        for (int c = 0; c < nc; ++c)
            for (int v : plan.cliques[c].vars) holder[v] = c, ++count[v];
        for (int v = 0; v < V; ++v) {
            if (count[v] == 0) return SetError(FBN_ERR_ARG, "variable %d appears in no clique", v);
            if (src_sep[v] < 0) {
                if (count[v] != 1) return SetError(FBN_ERR_ARG, "internal: variable %d in %d cliques, no separator", v, count[v]);
                priv[holder[v]].push_back(PosIn(plan.cliques[holder[v]].vars, v));
            }
        }
        for (auto &p : priv) std::sort(p.begin(), p.end());
    }

    const int budget_rows = std::max(0, lds_budget) / (JT_T_C * 8);
    // waves per workgroup sharing a case group (1 .. JT_T_W; FBN_JT_TW: tuning knob).  Default 1:
    // on the Munin-like tree 2 / 4 waves per case group measured 235 / 291 ms against 211 ms --
    // the passes' per-pass latency chain and imbalance outweigh the larger shared LDS stage
    const int TW = std::max(1, std::min(JT_T_W, getenv("FBN_JT_TW") ? atoi(getenv("FBN_JT_TW")) : 1));
    prog.waves = TW;
    int64_t max_x = 1, max_bins = 1;

    // one pass: clique c, output variables `opos` (positions) laid out by `ocum` (stride of each
    // output variable in the output's bin index), factors, destination
    auto build_pass = [&](int c, int kind, const std::vector<int> &opos, const std::vector<int64_t> &ocum,
                          int64_t nbins, const std::vector<Factor> &fac_in, int64_t dest_row, int64_t col_row,
                          int64_t dest_sc, int64_t col_sc_row, const std::vector<int> &mvars, bool first, int nstage,
                          int32_t stage_off) -> int {
        const Table &t = plan.cliques[c];
        const int nv = (int)t.vars.size(), nf = (int)fac_in.size();
        JtTPass P{};
        P.kind = kind;
        P.clique = c;
        P.nf = nf;
        // the LDS-resident factors first (the kernel reads factors 0 .. nl-1 from LDS)
        std::vector<Factor> fac(fac_in);
        std::stable_partition(fac.begin(), fac.end(), [](const Factor &f) { return f.lds_off >= 0; });
        P.nl = 0;
        for (const Factor &f : fac) P.nl += f.lds_off >= 0 ? 1 : 0;
        // G: output variables first (no partial bins), extra variables when the output is small
        std::vector<int> G;
        std::vector<int> others;
        for (int j = 0; j < nv; ++j)
            if (std::find(opos.begin(), opos.end(), j) == opos.end()) others.push_back(j);
        if (Prod(t, opos) >= JT_T_L || others.empty()) G = BestSubset(t, {}, opos, false);
        else G = BestSubset(t, opos, others, true);
        if (G.empty()) G = opos.empty() ? std::vector<int>{} : opos;
        std::vector<int> E, RO, RI;
        for (int j : G)
            if (std::find(opos.begin(), opos.end(), j) == opos.end()) E.push_back(j);
        for (int j : opos)
            if (std::find(G.begin(), G.end(), j) == G.end()) RO.push_back(j);
        for (int j = 0; j < nv; ++j)
            if (std::find(G.begin(), G.end(), j) == G.end() && std::find(RO.begin(), RO.end(), j) == RO.end())
                RI.push_back(j);
        const int64_t nE = Prod(t, E), nG = G.empty() ? 1 : Prod(t, G);
        P.nG = (int32_t)nG;
        P.rounds = (int32_t)((nG + JT_T_L - 1) / JT_T_L);
        P.nRo = (int32_t)Prod(t, RO);
        P.nRi = (int32_t)Prod(t, RI);
        P.nE = (int32_t)nE;
        P.nbins = (int32_t)nbins;
        {  // split the pass over the workgroup's waves by rounds or by outer configurations, whichever is shorter
            const int64_t by_rounds = (P.rounds + TW - 1) / TW * (int64_t)P.nRo;
            const int64_t by_outer = (int64_t)P.rounds * ((P.nRo + TW - 1) / TW);
            P.split = by_outer < by_rounds ? 1 : 0;
        }
        max_x = std::max(max_x, nbins * nE);
        max_bins = std::max(max_bins, nbins);
        // factor strides per clique variable
        std::vector<std::vector<int64_t>> fs(nf, std::vector<int64_t>(nv, 0));
        for (int j = 0; j < nf; ++j)
            for (int i = 0; i < nv; ++i) {
                const int l = PosIn(fac[j].sep->vars, t.vars[i]);
                fs[j][i] = l >= 0 ? fac[j].sep->cum[l] : 0;
            }
        // R order (outer, then inner; slowest first): a factor's row changes only when one of its
        // variables does, and the kernel reuses the row it loaded at the previous step, so the order
        // that minimizes the row changes of the wave-store factors (weight 1; LDS ones 1/8) is taken
        // -- exhaustively for small R, else by sorting (variables of many/large factors slowest)
        {
            // weight of a row change: an LDS factor 1/8; a wave-store factor that stays in the
            // wave's share of L2 (<= kCacheRows rows) 1/4; a larger one (its next row misses) 1
            static const int64_t kCacheRows = getenv("FBN_JT_ORDER_ROWS") ? atoll(getenv("FBN_JT_ORDER_ROWS")) : 64;
            auto wgt = [&](int j) {
                return j < P.nl ? 0.125 : fac[j].sep->size() <= kCacheRows ? 0.25 : 1.0;
            };
            auto changes = [&](const std::vector<int> &ord) {
                double cst = 0.0;
                for (int j = 0; j < nf; ++j) {
                    int64_t n = 1, seg = 1;
                    for (int i : ord) {
                        n *= t.dims[i];
                        if (fs[j][i] != 0) seg = n;
                    }
                    cst += wgt(j) * (double)seg;
                }
                return cst;
            };
            auto fact = [](size_t n) { size_t f = 1; for (size_t i = 2; i <= n; ++i) f *= i; return f; };
            if (nf > 0 && fact(RO.size()) * fact(RI.size()) <= 20000) {
                std::vector<int> ro = RO, ri = RI, best;
                std::sort(ro.begin(), ro.end());
                double bc = 1e300;
                do {
                    std::sort(ri.begin(), ri.end());
                    do {
                        std::vector<int> ord = ro;
                        ord.insert(ord.end(), ri.begin(), ri.end());
                        const double cst = changes(ord);
                        if (cst < bc - 1e-9) bc = cst, best = ord;
                    } while (std::next_permutation(ri.begin(), ri.end()));
                } while (std::next_permutation(ro.begin(), ro.end()));
                std::copy(best.begin(), best.begin() + RO.size(), RO.begin());
                std::copy(best.begin() + RO.size(), best.end(), RI.begin());
            } else if (nf > 0) {
                auto key = [&](int i) {
                    double k = 0.0;
                    for (int j = 0; j < nf; ++j)
                        if (fs[j][i] != 0) k += wgt(j);
                    return k;
                };
                auto by = [&](int a, int b) { return key(a) > key(b); };
                std::stable_sort(RO.begin(), RO.end(), by);
                std::stable_sort(RI.begin(), RI.end(), by);
            }
            // LRU refinement, for passes whose wave-store factors exceed the wave's share of L2
            // (kCacheRows rows): round 0's row stream (every slot's rows of every wave-store factor,
            // reused rows skipped as the kernel does) through a kCacheRows-row LRU, for candidate
            // orders -- all when few, else the order above, its adjacent swaps and seeded random
            // ones; the fewest misses wins (ties keep the order above).  FBN_JT_NO_LRU_ORDER: off.
            int64_t glob_rows = 0;
            for (int j = P.nl; j < nf; ++j) glob_rows += fac[j].sep->size();
            const int64_t nR_ = Prod(t, RO) * Prod(t, RI);
            static const bool no_lru = getenv("FBN_JT_NO_LRU_ORDER") != nullptr;
            if (!no_lru && nf > P.nl && glob_rows > kCacheRows && nR_ * P.rounds * (nf - P.nl) >= 8192) {
                std::vector<std::vector<int>> gd;
                ForEachConfig(t, G, [&](const std::vector<int> &d) {
                    if (gd.size() < (size_t)JT_T_L) gd.push_back(d);
                });
                if (G.empty()) gd.assign(1, {});
                std::vector<std::vector<int64_t>> gpart(nf, std::vector<int64_t>(gd.size(), 0));
                for (int j = P.nl; j < nf; ++j)
                    for (size_t sl = 0; sl < gd.size(); ++sl)
                        for (size_t i = 0; i < G.size(); ++i) gpart[j][sl] += gd[sl][i] * fs[j][G[i]];
                const int K = (int)std::min<int64_t>(256, kCacheRows);
                static const int64_t kLruSteps = getenv("FBN_JT_LRU_STEPS") ? atoll(getenv("FBN_JT_LRU_STEPS")) : 1024;
                auto misses = [&](const std::vector<int> &ord) -> int64_t {
                    const int nr = (int)ord.size();
                    std::vector<int> d(nr, 0);
                    std::vector<int64_t> prev(nf, -1);
                    int64_t keys[256];
                    uint64_t stamp[256];
                    int used = 0;
                    uint64_t clk = 0;
                    int64_t miss = 0;
                    for (int64_t k = 0; k < std::min<int64_t>(nR_, kLruSteps); ++k) {  // (a prefix: the
                        for (int j = P.nl; j < nf; ++j) {                              // stream is periodic)
                            int64_t r = 0;
                            for (int i = 0; i < nr; ++i) r += d[i] * fs[j][ord[i]];
                            if (r == prev[j]) continue;  // the kernel keeps the row it has
                            prev[j] = r;
                            for (size_t sl = 0; sl < gd.size(); ++sl) {
                                const int64_t key = ((int64_t)j << 40) | (gpart[j][sl] + r);
                                ++clk;
                                int hit = -1, lru = 0;
                                for (int q = 0; q < used; ++q) {
                                    if (keys[q] == key) { hit = q; break; }
                                    if (stamp[q] < stamp[lru]) lru = q;
                                }
                                if (hit >= 0) { stamp[hit] = clk; continue; }
                                ++miss;
                                if (used < K) keys[used] = key, stamp[used++] = clk;
                                else keys[lru] = key, stamp[lru] = clk;
                            }
                        }
                        for (int i = nr - 1; i >= 0; --i) {  // odometer, last fastest
                            if (++d[i] < t.dims[ord[i]]) break;
                            d[i] = 0;
                        }
                    }
                    return miss;
                };
                std::vector<std::pair<std::vector<int>, std::vector<int>>> cand;
                cand.push_back({RO, RI});
                if (fact(RO.size()) * fact(RI.size()) <= 48) {
                    std::vector<int> ro = RO, ri = RI;
                    std::sort(ro.begin(), ro.end());
                    do {
                        std::sort(ri.begin(), ri.end());
                        do cand.push_back({ro, ri});
                        while (std::next_permutation(ri.begin(), ri.end()));
                    } while (std::next_permutation(ro.begin(), ro.end()));
                } else {
                    for (size_t i = 0; i + 1 < RI.size(); ++i) {
                        auto ri = RI;
                        std::swap(ri[i], ri[i + 1]);
                        cand.push_back({RO, ri});
                    }
                    for (size_t i = 0; i + 1 < RO.size(); ++i) {
                        auto ro = RO;
                        std::swap(ro[i], ro[i + 1]);
                        cand.push_back({ro, RI});
                    }
                    uint64_t rs = 0x9E3779B97F4A7C15ull ^ (uint64_t)prog.passes.size();
                    auto rnd = [&]() { rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17; return rs; };
                    for (int q = 0; q < 24; ++q) {
                        auto ro = RO, ri = RI;
                        for (size_t i = ro.size(); i > 1; --i) std::swap(ro[i - 1], ro[rnd() % i]);
                        for (size_t i = ri.size(); i > 1; --i) std::swap(ri[i - 1], ri[rnd() % i]);
                        cand.push_back({ro, ri});
                    }
                }
                int64_t bm = -1;
                size_t bi = 0;
                for (size_t q = 0; q < cand.size(); ++q) {
                    std::vector<int> ord = cand[q].first;
                    ord.insert(ord.end(), cand[q].second.begin(), cand[q].second.end());
                    const int64_t m = misses(ord);
                    if (bm < 0 || m < bm) bm = m, bi = q;
                }
                RO = cand[bi].first;
                RI = cand[bi].second;
            }
        }
        std::vector<int64_t> ecum(nv, 0), ocum_p(nv, 0);
        {
            int64_t m = 1;
            for (int i = (int)E.size() - 1; i >= 0; --i) ecum[E[i]] = m, m *= t.dims[E[i]];
            for (size_t i = 0; i < opos.size(); ++i) ocum_p[opos[i]] = ocum[i];
        }
        auto fbase = [&](int j) -> int64_t { return fac[j].lds_off >= 0 ? fac[j].lds_off : fac[j].row * (JT_T_C * 8); };
        uint32_t gf = 0;
        for (int j : G) gf |= (uint32_t)fm[c][j] << sh[c][j];
        P.gfields = gf;
        // G records
        P.g_off = (int32_t)prog.tab.size();
        ForEachConfig(t, G, [&](const std::vector<int> &d) {
            int64_t e = 0, x = 0;
            uint32_t dw = 0;
            for (size_t i = 0; i < G.size(); ++i) {
                const int j = G[i];
                e += d[i] * t.cum[j];
                dw |= (uint32_t)d[i] << sh[c][j];
                x += d[i] * (ocum_p[j] * nE + ecum[j]);
            }
            prog.tab.push_back((int32_t)e);
            prog.tab.push_back((int32_t)dw);
            prog.tab.push_back((int32_t)x);
            prog.tab.push_back(0);
            for (int f = 0; f < nf; ++f) {
                int64_t o = fbase(f);
                for (size_t i = 0; i < G.size(); ++i) o += d[i] * fs[f][G[i]] * (JT_T_C * 8);
                prog.tab.push_back((int32_t)o);
            }
        });
        // the R stream = outer configurations (RO) x inner ones (RI); every map is the sum of an outer
        // and an inner part, so the kernel reads a small inner table (reused by every outer
        // configuration and round: it stays in the scalar cache) and one outer record per configuration
        auto emit = [&](const std::vector<int> &vars, bool outer) {  // odometer over `vars`, last fastest
            const int RS = outer ? 4 + nf : 2 + nf;
            const int64_t n = Prod(t, vars);
            const int nr = (int)vars.size();
            std::vector<int64_t> inc((size_t)nr * RS, 0);  // per variable: increments of every field
            for (int k = 0; k < nr; ++k) {
                const int j = vars[k];
                int64_t *q = &inc[(size_t)k * RS];
                q[0] = outer ? t.cum[j] : t.cum[j] * 8;  // inner: byte offsets (buffer soffset)
                q[1] = (int64_t)1 << sh[c][j];
                if (outer) q[2] = ocum_p[j] * nE;
                for (int f = 0; f < nf; ++f) q[(outer ? 4 : 2) + f] = fs[f][j] * (JT_T_C * 8);
            }
            const size_t base = prog.tab.size();
            prog.tab.resize(base + (size_t)n * RS);
            int32_t *out = prog.tab.data() + base;
            int64_t cur[4 + JT_T_MAXF] = {0};
            std::vector<int> d(nr, 0);
            for (int64_t k = 0; k < n; ++k) {
                for (int q = 0; q < RS; ++q) out[k * RS + q] = (int32_t)cur[q];
                int i2 = nr - 1;
                while (i2 >= 0) {
                    const int jv = vars[i2];
                    if (++d[i2] < t.dims[jv]) {
                        for (int q = 0; q < RS; ++q) cur[q] += inc[(size_t)i2 * RS + q];
                        break;
                    }
                    for (int q = 0; q < RS; ++q) cur[q] -= inc[(size_t)i2 * RS + q] * (t.dims[jv] - 1);
                    d[i2--] = 0;
                }
            }
        };
        P.o_off = (int32_t)prog.tab.size();
        emit(RO, true);
        P.i_off = (int32_t)prog.tab.size();
        emit(RI, false);
        {  // the flattened R stream (outer x inner): per step the entry's R part (bytes: the kernel's
           // per-lane gather), and a step record {factor soffsets [nf], digit word, bin offset of the
           // inner run that ends here or -1}
            const int64_t nRo_ = Prod(t, RO), nRi_ = Prod(t, RI);
            const int32_t *ro = prog.tab.data() + P.o_off, *ri = prog.tab.data() + P.i_off;
            // loop tiling of the inner range (one wave per case group only): a wave-store factor that
            // varies with the inner variables but not the outer ones re-reads the same nRi x 4 rows in
            // every outer configuration, a cyclic stream an LRU of the wave's L2 share (kCacheRows)
            // misses in full when the rows exceed it.  Chunk-major order (for each chunk of the inner
            // range, every outer configuration) keeps one chunk's rows resident; a run's sum then adds
            // into its bin after the first chunk.  The chunk length is chosen by the same LRU model
            // over a prefix of the stream.  Opt-in (FBN_JT_TILING=1, read per plan): on the Munin-like
            // network it tiles 181 of 2320 passes (39 % of the steps), yet the kernel's measured
            // FETCH_SIZE does not drop (+2 %) and the extra bin read-modify-writes cost time (125k
            // cases: 239 ms tiled vs 204 ms untiled) -- the L2 is not the per-wave
            // LRU the model assumes.
            int64_t chunk = nRi_;
            {
                const bool no_tiling = !getenv("FBN_JT_TILING") || atoi(getenv("FBN_JT_TILING")) == 0;
                static const int64_t kCacheRowsT = getenv("FBN_JT_ORDER_ROWS") ? atoll(getenv("FBN_JT_ORDER_ROWS")) : 64;
                int64_t glob = 0;
                for (int j = P.nl; j < nf; ++j) glob += fac[j].sep->size();
                if (!no_tiling && TW == 1 && nf > P.nl && nRi_ >= 4 && nRo_ >= 2 && glob > kCacheRowsT) {
                    std::vector<std::vector<int64_t>> gp(nf);  // round 0's G parts (slot) of each factor
                    for (int j = P.nl; j < nf; ++j)
                        for (int64_t sl = 0; sl < std::min<int64_t>(nG, JT_T_L); ++sl)
                            gp[j].push_back(prog.tab[P.g_off + sl * (4 + nf) + 4 + j]);
                    const int K = (int)std::min<int64_t>(256, kCacheRowsT);
                    const int64_t kSteps = std::min<int64_t>(nRo_ * nRi_, 16384);
                    auto seq_misses = [&](int64_t q) -> int64_t {
                        std::vector<int64_t> prev(nf, -1), keys(K);
                        std::vector<uint64_t> stamp(K);
                        int used = 0;
                        uint64_t clk = 0;
                        int64_t miss = 0, k = 0;
                        for (int64_t c0 = 0; c0 < nRi_ && k < kSteps; c0 += q)
                            for (int64_t o = 0; o < nRo_ && k < kSteps; ++o)
                                for (int64_t i = c0; i < std::min(nRi_, c0 + q) && k < kSteps; ++i, ++k) {
                                    const int32_t *oq = ro + o * (4 + nf), *iq = ri + i * (2 + nf);
                                    for (int j = P.nl; j < nf; ++j) {
                                        const int64_t r = (int64_t)oq[4 + j] + iq[2 + j];
                                        if (r == prev[j]) continue;  // the kernel keeps the row it has
                                        prev[j] = r;
                                        for (int64_t g0 : gp[j]) {
                                            const int64_t key = ((int64_t)j << 40) | (g0 + r);
                                            ++clk;
                                            int hit = -1, lru = 0;
                                            for (int q2 = 0; q2 < used; ++q2) {
                                                if (keys[q2] == key) { hit = q2; break; }
                                                if (stamp[q2] < stamp[lru]) lru = q2;
                                            }
                                            if (hit >= 0) { stamp[hit] = clk; continue; }
                                            ++miss;
                                            if (used < K) keys[used] = key, stamp[used++] = clk;
                                            else keys[lru] = key, stamp[lru] = clk;
                                        }
                                    }
                                }
                        return miss;
                    };
                    const int64_t base = seq_misses(nRi_);
                    int64_t best = base;
                    for (int64_t dv = 2; dv <= 64 && dv <= nRi_; ++dv) {
                        const int64_t q = (nRi_ + dv - 1) / dv;
                        if (q == chunk) continue;
                        const int64_t m = seq_misses(q);
                        if (m < best) best = m, chunk = q;
                    }
                    if (best * 5 > base * 4) chunk = nRi_;  // (less than 20 % fewer modeled misses: untiled)
                }
            }
            P.chunk = (int32_t)chunk;
            std::vector<int32_t> et((size_t)(nRo_ * nRi_)), sr((size_t)(nRo_ * nRi_ * (nf + 2)));
            int64_t k = 0;
            for (int64_t c0 = 0; c0 < nRi_; c0 += chunk)
                for (int64_t o = 0; o < nRo_; ++o)
                    for (int64_t i = c0; i < std::min(nRi_, c0 + chunk); ++i, ++k) {
                    const int32_t *oq = ro + o * (4 + nf), *iq = ri + i * (2 + nf);
                    et[k] = oq[0] * 8 + iq[0];
                    int32_t *q = &sr[k * (nf + 2)];
                    // a wave's first step (outer-configuration split) loads every factor
                    bool wave_start = k == 0;
                    if (P.split == 1)
                        for (int w = 1; w < TW; ++w) wave_start |= k == (int64_t)P.nRo * w / TW * nRi_;
                    for (int f = 0; f < nf; ++f) {
                        q[f] = oq[4 + f] + iq[2 + f];
                        // bit 0 (offsets are multiples of a 128-byte row): the same row as the step
                        // before -- the kernel keeps the value it loaded then
                        if (!wave_start && q[f] == (sr[(k - 1) * (nf + 2) + f] & ~1)) q[f] |= 1;
                    }
                    q[nf] = (int32_t)((uint32_t)oq[1] | (uint32_t)iq[1]);
                    // end of a run: write its bin (first chunk) or add into it (later chunks)
                    q[nf + 1] = i == std::min(nRi_, c0 + chunk) - 1 ? (c0 == 0 ? oq[2] : -(oq[2] + 2)) : -1;
                }
            // padded by one chunk (JT_T_C steps, zero offsets, no bin): the kernel reads whole chunks
            et.resize(et.size() + JT_T_C, 0);
            for (int pad = 0; pad < JT_T_C; ++pad) {
                for (int f = 0; f < nf; ++f) sr.push_back(0);
                sr.push_back(0);
                sr.push_back(-1);
            }
            P.et_off = (int32_t)prog.tab.size();
            prog.tab.insert(prog.tab.end(), et.begin(), et.end());
            P.st_off = (int32_t)prog.tab.size();
            prog.tab.insert(prog.tab.end(), sr.begin(), sr.end());
        }
        uint32_t of = 0;
        for (int j : RO) of |= (uint32_t)fm[c][j] << sh[c][j];
        P.ofields = of;
        P.dest_row = (int32_t)dest_row;
        P.col_row = (int32_t)col_row;
        P.dest_sc = (int32_t)dest_sc;
        P.col_sc = (int32_t)col_sc_row;
        P.fsc_off = (int32_t)prog.tab.size();  // the factors' scale rows, in factor order
        for (int j = 0; j < nf; ++j) prog.tab.push_back((int32_t)fac[j].srow);
        // packed digits of every output bin, fields of the output variables in output order
        P.bdig_off = (int32_t)prog.tab.size();
        std::vector<int> osh(opos.size()), ofm(opos.size());
        {
            int bits = 0;
            for (size_t i = 0; i < opos.size(); ++i) {
                int w = 1;
                while ((1 << w) < t.dims[opos[i]]) ++w;
                osh[i] = bits, ofm[i] = (1 << w) - 1, bits += w;
            }
        }
        if (!mvars.empty()) {
            std::vector<int32_t> bd((size_t)nbins, 0);
            ForEachConfig(t, opos, [&](const std::vector<int> &d) {
                int64_t b = 0;
                uint32_t w = 0;
                for (size_t i = 0; i < opos.size(); ++i) b += d[i] * ocum[i], w |= (uint32_t)d[i] << osh[i];
                bd[(size_t)b] = (int32_t)w;
            });
            prog.tab.insert(prog.tab.end(), bd.begin(), bd.end());
        }
        P.nmv = (int32_t)mvars.size();
        P.mv_off = (int32_t)prog.tab.size();
        for (int v : mvars) {
            const int i = PosIn(plan.cliques[c].vars, v);
            const int oi = (int)(std::find(opos.begin(), opos.end(), i) - opos.begin());
            prog.tab.push_back(v);
            prog.tab.push_back((int32_t)out_off[v]);
            prog.tab.push_back(plan.dom[v]);
            prog.tab.push_back(osh[oi]);
            prog.tab.push_back(ofm[oi]);
        }
        P.iv_off = iv_off[c];
        P.nv = nv;
        P.vars_off = vars_off[c];
        P.first = first ? 1 : 0;
        P.nstage = first ? nstage : 0;
        P.stage_off = stage_off;
        prog.passes.push_back(P);
        prog.entry_visits += t.size();
        if (prog.tab.size() > (size_t)INT32_MAX / 2) return SetError(FBN_ERR_LIMIT, "device program too large for the tiled variant");
        return FBN_OK;
    };

    // factor placement of one clique phase: the smallest factors in LDS while they fit the per-wave
    // budget, the rest read from the wave store; staging records for the LDS ones
    auto place = [&](std::vector<Factor> &fac, int *nstage, int32_t *stage_off) {
        std::vector<size_t> idx(fac.size());
        for (size_t j = 0; j < fac.size(); ++j) idx[j] = j;
        std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return fac[a].sep->size() < fac[b].sep->size(); });
        *stage_off = (int32_t)prog.tab.size();
        *nstage = 0;
        int64_t off = 0;
        for (size_t j : idx) {
            if (off + fac[j].sep->size() <= budget_rows) {
                fac[j].lds_off = (int)(off * JT_T_C * 8);
                prog.tab.push_back((int32_t)fac[j].row);
                prog.tab.push_back((int32_t)fac[j].sep->size());
                prog.tab.push_back(fac[j].lds_off);
                off += fac[j].sep->size();
                ++*nstage;
            } else {
                fac[j].lds_off = -1;
            }
        }
        prog.lds_bytes = std::max<int64_t>(prog.lds_bytes, off * JT_T_C * 8);
    };

    int rc;
    // ---- Collect (post-order, the root has no upstream separator)
    for (int c : post) {
        if (c == plan.root) continue;
        std::vector<Factor> fac;
        for (int s : plan.clique_down[c]) fac.push_back({&plan.seps[s], col[s], col_sc[s], -1});
        int nst;
        int32_t so;
        place(fac, &nst, &so);
        const int s = plan.clique_up[c];
        const Table &sp = plan.seps[s];
        std::vector<int> opos;
        for (int v : sp.vars) opos.push_back(PosIn(plan.cliques[c].vars, v));
        if ((rc = build_pass(c, JT_T_COL, opos, std::vector<int64_t>(sp.cum.begin(), sp.cum.end()), sp.size(), fac,
                             col[s], -1, col_sc[s], -1, {}, true, nst, so)))
            return rc;
    }
    // ---- Distribute (pre-order): one pass per child, then the private variables
    for (int c : pre) {
        const Table &t = plan.cliques[c];
        std::vector<Factor> fac;
        for (int s : plan.clique_down[c]) fac.push_back({&plan.seps[s], col[s], col_sc[s], -1});
        const bool has_parent = c != plan.root;
        if (has_parent)
            fac.push_back({&plan.seps[plan.clique_up[c]], dis[plan.clique_up[c]], dis_sc[plan.clique_up[c]], -1});
        int nst;
        int32_t so;
        place(fac, &nst, &so);
        bool first = true;
        for (size_t ci = 0; ci < plan.clique_down[c].size(); ++ci) {
            const int s = plan.clique_down[c][ci];
            const Table &sp = plan.seps[s];
            std::vector<int> opos, mv;
            for (int v : sp.vars) opos.push_back(PosIn(t.vars, v));
            for (int v : sp.vars)
                if (src_sep[v] == s) mv.push_back(v);
            // the child's own Collect message M_i is constant on each output bin b and cancels in
            // SEPDIS: tmp(b) = M_i(b) U(b) / S, dis(b) = tmp(b) / M_i(b) = U(b) / S (0 where M_i(b) = 0),
            // S = sum_b M_i(b) U(b) -- so the pass multiplies every other factor and the post sweep
            // forms S from the bins
            std::vector<Factor> sub;
            for (size_t j = 0; j < fac.size(); ++j)
                if (j != ci) sub.push_back(fac[j]);
            if ((rc = build_pass(c, JT_T_DIS, opos, std::vector<int64_t>(sp.cum.begin(), sp.cum.end()), sp.size(), sub,
                                 dis[s], col[s], dis_sc[s], col_sc[s], mv, first, nst, so)))
                return rc;
            first = false;
        }
        if (!priv[c].empty()) {
            std::vector<int64_t> ocum(priv[c].size());
            int64_t m = 1;
            for (int i = (int)priv[c].size() - 1; i >= 0; --i) ocum[i] = m, m *= t.dims[priv[c][i]];
            std::vector<int> mv;
            for (int j : priv[c]) mv.push_back(t.vars[j]);
            if ((rc = build_pass(c, JT_T_MARG, priv[c], ocum, m, fac, -1, -1, -1, -1, mv, first, nst, so)))
                return rc;
        }
    }
    prog.red_row = prog.scr_row + max_x;
    prog.store_rows = prog.red_row + max_bins;
    if (prog.store_rows * JT_T_C * 8 > INT32_MAX) return SetError(FBN_ERR_LIMIT, "junction tree too large for the tiled variant");
    return FBN_OK;
}

}  // namespace fbn
