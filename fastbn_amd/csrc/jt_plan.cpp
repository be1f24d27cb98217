// jt_plan.cpp -- case-independent junction-tree plan (host) and its compilation into the device
// program interpreted by jt_kernels.hip.
//
// BuildJTPlan reproduces the reference's tree exactly (the parity fixtures compare the dump with
// the reference's own, tests/golden/alarm_1k.plan): moralization, min-neighbour triangulation
// with lowest-index ties, Prim over separator candidates taken in creation order (the pointer
// order of the reference's std::set<Separator*>), root = first clique with the fewest BFS levels,
// MarkLevel order, CPT factors multiplied into the first containing clique in node order, and
// ReorganizeTableStorage putting each clique's upstream separator variables last.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <numeric>

#include "fbn_internal.h"

namespace fbn {

void Table::Rebuild() {
    const int nv = (int)vars.size();
    cum.assign(nv, 1);
    for (int i = nv - 2; i >= 0; --i) cum[i] = cum[i + 1] * dims[i + 1];  // src/PotentialTableBase.cpp:599-607
    pot.resize(nv ? (size_t)cum[0] * dims[0] : 1);
}

namespace {

// adjacency as one bitset row per node: cheap neighbour counts for the O(n^2) elimination loop
struct BitGraph {
    int n, words;
    std::vector<uint64_t> bits;
    explicit BitGraph(int n_) : n(n_), words((n_ + 63) / 64), bits((size_t)n_ * ((n_ + 63) / 64), 0) {}
    bool get(int i, int j) const { return (bits[(size_t)i * words + j / 64] >> (j % 64)) & 1; }
    void set(int i, int j, bool v) {
        uint64_t &w = bits[(size_t)i * words + j / 64];
        if (v) w |= 1ull << (j % 64);
        else w &= ~(1ull << (j % 64));
    }
    int degree(int i) const {
        int d = 0;
        for (int w = 0; w < words; ++w) d += __builtin_popcountll(bits[(size_t)i * words + w]);
        return d;
    }
};

int LocOf(const Table &t, int v) {
    for (size_t i = 0; i < t.vars.size(); ++i)
        if (t.vars[i] == v) return (int)i;
    return -1;
}

}  // namespace

int BuildJTPlan(const Network &net, JTPlanHost &plan) {
    const int n = net.n();
    plan = JTPlanHost();
    plan.num_nodes = n;
    plan.dom = net.dom;

    // moral graph (ConvertDAGNetworkToAdjacencyMatrix + Moralize, src/JunctionTreeStructure.cpp:70-115)
    BitGraph g(n);
    for (int c = 0; c < n; ++c)
        for (int p : net.parents_asc[c]) {
            g.set(p, c, true);
            g.set(c, p, true);
        }
    for (int c = 0; c < n; ++c) {
        const auto &pa = net.parents_asc[c];
        for (size_t a = 0; a < pa.size(); ++a)
            for (size_t b = a + 1; b < pa.size(); ++b) {
                g.set(pa[a], pa[b], true);
                g.set(pa[b], pa[a], true);
            }
    }

    // triangulation by repeated min-neighbour elimination (src/JunctionTreeStructure.cpp:128-222)
    std::vector<std::vector<int>> cliques;  // sorted variable lists, creation = container order
    std::vector<bool> done(n, false);
    for (int step = 0; step < n; ++step) {
        int best = -1, best_deg = INT_MAX;
        for (int i = 0; i < n; ++i) {
            if (done[i]) continue;
            int d = g.degree(i);
            if (d < best_deg) best_deg = d, best = i;
        }
        std::vector<int> nei;
        for (int j = 0; j < n; ++j)
            if (g.get(best, j)) nei.push_back(j);
        for (size_t a = 0; a < nei.size(); ++a)
            for (size_t b = a + 1; b < nei.size(); ++b) {
                g.set(nei[a], nei[b], true);
                g.set(nei[b], nei[a], true);
            }
        std::vector<int> cl = nei;
        cl.push_back(best);
        std::sort(cl.begin(), cl.end());
        bool subsumed = false;
        for (const auto &c : cliques)
            if (std::includes(c.begin(), c.end(), cl.begin(), cl.end())) {
                subsumed = true;
                break;
            }
        if (!subsumed) cliques.push_back(cl);
        done[best] = true;
        for (int j : nei) {
            g.set(best, j, false);
            g.set(j, best, false);
        }
    }
    const int nc = (int)cliques.size();

    // Prim maximum spanning tree over separator candidates (src/JunctionTreeStructure.cpp:228-306)
    struct Cand {
        int a, b;
        std::vector<int> vars;
    };
    std::vector<Cand> cand;
    for (int i = 0; i < nc; ++i)
        for (int j = i + 1; j < nc; ++j) {
            std::vector<int> common;
            std::set_intersection(cliques[i].begin(), cliques[i].end(), cliques[j].begin(), cliques[j].end(),
                                  std::back_inserter(common));
            if (!common.empty()) cand.push_back({i, j, std::move(common)});
        }
    std::vector<char> in_tree(nc, 0);
    in_tree[0] = 1;
    int n_in = 1;
    std::vector<int> chosen;
    while (n_in < nc) {
        int best = -1;
        size_t best_w = 0;
        for (int k = 0; k < (int)cand.size(); ++k) {
            if (in_tree[cand[k].a] == in_tree[cand[k].b]) continue;
            if (best < 0 || best_w < cand[k].vars.size()) best = k, best_w = cand[k].vars.size();
        }
        if (best < 0) return SetError(FBN_ERR_ARG, "moral graph is disconnected: junction forest unsupported");
        chosen.push_back(best);
        for (int c : {cand[best].a, cand[best].b})
            if (!in_tree[c]) in_tree[c] = 1, ++n_in;
    }
    const int ns = (int)chosen.size();
    std::vector<std::vector<int>> c_nbr(nc);  // separators of a clique in creation (pointer) order
    {
        std::vector<int> by_creation(ns);
        std::iota(by_creation.begin(), by_creation.end(), 0);
        std::sort(by_creation.begin(), by_creation.end(), [&](int x, int y) { return chosen[x] < chosen[y]; });
        for (int s : by_creation) {
            c_nbr[cand[chosen[s]].a].push_back(s);
            c_nbr[cand[chosen[s]].b].push_back(s);
        }
    }

    // initial clique potentials: all-ones tables times the CPT factors
    // (AssignPotentials src/JunctionTreeStructure.cpp:312-348, PotentialTable(node) ctor
    //  src/PotentialTable.cpp:16-77, TableMultiplication :636-657)
    plan.cliques.assign(nc, Table());
    for (int c = 0; c < nc; ++c) {
        Table &t = plan.cliques[c];
        t.vars = cliques[c];
        for (int v : t.vars) t.dims.push_back(net.dom[v]);
        t.Rebuild();
        std::fill(t.pot.begin(), t.pot.end(), 1.0);
    }
    for (int v = 0; v < n; ++v) {
        std::vector<int> fv = net.parents_asc[v];
        fv.push_back(v);
        std::sort(fv.begin(), fv.end());
        Table f;
        f.vars = fv;
        for (int u : fv) f.dims.push_back(net.dom[u]);
        f.Rebuild();
        const int fn = (int)fv.size();
        std::vector<int> cfg(fn), pv;
        for (int64_t i = 0; i < f.size(); ++i) {
            int64_t r = i;
            for (int j = 0; j < fn; ++j) cfg[j] = (int)(r / f.cum[j]), r %= f.cum[j];
            pv.clear();
            int q = 0;
            for (int j = 0; j < fn; ++j) {
                if (fv[j] == v) q = cfg[j];
                else pv.push_back(cfg[j]);
            }
            f.pot[i] = net.Prob(v, q, pv.data());
        }
        for (int c = 0; c < nc; ++c) {
            if (!std::includes(cliques[c].begin(), cliques[c].end(), fv.begin(), fv.end())) continue;
            Table &t = plan.cliques[c];
            const int tn = (int)t.vars.size();
            std::vector<int> loc(fn), tc(tn);
            for (int j = 0; j < fn; ++j) loc[j] = LocOf(t, fv[j]);
            for (int64_t e = 0; e < t.size(); ++e) {
                int64_t r = e;
                for (int j = 0; j < tn; ++j) tc[j] = (int)(r / t.cum[j]), r %= t.cum[j];
                int64_t fi = 0;
                for (int j = 0; j < fn; ++j) fi += (int64_t)tc[loc[j]] * f.cum[j];
                t.pot[e] *= f.pot[fi];
            }
            break;
        }
    }
    plan.seps.assign(ns, Table());
    for (int s = 0; s < ns; ++s) {
        Table &t = plan.seps[s];
        t.vars = cand[chosen[s]].vars;
        for (int v : t.vars) t.dims.push_back(net.dom[v]);
        t.Rebuild();
        std::fill(t.pot.begin(), t.pot.end(), 1.0);
    }

    // root selection and levelling (src/JunctionTree.cpp:15-24, 137-225)
    auto bfs = [&](int r, bool record) {
        std::vector<int> up_c(nc, -2), up_s(ns, -2);
        up_c[r] = -1;
        std::vector<int> cur{r};
        std::vector<std::vector<int>> lv{cur};
        bool sep_level = false;
        if (record) {
            plan.clique_down.assign(nc, {});
            plan.sep_down.assign(ns, -1);
        }
        while (!cur.empty()) {
            std::vector<int> nxt;
            for (int x : cur) {
                if (!sep_level) {
                    for (int s : c_nbr[x]) {
                        if (up_c[x] == s) continue;
                        up_s[s] = x;
                        nxt.push_back(s);
                        if (record) plan.clique_down[x].push_back(s);
                    }
                } else {
                    for (int c : {cand[chosen[x]].a, cand[chosen[x]].b}) {
                        if (up_s[x] == c) continue;
                        up_c[c] = x;
                        nxt.push_back(c);
                        if (record) plan.sep_down[x] = c;
                    }
                }
            }
            lv.push_back(nxt);
            cur.swap(nxt);
            sep_level = !sep_level;
        }
        lv.pop_back();
        if (record) {
            plan.levels = lv;
            plan.clique_up = up_c;
            plan.sep_up = up_s;
        }
        return (int)lv.size();
    };
    int root = 0, min_lv = bfs(0, false);
    for (int c = 1; c < nc; ++c) {
        int l = bfs(c, false);
        if (l < min_lv) min_lv = l, root = c;
    }
    plan.root = root;
    bfs(root, true);

    // ReorganizeTableStorage (src/JunctionTree.cpp:235-281, TableReorganizationPre/Main/Post
    // src/PotentialTable.cpp:215-292)
    for (int c = 0; c < nc; ++c) {
        int s = plan.clique_up[c];
        if (s < 0) continue;
        Table &t = plan.cliques[c];
        const Table &sp = plan.seps[s];
        const int nv = (int)t.vars.size(), nsv = (int)sp.vars.size();
        bool need = false;
        for (int j = 0; j < nsv; ++j)
            if (t.vars[nv - 1 - j] != sp.vars[nsv - 1 - j]) need = true;
        if (!need) continue;
        std::vector<int> from;
        for (int i = 0; i < nv; ++i)
            if (std::find(sp.vars.begin(), sp.vars.end(), t.vars[i]) == sp.vars.end()) from.push_back(i);
        for (int v : sp.vars) from.push_back(LocOf(t, v));
        Table nt;
        for (int i : from) nt.vars.push_back(t.vars[i]), nt.dims.push_back(t.dims[i]);
        nt.Rebuild();
        std::vector<int> oc(nv);
        for (int64_t k = 0; k < t.size(); ++k) {
            int64_t r = k;
            for (int j = 0; j < nv; ++j) oc[j] = (int)(r / t.cum[j]), r %= t.cum[j];
            int64_t ni = 0;
            for (int l = 0; l < nv; ++l) ni += (int64_t)oc[from[l]] * nt.cum[l];
            nt.pot[ni] = t.pot[k];
        }
        t = std::move(nt);
    }
    return FBN_OK;
}

// ---------------------------------------------------------------------------------------------
// program compiler
int CompileJTProgram(const JTPlanHost &plan, JTProgram &prog) {
    prog = JTProgram();
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size();
    std::vector<int64_t> coff(nc), soff(ns);
    int64_t off = 0;
    for (int c = 0; c < nc; ++c) coff[c] = off, off += plan.cliques[c].size();
    for (int s = 0; s < ns; ++s) soff[s] = off, off += plan.seps[s].size();
    const int64_t den0 = off;
    prog.state_entries = off + nc;
    prog.num_cliques = nc;
    if (prog.state_entries > INT32_MAX / 2) return SetError(FBN_ERR_LIMIT, "junction tree too large (%lld entries)", (long long)off);
    for (int d : plan.dom) prog.sum_dom += d;

    auto op = [&](int32_t type, int64_t a, int64_t b, int64_t c, int64_t d, int64_t e, int64_t f = 0, int64_t g = 0,
                  int64_t h = 0) {
        JtOp o{type, (int32_t)a, (int32_t)b, (int32_t)c, (int32_t)d, (int32_t)e, (int32_t)f, (int32_t)g, (int32_t)h, 0};
        prog.ops.push_back(o);
    };
    // INIT: masked initial potentials; digits packed 8 bits per variable slot, 8 slots per word
    auto emit_init = [&](const Table &t, int64_t toff, int den_idx, int clique_id) {
        const int nv = (int)t.vars.size();
        prog.max_vars = std::max(prog.max_vars, nv);
        if (nv > 8 * JT_MAX_DIG_WORDS) return SetError(FBN_ERR_LIMIT, "table with %d variables (max %d)", nv, 8 * JT_MAX_DIG_WORDS);
        const int nw = std::max(1, (nv + 7) / 8);
        int64_t vars_off = (int64_t)prog.aux.size();
        for (int v : t.vars) prog.aux.push_back(v);
        int64_t dig_off = (int64_t)prog.dig.size();
        for (int64_t e = 0; e < t.size(); ++e) {
            uint64_t w[JT_MAX_DIG_WORDS] = {0, 0, 0, 0};
            int64_t r = e;
            for (int j = 0; j < nv; ++j) {
                uint64_t digit = (uint64_t)(r / t.cum[j]);
                r %= t.cum[j];
                w[j / 8] |= digit << (8 * (j % 8));
            }
            for (int k = 0; k < nw; ++k) prog.dig.push_back(w[k]);
        }
        int64_t init_off = (int64_t)prog.initv.size();
        prog.initv.insert(prog.initv.end(), t.pot.begin(), t.pot.end());
        op(JT_OP_INIT, toff, t.size(), vars_off, nv, dig_off, den_idx, clique_id, init_off);
        return (int)FBN_OK;
    };
    for (int c = 0; c < nc; ++c) {
        int rc = emit_init(plan.cliques[c], coff[c], (int)(den0 + c), c);
        if (rc) return rc;
    }
    for (int s = 0; s < ns; ++s) {
        int rc = emit_init(plan.seps[s], soff[s], -1, -1);
        if (rc) return rc;
    }
    // map from a clique entry to the index of a separator over a subset of its variables
    auto sub_index = [&](const Table &t, const Table &sub, int64_t e) {
        int64_t r = e, idx = 0;
        for (size_t j = 0; j < t.vars.size(); ++j) {
            int64_t digit = r / t.cum[j];
            r %= t.cum[j];
            int l = LocOf(sub, t.vars[j]);
            if (l >= 0) idx += digit * sub.cum[l];
        }
        return idx;
    };
    const int L = (int)plan.levels.size();
    // Collect (src/JunctionTree.cpp:1240-1306)
    for (int i = L - 2; i >= 0; --i) {
        if (i % 2) {
            for (int s : plan.levels[i]) {
                int c = plan.sep_down[s];
                op(JT_OP_SEPCOL, soff[s], plan.seps[s].size(), coff[c], plan.cliques[c].size(), den0 + c);
            }
        } else {
            size_t maxch = 0;
            for (int c : plan.levels[i]) maxch = std::max(maxch, plan.clique_down[c].size());
            for (size_t k = 0; k < maxch; ++k)
                for (int c : plan.levels[i]) {
                    if (plan.clique_down[c].size() <= k) continue;
                    int s = plan.clique_down[c][k];
                    const Table &t = plan.cliques[c];
                    int64_t map_off = (int64_t)prog.aux.size();
                    for (int64_t e = 0; e < t.size(); ++e) prog.aux.push_back((int32_t)sub_index(t, plan.seps[s], e));
                    op(JT_OP_CLQMUL, coff[c], t.size(), den0 + c, soff[s], map_off);
                }
        }
    }
    // Distribute (src/JunctionTree.cpp:1308-1333)
    for (int i = 1; i < L; ++i) {
        if (i % 2) {
            for (int s : plan.levels[i]) {
                int c = plan.sep_up[s];
                const Table &t = plan.cliques[c];
                const int64_t Ts = plan.seps[s].size(), per = t.size() / Ts;
                std::vector<std::vector<int32_t>> lists(Ts);
                for (int64_t e = 0; e < t.size(); ++e) lists[sub_index(t, plan.seps[s], e)].push_back((int32_t)e);
                int64_t list_off = (int64_t)prog.aux.size();
                for (auto &l : lists) {
                    if ((int64_t)l.size() != per) return SetError(FBN_ERR_ARG, "internal: ragged separator map");
                    prog.aux.insert(prog.aux.end(), l.begin(), l.end());
                }
                op(JT_OP_SEPDIS, soff[s], Ts, coff[c], den0 + c, list_off, per);
            }
        } else {
            for (int c : plan.levels[i]) {
                int s = plan.clique_up[c];
                op(JT_OP_CLQDIS, coff[c], plan.cliques[c].size(), den0 + c, soff[s], plan.seps[s].size());
            }
        }
    }
    // outputs (GetProbabilitiesOneNode src/JunctionTree.cpp:1392-1454; InferenceUsingJT :1459-1467)
    int out_off = 0;
    for (int v = 0; v < plan.num_nodes; ++v) {
        int64_t cand_off = (int64_t)prog.aux.size();
        int ncand = 0;
        for (int c = 0; c < nc; ++c) {
            const Table &t = plan.cliques[c];
            int l = LocOf(t, v);
            if (l < 0) continue;
            prog.aux.insert(prog.aux.end(), {c, (int32_t)coff[c], (int32_t)(den0 + c), (int32_t)t.vars.size(),
                                             (int32_t)t.cum[l], (int32_t)t.size()});
            ++ncand;
        }
        if (ncand == 0) return SetError(FBN_ERR_ARG, "variable %d appears in no clique", v);
        op(JT_OP_MARG, out_off, plan.dom[v], cand_off, ncand, v, v == 0 ? 1 : 0);
        out_off += plan.dom[v];
    }
    if (prog.aux.size() > (size_t)INT32_MAX) return SetError(FBN_ERR_LIMIT, "device program too large");
    return FBN_OK;
}

}  // namespace fbn

// ---------------------------------------------------------------------------------------------
// LDS-resident program: cliques one at a time (see jt_program.h)
namespace fbn {

int CompileJTProgramLDS(const JTPlanHost &plan, JTProgramLDS &prog) {
    prog = JTProgramLDS();
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size();
    prog.num_cliques = nc;
    for (int d : plan.dom) prog.sum_dom += d;
    std::vector<int64_t> store_off(nc, -1), sep_off(ns);
    for (int c = 0; c < nc; ++c) {
        prog.max_table = std::max<int64_t>(prog.max_table, plan.cliques[c].size());
        if (c == plan.root) continue;  // the root never leaves LDS between the two phases
        store_off[c] = prog.store_entries;
        prog.store_entries += plan.cliques[c].size();
    }
    for (int s = 0; s < ns; ++s) sep_off[s] = prog.sep_entries, prog.sep_entries += plan.seps[s].size();
    if (prog.store_entries + prog.sep_entries + prog.max_table > INT32_MAX / 64)
        return SetError(FBN_ERR_LIMIT, "junction tree too large for the LDS program");

    auto op = [&](int32_t type, int64_t a, int64_t b, int64_t c, int64_t d, int64_t e, int64_t f = 0, int64_t g = 0,
                  int64_t h = 0, int64_t pad = 0) {
        prog.ops.push_back(JtOp{type, (int32_t)a, (int32_t)b, (int32_t)c, (int32_t)d, (int32_t)e, (int32_t)f,
                                (int32_t)g, (int32_t)h, (int32_t)pad});
    };
    auto sub_index = [&](const Table &t, const Table &sub, int64_t e) {
        int64_t r = e, idx = 0;
        for (size_t j = 0; j < t.vars.size(); ++j) {
            int64_t digit = r / t.cum[j];
            r %= t.cum[j];
            int l = LocOf(sub, t.vars[j]);
            if (l >= 0) idx += digit * sub.cum[l];
        }
        return idx;
    };
    auto emit_init = [&](int c) -> int {
        const Table &t = plan.cliques[c];
        const int nv = (int)t.vars.size();
        if (nv > 8 * JT_MAX_DIG_WORDS) return SetError(FBN_ERR_LIMIT, "clique with %d variables (max %d)", nv, 8 * JT_MAX_DIG_WORDS);
        const int nw = std::max(1, (nv + 7) / 8);
        int64_t vars_off = (int64_t)prog.aux.size();
        for (int v : t.vars) prog.aux.push_back(v);
        int64_t dig_off = (int64_t)prog.dig.size();
        for (int64_t e = 0; e < t.size(); ++e) {
            uint64_t w[JT_MAX_DIG_WORDS] = {0, 0, 0, 0};
            int64_t r = e;
            for (int j = 0; j < nv; ++j) {
                w[j / 8] |= (uint64_t)(r / t.cum[j]) << (8 * (j % 8));
                r %= t.cum[j];
            }
            for (int k = 0; k < nw; ++k) prog.dig.push_back(w[k]);
        }
        int64_t init_off = (int64_t)prog.initv.size();
        prog.initv.insert(prog.initv.end(), t.pot.begin(), t.pot.end());
        op(JT_L_INIT, 0, t.size(), vars_off, nv, dig_off, 0, c, init_off);
        return FBN_OK;
    };
    // candidate cliques per variable, container order (GetProbabilitiesOneNode's scan)
    std::vector<std::vector<int>> cand(plan.num_nodes);
    for (int c = 0; c < nc; ++c)
        for (int v : plan.cliques[c].vars) cand[v].push_back(c);
    std::vector<int64_t> cand_off(plan.num_nodes), out_off(plan.num_nodes);
    int64_t oo = 0;
    for (int v = 0; v < plan.num_nodes; ++v) {
        if (cand[v].empty()) return SetError(FBN_ERR_ARG, "variable %d appears in no clique", v);
        cand_off[v] = (int64_t)prog.aux.size();
        prog.aux.insert(prog.aux.end(), cand[v].begin(), cand[v].end());
        out_off[v] = oo;
        oo += plan.dom[v];
    }

    const int L = (int)plan.levels.size();
    // Collect: clique levels deepest first (src/JunctionTree.cpp:1240-1306)
    for (int i = ((L - 1) / 2) * 2; i >= 0; i -= 2) {
        for (int c : plan.levels[i]) {
            const Table &t = plan.cliques[c];
            int rc = emit_init(c);
            if (rc) return rc;
            for (int s : plan.clique_down[c]) {
                const int64_t Ts = plan.seps[s].size(), per = t.size() / Ts;
                std::vector<std::vector<int32_t>> lists(Ts);
                for (int64_t e = 0; e < t.size(); ++e) lists[sub_index(t, plan.seps[s], e)].push_back((int32_t)e);
                int64_t list_off = (int64_t)prog.aux.size();
                for (auto &l : lists) {
                    if ((int64_t)l.size() != per) return SetError(FBN_ERR_ARG, "internal: ragged separator map");
                    prog.aux.insert(prog.aux.end(), l.begin(), l.end());
                }
                op(JT_L_MUL, 0, t.size(), Ts, sep_off[s], list_off);
            }
            if (c != plan.root) {
                int s = plan.clique_up[c];
                op(JT_L_SEPCOL, sep_off[s], plan.seps[s].size(), t.size(), 0, 0);
                op(JT_L_STORE, store_off[c], t.size(), c, 0, 0);
            }
        }
    }
    // Distribute: clique levels root first (src/JunctionTree.cpp:1308-1333) + outputs
    for (int i = 0; i < L; i += 2) {
        for (int c : plan.levels[i]) {
            const Table &t = plan.cliques[c];
            if (c != plan.root) {
                int s = plan.clique_up[c];
                op(JT_L_LOAD, store_off[c], t.size(), c, 0, 0);
                op(JT_L_DMUL, 0, t.size(), 0, sep_off[s], plan.seps[s].size());
            }
            for (int s : plan.clique_down[c]) {
                const int64_t Ts = plan.seps[s].size(), per = t.size() / Ts;
                std::vector<std::vector<int32_t>> lists(Ts);
                for (int64_t e = 0; e < t.size(); ++e) lists[sub_index(t, plan.seps[s], e)].push_back((int32_t)e);
                int64_t list_off = (int64_t)prog.aux.size();
                for (auto &l : lists) {
                    if ((int64_t)l.size() != per) return SetError(FBN_ERR_ARG, "internal: ragged separator map");
                    prog.aux.insert(prog.aux.end(), l.begin(), l.end());
                }
                op(JT_L_SEPDIS, sep_off[s], Ts, 0, 0, list_off, per);
            }
            for (size_t j = 0; j < t.vars.size(); ++j) {
                int v = t.vars[j];
                op(JT_L_MARG, out_off[v], plan.dom[v], cand_off[v], (int64_t)cand[v].size(), v, v == 0 ? 1 : 0, c,
                   t.cum[j], t.size());
            }
        }
    }
    for (int v = 0; v < plan.num_nodes; ++v) op(JT_L_EVZERO, out_off[v], plan.dom[v], 0, 0, v);
    if (prog.aux.size() > (size_t)INT32_MAX) return SetError(FBN_ERR_LIMIT, "device program too large");
    return FBN_OK;
}

}  // namespace fbn
