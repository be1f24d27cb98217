// jt_oracle.cpp -- TEST INFRASTRUCTURE.  CPU restatement of the reference junction tree; every
// function cites the reference code it restates (paths relative to the reference root).
#include "jt_oracle.h"

#include <algorithm>
#include <climits>
#include <cstdio>
#include <set>

namespace oracle {

void PTable::Rebuild() {
    int nv = (int)vars.size();
    cum.assign(nv, 1);
    for (int i = nv - 2; i >= 0; --i) cum[i] = cum[i + 1] * dims[i + 1];
    int s = nv ? cum[0] * dims[0] : 1;
    pot.resize(s);
}

static void Decode(const PTable &t, int idx, int *cfg) {  // src/PotentialTableBase.cpp:547-555
    for (size_t i = 0; i < t.vars.size(); ++i) {
        cfg[i] = idx / t.cum[i];
        idx %= t.cum[i];
    }
}

static int Loc(const PTable &t, int v) {  // GetVariableIndex, src/PotentialTableBase.cpp:531-538
    for (size_t i = 0; i < t.vars.size(); ++i)
        if (t.vars[i] == v) return (int)i;
    return (int)t.vars.size();
}

static void Normalize(PTable &t) {  // src/PotentialTableBase.cpp:433-445
    double den = 0;
    for (double p : t.pot) den += p;
    for (double &p : t.pot) p /= den;
}

// ---------------------------------------------------------------------------------------------
// static plan
void JTree::Build(const BayesNet &net) {
    bn = net;
    const int n = bn.n;
    // ConvertDAGNetworkToAdjacencyMatrix + Moralize, src/JunctionTreeStructure.cpp:70-115
    std::vector<std::vector<int>> adj(n, std::vector<int>(n, 0));
    for (int c = 0; c < n; ++c)
        for (int p : bn.parents_asc[c]) adj[p][c] = 1;
    std::set<std::pair<int, int>> marry;
    for (int i = 0; i < n; ++i) {
        std::vector<int> par;
        for (int j = 0; j < n; ++j)
            if (j != i && adj[j][i] == 1) par.push_back(j);
        for (size_t a = 0; a < par.size(); ++a)
            for (size_t b = a + 1; b < par.size(); ++b) marry.insert({par[a], par[b]});
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j)
            if (adj[i][j] == 1 || adj[j][i] == 1) adj[i][j] = adj[j][i] = 1;
    for (auto &p : marry) adj[p.first][p.second] = adj[p.second][p.first] = 1;

    // Triangulate: min-neighbour elimination, lowest index wins ties, subsumed cliques dropped
    // (src/JunctionTreeStructure.cpp:128-222)
    std::vector<std::set<int>> cliques;
    std::vector<bool> done(n, false);
    for (int step = 0; step < n; ++step) {
        int best = -1, best_nei = INT_MAX;
        for (int i = 0; i < n; ++i) {
            if (done[i]) continue;
            int k = 0;
            for (int j = 0; j < n; ++j) k += (adj[i][j] == 1);
            if (k < best_nei) {
                best_nei = k;
                best = i;
            }
        }
        std::vector<int> nei;
        for (int j = 0; j < n; ++j)
            if (adj[best][j] == 1) nei.push_back(j);
        std::set<int> cl{best};
        for (size_t a = 0; a < nei.size(); ++a) {
            for (size_t b = a + 1; b < nei.size(); ++b) adj[nei[a]][nei[b]] = adj[nei[b]][nei[a]] = 1;
            cl.insert(nei[a]);
        }
        bool subsumed = false;
        for (auto &c : cliques)
            if (std::includes(c.begin(), c.end(), cl.begin(), cl.end())) {
                subsumed = true;
                break;
            }
        if (!subsumed) cliques.push_back(cl);
        done[best] = true;
        for (int j : nei) adj[best][j] = adj[j][best] = 0;
    }
    const int nc = (int)cliques.size();

    // FormJunctionTree: candidate separators in (i,j) creation order (= pointer order of the
    // reference's set<Separator*>), Prim from clique 0, strict '<' keeps the first maximum
    // (src/JunctionTreeStructure.cpp:228-306)
    struct Cand {
        int a, b;
        std::set<int> vars;
    };
    std::vector<Cand> cand;
    for (int i = 0; i < nc; ++i)
        for (int j = i + 1; j < nc; ++j) {
            std::set<int> common;
            std::set_intersection(cliques[i].begin(), cliques[i].end(), cliques[j].begin(), cliques[j].end(),
                                  std::inserter(common, common.begin()));
            if (!common.empty()) cand.push_back({i, j, common});
        }
    std::vector<bool> in_tree(nc, false);
    in_tree[0] = true;
    int n_in = 1;
    std::vector<int> chosen;  // candidate ids in container (selection) order
    while (n_in < nc) {
        int best = -1;
        for (int k = 0; k < (int)cand.size(); ++k) {
            bool ia = in_tree[cand[k].a], ib = in_tree[cand[k].b];
            if (ia != ib && (best < 0 || cand[best].vars.size() < cand[k].vars.size())) best = k;
        }
        chosen.push_back(best);
        if (!in_tree[cand[best].a]) ++n_in, in_tree[cand[best].a] = true;
        if (!in_tree[cand[best].b]) ++n_in, in_tree[cand[best].b] = true;
    }
    const int ns = (int)chosen.size();
    // neighbour sets ordered by pointer = creation order
    std::vector<std::vector<int>> c_nbr(nc);  // separator container ids, by candidate id
    {
        std::vector<int> order(ns);
        for (int s = 0; s < ns; ++s) order[s] = s;
        std::sort(order.begin(), order.end(), [&](int x, int y) { return chosen[x] < chosen[y]; });
        for (int s : order) {
            c_nbr[cand[chosen[s]].a].push_back(s);
            c_nbr[cand[chosen[s]].b].push_back(s);
        }
    }

    // AssignPotentials: factor of each node (ascending vars) multiplied into the first clique
    // containing it (src/JunctionTreeStructure.cpp:312-348, src/PotentialTable.cpp:16-77,636-657)
    clique_init.assign(nc, PTable());
    for (int c = 0; c < nc; ++c) {
        PTable &t = clique_init[c];
        t.vars.assign(cliques[c].begin(), cliques[c].end());
        for (int v : t.vars) t.dims.push_back(bn.dom[v]);
        t.Rebuild();
        std::fill(t.pot.begin(), t.pot.end(), 1.0);
    }
    for (int v = 0; v < n; ++v) {
        std::set<int> fv(bn.parents_asc[v].begin(), bn.parents_asc[v].end());
        fv.insert(v);
        PTable f;
        f.vars.assign(fv.begin(), fv.end());
        for (int u : f.vars) f.dims.push_back(bn.dom[u]);
        f.Rebuild();
        std::vector<int> cfg(f.vars.size()), pv;
        for (int i = 0; i < f.size(); ++i) {
            Decode(f, i, cfg.data());
            pv.clear();
            int q = 0;
            for (size_t j = 0; j < f.vars.size(); ++j) {
                if (f.vars[j] == v) q = cfg[j];
                else pv.push_back(cfg[j]);  // parents in ascending order
            }
            f.pot[i] = bn.Prob(v, q, pv);
        }
        for (int c = 0; c < nc; ++c) {
            if (!std::includes(cliques[c].begin(), cliques[c].end(), fv.begin(), fv.end())) continue;
            PTable &t = clique_init[c];
            std::vector<int> tc(t.vars.size()), loc(f.vars.size());
            for (size_t j = 0; j < f.vars.size(); ++j) loc[j] = Loc(t, f.vars[j]);
            for (int e = 0; e < t.size(); ++e) {  // TableExtension + multiply
                Decode(t, e, tc.data());
                int fi = 0;
                for (size_t j = 0; j < f.vars.size(); ++j) fi += tc[loc[j]] * f.cum[j];
                t.pot[e] *= f.pot[fi];
            }
            break;
        }
    }
    sep_init.assign(ns, PTable());
    sep_up.assign(ns, -1);
    sep_down.assign(ns, -1);
    for (int s = 0; s < ns; ++s) {
        PTable &t = sep_init[s];
        const auto &vs = cand[chosen[s]].vars;
        t.vars.assign(vs.begin(), vs.end());
        for (int v : t.vars) t.dims.push_back(bn.dom[v]);
        t.Rebuild();
        std::fill(t.pot.begin(), t.pot.end(), 1.0);
    }

    // root = first clique with the fewest BFS levels (src/JunctionTree.cpp:15-24,187-225)
    auto bfs = [&](int r, std::vector<std::vector<int>> *lv, std::vector<int> *cup,
                   std::vector<std::vector<int>> *cdown, std::vector<int> *sup, std::vector<int> *sdown) {
        std::vector<int> up_c(nc, -2), up_s(ns, -2);  // -2: none; ids of the upstream node
        std::vector<int> cur{r};
        bool cur_is_sep = false;
        std::vector<std::vector<int>> levels_local{cur};
        up_c[r] = -1;
        while (!cur.empty()) {
            std::vector<int> nxt;
            for (int x : cur) {
                if (!cur_is_sep) {
                    for (int s : c_nbr[x]) {
                        if (up_c[x] == s) continue;
                        up_s[s] = x;
                        nxt.push_back(s);
                        if (cdown) (*cdown)[x].push_back(s);
                    }
                } else {
                    int a = cand[chosen[x]].a, b = cand[chosen[x]].b;
                    for (int c : {a, b}) {
                        if (up_s[x] == c) continue;
                        up_c[c] = x;
                        nxt.push_back(c);
                        if (sdown) (*sdown)[x] = c;
                    }
                }
            }
            levels_local.push_back(nxt);
            cur = nxt;
            cur_is_sep = !cur_is_sep;
        }
        levels_local.pop_back();
        if (lv) *lv = levels_local;
        if (cup) *cup = up_c;
        if (sup) *sup = up_s;
        return (int)levels_local.size();
    };
    int best_root = 0, min_lv = bfs(0, nullptr, nullptr, nullptr, nullptr, nullptr);
    for (int c = 1; c < nc; ++c) {
        int l = bfs(c, nullptr, nullptr, nullptr, nullptr, nullptr);
        if (l < min_lv) {
            min_lv = l;
            best_root = c;
        }
    }
    root = best_root;
    clique_down.assign(nc, {});
    std::vector<int> cup;
    bfs(root, &levels, &cup, &clique_down, &sep_up, &sep_down);
    clique_up = cup;

    // ReorganizeTableStorage: upstream separator vars become the trailing vars
    // (src/JunctionTree.cpp:235-281, src/PotentialTable.cpp:215-292)
    for (int c = 0; c < nc; ++c) {
        int s = clique_up[c];
        if (s < 0) continue;
        PTable &t = clique_init[c];
        const PTable &sp = sep_init[s];
        int nv = (int)t.vars.size(), nsv = (int)sp.vars.size();
        bool need = false;
        for (int j = 0; j < nsv; ++j)
            if (t.vars[nv - j - 1] != sp.vars[nsv - j - 1]) need = true;
        if (!need) continue;
        PTable nt;
        std::vector<int> from;  // from[k] = position in old table of new var k
        for (int i = 0; i < nv; ++i)
            if (std::find(sp.vars.begin(), sp.vars.end(), t.vars[i]) == sp.vars.end()) from.push_back(i);
        for (int v : sp.vars) from.push_back(Loc(t, v));
        for (int i : from) {
            nt.vars.push_back(t.vars[i]);
            nt.dims.push_back(t.dims[i]);
        }
        nt.Rebuild();
        std::vector<int> oc(nv);
        for (int k = 0; k < t.size(); ++k) {
            Decode(t, k, oc.data());
            int ni = 0;
            for (int l = 0; l < nv; ++l) ni += oc[from[l]] * nt.cum[l];
            nt.pot[ni] = t.pot[k];
        }
        t = nt;
    }
}

void JTree::DumpPlan(const std::string &plan_path, const std::string &init_path) const {
    FILE *f = fopen(plan_path.c_str(), "w");
    fprintf(f, "cliques %zu\n", clique_init.size());
    for (size_t i = 0; i < clique_init.size(); ++i) {
        const PTable &t = clique_init[i];
        fprintf(f, "c %zu %zu %d", i, t.vars.size(), t.size());
        for (int v : t.vars) fprintf(f, " %d", v);
        fprintf(f, " | up %d | down", clique_up[i]);
        for (int d : clique_down[i]) fprintf(f, " %d", d);
        fprintf(f, "\n");
    }
    fprintf(f, "seps %zu\n", sep_init.size());
    for (size_t i = 0; i < sep_init.size(); ++i) {
        const PTable &t = sep_init[i];
        fprintf(f, "s %zu %zu %d", i, t.vars.size(), t.size());
        for (int v : t.vars) fprintf(f, " %d", v);
        fprintf(f, " | up %d | down %d\n", sep_up[i], sep_down[i]);
    }
    fprintf(f, "root %d\n", root);
    fprintf(f, "levels %zu\n", levels.size());
    for (size_t l = 0; l < levels.size(); ++l) {
        fprintf(f, "level %zu %c", l, (l % 2) ? 's' : 'c');
        for (int x : levels[l]) fprintf(f, " %d", x);
        fprintf(f, "\n");
    }
    fclose(f);
    f = fopen(init_path.c_str(), "w");
    for (size_t i = 0; i < clique_init.size(); ++i) {
        fprintf(f, "c %zu %d", i, clique_init[i].size());
        for (double p : clique_init[i].pot) fprintf(f, " %.17g", p);
        fprintf(f, "\n");
    }
    fclose(f);
}

// ---------------------------------------------------------------------------------------------
// per case
static void Reduce(PTable &t, int var, int val) {  // TableReductionPost, src/PotentialTable.cpp:354-396
    int loc = Loc(t, var);
    std::vector<double> np;
    std::vector<int> cfg(t.vars.size());
    for (int i = 0; i < t.size(); ++i) {
        Decode(t, i, cfg.data());
        if (cfg[loc] == val) np.push_back(t.pot[i]);
    }
    t.vars.erase(t.vars.begin() + loc);
    t.dims.erase(t.dims.begin() + loc);
    t.Rebuild();
    t.pot = np;
    if (t.vars.empty()) t.pot.resize(1);
}

// index of parent entry k in a table over `sub` (sub's vars all in `t`)
static int MapToSub(const PTable &t, const PTable &sub, int k, std::vector<int> &cfg) {
    Decode(t, k, cfg.data());
    int idx = 0;
    for (size_t j = 0; j < sub.vars.size(); ++j) idx += cfg[Loc(t, sub.vars[j])] * sub.cum[j];
    return idx;
}

int JTree::Infer(const int8_t *ev, double *marg) const {
    std::vector<PTable> C = clique_init, S = sep_init;
    // LoadDiscreteEvidence: evidence in ascending var order (src/JunctionTree.cpp:316-383)
    for (int v = 0; v < bn.n; ++v) {
        if (ev[v] < 0) continue;
        for (auto &t : C)
            if (Loc(t, v) < (int)t.vars.size()) Reduce(t, v, ev[v]);
        for (auto &t : S)
            if (Loc(t, v) < (int)t.vars.size()) Reduce(t, v, ev[v]);
    }
    for (auto &t : C) Normalize(t);  // src/JunctionTree.cpp:1479-1483
    std::vector<int> cfg(64);
    const int L = (int)levels.size();
    // Collect, src/JunctionTree.cpp:1240-1306
    for (int i = L - 2; i >= 0; --i) {
        if (i % 2) {
            for (int s : levels[i]) {  // SeparatorLevelCollectionOptimized :1056-1148
                const PTable &ch = C[sep_down[s]];
                PTable &sp = S[s];
                int Ts = sp.size();
                std::vector<double> tmp(Ts, 0.0);
                for (int k = 0; k < ch.size(); ++k) tmp[k % Ts] += ch.pot[k];
                for (int k = 0; k < Ts; ++k) sp.pot[k] = (sp.pot[k] == 0) ? 0 : tmp[k] / sp.pot[k];
            }
        } else {
            size_t maxch = 0;
            for (int c : levels[i]) maxch = std::max(maxch, clique_down[c].size());
            for (size_t k = 0; k < maxch; ++k) {  // CliqueLevelCollection :829-941
                for (int c : levels[i]) {
                    if (clique_down[c].size() <= k) continue;
                    PTable &p = C[c];
                    const PTable &sp = S[clique_down[c][k]];
                    cfg.resize(p.vars.size() + 1);
                    for (int e = 0; e < p.size(); ++e) p.pot[e] *= sp.pot[MapToSub(p, sp, e, cfg)];
                }
                for (int c : levels[i])
                    if (clique_down[c].size() > k) Normalize(C[c]);
            }
        }
    }
    // Distribute, src/JunctionTree.cpp:1308-1333
    for (int i = 1; i < L; ++i) {
        if (i % 2) {
            for (int s : levels[i]) {  // SeparatorLevelDistribution :700-816
                const PTable &p = C[sep_up[s]];
                PTable &sp = S[s];
                std::vector<double> tmp(sp.size(), 0.0);
                cfg.resize(p.vars.size() + 1);
                for (int k = 0; k < p.size(); ++k) tmp[MapToSub(p, sp, k, cfg)] += p.pot[k];
                for (int k = 0; k < sp.size(); ++k) sp.pot[k] = (sp.pot[k] == 0) ? 0 : tmp[k] / sp.pot[k];
            }
        } else {
            for (int c : levels[i]) {  // CliqueLevelDistributionOptimized :1150-1238
                PTable &t = C[c];
                const PTable &sp = S[clique_up[c]];
                int Ts = sp.size();
                for (int k = 0; k < t.size(); ++k) t.pot[k] *= sp.pot[k % Ts];
                Normalize(t);
            }
        }
    }
    // outputs: GetProbabilitiesOneNode (:1392-1454) and InferenceUsingJT/ArgMax
    // (:1339-1380,1459-1467; src/Inference.cpp:92-102)
    int label = 0;
    int off = 0;
    for (int v = 0; v < bn.n; ++v) {
        int d = bn.dom[v];
        for (int j = 0; j < d; ++j) marg[off + j] = 0.0;
        if (ev[v] >= 0) {
            off += d;
            continue;
        }
        int best = -1, best_nv = INT_MAX;
        for (int c = 0; c < (int)C.size(); ++c) {
            int nv = (int)C[c].vars.size();
            if (nv >= best_nv) continue;
            if (Loc(C[c], v) == nv) continue;
            best = c;
            best_nv = nv;
        }
        const PTable &t = C[best];
        PTable pt;
        if (best_nv > 1) {
            pt.vars = {v};
            pt.dims = {d};
            pt.Rebuild();
            std::fill(pt.pot.begin(), pt.pot.end(), 0.0);
            int loc = Loc(t, v);
            cfg.resize(t.vars.size() + 1);
            for (int k = 0; k < t.size(); ++k) {
                Decode(t, k, cfg.data());
                pt.pot[cfg[loc]] += t.pot[k];
            }
        } else {
            pt = t;
        }
        if (v == 0) {
            // CalculateMarginalProbability returns the clique table itself (not re-normalized)
            // when it has 1 variable; otherwise the normalized marginal.  ArgMax: strict '>'.
            PTable q = pt;
            if (best_nv > 1) Normalize(q);
            double mp = 0;
            for (int i = 0; i < q.size(); ++i)
                if (q.pot[i] > mp) {
                    mp = q.pot[i];
                    label = i;
                }
        }
        Normalize(pt);
        for (int j = 0; j < d; ++j) marg[off + j] = pt.pot[j];
        off += d;
    }
    return label;
}

double Round7(double number) {  // src/Inference.cpp:195-206
    long long integerpart = (long long)number;
    number -= integerpart;
    for (unsigned i = 0; i < 7; ++i) number *= 10;
    number = (double)(long long)(number + 0.5);
    for (unsigned i = 0; i < 7; ++i) number /= 10;
    return integerpart + number;
}

}  // namespace oracle
