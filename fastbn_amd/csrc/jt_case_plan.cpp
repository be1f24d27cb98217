// jt_case_plan.cpp -- compiles the host plan into the per-case program of jt_case.hip (layout:
// jt_program.h, JtCClique / JT_C_VREC).
//
// What the kernel needs per clique is only index arithmetic: for every clique variable its
// domain, its stride in the clique table (row-major, left-most variable most significant, as
// ReorganizeTableStorage leaves it, src/JunctionTree.cpp:235-281) and its stride in each adjacent
// separator table (0 when the separator does not hold it).  Entry e of a case then meets
// separator entry sum_j digit_j(e) * stride_j -- the reference's Compute2DIndex / VariableIndex
// maps (src/PotentialTableBase.cpp, src/JunctionTree.cpp:700-816) as strides instead of tables.
// Schedules: Collect in DFS post-order (a clique after its children; the root needs no Collect
// pass of its own), Distribute in DFS pre-order, children in clique_down order (the reference's
// multiplication order of child messages, src/JunctionTree.cpp:1282-1302).
#include <algorithm>
#include <climits>

#include "fbn_internal.h"

namespace fbn {

namespace {
int PosOf(const Table &t, int v) {
    for (size_t i = 0; i < t.vars.size(); ++i)
        if (t.vars[i] == v) return (int)i;
    return -1;
}
}  // namespace

int CompileJTProgramC(const JTPlanHost &plan, JTProgramC &prog) {
    prog = JTProgramC();
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size(), V = plan.num_nodes;
    if (nc > 65535) return SetError(FBN_ERR_LIMIT, "%d cliques (per-case variant: max 65535)", nc);
    for (int d : plan.dom)
        if (d < 1 || d > 64) return SetError(FBN_ERR_LIMIT, "a domain of %d states (per-case variant: 1..64)", d);
    prog.num_cliques = nc;
    std::vector<int64_t> out_off(V);
    for (int v = 0; v < V; ++v) out_off[v] = prog.sum_dom, prog.sum_dom += plan.dom[v];
    // message slice: Collect messages of every separator, then the Distribute ones
    std::vector<int64_t> col(ns), dis(ns);
    int64_t m = 0;
    for (int s = 0; s < ns; ++s) col[s] = m, m += plan.seps[s].size();
    for (int s = 0; s < ns; ++s) dis[s] = m, m += plan.seps[s].size();
    if (m > INT32_MAX / 8) return SetError(FBN_ERR_LIMIT, "separators too large for the per-case variant");
    prog.msg_doubles = m;

    int64_t ivn = 0;
    for (int c = 0; c < nc; ++c) {
        const Table &t = plan.cliques[c];
        const int k = (int)plan.clique_down[c].size();
        if (k > JT_C_MAX_CHILDREN)
            return SetError(FBN_ERR_LIMIT, "clique %d has %d children (per-case variant: max %d)", c, k,
                            JT_C_MAX_CHILDREN);
        if (t.vars.size() > 64) return SetError(FBN_ERR_LIMIT, "clique with %zu variables (max 64)", t.vars.size());
        if (t.size() >= ((int64_t)1 << 26)) return SetError(FBN_ERR_LIMIT, "clique table of %lld entries", (long long)t.size());
        ivn += t.size();
        if (ivn > INT32_MAX / 8) return SetError(FBN_ERR_LIMIT, "clique tables too large for the per-case variant");
    }

    prog.cl.resize(nc);
    for (int c = 0; c < nc; ++c) {
        const Table &t = plan.cliques[c];
        const int nv = (int)t.vars.size(), k = (int)plan.clique_down[c].size();
        JtCClique &q = prog.cl[c];
        q.T = (int32_t)t.size();
        q.nv = nv;
        q.k = k;
        q.root = c == plan.root ? 1 : 0;
        q.id = c;
        q.iv_off = (int32_t)prog.initv.size();
        prog.initv.insert(prog.initv.end(), t.pot.begin(), t.pot.end());
        const Table *up = q.root ? nullptr : &plan.seps[plan.clique_up[c]];
        if (up) {
            const int s = plan.clique_up[c];
            q.up_Ts = (int32_t)up->size();
            q.up_col = (int32_t)col[s];
            q.up_dis = (int32_t)dis[s];
        }
        q.var_off = (int32_t)(prog.vrec.size() / JT_C_VREC);
        int maxdim = 1;
        for (int j = 0; j < nv; ++j) {
            const int v = t.vars[j];
            int32_t r[JT_C_VREC] = {0};
            r[0] = v;
            r[1] = t.dims[j];
            r[2] = t.cum[j];
            if (up) {
                const int l = PosOf(*up, v);
                r[3] = l >= 0 ? up->cum[l] : 0;
            }
            for (int i = 0; i < k; ++i) {
                const Table &sp = plan.seps[plan.clique_down[c][i]];
                const int l = PosOf(sp, v);
                r[4 + i] = l >= 0 ? sp.cum[l] : 0;
            }
            r[4 + JT_C_MAX_CHILDREN] = (int32_t)out_off[v];
            // division magic of the domain (jt_case.hip udiv_small): ceil(2^32 / d), 0 for d == 1
            r[5 + JT_C_MAX_CHILDREN] = t.dims[j] > 1 ? (int32_t)(uint32_t)((((uint64_t)1 << 32) + t.dims[j] - 1) / t.dims[j]) : 0;
            prog.vrec.insert(prog.vrec.end(), r, r + JT_C_VREC);
            maxdim = std::max(maxdim, t.dims[j]);
        }
        q.child_off = (int32_t)prog.aux.size();
        int64_t bins = 0;
        for (int i = 0; i < k; ++i) {
            const int s = plan.clique_down[c][i];
            prog.aux.push_back((int32_t)plan.seps[s].size());
            prog.aux.push_back((int32_t)col[s]);
            prog.aux.push_back((int32_t)dis[s]);
            bins += plan.seps[s].size();
        }
        bins += 4 * maxdim;  // up to 4 marginals ride on one Distribute pass
        q.dbins = (int32_t)bins;
        prog.max_bins = (int32_t)std::max<int64_t>(prog.max_bins, std::max<int64_t>(bins, q.up_Ts));
    }

    // DFS orders (iterative)
    {
        std::vector<std::pair<int, size_t>> st{{plan.root, 0}};
        while (!st.empty()) {
            auto &top = st.back();
            const int c = top.first;
            if (top.second == 0) prog.pre.push_back(c);
            if (top.second < plan.clique_down[c].size()) {
                const int ch = plan.sep_down[plan.clique_down[c][top.second++]];
                st.push_back({ch, 0});
            } else {
                if (c != plan.root) prog.post.push_back(c);
                st.pop_back();
            }
        }
        if ((int)prog.pre.size() != nc)
            return SetError(FBN_ERR_LIMIT, "tree traversal covers %zu of %d cliques", prog.pre.size(), nc);
    }

    // per variable: candidate cliques in container order (GetProbabilitiesOneNode's scan,
    // src/JunctionTree.cpp:1412-1434) and the output slot
    std::vector<std::vector<int>> cand(V);
    for (int c = 0; c < nc; ++c)
        for (int v : plan.cliques[c].vars) cand[v].push_back(c);
    for (int v = 0; v < V; ++v) {
        if (cand[v].empty()) return SetError(FBN_ERR_ARG, "variable %d appears in no clique", v);
        prog.vsel.push_back((int32_t)prog.aux.size());
        prog.vsel.push_back((int32_t)cand[v].size());
        prog.vsel.push_back((int32_t)out_off[v]);
        prog.vsel.push_back(plan.dom[v]);
        prog.aux.insert(prog.aux.end(), cand[v].begin(), cand[v].end());
    }
    if (prog.aux.size() > (size_t)INT32_MAX) return SetError(FBN_ERR_LIMIT, "device program too large");
    return FBN_OK;
}

}  // namespace fbn
