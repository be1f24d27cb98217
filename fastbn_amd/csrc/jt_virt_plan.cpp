// jt_virt_plan.cpp -- compiles the host plan into the streamed ("virtual table") program of
// jt_virt.hip (descriptor layout: jt_program.h, JtVClique).
//
// Per-wave store rows (64 lanes x fp64 each): [Collect messages | Distribute messages | step
// denominators].  Collect visits the cliques in DFS post-order, Distribute in DFS pre-order: a
// clique's Collect result depends only on its subtree and the fixed order of its child messages
// (clique_down = the reference's k-th-child rounds, src/JunctionTree.cpp:1282-1302), its Distribute
// result only on its parent's message, so the values are the reference's level-order values.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "fbn_internal.h"

namespace fbn {

namespace {

int LocOfV(const Table &t, int v) {
    for (size_t i = 0; i < t.vars.size(); ++i)
        if (t.vars[i] == v) return (int)i;
    return -1;
}

// index into `sub` of entry e of `t` (sub's variables are a subset of t's)
int64_t SubIndex(const Table &t, const Table &sub, int64_t e) {
    int64_t r = e, idx = 0;
    for (size_t j = 0; j < t.vars.size(); ++j) {
        const int64_t digit = r / t.cum[j];
        r %= t.cum[j];
        const int l = LocOfV(sub, t.vars[j]);
        if (l >= 0) idx += digit * sub.cum[l];
    }
    return idx;
}

}  // namespace

int CompileJTProgramV(const JTPlanHost &plan, JTProgramV &prog) {
    prog = JTProgramV();
    const int nc = (int)plan.cliques.size(), ns = (int)plan.seps.size(), V = plan.num_nodes;
    prog.num_cliques = nc;
    for (int d : plan.dom) prog.sum_dom += d;
    for (int c = 0; c < nc; ++c) {
        if ((int)plan.clique_down[c].size() > JT_V_MAX_CHILDREN)
            return SetError(FBN_ERR_LIMIT, "clique %d has %zu children (streamed variant: max %d)", c,
                            plan.clique_down[c].size(), JT_V_MAX_CHILDREN);
        if ((int)plan.cliques[c].vars.size() > 8 * JT_MAX_DIG_WORDS)
            return SetError(FBN_ERR_LIMIT, "clique with %zu variables (max %d)", plan.cliques[c].vars.size(),
                            8 * JT_MAX_DIG_WORDS);
        if (plan.cliques[c].size() > (int64_t)1 << 28)
            return SetError(FBN_ERR_LIMIT, "clique table of %lld entries", (long long)plan.cliques[c].size());
    }
    // store rows
    std::vector<int64_t> col_row(ns), dis_row(ns), den_row(nc);
    int64_t rows = 0;
    for (int s = 0; s < ns; ++s) col_row[s] = rows, rows += plan.seps[s].size();
    for (int s = 0; s < ns; ++s) dis_row[s] = rows, rows += plan.seps[s].size();
    for (int c = 0; c < nc; ++c) den_row[c] = rows, rows += (int64_t)plan.clique_down[c].size() + 2;
    // one scratch table per wave of the block (the Collect / Distribute table of the clique in
    // flight, read by its SEPCOL / SEPDIS / MARG passes)
    prog.scratch_row = rows;
    int64_t scr = 1;
    for (int c = 0; c < nc; ++c)
        if (!plan.clique_down[c].empty()) scr = std::max<int64_t>(scr, plan.cliques[c].size());
    prog.scratch_rows = scr;
    rows += JT_V_WAVES * scr;
    // message maps hold byte offsets into the block's store (buffer-load soffset)
    if (rows > INT32_MAX / 512) return SetError(FBN_ERR_LIMIT, "junction tree too large for the streamed variant");
    prog.store_rows = rows;

    // DFS orders (iterative)
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
    }
    if ((int)post.size() != nc)
        return SetError(FBN_ERR_LIMIT, "tree traversal covers %zu of %d cliques", post.size(), nc);
    // the JT_V_WAVES waves of a block split the tree: disjoint subtrees (one list per wave, run in
    // parallel) and the "top" cliques above them (one wave).  Greedy: expand the costliest subtree
    // while it exceeds 1/W of the total, then longest-processing-time assignment to the waves.
    {
        std::vector<int64_t> cost(nc), sub(nc);
        for (int c = 0; c < nc; ++c)
            cost[c] = plan.cliques[c].size() * (2 * (int64_t)plan.clique_down[c].size() + 3);
        for (int c : post) {
            sub[c] = cost[c];
            for (int s : plan.clique_down[c]) sub[c] += sub[plan.sep_down[s]];
        }
        const int64_t total = sub[plan.root];
        std::vector<int> cand{plan.root};
        std::vector<char> top(nc, 0);
        while (JT_V_WAVES > 1) {
            size_t bi = 0;
            for (size_t i = 1; i < cand.size(); ++i)
                if (sub[cand[i]] > sub[cand[bi]]) bi = i;
            const int c = cand[bi];
            if (sub[c] * JT_V_WAVES <= total || plan.clique_down[c].empty()) break;
            cand.erase(cand.begin() + bi);
            top[c] = 1;
            for (int s : plan.clique_down[c]) cand.push_back(plan.sep_down[s]);
        }
        std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) { return sub[a] > sub[b]; });
        std::vector<int64_t> load(JT_V_WAVES, 0);
        std::vector<int> owner(nc, -1);  // wave of each non-top clique
        for (int c : cand) {
            int w = 0;
            for (int i = 1; i < JT_V_WAVES; ++i)
                if (load[i] < load[w]) w = i;
            load[w] += sub[c];
            owner[c] = w;
        }
        for (int c : pre)  // propagate subtree ownership down (pre-order: parents first)
            for (int s : plan.clique_down[c]) {
                const int ch = plan.sep_down[s];
                if (!top[ch] && owner[ch] < 0) owner[ch] = owner[c];
            }
        // segments: collect per wave | collect top | distribute top | distribute per wave
        prog.sched.clear();
        prog.order.clear();
        for (int w = 0; w < JT_V_WAVES; ++w) {
            prog.sched.push_back((int32_t)prog.order.size());
            for (int c : post)
                if (!top[c] && owner[c] == w) prog.order.push_back(c);
        }
        prog.sched.push_back((int32_t)prog.order.size());
        for (int c : post)
            if (top[c] || JT_V_WAVES == 1) prog.order.push_back(c);
        prog.sched.push_back((int32_t)prog.order.size());
        for (int c : pre)
            if (top[c] || JT_V_WAVES == 1) prog.order.push_back(c);
        for (int w = 0; w < JT_V_WAVES; ++w) {
            prog.sched.push_back((int32_t)prog.order.size());
            for (int c : pre)
                if (!top[c] && owner[c] == w) prog.order.push_back(c);
        }
        prog.sched.push_back((int32_t)prog.order.size());
        if ((int)prog.order.size() != 2 * nc) return SetError(FBN_ERR_ARG, "internal: streamed schedule covers %zu of %d", prog.order.size(), 2 * nc);
        int64_t top_cost = 0;
        for (int c = 0; c < nc; ++c) top_cost += top[c] ? cost[c] : 0;
        int64_t mx = 0;
        for (auto l : load) mx = std::max(mx, l);
        prog.split_efficiency = (double)total / JT_V_WAVES / (double)std::max<int64_t>(1, mx + top_cost);
    }

    // per variable: candidate cliques in container order (GetProbabilitiesOneNode's scan,
    // src/JunctionTree.cpp:1412-1434) and the output slot
    std::vector<std::vector<int>> cand(V);
    for (int c = 0; c < nc; ++c)
        for (int v : plan.cliques[c].vars) cand[v].push_back(c);
    std::vector<int64_t> out_off(V);
    int64_t oo = 0;
    for (int v = 0; v < V; ++v) {
        if (cand[v].empty()) return SetError(FBN_ERR_ARG, "variable %d appears in no clique", v);
        prog.vsel.push_back((int32_t)prog.aux.size());
        prog.vsel.push_back((int32_t)cand[v].size());
        prog.aux.insert(prog.aux.end(), cand[v].begin(), cand[v].end());
        out_off[v] = oo;
        prog.vsel.push_back((int32_t)oo);
        prog.vsel.push_back(plan.dom[v]);
        oo += plan.dom[v];
    }

    prog.cl.resize(nc);
    for (int c = 0; c < nc; ++c) {
        const Table &t = plan.cliques[c];
        const int64_t T = t.size();
        const int nv = (int)t.vars.size();
        const int k = (int)plan.clique_down[c].size();
        const bool root = c == plan.root;
        JtVClique &q = prog.cl[c];
        q.T = (int32_t)T;
        q.nv = nv;
        q.k = k;
        q.root = root ? 1 : 0;
        q.id = c;
        // the Distribute table goes to the per-wave scratch for SEPDIS / MARG when the clique has
        // >= 2 children; with one child its two passes recompute the entries from the messages
        // (3 reads of L2-friendly message rows per entry instead of a scratch write + 2 reads that
        // reach HBM): 369 -> 364 ms per 125k Munin-like cases (FBN_JT_VDEBUG bit 512 measured it)
        static const int mat_min = getenv("FBN_JT_VMATK") ? atoi(getenv("FBN_JT_VMATK")) : 2;  // (tuning knob)
        q.mat = (!root && k >= mat_min) ? 1 : 0;
        static const int cmat_min = getenv("FBN_JT_VCMATK") ? atoi(getenv("FBN_JT_VCMATK")) : 2;  // (tuning knob)
        q.cmat = (!root && k >= cmat_min) ? 1 : 0;
        q.iv_off = (int32_t)prog.initv.size();
        prog.initv.insert(prog.initv.end(), t.pot.begin(), t.pot.end());
        // digits of every entry for the evidence test: packed into one 32-bit word with the
        // narrowest fields when they fit (nw = 0), else 8 bits per digit in nw 64-bit words
        std::vector<int> sh(nv), fm(nv);
        int bits = 0;
        for (int j = 0; j < nv; ++j) {
            int w = 1;
            while ((1 << w) < t.dims[j]) ++w;
            sh[j] = bits, fm[j] = (1 << w) - 1, bits += w;
        }
        const bool packed = bits <= 32 && nv <= 32;
        q.nw = packed ? 0 : std::max(1, (nv + 7) / 8);
        if (!packed) {
            for (int j = 0; j < nv; ++j) sh[j] = 8 * (j % 8), fm[j] = 0xFF;
            if (nv > 8 * JT_MAX_DIG_WORDS) return SetError(FBN_ERR_LIMIT, "clique with %d variables", nv);
        }
        q.dig_off = (int32_t)prog.dig.size();
        if (packed) {  // two entries per uint64 slot: entry e at 32-bit word dig_off * 2 + e
            std::vector<uint32_t> w32(T);
            for (int64_t e = 0; e < T; ++e) {
                uint32_t w = 0;
                int64_t r = e;
                for (int j = 0; j < nv; ++j) {
                    w |= (uint32_t)(r / t.cum[j]) << sh[j];
                    r %= t.cum[j];
                }
                w32[e] = w;
            }
            for (int64_t e = 0; e < T; e += 2)
                prog.dig.push_back((uint64_t)w32[e] | ((e + 1 < T ? (uint64_t)w32[e + 1] : 0ull) << 32));
        } else {
            for (int64_t e = 0; e < T; ++e) {
                uint64_t w[JT_MAX_DIG_WORDS] = {0, 0, 0, 0};
                int64_t r = e;
                for (int j = 0; j < nv; ++j) {
                    w[j / 8] |= (uint64_t)(r / t.cum[j]) << sh[j];
                    r %= t.cum[j];
                }
                for (int i = 0; i < q.nw; ++i) prog.dig.push_back(w[i]);
            }
        }
        q.vars_off = (int32_t)prog.aux.size();  // records {var, shift, field mask}
        for (int j = 0; j < nv; ++j) {
            prog.aux.push_back(t.vars[j]);
            prog.aux.push_back(sh[j]);
            prog.aux.push_back(fm[j]);
        }
        q.den_row = (int32_t)den_row[c];
        // message maps: child Collect messages in multiplication order, then the parent's message
        q.map_off = (int32_t)prog.aux.size();
        for (int s : plan.clique_down[c])
            for (int64_t e = 0; e < T; ++e)
                prog.aux.push_back((int32_t)((col_row[s] + SubIndex(t, plan.seps[s], e)) * 512));
        if (!root) {
            const int s = plan.clique_up[c];
            const int64_t Ts = plan.seps[s].size();
            // the upstream separator's variables are the clique's trailing ones
            // (ReorganizeTableStorage, src/JunctionTree.cpp:235-281): entry e meets separator entry e % Ts
            for (int64_t e = 0; e < T; ++e) {
                if (SubIndex(t, plan.seps[s], e) != e % Ts)
                    return SetError(FBN_ERR_ARG, "internal: upstream separator of clique %d is not trailing", c);
                prog.aux.push_back((int32_t)((dis_row[s] + e % Ts) * 512));
            }
            q.up_Ts = (int32_t)Ts;
            q.up_col_row = (int32_t)col_row[s];
        }
        // children: Distribute message targets, entry lists grouped by separator entry
        q.child_off = (int32_t)prog.aux.size();
        std::vector<int64_t> list_pos;
        for (int s : plan.clique_down[c]) {
            const int64_t Ts = plan.seps[s].size();
            prog.aux.push_back((int32_t)Ts);
            prog.aux.push_back((int32_t)(T / Ts));
            list_pos.push_back((int64_t)prog.aux.size());
            prog.aux.push_back(0);  // list_off, patched below
            prog.aux.push_back((int32_t)col_row[s]);
            prog.aux.push_back((int32_t)dis_row[s]);
        }
        for (int i = 0; i < k; ++i) {
            const int s = plan.clique_down[c][i];
            const int64_t Ts = plan.seps[s].size(), per = T / Ts;
            std::vector<std::vector<int32_t>> lists(Ts);
            for (int64_t e = 0; e < T; ++e) lists[SubIndex(t, plan.seps[s], e)].push_back((int32_t)e);
            prog.aux[list_pos[i]] = (int32_t)prog.aux.size();
            for (auto &l : lists) {
                if ((int64_t)l.size() != per) return SetError(FBN_ERR_ARG, "internal: ragged separator map");
                prog.aux.insert(prog.aux.end(), l.begin(), l.end());
            }
        }
        // marginals this clique may have to produce (every variable it holds; the per-case choice
        // of clique is made in the kernel)
        q.marg_off = (int32_t)prog.aux.size();
        q.nmarg = nv;
        for (int j = 0; j < nv; ++j) {
            const int v = t.vars[j];
            prog.aux.push_back((int32_t)out_off[v]);
            prog.aux.push_back(plan.dom[v]);
            prog.aux.push_back(v);
            prog.aux.push_back((int32_t)t.cum[j]);
        }
        if (prog.aux.size() > (size_t)INT32_MAX || prog.initv.size() > (size_t)INT32_MAX ||
            prog.dig.size() > (size_t)INT32_MAX)
            return SetError(FBN_ERR_LIMIT, "device program too large for the streamed variant");
    }
    return FBN_OK;
}

}  // namespace fbn
