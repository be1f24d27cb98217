// pc_oracle.cpp -- TEST INFRASTRUCTURE.  See pc_oracle.h; each function cites the reference code
// it restates.
#include "pc_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>

namespace oracle {

// Regularized lower incomplete gamma P(a, x): series for x < a + 1, modified Lentz continued
// fraction for Q = 1 - P otherwise -- converged to full double precision.  stats::pchisq (the
// reference's p-value, src/IndependenceTest.cpp:146,268,355) is un-vendored: parity unpinned.
static double GammaP(double a, double x) {
    if (x <= 0) return 0.0;
    double lg = std::lgamma(a);
    if (x < a + 1.0) {
        double ap = a, sum = 1.0 / a, del = sum;
        for (int n = 0; n < 2000; ++n) {
            ap += 1.0;
            del *= x / ap;
            sum += del;
            if (std::fabs(del) < std::fabs(sum) * 1e-17) break;
        }
        return sum * std::exp(-x + a * std::log(x) - lg);
    }
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 2000; ++i) {
        double an = -i * (i - a);
        b += 2.0;
        d = an * d + b;
        if (std::fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (std::fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        double del = d * c;
        h *= del;
        if (std::fabs(del - 1.0) < 1e-17) break;
    }
    return 1.0 - std::exp(-x + a * std::log(x) - lg) * h;
}

// p = 1.0 - pchisq(g2, df), formed as the reference forms it (a CDF that rounds to 1 gives 0)
double ChiSquarePValue(double g2, int df) { return 1.0 - GammaP(0.5 * df, 0.5 * g2); }

CIResult CITest(const CodedDataset &ds, int x, int y, const int *z, int d, double alpha,
                std::vector<int> *counts_out) {
    const int dx = ds.dims[x], dy = ds.dims[y];
    // Counts3D ctor: z index = mixed radix, first conditioning var most significant
    // (src/CellTable.cpp:23-51, 268-291)
    std::vector<int> cum(d > 0 ? d : 1, 1);
    int dimz = 1;
    for (int j = d - 1; j >= 0; --j) {
        cum[j] = dimz;
        dimz *= ds.dims[z[j]];
    }
    std::vector<int> n((size_t)dimz * dx * dy, 0);
    const uint8_t *cx = ds.col[x].data(), *cy = ds.col[y].data();
    for (int64_t k = 0; k < ds.num_samples; ++k) {
        int zi = 0;
        for (int j = 0; j < d; ++j) zi += ds.col[z[j]][k] * cum[j];
        n[((size_t)zi * dx + cx[k]) * dy + cy[k]]++;
    }
    std::vector<int> ni((size_t)dimz * dx, 0), nj((size_t)dimz * dy, 0), nk(dimz, 0);
    for (int k = 0; k < dimz; ++k)  // marginals, src/CellTable.cpp:242-250
        for (int i = 0; i < dx; ++i)
            for (int j = 0; j < dy; ++j) {
                int c = n[((size_t)k * dx + i) * dy + j];
                ni[k * dx + i] += c;
                nj[k * dy + j] += c;
                nk[k] += c;
            }
    if (counts_out) *counts_out = n;
    CIResult r;
    r.g2 = 0.0;
    r.df = 0;
    for (int k = 0; k < dimz; ++k) {  // src/IndependenceTest.cpp:94-138 (XY: :309-347)
        int alx = 0, aly = 0;
        for (int i = 0; i < dx; ++i) alx += (ni[k * dx + i] > 0);
        for (int j = 0; j < dy; ++j) aly += (nj[k * dy + j] > 0);
        alx = alx >= 1 ? alx : 1;
        aly = aly >= 1 ? aly : 1;
        r.df += (alx - 1) * (aly - 1);
        long total = (d == 0) ? (long)ds.num_samples : (long)nk[k];
        if (total == 0) continue;
        for (int i = 0; i < dx; ++i) {
            long sum_row = ni[k * dx + i];
            if (sum_row == 0) continue;
            for (int j = 0; j < dy; ++j) {
                long sum_col = nj[k * dy + j];
                long observed = n[((size_t)k * dx + i) * dy + j];
                if (sum_col == 0 || observed == 0) continue;
                double expected = (double)sum_col * (double)sum_row / (double)total;
                r.g2 += 2.0 * observed * std::log(observed / expected);
            }
        }
    }
    if (r.df == 0) {  // df == 0 -> independent, p = 1 (:149-151, :349-351)
        r.p = 1.0;
        r.indep = true;
        return r;
    }
    r.p = ChiSquarePValue(r.g2, r.df);
    r.indep = r.p > alpha;
    return r;
}

// ---------------------------------------------------------------------------------------------
// PC-stable skeleton (src/PCStable.cpp:49-178, 209-563)
PCResult PCStableSkeleton(const CodedDataset &ds, double alpha, int depth, int group_size, bool keep_log) {
    PCResult res;
    const int n = ds.num_vars;
    std::vector<std::pair<int, int>> edges;  // GenerateUndirectedCompleteGraph order
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) edges.push_back({i, j});
    std::vector<std::set<int>> adj(n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j) adj[i].insert(j);

    auto remove_marked = [&](std::vector<char> &rm) {  // erase loop :131-147 / :310-326
        std::vector<std::pair<int, int>> keep;
        for (size_t e = 0; e < edges.size(); ++e) {
            if (rm[e]) {
                adj[edges[e].first].erase(edges[e].second);
                adj[edges[e].second].erase(edges[e].first);
            } else {
                keep.push_back(edges[e]);
            }
        }
        edges.swap(keep);
    };

    // level 0
    {
        std::vector<char> rm(edges.size(), 0);
        long long cnt = 0;
        for (size_t e = 0; e < edges.size(); ++e) {
            int x = edges[e].first, y = edges[e].second;
            CIResult r = CITest(ds, x, y, nullptr, 0, alpha);
            ++cnt;
            if (keep_log) res.log.push_back({0, x, y, {}, r});
            if (r.indep) {
                rm[e] = 1;
                res.sepset.insert({{x, y}, {}});
            }
        }
        remove_marked(rm);
        res.tests_per_level.push_back(cnt);
    }
    for (int d = 1; d < depth; ++d) {
        std::vector<std::set<int>> snap = adj;  // adjacencies_copy (:215)
        std::vector<char> rm(edges.size(), 0);
        long long cnt = 0;
        for (size_t e = 0; e < edges.size(); ++e) {
            int x = edges[e].first, y = edges[e].second;
            bool removed = false;
            for (int side = 0; side < 2 && !removed; ++side) {  // NODE1 then NODE2 (:351-399)
                int a = side ? y : x, b = side ? x : y;
                std::vector<int> A;
                for (int u : snap[a])
                    if (u != b) A.push_back(u);
                int m = (int)A.size();
                if (m < d) continue;
                // ChoiceGenerator lexicographic order (src/ChoiceGenerator.cpp:14-85)
                std::vector<int> ch(d);
                for (int i = 0; i < d; ++i) ch[i] = i;
                bool more = true;
                std::vector<std::vector<int>> group;
                auto flush = [&]() {
                    // one Testing() call (:465-551): group of up to group_size sets
                    int gsz = (int)group.size();
                    cnt += gsz;
                    int first = -1;
                    for (int g = 0; g < gsz; ++g) {
                        CIResult r = CITest(ds, x, y, group[g].data(), d, alpha);
                        if (gsz > 1 && r.df == 0) {
                            // ComputeGSquareXYZGroup overwrites results[m] with p > alpha and
                            // 1 - pchisq(g2, 0) = 0 (src/IndependenceTest.cpp:262-271)
                            r.p = 0.0;
                            r.indep = false;
                        }
                        if (keep_log) res.log.push_back({d, x, y, group[g], r});
                        if (r.indep && first < 0) first = g;
                    }
                    if (first >= 0) {
                        std::set<int> zs(group[first].begin(), group[first].end());
                        res.sepset.insert({{std::min(x, y), std::max(x, y)}, zs});
                        removed = true;
                    }
                    group.clear();
                };
                while (more && !removed) {
                    std::vector<int> Z(d);
                    for (int i = 0; i < d; ++i) Z[i] = A[ch[i]];
                    group.push_back(Z);
                    if ((int)group.size() == group_size) flush();
                    int i = d - 1;
                    while (i >= 0 && ch[i] == m - d + i) --i;
                    if (i < 0) {
                        more = false;
                    } else {
                        ++ch[i];
                        for (int k = i + 1; k < d; ++k) ch[k] = ch[k - 1] + 1;
                    }
                }
                if (!removed && !group.empty()) flush();
            }
            rm[e] = removed;
        }
        remove_marked(rm);
        res.tests_per_level.push_back(cnt);
        size_t maxdeg = 0;  // FreeDegree (:557-563)
        for (int i = 0; i < n; ++i) maxdeg = std::max(maxdeg, adj[i].size());
        if (!((int)maxdeg - 1 > d)) break;
    }
    res.edges = edges;
    for (long long c : res.tests_per_level) res.num_ci_test += c;
    return res;
}

}  // namespace oracle
