// io.cpp -- host-side inputs of the hot paths: XMLBIF networks, CSV training sets, LIBSVM test
// sets, plus the thread-local error channel.  Semantics follow the reference loaders (cited per
// function); the implementations are single-pass scanners over the file bytes.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <fstream>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "fbn_internal.h"

namespace fbn {

static thread_local std::string g_last_error;

int SetError(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

const char *LastError() { return g_last_error.c_str(); }

static bool ReadFile(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

static std::string Trim(const std::string &s) {  // chars < 33 (src/common.cpp:145-177)
    size_t b = 0, e = s.size();
    while (b < e && (unsigned char)s[b] < 33) ++b;
    while (e > b && (unsigned char)s[e - 1] < 33) --e;
    return s.substr(b, e - b);
}

// ---------------------------------------------------------------------------------------------
// XMLBIF.  A flat scanner: we only need the text of NAME/TYPE/VALUE inside VARIABLE and of
// FOR/GIVEN/TABLE inside PROBABILITY, in document order.
namespace {
struct Tok {
    bool close;
    std::string name;
    size_t text_begin, text_end;  // text after the tag up to the next '<'
};

bool ScanTags(const std::string &s, std::vector<Tok> &toks) {
    size_t i = 0, n = s.size();
    while (i < n) {
        size_t lt = s.find('<', i);
        if (lt == std::string::npos) break;
        if (s.compare(lt, 4, "<!--") == 0) {
            size_t e = s.find("-->", lt);
            if (e == std::string::npos) return false;
            i = e + 3;
            continue;
        }
        size_t gt = s.find('>', lt);
        if (gt == std::string::npos) return false;
        if (s[lt + 1] == '?' || s[lt + 1] == '!') {
            i = gt + 1;
            continue;
        }
        Tok t;
        t.close = s[lt + 1] == '/';
        size_t nb = lt + 1 + (t.close ? 1 : 0), ne = nb;
        while (ne < gt && !isspace((unsigned char)s[ne]) && s[ne] != '/') ++ne;
        t.name = s.substr(nb, ne - nb);
        bool self_close = s[gt - 1] == '/';
        t.text_begin = gt + 1;
        size_t nx = s.find('<', gt + 1);
        t.text_end = nx == std::string::npos ? n : nx;
        toks.push_back(t);
        if (self_close) toks.push_back({true, t.name, gt + 1, gt + 1});
        i = gt + 1;
    }
    return true;
}
}  // namespace

double Network::Prob(int v, int q, const int *pv) const {
    // DiscreteNode::GetProbability (src/DiscreteNode.cpp:152-161): (count + 1) / (total + 1*|dom|)
    int64_t pc = 0;
    for (size_t j = 0; j < parents_asc[v].size(); ++j) pc = pc * dom[parents_asc[v][j]] + pv[j];
    int64_t npc = (int64_t)totals[v].size();
    return ((double)counts[v][q * npc + pc] + 1.0) / ((double)totals[v][pc] + 1.0 * (double)dom[v]);
}

// A network given in memory: what a reference `Network` of DiscreteNodes holds after
// InitializeCPT + AddCount (src/DiscreteNode.cpp:114-147): per node its state count, its parents
// (the order given = the node's own parent order, used by the seeded generators) and the count map
// map_cond_prob_table_statistics[value][parent config], parent configurations over the parents in
// ascending index order, last fastest (a DiscreteConfig is an ordered set of (var, value) pairs).
// map_total_count_under_parents_config is the sum over the values, as AddCount keeps it; the
// probabilities follow GetProbability (:154-164) with laplace_smooth = 1, as for the XMLBIF path.
int BuildNetwork(int n, const int32_t *dims, const int32_t *parent_off, const int32_t *parents, const int64_t *counts,
                 const char *const *names, Network &net) {
    if (n < 1 || !dims || !parent_off || (!parents && parent_off[n] > 0) || !counts)
        return SetError(FBN_ERR_ARG, "network: bad arguments");
    net = Network();
    net.dom.assign(dims, dims + n);
    for (int v = 0; v < n; ++v) {
        if (net.dom[v] < 1 || net.dom[v] > 127) return SetError(FBN_ERR_LIMIT, "node %d has %d states (supported 1..127)", v, net.dom[v]);
        net.names.push_back(names && names[v] ? std::string(names[v]) : "X" + std::to_string(v));
    }
    net.given.assign(n, {});
    net.parents_asc.assign(n, {});
    net.counts.assign(n, {});
    net.totals.assign(n, {});
    int64_t off = 0;
    for (int v = 0; v < n; ++v) {
        if (parent_off[v + 1] < parent_off[v]) return SetError(FBN_ERR_ARG, "node %d: parent offsets decrease", v);
        for (int32_t k = parent_off[v]; k < parent_off[v + 1]; ++k) {
            const int q = parents[k];
            if (q < 0 || q >= n || q == v) return SetError(FBN_ERR_ARG, "node %d: bad parent %d", v, q);
            net.given[v].push_back(q);
        }
        std::set<int> ps(net.given[v].begin(), net.given[v].end());
        if (ps.size() != net.given[v].size()) return SetError(FBN_ERR_ARG, "node %d: repeated parent", v);
        net.parents_asc[v].assign(ps.begin(), ps.end());
        int64_t npc = 1;
        for (int q : net.parents_asc[v]) npc *= net.dom[q];
        net.counts[v].assign(counts + off, counts + off + net.dom[v] * npc);
        net.totals[v].assign((size_t)npc, 0);
        for (int q = 0; q < net.dom[v]; ++q)
            for (int64_t pc = 0; pc < npc; ++pc) {
                const int64_t c = net.counts[v][q * npc + pc];
                if (c < 0) return SetError(FBN_ERR_ARG, "node %d: negative count", v);
                net.totals[v][pc] += c;
            }
        off += net.dom[v] * npc;
    }
    // a DAG (the junction tree and the generators need one)
    std::vector<int> indeg(n, 0), order;
    std::vector<std::vector<int>> ch(n);
    for (int v = 0; v < n; ++v)
        for (int q : net.parents_asc[v]) ch[q].push_back(v), ++indeg[v];
    for (int v = 0; v < n; ++v)
        if (!indeg[v]) order.push_back(v);
    for (size_t i = 0; i < order.size(); ++i)
        for (int c : ch[order[i]])
            if (--indeg[c] == 0) order.push_back(c);
    if ((int)order.size() != n) return SetError(FBN_ERR_ARG, "network: the parent lists form a cycle");
    return FBN_OK;
}

// the count map of node v (layout as BuildNetwork's), parents in ascending order
int NodeCounts(const Network &net, int v, int32_t *parents_asc, int64_t *counts, int *nparents, int64_t *ncounts) {
    if (v < 0 || v >= net.n()) return SetError(FBN_ERR_ARG, "node %d out of range", v);
    if (nparents) *nparents = (int)net.parents_asc[v].size();
    if (ncounts) *ncounts = (int64_t)net.counts[v].size();
    if (parents_asc) std::copy(net.parents_asc[v].begin(), net.parents_asc[v].end(), parents_asc);
    if (counts) std::copy(net.counts[v].begin(), net.counts[v].end(), counts);
    return FBN_OK;
}

int LoadXmlbif(const std::string &path, Network &net) {
    std::string s;
    if (!ReadFile(path, s)) return SetError(FBN_ERR_IO, "cannot open %s", path.c_str());
    std::vector<Tok> toks;
    if (!ScanTags(s, toks)) return SetError(FBN_ERR_IO, "%s: malformed XML", path.c_str());
    auto text = [&](const Tok &t) { return Trim(s.substr(t.text_begin, t.text_end - t.text_begin)); };

    struct Var {
        std::string name, type;
        int nvals = 0;
    };
    struct Prob {
        std::string for_;
        std::vector<std::string> given;
        std::string table;
    };
    std::vector<Var> vars;
    std::vector<Prob> probs;
    int in_var = 0, in_prob = 0;
    for (const Tok &t : toks) {
        if (t.name == "VARIABLE") {
            in_var = !t.close;
            if (!t.close) vars.emplace_back();
        } else if (t.name == "PROBABILITY") {
            in_prob = !t.close;
            if (!t.close) probs.emplace_back();
        } else if (!t.close && in_var) {
            if (t.name == "NAME") vars.back().name = text(t);
            else if (t.name == "TYPE") vars.back().type = text(t);
            else if (t.name == "VALUE") vars.back().nvals++;
        } else if (!t.close && in_prob) {
            if (t.name == "FOR") probs.back().for_ = text(t);
            else if (t.name == "GIVEN") probs.back().given.push_back(text(t));
            else if (t.name == "TABLE") probs.back().table = text(t);
        }
    }
    // node index = order of the discrete <VARIABLE> elements (src/XMLBIFParser.cpp:33-68)
    std::unordered_map<std::string, int> idx;
    net = Network();
    for (const Var &v : vars) {
        if (v.type != "discrete") continue;
        idx[v.name] = (int)net.dom.size();
        net.names.push_back(v.name);
        net.dom.push_back(v.nvals);
    }
    const int n = net.n();
    if (n == 0) return SetError(FBN_ERR_IO, "%s: no discrete variables", path.c_str());
    for (int v = 0; v < n; ++v)
        if (net.dom[v] < 1 || net.dom[v] > 127)
            return SetError(FBN_ERR_LIMIT, "%s: variable %s has %d states (supported 1..127)", path.c_str(),
                            net.names[v].c_str(), net.dom[v]);
    net.given.assign(n, {});
    net.parents_asc.assign(n, {});
    net.counts.assign(n, {});
    net.totals.assign(n, {});
    std::vector<bool> seen(n, false);
    // src/XMLBIFParser.cpp:73-179
    for (const Prob &p : probs) {
        auto it = idx.find(p.for_);
        if (it == idx.end()) return SetError(FBN_ERR_IO, "%s: PROBABILITY for unknown %s", path.c_str(), p.for_.c_str());
        int v = it->second;
        seen[v] = true;
        std::vector<int> given;
        for (auto &g : p.given) {
            auto gi = idx.find(g);
            if (gi == idx.end()) return SetError(FBN_ERR_IO, "%s: GIVEN %s unknown", path.c_str(), g.c_str());
            given.push_back(gi->second);
        }
        std::set<int> ps(given.begin(), given.end());
        net.given[v] = given;
        net.parents_asc[v].assign(ps.begin(), ps.end());
        int64_t npc = 1;
        for (int q : net.parents_asc[v]) npc *= net.dom[q];
        net.counts[v].assign((size_t)(net.dom[v] * npc), 0);
        net.totals[v].assign((size_t)npc, 0);
        // positions of each ascending parent inside the GIVEN list (last occurrence wins)
        std::vector<int> pos_in_given(net.parents_asc[v].size(), 0);
        for (size_t a = 0; a < net.parents_asc[v].size(); ++a)
            for (size_t j = 0; j < given.size(); ++j)
                if (given[j] == net.parents_asc[v][a]) pos_in_given[a] = (int)j;
        std::vector<int> range{net.dom[v]};
        for (int g : given) range.push_back(net.dom[g]);
        int64_t total = 1;
        for (int r : range) total *= r;
        // TABLE: split on single spaces (src/common.cpp:182-190 via src/XMLBIFParser.cpp:123-130),
        // digit 0 = this node, then GIVEN order, last fastest (NaryCount src/common.cpp:193-232)
        const std::string &tb = p.table;
        std::vector<int> digit(range.size(), 0);
        size_t pos = 0;
        for (int64_t i = 0; i < total; ++i) {
            if (pos > tb.size()) return SetError(FBN_ERR_IO, "%s: TABLE of %s too short", path.c_str(), p.for_.c_str());
            size_t sp = tb.find(' ', pos);
            if (sp == std::string::npos) sp = tb.size();
            std::string tokn = tb.substr(pos, sp - pos);
            char *endp = nullptr;
            double pr = strtod(tokn.c_str(), &endp);
            if (tokn.empty() || endp == tokn.c_str())
                return SetError(FBN_ERR_IO, "%s: bad TABLE entry '%s' for %s", path.c_str(), tokn.c_str(), p.for_.c_str());
            pos = sp + 1;
            int cnt = (int)(pr * 10000);  // DiscreteNode::AddCount(int) truncation (:176)
            int64_t pc = 0;
            for (size_t a = 0; a < net.parents_asc[v].size(); ++a)
                pc = pc * net.dom[net.parents_asc[v][a]] + digit[pos_in_given[a] + 1];
            net.counts[v][digit[0] * npc + pc] += cnt;
            net.totals[v][pc] += cnt;
            for (int d = (int)range.size() - 1; d >= 0; --d) {
                if (++digit[d] < range[d]) break;
                digit[d] = 0;
            }
        }
        if (pos <= tb.size()) return SetError(FBN_ERR_IO, "%s: TABLE of %s too long", path.c_str(), p.for_.c_str());
    }
    for (int v = 0; v < n; ++v)  // the reference requires one PROBABILITY per VARIABLE (:20-23)
        if (!seen[v]) return SetError(FBN_ERR_IO, "%s: no PROBABILITY for %s", path.c_str(), net.names[v].c_str());
    return FBN_OK;
}

// ---------------------------------------------------------------------------------------------
// Streaming, multi-threaded text scanning: the file is read in blocks of kBlock bytes; each block's
// complete lines are cut into one part per thread at line boundaries and parsed in parallel; the
// parts are then merged in file order (so every order-dependent result -- first-appearance codes,
// row indices -- is the sequential one).  Memory: one block plus the outputs.
namespace {

constexpr size_t kBlock = 64u << 20;

int NumThreads() {
    const unsigned hc = std::thread::hardware_concurrency();
    int t = (int)std::max(1u, std::min(16u, hc ? hc : 1u));  // the GPU box's CPU share is 16
    if (const char *e = getenv("OMP_NUM_THREADS")) t = std::max(1, std::min(t, atoi(e)));
    return t;
}

// calls fn(lines_begin, lines_end, is_last_block) for consecutive blocks of complete lines; the
// final unterminated line (if any) is passed as the last block's tail
template <class F>
int ForEachBlock(const std::string &path, F fn) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return SetError(FBN_ERR_IO, "cannot open %s", path.c_str());
    std::vector<char> buf;
    size_t carry = 0;
    while (true) {
        buf.resize(carry + kBlock);
        const size_t got = fread(buf.data() + carry, 1, kBlock, f);
        const size_t have = carry + got;
        const bool eof = got < kBlock;
        size_t end = have;
        if (!eof) {  // cut after the last newline; the rest carries over
            const char *p = buf.data();
            size_t k = have;
            while (k > 0 && p[k - 1] != '\n') --k;
            if (k == 0) {  // one line longer than a block: read on
                carry = have;
                continue;
            }
            end = k;
        }
        int rc = fn(buf.data(), buf.data() + end, eof);
        if (rc) {
            fclose(f);
            return rc;
        }
        if (eof) break;
        carry = have - end;
        memmove(buf.data(), buf.data() + end, carry);
    }
    fclose(f);
    return FBN_OK;
}

// cut [b, e) into up to T parts at line boundaries
std::vector<std::pair<const char *, const char *>> CutLines(const char *b, const char *e, int T) {
    std::vector<std::pair<const char *, const char *>> parts;
    const char *p = b;
    for (int t = 0; t < T && p < e; ++t) {
        const char *q = t == T - 1 ? e : std::min(e, p + (e - b) / T + 1);
        if (q < e) {
            const char *nl = (const char *)memchr(q, '\n', (size_t)(e - q));
            q = nl ? nl + 1 : e;
        }
        parts.push_back({p, q});
        p = q;
    }
    return parts;
}

template <class F>
void Parallel(int n, F fn) {
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i) th.emplace_back(fn, i);
    fn(0);
    for (auto &t : th) t.join();
}

// one line [b, e) without its '\n', right-trimmed (chars < 33, as the reference's Trim)
inline void TrimRight(const char *b, const char *&e) {
    while (e > b && (unsigned char)e[-1] < 33) --e;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// CSV training set: header + string values coded by first appearance per column
// (src/Dataset.cpp:267-414).  Trailing empty lines are ignored (the reference would read past the
// end of the row vector there).  A row's last variable ends at the next ',' if the row
// has extra fields (they are ignored); a row with fewer fields is an error.
int LoadCsv(const std::string &path, Dataset &ds) {
    ds = Dataset();
    const int T = NumThreads();
    bool header_done = false;
    std::vector<std::vector<std::string>> gdict;     // global first-appearance dictionaries
    std::vector<std::vector<uint8_t>> colv;          // per-column codes, file order
    struct Part {
        std::vector<uint8_t> rows;                   // row-major local codes
        std::vector<std::vector<std::string>> dict;  // local dictionaries
        int64_t nrows = 0;
        int err = 0, err_var = 0;
        int64_t err_row = 0;
    };
    int rc = ForEachBlock(path, [&](const char *b, const char *e, bool) -> int {
        if (!header_done) {
            const char *nl = (const char *)memchr(b, '\n', (size_t)(e - b));
            const char *he = nl ? nl : e;
            TrimRight(b, he);
            const char *p = b;
            while (true) {
                const char *c = (const char *)memchr(p, ',', (size_t)(he - p));
                ds.names.emplace_back(p, c ? c : he);
                if (!c) break;
                p = c + 1;
            }
            if (b == e) return SetError(FBN_ERR_IO, "%s: empty file", path.c_str());
            ds.nvars = (int)ds.names.size();
            gdict.assign(ds.nvars, {});
            colv.assign(ds.nvars, {});
            header_done = true;
            b = nl ? nl + 1 : e;
        }
        const int V = ds.nvars;
        auto parts = CutLines(b, e, T);
        std::vector<Part> P(parts.size());
        Parallel((int)parts.size(), [&](int t) {
            Part &pt = P[t];
            pt.dict.assign(V, {});
            const char *p = parts[t].first, *pe = parts[t].second;
            while (p < pe && !pt.err) {
                const char *nl = (const char *)memchr(p, '\n', (size_t)(pe - p));
                const char *le = nl ? nl : pe;
                const char *ls = p;
                p = nl ? nl + 1 : pe;
                TrimRight(ls, le);
                if (ls == le) continue;  // empty line
                const char *f = ls;
                for (int v = 0; v < V; ++v) {
                    const char *c = (const char *)memchr(f, ',', (size_t)(le - f));
                    if (!c) {
                        if (v != V - 1) {
                            pt.err = 1, pt.err_row = pt.nrows;
                            break;
                        }
                        c = le;
                    }
                    const size_t len = (size_t)(c - f);
                    auto &d = pt.dict[v];
                    size_t k = 0;
                    while (k < d.size() && !(d[k].size() == len && memcmp(d[k].data(), f, len) == 0)) ++k;
                    if (k == d.size()) {
                        if (k >= 256) {
                            pt.err = 2, pt.err_var = v;
                            break;
                        }
                        d.emplace_back(f, len);
                    }
                    pt.rows.push_back((uint8_t)k);
                    f = c + 1;
                }
                if (!pt.err) ++pt.nrows;
            }
        });
        // merge in file order: local -> global codes (first appearance), append per column
        int64_t base = ds.nsamples;
        for (auto &pt : P) {
            if (pt.err == 1)
                return SetError(FBN_ERR_IO, "%s: short row at sample %lld", path.c_str(), (long long)(base + pt.err_row));
            if (pt.err == 2) return SetError(FBN_ERR_LIMIT, "%s: column %d has more than 256 values", path.c_str(), pt.err_var);
            base += pt.nrows;
        }
        std::vector<std::vector<uint8_t>> remap(P.size(), std::vector<uint8_t>((size_t)V * 256));
        for (size_t t = 0; t < P.size(); ++t)
            for (int v = 0; v < V; ++v)
                for (size_t k = 0; k < P[t].dict[v].size(); ++k) {
                    auto &g = gdict[v];
                    size_t j = 0;
                    while (j < g.size() && g[j] != P[t].dict[v][k]) ++j;
                    if (j == g.size()) {
                        if (j >= 256) return SetError(FBN_ERR_LIMIT, "%s: column %d has more than 256 values", path.c_str(), v);
                        g.push_back(P[t].dict[v][k]);
                    }
                    remap[t][(size_t)v * 256 + k] = (uint8_t)j;
                }
        std::vector<int64_t> row0(P.size() + 1, ds.nsamples);
        for (size_t t = 0; t < P.size(); ++t) row0[t + 1] = row0[t] + P[t].nrows;
        for (int v = 0; v < V; ++v) colv[v].resize((size_t)row0.back());
        Parallel((int)P.size(), [&](int t) {
            const uint8_t *r = P[t].rows.data();
            const uint8_t *m = remap[t].data();
            for (int64_t i = 0; i < P[t].nrows; ++i, r += V)
                for (int v = 0; v < V; ++v) colv[v][(size_t)(row0[t] + i)] = m[(size_t)v * 256 + r[v]];
        });
        ds.nsamples = row0.back();
        return FBN_OK;
    });
    if (rc) return rc;
    if (!header_done) return SetError(FBN_ERR_IO, "%s: empty file", path.c_str());
    ds.cols.resize((size_t)ds.nvars * ds.nsamples);
    for (int v = 0; v < ds.nvars; ++v) {
        std::copy(colv[v].begin(), colv[v].end(), ds.cols.begin() + (size_t)v * ds.nsamples);
        ds.dims.push_back((int32_t)gdict[v].size());
    }
    return FBN_OK;
}

// ---------------------------------------------------------------------------------------------
// LIBSVM test set -> evidence (src/Dataset.cpp:162-262, src/Inference.cpp:13-42).  The reference's
// `getline; while(!eof)` loop skips a final line without '\n'; reproduced.  Features with an index
// >= num_nodes are ignored (src/JunctionTree.cpp:326-331).  ev == nullptr: count the rows only;
// otherwise the first min(rows, cap) rows are written to ev [row][num_nodes] / labels.
int LoadLibsvm(const std::string &path, int num_nodes, int8_t *ev, int32_t *labels, int64_t cap, int64_t *nrows) {
    const int T = NumThreads();
    int64_t row = 0;
    int rc = ForEachBlock(path, [&](const char *b, const char *e, bool last) -> int {
        if (last) {  // drop an unterminated final line
            const char *k = e;
            while (k > b && k[-1] != '\n') --k;
            e = k;
        }
        auto parts = CutLines(b, e, T);
        std::vector<int64_t> cnt(parts.size(), 0);
        Parallel((int)parts.size(), [&](int t) {
            for (const char *p = parts[t].first; p < parts[t].second;) {
                const char *nl = (const char *)memchr(p, '\n', (size_t)(parts[t].second - p));
                if (!nl) break;
                ++cnt[t];
                p = nl + 1;
            }
        });
        std::vector<int64_t> r0(parts.size() + 1, row);
        for (size_t t = 0; t < parts.size(); ++t) r0[t + 1] = r0[t] + cnt[t];
        if (ev && row < cap) {
            std::vector<std::string> errs(parts.size());
            Parallel((int)parts.size(), [&](int t) {
                int64_t r = r0[t];
                for (const char *p = parts[t].first; p < parts[t].second && r < cap; ++r) {
                    const char *nl = (const char *)memchr(p, '\n', (size_t)(parts[t].second - p));
                    const char *ls = p, *le = nl;
                    p = nl + 1;
                    TrimRight(ls, le);
                    int8_t *out = ev + (size_t)r * num_nodes;
                    memset(out, -1, (size_t)num_nodes);
                    // tokens separated by single spaces: the label, then idx:val features
                    const char *q = ls;
                    bool first = true;
                    while (true) {
                        const char *sp = (const char *)memchr(q, ' ', (size_t)(le - q));
                        const char *te = sp ? sp : le;
                        if (first) {
                            if (labels) labels[r] = atoi(std::string(q, te).c_str());
                            first = false;
                        } else {
                            const char *c = (const char *)memchr(q, ':', (size_t)(te - q));
                            if (!c) {
                                errs[t] = std::string(q, te);
                                return;
                            }
                            const int idx = atoi(std::string(q, c).c_str());
                            const int val = atoi(std::string(c + 1, te).c_str());
                            if (idx >= 0 && idx < num_nodes) out[idx] = (int8_t)val;
                        }
                        if (!sp) break;
                        q = sp + 1;
                    }
                }
            });
            for (auto &m : errs)
                if (!m.empty()) return SetError(FBN_ERR_IO, "%s: bad feature '%s'", path.c_str(), m.c_str());
        }
        row = r0.back();
        return FBN_OK;
    });
    if (rc) return rc;
    if (nrows) *nrows = row;
    return FBN_OK;
}

}  // namespace fbn
