// io.cpp -- host-side inputs of the hot paths: XMLBIF networks, CSV training sets, LIBSVM test
// sets, plus the thread-local error channel.  Semantics follow the reference loaders (cited per
// function); the implementations are single-pass scanners over the file bytes.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
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
// CSV training set: header + string values coded by first appearance per column
// (src/Dataset.cpp:267-414).  Trailing empty lines are ignored (the reference would read past the
// end of the row vector there).
int LoadCsv(const std::string &path, Dataset &ds) {
    std::string s;
    if (!ReadFile(path, s)) return SetError(FBN_ERR_IO, "cannot open %s", path.c_str());
    ds = Dataset();
    size_t pos = 0, n = s.size();
    auto next_line = [&](std::string &line) {
        if (pos >= n) return false;
        size_t e = s.find('\n', pos);
        if (e == std::string::npos) e = n;
        line.assign(s, pos, e - pos);
        pos = e + 1;
        size_t t = line.size();
        while (t > 0 && (unsigned char)line[t - 1] < 33) --t;  // TrimRight
        line.resize(t);
        return true;
    };
    std::string line;
    if (!next_line(line)) return SetError(FBN_ERR_IO, "%s: empty file", path.c_str());
    {
        size_t b = 0, e;
        while ((e = line.find(',', b)) != std::string::npos) {
            ds.names.push_back(line.substr(b, e - b));
            b = e + 1;
        }
        ds.names.push_back(line.substr(b));
    }
    ds.nvars = (int)ds.names.size();
    std::vector<std::unordered_map<std::string, int>> code(ds.nvars);
    std::vector<std::vector<uint8_t>> rows(ds.nvars);
    while (next_line(line)) {
        if (line.empty()) continue;
        size_t b = 0;
        for (int v = 0; v < ds.nvars; ++v) {
            size_t e = line.find(',', b);
            if (e == std::string::npos) {
                if (v != ds.nvars - 1) return SetError(FBN_ERR_IO, "%s: short row at sample %lld", path.c_str(), (long long)ds.nsamples);
                e = line.size();
            }
            std::string f = line.substr(b, e - b);
            b = e + 1;
            auto it = code[v].find(f);
            int c;
            if (it == code[v].end()) {
                c = (int)code[v].size();
                if (c > 255) return SetError(FBN_ERR_LIMIT, "%s: column %d has more than 256 values", path.c_str(), v);
                code[v].emplace(f, c);
            } else {
                c = it->second;
            }
            rows[v].push_back((uint8_t)c);
        }
        ds.nsamples++;
    }
    ds.cols.resize((size_t)ds.nvars * ds.nsamples);
    for (int v = 0; v < ds.nvars; ++v) {
        std::copy(rows[v].begin(), rows[v].end(), ds.cols.begin() + (size_t)v * ds.nsamples);
        ds.dims.push_back((int32_t)code[v].size());
    }
    return FBN_OK;
}

// ---------------------------------------------------------------------------------------------
// LIBSVM test set -> evidence (src/Dataset.cpp:162-262, src/Inference.cpp:13-42).  The reference's
// `getline; while(!eof)` loop skips a final line without '\n'; reproduced.  Features with an index
// >= num_nodes are ignored (src/JunctionTree.cpp:326-331).
int LoadLibsvm(const std::string &path, int num_nodes, std::vector<int8_t> &ev, std::vector<int32_t> &labels) {
    std::string s;
    if (!ReadFile(path, s)) return SetError(FBN_ERR_IO, "cannot open %s", path.c_str());
    ev.clear();
    labels.clear();
    size_t pos = 0, n = s.size();
    while (pos < n) {
        size_t e = s.find('\n', pos);
        if (e == std::string::npos) break;  // unterminated last line: not read by the reference
        std::string line = s.substr(pos, e - pos);
        pos = e + 1;
        size_t t = line.size();
        while (t > 0 && (unsigned char)line[t - 1] < 33) --t;
        line.resize(t);
        std::vector<int8_t> row(num_nodes, -1);
        size_t b = 0;
        bool first = true;
        while (true) {
            size_t sp = line.find(' ', b);
            std::string tok = line.substr(b, sp == std::string::npos ? std::string::npos : sp - b);
            if (first) {
                labels.push_back(atoi(tok.c_str()));
                first = false;
            } else {
                size_t c = tok.find(':');
                if (c == std::string::npos) return SetError(FBN_ERR_IO, "%s: bad feature '%s'", path.c_str(), tok.c_str());
                int idx = atoi(tok.substr(0, c).c_str());
                int val = atoi(tok.substr(c + 1).c_str());
                if (idx >= 0 && idx < num_nodes) row[idx] = (int8_t)val;
            }
            if (sp == std::string::npos) break;
            b = sp + 1;
        }
        ev.insert(ev.end(), row.begin(), row.end());
    }
    return FBN_OK;
}

}  // namespace fbn
