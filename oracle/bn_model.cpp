// bn_model.cpp -- TEST INFRASTRUCTURE (CPU oracle).  See bn_model.h for the reference sites.
#include "bn_model.h"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <set>
#include <sstream>

#include "mini_xml.h"

namespace oracle {

static std::string TrimWs(const std::string &s) {  // src/common.cpp:145-177 (chars < 33)
    size_t b = 0, e = s.size();
    while (b < e && (unsigned char)s[b] < 33) ++b;
    while (e > b && (unsigned char)s[e - 1] < 33) --e;
    return s.substr(b, e - b);
}

static std::vector<std::string> SplitAny(const std::string &s, const std::string &delims) {
    std::vector<std::string> out;  // src/common.cpp:182-190: empty fields are kept
    size_t begin = 0, end;
    while ((end = s.find_first_of(delims, begin)) != std::string::npos) {
        out.push_back(s.substr(begin, end - begin));
        begin = end + 1;
    }
    out.push_back(s.substr(begin));
    return out;
}

double BayesNet::Prob(int v, int q, const std::vector<int> &pv) const {
    // src/DiscreteNode.cpp:152-161: (frequency_count + 1) / (total + 1 * |dom|), int counts
    long long pc = 0;
    for (size_t j = 0; j < parents_asc[v].size(); ++j) pc = pc * dom[parents_asc[v][j]] + pv[j];
    long long npc = (long long)totals[v].size();
    long long fc = counts[v][q * npc + pc];
    long long tot = totals[v][pc];
    return ((double)fc + 1.0) / ((double)tot + 1.0 * (double)dom[v]);
}

BayesNet LoadXmlbif(const std::string &path) {
    BayesNet bn;
    std::unique_ptr<mini_xml::Element> doc;
    try {
        doc = mini_xml::parse_file(path);
    } catch (const std::exception &e) {
        fprintf(stderr, "oracle: %s\n", e.what());
        exit(1);
    }
    const mini_xml::Element *bif = doc->first("BIF");
    const mini_xml::Element *net = bif ? bif->first("NETWORK") : nullptr;
    if (!net) {
        fprintf(stderr, "oracle: %s is not XMLBIF\n", path.c_str());
        exit(1);
    }
    // src/XMLBIFParser.cpp:33-68 -- node index = order of discrete <VARIABLE> elements
    for (const mini_xml::Element *xv : net->all("VARIABLE")) {
        if (TrimWs(xv->first("TYPE")->text) != "discrete") continue;
        bn.names.push_back(TrimWs(xv->first("NAME")->text));
        bn.dom.push_back((int)xv->all("VALUE").size());
    }
    bn.n = (int)bn.names.size();
    bn.given.assign(bn.n, {});
    bn.parents_asc.assign(bn.n, {});
    bn.counts.assign(bn.n, {});
    bn.totals.assign(bn.n, {});
    auto find = [&](const std::string &raw) {
        std::string nm = TrimWs(raw);
        for (int i = 0; i < bn.n; ++i)
            if (bn.names[i] == nm) return i;
        fprintf(stderr, "oracle: unknown variable '%s'\n", nm.c_str());
        exit(1);
    };
    // src/XMLBIFParser.cpp:73-179
    for (const mini_xml::Element *xp : net->all("PROBABILITY")) {
        int v = find(xp->first("FOR")->text);
        std::vector<int> given;
        for (const mini_xml::Element *g : xp->all("GIVEN")) given.push_back(find(g->text));
        bn.given[v] = given;
        std::set<int> ps(given.begin(), given.end());
        bn.parents_asc[v].assign(ps.begin(), ps.end());
        const auto &pa = bn.parents_asc[v];
        long long npc = 1;
        for (int p : pa) npc *= bn.dom[p];
        bn.counts[v].assign((size_t)(bn.dom[v] * npc), 0);
        bn.totals[v].assign((size_t)npc, 0);

        std::vector<std::string> toks = SplitAny(TrimWs(xp->first("TABLE")->text), " ");
        // NaryCount (src/common.cpp:193-232): digit 0 = this node, then GIVEN order, last fastest
        std::vector<int> range{bn.dom[v]};
        for (int g : given) range.push_back(bn.dom[g]);
        long long total = 1;
        for (int r : range) total *= r;
        if ((long long)toks.size() != total) {
            fprintf(stderr, "oracle: table of %s has %zu entries, expected %lld\n", bn.names[v].c_str(),
                    toks.size(), total);
            exit(1);
        }
        std::vector<int> digit(range.size(), 0);
        for (long long i = 0; i < total; ++i) {
            double p = strtod(toks[i].c_str(), nullptr);
            int cnt = (int)(p * 10000);  // AddCount(int count) truncation, src/XMLBIFParser.cpp:176
            // map GIVEN-order digits to the ascending parent index
            long long pc = 0;
            for (int par : pa) {
                int val = 0;
                for (size_t j = 0; j < given.size(); ++j)
                    if (given[j] == par) val = digit[j + 1];
                pc = pc * bn.dom[par] + val;
            }
            bn.counts[v][digit[0] * npc + pc] += cnt;
            bn.totals[v][pc] += cnt;
            for (int d = (int)range.size() - 1; d >= 0; --d) {
                if (++digit[d] < range[d]) break;
                digit[d] = 0;
            }
        }
    }
    return bn;
}

CodedDataset LoadCsv(const std::string &path) {
    CodedDataset ds;
    std::ifstream in(path);
    if (!in) {
        fprintf(stderr, "oracle: cannot open %s\n", path.c_str());
        exit(1);
    }
    std::string line;
    std::getline(in, line);
    line = TrimWs(line);
    ds.var_names = SplitAny(line, ",");
    ds.num_vars = (int)ds.var_names.size();
    std::vector<std::map<std::string, int>> code(ds.num_vars);
    ds.col.assign(ds.num_vars, {});
    while (std::getline(in, line)) {
        // TrimRight only (src/Dataset.cpp:322,390); empty lines are skipped (the reference would
        // read past the row end on a trailing newline)
        size_t e = line.size();
        while (e > 0 && (unsigned char)line[e - 1] < 33) --e;
        line.resize(e);
        if (line.empty()) continue;
        std::vector<std::string> f = SplitAny(line, ",");
        if ((int)f.size() < ds.num_vars) {
            fprintf(stderr, "oracle: short CSV row\n");
            exit(1);
        }
        for (int v = 0; v < ds.num_vars; ++v) {
            auto it = code[v].find(f[v]);
            int c;
            if (it == code[v].end()) {
                c = (int)code[v].size();  // first-appearance coding, src/Dataset.cpp:334-342
                code[v][f[v]] = c;
            } else {
                c = it->second;
            }
            ds.col[v].push_back((uint8_t)c);
        }
        ds.num_samples++;
    }
    for (int v = 0; v < ds.num_vars; ++v) ds.dims.push_back((int)code[v].size());
    return ds;
}

int64_t LoadLibsvmEvidence(const std::string &path, int num_nodes, std::vector<int8_t> &ev,
                           std::vector<int> &labels) {
    std::ifstream in(path);
    if (!in) {
        fprintf(stderr, "oracle: cannot open %s\n", path.c_str());
        exit(1);
    }
    ev.clear();
    labels.clear();
    std::string line;
    // src/Dataset.cpp:182-227: getline; while(!eof){...; getline} -> a final line without '\n'
    // is not read.  Reproduced.
    std::getline(in, line);
    while (!in.eof()) {
        size_t e = line.size();
        while (e > 0 && (unsigned char)line[e - 1] < 33) --e;
        line.resize(e);
        std::vector<std::string> tok = SplitAny(line, " ");
        labels.push_back(atoi(tok[0].c_str()));
        std::vector<int8_t> row(num_nodes, -1);
        for (size_t i = 1; i < tok.size(); ++i) {
            size_t c = tok[i].find(':');
            int idx = atoi(tok[i].substr(0, c).c_str());
            int val = atoi(tok[i].substr(c + 1).c_str());
            if (idx >= num_nodes) continue;  // src/JunctionTree.cpp:326-331
            row[idx] = (int8_t)val;
        }
        ev.insert(ev.end(), row.begin(), row.end());
        std::getline(in, line);
    }
    return (int64_t)labels.size();
}

}  // namespace oracle
