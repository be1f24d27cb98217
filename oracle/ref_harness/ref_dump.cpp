// ref_dump.cpp -- TEST INFRASTRUCTURE.  Harness that links the *unmodified* reference sources
// (compiled in place from /root/reference/src by oracle/Makefile target `ref`) and dumps golden
// vectors for the parity tests.  Nothing here ships: the binary lands in oracle/_ref/ (gitignored)
// and only the text fixtures it writes are committed under tests/golden/.
//
// The reference reads XMLBIF through tinyxml2, which is absent from this image, so the network
// is populated here through the reference's own public model API in exactly the order
// XMLBIFParser does it (src/XMLBIFParser.cpp:33-179): nodes in <VARIABLE> order,
// AddParent/AddChild in <GIVEN> order, TABLE read node-major with NaryCount
// (src/common.cpp:193-232) and AddCount(query, parents, p*10000) (src/XMLBIFParser.cpp:176).
//
// Modes
//   jt  <net.xml> <libsvm test set> <pt file|-> <out prefix> [max_cases] [eval set]
//       writes <prefix>.plan (junction-tree plan after ReorganizeTableStorage),
//              <prefix>.init (initial clique potentials, %.17g),
//              <prefix>.marg (per case: label + all node marginals, %.17g)
//   jtbench / pcbench   timing of the reference's own loops for bench.py's cpu_baseline (below)
//   ci  <csv> <tests file> <out>
//       counts N_xyz for every (x, y, Z) line of <tests file> with the reference Counts2D/Counts3D
//       (src/CellTable.cpp:174-291,430-455) and writes them with the dataset's domains.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <set>
#include <stack>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "BNSLComparison.h"
#include "CellTable.h"
#include "Dataset.h"
#include "DiscreteNode.h"
#include "JunctionTree.h"
#include "Network.h"
#include "Timer.h"
#include "common.h"

#include "../mini_xml.h"

// ---------------------------------------------------------------------------------------------
// network population through the reference API
static Network *LoadXmlbifIntoReference(const std::string &path) {
    auto doc = mini_xml::parse_file(path);
    const mini_xml::Element *net = doc->first("BIF")->first("NETWORK");
    std::vector<Node *> nodes;
    for (const mini_xml::Element *xv : net->all("VARIABLE")) {
        if (Trim(const_cast<std::string &>(xv->first("TYPE")->text)) != "discrete") continue;
        auto *n = new DiscreteNode((int)nodes.size());
        std::string nm = xv->first("NAME")->text;
        n->node_name = Trim(nm);
        for (const mini_xml::Element *val : xv->all("VALUE")) {
            std::string v = val->text;
            n->vec_str_potential_vals.push_back(Trim(v));
        }
        n->SetDomainSize((int)n->vec_str_potential_vals.size());
        nodes.push_back(n);
    }
    auto find = [&](std::string name) -> Node * {
        name = Trim(name);
        for (Node *p : nodes)
            if (p->node_name == name) return p;
        fprintf(stderr, "unknown variable %s\n", name.c_str());
        exit(1);
    };
    for (const mini_xml::Element *xp : net->all("PROBABILITY")) {
        auto *for_np = dynamic_cast<DiscreteNode *>(find(xp->first("FOR")->text));
        std::vector<Node *> given;
        for (const mini_xml::Element *g : xp->all("GIVEN")) given.push_back(find(g->text));
        for (Node *g : given) {
            for_np->AddParent(g);
            g->AddChild(for_np);
        }
        std::string table = xp->first("TABLE")->text;
        table = Trim(table);
        std::vector<std::string> toks = Split(table, " ");
        std::vector<double> entries;
        for (auto &t : toks) entries.push_back(stod(t));
        std::vector<int> range;
        range.push_back(for_np->GetDomainSize());
        for (Node *g : given) range.push_back(dynamic_cast<DiscreteNode *>(g)->GetDomainSize());
        std::vector<std::vector<int>> counts = NaryCount(range);
        if (counts.size() != entries.size()) {
            fprintf(stderr, "table size mismatch for %s\n", for_np->node_name.c_str());
            exit(1);
        }
        for (size_t i = 0; i < counts.size(); ++i) {
            DiscreteConfig comb;
            for (size_t j = 1; j < counts[i].size(); ++j)
                comb.insert(std::pair<int, int>(given[j - 1]->GetNodeIndex(), counts[i][j]));
            for_np->AddCount(counts[i][0], comb, entries.at(i) * 10000);
        }
    }
    Network *network = new Network(nodes, "xmlbif");
    network->GetTopoOrd();
    return network;
}

// ---------------------------------------------------------------------------------------------
class JTHarness : public JunctionTree {
public:
    JTHarness(Network *net, Dataset *dts) : JunctionTree(net, dts, false) {}

    void DumpPlan(const std::string &path_plan, const std::string &path_init) {
        std::map<const Clique *, int> cid, sid;
        auto &C = tree->vector_clique_ptr_container;
        auto &S = tree->vector_separator_ptr_container;
        for (size_t i = 0; i < C.size(); ++i) cid[C[i]] = (int)i;
        for (size_t i = 0; i < S.size(); ++i) sid[S[i]] = (int)i;
        FILE *f = fopen(path_plan.c_str(), "w");
        fprintf(f, "cliques %zu\n", C.size());
        for (size_t i = 0; i < C.size(); ++i) {
            const PotentialTable &t = clique_backup[i].p_table;
            fprintf(f, "c %zu %d %d", i, t.num_variables, t.table_size);
            for (int v : t.vec_related_variables) fprintf(f, " %d", v);
            fprintf(f, " | up %d | down", C[i]->ptr_upstream_clique ? sid[C[i]->ptr_upstream_clique] : -1);
            for (auto *d : C[i]->ptr_downstream_cliques) fprintf(f, " %d", sid[d]);
            fprintf(f, "\n");
        }
        fprintf(f, "seps %zu\n", S.size());
        for (size_t i = 0; i < S.size(); ++i) {
            const PotentialTable &t = separator_backup[i].p_table;
            fprintf(f, "s %zu %d %d", i, t.num_variables, t.table_size);
            for (int v : t.vec_related_variables) fprintf(f, " %d", v);
            fprintf(f, " | up %d | down", cid[S[i]->ptr_upstream_clique]);
            for (auto *d : S[i]->ptr_downstream_cliques) fprintf(f, " %d", cid[d]);
            fprintf(f, "\n");
        }
        fprintf(f, "root %d\n", cid[jt_root]);
        fprintf(f, "levels %d\n", max_level);
        for (int l = 0; l < max_level; ++l) {
            fprintf(f, "level %d %c", l, (l % 2) ? 's' : 'c');
            for (auto *n : nodes_by_level[l]) fprintf(f, " %d", (l % 2) ? sid[n] : cid[n]);
            fprintf(f, "\n");
        }
        fclose(f);
        f = fopen(path_init.c_str(), "w");
        for (size_t i = 0; i < C.size(); ++i) {
            const PotentialTable &t = clique_backup[i].p_table;
            fprintf(f, "c %zu %d", i, t.table_size);
            for (double p : t.potentials) fprintf(f, " %.17g", p);
            fprintf(f, "\n");
        }
        fclose(f);
    }

    void DumpCases(const std::string &pt_path, const std::string &out_path, int max_cases) {
        if (pt_path != "-") {
            LoadGroundTruthProbabilityTable(pt_path);
        } else {
            ground_truth_probability_tables.assign(num_instances, std::vector<std::vector<double>>());
            for (auto &c : ground_truth_probability_tables) {
                c.resize(network->num_nodes);
                for (int j = 0; j < network->num_nodes; ++j)
                    c[j].assign(dynamic_cast<DiscreteNode *>(network->FindNodePtrByIndex(j))->GetDomainSize(), 0.0);
            }
        }
        int n = num_instances;
        if (max_cases > 0 && max_cases < n) n = max_cases;
        Timer timer;
        double mse = 0.0, hd = 0.0;
        FILE *f = fopen(out_path.c_str(), "w");
        for (int i = 0; i < n; ++i) {
            int label = PredictUseJTInfer(evidences.at(i), i, mse, hd, 1, &timer);
            fprintf(f, "case %d label %d\n", i, label);
            for (int v = 0; v < network->num_nodes; ++v) {
                for (size_t d = 0; d < probs_one_sample[v].size(); ++d)
                    fprintf(f, "%s%.17g", d ? " " : "", probs_one_sample[v][d]);
                fprintf(f, "\n");
            }
        }
        fprintf(f, "mse_sum %.17g hd_sum %.17g\n", mse, hd);
        fclose(f);
    }

    // evaluate a different case list on the same tree: the reference's tree shape depends on the
    // heap addresses of its cliques/separators (pointer-ordered std::set, src/JunctionTreeStructure.cpp:231,
    // include/Clique.h:22), so the tree is always built after loading the same test set
    double TimeCases(int n, int threads = 1) {
        if (n > num_instances) n = num_instances;
        ground_truth_probability_tables.assign(num_instances, std::vector<std::vector<double>>());
        for (auto &c : ground_truth_probability_tables) {
            c.resize(network->num_nodes);
            for (int j = 0; j < network->num_nodes; ++j)
                c[j].assign(dynamic_cast<DiscreteNode *>(network->FindNodePtrByIndex(j))->GetDomainSize(), 0.0);
        }
        Timer timer;
        double mse = 0.0, hd = 0.0, t0 = omp_get_wtime();
        long sink = 0;
        for (int i = 0; i < n; ++i) sink += PredictUseJTInfer(evidences.at(i), i, mse, hd, threads, &timer);
        double t = omp_get_wtime() - t0;
        if (sink < 0) printf("%ld", sink);
        return t;
    }
    struct CaseList : Inference {  // the reference's own evidence extraction (src/Inference.cpp:13-42)
        CaseList(Network *n, Dataset *d) : Inference(n, d, false) {}
        double EvaluateAccuracy(string, int) override { return 0; }
    };
    void SwapCases(Dataset *other) {
        CaseList tmp(network, other);
        evidences = tmp.evidences;
        ground_truths = tmp.ground_truths;
        num_instances = tmp.num_instances;
    }
};

static int RunJT(int argc, char **argv) {
    if (argc < 6) return 2;
    Network *net = LoadXmlbifIntoReference(argv[2]);
    auto *tester = new Dataset();
    tester->LoadLIBSVMDataKnownNetwork(argv[3], net->num_nodes);
    JTHarness jt(net, tester);
    std::string prefix = argv[5];
    jt.DumpPlan(prefix + ".plan", prefix + ".init");
    if (argc > 7) {
        auto *other = new Dataset();
        other->LoadLIBSVMDataKnownNetwork(argv[7], net->num_nodes);
        jt.SwapCases(other);
    }
    jt.DumpCases(argv[4], prefix + ".marg", argc > 6 ? atoi(argv[6]) : 0);
    return 0;
}

// ---------------------------------------------------------------------------------------------
static unsigned long long Fnv1a(const int *col, int n) {
    unsigned long long h = 1469598103934665603ull;
    for (int i = 0; i < n; ++i) {
        h ^= (unsigned long long)(unsigned)col[i];
        h *= 1099511628211ull;
    }
    return h;
}

// "cols:<file>" (int32 nvars, int64 nsamples, int32 dims[nvars], uint8 codes [nvars][nsamples]) into
// the reference's Dataset (dataset_columns int32 [var][sample], as LoadCSVData leaves them), or a CSV
// through the reference's own LoadCSVData; nullptr on a read error
static Dataset *LoadColsOrCsv(const std::string &src) {
    auto *dts = new Dataset();
    if (src.rfind("cols:", 0) != 0) {
        dts->LoadCSVData(src, true, true, 0);
        return dts;
    }
    FILE *f = fopen(src.c_str() + 5, "rb");
    if (!f) return nullptr;
    int32_t V;
    int64_t N;
    if (fread(&V, 4, 1, f) != 1 || fread(&N, 8, 1, f) != 1) return nullptr;
    dts->num_vars = V;
    dts->num_instance = (int)N;
    dts->num_of_possible_values_of_disc_vars.resize(V);
    if (fread(dts->num_of_possible_values_of_disc_vars.data(), 4, V, f) != (size_t)V) return nullptr;
    dts->dataset_columns = new int *[V];
    std::vector<uint8_t> buf(N);
    for (int v = 0; v < V; ++v) {
        if (fread(buf.data(), 1, N, f) != (size_t)N) return nullptr;
        dts->dataset_columns[v] = new int[N];
        for (int64_t k = 0; k < N; ++k) dts->dataset_columns[v][k] = buf[k];
    }
    fclose(f);
    return dts;
}

// ci <csv | cols:file> <tests file> <out>: the reference's Counts2D / Counts3D::FillTable
// (src/CellTable.cpp) for every listed test (x y z...), plus the FNV-1a hash of every column it saw
static int RunCI(int argc, char **argv) {
    if (argc < 5) return 2;
    Dataset *dts = LoadColsOrCsv(argv[2]);
    if (!dts) return 3;
    std::ifstream tin(argv[3]);
    FILE *f = fopen(argv[4], "w");
    fprintf(f, "vars %d samples %d\n", dts->num_vars, dts->num_instance);
    fprintf(f, "dims");
    for (int v = 0; v < dts->num_vars; ++v) fprintf(f, " %d", dts->num_of_possible_values_of_disc_vars[v]);
    fprintf(f, "\n");
    for (int v = 0; v < dts->num_vars; ++v)
        fprintf(f, "colhash %d %llu\n", v, Fnv1a(dts->dataset_columns[v], dts->num_instance));
    std::string line;
    Timer timer;
    while (std::getline(tin, line)) {
        line = Trim(line);
        if (line.empty()) continue;
        std::vector<std::string> tok = Split(line, " ");
        int x = stoi(tok[0]), y = stoi(tok[1]);
        std::vector<int> z;
        for (size_t i = 2; i < tok.size(); ++i) z.push_back(stoi(tok[i]));
        int dx = dts->num_of_possible_values_of_disc_vars[x];
        int dy = dts->num_of_possible_values_of_disc_vars[y];
        fprintf(f, "test %d %d %zu", x, y, z.size());
        for (int zz : z) fprintf(f, " %d", zz);
        if (z.empty()) {
            Counts2D t(dx, dy, x, y);
            t.FillTable(dts, &timer);
            fprintf(f, " cells %d :", dx * dy);
            for (int i = 0; i < dx * dy; ++i) fprintf(f, " %d", t.n[i]);
        } else {
            std::vector<int> cd;
            for (int zz : z) cd.push_back(dts->num_of_possible_values_of_disc_vars[zz]);
            Counts3D t(dx, dy, x, y, cd, z);
            t.FillTable(dts, &timer);
            fprintf(f, " cells %d :", t.dimz * dx * dy);
            for (int i = 0; i < t.dimz * dx * dy; ++i) fprintf(f, " %d", t.n[i]);
        }
        fprintf(f, "\n");
    }
    fclose(f);
    return 0;
}

// jtbench <net.xml> <tree set> <eval set> <max_cases> [threads]: wall time of the reference's
// per-case loop (PredictUseJTInfer with num_threads = threads, default 1, as EvaluateAccuracy runs
// it) -- bench.py's cpu_baseline "reference"
static int RunJTBench(int argc, char **argv) {
    if (argc < 6) return 2;
    std::streambuf *old = std::cout.rdbuf(nullptr);  // silence the reference's progress output
    Network *net = LoadXmlbifIntoReference(argv[2]);
    auto *tester = new Dataset();
    tester->LoadLIBSVMDataKnownNetwork(argv[3], net->num_nodes);
    JTHarness jt(net, tester);
    auto *other = new Dataset();
    other->LoadLIBSVMDataKnownNetwork(argv[4], net->num_nodes);
    jt.SwapCases(other);
    std::cout.rdbuf(old);
    int n = atoi(argv[5]);
    const int threads = argc > 6 ? atoi(argv[6]) : 1;
    double s = jt.TimeCases(n, threads);
    printf("cases %d seconds %.6f threads %d\n", n, s, threads);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// shd <bif> <learned>: the reference's own BNSLComparison::GetSHD (src/BNSLComparison.cpp:12-121).
// The true DAG is built from the BIF through the public Network API in CustomNetwork::LoadBIFFile's
// order (variables in declaration order, arcs per `probability` line, parents as listed) -- that
// loader itself needs tinyxml2 and is not compiled; <learned> lines are "from to directed".
static Network *NewNet(int n) {
    auto *net = new Network(true);
    for (int i = 0; i < n; ++i) {
        auto *node = new DiscreteNode(i);
        net->map_idx_node_ptr[i] = node;
    }
    net->num_nodes = n;
    return net;
}

static int RunSHD(int argc, char **argv) {
    if (argc < 4) return 2;
    std::ifstream bif(argv[2]);
    std::map<std::string, int> id;
    std::vector<std::pair<int, int>> arcs;
    std::string line;
    auto trim = [](std::string t) {
        size_t a = t.find_first_not_of(" \t\r"), b = t.find_last_not_of(" \t\r,");
        return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
    };
    while (std::getline(bif, line)) {
        line = trim(line);
        if (line.rfind("variable ", 0) == 0) {
            std::string name = line.substr(9);
            name = name.substr(0, name.find(' '));
            int k = (int)id.size();
            id[name] = k;
        } else if (line.rfind("probability", 0) == 0) {
            std::string in = line.substr(line.find('(') + 1);
            in = in.substr(0, in.find(')'));
            size_t bar = in.find('|');
            std::string child = trim(in.substr(0, bar));
            if (bar == std::string::npos) continue;
            std::string rest = in.substr(bar + 1);
            size_t pos = 0;
            while (pos < rest.size()) {
                size_t q = rest.find(',', pos);
                if (q == std::string::npos) q = rest.size();
                std::string p = trim(rest.substr(pos, q - pos));
                if (!p.empty()) arcs.push_back({id.at(p), id.at(child)});
                pos = q + 1;
            }
        }
    }
    const int n = (int)id.size();
    Network *truth = NewNet(n), *learned = NewNet(n);
    for (auto &a : arcs) {
        truth->SetParentChild(a.first, a.second);
        truth->vec_edges.push_back(Edge(truth->FindNodePtrByIndex(a.first), truth->FindNodePtrByIndex(a.second), TAIL, ARROW));
        ++truth->num_edges;
    }
    std::ifstream le(argv[3]);
    int a, b, d;
    while (le >> a >> b >> d) {
        if (d) {
            learned->SetParentChild(a, b);
            learned->vec_edges.push_back(Edge(learned->FindNodePtrByIndex(a), learned->FindNodePtrByIndex(b), TAIL, ARROW));
        } else {
            learned->vec_edges.push_back(Edge(learned->FindNodePtrByIndex(a), learned->FindNodePtrByIndex(b)));
        }
        ++learned->num_edges;
    }
    std::streambuf *old = std::cout.rdbuf(nullptr);
    BNSLComparison comp(truth, learned);
    int shd = comp.GetSHD();
    std::cout.rdbuf(old);
    printf("SHD %d\n", shd);
    return 0;
}


// ---------------------------------------------------------------------------------------------
// pcbench <csv | cols:file> <alpha> <depth> <group_size> <threads> [noerase]
// The reference's PC-stable skeleton phase timed with the reference's own data structures and
// counting code: Dataset::dataset_columns (int32 [var][sample], LoadCSVData for a CSV), Network's
// vec_edges of Edge objects + ChoiceGenerator + map adjacencies, Counts2D / Counts3D /
// Counts3DGroup::FillTable (src/CellTable.cpp), and its OpenMP structure: level 0 one
// `omp parallel for` over the edges (src/PCStable.cpp:83-129), levels >= 1 rounds of 128 popped
// edges, one CheckEdge (= one group of tests) each (:209-265), the vec_edges.erase loops after
// every level (:131-147, :310-326).  PCStable.cpp / IndependenceTest.cpp themselves need the
// absent stats/gcem headers, so the driver and the G^2 / df arithmetic
// (src/IndependenceTest.cpp:65-364) are restated here (p = 1 - P(df/2, G^2/2), parity unpinned);
// the shared counters / sepset map the reference updates racily are updated atomically here.
// "cols:<file>": int32 nvars, int64 nsamples, int32 dims[nvars], uint8 codes [nvars][nsamples].
// noerase: removals by one stable compaction instead of the O(E^2) erase loop (CI-only timing).
// Prints: tests per level, remaining edges, seconds: step 1 total, in CI rounds, in erase loops.
namespace pcb {

double GammaP(double a, double x) {
    if (x <= 0) return 0.0;
    const double lg = std::lgamma(a);
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
        const double an = -i * (i - a);
        b += 2.0;
        d = an * d + b;
        if (std::fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (std::fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (std::fabs(del - 1.0) < 1e-17) break;
    }
    return 1.0 - std::exp(-x + a * std::log(x) - lg) * h;
}

struct Res {
    bool indep;
    int first;
};

// G^2 + adjusted df over one table slice (src/IndependenceTest.cpp:94-138 / :309-347)
double G2Slice(const int *n, const int *ni, const int *nj, const int *nk, int dimz, int dimx, int dimy, long n_all,
               bool xy, int *df) {
    double g2 = 0.0;
    *df = 0;
    for (int k = 0; k < dimz; ++k) {
        int alx = 0, aly = 0;
        for (int i = 0; i < dimx; ++i) alx += (ni[k * dimx + i] > 0);
        for (int j = 0; j < dimy; ++j) aly += (nj[k * dimy + j] > 0);
        alx = (alx >= 1) ? alx : 1;
        aly = (aly >= 1) ? aly : 1;
        *df += (alx - 1) * (aly - 1);
        const long total = xy ? n_all : nk[k];
        if (total == 0) continue;
        for (int i = 0; i < dimx; ++i) {
            const long sum_row = ni[k * dimx + i];
            if (sum_row == 0) continue;
            for (int j = 0; j < dimy; ++j) {
                const long sum_col = nj[k * dimy + j];
                const long observed = n[k * dimx * dimy + i * dimy + j];
                if (sum_col == 0 || observed == 0) continue;
                const double expected = (double)sum_col * (double)sum_row / (double)total;
                g2 += 2.0 * observed * log(observed / expected);
            }
        }
    }
    return g2;
}

// IndependenceTest::IndependenceResult dispatch (src/IndependenceTest.cpp:35-58)
Res IndependenceResult(Dataset *dts, int x, int y, const vector<int> &z, int c_size, double alpha, Timer *timer) {
    const int dx = dts->num_of_possible_values_of_disc_vars[x], dy = dts->num_of_possible_values_of_disc_vars[y];
    int df = 0;
    if (z.empty()) {
        Counts2D t(dx, dy, x, y);
        t.FillTable(dts, timer);
        const double g2 = G2Slice(t.n, t.ni, t.nj, nullptr, 1, dx, dy, dts->num_instance, true, &df);
        if (df == 0) return {true, 0};
        return {1.0 - GammaP(0.5 * df, 0.5 * g2) > alpha, 0};
    }
    vector<int> cd;
    for (int v : z) cd.push_back(dts->num_of_possible_values_of_disc_vars[v]);
    if (c_size == 1) {
        Counts3D t(dx, dy, x, y, cd, z);
        t.FillTable(dts, timer);
        const double g2 = G2Slice(t.n, t.ni, t.nj, t.nk, t.dimz, dx, dy, 0, false, &df);
        if (df == 0) return {true, 0};
        return {1.0 - GammaP(0.5 * df, 0.5 * g2) > alpha, 0};
    }
    Counts3DGroup t(dx, dy, x, y, cd, z, c_size);
    t.FillTableGroup(dts, c_size, timer);
    for (int m = 0; m < c_size; ++m) {  // src/IndependenceTest.cpp:189-287 (df == 0 overwritten)
        const int off = t.cum_dims[m];
        const double g2 = G2Slice(t.n + off * dx * dy, t.ni + off * dx, t.nj + off * dy, t.nk + off, t.dimz[m], dx,
                                  dy, 0, false, &df);
        if (1.0 - GammaP(0.5 * df, 0.5 * g2) > alpha) return {true, m};
    }
    return {false, 0};
}

struct Run {
    Dataset *dts;
    Network *net;
    double alpha;
    int group_size;
    std::map<std::pair<int, int>, std::set<int>> sepset;
    long long num_ci_test = 0;
    double ci_s = 0.0, erase_s = 0.0;
    bool erase = true;
    Timer timer;
};

void FindAdjacencies(Run &R, const map<int, map<int, double>> &adj, int e, int x, int y) {  // :439-454
    set<int> s;
    for (auto &kv : adj.at(x)) s.insert(kv.first);
    s.erase(y);
    R.net->vec_edges[e].vec_adj.assign(s.begin(), s.end());
}

bool Testing(Run &R, int d, int e, int x, int y) {  // :465-551
    Edge &E = R.net->vec_edges[e];
    vector<vector<int>> choices = E.cg->NextN(R.group_size);
    if (!choices[0].empty()) {
        vector<int> Z;
        int i;
        for (i = 0; i < R.group_size; ++i) {
            if (choices[i].empty()) break;
            for (int j = 0; j < d; ++j) Z.push_back(E.vec_adj[choices[i][j]]);
        }
#pragma omp atomic
        R.num_ci_test += i;
        Res r = IndependenceResult(R.dts, x, y, Z, i, R.alpha, &R.timer);
        if (r.indep) {
            set<int> cs;
            for (int j = 0; j < d; ++j) cs.insert(E.vec_adj[choices[r.first][j]]);
#pragma omp critical(pcb_sepset)
            R.sepset.insert(make_pair(make_pair(std::min(x, y), std::max(x, y)), cs));
            return true;
        }
        E.finish = (i != R.group_size);
        return false;
    }
    E.finish = true;
    return false;
}

bool CheckEdge(Run &R, const map<int, map<int, double>> &adj, int d, int e) {  // :339-433
    Edge &E = R.net->vec_edges[e];
    const int x = E.GetNode1()->GetNodeIndex(), y = E.GetNode2()->GetNodeIndex();
    if (E.process == NO) {
        FindAdjacencies(R, adj, e, x, y);
        if ((int)E.vec_adj.size() >= d) {
            E.cg = new ChoiceGenerator((int)E.vec_adj.size(), d);
            E.process = NODE1;
        } else {
            FindAdjacencies(R, adj, e, y, x);
            if ((int)E.vec_adj.size() >= d) {
                E.cg = new ChoiceGenerator((int)E.vec_adj.size(), d);
                E.process = NODE2;
            } else {
                E.need_remove = false;
                return false;
            }
        }
    } else if (E.process == ENODE1) {
        FindAdjacencies(R, adj, e, y, x);
        if ((int)E.vec_adj.size() >= d) {
            E.cg = new ChoiceGenerator((int)E.vec_adj.size(), d);
            E.process = NODE2;
        } else {
            E.need_remove = false;
            return false;
        }
    }
    const bool ind = Testing(R, d, e, x, y);
    if (ind) {
        delete E.cg;
        E.cg = nullptr;
        E.need_remove = true;
        return false;
    }
    if (!E.finish) return true;
    delete E.cg;
    E.cg = nullptr;
    if (E.process == NODE1) {
        E.process = ENODE1;
        return true;
    }
    E.need_remove = false;
    return false;
}

void RemoveMarked(Run &R) {  // :131-147, :310-326 (or one stable compaction with noerase)
    double t0 = omp_get_wtime();
    Network *net = R.net;
    if (R.erase) {
        for (int i = 0; i < net->num_edges; ++i) {
            if (net->vec_edges[i].need_remove) {
                const int a = net->vec_edges[i].GetNode1()->GetNodeIndex(), b = net->vec_edges[i].GetNode2()->GetNodeIndex();
                net->vec_edges.erase(net->vec_edges.begin() + i);
                --net->num_edges;
                net->adjacencies[a].erase(b);
                net->adjacencies[b].erase(a);
                i--;
            }
        }
    } else {
        size_t o = 0;
        for (size_t i = 0; i < net->vec_edges.size(); ++i) {
            Edge &E = net->vec_edges[i];
            if (E.need_remove) {
                const int a = E.GetNode1()->GetNodeIndex(), b = E.GetNode2()->GetNodeIndex();
                net->adjacencies[a].erase(b);
                net->adjacencies[b].erase(a);
            } else {
                if (o != i) net->vec_edges[o] = std::move(E);
                ++o;
            }
        }
        net->vec_edges.resize(o);
        net->num_edges = (int)o;
    }
    R.erase_s += omp_get_wtime() - t0;
}

bool SearchAtDepth(Run &R, int d, int threads) {  // :209-328
    Network *net = R.net;
    map<int, map<int, double>> adj = net->adjacencies;
    std::stack<int> st;
    for (int i = net->num_edges - 1; i >= 0; --i) {
        net->vec_edges[i].process = NO;
        st.push(i);
    }
    int ids[128];
    bool push[128];
    while (!st.empty()) {
        const int size = st.size() >= 128 ? 128 : (int)st.size();
        for (int i = 0; i < size; ++i) ids[i] = st.top(), st.pop();
        const int p = size == 128 ? threads : std::min(size, threads);
        double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(p)
        for (int i = 0; i < size; ++i) push[i] = CheckEdge(R, adj, d, ids[i]);
        R.ci_s += omp_get_wtime() - t0;
        for (int i = size - 1; i >= 0; --i)
            if (push[i]) st.push(ids[i]);
    }
    RemoveMarked(R);
    int mx = 0;
    for (int i = 0; i < net->num_nodes; ++i) mx = std::max<int>(mx, (int)net->adjacencies.at(i).size());
    return mx - 1 > d;  // FreeDegree (:557-563)
}

}  // namespace pcb

static int RunPCBench(int argc, char **argv) {
    if (argc < 7) return 2;
    std::streambuf *old = std::cout.rdbuf(nullptr);
    Dataset *dts = LoadColsOrCsv(argv[2]);
    std::cout.rdbuf(old);
    if (!dts) return 3;
    pcb::Run R;
    R.dts = dts;
    R.alpha = atof(argv[3]);
    const int depth = atoi(argv[4]);
    R.group_size = atoi(argv[5]);
    const int threads = atoi(argv[6]);
    R.erase = !(argc > 7 && std::string(argv[7]) == "noerase");
    R.net = NewNet(dts->num_vars);
    Network *net = R.net;
    double t_start = omp_get_wtime();
    net->GenerateUndirectedCompleteGraph();  // step 0 (:49-65), timed with step 1 here
    for (int i = 0; i < net->num_nodes; ++i) {  // :73-81
        map<int, double> a;
        for (int j = 0; j < net->num_nodes; ++j)
            if (i != j) a.insert(make_pair(j, 1.0));
        net->adjacencies.insert(make_pair(i, a));
    }
    std::vector<long long> per_level;
    {  // level 0 (:83-129)
        long long cnt = 0;
        double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) reduction(+ : cnt)
        for (int i = 0; i < net->num_edges; ++i) {
            const int a = net->vec_edges[i].GetNode1()->GetNodeIndex(), b = net->vec_edges[i].GetNode2()->GetNodeIndex();
            ++cnt;
            pcb::Res r = pcb::IndependenceResult(dts, a, b, vector<int>(), 1, R.alpha, &R.timer);
            if (r.indep) {
                net->vec_edges[i].need_remove = true;
#pragma omp critical(pcb_sepset)
                R.sepset.insert(make_pair(make_pair(a, b), set<int>()));
            }
        }
        R.ci_s += omp_get_wtime() - t0;
        R.num_ci_test = cnt;
        pcb::RemoveMarked(R);
        per_level.push_back(cnt);
    }
    for (int d = 1; d < depth; ++d) {
        const long long before = R.num_ci_test;
        const bool more = pcb::SearchAtDepth(R, d, threads);
        per_level.push_back(R.num_ci_test - before);
        if (!more) break;
    }
    const double total = omp_get_wtime() - t_start;
    printf("tests");
    for (long long c : per_level) printf(" %lld", c);
    printf(" | edges %d | total_s %.6f ci_s %.6f erase_s %.6f threads %d\n", net->num_edges, total, R.ci_s, R.erase_s,
           threads);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && std::string(argv[1]) == "shd") return RunSHD(argc, argv);
    if (argc >= 2 && std::string(argv[1]) == "jtbench") return RunJTBench(argc, argv);
    if (argc >= 2 && std::string(argv[1]) == "jt") return RunJT(argc, argv);
    if (argc >= 2 && std::string(argv[1]) == "ci") return RunCI(argc, argv);
    if (argc >= 2 && std::string(argv[1]) == "pcbench") return RunPCBench(argc, argv);
    fprintf(stderr, "usage: ref_dump jt|ci ...\n");
    return 2;
}
