// pc_orient.cpp -- PC-stable orientation (v-structures + Meek rules 1-3) and the SHD against a
// reference BIF graph, host side.  Mirrors the reference's graph-edit semantics exactly, including
// the order-dependent details that decide the final DAG/CPDAG:
//   * OrientVStructure (src/PCStable.cpp:576-668): nodes b ascending, pairs of b's (skeleton)
//     neighbours in ChoiceGenerator order; conflicting directions are overwritten, and an edit that
//     would close a cycle is rolled back to the edge it replaced;
//   * OrientImplied (src/PCStable.cpp:679-703): sweeps over vec_edges by position until a sweep
//     orients nothing; an oriented edge is erased at its position and re-appended, and a rejected
//     Direct() re-appends the undirected edge -- the sweep then advances past the element that slid
//     into the current position (the reference's iterator arithmetic, reproduced);
//   * Rule3 (src/PCStable.cpp:812-843) indexes nodes by *position* in the common-neighbour set,
//     not by node id -- reproduced;
//   * cycle checks: Kahn's algorithm over the directed part (Network::ContainCircle, src/Network.cpp:670);
//   * SHD (src/BNSLComparison.cpp:12-121): true DAG from BIF (CustomNetwork::LoadBIFFile,
//     src/CustomNetwork.cpp:49-160) -> Chickering edge ordering + compelled/reversible labelling
//     (src/Network.cpp:731-869) -> reversible edges undirected -> one error per node pair whose
//     first matching edge (undirected, x->y, y->x) differs.
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <fstream>
#include <map>
#include <queue>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "fbn_internal.h"
#include "pc_internal.h"

namespace fbn {

namespace {

enum { ARROW = 0, TAIL = 1 };

// a node's parents / children / skeleton neighbours: a sorted array (iteration in ascending node
// index, as the reference's node-pointer sets).  Degrees are small, so the first kInline members
// live inline: building 3n sets and editing a few hundred arcs then allocates nothing (a vector per
// set cost ~0.1 ms of a 1000-variable orientation in allocations alone)
class IntSet {
  public:
    bool insert(int x) {
        int *b = data(), *e = b + n_;
        int *it = std::lower_bound(b, e, x);
        if (it != e && *it == x) return false;
        const size_t at = (size_t)(it - b);
        if (!big_ && n_ == kInline) heap_.assign(inl_, inl_ + n_), big_ = true;
        if (big_) {
            heap_.insert(heap_.begin() + at, x);
        } else {
            std::copy_backward(inl_ + at, inl_ + n_, inl_ + n_ + 1);
            inl_[at] = x;
        }
        ++n_;
        return true;
    }
    bool erase(int x) {
        int *b = data(), *e = b + n_;
        int *it = std::lower_bound(b, e, x);
        if (it == e || *it != x) return false;
        if (big_) heap_.erase(heap_.begin() + (it - b));
        else std::copy(it + 1, e, it);
        --n_;
        return true;
    }
    size_t count(int x) const { return std::binary_search(begin(), end(), x) ? 1 : 0; }
    size_t size() const { return (size_t)n_; }
    const int *begin() const { return big_ ? heap_.data() : inl_; }
    const int *end() const { return begin() + n_; }

  private:
    static constexpr int kInline = 6;
    int *data() { return big_ ? heap_.data() : inl_; }
    int n_ = 0;
    bool big_ = false;  // once spilled, the members stay in heap_
    int inl_[kInline];
    std::vector<int> heap_;
};

struct GEdge {
    int n1, n2, ep1, ep2;
    bool operator==(const GEdge &o) const { return n1 == o.n1 && n2 == o.n2 && ep1 == o.ep1 && ep2 == o.ep2; }
    bool directed() const { return (ep1 == ARROW && ep2 == TAIL) || (ep2 == ARROW && ep1 == TAIL); }
};

GEdge Undirected(int a, int b) { return GEdge{std::min(a, b), std::max(a, b), TAIL, TAIL}; }
GEdge Directed(int p, int c) { return GEdge{p, c, TAIL, ARROW}; }

// The reference's vec_edges (a std::vector of edges: push_back, erase of the first equal element
// found by a linear search, positional sweeps) with the same order semantics in O(1) / O(log E)
// per operation: edges live in append-only slots, an erased slot becomes a tombstone, a Fenwick
// tree over the live flags maps a position to its slot, and an open-addressing table maps every
// edge to the chain of its live slots in ascending order (its head = the linear search's hit).
class EdgeSeq {
  public:
    int size() const { return nlive_; }
    int slots() const { return (int)e_.size(); }
    bool live(int s) const { return live_[s] != 0; }
    const GEdge &at_slot(int s) const { return e_[s]; }
    int64_t erasures() const { return nerased_; }
    void reserve(size_t n) {
        e_.reserve(n), live_.reserve(n), next_.reserve(n);
        Rehash(4 * n);
    }
    void push(const GEdge &g) {
        const int s = (int)e_.size();
        e_.push_back(g), live_.push_back(1), next_.push_back(-1);
        if ((int)e_.size() > cap_) Rebuild();
        else FenAdd(s, 1);
        ++nlive_;
        Ent &h = Insert(Key(g));
        if (h.head < 0) h.head = h.tail = s;
        else next_[h.tail] = s, h.tail = s;
    }
    int find(const GEdge &g) const {  // slot of the first live equal edge, -1 if none
        const Ent *h = Lookup(Key(g));
        return h ? h->head : -1;
    }
    bool erase_first(const GEdge &g) {
        const uint64_t k = Key(g);
        Ent *h = const_cast<Ent *>(Lookup(k));
        if (!h) return false;
        const int s = h->head;
        h->head = next_[s];
        if (h->head < 0) Remove(k);
        live_[s] = 0;
        FenAdd(s, -1);
        --nlive_, ++nerased_;
        return true;
    }
    int slot_at(int pos) const {  // the slot at position pos (0-based among live slots)
        int idx = 0, rem = pos + 1;
        for (int step = cap_; step > 0; step >>= 1)
            if (idx + step <= cap_ && fen_[idx + step] < rem) idx += step, rem -= fen_[idx];
        return idx;
    }
    int next_live(int s) const {  // first live slot after s (slots() if none)
        do ++s;
        while (s < (int)e_.size() && !live_[s]);
        return s;
    }
    // overwrite the edge of a slot alone in its chain (the SHD's reversible arcs of a DAG)
    void replace_single(int s, const GEdge &g) {
        Remove(Key(e_[s]));
        e_[s] = g;
        Ent &h = Insert(Key(g));
        if (h.head < 0) h.head = h.tail = s;
        else next_[h.tail] = s, h.tail = s;
    }

  private:
    struct Ent {
        int head = -1, tail = -1;
    };
    static uint64_t Key(const GEdge &g) {
        return (uint64_t)(uint32_t)g.n1 << 34 ^ (uint64_t)(uint32_t)g.n2 << 2 ^ (uint64_t)(g.ep1 << 1 | g.ep2);
    }
    static size_t Hash(uint64_t k) {
        k ^= k >> 33, k *= 0xff51afd7ed558ccdull, k ^= k >> 33;
        return (size_t)k;
    }
    // open addressing, linear probing; state 0 empty, 1 full, 2 deleted
    std::vector<uint64_t> keys_;
    std::vector<Ent> vals_;
    std::vector<uint8_t> state_;
    size_t used_ = 0;  // full + deleted
    const Ent *Lookup(uint64_t k) const {
        if (keys_.empty()) return nullptr;
        const size_t m = keys_.size() - 1;
        for (size_t i = Hash(k) & m;; i = (i + 1) & m) {
            if (state_[i] == 0) return nullptr;
            if (state_[i] == 1 && keys_[i] == k) return &vals_[i];
        }
    }
    Ent &Insert(uint64_t k) {
        if (keys_.empty() || 2 * (used_ + 1) > keys_.size()) Rehash(4 * (used_ + 1));
        const size_t m = keys_.size() - 1;
        size_t tomb = SIZE_MAX;
        for (size_t i = Hash(k) & m;; i = (i + 1) & m) {
            if (state_[i] == 1 && keys_[i] == k) return vals_[i];
            if (state_[i] == 2 && tomb == SIZE_MAX) tomb = i;
            if (state_[i] == 0) {
                const size_t j = tomb != SIZE_MAX ? tomb : i;
                if (state_[j] == 0) ++used_;
                state_[j] = 1, keys_[j] = k, vals_[j] = Ent();
                return vals_[j];
            }
        }
    }
    void Remove(uint64_t k) {
        const size_t m = keys_.size() - 1;
        for (size_t i = Hash(k) & m;; i = (i + 1) & m) {
            if (state_[i] == 0) return;
            if (state_[i] == 1 && keys_[i] == k) {
                state_[i] = 2;
                return;
            }
        }
    }
    void Rehash(size_t want) {
        size_t cap = 64;
        while (cap < want) cap <<= 1;
        std::vector<uint64_t> k0(cap, 0);
        std::vector<Ent> v0(cap);
        std::vector<uint8_t> s0(cap, 0);
        k0.swap(keys_), v0.swap(vals_), s0.swap(state_);
        used_ = 0;
        for (size_t i = 0; i < s0.size(); ++i)
            if (s0[i] == 1) Insert(k0[i]) = v0[i];
    }
    // Fenwick tree over live_ (1-based, cap_ a power of two)
    std::vector<GEdge> e_;
    std::vector<uint8_t> live_;
    std::vector<int> next_, fen_;
    int cap_ = 0, nlive_ = 0;
    int64_t nerased_ = 0;
    void FenAdd(int s, int v) {
        for (int i = s + 1; i <= cap_; i += i & -i) fen_[i] += v;
    }
    void Rebuild() {
        int cap = std::max(cap_, 64);
        while (cap < (int)e_.size()) cap <<= 1;
        cap_ = cap;
        fen_.assign(cap_ + 1, 0);
        for (size_t s = 0; s < live_.size(); ++s) fen_[s + 1] = live_[s];
        for (int i = 1; i <= cap_; ++i) {
            const int j = i + (i & -i);
            if (j <= cap_) fen_[j] += fen_[i];
        }
    }
};

// the reference's Network state used by orientation: edge list + parent/child sets
struct Graph {
    int n = 0;
    EdgeSeq edges;  // vec_edges
    std::vector<IntSet> parents, children;
    explicit Graph(int nn) : n(nn), parents(nn), children(nn) {}

    int Find(const GEdge &e) const { return edges.find(e); }  // slot of the first equal edge, -1 if none
    bool ContainCircle() const {
        std::vector<int> indeg(n, 0);
        for (int i = 0; i < n; ++i)
            for (int c : children[i]) ++indeg[c];
        std::queue<int> q;
        for (int i = 0; i < n; ++i)
            if (!indeg[i]) q.push(i);
        int visited = 0;
        while (!q.empty()) {
            const int u = q.front();
            q.pop();
            ++visited;
            for (int c : children[u])
                if (--indeg[c] == 0) q.push(c);
        }
        return visited != n;
    }
    // A topological order of the directed part kept up to date (Pearce & Kelly's dynamic order):
    // ord[v] = position of v, at[i] = node at position i.  Deletions keep an order valid; an added
    // p -> c with ord[p] < ord[c] cannot close a cycle; otherwise c reaches p iff a forward search
    // from c through positions <= ord[p] finds p, and if not the nodes found forward from c and
    // backward from p are re-slotted (backward ones first) into the positions they occupied.
    std::vector<int> ord, at, stamp, stack, fw, bw, slots;
    int epoch = 0;
    void InitOrder() {
        if (ord.size() == (size_t)n) return;
        ord.resize(n), at.resize(n), stamp.assign(n, 0);
        for (int i = 0; i < n; ++i) ord[i] = at[i] = i;
    }
    // does c reach p?  (true: the add would close a cycle); if not, the order is fixed for p -> c
    bool ClosesCycle(int p, int c) {
        InitOrder();
        if (p == c) return true;
        if (ord[p] < ord[c]) return false;
        const int ub = ord[p], lb = ord[c];
        ++epoch;
        fw.clear(), stack.clear();
        stack.push_back(c), stamp[c] = epoch;
        while (!stack.empty()) {
            const int u = stack.back();
            stack.pop_back();
            if (u == p) return true;
            fw.push_back(u);
            for (int v : children[u])
                if (stamp[v] != epoch && ord[v] <= ub) stamp[v] = epoch, stack.push_back(v);
        }
        ++epoch;
        bw.clear();
        stack.push_back(p), stamp[p] = epoch;
        while (!stack.empty()) {
            const int u = stack.back();
            stack.pop_back();
            bw.push_back(u);
            for (int v : parents[u])
                if (stamp[v] != epoch && ord[v] >= lb) stamp[v] = epoch, stack.push_back(v);
        }
        auto by_ord = [&](int a, int b) { return ord[a] < ord[b]; };
        std::sort(fw.begin(), fw.end(), by_ord);
        std::sort(bw.begin(), bw.end(), by_ord);
        slots.clear();
        for (int v : bw) slots.push_back(ord[v]);
        for (int v : fw) slots.push_back(ord[v]);
        std::sort(slots.begin(), slots.end());
        size_t k = 0;
        for (int v : bw) ord[v] = slots[k], at[slots[k]] = v, ++k;
        for (int v : fw) ord[v] = slots[k], at[slots[k]] = v, ++k;
        return false;
    }
    // the reference adds the edge and rolls it back if Network::ContainCircle() then holds.  Every
    // cycle-closing add is rolled back and deletions close no cycle, so the graph is acyclic before
    // each add, and the new edge p -> c closes a cycle iff c already reaches p: the same answer as a
    // whole-graph Kahn pass (ContainCircle above), usually without any search (ClosesCycle)
    bool AddDirected(int p, int c) {
        const bool cyc = ClosesCycle(p, c);
        parents[c].insert(p);
        children[p].insert(c);
        edges.push(Directed(p, c));
        if (cyc) DeleteDirected(p, c);
        return !cyc;
    }
    bool DeleteDirected(int p, int c) {
        if (!parents[c].count(p)) return false;
        if (!edges.erase_first(Directed(p, c))) return false;
        parents[c].erase(p);
        children[p].erase(c);
        return true;
    }
    void AddUndirected(int a, int b) { edges.push(Undirected(a, b)); }
    bool DeleteUndirected(int a, int b) { return edges.erase_first(Undirected(a, b)); }
    bool IsDirectedFromTo(int a, int b) const { return parents[b].count(a) != 0; }
    // first matching edge for the SHD: undirected, a->b, b->a
    int GetEdge(int a, int b) const {
        int pos = Find(Undirected(a, b));
        if (pos < 0) pos = Find(Directed(a, b));
        if (pos < 0) pos = Find(Directed(b, a));
        return pos;
    }
};

struct Orienter {
    Graph g;
    std::vector<IntSet> adj;  // skeleton adjacencies (fixed during orientation)
    const SepsetMap &sepset;

    Orienter(int n, const std::vector<std::pair<int, int>> &skeleton,
             const SepsetMap &ss)
        : g(n), adj(n), sepset(ss) {
        g.edges.reserve(2 * skeleton.size() + 16);
        for (auto &e : skeleton) {
            g.AddUndirected(e.first, e.second);
            adj[e.first].insert(e.second);
            adj[e.second].insert(e.first);
        }
    }
    bool IsAdjacentTo(int a, int b) const { return a >= 0 && a < g.n && adj[a].count(b) != 0; }
    bool IsUndirectedFromTo(int a, int b) const {
        return IsAdjacentTo(a, b) && !g.IsDirectedFromTo(a, b) && !g.IsDirectedFromTo(b, a);
    }
    void VStructures() {
        // the skeleton adjacencies and the sepsets stay fixed while edges are oriented, so which
        // triples a - b - c are unshielded with b outside sepset(a, c) is known up front: collected
        // in the reference's visiting order, their sepsets looked up in one batch (find_many), then
        // the edits applied in that order
        struct Triple {
            int a, b, c;
        };
        std::vector<Triple> tri;
        std::vector<std::pair<int, int>> keys;
        for (int b = 0; b < g.n; ++b) {
            const int *nb = adj[b].begin();  // ascending, as the reference's neighbour set
            const size_t nn = adj[b].size();
            for (size_t i = 0; i < nn; ++i)
                for (size_t j = i + 1; j < nn; ++j) {  // ChoiceGenerator(k, 2) order
                    const int a = nb[i], c = nb[j];
                    if (IsAdjacentTo(a, c)) continue;
                    tri.push_back({a, b, c});
                    keys.push_back({a, c});
                }
        }
        std::vector<SepsetMap::View> z(tri.size());
        std::vector<char> found(tri.size());
        auto tq = std::chrono::steady_clock::now();
        sepset.find_many(keys.data(), keys.size(), z.data(), found.data());
        auto tr = std::chrono::steady_clock::now();
        if (getenv("FBN_PC_TIMING"))
            fprintf(stderr, "orient: %zu unshielded triples, sepset lookups %.3f ms\n", tri.size(),
                    std::chrono::duration<double, std::milli>(tr - tq).count());
        for (size_t t = 0; t < tri.size(); ++t) {
            const int a = tri[t].a, b = tri[t].b, c = tri[t].c;
            if (found[t] && std::find(z[t].begin(), z[t].end(), b) != z[t].end()) continue;
            const bool dd1 = g.DeleteDirected(b, a);
            const bool du1 = dd1 ? false : g.DeleteUndirected(a, b);
            const bool add1 = dd1 || du1;
            const bool dd2 = g.DeleteDirected(b, c);
            const bool du2 = dd2 ? false : g.DeleteUndirected(c, b);
            const bool add2 = dd2 || du2;
            const bool ok1 = add1 ? g.AddDirected(a, b) : false;
            const bool ok2 = add2 ? g.AddDirected(c, b) : false;
            if (add1 && !ok1) {
                if (dd1) g.AddDirected(b, a);
                else g.AddUndirected(a, b);
            }
            if (add2 && !ok2) {
                if (dd2) g.AddDirected(b, c);
                else g.AddUndirected(c, b);
            }
        }
    }
    bool Direct(int a, int c) {
        g.DeleteUndirected(a, c);
        const bool added = g.AddDirected(a, c);
        if (!added) g.AddUndirected(a, c);
        return added;
    }
    // common skeleton neighbours into a caller's reused buffer (Rule2 / Rule3 run per edge and sweep)
    const std::vector<int> &Common(int x, int y, std::vector<int> &r) const {
        r.clear();
        std::set_intersection(adj[x].begin(), adj[x].end(), adj[y].begin(), adj[y].end(), std::back_inserter(r));
        return r;
    }
    std::vector<int> common2_, common3_;
    bool Rule1(int b, int c) {
        // node-pointer order == index order; Direct(b, c) edits parents[c] / children[b] only, so
        // b's parent set is stable while it is walked
        const IntSet &par = g.parents[b];
        for (int a : par) {
            if (IsAdjacentTo(c, a)) continue;
            if (Direct(b, c)) return true;
        }
        return false;
    }
    bool Rule2(int a, int c) {
        for (int b : Common(a, c, common2_))
            if (g.IsDirectedFromTo(a, b) && g.IsDirectedFromTo(b, c) && Direct(a, c)) return true;
        return false;
    }
    bool Rule3(int d, int a) {
        const std::vector<int> &common = Common(a, d, common3_);
        if (common.size() < 2) return false;
        // positions in the common set used as node ids, as in the reference
        for (int b = 0; b < (int)common.size(); ++b)
            for (int c = b + 1; c < (int)common.size(); ++c)
                if (!IsAdjacentTo(b, c) && IsUndirectedFromTo(d, b) && IsUndirectedFromTo(d, c) &&
                    g.IsDirectedFromTo(b, a) && g.IsDirectedFromTo(c, a) && Direct(d, a))
                    return true;
        return false;
    }
    void Implied() {
        bool oriented = true;
        while (oriented) {
            oriented = false;
            // position i of vec_edges = live slot s; a step that erased nothing moves to the next
            // live slot, otherwise the slot of the step's next position is looked up
            int s = g.edges.size() ? g.edges.slot_at(0) : 0;
            for (int i = 0; i < g.edges.size();) {
                const int x = g.edges.at_slot(s).n1, y = g.edges.at_slot(s).n2;
                const int64_t er = g.edges.erasures();
                bool stay = false;
                if (IsUndirectedFromTo(x, y)) {
                    if (Rule1(x, y) || Rule1(y, x) || Rule2(x, y) || Rule2(y, x) || Rule3(x, y) || Rule3(y, x))
                        oriented = stay = true;  // edge at i erased: i now holds the next one
                }
                if (!stay) ++i;
                if (!stay && g.edges.erasures() == er) s = g.edges.next_live(s);
                else if (i < g.edges.size()) s = g.edges.slot_at(i);
            }
        }
    }
};

std::string Trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

}  // namespace

int OrientPC(int nvars, PCResultHost &r) {
    static const bool timing = getenv("FBN_PC_TIMING") != nullptr;  // diagnostic
    auto t0 = std::chrono::steady_clock::now();
    Orienter o(nvars, r.edges, r.sepset);
    auto t1 = std::chrono::steady_clock::now();
    o.VStructures();
    auto t2 = std::chrono::steady_clock::now();
    o.Implied();
    if (timing) {
        auto t3 = std::chrono::steady_clock::now();
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        fprintf(stderr, "orient: setup %.3f ms, v-structures %.3f ms, implied %.3f ms\n", ms(t0, t1), ms(t1, t2),
                ms(t2, t3));
    }
    r.oriented.clear();
    for (int sl = 0; sl < o.g.edges.slots(); ++sl) {
        if (!o.g.edges.live(sl)) continue;
        const GEdge &e = o.g.edges.at_slot(sl);
        if (!e.directed()) r.oriented.push_back({e.n1, e.n2, 0});
        else if (e.ep1 == TAIL) r.oriented.push_back({e.n1, e.n2, 1});
        else r.oriented.push_back({e.n2, e.n1, 1});
    }
    r.num_nodes = nvars;
    return FBN_OK;
}

// true DAG from a BIF file: node ids in `variable` declaration order, arcs from `probability` lines
int LoadBifGraph(const std::string &path, std::vector<std::string> &names, std::vector<std::pair<int, int>> &arcs) {
    std::ifstream in(path);
    if (!in) return SetError(FBN_ERR_IO, "cannot open %s", path.c_str());
    std::map<std::string, int> id;
    std::string line;
    names.clear();
    arcs.clear();
    while (std::getline(in, line)) {
        line = Trim(line);
        if (line.compare(0, 9, "variable ") == 0) {
            std::istringstream ss(line.substr(9));
            std::string name;
            ss >> name;
            id[name] = (int)names.size();
            names.push_back(name);
        } else if (line.compare(0, 11, "probability") == 0) {
            const size_t lp = line.find('('), rp = line.find(')');
            if (lp == std::string::npos || rp == std::string::npos) return SetError(FBN_ERR_IO, "%s: bad line '%s'", path.c_str(), line.c_str());
            std::string inner = line.substr(lp + 1, rp - lp - 1);
            const size_t bar = inner.find('|');
            const std::string child = Trim(inner.substr(0, bar));
            if (!id.count(child)) return SetError(FBN_ERR_IO, "%s: unknown variable %s", path.c_str(), child.c_str());
            if (bar == std::string::npos) continue;
            std::string rest = inner.substr(bar + 1);
            std::istringstream ps(rest);
            std::string tok;
            while (std::getline(ps, tok, ',')) {
                const std::string p = Trim(tok);
                if (p.empty()) continue;
                if (!id.count(p)) return SetError(FBN_ERR_IO, "%s: unknown variable %s", path.c_str(), p.c_str());
                arcs.push_back({id[p], id[child]});
            }
        }
    }
    if (names.empty()) return SetError(FBN_ERR_IO, "%s: no variables", path.c_str());
    return FBN_OK;
}

// SHD between the learned (oriented) graph and the CPDAG of a true DAG
int ComputeSHD(int n, const std::vector<std::pair<int, int>> &arcs, const std::vector<std::array<int, 3>> &learned,
               int *shd, int *unlabelled) {
    int r_unlabelled = 0;
    Graph t(n);
    for (auto &a : arcs) {
        t.parents[a.second].insert(a.first);
        t.children[a.first].insert(a.second);
        t.edges.push(Directed(a.first, a.second));
    }
    if (t.ContainCircle()) return SetError(FBN_ERR_ARG, "true graph is not a DAG");
    // topological order: Kahn, queue, children scanned by ascending index (TopoSortOfDAGZeroInDegreeFirst)
    std::vector<int> indeg(n, 0), topo;
    for (int i = 0; i < n; ++i)
        for (int c : t.children[i]) ++indeg[c];
    std::queue<int> q;
    for (int i = 0; i < n; ++i)
        if (!indeg[i]) q.push(i);
    while (!q.empty()) {
        const int u = q.front();
        q.pop();
        topo.push_back(u);
        for (int c : t.children[u])
            if (--indeg[c] == 0) q.push(c);
    }
    // OrderEdge: for y in topo order, parents x from the highest-ordered down
    std::vector<GEdge> order;
    std::vector<bool> ordered(t.edges.size(), false);
    for (size_t j = 0; j < topo.size(); ++j) {
        const int y = topo[j];
        for (int k = (int)j - 1; k >= 0; --k) {
            const int x = topo[k];
            if (!t.parents[y].count(x)) continue;
            const int pos = t.Find(Directed(x, y));
            if (!ordered[pos]) ordered[pos] = true, order.push_back(t.edges.at_slot(pos));
        }
    }
    if (order.size() != (size_t)t.edges.size()) return SetError(FBN_ERR_ARG, "true graph has duplicate arcs");
    // FindCompelled (Chickering 1995)
    enum { UNKNOWN = 0, COMPELLED = 1, REVERSIBLE = 2 };
    std::vector<int> label(t.edges.size(), UNKNOWN);
    auto in_order = [&](int p, int c) {
        auto it = std::find(order.begin(), order.end(), Directed(p, c));
        return it == order.end() ? -1 : (int)(it - order.begin());
    };
    auto lab = [&](int p, int c) -> int & { return label[t.Find(Directed(p, c))]; };
    while (!order.empty()) {
        const int x = order[0].n1, y = order[0].n2;
        bool done = false;
        for (int w : t.parents[x]) {
            if (lab(w, x) != COMPELLED) continue;
            if (!t.parents[y].count(w)) {
                done = true;
                lab(x, y) = COMPELLED;
                order.erase(order.begin());
                for (int py : t.parents[y]) {
                    const int po = in_order(py, y);
                    lab(py, y) = COMPELLED;
                    if (po >= 0) order.erase(order.begin() + po);
                }
                break;
            } else {
                const int po = in_order(w, y);
                if (po >= 0) lab(w, y) = COMPELLED, order.erase(order.begin() + po);
            }
        }
        if (done) continue;
        bool found = false;
        const IntSet py_set = t.parents[y];
        for (int z : py_set) {
            if (z == x || t.parents[x].count(z)) continue;
            // as in the reference (src/Network.cpp:828-845): x->y is labelled and the *front* of the
            // order is erased on every hit; a second hit drops an unrelated edge unlabelled
            if (found && !order.empty()) ++r_unlabelled;
            found = true;
            lab(x, y) = COMPELLED;
            if (!order.empty()) order.erase(order.begin());
            for (int py : t.parents[y]) {
                const int po = in_order(py, y);
                if (po >= 0) lab(py, y) = COMPELLED, order.erase(order.begin() + po);
            }
        }
        if (!found) {
            lab(x, y) = REVERSIBLE;
            order.erase(order.begin());
            for (int py : t.parents[y]) {
                const int po = in_order(py, y);
                if (po >= 0) lab(py, y) = REVERSIBLE, order.erase(order.begin() + po);
            }
        }
    }
    for (int i = 0; i < t.edges.slots(); ++i)  // (no erasures in t: slot = position)
        if (label[i] == REVERSIBLE) t.edges.replace_single(i, Undirected(t.edges.at_slot(i).n1, t.edges.at_slot(i).n2));
    Graph l(n);
    for (auto &e : learned) l.edges.push(e[2] ? Directed(e[0], e[1]) : Undirected(e[0], e[1]));
    int err = 0;
    for (int a = 0; a < n; ++a)
        for (int b = a + 1; b < n; ++b) {
            const int p1 = t.GetEdge(a, b), p2 = l.GetEdge(a, b);
            if (p1 < 0 && p2 < 0) continue;
            if (p1 >= 0 && p2 >= 0 && t.edges.at_slot(p1) == l.edges.at_slot(p2)) continue;
            ++err;
        }
    *shd = err;
    if (unlabelled) *unlabelled = r_unlabelled;
    return FBN_OK;
}

}  // namespace fbn
