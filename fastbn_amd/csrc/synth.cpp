// synth.cpp -- seeded synthetic workloads, native (§8(f) rank 4).
//
// The reference's own generator (src/SampleSetGenerator.cpp) is wall-clock seeded and unreachable
// from its CLI, so the workloads are defined by this repository: forward (ancestral) sampling of
// complete cases from a network's CPTs (the reference's (count+1)/(total+|dom|) convention), and
// evidence cases that observe k variables per case drawn without replacement (never the query).
// The native generators draw exactly the numbers numpy's PCG64(seed) draws in
// fastbn_amd/synth.py (SeedSequence -> PCG64 XSL-RR 128/64 -> 53-bit doubles), so both produce
// bit-identical datasets and the committed fixtures hold for either (tests/test_host.py).  Also:
// writers of the CSV / LIBSVM text formats the reference loads (src/Dataset.cpp:35-414), used to
// time the loaders at benchmark scale.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "fbn_internal.h"

namespace fbn {

namespace {

// numpy.random.SeedSequence(seed).generate_state(4, uint64) (pool size 4, no spawn key)
void SeedSequenceState(uint64_t seed, uint64_t out[4]) {
    const uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
    const uint32_t MIX_MULT_L = 0xca01f9ddu, MIX_MULT_R = 0x4973f715u;
    std::vector<uint32_t> entropy;
    do {  // the integer as little-endian 32-bit words (0 -> [0])
        entropy.push_back((uint32_t)(seed & 0xFFFFFFFFu));
        seed >>= 32;
    } while (seed);
    uint32_t hash_const = INIT_A;
    auto hashmix = [&](uint32_t v) {
        v ^= hash_const;
        hash_const *= MULT_A;
        v *= hash_const;
        v ^= v >> 16;
        return v;
    };
    auto mix = [&](uint32_t x, uint32_t y) {
        uint32_t r = MIX_MULT_L * x - MIX_MULT_R * y;
        r ^= r >> 16;
        return r;
    };
    uint32_t pool[4];
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < (int)entropy.size() ? entropy[i] : 0u);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
    for (size_t s = 4; s < entropy.size(); ++s)
        for (int d = 0; d < 4; ++d) pool[d] = mix(pool[d], hashmix(entropy[s]));
    uint32_t hb = INIT_B, words[8];
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i % 4];
        v ^= hb;
        hb *= MULT_B;
        v *= hb;
        v ^= v >> 16;
        words[i] = v;
    }
    for (int i = 0; i < 4; ++i) out[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
}

// numpy.random.PCG64: 128-bit LCG, XSL-RR output; random() = (next64 >> 11) * 2^-53
struct Pcg64 {
    unsigned __int128 state, inc;
    static constexpr unsigned __int128 kMult =
        ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | (unsigned __int128)0x4385DF649FCCF645ull;
    explicit Pcg64(uint64_t seed) {
        uint64_t v[4];
        SeedSequenceState(seed, v);
        const unsigned __int128 initstate = ((unsigned __int128)v[0] << 64) | v[1];
        const unsigned __int128 initseq = ((unsigned __int128)v[2] << 64) | v[3];
        state = 0;
        inc = (initseq << 1) | 1;
        step();
        state += initstate;
        step();
    }
    void step() { state = state * kMult + inc; }
    // jump ahead by `delta` steps (the LCG's affine map composed by squaring, O(log delta))
    void advance(uint64_t delta) {
        unsigned __int128 acc_mult = 1, acc_plus = 0, cur_mult = kMult, cur_plus = inc;
        while (delta) {
            if (delta & 1) acc_mult *= cur_mult, acc_plus = acc_plus * cur_mult + cur_plus;
            cur_plus = (cur_mult + 1) * cur_plus;
            cur_mult *= cur_mult;
            delta >>= 1;
        }
        state = acc_mult * state + acc_plus;
    }
    uint64_t next64() {
        step();
        const uint64_t hi = (uint64_t)(state >> 64), lo = (uint64_t)state;
        const unsigned rot = (unsigned)(state >> 122);
        const uint64_t x = hi ^ lo;
        return (x >> rot) | (x << ((64 - rot) & 63));
    }
    double random() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }
};

// synth.py _topo: Kahn's algorithm with a LIFO stack, children in ascending order
std::vector<int> TopoOrder(const Network &net) {
    const int n = net.n();
    std::vector<int> indeg(n, 0);
    std::vector<std::vector<int>> children(n);
    for (int c = 0; c < n; ++c) {
        std::vector<int> ps(net.given[c]);
        std::sort(ps.begin(), ps.end());
        ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
        indeg[c] = (int)ps.size();
        for (int p : ps) children[p].push_back(c);
    }
    std::vector<int> order, st;
    for (int i = n - 1; i >= 0; --i)
        if (indeg[i] == 0) st.push_back(i);
    while (!st.empty()) {
        const int u = st.back();
        st.pop_back();
        order.push_back(u);
        for (int c : children[u])
            if (--indeg[c] == 0) st.push_back(c);
    }
    return order;
}

int GenThreads() {
    const unsigned hc = std::thread::hardware_concurrency();
    int t = (int)std::max(1u, std::min(16u, hc ? hc : 1u));
    if (const char *e = getenv("OMP_NUM_THREADS")) t = std::max(1, std::min(t, atoi(e)));
    return t;
}

// fn(t, begin, end) over [0, n) in T contiguous ranges, in parallel
template <class F>
void ParallelRanges(int64_t n, F fn) {
    const int T = (int)std::min<int64_t>(GenThreads(), std::max<int64_t>(1, n / 4096));
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(fn, t, n * t / T, n * (t + 1) / T);
    fn(0, 0, n / T);
    for (auto &x : th) x.join();
}

}  // namespace

int ForwardSample(const Network &net, int64_t n, uint64_t seed, uint8_t *cols) {
    const int V = net.n();
    std::vector<int> order = TopoOrder(net);
    if ((int)order.size() != V) return SetError(FBN_ERR_ARG, "network has a cycle");
    Pcg64 rng(seed);
    for (int v : order) {
        // cdf rows of every parent configuration (GIVEN order, last fastest), values in order
        const std::vector<int> &g = net.given[v];
        int64_t ncfg = 1;
        for (int p : g) ncfg *= net.dom[p];
        const int d = net.dom[v];
        std::vector<double> cdf((size_t)(ncfg * d));
        std::vector<int> gv(g.size(), 0), asc(net.parents_asc[v].size(), 0);
        for (int64_t pc = 0; pc < ncfg; ++pc) {
            for (size_t a = 0; a < asc.size(); ++a)  // ascending-parent values of this GIVEN config
                for (size_t j = 0; j < g.size(); ++j)
                    if (g[j] == net.parents_asc[v][a]) asc[a] = gv[j];
            double acc = 0.0;
            for (int q = 0; q < d; ++q) {
                acc += net.Prob(v, q, asc.data());
                cdf[pc * d + q] = acc;
            }
            for (int j = (int)g.size() - 1; j >= 0; --j) {
                if (++gv[j] < net.dom[g[j]]) break;
                gv[j] = 0;
            }
        }
        // this variable's n draws: the stream positions [k n, (k + 1) n) of the k-th sampled
        // variable, split over threads by jumping ahead
        uint8_t *out = cols + (size_t)v * n;
        ParallelRanges(n, [&](int, int64_t a, int64_t b) {
            Pcg64 r = rng;
            r.advance((uint64_t)a);
            for (int64_t i = a; i < b; ++i) {
                int64_t pc = 0;
                for (int p : g) pc = pc * net.dom[p] + cols[(size_t)p * n + i];
                const double *c = cdf.data() + pc * d;
                const double x = r.random() * c[d - 1];
                int cnt = 0;
                for (int q = 0; q < d; ++q) cnt += x >= c[q];
                out[i] = (uint8_t)std::min(cnt, d - 1);
            }
        });
        rng.advance((uint64_t)n);
    }
    return FBN_OK;
}

int EvidenceCases(const Network &net, int64_t n, int k, uint64_t seed, int query, int8_t *ev) {
    const int V = net.n();
    std::vector<uint8_t> full((size_t)V * n);
    int rc = ForwardSample(net, n, seed, full.data());
    if (rc) return rc;
    std::vector<int> cand;
    for (int v = 0; v < V; ++v)
        if (v != query) cand.push_back(v);
    const int nc = (int)cand.size();
    const Pcg64 rng0(seed + 1);
    const int kk = std::max(0, std::min(k, nc));
    ParallelRanges(n, [&](int, int64_t a, int64_t b) {
        Pcg64 rng = rng0;
        rng.advance((uint64_t)a * (uint64_t)nc);  // row-major draws, as keys[n][nc]
        std::vector<double> keys(nc);
        std::vector<int> idx(nc);
        for (int64_t r = a; r < b; ++r) {
            for (int j = 0; j < nc; ++j) keys[j] = rng.random();
            int8_t *row = ev + (size_t)r * V;
            std::fill(row, row + V, (int8_t)-1);
            if (kk == 0) continue;
            std::iota(idx.begin(), idx.end(), 0);
            // the k smallest keys (a set: argpartition and a full sort pick the same candidates)
            if (kk < nc)
                std::nth_element(idx.begin(), idx.begin() + (kk - 1), idx.end(),
                                 [&](int x, int y) { return keys[x] < keys[y] || (keys[x] == keys[y] && x < y); });
            for (int j = 0; j < kk; ++j) {
                const int v = cand[idx[j]];
                row[v] = (int8_t)full[(size_t)v * n + r];
            }
        }
    });
    return FBN_OK;
}

namespace {
// write `nchunks` text chunks produced in parallel, in order
template <class F>
int WriteChunked(const std::string &path, int64_t nrows, const std::string &header, F render) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return SetError(FBN_ERR_IO, "cannot write %s", path.c_str());
    if (!header.empty() && fwrite(header.data(), 1, header.size(), f) != header.size()) {
        fclose(f);
        return SetError(FBN_ERR_IO, "write failed: %s", path.c_str());
    }
    const int T = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t rows_per = 16384;
    for (int64_t r0 = 0; r0 < nrows; r0 += rows_per * T) {
        std::vector<std::string> bufs(T);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const int64_t a = r0 + t * rows_per, b = std::min(nrows, a + rows_per);
                for (int64_t r = a; r < b; ++r) render(r, bufs[t]);
            });
        for (auto &x : th) x.join();
        for (auto &b : bufs)
            if (!b.empty() && fwrite(b.data(), 1, b.size(), f) != b.size()) {
                fclose(f);
                return SetError(FBN_ERR_IO, "write failed: %s", path.c_str());
            }
    }
    if (fclose(f) != 0) return SetError(FBN_ERR_IO, "write failed: %s", path.c_str());
    return FBN_OK;
}

void AppendInt(std::string &s, int v) {
    char b[16];
    int n = 0;
    if (v < 0) s.push_back('-'), v = -v;
    do b[n++] = (char)('0' + v % 10), v /= 10;
    while (v);
    while (n) s.push_back(b[--n]);
}
}  // namespace

}  // namespace fbn

namespace fbn {
int WriteCsv(const std::string &path, const uint8_t *cols, int nvars, int64_t n, const std::vector<std::string> &names,
             const std::vector<std::vector<std::string>> &values) {
    std::string header;
    for (int v = 0; v < nvars; ++v) {
        if (v) header.push_back(',');
        header += names[v];
    }
    header.push_back('\n');
    return WriteChunked(path, n, header, [&](int64_t r, std::string &s) {
        for (int v = 0; v < nvars; ++v) {
            if (v) s.push_back(',');
            s += values[v][cols[(size_t)v * n + r]];
        }
        s.push_back('\n');
    });
}

int WriteLibsvm(const std::string &path, const int8_t *ev, int64_t n, int V, const int32_t *labels) {
    return WriteChunked(path, n, std::string(), [&](int64_t r, std::string &s) {
        AppendInt(s, labels ? labels[r] : 0);
        const int8_t *row = ev + (size_t)r * V;
        for (int v = 0; v < V; ++v)
            if (row[v] >= 0) {
                s.push_back(' ');
                AppendInt(s, v);
                s.push_back(':');
                AppendInt(s, row[v]);
            }
        s += " \n";
    });
}
}  // namespace fbn

// ------------------------------------------------------------------ C-ABI (include/fastbn.h)
using fbn::SetError;
extern "C" {

int fbn_synth_forward_sample(const fbn_network *net, int64_t n, uint64_t seed, uint8_t *cols) {
    if (!net || n < 0 || (n > 0 && !cols)) return SetError(FBN_ERR_ARG, "bad argument");
    return fbn::ForwardSample(net->net, n, seed, cols);
}

int fbn_synth_evidence(const fbn_network *net, int64_t n, int k, uint64_t seed, int query, int8_t *evidence) {
    if (!net || n < 0 || k < 0 || (n > 0 && !evidence)) return SetError(FBN_ERR_ARG, "bad argument");
    return fbn::EvidenceCases(net->net, n, k, seed, query, evidence);
}

int fbn_write_csv(const char *path, const uint8_t *cols, int nvars, int64_t n, const fbn_network *net) {
    if (!path || nvars <= 0 || n < 0 || (n > 0 && !cols)) return SetError(FBN_ERR_ARG, "bad argument");
    if (net && net->net.n() != nvars) return SetError(FBN_ERR_ARG, "network has %d variables, columns %d", net->net.n(), nvars);
    std::vector<std::string> names(nvars);
    std::vector<std::vector<std::string>> values(nvars);
    for (int v = 0; v < nvars; ++v) {
        names[v] = net ? net->net.names[v] : "X" + std::to_string(v);
        for (int c = 0; c < 256; ++c) values[v].push_back("s" + std::to_string(c));
    }
    return fbn::WriteCsv(path, cols, nvars, n, names, values);
}

int fbn_write_libsvm(const char *path, const int8_t *evidence, int64_t n, int num_nodes, const int32_t *labels) {
    if (!path || num_nodes <= 0 || n < 0 || (n > 0 && !evidence)) return SetError(FBN_ERR_ARG, "bad argument");
    return fbn::WriteLibsvm(path, evidence, n, num_nodes, labels);
}

}  // extern "C"
