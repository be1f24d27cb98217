// ThreadSanitizer driver for the multi-threaded host code of libfastbn (SURVEY §5 race detection:
// the reference's OpenMP loops race on shared counters / maps; ours must not).  Built by
// tests/test_host.py::test_host_threads_under_tsan with g++ -fsanitize=thread from io.cpp and
// synth.cpp directly (no HIP): threaded forward sampling and evidence generation, the chunked
// parallel CSV / LIBSVM writers, and the block-parallel CSV / LIBSVM parsers, round-tripped.
// usage: host_tsan <network.xml> <scratch dir>
#include <cstdio>
#include <string>
#include <vector>

#include "../../fastbn_amd/csrc/fbn_internal.h"

#define CHECK(c)                                                 \
    do {                                                         \
        if (!(c)) {                                              \
            std::fprintf(stderr, "check failed: %s:%d %s\n", __FILE__, __LINE__, #c); \
            return 1;                                            \
        }                                                        \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    fbn_network net;
    CHECK(fbn::LoadXmlbif(argv[1], net.net) == 0);
    const int V = net.net.n();
    const int64_t n = 150000;  // several parser blocks' worth of rows per thread
    std::vector<uint8_t> cols((size_t)V * n);
    CHECK(fbn::ForwardSample(net.net, n, 7, cols.data()) == 0);
    const std::string csv = std::string(argv[2]) + "/tsan.csv", svm = std::string(argv[2]) + "/tsan.libsvm";
    CHECK(fbn_write_csv(csv.c_str(), cols.data(), V, n, &net) == 0);
    fbn::Dataset ds;
    CHECK(fbn::LoadCsv(csv, ds) == 0);
    CHECK(ds.nvars == V && ds.nsamples == n);
    // state names "s<c>": the parser numbers states in order of first appearance, so compare the
    // columns up to that relabelling
    for (int v = 0; v < V; ++v) {
        std::vector<int> map(256, -1);
        for (int64_t r = 0; r < n; ++r) {
            int &m = map[cols[(size_t)v * n + r]];
            if (m < 0) m = ds.cols[(size_t)v * n + r];
            CHECK(m == ds.cols[(size_t)v * n + r]);
        }
    }
    std::vector<int8_t> ev((size_t)V * n), back((size_t)V * n);
    std::vector<int32_t> lab(n), lab2(n);
    CHECK(fbn::EvidenceCases(net.net, n, 5, 11, -1, ev.data()) == 0);
    for (int64_t r = 0; r < n; ++r) lab[r] = (int32_t)(r % 3);
    CHECK(fbn_write_libsvm(svm.c_str(), ev.data(), n, V, lab.data()) == 0);
    int64_t rows = 0;
    CHECK(fbn::LoadLibsvm(svm, V, back.data(), lab2.data(), n, &rows) == 0);
    CHECK(rows == n && back == ev && lab2 == lab);
    std::printf("host_tsan ok: %d variables, %lld rows\n", V, (long long)n);
    return 0;
}
