// gram4_bench.cpp -- diagnostic: the level-0 FP4 MFMA Gram (ci_gram_mfma.hip, through libfastbn.so's
// fbn_ci_onehot4_build / fbn_ci_gram4) in isolation on config-5's shape: 1000 three-state variables
// (2000 leading rows) x 100k samples, 36 upper 256 x 256 tiles, split-K S (argv[1], default 7).
// Prints the mean time of the Gram + reduce pair over 20 launches.
//   g++ -O2 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/micro/gram4_bench.cpp -o tools/micro/gram4_bench \
//       -L fastbn_amd -lfastbn -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../../fastbn_amd'
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

extern "C" hipError_t fbn_ci_onehot4_build(const uint8_t *cols, const int32_t *dims, const int32_t *lead0, long long N,
                                           long long KS, long long Rp, int nvars, uint8_t *O4, hipStream_t s);
extern "C" hipError_t fbn_ci_gram4(const uint8_t *O4, long long Rp, const int2 *tasks, int nt, int S, int KS,
                                   uint16_t *slab, int R, long long ld, int32_t *gram, hipStream_t s);

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main(int argc, char **argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 7;
    const int nv = 1000, R = 2000, Rp = 2048;
    const long long N = 100000, KS = (N + 127) / 128, Kb = KS * 64;
    std::vector<uint8_t> cols((size_t)nv * N);
    std::mt19937 g(7);
    for (auto &c : cols) c = (uint8_t)(g() % 3);
    std::vector<int32_t> dims(nv, 3), lead0(nv);
    for (int v = 0; v < nv; ++v) lead0[v] = 2 * v;
    std::vector<int32_t> tasks;
    for (int I = 0; I < Rp / 256; ++I)
        for (int J = I; J < Rp / 256; ++J) tasks.push_back(I), tasks.push_back(J);
    const int nt = (int)tasks.size() / 2;
    uint8_t *dcols, *O4;
    int32_t *ddims, *dlead, *dtasks, *gram;
    uint16_t *slab;
    CK(hipMalloc(&dcols, cols.size()));
    CK(hipMalloc(&O4, (size_t)Rp * Kb));
    CK(hipMalloc(&ddims, nv * 4));
    CK(hipMalloc(&dlead, nv * 4));
    CK(hipMalloc(&dtasks, tasks.size() * 4));
    CK(hipMalloc(&gram, (size_t)R * R * 4));
    CK(hipMalloc(&slab, (size_t)nt * S * 65536 * 2));
    CK(hipMemcpy(dcols, cols.data(), cols.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(ddims, dims.data(), nv * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlead, lead0.data(), nv * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtasks, tasks.data(), tasks.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(O4, 0, (size_t)Rp * Kb));
    CK(fbn_ci_onehot4_build(dcols, ddims, dlead, N, KS, Rp, nv, O4, 0));
    CK(fbn_ci_gram4(O4, Rp, (const int2 *)dtasks, nt, S, (int)KS, slab, R, R, gram, 0));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < 20; ++r) CK(fbn_ci_gram4(O4, Rp, (const int2 *)dtasks, nt, S, (int)KS, slab, R, R, gram, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // spot check: G[0][2] = #samples with v0 == 0 and v1 == 0
    int32_t g02 = 0;
    CK(hipMemcpy(&g02, gram + 2, 4, hipMemcpyDeviceToHost));
    long long ref = 0;
    for (long long s = 0; s < N; ++s) ref += cols[s] == 0 && cols[N + s] == 0;
    printf("S %d tiles %d: gram+reduce %.1f us per call  G[0][2] %d (ref %lld)\n", S, nt, 1e3 * ms / 20, g02, ref);
    return g02 == ref ? 0 : 2;
}
