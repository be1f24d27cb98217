// Time a (possibly hand-edited) specialized JT code object in isolation:
//   gen_bench <hsaco> <ncases> <wave_entries> <lds_bytes> <niv> [grid]
// Inputs are synthetic (no evidence, constant potentials); only the timing is meaningful.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    const long long n = atoll(argv[2]), we = atoll(argv[3]), lds = atoll(argv[4]), niv = atoll(argv[5]);
    int grid = argc > 6 ? atoi(argv[6]) : 1024;
    const long long nblk = (n + 63) / 64;
    if (grid > nblk) grid = (int)nblk;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 3;
    std::vector<char> code;
    fseek(f, 0, SEEK_END);
    code.resize(ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(code.data(), 1, code.size(), f) != code.size()) return 4;
    fclose(f);
    hipModule_t mod;
    hipFunction_t fn;
    CK(hipModuleLoadData(&mod, code.data()));
    CK(hipModuleGetFunction(&fn, mod, "fbn_jt_gen"));
    signed char *ev;
    double *marg, *ws, *iv;
    int *lab, *flags;
    CK(hipMalloc(&ev, n * 64));
    CK(hipMemset(ev, 0xff, n * 64));  // no evidence (all -1) for any V <= 64
    CK(hipMalloc(&marg, n * 8 * 1024));
    CK(hipMalloc(&lab, n * 4));
    CK(hipMalloc(&flags, nblk * 4));
    CK(hipMalloc(&ws, (size_t)grid * we * 64 * 8));
    std::vector<double> h(niv, 0.5);
    CK(hipMalloc(&iv, niv * 8));
    CK(hipMemcpy(iv, h.data(), niv * 8, hipMemcpyHostToDevice));
    unsigned long long *prof = nullptr;
    void *args[] = {&ev, &marg, &lab, &ws, &flags, &iv, (void *)&n, &prof};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
        CK(hipEventRecord(a, 0));
        CK(hipModuleLaunchKernel(fn, grid, 1, 1, 64, 1, 1, (unsigned)lds, 0, args, nullptr));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r > 1 && ms < best) best = ms;
    }
    printf("%s: %.4f ms (best of 8), %.1f Mcases/s\n", argv[1], best, n / best / 1e3);
    return 0;
}
