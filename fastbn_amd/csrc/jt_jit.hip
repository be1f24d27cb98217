// jt_jit.hip -- compile + cache + load of plan-specialized kernels (jt_codegen.cpp output).
//
// Code objects are cached on disk under a key = FNV-1a-64 of (source, options): $FBN_KERNEL_CACHE,
// else <directory of libfastbn.so>/kcache (in-tree, so kernels prebuilt by __graft_entry__.build()
// travel with the repository).  A miss compiles with hiprtc, resolved at run time with dlopen so
// that a process which already carries a hiprtc (e.g. PyTorch's) reuses that one.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "fbn_internal.h"

namespace fbn {

extern const char *kJitOptions[];
const char *kJitOptions[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"};
extern const int kJitNumOptions = 4;

namespace {

struct Rtc {
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) log = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) code = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    bool ok = false;
};

Rtc &GetRtc() {
    static Rtc r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("libhiprtc.so.7", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/libhiprtc.so.7", RTLD_NOW);
        if (!h) return;
        r.create = (decltype(r.create))dlsym(h, "hiprtcCreateProgram");
        r.compile = (decltype(r.compile))dlsym(h, "hiprtcCompileProgram");
        r.log_size = (decltype(r.log_size))dlsym(h, "hiprtcGetProgramLogSize");
        r.log = (decltype(r.log))dlsym(h, "hiprtcGetProgramLog");
        r.code_size = (decltype(r.code_size))dlsym(h, "hiprtcGetCodeSize");
        r.code = (decltype(r.code))dlsym(h, "hiprtcGetCode");
        r.destroy = (decltype(r.destroy))dlsym(h, "hiprtcDestroyProgram");
        r.ok = r.create && r.compile && r.log_size && r.log && r.code_size && r.code && r.destroy;
    });
    return r;
}

uint64_t Fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

std::string CacheDir() {
    if (const char *e = getenv("FBN_KERNEL_CACHE")) return e;
    Dl_info info;
    if (dladdr((void *)&CacheDir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t k = p.rfind('/');
        return (k == std::string::npos ? std::string(".") : p.substr(0, k)) + "/kcache";
    }
    return "kcache";
}

bool ReadFile(const std::string &path, std::vector<char> &out) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    bool good = n > 0 && fread(out.data(), 1, out.size(), f) == out.size();
    fclose(f);
    return good;
}

void WriteFileAtomic(const std::string &dir, const std::string &path, const std::vector<char> &data) {
    mkdir(dir.c_str(), 0755);
    std::string tmp = path + ".tmp." + std::to_string((long)getpid());
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;  // read-only location: the cache is an optimization only
    bool good = fwrite(data.data(), 1, data.size(), f) == data.size();
    good = (fclose(f) == 0) && good;
    if (good) rename(tmp.c_str(), path.c_str());
    else unlink(tmp.c_str());
}

}  // namespace

std::string JitCacheKey(const std::string &src) {
    std::string opts;
    for (int i = 0; i < kJitNumOptions; ++i) opts += std::string(kJitOptions[i]) + "\n";
    char b[32];
    snprintf(b, sizeof b, "%016llx", (unsigned long long)Fnv1a(src, Fnv1a(opts)));
    return b;
}

std::string JitCachePath(const std::string &src) { return CacheDir() + "/fbn_jt_" + JitCacheKey(src) + ".hsaco"; }

// code object for `src` (cache hit or hiprtc compile); FBN_OK or an error with the compile log
int JitCodeObject(const std::string &src, std::vector<char> &code) {
    const std::string path = JitCachePath(src);
    if (ReadFile(path, code)) return FBN_OK;
    Rtc &r = GetRtc();
    if (!r.ok) return SetError(FBN_ERR_HIP, "specialized kernel: %s not cached and libhiprtc unavailable", path.c_str());
    hiprtcProgram prog;
    if (r.create(&prog, src.c_str(), "fbn_jt_gen.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        return SetError(FBN_ERR_HIP, "hiprtcCreateProgram failed");
    hiprtcResult cr = r.compile(prog, kJitNumOptions, kJitOptions);
    if (cr != HIPRTC_SUCCESS) {
        size_t n = 0;
        r.log_size(prog, &n);
        std::string log(n, '\0');
        if (n) r.log(prog, &log[0]);
        r.destroy(&prog);
        if (log.size() > 2000) log.resize(2000);
        return SetError(FBN_ERR_HIP, "hiprtc compile of the specialized kernel failed: %s", log.c_str());
    }
    size_t n = 0;
    r.code_size(prog, &n);
    code.resize(n);
    r.code(prog, code.data());
    r.destroy(&prog);
    std::string dir = path.substr(0, path.rfind('/'));
    WriteFileAtomic(dir, path, code);
    return FBN_OK;
}

}  // namespace fbn
