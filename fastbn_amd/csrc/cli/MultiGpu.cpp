// MultiGpu.cpp -- see MultiGpu.h
#include "MultiGpu.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

std::string NcclErr(ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return std::string();
    return std::string(what) + ": " + ncclGetErrorString(r);
}

std::string HipErr(hipError_t e, const char *what) {
    if (e == hipSuccess) return std::string();
    return std::string(what) + ": " + hipGetErrorString(e);
}

bool ForceExchange() {
    const char *v = getenv("FBN_PC_DIST_FORCE_EXCHANGE");
    return v && *v && strcmp(v, "0") != 0;
}

GpuGroup::GpuGroup(int n, int first_device) : first_(first_device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || n < 1 || first_device < 0 || first_device + n > count) {
        err_ = "--gpus " + std::to_string(n) + " from device " + std::to_string(first_device) + ": " +
               std::to_string(count) + " HIP device(s) visible";
        return;
    }
    std::vector<int> devs(n);
    for (int r = 0; r < n; ++r) devs[r] = first_device + r;
    comms_.assign(n, nullptr);
    if ((err_ = NcclErr(ncclCommInitAll(comms_.data(), n, devs.data()), "ncclCommInitAll")).size()) {
        comms_.clear();
        return;
    }
    streams_.assign(n, nullptr);
    for (int r = 0; r < n; ++r) {
        if ((err_ = HipErr(hipSetDevice(devs[r]), "hipSetDevice")).size()) return;
        if ((err_ = HipErr(hipStreamCreateWithFlags(&streams_[r], hipStreamNonBlocking), "hipStreamCreate")).size())
            return;
    }
}

GpuGroup::~GpuGroup() {
    for (size_t r = 0; r < streams_.size(); ++r)
        if (streams_[r]) {
            (void)hipSetDevice(first_ + (int)r);
            (void)hipStreamDestroy(streams_[r]);
        }
    if (!aborted_)
        for (auto c : comms_)
            if (c) (void)ncclCommDestroy(c);
}

std::string GpuGroup::Run(const std::function<std::string(int)> &fn) {
    std::mutex mu;
    std::string first_err;
    std::vector<std::thread> th;
    for (int r = 0; r < size(); ++r)
        th.emplace_back([&, r] {
            std::string e = HipErr(hipSetDevice(device(r)), "hipSetDevice");
            if (e.empty()) e = fn(r);
            if (!e.empty()) {
                std::lock_guard<std::mutex> g(mu);
                if (first_err.empty()) {
                    first_err = "rank " + std::to_string(r) + ": " + e;
                    // the other ranks may be waiting in a collective this rank will never join:
                    // abort every communicator so their in-flight collectives return
                    for (auto c : comms_)
                        if (c) (void)ncclCommAbort(c);
                    aborted_ = true;
                }
            }
        });
    for (auto &t : th) t.join();
    return first_err;
}
