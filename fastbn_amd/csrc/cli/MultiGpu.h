// MultiGpu.h -- the drop-in CLI's multi-GPU layer: one host thread per GPU of this
// node, one RCCL communicator per GPU (ncclCommInitAll, single process), collectives on each
// rank's own HIP stream over xGMI.  The reference runs one process with OpenMP threads
// (src/main.cpp:31-82); `--gpus N` keeps that process model and drives N devices from it.
//
//   JT (-a 2):  the cases are cut into N contiguous shards; each rank builds its plan on its device
//               from the parsed network, runs its shard from device memory and forms every case's
//               MSE / HD terms there (fbn_jt_score_terms_device, against its golden slice uploaded
//               once); all-gathers (RCCL) of the labels and of the 16-byte per-case terms let rank 0
//               add them in the reference's case order (src/Inference.cpp:153-206) -- the marginals
//               never leave their device.
//   PC (-a 0):  rank 0 uploads the column store, ONE broadcast (RCCL) places it in every rank's
//               device memory, and the native session fbn_pc_dist_* cuts each level by edges; per
//               level one all-gather of the fixed-size records (and at level 0 of the pair tables,
//               device to device) -- INTEGRATION.md "Multi-GPU".
#ifndef FBN_CLI_MULTIGPU_H
#define FBN_CLI_MULTIGPU_H

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <functional>
#include <string>
#include <vector>

class GpuGroup {
public:
    // ranks 0..n-1 on devices first_device .. first_device + n - 1
    GpuGroup(int n, int first_device);
    ~GpuGroup();
    bool ok() const { return err_.empty(); }
    const std::string &error() const { return err_; }
    int size() const { return (int)comms_.size(); }
    int device(int rank) const { return first_ + rank; }
    ncclComm_t comm(int rank) const { return comms_[rank]; }
    hipStream_t stream(int rank) const { return streams_[rank]; }
    // fn(rank) on one host thread per rank (device already selected); returns 0 or the first error
    // message of any rank (every rank runs to completion or to its own error)
    std::string Run(const std::function<std::string(int rank)> &fn);

private:
    int first_ = 0;
    std::vector<ncclComm_t> comms_;
    std::vector<hipStream_t> streams_;
    std::string err_;
    bool aborted_ = false;
};

// error text of an RCCL / HIP call, empty on success
std::string NcclErr(ncclResult_t r, const char *what);
std::string HipErr(hipError_t e, const char *what);

// FBN_PC_DIST_FORCE_EXCHANGE=1: take the RCCL path (and every collective of it) even with one GPU,
// so a one-GPU machine executes the multi-GPU data paths (testing / rehearsal)
bool ForceExchange();

#endif
