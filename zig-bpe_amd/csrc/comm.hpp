// Collectives used by the sharded trainer (one process per GPU). Two implementations:
//   RcclComm  -- RCCL (NCCL API on ROCm) over xGMI, enqueued on the engine stream;
//   HostComm  -- a host callback (e.g. torch.distributed gloo) on staged host copies, used to test
//                the multi-rank logic with several ranks sharing one GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <cstring>
#include <vector>

#include "../../include/zbpe.h"

namespace zbpe {

enum CommOp { COMM_SUM_U32 = 0, COMM_MIN_U32 = 1, COMM_ALLGATHER = 2 };

struct Comm {
    int rank = 0, world = 1;
    virtual ~Comm() {}
    // in place on device memory, stream-ordered
    virtual bool allreduce_u32(uint32_t *d, size_t n, CommOp op, hipStream_t s) = 0;
    // d_out holds world * bytes; this rank's `bytes` come from d_in
    virtual bool allgather(const void *d_in, void *d_out, size_t bytes, hipStream_t s) = 0;
};

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) ncclCommDestroy(comm);
    }
    bool init(int r, int w, const void *uid) {
        rank = r;
        world = w;
        ncclUniqueId id;
        memcpy(&id, uid, sizeof(id));
        return ncclCommInitRank(&comm, w, id, r) == ncclSuccess;
    }
    bool allreduce_u32(uint32_t *d, size_t n, CommOp op, hipStream_t s) override {
        return ncclAllReduce(d, d, n, ncclUint32, op == COMM_MIN_U32 ? ncclMin : ncclSum, comm, s) == ncclSuccess;
    }
    bool allgather(const void *d_in, void *d_out, size_t bytes, hipStream_t s) override {
        return ncclAllGather(d_in, d_out, bytes, ncclUint8, comm, s) == ncclSuccess;
    }
};

struct HostComm : Comm {
    zbpe_collective_fn fn = nullptr;
    void *user = nullptr;
    std::vector<uint8_t> buf;
    bool allreduce_u32(uint32_t *d, size_t n, CommOp op, hipStream_t s) override {
        buf.resize(n * 4);
        if (hipMemcpyAsync(buf.data(), d, n * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        if (fn(user, (int)op, buf.data(), n) != 0) return false;
        if (hipMemcpyAsync(d, buf.data(), n * 4, hipMemcpyHostToDevice, s) != hipSuccess) return false;
        return hipStreamSynchronize(s) == hipSuccess;
    }
    bool allgather(const void *d_in, void *d_out, size_t bytes, hipStream_t s) override {
        buf.assign(bytes * world, 0);
        if (hipMemcpyAsync(buf.data() + bytes * rank, d_in, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        if (fn(user, (int)COMM_ALLGATHER, buf.data(), bytes) != 0) return false;
        if (hipMemcpyAsync(d_out, buf.data(), bytes * world, hipMemcpyHostToDevice, s) != hipSuccess) return false;
        return hipStreamSynchronize(s) == hipSuccess;
    }
};

}  // namespace zbpe
