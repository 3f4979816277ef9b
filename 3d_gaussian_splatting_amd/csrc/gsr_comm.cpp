// gsr_comm.cpp -- RCCL transport of the multi-GPU step (include/gsr/gsr_comm.h).
// Built into libgsr_hip.so with hipcc, so a C++ caller reaches RCCL, like the kernels, through
// the C ABI only (one HIP runtime and one RCCL per process: the executables link libtorch's).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>
#include <string>

#include "gsr/gsr_comm.h"

namespace gsr {
int set_error(int code, const char* msg);  // gsr_api.cpp: the thread-local gsr_last_error text
}

static_assert(GSR_COMM_ID_BYTES == sizeof(ncclUniqueId), "ncclUniqueId size");

struct gsr_comm {
    ncclComm_t comm = nullptr;
    int32_t world = 0, rank = 0;
};

namespace {
thread_local std::string t_msg;
int nccl_err(ncclResult_t r, const char* what) {
    t_msg = std::string(what) + ": " + ncclGetErrorString(r);
    return gsr::set_error(-1, t_msg.c_str());
}
}  // namespace

extern "C" {

int gsr_comm_unique_id(uint8_t id[GSR_COMM_ID_BYTES]) {
    if (!id) return gsr::set_error(-1, "gsr_comm_unique_id: null id");
    ncclUniqueId u;
    if (ncclResult_t r = ncclGetUniqueId(&u)) return nccl_err(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return 0;
}

int gsr_comm_init(gsr_comm** comm, const uint8_t id[GSR_COMM_ID_BYTES], int32_t world, int32_t rank) {
    if (!comm || !id) return gsr::set_error(-1, "gsr_comm_init: null argument");
    if (world < 1 || rank < 0 || rank >= world) return gsr::set_error(-1, "gsr_comm_init: bad rank / world");
    auto* c = new (std::nothrow) gsr_comm;
    if (!c) return gsr::set_error(-1, "gsr_comm_init: out of memory");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    if (ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank)) {
        delete c;
        return nccl_err(r, "ncclCommInitRank");
    }
    c->world = world;
    c->rank = rank;
    *comm = c;
    return 0;
}

int gsr_comm_destroy(gsr_comm* comm) {
    if (!comm) return 0;
    ncclResult_t r = comm->comm ? ncclCommDestroy(comm->comm) : ncclSuccess;
    delete comm;
    return r == ncclSuccess ? 0 : nccl_err(r, "ncclCommDestroy");
}

int gsr_comm_size(gsr_comm* c, int32_t* world, int32_t* rank) {
    if (!c || !c->comm || !world || !rank) return gsr::set_error(-1, "gsr_comm_size: null argument");
    int n = 0, r = 0;
    if (ncclResult_t e = ncclCommCount(c->comm, &n)) return nccl_err(e, "ncclCommCount");
    if (ncclResult_t e = ncclCommUserRank(c->comm, &r)) return nccl_err(e, "ncclCommUserRank");
    *world = n;
    *rank = r;
    return 0;
}

int gsr_comm_all_to_all(gsr_comm* c, const void* send, void* recv, size_t bb, void* stream) {
    if (!c || (!send && bb) || (!recv && bb)) return gsr::set_error(-1, "gsr_comm_all_to_all: null argument");
    const hipStream_t s = (hipStream_t)stream;
    if (ncclResult_t r = ncclGroupStart()) return nccl_err(r, "ncclGroupStart");
    for (int p = 0; p < c->world; ++p) {
        if (ncclResult_t r = ncclSend(static_cast<const char*>(send) + (size_t)p * bb, bb, ncclChar, p, c->comm, s)) {
            (void)ncclGroupEnd();
            return nccl_err(r, "ncclSend");
        }
        if (ncclResult_t r = ncclRecv(static_cast<char*>(recv) + (size_t)p * bb, bb, ncclChar, p, c->comm, s)) {
            (void)ncclGroupEnd();
            return nccl_err(r, "ncclRecv");
        }
    }
    if (ncclResult_t r = ncclGroupEnd()) return nccl_err(r, "ncclGroupEnd");
    return 0;
}

int gsr_comm_all_gather(gsr_comm* c, const void* send, void* recv, size_t bytes, void* stream) {
    if (!c) return gsr::set_error(-1, "gsr_comm_all_gather: null comm");
    if (ncclResult_t r = ncclAllGather(send, recv, bytes, ncclChar, c->comm, (hipStream_t)stream))
        return nccl_err(r, "ncclAllGather");
    return 0;
}

int gsr_comm_all_reduce_i64(gsr_comm* c, int64_t* buf, size_t n, int32_t op, void* stream) {
    if (!c) return gsr::set_error(-1, "gsr_comm_all_reduce_i64: null comm");
    if (ncclResult_t r = ncclAllReduce(buf, buf, n, ncclInt64, op ? ncclMax : ncclSum, c->comm, (hipStream_t)stream))
        return nccl_err(r, "ncclAllReduce");
    return 0;
}

}  // extern "C"
