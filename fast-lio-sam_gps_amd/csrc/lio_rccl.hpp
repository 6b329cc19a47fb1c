// lio_rccl.hpp — the few RCCL entry points the loop ICP uses, resolved from librccl at run time (rccl.h
// ABI; the library loads without RCCL and reuses a copy already in the process).
#pragma once
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

namespace lio {

typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;  // ncclSuccess = 0
struct ncclUniqueId {
    char internal[128];  // NCCL_UNIQUE_ID_BYTES
};
constexpr int kNcclDouble = 8;  // ncclFloat64

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

inline bool load_rccl(Rccl& r, std::string& why) {
    const char* env = std::getenv("LIO_RCCL_LIB");
    const char* names[] = {env, "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
        if (!n) continue;
        r.so = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (r.so) break;
    }
    if (!r.so) {
        why = "librccl not found (set LIO_RCCL_LIB or LIO_ICP_EXCHANGE=host)";
        return false;
    }
    r.CommInitAll = (decltype(r.CommInitAll))dlsym(r.so, "ncclCommInitAll");
    r.CommInitRank = (decltype(r.CommInitRank))dlsym(r.so, "ncclCommInitRank");
    r.GetUniqueId = (decltype(r.GetUniqueId))dlsym(r.so, "ncclGetUniqueId");
    r.CommDestroy = (decltype(r.CommDestroy))dlsym(r.so, "ncclCommDestroy");
    r.CommAbort = (decltype(r.CommAbort))dlsym(r.so, "ncclCommAbort");
    r.AllGather = (decltype(r.AllGather))dlsym(r.so, "ncclAllGather");
    r.GroupStart = (decltype(r.GroupStart))dlsym(r.so, "ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))dlsym(r.so, "ncclGroupEnd");
    r.GetErrorString = (decltype(r.GetErrorString))dlsym(r.so, "ncclGetErrorString");
    if (!r.CommInitAll || !r.CommInitRank || !r.GetUniqueId || !r.CommDestroy || !r.CommAbort || !r.AllGather ||
        !r.GroupStart || !r.GroupEnd || !r.GetErrorString) {
        why = "librccl lacks the communicator / all-gather entry points";
        return false;
    }
    return true;
}

}  // namespace lio
