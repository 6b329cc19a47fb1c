// lio_icp_group.cpp — single-process multi-GPU loop ICP: the
// form a C++ host uses, e.g. fast_lio_sam's loop-closure thread
// (fast_lio_sam/src/main.cpp:10 AsyncSpinner, fast_lio_sam.cpp:698 ->
// loop_closure.cpp:69-92 icpAlignment).
//
// n_gpus lio_icp handles, one per device, the source sharded over them in
// whole 4096-point records (lio_icp_set_shard); the target is replicated.  A
// group alignment runs every rank's lio_icp_align on its own host thread; per
// ICP iteration each rank publishes its records' Umeyama statistics and the
// group all-gathers them:
//   * RCCL (default when the devices are distinct): one communicator per
//     device from ncclCommInitAll; each handle's statistics kernel writes its
//     records into a device buffer, ncclAllGather moves them over xGMI on the
//     handle's own stream and a one-block kernel sums them in record order
//     behind it (lio_icp_set_shard_device: no host copies, one host wait per
//     pass).  librccl is opened at group creation, not linked: the library
//     loads without it and reuses a copy already in the process;
//   * host (LIO_ICP_EXCHANGE=host, or several ranks on one device): the
//     ranks' threads swap the records through shared memory behind a barrier.
// Every rank then sums all records in record order (lio_icp_combine), so every
// rank — and every n_gpus — computes the bit-identical transform.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lio_gpu.h"
#include "lio_error.hpp"
#include "lio_rccl.hpp"

namespace {

int gfail(int code, const std::string& msg) {
    lio::last_error() = msg;
    return code;
}

using lio::kNcclDouble;
using lio::ncclComm_t;
using lio::ncclResult_t;
using lio::Rccl;

}  // namespace

struct lio_icp_group;

struct IcpRank {
    lio_icp_group* g = nullptr;
    int rank = 0;
};

struct lio_icp_group {
    int world = 0;
    bool use_rccl = false;
    std::vector<int> dev;
    std::vector<lio_icp*> h;
    std::vector<IcpRank> rk;
    Rccl rccl;
    std::vector<ncclComm_t> comms;
    int64_t ns = 0;
    // host exchange: generation-counted barrier; `failed` releases every waiter
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool failed = false;
    bool aborted = false;  // communicators aborted (and freed) once; destroy skips them
    std::vector<const double*> slots;
};

namespace {

// false when the group failed while waiting (the caller returns an error)
bool host_barrier(lio_icp_group* g) {
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->failed) return false;
    const uint64_t my = g->gen;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return true;
    }
    g->cv.wait(lk, [&] { return g->gen != my || g->failed; });
    return !g->failed;
}

// Every rank that fails calls this; the communicators are aborted exactly once (ncclCommAbort frees
// them: a second abort, or ncclCommDestroy afterwards, would be a use after free), under the lock.
void fail_group(lio_icp_group* g) {
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->failed = true;
        if (g->use_rccl && !g->aborted) {
            g->aborted = true;
            // ranks waiting on an all-gather's stream return once their communicators abort
            for (ncclComm_t c : g->comms)
                if (c) (void)g->rccl.CommAbort(c);
            g->comms.clear();  // destroy sees no communicator
        }
    }
    g->cv.notify_all();
}

// host exchange (LIO_ICP_EXCHANGE=host, or ranks sharing a device): lio_allgather_fn of rank r,
// `n` doubles from every rank in rank order, through shared host memory behind a barrier
int group_allgather(const double* send, int64_t n, double* recv, void* user) {
    IcpRank* r = static_cast<IcpRank*>(user);
    lio_icp_group* g = r->g;
    g->slots[r->rank] = send;
    if (!host_barrier(g)) return -1;  // every rank's send is published
    for (int k = 0; k < g->world; ++k) std::memcpy(recv + (size_t)k * n, g->slots[k], (size_t)n * sizeof(double));
    return host_barrier(g) ? 0 : -1;  // every rank has copied before the sends change
}

// RCCL exchange: lio_allgather_dev_fn of rank r — the handle's device send buffer all-gathered into its
// device recv buffer on the handle's own stream (enqueued only; the handle sums the records behind it
// and waits once per pass).  The enqueue runs under the lock fail_group aborts under, so it never
// touches a communicator an abort has freed.
int group_allgather_dev(const double* d_send, int64_t n, double* d_recv, void* stream, void* user) {
    IcpRank* r = static_cast<IcpRank*>(user);
    lio_icp_group* g = r->g;
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->failed || g->comms.empty()) return -1;  // another rank failed: its abort freed the comms
    return g->rccl.AllGather(d_send, d_recv, (size_t)n, kNcclDouble, g->comms[r->rank], (hipStream_t)stream) == 0 ? 0
                                                                                                                 : -1;
}

// One all-gather on every communicator from this thread, inside a group call: the connections RCCL
// sets up lazily at a communicator's first collective (a step that waits for every peer) exist before
// the ranks' threads enqueue theirs one at a time under the group lock.
int rccl_warmup(lio_icp_group* g) {
    const int n = g->world;
    std::vector<double*> buf(n, nullptr);
    int rc = LIO_OK;
    for (int r = 0; r < n && rc == LIO_OK; ++r) {
        if (hipSetDevice(g->dev[r]) != hipSuccess || hipMalloc(&buf[r], (size_t)(n + 1) * sizeof(double)) != hipSuccess)
            rc = gfail(LIO_ERR_NOMEM, "lio_icp_group_create: warm-up buffers");
        else if (hipMemset(buf[r], 0, (size_t)(n + 1) * sizeof(double)) != hipSuccess)
            rc = gfail(LIO_ERR_HIP, "lio_icp_group_create: warm-up buffers");
    }
    if (rc == LIO_OK) {
        ncclResult_t nr = g->rccl.GroupStart();
        for (int r = 0; r < n && nr == 0; ++r)
            nr = g->rccl.AllGather(buf[r] + n, buf[r], 1, kNcclDouble, g->comms[r], nullptr);
        const ncclResult_t ne = g->rccl.GroupEnd();
        if (nr == 0) nr = ne;
        if (nr != 0) rc = gfail(LIO_ERR_STATE, std::string("RCCL warm-up all-gather: ") + g->rccl.GetErrorString(nr));
    }
    for (int r = 0; r < n; ++r) {
        if (!buf[r]) continue;
        (void)hipSetDevice(g->dev[r]);
        if (hipDeviceSynchronize() != hipSuccess && rc == LIO_OK) rc = gfail(LIO_ERR_HIP, "RCCL warm-up: device error");
        (void)hipFree(buf[r]);
    }
    return rc;
}

}  // namespace

extern "C" {

int lio_icp_group_create(const lio_icp_params* p, int n_gpus, const int* devices, lio_icp_group** out) {
    if (!p || !out || n_gpus < 1 || n_gpus > 64) return gfail(LIO_ERR_ARG, "lio_icp_group_create: bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return gfail(LIO_ERR_NODEV, "lio_icp_group_create: no HIP device (no CPU path)");
    auto* g = new lio_icp_group();
    g->world = n_gpus;
    g->dev.resize(n_gpus);
    bool distinct = true;
    for (int r = 0; r < n_gpus; ++r) {
        g->dev[r] = devices ? devices[r] : r;
        for (int q = 0; q < r; ++q) distinct = distinct && g->dev[q] != g->dev[r];
    }
    const char* ex = std::getenv("LIO_ICP_EXCHANGE");
    g->use_rccl = n_gpus > 1 && distinct && !(ex && std::string(ex) == "host");
    g->h.assign(n_gpus, nullptr);
    g->rk.resize(n_gpus);
    g->slots.assign(n_gpus, nullptr);
    int rc = LIO_OK;
    for (int r = 0; r < n_gpus && rc == LIO_OK; ++r) {
        lio_icp_params pr = *p;
        pr.device = g->dev[r];
        rc = lio_icp_create(&pr, &g->h[r]);
        g->rk[r].g = g;
        g->rk[r].rank = r;
        if (rc == LIO_OK && n_gpus > 1)
            rc = g->use_rccl ? lio_icp_set_shard_device(g->h[r], r, n_gpus, group_allgather_dev, &g->rk[r])
                             : lio_icp_set_shard(g->h[r], r, n_gpus, group_allgather, &g->rk[r]);
    }
    if (rc == LIO_OK && g->use_rccl) {
        std::string why;
        if (!lio::load_rccl(g->rccl, why)) {
            rc = gfail(LIO_ERR_STATE, "lio_icp_group_create: " + why);
        } else {
            g->comms.assign(n_gpus, nullptr);
            const ncclResult_t nr = g->rccl.CommInitAll(g->comms.data(), n_gpus, g->dev.data());
            if (nr != 0) {
                g->comms.clear();
                rc = gfail(LIO_ERR_STATE, std::string("ncclCommInitAll: ") + g->rccl.GetErrorString(nr));
            } else {
                rc = rccl_warmup(g);
            }
        }
    }
    if (rc != LIO_OK) {
        lio_icp_group_destroy(g);
        return rc;
    }
    *out = g;
    return LIO_OK;
}

int lio_icp_group_destroy(lio_icp_group* g) {
    if (!g) return LIO_OK;
    for (lio_icp* h : g->h) lio_icp_destroy(h);  // drains each handle's stream first
    for (ncclComm_t c : g->comms)
        if (c) (void)g->rccl.CommDestroy(c);
    delete g;  // librccl stays loaded (other users in the process may share it)
    return LIO_OK;
}

int lio_icp_group_size(const lio_icp_group* g) { return g ? g->world : 0; }
int lio_icp_group_uses_rccl(const lio_icp_group* g) { return g && g->use_rccl ? 1 : 0; }

int lio_icp_group_set_target(lio_icp_group* g, const float* xyz, int64_t n) {
    if (!g) return gfail(LIO_ERR_ARG, "lio_icp_group_set_target: NULL group");
    for (lio_icp* h : g->h) {  // replicated on every device
        const int rc = lio_icp_set_target(h, xyz, n);
        if (rc) return rc;
    }
    return LIO_OK;
}

int lio_icp_group_set_source(lio_icp_group* g, const float* xyz, int64_t n) {
    if (!g) return gfail(LIO_ERR_ARG, "lio_icp_group_set_source: NULL group");
    for (lio_icp* h : g->h) {  // each handle keeps the full source on the host and uploads its shard
        const int rc = lio_icp_set_source(h, xyz, n);
        if (rc) return rc;
    }
    g->ns = n;
    return LIO_OK;
}

int lio_icp_group_align(lio_icp_group* g, const float* guess16, lio_icp_result* out, float* aligned_opt) {
    if (!g || !out) return gfail(LIO_ERR_ARG, "lio_icp_group_align: bad arguments");
    if (g->world == 1) return lio_icp_align(g->h[0], guess16, out, aligned_opt);
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->failed) return gfail(LIO_ERR_STATE, "lio_icp_group_align: the group failed earlier (recreate it)");
        g->arrived = 0;
    }
    std::vector<lio_icp_result> res(g->world);
    std::vector<int> rcs(g->world, LIO_OK);
    std::vector<std::string> errs(g->world);
    std::vector<std::thread> th;
    for (int r = 0; r < g->world; ++r)
        th.emplace_back([&, r] {
            int64_t b = 0, cnt = 0;
            lio_icp_shard_range(g->ns, r, g->world, &b, &cnt);
            rcs[r] = lio_icp_align(g->h[r], guess16, &res[r], aligned_opt ? aligned_opt + 3 * b : nullptr);
            if (rcs[r] != LIO_OK) {
                errs[r] = lio::last_error();
                fail_group(g);
            }
        });
    for (std::thread& t : th) t.join();
    for (int r = 0; r < g->world; ++r)
        if (rcs[r] != LIO_OK) return gfail(rcs[r], "lio_icp_group_align: rank " + std::to_string(r) + ": " + errs[r]);
    for (int r = 1; r < g->world; ++r)  // every rank summed the same records in the same order
        if (std::memcmp(res[r].T, res[0].T, sizeof(res[0].T)) != 0 || res[r].iterations != res[0].iterations)
            return gfail(LIO_ERR_STATE, "lio_icp_group_align: ranks disagree (not bit-identical)");
    *out = res[0];
    return LIO_OK;
}

}  // extern "C"
