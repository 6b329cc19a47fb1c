// lio_icp_mp.cpp — the multi-process loop-ICP exchanges, with no Python in the per-pass loop.
//
// One process per GPU shards the source in 4096-point records (lio_icp_set_shard*); per ICP pass every rank
// all-gathers every rank's records and sums them in record order, so every rank computes the transform of
// one GPU bit for bit.  The reference's loop closure is one C++ node (fast_lio_sam/src/main.cpp:10,
// fast_lio_sam.cpp:698 -> loop_closure.cpp:69-92); the exchanges here are C++ end to end:
//
//   * RCCL (one communicator per rank, ncclCommInitRank from a ncclUniqueId that the caller broadcasts once,
//     e.g. through torch.distributed): the statistics kernel writes the rank's records into a device send
//     buffer, ncclAllGather is enqueued from C++ on the ICP handle's own stream, the record-order sum runs
//     behind it on the device — one host wait per pass (lio_icp_set_shard_rccl);
//   * shared memory (several ranks on ONE node without RCCL — RCCL refuses two ranks on one device — the
//     one-GPU rehearsal): a POSIX shm segment with two record buffers per rank (alternating by pass) and a
//     generation barrier; each rank copies its host-mapped records in, waits once, sums every rank's
//     records in order (lio_icp_set_shard_shm; the primitive is lio_shm_exchange_*).
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <string>

#include "../../include/lio_gpu.h"
#include "lio_error.hpp"
#include "lio_rccl.hpp"

extern "C" void lio_icp_set_exchange_owner(lio_icp* h, void* owner, void (*free_fn)(void*));
extern "C" int lio_icp_device(const lio_icp* h);

namespace {

int mfail(int code, const std::string& msg) {
    lio::last_error() = msg;
    return code;
}

// ------------------------------------------------------------------ shared-memory all-gather
constexpr uint32_t kShmMagic = 0x4c494f58u;  // rank 0 has written world / n

struct ShmHdr {
    std::atomic<uint64_t> arrive;
    std::atomic<uint64_t> gen;
    std::atomic<int> attached;
    std::atomic<int> poisoned;   // a barrier timed out: the arrival count can no longer be trusted
    std::atomic<uint32_t> magic;
    int world;
    int64_t n;
    char pad[256 - 2 * sizeof(std::atomic<uint64_t>) - 2 * sizeof(std::atomic<int>) - sizeof(std::atomic<uint32_t>) -
             sizeof(int) - sizeof(int64_t) - 4];
};
static_assert(sizeof(ShmHdr) == 256, "shm header layout");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "shared-memory atomics must be lock-free");

struct ShmEx {
    std::string name;
    int rank = 0, world = 1;
    int64_t n = 0;  // doubles per rank
    size_t bytes = 0;
    ShmHdr* hdr = nullptr;
    double* data = nullptr;  // 2 x world x n
    uint64_t round = 0;
    ino_t ino = 0;           // the segment's inode: a name is only unlinked while it still names THIS segment
    double timeout_s = 60.0;
};

// unlink `name` if it still refers to the segment with inode `ino` (a later open of the same name may have
// replaced it: that segment belongs to someone else)
void unlink_if_ours(const std::string& name, ino_t ino) {
    const int fd = shm_open(name.c_str(), O_RDONLY, 0600);
    if (fd < 0) return;
    struct stat sb;
    const bool ours = fstat(fd, &sb) == 0 && sb.st_ino == ino;
    close(fd);
    if (ours) shm_unlink(name.c_str());
}

void shm_close(ShmEx* e) {
    if (!e) return;
    // the name was unlinked when the last rank attached; a segment some rank never attached to is removed by
    // rank 0 here, and only while the name still refers to it
    if (e->hdr && e->rank == 0 && e->hdr->attached.load(std::memory_order_acquire) < e->world)
        unlink_if_ours(e->name, e->ino);
    if (e->hdr) munmap(e->hdr, e->bytes);
    delete e;
}

// rank 0 creates the segment (a stale one of the same name is removed first); the other ranks open it
// after rank 0 has (the caller orders the opens, e.g. a process-group barrier), retrying for a few seconds,
// and check that it was made for the same world size and at least their message size.  The rank whose
// attach completes the world unlinks the name at once, so no later close can remove a newer segment that
// reuses it.
int shm_open_ex(const char* name, int rank, int world, int64_t n, ShmEx** out) {
    if (!name || name[0] != '/' || rank < 0 || rank >= world || n < 1) return mfail(LIO_ERR_ARG, "lio_shm_exchange_open: bad arguments");
    auto* e = new ShmEx();
    e->name = name;
    e->rank = rank;
    e->world = world;
    e->n = n;
    e->bytes = sizeof(ShmHdr) + 2 * (size_t)world * (size_t)n * sizeof(double);
    int fd = -1;
    if (rank == 0) {
        shm_unlink(name);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0 && ftruncate(fd, (off_t)e->bytes) != 0) {
            close(fd);
            fd = -1;
        }
    } else {
        for (int t = 0; t < 500 && fd < 0; ++t) {  // <= 5 s for rank 0's segment to appear with its size
            fd = shm_open(name, O_RDWR, 0600);
            struct stat sb;
            if (fd >= 0 && (fstat(fd, &sb) != 0 || (size_t)sb.st_size < e->bytes)) {
                close(fd);
                fd = -1;
            }
            if (fd < 0) usleep(10000);
        }
    }
    if (fd < 0) {
        const std::string nm = name;
        delete e;
        return mfail(LIO_ERR_STATE, "lio_shm_exchange_open: cannot open shared memory " + nm);
    }
    struct stat sb;
    if (fstat(fd, &sb) == 0) e->ino = sb.st_ino;
    void* p = mmap(nullptr, e->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete e;
        return mfail(LIO_ERR_NOMEM, "lio_shm_exchange_open: mmap failed");
    }
    e->hdr = static_cast<ShmHdr*>(p);
    e->data = reinterpret_cast<double*>(static_cast<char*>(p) + sizeof(ShmHdr));
    if (rank == 0) {
        e->hdr->world = world;
        e->hdr->n = n;
        e->hdr->magic.store(kShmMagic, std::memory_order_release);
    } else {
        for (int t = 0; t < 500 && e->hdr->magic.load(std::memory_order_acquire) != kShmMagic; ++t) usleep(10000);
        if (e->hdr->magic.load(std::memory_order_acquire) != kShmMagic || e->hdr->world != world || e->hdr->n < n) {
            const std::string msg = "lio_shm_exchange_open: segment " + e->name + " was made for another world size or "
                                    "a smaller message (world " + std::to_string(e->hdr->world) + ", n " +
                                    std::to_string(e->hdr->n) + ")";
            munmap(e->hdr, e->bytes);
            delete e;
            return mfail(LIO_ERR_STATE, msg);
        }
    }
    if (e->hdr->attached.fetch_add(1, std::memory_order_acq_rel) + 1 == world) unlink_if_ours(e->name, e->ino);
    *out = e;
    return LIO_OK;
}

// generation barrier over the ranks of the segment; false after the timeout (a rank died) — and then the
// segment is poisoned for every rank: this rank's arrival stays counted, so a later barrier could release
// before every rank has written its records
bool shm_barrier(ShmEx* e) {
    ShmHdr* h = e->hdr;
    if (h->poisoned.load(std::memory_order_acquire)) return false;
    const uint64_t g = h->gen.load(std::memory_order_acquire);
    if (h->arrive.fetch_add(1, std::memory_order_acq_rel) == (uint64_t)e->world - 1) {
        h->arrive.store(0, std::memory_order_relaxed);
        h->gen.fetch_add(1, std::memory_order_release);
        return true;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = std::chrono::duration<double>(e->timeout_s);
    for (uint64_t it = 0; h->gen.load(std::memory_order_acquire) == g; ++it) {
        if (h->poisoned.load(std::memory_order_acquire)) return false;
        if (it > 2000) {
            sched_yield();
            if ((it & 1023) == 0 && std::chrono::steady_clock::now() - t0 > limit) {
                h->poisoned.store(1, std::memory_order_release);
                return false;
            }
        }
    }
    return true;
}

// n doubles from every rank in rank order; two buffer sets alternate by round, so ONE barrier per round is
// enough: a rank can only reuse a set after passing the next round's barrier, which every rank reaches
// after it has read this round's set
int shm_allgather(ShmEx* e, const double* send, int64_t n, double* recv) {
    if (n > e->n) return mfail(LIO_ERR_ARG, "shared-memory exchange: more doubles than the segment holds");
    if (e->hdr->poisoned.load(std::memory_order_acquire))
        return mfail(LIO_ERR_STATE, "shared-memory exchange: the segment is poisoned (an earlier barrier timed out)");
    double* set = e->data + (size_t)(e->round & 1) * (size_t)e->world * (size_t)e->n;
    std::memcpy(set + (size_t)e->rank * (size_t)e->n, send, (size_t)n * sizeof(double));
    if (!shm_barrier(e))
        return mfail(LIO_ERR_STATE, "shared-memory exchange: a rank did not arrive in time (segment poisoned)");
    for (int r = 0; r < e->world; ++r)
        std::memcpy(recv + (size_t)r * (size_t)n, set + (size_t)r * (size_t)e->n, (size_t)n * sizeof(double));
    ++e->round;
    return LIO_OK;
}

// lio_allgather_fn for the ICP handle
int shm_allgather_fn(const double* send, int64_t n, double* recv, void* user) {
    return shm_allgather(static_cast<ShmEx*>(user), send, n, recv) == LIO_OK ? 0 : -1;
}

// ------------------------------------------------------------------ per-process RCCL communicator
struct RcclRank {
    lio::Rccl lib;
    lio::ncclComm_t comm = nullptr;
    int dev = 0;
};

void rccl_free(void* p) {
    auto* r = static_cast<RcclRank*>(p);
    if (r->comm) {
        (void)hipSetDevice(r->dev);
        (void)r->lib.CommDestroy(r->comm);
    }
    delete r;
}

// lio_allgather_dev_fn: the rank's device records all-gathered on the handle's stream (enqueued only)
int rccl_allgather_dev(const double* d_send, int64_t n, double* d_recv, void* stream, void* user) {
    auto* r = static_cast<RcclRank*>(user);
    return r->lib.AllGather(d_send, d_recv, (size_t)n, lio::kNcclDouble, r->comm, (hipStream_t)stream) == 0 ? 0 : -1;
}

}  // namespace

extern "C" {

int lio_shm_exchange_open(const char* name, int rank, int world, int64_t n_per_rank, void** out) {
    if (!out) return mfail(LIO_ERR_ARG, "lio_shm_exchange_open: out is NULL");
    *out = nullptr;
    ShmEx* e = nullptr;
    const int rc = shm_open_ex(name, rank, world, n_per_rank, &e);
    if (rc == LIO_OK) *out = e;
    return rc;
}

int lio_shm_exchange_allgather(void* ex, const double* send, int64_t n, double* recv) {
    if (!ex || !send || !recv || n < 0) return mfail(LIO_ERR_ARG, "lio_shm_exchange_allgather: bad arguments");
    return shm_allgather(static_cast<ShmEx*>(ex), send, n, recv);
}

int lio_shm_exchange_close(void* ex) {
    shm_close(static_cast<ShmEx*>(ex));
    return LIO_OK;
}

int lio_shm_exchange_set_timeout(void* ex, double seconds) {
    if (!ex || !(seconds > 0.0)) return mfail(LIO_ERR_ARG, "lio_shm_exchange_set_timeout: bad arguments");
    static_cast<ShmEx*>(ex)->timeout_s = seconds;
    return LIO_OK;
}

int lio_icp_set_shard_shm(lio_icp* h, int rank, int world, const char* name, int64_t max_source_points) {
    if (!h || world < 1 || rank < 0 || rank >= world || max_source_points < 1)
        return mfail(LIO_ERR_ARG, "lio_icp_set_shard_shm: bad arguments");
    if (world == 1) return lio_icp_set_shard(h, 0, 1, nullptr, nullptr);
    int64_t n = 0;
    int rc = lio_icp_exchange_len(max_source_points, world, &n);
    if (rc) return rc;
    ShmEx* e = nullptr;
    rc = shm_open_ex(name, rank, world, n, &e);
    if (rc) return rc;
    rc = lio_icp_set_shard(h, rank, world, shm_allgather_fn, e);
    if (rc) {
        shm_close(e);
        return rc;
    }
    lio_icp_set_exchange_owner(h, e, [](void* p) { shm_close(static_cast<ShmEx*>(p)); });
    return LIO_OK;
}

int lio_rccl_unique_id(uint8_t* id128) {
    if (!id128) return mfail(LIO_ERR_ARG, "lio_rccl_unique_id: NULL");
    static lio::Rccl lib;
    static std::string why;
    if (!lib.so && !lio::load_rccl(lib, why)) return mfail(LIO_ERR_STATE, "lio_rccl_unique_id: " + why);
    lio::ncclUniqueId u;
    const lio::ncclResult_t r = lib.GetUniqueId(&u);
    if (r != 0) return mfail(LIO_ERR_STATE, std::string("ncclGetUniqueId: ") + lib.GetErrorString(r));
    std::memcpy(id128, u.internal, sizeof(u.internal));
    return LIO_OK;
}

int lio_icp_set_shard_rccl(lio_icp* h, int rank, int world, const uint8_t* id128) {
    if (!h || !id128 || world < 1 || rank < 0 || rank >= world) return mfail(LIO_ERR_ARG, "lio_icp_set_shard_rccl: bad arguments");
    if (world == 1) return lio_icp_set_shard(h, 0, 1, nullptr, nullptr);
    auto* r = new RcclRank();
    std::string why;
    if (!lio::load_rccl(r->lib, why)) {
        delete r;
        return mfail(LIO_ERR_STATE, "lio_icp_set_shard_rccl: " + why);
    }
    r->dev = lio_icp_device(h);
    if (hipSetDevice(r->dev) != hipSuccess) {
        delete r;
        return mfail(LIO_ERR_HIP, "lio_icp_set_shard_rccl: hipSetDevice");
    }
    lio::ncclUniqueId u;
    std::memcpy(u.internal, id128, sizeof(u.internal));
    const lio::ncclResult_t nr = r->lib.CommInitRank(&r->comm, world, u, rank);  // collective: every rank joins
    if (nr != 0) {
        const std::string msg = std::string("ncclCommInitRank: ") + r->lib.GetErrorString(nr);
        r->comm = nullptr;
        delete r;
        return mfail(LIO_ERR_STATE, msg);
    }
    const int rc = lio_icp_set_shard_device(h, rank, world, rccl_allgather_dev, r);
    if (rc) {
        rccl_free(r);
        return rc;
    }
    lio_icp_set_exchange_owner(h, r, rccl_free);
    return LIO_OK;
}

}  // extern "C"
