// lio_icp_host.cpp — LoopClosure::icpAlignment replacement (C-ABI lio_icp_*).
//
// Host loop = pcl::IterativeClosestPoint::computeTransformation as configured at
// /root/reference/fast_lio_sam/src/loop_closure.cpp:3-14 (PCL 1.10 semantics [U]):
//   repeat { correspondences (1-NN, d2 <= max_corr_dist^2) on the incrementally
//            transformed source; < 3 => not converged, stop;
//            T_inc = Umeyama(src_corr, tgt_corr) (TransformationEstimationSVD);
//            transform source by T_inc; final = T_inc * final; ++iter;
//            DefaultConvergenceCriteria }
//   score = getFitnessScore() (unbounded 1-NN of src*final), is_valid =
//   converged && score < icp_score_threshold (loop_closure.cpp:85-90).
// Per iteration the GPU returns Umeyama sufficient statistics per 4096-point
// record; ranks all-gather the records and every rank sums them in record
// order, so the result is bit-identical for any number of ranks.
#include <hip/hip_runtime.h>

#include "lio_pcl.hpp"
#include "lio_pool.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lio_gpu.h"
#include "lio_error.hpp"
#include "lio_kernels.hpp"

namespace {
int ifail(int code, const std::string& m) {
    lio::last_error() = m;
    return code;
}
#define IHIP(expr)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return ifail(LIO_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- 3x3 SVD by one-sided Jacobi (Hestenes) on the columns of A: A = U S V^T
void svd3(const double A[9], double U[9], double S[3], double V[9]) {
    double W[9];
    std::memcpy(W, A, sizeof(W));
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int r = 0; r < 3; ++r) {
                    al += W[3 * r + p] * W[3 * r + p];
                    be += W[3 * r + q] * W[3 * r + q];
                    ga += W[3 * r + p] * W[3 * r + q];
                }
                if (ga == 0.0) continue;
                off = std::max(off, std::fabs(ga) / std::sqrt(al * be + 1e-300));
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                for (int r = 0; r < 3; ++r) {
                    const double wp = W[3 * r + p], wq = W[3 * r + q];
                    W[3 * r + p] = c * wp - s * wq;
                    W[3 * r + q] = s * wp + c * wq;
                    const double vp = V[3 * r + p], vq = V[3 * r + q];
                    V[3 * r + p] = c * vp - s * vq;
                    V[3 * r + q] = s * vp + c * vq;
                }
            }
        if (off < 1e-15) break;
    }
    double sv[3];
    for (int c = 0; c < 3; ++c) sv[c] = std::sqrt(W[c] * W[c] + W[3 + c] * W[3 + c] + W[6 + c] * W[6 + c]);
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int a, int b) { return sv[a] > sv[b]; });
    double Vs[9], Us[9];
    for (int k = 0; k < 3; ++k) {
        const int c = ord[k];
        S[k] = sv[c];
        for (int r = 0; r < 3; ++r) {
            Vs[3 * r + k] = V[3 * r + c];
            Us[3 * r + k] = sv[c] > 0 ? W[3 * r + c] / sv[c] : 0.0;
        }
    }
    // complete U to an orthonormal basis where sigma vanished
    if (!(S[2] > 1e-300 * S[0])) {
        Us[2] = Us[3] * Us[7] - Us[6] * Us[4];
        Us[5] = Us[6] * Us[1] - Us[0] * Us[7];
        Us[8] = Us[0] * Us[4] - Us[3] * Us[1];
    }
    std::memcpy(U, Us, sizeof(Us));
    std::memcpy(V, Vs, sizeof(Vs));
}
double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// Umeyama without scaling (Eigen::umeyama(src, dst, false)) from statistics:
// st[0]=n, st[1..3]=sum p, st[4..6]=sum q, st[7..15]=sum q p^T, all about c0.
void umeyama(const double* st, const double c0[3], float Ti[16]) {
    const double inv_n = 1.0 / st[0];
    double pm[3], qm[3], Sg[9];
    for (int d = 0; d < 3; ++d) {
        pm[d] = st[1 + d] * inv_n;
        qm[d] = st[4 + d] * inv_n;
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Sg[3 * r + c] = st[7 + 3 * r + c] * inv_n - qm[r] * pm[c];
    double U[9], S[3], V[9];
    svd3(Sg, U, S, V);
    const double D = (det3(U) * det3(V) < 0) ? -1.0 : 1.0;
    double R[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] = U[3 * r] * V[3 * c] + U[3 * r + 1] * V[3 * c + 1] + D * U[3 * r + 2] * V[3 * c + 2];
    std::memset(Ti, 0, 16 * sizeof(float));
    for (int r = 0; r < 3; ++r) {
        const double t = (qm[r] + c0[r]) -
                         (R[3 * r] * (pm[0] + c0[0]) + R[3 * r + 1] * (pm[1] + c0[1]) + R[3 * r + 2] * (pm[2] + c0[2]));
        for (int c = 0; c < 3; ++c) Ti[4 * r + c] = (float)R[3 * r + c];
        Ti[4 * r + 3] = (float)t;
    }
    Ti[15] = 1.f;
}

// ---- PCL-order fidelity mode (lio_icp_params.umeyama_float): the host half of pcl::umeyama(src, dst,
// false) in float [U] (Eigen 3.3 Umeyama.h / JacobiSVD.h / Jacobi.h as PCL 1.10 instantiates them for
// Scalar = float, no FMA).  The GPU returns the sequential float sums (means) and the sequential
// sigma accumulator (lio_icp.hip icp_pcl_*); here: sigma = one_over_n * acc, the two-sided Jacobi SVD
// of the 3x3, R = U S V^T (S(2) = -1 when det U det V < 0), t = dst_mean - R src_mean.
struct Rot2 {
    float c, s;
};

// JacobiRotation::makeJacobi(x, y, z) for real scalars
Rot2 make_jacobi_f(float x, float y, float z) {
    const float deno = 2.f * std::fabs(y);
    if (deno < FLT_MIN) return {1.f, 0.f};
    const float tau = (x - z) / deno;
    const float w = std::sqrt(tau * tau + 1.f);
    const float t = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
    const float sign_t = t > 0.f ? 1.f : -1.f;
    const float n = 1.f / std::sqrt(t * t + 1.f);
    return {n, ((-sign_t) * (y / std::fabs(y))) * std::fabs(t) * n};
}

// apply_rotation_in_the_plane(x, y, j) over 3 elements with stride `inc` (a no-op for the identity)
void plane_rot(float* x, float* y, int inc, Rot2 j) {
    if (j.c == 1.f && j.s == 0.f) return;
    for (int i = 0; i < 3; ++i) {
        const float xi = x[i * inc], yi = y[i * inc];
        x[i * inc] = j.c * xi + j.s * yi;
        y[i * inc] = -j.s * xi + j.c * yi;
    }
}

// JacobiSVD<Matrix3f>(A, ComputeFullU | ComputeFullV), column-major storage M[3 * col + row]
void jacobi_svd3_f(const float* A, float* U, float* V, float* sv) {
    float scale = 0.f;
    for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(A[i]));
    if (scale == 0.f) scale = 1.f;
    float W[9];
    for (int i = 0; i < 9; ++i) {
        W[i] = A[i] / scale;
        U[i] = V[i] = (i % 4 == 0) ? 1.f : 0.f;
    }
    auto at = [&](int r, int c) -> float& { return W[3 * c + r]; };
    const float precision = 2.f * FLT_EPSILON;
    float max_diag = std::max(std::max(std::fabs(at(0, 0)), std::fabs(at(1, 1))), std::fabs(at(2, 2)));
    for (bool finished = false; !finished;) {
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const float thr = std::max(FLT_MIN, precision * max_diag);
                if (!(std::fabs(at(p, q)) > thr || std::fabs(at(q, p)) > thr)) continue;
                finished = false;
                // real_2x2_jacobi_svd: rot1 makes the 2x2 block symmetric, then makeJacobi on it
                float m00 = at(p, p), m01 = at(p, q), m10 = at(q, p), m11 = at(q, q);
                Rot2 rot1{1.f, 0.f};
                const float t = m00 + m11, d = m10 - m01;
                if (!(std::fabs(d) < FLT_MIN)) {
                    const float u = t / d;
                    const float tmp = std::sqrt(1.f + u * u);
                    rot1 = {u / tmp, 1.f / tmp};
                }
                if (!(rot1.c == 1.f && rot1.s == 0.f)) {  // m.applyOnTheLeft(0, 1, rot1)
                    const float a0 = m00, b0 = m10, a1 = m01, b1 = m11;
                    m00 = rot1.c * a0 + rot1.s * b0;
                    m10 = -rot1.s * a0 + rot1.c * b0;
                    m01 = rot1.c * a1 + rot1.s * b1;
                    m11 = -rot1.s * a1 + rot1.c * b1;
                }
                const Rot2 jr = make_jacobi_f(m00, m01, m11);
                const Rot2 jrt{jr.c, -jr.s};
                const Rot2 jl{rot1.c * jrt.c - rot1.s * jrt.s, rot1.c * jrt.s + rot1.s * jrt.c};  // rot1 * j_right^T
                plane_rot(W + p, W + q, 3, jl);            // W.applyOnTheLeft(p, q, j_left): rows
                // U.applyOnTheRight(p, q, j_left^T): columns, and applyOnTheRight rotates by the transpose of
                // its argument, so the plane rotation is j_left itself
                plane_rot(U + 3 * p, U + 3 * q, 1, jl);
                plane_rot(W + 3 * p, W + 3 * q, 1, {jr.c, -jr.s});  // W.applyOnTheRight(p, q, j_right)
                plane_rot(V + 3 * p, V + 3 * q, 1, {jr.c, -jr.s});  // V.applyOnTheRight(p, q, j_right)
                max_diag = std::max(max_diag, std::max(std::fabs(at(p, p)), std::fabs(at(q, q))));
            }
    }
    for (int i = 0; i < 3; ++i) {
        const float a = at(i, i);
        sv[i] = std::fabs(a);
        if (a < 0.f)
            for (int r = 0; r < 3; ++r) U[3 * i + r] = -U[3 * i + r];
    }
    for (int i = 0; i < 3; ++i) sv[i] *= scale;
    for (int i = 0; i < 3; ++i) {  // descending; maxCoeff keeps the first maximum
        int pos = i;
        for (int k = i + 1; k < 3; ++k)
            if (sv[k] > sv[pos]) pos = k;
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int r = 0; r < 3; ++r) {
                std::swap(U[3 * i + r], U[3 * pos + r]);
                std::swap(V[3 * i + r], V[3 * pos + r]);
            }
        }
    }
}

float det3_f(const float* M) {  // column-major; Eigen determinant_impl<3>
    auto m = [&](int r, int c) { return M[3 * c + r]; };
    auto h = [&](int a, int b, int c) { return m(a, 0) * (m(b, 1) * m(c, 2) - m(b, 2) * m(c, 1)); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// out16 from the fidelity statistics -> the incremental transform (row-major 4x4 float); order 1 returns
// the raw sequential sigma accumulator (scaled here), orders 2 / 3 sigma as Eigen's GEMM leaves it
void umeyama_pcl_float(const float* out16, float Ti[16], int order = 1) {
    const uint32_t n = [&] {
        uint32_t u;
        std::memcpy(&u, out16 + 6, sizeof(u));
        return u;
    }();
    const float one_over_n = 1.f / (float)n;
    float sm[3], dm[3];
    for (int d = 0; d < 3; ++d) {
        sm[d] = out16[d] * one_over_n;
        dm[d] = out16[3 + d] * one_over_n;
    }
    float sigma[9];  // column-major
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) sigma[3 * c + r] = order == 1 ? one_over_n * out16[7 + 3 * r + c] : out16[7 + 3 * r + c];
    float U[9], V[9], sv[3];
    jacobi_svd3_f(sigma, U, V, sv);
    const float S2 = det3_f(U) * det3_f(V) < 0.f ? -1.f : 1.f;
    std::memset(Ti, 0, 16 * sizeof(float));
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {  // (U S) V^T, each entry e0 + (e1 + e2)
            const float e0 = U[r] * V[c], e1 = U[3 + r] * V[3 + c], e2 = (U[6 + r] * S2) * V[6 + c];
            Ti[4 * r + c] = e0 + (e1 + e2);
        }
    }
    for (int r = 0; r < 3; ++r)
        Ti[4 * r + 3] = dm[r] - (Ti[4 * r] * sm[0] + (Ti[4 * r + 1] * sm[1] + Ti[4 * r + 2] * sm[2]));
    Ti[15] = 1.f;
}

struct EvPair {
    hipEvent_t a = nullptr, b = nullptr;
    hipEvent_t m = nullptr;     // between the correspondence and statistics kernels
    hipEvent_t done = nullptr;  // a pass's statistics have reached the host
};

}  // namespace

struct lio_icp {
    int dev = 0;
    hipStream_t st = nullptr;
    lio_icp_params p{};
    lio::GridBuf tgt;
    float* d_tgt = nullptr;
    int64_t tgt_cap = 0;
    int64_t nt = 0;
    bool tgt_dirty = false;      // setInputTarget staged; uploaded and gridded at the next align (as PCL builds
                                 // its kd-tree lazily in align), on st2, overlapped with the source preparation
    hipStream_t st2 = nullptr;
    float* h_tgt = nullptr;      // pinned staging: the target, the full source
    int64_t h_tgt_cap = 0;
    float* h_src = nullptr;
    int64_t h_src_cap = 0;
    double c0[3] = {0, 0, 0};
    int64_t ns = 0;
    int rank = 0, world = 1;
    lio_allgather_fn fn = nullptr;
    void* user = nullptr;
    lio_allgather_dev_fn fn_dev = nullptr;  // device-side exchange (lio_icp_set_shard_device)
    void* user_dev = nullptr;
    double* d_xsend = nullptr;  // exchange buffers: this rank's records / all ranks' (device)
    double* d_xrecv = nullptr;
    int64_t x_len = 0;          // doubles per rank they hold
    bool x_ext = false;         // caller-owned (lio_icp_set_exchange_buffers)
    double* h_out17 = nullptr;  // host-mapped record-order sums (device exchange)
    double* h_out17_dev = nullptr;
    // shard buffers
    int64_t sh_begin = 0, sh_n = 0, cap = 0;
    float* d_src = nullptr;
    float* d_cur = nullptr;
    float* d_thist = nullptr;  // transforms applied this alignment (the correspondence kernel's history)
    int thist_cap = 0, nT = 0;
    float* d_fd2 = nullptr;
    int* d_fid = nullptr;
    lio::GridBuf qgrid;      // the shard's source binned by tile cell (icp_build_tiles)
    uint2* d_tiles = nullptr;
    uint32_t* d_tscratch = nullptr;
    void* d_ttmp = nullptr;
    size_t ttmp_bytes = 0;
    int64_t tiles_cap = 0, tscratch_cap = 0;
    int ntiles = 0;
    float tile_cell = 2.0f;
    bool have_prior = false;  // nn ids of this alignment's previous pass are in d_fid
    uint32_t* d_tcost = nullptr;  // per tile: candidates of the last pass
    uint32_t* d_order = nullptr;  // longest-first tile order (valid when have_order)
    bool have_order = false;
    unsigned long long* d_dbg = nullptr;  // search counters (diagnostics build: LIO_DIAG + LIO_ICP_DEBUG)
    size_t dbg_bytes = 0;
    double* h_super = nullptr;      // pinned, host-mapped: the pass's 4096-point records
    double* h_super_dev = nullptr;  // device view of h_super (the statistics kernel writes it, zero-copy)
    int64_t super_cap = 0;
    bool src_dirty = true;
    float* d_pcl16 = nullptr;  // umeyama_float: the serial float sums (launch_icp_pcl_stats: the fallback)
    float* h_pcl16 = nullptr;  // pinned copy
    lio::PclBuf pcl;           // umeyama_float: compacted pairs + seqsum chains
    float* d_pclout = nullptr; // pcl_pack output (kPclOutWords)
    float* h_pclout = nullptr; // pinned, host-mapped: a copy, or the pack's own stores (pcl_wait polls [23])
    float* h_pclout_dev = nullptr;
    uint32_t pcl_seq = 0;      // the last sequence number handed to the pack
    void* x_owner = nullptr;   // exchange state owned by the handle (lio_icp_mp.cpp: shm segment, RCCL comm)
    void (*x_owner_free)(void*) = nullptr;
    // sharded PCL float modes (fid_sharded): only this rank's shard on the device; the float chains split by
    // window (lio_seqsum.hpp), the per-rank event-list slot of the exchange (grown from what the last pass
    // needed, the same on every rank), pinned staging for a host exchange, the serial fallback's gathered pairs
    int ev_slot = 2048, ev_slot_s = 2048;
    double* h_xs = nullptr;
    double* h_xr = nullptr;
    int64_t hx_cap = 0;
    lio::PclBuf pg;
    int64_t fid_stats[4] = {0, 0, 0, 0};  // re-passes, serial fallbacks, events of the last pass, passes
    int fid_flags = 0;
    int64_t fid_evcap = 0;
    bool timing = false;
    lio_kernel_timing tm{};
    EvPair ev;
    // set-up started by lio_icp_set_target / _set_source that runs on behind the caller (the target's upload
    // and grid on st2, the source's upload and binning on st): every other entry point joins them first; a
    // failure leaves the dirty flag set, so lio_icp_align repeats the step and reports it
    std::thread bg_tgt, bg_src;
    std::string bg_tgt_err, bg_src_err;  // why a background set-up failed (reported if align's retry fails too)
};

static void icp_join(lio_icp* h) {
    if (h->bg_src.joinable()) h->bg_src.join();
    if (h->bg_tgt.joinable()) h->bg_tgt.join();
}
// the two set-ups touch disjoint state (target: st2, d_tgt, tgt grid, c0; source: st, the shard buffers),
// so a new target only waits for the previous target's thread and a new source for the previous source's
static void icp_join_tgt(lio_icp* h) {
    if (h->bg_tgt.joinable()) h->bg_tgt.join();
}
static void icp_join_src(lio_icp* h) {
    if (h->bg_src.joinable()) h->bg_src.join();
}

// the PCL float modes with more than one rank: the float chains run split over the ranks' windows
static bool fid_sharded(const lio_icp* h) { return h->p.umeyama_float > 0 && h->world > 1; }

// Capacities grow geometrically from a floor sized for the reference's largest submaps (C4: 500 k points): a
// loop-closure node whose submaps change size on every 2 Hz loopTimerFunc call (fast_lio_sam.cpp:682-730) then
// allocates on its first call and (almost) never again — a hipFree synchronises the device, and a re-allocation
// per call showed up as a 9 ms cold loop leg against 1.1 ms warm.
constexpr int64_t kIcpCapFloor = (int64_t)1 << 19;
static int64_t icp_cap(int64_t need, int64_t cap) { return std::max(std::max(need + need / 2, 2 * cap), kIcpCapFloor); }

static int icp_check_dev(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ifail(LIO_ERR_NODEV, "no HIP device (no CPU path)");
    if (dev < 0 || dev >= n) return ifail(LIO_ERR_ARG, "device ordinal out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return ifail(LIO_ERR_HIP, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ifail(LIO_ERR_NODEV, "device is not gfx950");
    return LIO_OK;
}

static void shard_range(int64_t ns, int rank, int world, int64_t& b, int64_t& n) {
    const int64_t nsup = (ns + lio::kIcpSuper - 1) / lio::kIcpSuper;
    const int64_t s0 = nsup * rank / world, s1 = nsup * (rank + 1) / world;
    b = std::min<int64_t>(s0 * lio::kIcpSuper, ns);
    n = std::min<int64_t>(s1 * lio::kIcpSuper, ns) - b;
}

extern "C" {

int lio_icp_create(const lio_icp_params* p, lio_icp** out) {
    if (!p || !out) return ifail(LIO_ERR_ARG, "bad arguments");
    *out = nullptr;
    if (p->umeyama_float < LIO_ICP_UMEYAMA_DOUBLE || p->umeyama_float > LIO_ICP_UMEYAMA_PCL_GEMM48)
        return ifail(LIO_ERR_ARG, "lio_icp_create: umeyama_float must be -1 (double statistics), 0 (default) or 1..3");
    int rc = icp_check_dev(p->device);
    if (rc) return rc;
    IHIP(hipSetDevice(p->device));
    auto* h = new lio_icp();
    h->dev = p->device;
    h->p = *p;
    // the default is the reference's float arithmetic (Eigen 3.3 GEMM order, loop_closure.h:42); the double
    // statistics are an explicit opt-in (-1), stored as 0 from here on
    if (h->p.umeyama_float == LIO_ICP_UMEYAMA_DEFAULT) h->p.umeyama_float = LIO_ICP_UMEYAMA_PCL_GEMM32;
    else if (h->p.umeyama_float == LIO_ICP_UMEYAMA_DOUBLE) h->p.umeyama_float = 0;
    if (!(h->p.cell_size > 0.f)) h->p.cell_size = 1.0f;  // 0.3 m voxelised submaps: 1 m target cells (scripts/icp_cells.py)
    // the grids' capacity floors: a C4-sized submap (500 k points, ~1 M target cells at 1 m) fits from the start
    h->tgt.min_entries = h->qgrid.min_entries = kIcpCapFloor;
    h->tgt.min_cells = 1u << 20;
    h->qgrid.min_cells = 1u << 17;
    if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking) != hipSuccess) {
        if (h->st) (void)hipStreamDestroy(h->st);
        delete h;
        return ifail(LIO_ERR_HIP, "icp stream/alloc failed");
    }
    (void)hipEventCreate(&h->ev.a);
    (void)hipEventCreate(&h->ev.b);
    (void)hipEventCreate(&h->ev.m);
    (void)hipEventCreateWithFlags(&h->ev.done, hipEventDisableTiming);
    *out = h;
    return LIO_OK;
}

// internal (lio_icp_mp.cpp): hand the exchange state of a multi-process shard to the handle (freed with it,
// or when another exchange replaces it)
void lio_icp_set_exchange_owner(lio_icp* h, void* owner, void (*free_fn)(void*)) {
    icp_join(h);
    if (h->x_owner && h->x_owner_free) {
        (void)hipSetDevice(h->dev);
        (void)hipStreamSynchronize(h->st);
        h->x_owner_free(h->x_owner);
    }
    h->x_owner = owner;
    h->x_owner_free = free_fn;
}

int lio_icp_device(const lio_icp* h) { return h->dev; }

int lio_icp_destroy(lio_icp* h) {
    if (!h) return LIO_OK;
    icp_join(h);
    (void)hipSetDevice(h->dev);
    (void)hipStreamSynchronize(h->st);
    lio_icp_set_exchange_owner(h, nullptr, nullptr);
    lio::grid_free(h->tgt);
    lio::grid_free(h->qgrid);
    void* ptrs[] = {h->d_thist, h->d_tgt,   h->d_src,   h->d_cur,   h->d_fd2,  h->d_fid, h->d_tiles,
                    h->d_tscratch, h->d_ttmp, h->d_dbg, h->d_tcost, h->d_order, h->d_pcl16};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    lio::pcl_free(h->pg);
    if (h->h_xs) (void)hipHostFree(h->h_xs);
    if (h->h_xr) (void)hipHostFree(h->h_xr);
    if (h->h_super) (void)hipHostFree(h->h_super);
    if (h->h_pcl16) (void)hipHostFree(h->h_pcl16);
    lio::pcl_free(h->pcl);
    if (h->d_pclout) (void)hipFree(h->d_pclout);
    if (h->h_pclout) (void)hipHostFree(h->h_pclout);
    if (h->h_out17) (void)hipHostFree(h->h_out17);
    if (!h->x_ext) {
        if (h->d_xsend) (void)hipFree(h->d_xsend);
        if (h->d_xrecv) (void)hipFree(h->d_xrecv);
    }
    if (h->ev.a) (void)hipEventDestroy(h->ev.a);
    if (h->ev.b) (void)hipEventDestroy(h->ev.b);
    if (h->ev.m) (void)hipEventDestroy(h->ev.m);
    if (h->ev.done) (void)hipEventDestroy(h->ev.done);
    if (h->h_tgt) (void)hipHostFree(h->h_tgt);
    if (h->h_src) (void)hipHostFree(h->h_src);
    (void)hipStreamSynchronize(h->st2);
    (void)hipStreamDestroy(h->st2);
    (void)hipStreamDestroy(h->st);
    delete h;
    return LIO_OK;
}

// host copy into the handle's pinned staging buffer (grown geometrically), split over a few threads for
// large clouds: the caller's buffer may go away after the call (PCL copies the cloud too)
static int stage_pinned(float*& buf, int64_t& cap, const float* xyz, int64_t n) {
    if (n > cap || !buf) {
        if (buf) (void)hipHostFree(buf);
        buf = nullptr;
        cap = 0;
        const int64_t c = icp_cap(n, cap);
        lio::count_alloc();
        if (hipHostMalloc(reinterpret_cast<void**>(&buf), (size_t)c * 3 * sizeof(float), hipHostMallocDefault) != hipSuccess)
            return ifail(LIO_ERR_NOMEM, "ICP staging: hipHostMalloc failed");
        cap = c;
    }
    const size_t bytes = (size_t)n * 3 * sizeof(float);
    const int nt = bytes >= ((size_t)1 << 20) ? 4 : 1;  // the host pool's threads (no thread created per call)
    if (nt == 1) {
        std::memcpy(buf, xyz, bytes);
    } else {
        const int64_t per = (3 * n + nt - 1) / nt;
        lio::HostPool::get().parallel_for(nt, [&](int t) {
            const int64_t b = std::min<int64_t>(3 * n, t * per), e = std::min<int64_t>(3 * n, b + per);
            std::memcpy(buf + b, xyz + b, (size_t)(e - b) * sizeof(float));
        });
    }
    return LIO_OK;
}

static int target_build(lio_icp* h);
static int icp_prepare(lio_icp* h);

int lio_icp_set_target(lio_icp* h, const float* xyz, int64_t n) {
    if (!h || n <= 0 || !xyz) return ifail(LIO_ERR_ARG, "lio_icp_set_target: bad arguments");
    icp_join_tgt(h);
    IHIP(hipSetDevice(h->dev));
    IHIP(hipStreamSynchronize(h->st2));  // a previous target upload may still read the staging buffer
    const int rc = stage_pinned(h->h_tgt, h->h_tgt_cap, xyz, n);
    if (rc) return rc;
    h->nt = n;
    h->tgt_dirty = true;
    h->bg_tgt_err.clear();
    // upload + grid on st2 behind the caller: overlaps the source's set-up and whatever the caller does next
    // (no thread: the set-up runs here; a failure of either form leaves tgt_dirty for align to retry)
    auto job = [h] {
        if (target_build(h) != LIO_OK) h->bg_tgt_err = lio::last_error();
    };
    try {
        h->bg_tgt = std::thread(job);
    } catch (...) {
        job();
    }
    return LIO_OK;
}

// the staged target: upload + grid + accumulation centre, on st2 (called from a helper thread)
static int target_build(lio_icp* h) {
    IHIP(hipSetDevice(h->dev));
    const int64_t n = h->nt;
    if (n > h->tgt_cap || !h->d_tgt) {
        if (h->d_tgt) IHIP(hipFree(h->d_tgt));
        h->d_tgt = nullptr;
        const int64_t c = icp_cap(n, h->tgt_cap);
        h->tgt_cap = 0;
        lio::count_alloc();
        IHIP(hipMalloc(&h->d_tgt, (size_t)c * 3 * sizeof(float)));
        h->tgt_cap = c;
    }
    IHIP(hipMemcpyAsync(h->d_tgt, h->h_tgt, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, h->st2));
    int rc = lio::grid_build(h->tgt, h->d_tgt, n, h->p.cell_size, h->st2);
    if (rc) return ifail(rc == -5 ? LIO_ERR_NOMEM : LIO_ERR_HIP, "target grid build failed");
    IHIP(hipStreamSynchronize(h->st2));
    // fixed accumulation centre: target bounding-box centre (float)
    const float* bb = h->tgt.aabb_host;
    for (int d = 0; d < 3; ++d) h->c0[d] = (double)(0.5f * (bb[d] + bb[3 + d]));
    h->tgt_dirty = false;
    return LIO_OK;
}

int lio_icp_set_source(lio_icp* h, const float* xyz, int64_t n) {
    if (!h || n < 0 || (n > 0 && !xyz) || n >= (int64_t)1 << 30) return ifail(LIO_ERR_ARG, "lio_icp_set_source: bad arguments");
    icp_join_src(h);
    IHIP(hipSetDevice(h->dev));
    IHIP(hipStreamSynchronize(h->st));  // the previous source upload may still read the staging buffer
    if (n > 0) {
        const int rc = stage_pinned(h->h_src, h->h_src_cap, xyz, n);
        if (rc) return rc;
    }
    h->ns = n;
    h->src_dirty = true;
    h->bg_src_err.clear();
    // this rank's shard uploaded and binned on st behind the caller (a later lio_icp_set_shard* marks it
    // dirty again and align repeats it for the new shard)
    auto job = [h] {
        if (hipSetDevice(h->dev) != hipSuccess) h->bg_src_err = "hipSetDevice";
        else if (icp_prepare(h) != LIO_OK) h->bg_src_err = lio::last_error();
    };
    try {
        h->bg_src = std::thread(job);
    } catch (...) {
        job();
    }
    return LIO_OK;
}

int lio_icp_set_shard(lio_icp* h, int rank, int world, lio_allgather_fn fn, void* user) {
    if (!h || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn))
        return ifail(LIO_ERR_ARG, "lio_icp_set_shard: bad arguments");
    icp_join(h);
    h->rank = rank;
    h->world = world;
    h->fn = fn;
    h->user = user;
    h->fn_dev = nullptr;
    h->user_dev = nullptr;
    h->src_dirty = true;
    return LIO_OK;
}

int lio_icp_set_shard_device(lio_icp* h, int rank, int world, lio_allgather_dev_fn fn, void* user) {
    if (!h || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn))
        return ifail(LIO_ERR_ARG, "lio_icp_set_shard_device: bad arguments");
    icp_join(h);
    h->rank = rank;
    h->world = world;
    h->fn = nullptr;
    h->user = nullptr;
    h->fn_dev = fn;
    h->user_dev = user;
    h->src_dirty = true;
    return LIO_OK;
}

// Exchange messages of one rank, in doubles (all-gathered, rank r's at r * count of the receive buffer):
//   records   every pass: its 4096-point records (slot = ceil(records / world) of kIcpStride); in the sharded
//             PCL float modes followed by its windows' chain totals (lio_seqsum.hpp, kTotPad)
//   events    sharded PCL float modes: the seqsum event message of its window (ev_slot events per chain),
//             for the means with its first kPclMaxKc pairs (SeqHeads, lio_seqsum.hpp)
//   blocks    sharded orders 2 / 3: its depth blocks of sigma and the verification statuses
//   gather    the sharded serial fallback: its pairs in rounds
// exchange_len is the capacity of every one of them (the event slot up to ev_slot_cap).
static int64_t exchange_slot(int64_t ns, int world) {
    const int64_t nsup = (ns + lio::kIcpSuper - 1) / lio::kIcpSuper;
    return (nsup + world - 1) / world;
}
static int64_t shard_points_max(int64_t ns, int world) { return exchange_slot(ns, world) * lio::kIcpSuper; }
static int64_t ev_slot_cap(int64_t ns, int world) { return std::max<int64_t>(4096, shard_points_max(ns, world) / 8); }
static int64_t records_count(int64_t ns, int world) { return exchange_slot(ns, world) * lio::kIcpStride; }
// blocks of a window in the block-sum message (seq_bsum's tot_out)
static int64_t tot_blocks(int64_t ns, int world) { return (shard_points_max(ns, world) + lio::kSeqBlock - 1) / lio::kSeqBlock + 1; }
static int64_t tot_words(int64_t ns, int world, int nch) { return lio::seq_tot_words(nch, tot_blocks(ns, world)); }
static int64_t exchange_len_fsh(int64_t ns, int world) {
    const int64_t rec = records_count(ns, world) + tot_words(ns, world, lio::kSeqMaxChains);
    const int64_t ev = lio::seqsum_msg_words(lio::kSeqMaxChains, (int)ev_slot_cap(ns, world)) + lio::pcl_heads_words();  // >= 6 chains' heads
    const int64_t x3 = lio::pcl_x3_words(lio::pcl_blocks_slot(shard_points_max(ns, world)));
    return std::max(std::max(rec, ev), std::max(x3, (int64_t)4096));
}
static int64_t exchange_len(int64_t ns, int world) { return exchange_len_fsh(ns, world); }

// the records of every rank (rank r at recv + r * stride doubles) summed in global record order
static void combine_records(const double* recv, int64_t ns, int world, int64_t stride, double out17[17]) {
    const int64_t nsup = (ns + lio::kIcpSuper - 1) / lio::kIcpSuper;
    for (int k = 0; k < 17; ++k) out17[k] = 0.0;
    for (int r = 0; r < world; ++r) {
        const int64_t s0 = nsup * r / world, s1 = nsup * (r + 1) / world;
        for (int64_t s = s0; s < s1; ++s) {
            const double* rec = &recv[(size_t)r * (size_t)stride + (size_t)(s - s0) * lio::kIcpStride];
            for (int k = 0; k < 17; ++k) out17[k] += rec[k];
        }
    }
}

int lio_icp_exchange_len(int64_t n_source, int world, int64_t* n_per_rank) {
    if (n_source < 0 || world < 1 || !n_per_rank) return ifail(LIO_ERR_ARG, "lio_icp_exchange_len: bad arguments");
    *n_per_rank = std::max<int64_t>(exchange_len(n_source, world), lio::kIcpStride);
    return LIO_OK;
}

int lio_icp_set_exchange_buffers(lio_icp* h, double* d_send, double* d_recv, int64_t n_per_rank) {
    if (!h || !d_send || !d_recv || n_per_rank <= 0) return ifail(LIO_ERR_ARG, "lio_icp_set_exchange_buffers: bad arguments");
    icp_join(h);
    IHIP(hipSetDevice(h->dev));
    if (!h->x_ext) {
        if (h->d_xsend) IHIP(hipFree(h->d_xsend));
        if (h->d_xrecv) IHIP(hipFree(h->d_xrecv));
    }
    h->d_xsend = d_send;
    h->d_xrecv = d_recv;
    h->x_len = n_per_rank;
    h->x_ext = true;
    return LIO_OK;
}

// device exchange buffers for the current source (the handle's own unless the caller's are large enough): the
// sharded PCL float modes need exchange_len, the double statistics only the records
static int exchange_reserve(lio_icp* h) {
    const int64_t need = std::max<int64_t>(fid_sharded(h) ? exchange_len(h->ns, h->world) : records_count(h->ns, h->world),
                                           lio::kIcpStride);
    if (!h->h_out17) {  // the record-order sums land here whoever owns the exchange buffers
        IHIP(hipHostMalloc(&h->h_out17, 32 * sizeof(double), hipHostMallocMapped));
        IHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_out17_dev), h->h_out17, 0));
    }
    if (!h->h_out17_dev) return ifail(LIO_ERR_STATE, "lio_icp_align: no device view of the result block");
    if (h->x_ext) {
        if (h->x_len < need)
            return ifail(LIO_ERR_ARG, "lio_icp_align: caller exchange buffers too small (lio_icp_exchange_len: " +
                                          std::to_string(need) + " doubles per rank)");
        return LIO_OK;
    }
    if (h->x_len < need || !h->d_xsend || !h->d_xrecv) {
        if (h->d_xsend) IHIP(hipFree(h->d_xsend));
        if (h->d_xrecv) IHIP(hipFree(h->d_xrecv));
        h->d_xsend = h->d_xrecv = nullptr;
        const int64_t c = std::max(need + need / 2, 2 * h->x_len);
        h->x_len = 0;
        lio::count_alloc(2);
        IHIP(hipMalloc(&h->d_xsend, (size_t)c * sizeof(double)));
        IHIP(hipMalloc(&h->d_xrecv, (size_t)c * h->world * sizeof(double)));
        h->x_len = c;
    }
    return LIO_OK;
}

static int icp_prepare(lio_icp* h) {
    if (!h->src_dirty) return LIO_OK;
    shard_range(h->ns, h->rank, h->world, h->sh_begin, h->sh_n);
    if (h->sh_n > h->cap || !h->d_src) {
        void** ptrs[] = {(void**)&h->d_src,   (void**)&h->d_cur,   (void**)&h->d_fd2,  (void**)&h->d_fid,
                         (void**)&h->d_tiles, (void**)&h->d_tcost, (void**)&h->d_order};
        const int64_t n = icp_cap(h->sh_n, h->cap);
        h->cap = 0;  // a failed allocation below leaves no buffer that looks usable (and nothing freed twice)
        for (void** q : ptrs) {
            if (*q) (void)hipFree(*q);
            *q = nullptr;
        }
        lio::count_alloc(7);
        IHIP(hipMalloc(&h->d_src, n * 3 * sizeof(float)));
        IHIP(hipMalloc(&h->d_cur, n * 3 * sizeof(float)));
        IHIP(hipMalloc(&h->d_fd2, n * sizeof(float)));
        IHIP(hipMalloc(&h->d_fid, n * sizeof(int)));
        IHIP(hipMalloc(&h->d_tiles, (n + n / lio::kIcpTileQ + 1) * sizeof(uint2)));
        IHIP(hipMalloc(&h->d_tcost, (n + n / lio::kIcpTileQ + 1) * sizeof(uint32_t)));
        IHIP(hipMalloc(&h->d_order, (n + n / lio::kIcpTileQ + 64) * sizeof(uint32_t)));  // + the 9 share offsets
        h->cap = n;
    }
    const int64_t nsup_all = (h->ns + lio::kIcpSuper - 1) / lio::kIcpSuper + 1;
    if (nsup_all > h->super_cap) {
        if (h->h_super) (void)hipHostFree(h->h_super);
        h->h_super = nullptr;
        h->h_super_dev = nullptr;
        const int64_t c = icp_cap(nsup_all, h->super_cap * lio::kIcpSuper) / lio::kIcpSuper + 1;
        h->super_cap = 0;
        lio::count_alloc();
        IHIP(hipHostMalloc(&h->h_super, c * lio::kIcpStride * sizeof(double), hipHostMallocMapped));
        IHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_super_dev), h->h_super, 0));
        h->super_cap = c;
    }
    h->ntiles = 0;
    h->have_order = false;  // new tiles: cell order until a pass has measured them
    if (h->sh_n > 0) {
        IHIP(hipMemcpyAsync(h->d_src, h->h_src + 3 * h->sh_begin, h->sh_n * 3 * sizeof(float),
                            hipMemcpyHostToDevice, h->st));
        // bin the shard by tile cell: tiles of <= 64 spatially compact queries (perf only: every
        // query's 1-NN is exact whatever tile it is in)
        int rc = lio::grid_build(h->qgrid, h->d_src, h->sh_n, h->tile_cell, h->st);
        if (rc) return ifail(rc == -5 ? LIO_ERR_NOMEM : LIO_ERR_HIP, "source binning failed");
        const int64_t need = 6 * ((int64_t)h->qgrid.geom.ncells + 1);  // icp_build_tiles' scratch
        if (need > h->tscratch_cap) {
            if (h->d_tscratch) IHIP(hipFree(h->d_tscratch));
            h->d_tscratch = nullptr;
            const int64_t c = std::max(need + need / 2, 2 * h->tscratch_cap);
            h->tscratch_cap = 0;
            lio::count_alloc();
            IHIP(hipMalloc(&h->d_tscratch, c * sizeof(uint32_t)));
            h->tscratch_cap = c;
        }
        const int nt = lio::icp_build_tiles(h->qgrid, h->d_tiles, h->d_tscratch, h->d_ttmp, h->ttmp_bytes, h->st);
        if (nt < 0) return ifail(nt == -5 ? LIO_ERR_NOMEM : LIO_ERR_HIP, "tile list failed");
        h->ntiles = nt;
    }
    h->src_dirty = false;
    return LIO_OK;
}

// Float fidelity statistics of the pass (h_pclout after the pass's wait): a chain that failed its
// verification is re-run with the predictions of its reconstruction (passes 2, 3); an event-list overflow
// or a third failure falls back to the serial kernels (one lane per chain, the sums in order).
static uint32_t pcl_word(const lio_icp* h, int w) {
    uint32_t u;
    std::memcpy(&u, h->h_pclout + 16 + w, sizeof(u));
    return u;
}

// one rank: the pack stores its words straight into h_pclout (host-mapped) and its sequence number last; the host
// polls that word instead of a copy launch and an event wait (the pass's last launch is the pack)
static uint32_t pcl_next_seq(lio_icp* h) {
    if (++h->pcl_seq == 0) h->pcl_seq = 1;
    return h->pcl_seq;
}
static int pcl_wait(lio_icp* h, uint32_t seq) {
    const volatile uint32_t* w = reinterpret_cast<const volatile uint32_t*>(h->h_pclout + 23);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; *w != seq; ++spin) {
        if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            IHIP(hipStreamSynchronize(h->st));  // a failed launch reports here
            if (*w != seq) return ifail(LIO_ERR_STATE, "lio_icp_align: the statistics never arrived");
            break;
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return LIO_OK;
}

static int pcl_finish(lio_icp* h, const lio::IcpArgs& a) {
    const int order = h->p.umeyama_float;
    // the compaction's look-back timed out (h_pclout[19]; never expected): its pairs cannot be trusted, so the
    // serial kernels below re-compact them; the flag is cleared here, or every later pass would see it
    const bool lb_timeout = pcl_word(h, 3) != 0;
    if (lb_timeout) IHIP(hipMemsetAsync(h->pcl.small + lio::kPclTicket + 1, 0, sizeof(uint32_t), h->st));
    ++h->fid_stats[3];
    {
        int ev;
        std::memcpy(&ev, h->h_pclout + 18, sizeof(ev));
        h->fid_stats[2] = ev;
    }
    constexpr int kMaxPasses = 4;  // per chain set; the verification makes any pass count safe
    int mpass = 1, spass = 1;
    while (!lb_timeout && (pcl_word(h, 0) | pcl_word(h, 1)) != 0) {
        const uint32_t bad = pcl_word(h, 0), over = pcl_word(h, 1);
        // a failed verification set forced-event bits: whatever runs next (a re-pass, a restarted sigma pass 1,
        // the serial fallback), the next pass 1 must clear them (stale bits only add events)
        if (bad) h->pcl.means.forced_dirty = h->pcl.sig.forced_dirty = true;
        if (over) break;  // more passes only add events
        if (bad & 0x3fu) {  // the means (sigma depends on them: its chains restart from pass 1)
            if (mpass >= kMaxPasses) break;
            lio::launch_pcl_means(h->pcl, ++mpass, h->st);
            spass = 1;
            lio::launch_pcl_sigma(h->pcl, order, spass, h->st);
        } else {
            if (spass >= kMaxPasses) break;
            lio::launch_pcl_sigma(h->pcl, order, ++spass, h->st);
        }
        ++h->fid_stats[0];
        ++h->fid_stats[3];
        const uint32_t seq = pcl_next_seq(h);
        lio::launch_pcl_pack(h->pcl, order, h->h_pclout_dev, h->st, nullptr, seq);
        const int rc = pcl_wait(h, seq);
        if (rc) return rc;
    }
    if (lb_timeout || (pcl_word(h, 0) | pcl_word(h, 1)) != 0) {  // the serial kernels: one lane per chain
        ++h->fid_stats[1];
        if (order == lio::kPclSeq) {
            lio::launch_icp_pcl_stats(a, h->pcl.pairs, h->pcl.cap, h->d_pcl16, h->st);
            IHIP(hipMemcpyAsync(h->h_pclout, h->d_pcl16, 16 * sizeof(float), hipMemcpyDeviceToHost, h->st));
        } else {
            lio::launch_icp_pcl_means_serial(a, h->pcl.pairs, h->pcl.cap, h->d_pcl16, h->st);
            lio::launch_pcl_sigma(h->pcl, order, 1, h->st, h->d_pcl16);
            lio::launch_pcl_pack(h->pcl, order, h->d_pclout, h->st, h->d_pcl16);
            IHIP(hipMemcpyAsync(h->h_pclout, h->d_pclout, lio::kPclOutWords * sizeof(float), hipMemcpyDeviceToHost, h->st));
        }
        IHIP(hipStreamSynchronize(h->st));
        h->h_pclout[16] = h->h_pclout[17] = 0.f;
    }
    IHIP(hipGetLastError());
    return LIO_OK;
}

// the float statistics of the pass's accepted pairs (pa: this rank's correspondences, or with the source
// sharded all ranks' gathered ids over the whole cloud), enqueued; h_pclout once the stream gets there
static int enqueue_pcl(lio_icp* h, const lio::IcpArgs& pa) {
    const int order = h->p.umeyama_float;
    (void)pa;  // the pairs were compacted by the statistics launch (icp_pass: launch_icp_stats with IcpCompact)
    if (h->fid_flags & 4)  // test hook (lio_icp_set_fidelity_debug): report a look-back time-out for this pass
        IHIP(hipMemsetAsync(h->pcl.small + lio::kPclTicket + 1, 1, sizeof(uint32_t), h->st));
    lio::launch_pcl_means(h->pcl, 1, h->st);
    lio::launch_pcl_sigma(h->pcl, order, 1, h->st);
    lio::launch_pcl_pack(h->pcl, order, h->h_pclout_dev, h->st, nullptr, pcl_next_seq(h));
    return LIO_OK;
}

// ---------------------------------------------------------------- the sharded PCL float statistics
// Per correspondence pass (world > 1, umeyama_float 1..3), three all-gathers on the handle's stream:
//   records   the tile kernel, the records, the window's compaction, the means chains' block sums and the
//             window's totals -> all-gather -> the records' sum (MSE, counts) and every window's place in the
//             chains (seq_shard_offsets)
//   events    the means chains counted and their events listed on the window -> all-gather (+ each window's
//             first kPclMaxKc pairs) -> the global event lists, the walk over all of them (every rank: the serial
//             floor), the window verified
//   blocks    orders 2 / 3: the GEMM depth blocks starting in the window -> all-gather -> res += alpha * C_b over
//             all blocks in order (order 1: the sigma chains take the means' three steps themselves)
// so per-rank work and memory follow the window (source / world) except the walk and the order-of-blocks
// sums, and every rank gets the one-rank transform bit for bit (the verification covers every element).

// all-gather `cnt` doubles per rank from d_xsend into d_xrecv (rank r's at r * cnt) in the handle's stream order:
// the device callback enqueues it (RCCL / torch on an external stream); a host callback goes through pinned
// staging, one wait per call
static int xchg(lio_icp* h, int64_t cnt) {
    if (cnt > h->x_len) return ifail(LIO_ERR_STATE, "lio_icp_align: an exchange message is larger than the buffers");
    if (h->fn_dev) {
        if (h->fn_dev(h->d_xsend, cnt, h->d_xrecv, (void*)h->st, h->user_dev) != 0)
            return ifail(LIO_ERR_STATE, "device all-gather callback failed");
        return LIO_OK;
    }
    if (!h->fn) return ifail(LIO_ERR_STATE, "lio_icp_align: sharded without an exchange");
    if (h->hx_cap < h->x_len) {
        if (h->h_xs) (void)hipHostFree(h->h_xs);
        if (h->h_xr) (void)hipHostFree(h->h_xr);
        h->h_xs = h->h_xr = nullptr;
        h->hx_cap = 0;
        lio::count_alloc(2);
        IHIP(hipHostMalloc(&h->h_xs, (size_t)h->x_len * sizeof(double), hipHostMallocDefault));
        IHIP(hipHostMalloc(&h->h_xr, (size_t)h->x_len * h->world * sizeof(double), hipHostMallocDefault));
        h->hx_cap = h->x_len;
    }
    IHIP(hipMemcpyAsync(h->h_xs, h->d_xsend, (size_t)cnt * sizeof(double), hipMemcpyDeviceToHost, h->st));
    IHIP(hipStreamSynchronize(h->st));
    if (h->fn(h->h_xs, cnt, h->h_xr, h->user) != 0) return ifail(LIO_ERR_STATE, "allgather callback failed");
    IHIP(hipMemcpyAsync(h->d_xrecv, h->h_xr, (size_t)cnt * h->world * sizeof(double), hipMemcpyHostToDevice, h->st));
    return LIO_OK;
}

static lio::SeqPairs fsh_means_src(const lio_icp* h) { return lio::SeqPairs{h->pcl.pairs, h->pcl.cap}; }
static lio::SeqSigma fsh_sigma_src(const lio_icp* h) { return lio::SeqSigma{h->pcl.pairs, h->pcl.mean6, h->pcl.cap}; }

// the means' event message is packed (seqsum_shard_mid / _repack): + the window's first pairs -> all-gather ->
// the pairs after the window appended, the global lists, the walk, the window's verification
static int fsh_heads(const lio_icp* h) { return h->p.umeyama_float != 1 ? lio::kPclMaxKc : 0; }
static int fsh_means_events(lio_icp* h, int pass) {
    lio::PclBuf& P = h->pcl;
    const int64_t m2 = lio::seqsum_msg_words(6, h->ev_slot, fsh_heads(h));
    int rc = xchg(h, m2);
    if (rc) return rc;
    lio::SeqHeads hd;
    if (fsh_heads(h)) hd = lio::SeqHeads{lio::kPclMaxKc, P.pairs, P.cap, P.ghead, lio::kPclTinyN};
    lio::seqsum_shard_tail(fsh_means_src(h), 6, P.small + lio::kPclN, P.means, pass, h->d_xrecv, m2, h->rank, h->world,
                           h->ev_slot, hd, h->st);
    return LIO_OK;
}

// sigma and the result: order 1 the nine sigma chains sharded like the means (stage 0: from pass spass's block
// sums; stage 1: the same lists exchanged again with a larger slot), orders 2 / 3 the depth blocks; then the
// block exchange, the statuses combined, pcl_pack, and the pass's output on the host (one wait)
static int fsh_sigma_pack(lio_icp* h, int spass, int stage = 0) {
    lio::PclBuf& P = h->pcl;
    const int order = h->p.umeyama_float;
    const uint32_t* dn = P.small + lio::kPclN;
    const int64_t nq_slot = lio::pcl_blocks_slot(shard_points_max(h->ns, h->world));
    int rc = LIO_OK;
    if (order == 1) {
        const lio::SeqSigma ss = fsh_sigma_src(h);
        if (stage == 0) {
            lio::launch_pcl_mean6(P, P.means.result, h->st);
            const int64_t nbs = tot_blocks(h->ns, h->world), tw = tot_words(h->ns, h->world, 9);
            if (spass <= 1) {
                lio::seqsum_shard_head(ss, 9, dn, P.sig, h->d_xsend, nbs, h->st);
                if ((rc = xchg(h, tw))) return rc;
            }
            lio::seqsum_shard_mid(ss, 9, dn, P.sig, spass, h->d_xrecv, tw, nbs, h->rank, h->world, h->d_xsend,
                                  h->ev_slot_s, 0, h->st);
        } else {
            IHIP(hipMemsetAsync(P.sig.status + 1, 0, sizeof(uint32_t), h->st));
            lio::seqsum_shard_repack(ss, 9, dn, P.sig, h->d_xsend, h->ev_slot_s, 0, h->st);
        }
        const int64_t m = lio::seqsum_msg_words(9, h->ev_slot_s);
        if ((rc = xchg(h, m))) return rc;
        lio::seqsum_shard_tail(ss, 9, dn, P.sig, spass, h->d_xrecv, m, h->rank, h->world, h->ev_slot_s, lio::SeqHeads{},
                               h->st);
    }
    lio::launch_pcl_sigma_shard(P, order, h->d_xsend, nq_slot, h->st);
    const int64_t m3 = order == 1 ? lio::kPclX3Hdr : lio::pcl_x3_words(nq_slot);
    if ((rc = xchg(h, m3))) return rc;
    lio::launch_pcl_x3_merge(P, order, h->d_xrecv, m3, h->world, nq_slot, h->d_pclout, h->st);
    lio::launch_pcl_pack_shard(P, order, h->d_pclout, h->st);
    IHIP(hipMemcpyAsync(h->h_pclout, h->d_pclout, lio::kPclOutWords * sizeof(float), hipMemcpyDeviceToHost, h->st));
    IHIP(hipStreamSynchronize(h->st));
    return LIO_OK;
}

// the serial fallback, sharded: every window's pairs gathered on every rank (in rounds that fit the exchange
// buffers; O(source) memory for this path only), the serial chains over them
static int fsh_serial(lio_icp* h, const lio::IcpArgs& a, bool lb_timeout) {
    ++h->fid_stats[1];
    lio::PclBuf& P = h->pcl;
    lio::PclBuf& G = h->pg;
    const int order = h->p.umeyama_float;
    const uint32_t* dn = P.small + lio::kPclN;
    if (lb_timeout) {  // the window's pairs re-compacted by the serial kernel (its count lands in d_pcl16[6])
        lio::launch_icp_pcl_means_serial(a, P.pairs, P.cap, h->d_pcl16, h->st);
        dn = reinterpret_cast<const uint32_t*>(h->d_pcl16 + 6);
        IHIP(hipMemsetAsync(P.small + lio::kPclTicket + 1, 0, sizeof(uint32_t), h->st));
    }
    if (lio::pcl_reserve_plain(G, std::max<int64_t>(h->ns, 1), h->st)) return ifail(LIO_ERR_NOMEM, "lio_icp_align: fallback pairs");
    const int64_t chunk = (exchange_len(h->ns, h->world) - 2) / 3;  // the capacity every exchange offers
    const int64_t rounds = (shard_points_max(h->ns, h->world) + chunk - 1) / chunk;
    for (int64_t t = 0; t < rounds; ++t) {
        lio::launch_pcl_gather_pack(P, dn, t, chunk, h->d_xsend, h->st);
        const int rc = xchg(h, lio::pcl_gather_words(chunk));
        if (rc) return rc;
        lio::launch_pcl_gather_unpack(G, h->d_xrecv, lio::pcl_gather_words(chunk), h->world, t, chunk, h->st);
    }
    const uint32_t* gn = G.small + lio::kPclN;
    lio::launch_icp_pcl_means_pairs(G.pairs, G.cap, gn, h->d_pcl16, h->st);
    if (order == lio::kPclSeq) {
        lio::launch_icp_pcl_sigma_serial(G.pairs, G.cap, h->d_pcl16, h->st);
        IHIP(hipMemcpyAsync(h->h_pclout, h->d_pcl16, 16 * sizeof(float), hipMemcpyDeviceToHost, h->st));
    } else {
        lio::launch_pcl_sigma(G, order, 1, h->st, h->d_pcl16);
        lio::launch_pcl_pack(G, order, h->d_pclout, h->st, h->d_pcl16);
        IHIP(hipMemcpyAsync(h->h_pclout, h->d_pclout, lio::kPclOutWords * sizeof(float), hipMemcpyDeviceToHost, h->st));
    }
    IHIP(hipStreamSynchronize(h->st));
    h->h_pclout[16] = h->h_pclout[17] = 0.f;
    IHIP(hipGetLastError());
    return LIO_OK;
}

// the per-rank event slot for the next exchange: 1.5 x the longest list of this one (every rank saw the same
// lists, so every rank picks the same slot), at least 1024, at most the capacity, and never below the current
// slot (a pass-1 list is longer than a later pass's: a slot that shrank in between would make every alignment's
// first pass re-exchange)
static int next_slot(const lio_icp* h, int longest, int cur) {
    const int64_t want = ((int64_t)longest * 3 / 2 + 256 + 255) / 256 * 256;
    return (int)std::min<int64_t>(std::max<int64_t>(std::max<int64_t>(want, 1024), cur), ev_slot_cap(h->ns, h->world));
}

// pcl_finish for the sharded modes: the same re-pass policy (the statuses are every rank's, combined), plus a
// re-exchange when a list only outgrew its slot; the serial fallback gathers the pairs
static int pcl_finish_fsh(lio_icp* h, const lio::IcpArgs& a) {
    const int order = h->p.umeyama_float;
    lio::PclBuf& P = h->pcl;
    const uint32_t* dn = P.small + lio::kPclN;
    ++h->fid_stats[3];
    {
        int ev;
        std::memcpy(&ev, h->h_pclout + 18, sizeof(ev));
        h->fid_stats[2] = ev;
    }
    const bool lb_timeout = pcl_word(h, 3) != 0;
    constexpr int kMaxPasses = 4;
    int mpass = 1, spass = 1, reexchanges = 0;
    static const bool trace = std::getenv("LIO_FSH_TRACE") != nullptr;  // diagnostics: the re-pass decisions
    while (!lb_timeout) {
        const uint32_t bad = pcl_word(h, 0), over = pcl_word(h, 1), xf = pcl_word(h, 4);
        const int mm = (int)pcl_word(h, 5), ms = (int)pcl_word(h, 6);
        if (trace)
            std::fprintf(stderr, "fsh rank %d: bad %x over %x xflags %x longest %d/%d mpass %d spass %d slot %d\n", h->rank,
                         bad, over, xf, mm, ms, mpass, spass, h->ev_slot);
        h->ev_slot = next_slot(h, mm, h->ev_slot);
        if (order == 1 && ms > 0) h->ev_slot_s = next_slot(h, ms, h->ev_slot_s);
        if ((bad | over) == 0) break;
        if (bad) P.means.forced_dirty = P.sig.forced_dirty = true;
        const bool hard = (xf & (2u | 4u | 0x200u)) != 0;
        const int64_t cap = ev_slot_cap(h->ns, h->world);
        if (!hard && (xf & (1u | 0x100u)) && mm <= cap && ms <= cap && reexchanges < 2) {
            // a list longer than its slot, nothing else: the same lists again with the slot they need
            ++reexchanges;
            if (xf & 1u) {
                IHIP(hipMemsetAsync(P.means.status + 1, 0, sizeof(uint32_t), h->st));
                lio::seqsum_shard_repack(fsh_means_src(h), 6, dn, P.means, h->d_xsend, h->ev_slot, fsh_heads(h), h->st);
                int rc = fsh_means_events(h, mpass);
                if (rc) return rc;
                spass = 1;
                rc = fsh_sigma_pack(h, 1);
                if (rc) return rc;
            } else {
                const int rc = fsh_sigma_pack(h, spass, 1);
                if (rc) return rc;
            }
            continue;
        }
        if (over) break;  // a list over its capacity: more passes only add events
        if (bad & 0x3fu) {  // the means (sigma depends on them: its chains restart from pass 1)
            if (mpass >= kMaxPasses) break;
            ++mpass;
            lio::seqsum_shard_mid(fsh_means_src(h), 6, dn, P.means, mpass, nullptr, 0, 0, h->rank, h->world,
                                  h->d_xsend, h->ev_slot, fsh_heads(h), h->st);
            int rc = fsh_means_events(h, mpass);
            if (rc) return rc;
            spass = 1;
            rc = fsh_sigma_pack(h, spass);
            if (rc) return rc;
        } else {
            if (spass >= kMaxPasses) break;
            const int rc = fsh_sigma_pack(h, ++spass);
            if (rc) return rc;
        }
        ++h->fid_stats[0];
        ++h->fid_stats[3];
    }
    if (lb_timeout || (pcl_word(h, 0) | pcl_word(h, 1)) != 0) {
        if (trace) std::fprintf(stderr, "fsh rank %d: serial fallback (look-back %d)\n", h->rank, (int)lb_timeout);
        const int rc = fsh_serial(h, a, lb_timeout);
        if (rc) return rc;
    }
    IHIP(hipGetLastError());
    return LIO_OK;
}

// one correspondence pass of the sharded PCL float modes (a: this rank's shard, as icp_pass built it)
static int icp_pass_fsh(lio_icp* h, const lio::IcpArgs& a, bool apply_T, double out17[17], float* pcl16) {
    if (h->world > 64) return ifail(LIO_ERR_ARG, "lio_icp_align: the sharded float statistics take at most 64 ranks");
    int rc = exchange_reserve(h);
    if (rc) return rc;
    lio::PclBuf& P = h->pcl;
    const uint32_t* dn = P.small + lio::kPclN;
    const int64_t rec = records_count(h->ns, h->world), nbs = tot_blocks(h->ns, h->world);
    const int64_t cnt1 = rec + tot_words(h->ns, h->world, 6);
    const int64_t nsup = (h->ns + lio::kIcpSuper - 1) / lio::kIcpSuper;
    if (h->timing) IHIP(hipEventRecord(h->ev.a, h->st));
    if (h->sh_n > 0) lio::launch_icp_tiles(a, h->ntiles, h->st);
    if (h->timing) IHIP(hipEventRecord(h->ev.m, h->st));
    const lio::IcpCompact cpa = lio::pcl_compact_args(P);  // the window's pairs compacted by the same launch
    if (h->sh_n > 0) lio::launch_icp_stats(a, h->d_xsend, h->st, h->d_order, h->ntiles, &cpa);
    else IHIP(hipMemsetAsync(cpa.d_n, 0, sizeof(uint32_t), h->st));  // an empty window: no pairs
    if (h->timing) IHIP(hipEventRecord(h->ev.b, h->st));
    if (h->fid_flags & 4)  // test hook (lio_icp_set_fidelity_debug): report a look-back time-out for this pass
        IHIP(hipMemsetAsync(P.small + lio::kPclTicket + 1, 1, sizeof(uint32_t), h->st));
    lio::seqsum_shard_head(fsh_means_src(h), 6, dn, P.means, h->d_xsend + rec, nbs, h->st);
    if ((rc = xchg(h, cnt1))) return rc;
    // the records' sum in record order rides the offsets launch (lio_icp_combine's order)
    lio::SeqRecordSum rs;
    rs.recv = h->d_xrecv;
    rs.nrec = nsup;
    rs.world = h->world;
    rs.stride = cnt1;
    rs.width = lio::kIcpStride;
    rs.nval = 17;
    rs.out = h->h_out17_dev;
    lio::seqsum_shard_mid(fsh_means_src(h), 6, dn, P.means, 1, h->d_xrecv + rec, cnt1, nbs, h->rank, h->world,
                          h->d_xsend, h->ev_slot, fsh_heads(h), h->st, &rs);
    if ((rc = fsh_means_events(h, 1))) return rc;
    if ((rc = fsh_sigma_pack(h, 1))) return rc;  // waits for the pass
    IHIP(hipGetLastError());
    h->have_prior = true;
    if (h->sh_n > 0) h->have_order = true;
    if (apply_T) ++h->nT;
    if (h->timing && h->sh_n > 0) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, h->ev.a, h->ev.b) == hipSuccess) {
            h->tm.icp_ms += ms;
            ++h->tm.icp_launches;
        }
        if (hipEventElapsedTime(&ms, h->ev.a, h->ev.m) == hipSuccess) {
            h->tm.icp_nn_ms += ms;
            ++h->tm.icp_nn_launches;
        }
    }
    std::memcpy(out17, h->h_out17, 17 * sizeof(double));
    if ((rc = pcl_finish_fsh(h, a))) return rc;
    std::memcpy(pcl16, h->h_pclout, 16 * sizeof(float));
    return LIO_OK;
}

// One correspondence (or fitness) pass: GPU kernels + exchange + ordered sum.
static int icp_pass(lio_icp* h, bool fitness, bool apply_T, const float* T, double max_d2, double out17[17],
                    float* pcl16 = nullptr) {
    lio::IcpArgs a{};
    a.grid = lio::grid_view(h->tgt);
    a.tgt_by_id = h->tgt.by_id;
    a.cur = h->d_cur;
    a.src = h->d_src;
    a.thist = h->d_thist;
    a.nT = h->nT;
    if (!fitness && apply_T && h->nT >= h->thist_cap) return ifail(LIO_ERR_STATE, "lio_icp_align: transform history full");
    a.n = (int)h->sh_n;
    a.apply_T = apply_T ? 1 : 0;
    std::memcpy(a.T, T, sizeof(a.T));
    std::memcpy(a.c0, h->c0, sizeof(a.c0));
    a.max_d2 = max_d2;
    a.fitness = fitness ? 1 : 0;
    a.prior = h->have_prior ? 1 : 0;
    // first bound box: the tile's own cells (r0 = 0; with the per-batch bound and the centre-out rows, pair A
    // 0.221 -> 0.212 ms per alignment against r0 = 1, pair B unchanged: profiles/r05_icp_r0_ab.txt)
    a.r0 = 0;
    a.nn_d2 = h->d_fd2;
    a.nn_id = h->d_fid;
    a.qpts = h->qgrid.pts;
    a.tiles = h->d_tiles;
    a.tile_cost = h->d_tcost;
    a.order = h->have_order ? h->d_order : nullptr;
#ifdef LIO_DIAG
    static const bool dbg_on = std::getenv("LIO_ICP_DEBUG") != nullptr;  // diagnostics build: search statistics
    if (dbg_on) {
        // 8 counters + (start, end) wall clock per tile + (growth candidates, final candidates, final rows, rounds)
        const size_t bytes = (8 + 6 * (size_t)std::max(h->ntiles, 1)) * sizeof(unsigned long long);
        if (h->d_dbg && h->dbg_bytes < bytes) {
            IHIP(hipFree(h->d_dbg));
            h->d_dbg = nullptr;
        }
        if (!h->d_dbg) {
            IHIP(hipMalloc(&h->d_dbg, bytes));
            h->dbg_bytes = bytes;
        }
        IHIP(hipMemsetAsync(h->d_dbg, 0, bytes, h->st));
        a.dbg = h->d_dbg;
    }
#endif
    const int nsup_loc = (int)((h->sh_n + lio::kIcpSuper - 1) / lio::kIcpSuper);
    const bool dev_x = h->world > 1 && h->fn_dev;  // device-side exchange: records stay on the device
    // the sharded PCL float modes' correspondence passes: icp_pass_fsh (the chains split over the ranks' windows)
    if (pcl16 && fid_sharded(h) && !fitness) return icp_pass_fsh(h, a, apply_T, out17, pcl16);
    const int64_t cnt = records_count(h->ns, h->world);  // doubles per rank this pass
    if (dev_x) {
        const int rc = exchange_reserve(h);
        if (rc) return rc;
    }
    if (h->sh_n > 0 || dev_x) {
        if (h->timing) IHIP(hipEventRecord(h->ev.a, h->st));
        if (h->sh_n > 0) lio::launch_icp_tiles(a, h->ntiles, h->st);
        if (h->timing) IHIP(hipEventRecord(h->ev.m, h->st));
        // the PCL float modes: the accepted pairs compacted by the same launch (one rank: the whole source)
        lio::IcpCompact cpa;
        if (pcl16 && !fitness) cpa = lio::pcl_compact_args(h->pcl);
        const lio::IcpCompact* cp = pcl16 && !fitness ? &cpa : nullptr;
        if (dev_x) {  // records -> device send buffer -> in-stream all-gather -> record-order sum
            if (h->sh_n > 0) lio::launch_icp_stats(a, h->d_xsend, h->st, fitness ? nullptr : h->d_order, h->ntiles, cp);
            IHIP(hipGetLastError());
            if (h->fn_dev(h->d_xsend, cnt, h->d_xrecv, (void*)h->st, h->user_dev) != 0)
                return ifail(LIO_ERR_STATE, "device all-gather callback failed");
            const int64_t nsup = (h->ns + lio::kIcpSuper - 1) / lio::kIcpSuper;
            lio::launch_icp_combine(h->d_xrecv, nsup, h->world, cnt, h->h_out17_dev, h->st);
        } else if (h->sh_n > 0) {
            // records straight to host memory; the next pass's tile order in the same launch
            lio::launch_icp_stats(a, h->h_super_dev, h->st, fitness ? nullptr : h->d_order, h->ntiles, cp);
        }
        if (cp && h->sh_n == 0) IHIP(hipMemsetAsync(cp->d_n, 0, sizeof(uint32_t), h->st));  // no pairs
        if (h->timing) IHIP(hipEventRecord(h->ev.b, h->st));
        if (pcl16) {  // one rank: the float statistics of its correspondences
            const int rc = enqueue_pcl(h, a);
            if (rc) return rc;
        }
        IHIP(hipGetLastError());
        if (pcl16 && !h->timing) {  // the pack's sequence number (it is the pass's last launch)
            const int rc = pcl_wait(h, h->pcl_seq);
            if (rc) return rc;
        } else {
            IHIP(hipEventRecord(h->ev.done, h->st));
            IHIP(hipEventSynchronize(h->ev.done));
        }
    } else {
        IHIP(hipStreamSynchronize(h->st));
    }
    h->have_prior = true;
    if (!fitness && h->sh_n > 0) h->have_order = true;
    if (!fitness && apply_T) ++h->nT;
#ifdef LIO_DIAG
    if (dbg_on) {
        unsigned long long c[5];
        IHIP(hipMemcpy(c, h->d_dbg, sizeof(c), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "icp dbg: tiles|waves %llu lanes %llu cand/tile %.1f tested/tile %.1f rounds/tile %.2f cand/lane %.1f\n",
                     c[2], c[3], (double)c[0] / c[2], (double)c[4] / c[2], (double)c[1] / c[2], (double)c[0] / c[3]);
        // per-tile timeline (wall clock, 100 MHz): span, duration percentiles, the tail
        std::vector<unsigned long long> tt(2 * (size_t)h->ntiles);
        std::vector<uint32_t> cost(h->ntiles);
        IHIP(hipMemcpy(tt.data(), h->d_dbg + 8, tt.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        IHIP(hipMemcpy(cost.data(), h->d_tcost, cost.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0;
        std::vector<double> dur(h->ntiles);
        int imax = 0;
        for (int t = 0; t < h->ntiles; ++t) {
            t0 = std::min(t0, tt[2 * t]);
            t1 = std::max(t1, tt[2 * t + 1]);
            dur[t] = (double)(tt[2 * t + 1] - tt[2 * t]) * 0.01;  // us
            if (dur[t] > dur[imax]) imax = t;
        }
        unsigned long long last_start = 0;
        int late = 0;
        for (int t = 0; t < h->ntiles; ++t) {
            last_start = std::max(last_start, tt[2 * t]);
            if (tt[2 * t] > t0 + (t1 - t0) / 2) ++late;
        }
        std::vector<double> sd = dur;
        std::sort(sd.begin(), sd.end());
        auto pct = [&](double q) { return sd[std::min(sd.size() - 1, (size_t)(q * (double)sd.size()))]; };
        std::fprintf(stderr,
                     "icp tiles: span %.1f us | tile us p50 %.2f p90 %.2f p99 %.2f max %.2f (cost %u, median cost %u) | "
                     "last tile starts at %.1f us | tiles starting in the second half %d of %d\n",
                     (double)(t1 - t0) * 0.01, pct(0.5), pct(0.9), pct(0.99), sd.back(), cost[imax],
                     [&] { std::vector<uint32_t> c2 = cost; std::nth_element(c2.begin(), c2.begin() + c2.size() / 2, c2.end()); return c2[c2.size() / 2]; }(),
                     (double)(last_start - t0) * 0.01, late, h->ntiles);
        // the slowest tiles' search: candidates streamed while growing / in the final round, final rows, rounds
        std::vector<unsigned long long> ex(4 * (size_t)h->ntiles);
        IHIP(hipMemcpy(ex.data(), h->d_dbg + 8 + 2 * (size_t)h->ntiles, ex.size() * sizeof(unsigned long long),
                       hipMemcpyDeviceToHost));
        std::vector<int> idx(h->ntiles);
        for (int t = 0; t < h->ntiles; ++t) idx[t] = t;
        const int nshow = std::min(5, h->ntiles);
        std::partial_sort(idx.begin(), idx.begin() + nshow, idx.end(), [&](int u, int v) { return dur[u] > dur[v]; });
        for (int k = 0; k < nshow; ++k) {
            const int t = idx[k];
            std::fprintf(stderr, "  slow tile %d: %.1f us, starts %.1f us, growth cand %llu, final cand %llu, final rows %llu, rounds %llu, cost %u\n",
                         t, dur[t], (double)(tt[2 * t] - t0) * 0.01, ex[4 * t], ex[4 * t + 1], ex[4 * t + 2], ex[4 * t + 3], cost[t]);
        }
    }
#endif
    if (h->timing && h->sh_n > 0) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, h->ev.a, h->ev.b) == hipSuccess) {
            h->tm.icp_ms += ms;
            ++h->tm.icp_launches;
        }
        if (hipEventElapsedTime(&ms, h->ev.a, h->ev.m) == hipSuccess) {
            h->tm.icp_nn_ms += ms;
            ++h->tm.icp_nn_launches;
        }
    }
    if (!dev_x && h->world > 1) {
        // host exchange: fixed-size slots (max records per rank), summed in global record order
        std::vector<double> send((size_t)cnt, 0.0), recv((size_t)cnt * h->world);
        std::memcpy(send.data(), h->h_super, (size_t)nsup_loc * lio::kIcpStride * sizeof(double));
        if (h->fn(send.data(), cnt, recv.data(), h->user) != 0) return ifail(LIO_ERR_STATE, "allgather callback failed");
        combine_records(recv.data(), h->ns, h->world, cnt, out17);
    } else if (dev_x) {  // the record-order sums of every rank's records, computed on the device
        std::memcpy(out17, h->h_out17, 17 * sizeof(double));
    } else {
        for (int k = 0; k < 17; ++k) out17[k] = 0.0;
        for (int s = 0; s < nsup_loc; ++s)
            for (int k = 0; k < 17; ++k) out17[k] += h->h_super[(size_t)s * lio::kIcpStride + k];
    }
    if (pcl16) {
        const int rc = pcl_finish(h, a);
        if (rc) return rc;
        std::memcpy(pcl16, h->h_pclout, 16 * sizeof(float));
    }
    return LIO_OK;
}

extern "C" int64_t lio_alloc_count(void) { return lio::alloc_counter().load(std::memory_order_relaxed); }

extern "C" int lio_icp_shard_range(int64_t ns, int rank, int world, int64_t* begin, int64_t* count) {
    if (ns < 0 || world < 1 || rank < 0 || rank >= world || !begin || !count)
        return ifail(LIO_ERR_ARG, "lio_icp_shard_range: bad arguments");
    shard_range(ns, rank, world, *begin, *count);
    return LIO_OK;
}

extern "C" int lio_icp_umeyama_pcl_float(const float* sums16, float* T16) {
    if (!sums16 || !T16) return ifail(LIO_ERR_ARG, "lio_icp_umeyama_pcl_float: bad arguments");
    umeyama_pcl_float(sums16, T16);
    return LIO_OK;
}

extern "C" int lio_icp_umeyama_pcl_float_order(const float* sums16, int order, float* T16) {
    if (!sums16 || !T16 || order < 1 || order > 3) return ifail(LIO_ERR_ARG, "lio_icp_umeyama_pcl_float_order: bad arguments");
    umeyama_pcl_float(sums16, T16, order);
    return LIO_OK;
}

extern "C" int lio_icp_get_fidelity_stats(lio_icp* h, int64_t* out4) {
    if (!h || !out4) return ifail(LIO_ERR_ARG, "lio_icp_get_fidelity_stats: bad arguments");
    icp_join(h);
    std::memcpy(out4, h->fid_stats, sizeof(h->fid_stats));
    return LIO_OK;
}

extern "C" int lio_icp_set_fidelity_debug(lio_icp* h, int flags, int64_t evcap) {
    if (!h || evcap < 0) return ifail(LIO_ERR_ARG, "lio_icp_set_fidelity_debug: bad arguments");
    icp_join(h);
    h->fid_flags = flags;
    h->fid_evcap = evcap;
    return LIO_OK;
}

// test hook: the seqsum path on 6 interleaved chains, re-passes as in pcl_finish; -1 passes: serial needed
extern "C" int lio_seqsum6(int device, const float* x, int64_t n, int flags, float* sums6, int* passes_out) {
    if (!x || n < 1 || !sums6 || n >= ((int64_t)1 << 31)) return ifail(LIO_ERR_ARG, "lio_seqsum6: bad arguments");
    int rc = icp_check_dev(device);
    if (rc) return rc;
    IHIP(hipSetDevice(device));
    hipStream_t st;
    IHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    lio::SeqSumBuf b;
    b.dbg_noinc = flags & 1;
    float* d_x = nullptr;
    uint32_t* d_n = nullptr;
    uint32_t stat[2] = {0, 0};
    int passes = 0;
    const uint32_t n32 = (uint32_t)n;
    auto done = [&](int code, const char* msg) {
        lio::seqsum_free(b);
        if (d_x) (void)hipFree(d_x);
        if (d_n) (void)hipFree(d_n);
        (void)hipStreamDestroy(st);
        return code ? ifail(code, msg) : LIO_OK;
    };
    if (lio::seqsum_reserve(b, 6, n, st) || hipMalloc(&d_x, (size_t)n * 6 * sizeof(float)) != hipSuccess ||
        hipMalloc(&d_n, sizeof(uint32_t)) != hipSuccess)
        return done(LIO_ERR_NOMEM, "lio_seqsum6: allocation");
    if (flags & 2) b.evcap = std::min<int64_t>(4, b.evcap_alloc);  // overflow: the caller's serial fallback
    if (hipMemcpyAsync(d_x, x, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_n, &n32, sizeof(n32), hipMemcpyHostToDevice, st) != hipSuccess)
        return done(LIO_ERR_HIP, "lio_seqsum6: upload");
    for (int pass = 1; pass <= 3; ++pass) {
        lio::seqsum_launch(lio::SeqPairs{d_x}, 6, d_n, b, pass, st);
        if (hipMemcpyAsync(stat, b.status, sizeof(stat), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(sums6, b.result, 6 * sizeof(float), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return done(LIO_ERR_HIP, "lio_seqsum6: kernels");
        passes = pass;
        if ((stat[0] | stat[1]) == 0 || stat[1]) break;
    }
    if (passes_out) *passes_out = (stat[0] | stat[1]) ? -1 : passes;
    return done(LIO_OK, "");
}

// host mirrors of the sharded float chains' exchange logic (the device kernels run the same seq_shard_* helpers,
// lio_seqsum.hpp): the gathered totals -> one window's offsets; the gathered event messages -> one chain's global
// event lists.  tests/test_dist_gloo.py drives them with messages all-gathered over gloo.
extern "C" int lio_seq_shard_offsets(const double* recv, int64_t stride, int64_t nb_slot, int rank, int world, int nch,
                                     double* off0, double* var0, int32_t* floor_e, int64_t* gbase_nglobal) {
    if (!recv || !off0 || !var0 || !floor_e || !gbase_nglobal || world < 1 || rank < 0 || rank >= world || nch < 1 ||
        nch > lio::kSeqMaxChains || nb_slot < 1 || stride < lio::seq_tot_words(nch, nb_slot))
        return ifail(LIO_ERR_ARG, "lio_seq_shard_offsets: bad arguments");
    for (int c = 0; c < nch; ++c) {
        int fl;
        lio::seq_shard_offsets_chain(recv, stride, nb_slot, rank, world, c, off0[c], var0[c], fl, gbase_nglobal[0],
                                     gbase_nglobal[1]);
        floor_e[c] = fl;
    }
    return LIO_OK;
}

extern "C" int lio_seq_shard_merge(const double* recv, int64_t stride, int world, int slot, int chain, int64_t evs,
                                   int32_t* pos, uint64_t* P, float* x, int32_t* nev_ptot_bad, uint64_t* ptot, float* x0) {
    if (!recv || !pos || !P || !x || !nev_ptot_bad || !ptot || !x0 || world < 1 || world > 64 || slot < 0 || chain < 0 ||
        chain >= lio::kSeqMaxChains || stride < lio::seqsum_msg_words(chain + 1, slot))
        return ifail(LIO_ERR_ARG, "lio_seq_shard_merge: bad arguments");
    int eoff[65];
    uint64_t poff[65];
    int64_t ppos[65];
    int mx = 0;
    const int bad = lio::seq_shard_merge_chain(recv, stride, world, slot, chain, evs, eoff, poff, ppos, *x0, mx);
    nev_ptot_bad[0] = eoff[world];
    nev_ptot_bad[1] = mx;
    nev_ptot_bad[2] = bad;
    *ptot = poff[world];
    if (bad) return LIO_OK;
    for (int r = 0; r < world; ++r) {  // seq_shard_merge's copy: every rank's events moved by the ranks before it
        const double* ev = recv + (int64_t)r * stride + lio::kSeqHdrWords + (int64_t)chain * 2 * slot;
        for (int j = 0; j < eoff[r + 1] - eoff[r]; ++j) {
            const uint64_t w = (uint64_t)lio::seq_bits(ev[2 * j + 1]);
            P[eoff[r] + j] = poff[r] + (uint64_t)lio::seq_bits(ev[2 * j]);
            pos[eoff[r] + j] = (int32_t)(ppos[r] + (int64_t)(uint32_t)w);
            uint32_t xb = (uint32_t)(w >> 32);
            std::memcpy(&x[eoff[r] + j], &xb, sizeof(float));
        }
    }
    return LIO_OK;
}

extern "C" int lio_icp_combine(const double* recv, int64_t ns, int world, double* out17) {
    if (!recv || !out17 || world < 1 || ns < 0) return ifail(LIO_ERR_ARG, "lio_icp_combine: bad arguments");
    combine_records(recv, ns, world, records_count(ns, world), out17);
    return LIO_OK;
}

int lio_icp_align(lio_icp* h, const float* guess16, lio_icp_result* out, float* aligned) {
    if (!h || !out) return ifail(LIO_ERR_ARG, "lio_icp_align: bad arguments");
    icp_join(h);
    if (h->nt == 0) return ifail(LIO_ERR_STATE, "lio_icp_align: no target");
    IHIP(hipSetDevice(h->dev));
    const bool pcl_float = h->p.umeyama_float > 0;  // (normalised at create: 0 = the double statistics)
    // the target (st2, helper thread) and the source (st, this thread) prepared side by side
    int rc = LIO_OK, trc = LIO_OK;
    std::string terr;
    std::thread tth;
    if (h->tgt_dirty) {
        auto job = [&] {
            trc = target_build(h);
            if (trc) terr = lio::last_error();
        };
        try {
            tth = std::thread(job);
        } catch (...) {
            job();
        }
    }
    rc = icp_prepare(h);
    if (tth.joinable()) tth.join();
    // a set-up that failed in the background and again here: both reasons
    if (trc) return ifail(trc, terr + (h->bg_tgt_err.empty() ? "" : " (setInputTarget: " + h->bg_tgt_err + ")"));
    if (rc) return ifail(rc, lio::last_error() + (h->bg_src_err.empty() ? "" : " (setInputSource: " + h->bg_src_err + ")"));
    h->bg_tgt_err.clear();
    h->bg_src_err.clear();
    if (pcl_float) {
        // the window's pairs (sharded: + the kPclMaxKc pairs of the ranks after it, for the depth blocks that
        // start in the window and end in the next)
        const bool fsh = fid_sharded(h);
        lio::PclBuf& P = h->pcl;
        if (lio::pcl_reserve(P, std::max<int64_t>(h->sh_n + (fsh ? lio::kPclMaxKc : 0), kIcpCapFloor), h->p.umeyama_float, h->st))
            return ifail(LIO_ERR_NOMEM, "lio_icp_align: fidelity buffers");
        P.means.dbg_noinc = P.sig.dbg_noinc = h->fid_flags & 1;
        P.n_hint = fsh ? 0 : h->sh_n;  // one rank: the accepted pairs are a subset of the source
        for (lio::SeqSumBuf* b : {&P.means, &P.sig})
            b->evcap = h->fid_evcap > 0 ? std::min(h->fid_evcap, b->evcap_alloc) : b->evcap_alloc;
        P.mean6 = reinterpret_cast<float*>(P.small + lio::kPclMean6);
        if (lio::seqsum_shard(P.means, fsh, h->st) ||
            (h->p.umeyama_float == lio::kPclSeq && lio::seqsum_shard(P.sig, fsh, h->st)) ||
            (fsh && lio::pcl_shard_reserve(P, h->ns / 340 + 4, h->st)))
            return ifail(LIO_ERR_NOMEM, "lio_icp_align: sharded fidelity buffers");
        P.n_all = fsh ? reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(P.means.sh) +
                                                          offsetof(lio::SeqShard, n32))
                      : nullptr;
        if (fsh) {
            const int cap = (int)ev_slot_cap(h->ns, h->world);
            h->ev_slot = std::min(h->ev_slot, cap);
            h->ev_slot_s = std::min(h->ev_slot_s, cap);
        }
        if (!h->d_pcl16) IHIP(hipMalloc(&h->d_pcl16, 16 * sizeof(float)));
        if (!h->d_pclout) IHIP(hipMalloc(&h->d_pclout, 32 * sizeof(float)));
        if (!h->h_pclout) {
            IHIP(hipHostMalloc(&h->h_pclout, 32 * sizeof(float), hipHostMallocMapped));
            IHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_pclout_dev), h->h_pclout, 0));
        }
    }
    float fin[16], G[16];
    bool ident = true;
    for (int i = 0; i < 16; ++i) {
        G[i] = guess16 ? guess16[i] : ((i % 5 == 0) ? 1.f : 0.f);
        fin[i] = G[i];
        if (G[i] != ((i % 5 == 0) ? 1.f : 0.f)) ident = false;
    }
    if (h->sh_n > 0)
        IHIP(hipMemcpyAsync(h->d_cur, h->d_src, h->sh_n * 3 * sizeof(float), hipMemcpyDeviceToDevice, h->st));
    const int hist_need = std::max(h->p.max_iter, 1) + 4;  // one T per iteration plus the guess
    if (hist_need > h->thist_cap) {
        if (h->d_thist) IHIP(hipFree(h->d_thist));
        h->d_thist = nullptr;
        h->thist_cap = 0;
        IHIP(hipMalloc(&h->d_thist, (size_t)hist_need * 16 * sizeof(float)));
        h->thist_cap = hist_need;
    }
    h->nT = 0;
    h->have_prior = false;
    h->have_order = false;  // every alignment starts in cell order (its first pass measures the tiles)
    const double max_d2 = h->p.max_corr_dist * h->p.max_corr_dist;
    const double rot_thr = h->p.rot_eps > 0 ? h->p.rot_eps : 1.0 - h->p.trans_eps;
    double prev_mse = std::numeric_limits<double>::max();
    int iters = 0, similar = 0;
    bool apply = !ident;
    float Tapply[16];
    std::memcpy(Tapply, G, sizeof(G));
    std::memset(out, 0, sizeof(*out));
    out->state = 0;
    out->is_converged = 0;
    for (;;) {
        double st[17];
        float pcl16[16];
        rc = icp_pass(h, false, apply, Tapply, max_d2, st, pcl_float ? pcl16 : nullptr);
        if (rc) return rc;
        out->last_corr = (int64_t)st[0];
        if (st[0] < 3) {
            out->is_converged = 0;
            out->state = 5;
            break;
        }
        float Ti[16];
        if (pcl_float)
            umeyama_pcl_float(pcl16, Ti, h->p.umeyama_float);
        else
            umeyama(st, h->c0, Ti);
        float nf[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                float s = Ti[4 * r] * fin[c];
                s += Ti[4 * r + 1] * fin[4 + c];
                s += Ti[4 * r + 2] * fin[8 + c];
                s += Ti[4 * r + 3] * fin[12 + c];
                nf[4 * r + c] = s;
            }
        std::memcpy(fin, nf, sizeof(fin));
        ++iters;
        const double mse = st[16] / st[0];
        out->last_mse = mse;
        // DefaultConvergenceCriteria (max_iterations_similar_transforms_ = 0)
        bool done = false, is_similar = false;
        if (iters >= h->p.max_iter) {
            out->state = 1;
            done = true;
        } else {
            // PCL 1.10 DefaultConvergenceCriteria<float>: the coefficients of the Matrix4f are summed and
            // squared in float, then widened (0.5 * float -> double; float -> double translation_sqr)
            const float tr_f = Ti[0] + Ti[5] + Ti[10] - 1.f;
            const float tsq_f = Ti[3] * Ti[3] + Ti[7] * Ti[7] + Ti[11] * Ti[11];
            const double cosang = 0.5 * (double)tr_f;
            const double tsq = (double)tsq_f;
            if (cosang >= rot_thr && tsq <= h->p.trans_eps) {
                out->state = 2;
                done = true;
                is_similar = true;
            }
            if (!done && std::fabs(mse - prev_mse) < 1e-12) {
                out->state = 3;
                done = true;
            }
            if (!done && std::fabs(mse - prev_mse) / prev_mse < h->p.fitness_eps) {
                out->state = 4;
                done = true;
            }
            if (!done) {
                similar = is_similar ? similar + 1 : 0;
                prev_mse = mse;
            }
        }
        std::memcpy(Tapply, Ti, sizeof(Ti));
        apply = true;
        if (done) {
            out->is_converged = 1;
            break;
        }
    }
    (void)similar;
    out->iterations = iters;
    std::memcpy(out->T, fin, sizeof(fin));
    // getFitnessScore(): original source * final, unbounded 1-NN
    double fs[17];
    rc = icp_pass(h, true, true, fin, std::numeric_limits<double>::infinity(), fs);
    if (rc) return rc;
    out->score = fs[0] > 0 ? fs[16] / fs[0] : std::numeric_limits<double>::max();
    out->is_valid = (out->is_converged && out->score < h->p.score_threshold) ? 1 : 0;
    if (aligned && h->sh_n > 0) {
        IHIP(hipMemcpyAsync(aligned, h->d_cur, h->sh_n * 3 * sizeof(float), hipMemcpyDeviceToHost, h->st));
        IHIP(hipStreamSynchronize(h->st));
    }
    return LIO_OK;
}

int icp_align(const float* src, int64_t ns, const float* dst, int64_t nd, const lio_icp_params* p, int n_gpus,
              float* T_out, double* fitness, int* converged, int* iters, float* aligned) {
    if (!p) return ifail(LIO_ERR_ARG, "icp_align: NULL params");
    // n_gpus > 1: devices p->device .. p->device + n_gpus - 1, source sharded, records all-gathered over
    // RCCL (lio_icp_group); n_gpus <= 1: one handle on p->device
    const int ng = n_gpus > 1 ? n_gpus : 1;
    std::vector<int> devs(ng);
    for (int r = 0; r < ng; ++r) devs[r] = p->device + r;
    lio_icp_group* g = nullptr;
    int rc = lio_icp_group_create(p, ng, devs.data(), &g);
    if (rc) return rc;
    rc = lio_icp_group_set_target(g, dst, nd);
    if (!rc) rc = lio_icp_group_set_source(g, src, ns);
    lio_icp_result r{};
    if (!rc) rc = lio_icp_group_align(g, nullptr, &r, aligned);
    if (!rc) {
        if (T_out) std::memcpy(T_out, r.T, sizeof(r.T));
        if (fitness) *fitness = r.score;
        if (converged) *converged = r.is_converged;
        if (iters) *iters = r.iterations;
    }
    lio_icp_group_destroy(g);
    return rc;
}

int lio_icp_get_correspondences(lio_icp* h, int32_t* ids, float* d2) {
    if (!h || !ids || !d2) return ifail(LIO_ERR_ARG, "bad arguments");
    icp_join(h);
    if (!h->have_prior) return ifail(LIO_ERR_STATE, "lio_icp_get_correspondences: no pass run yet");
    IHIP(hipSetDevice(h->dev));
    if (h->sh_n > 0) {
        IHIP(hipMemcpyAsync(ids, h->d_fid, h->sh_n * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
        IHIP(hipMemcpyAsync(d2, h->d_fd2, h->sh_n * sizeof(float), hipMemcpyDeviceToHost, h->st));
        IHIP(hipStreamSynchronize(h->st));
    }
    return LIO_OK;
}

int lio_icp_set_timing(lio_icp* h, int enable) {
    if (!h) return ifail(LIO_ERR_ARG, "NULL handle");
    icp_join(h);
    h->timing = enable != 0;
    return LIO_OK;
}
int lio_icp_get_timing(lio_icp* h, lio_kernel_timing* out) {
    if (!h || !out) return ifail(LIO_ERR_ARG, "bad arguments");
    icp_join(h);
    *out = h->tm;
    return LIO_OK;
}

}  // extern "C"
