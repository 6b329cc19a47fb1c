// lio_capi.cpp — the C-ABI (include/lio_gpu.h): handles, streams, device
// buffers, and the host drivers (IESKF update, PCL-semantics ICP loop).
// There is deliberately no CPU compute path: every compute entry point runs
// the gfx950 kernels or fails with LIO_ERR_NODEV / LIO_ERR_HIP.
#include "../../include/lio_gpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "ieskf.hpp"
#include "lio_error.hpp"
#include "lio_kernels.hpp"
#include "lio_filter.hpp"
#include "lio_pool.hpp"
#include "lio_mapupd.hpp"

namespace {

int fail(int code, const std::string& msg) {
    lio::last_error() = msg;
    return code;
}

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return fail(LIO_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(LIO_ERR_NODEV, "no HIP device visible (this library has no CPU path)");
    if (dev < 0 || dev >= n) return fail(LIO_ERR_ARG, "device ordinal out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(LIO_ERR_HIP, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(LIO_ERR_NODEV, std::string("built for gfx950, device is ") + prop.gcnArchName);
    return LIO_OK;
}

template <class T>
int grow(T** p, int64_t& cap, int64_t need, size_t elems_per = 1) {
    if (need <= cap && *p) return LIO_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    int64_t c = std::max<int64_t>(need, cap + cap / 2);
    lio::count_alloc();
    if (hipMalloc(p, (size_t)c * elems_per * sizeof(T)) != hipSuccess) {
        cap = 0;
        return fail(LIO_ERR_NOMEM, "hipMalloc failed");
    }
    cap = c;
    return LIO_OK;
}

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};

// Eigen 3.3 quaternionbase_assign_impl<Other,3,3>::run (Geometry/Quaternion.h): rotation matrix ->
// quaternion (w, x, y, z), trace = m00 + (m11 + m22).  Only for callers that hand over matrices
// without the state quaternion (lio_pose.q all zero); the oracle derives it the same way.
void mat_to_quat(const double* m, double* q) {
    auto M = [&](int r, int c) { return m[3 * r + c]; };
    double t = M(0, 0) + (M(1, 1) + M(2, 2));
    double c[4];  // x, y, z, w
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        c[3] = 0.5 * t;
        t = 0.5 / t;
        c[0] = (M(2, 1) - M(1, 2)) * t;
        c[1] = (M(0, 2) - M(2, 0)) * t;
        c[2] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        c[3] = (M(k, j) - M(j, k)) * t;
        c[j] = (M(j, i) + M(i, j)) * t;
        c[k] = (M(k, i) + M(i, k)) * t;
    }
    q[0] = c[3], q[1] = c[0], q[2] = c[1], q[3] = c[2];
}

bool quat_zero(const double* q) { return q[0] == 0.0 && q[1] == 0.0 && q[2] == 0.0 && q[3] == 0.0; }

// The quaternions take precedence over R / R_LI (include/lio_gpu.h lio_pose): the kernels rotate with
// q / q_LI; a caller that fills only the matrices gets q derived from them.
lio_pose filled(const lio_pose& p) {
    lio_pose o = p;
    if (quat_zero(o.q)) mat_to_quat(o.R, o.q);
    if (quat_zero(o.q_LI)) mat_to_quat(o.R_LI, o.q_LI);
    return o;
}

// Eigen QuaternionBase::toRotationMatrix (q = w, x, y, z; any norm is used as given)
void quat_to_mat(const double* q, double* R) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz), R[1] = txy - twz, R[2] = txz + twy;
    R[3] = txy + twz, R[4] = 1 - (txx + tzz), R[5] = tyz - twx;
    R[6] = txz - twy, R[7] = tyz + twx, R[8] = 1 - (txx + tyy);
}

}  // namespace

// =============================================================================
// map
// =============================================================================
struct lio_map {
    uint64_t version = 0;  // bumped by every change of the point set (seeded kNN validity)
    std::atomic<int> n_ctx{0};  // live lio_ctx handles on this map (destroy refuses while > 0)
    int dev = 0;
    hipStream_t st = nullptr;
    lio_map_params p{};
    lio::GridBuf grid;
    lio::MapUpdBuf upd;
    float* d_xyz = nullptr;
    int64_t xyz_cap = 0;
    int64_t n = 0;  // alive points (== grid.n)
    int32_t* d_qidx = nullptr;  // lio_map_nearest_search results
    int64_t qidx_cap = 0;
    float* d_qd2 = nullptr;
    int64_t qd2_cap = 0;
};

// geometry slack when an insert leaves the grid: the rebuild reserves room
// around the map (half a local-map cube of travel at the usual 1 m cells)
static float map_slack(const lio_map* m) { return 64.f * m->grid.geom.cell; }

struct lio_ctx {
    lio_map* map = nullptr;
    double last_launch_ms = 0.0, last_wait_ms = 0.0;  // host side of the last lio_match
    lio_match_params p{};
    int64_t n = 0, cap = 0;
    float* d_body = nullptr;
    const float* body_ext = nullptr;  // lio_scan_bind_device: caller-owned scan (no copy)
    int32_t* d_nn = nullptr;
    float4* d_planes = nullptr;
    uint8_t* d_sel = nullptr;
    double* d_partials = nullptr;
    int64_t part_cap = 0;
    double* d_sums = nullptr;
    double* h_sums = nullptr;    // pinned, host-mapped: [0,32) sums, [32] sequence number, [33] checksum
    double* h_sums_dev = nullptr;  // device view of h_sums
    unsigned long long seq = 0;
    double* d_rows = nullptr;
    int64_t rows_cap = 0;
    int64_t* d_nrows = nullptr;
    lio_pose last_pose{};
    lio_pose knn_pose{};  // pose of the last kNN evaluation (Nearest_Points)
    int* d_far_list = nullptr;  // far-pass queue (cap), its length, and queued lists (cap*5)
    int* d_far_count = nullptr;
    unsigned* d_done = nullptr;  // plane/reuse block counter (last block publishes)
    float* d_far_d = nullptr;
    int* d_far_id = nullptr;
    float* d_d5 = nullptr;  // per point: 5th neighbour d2 of the last kNN (seeds the next one)
    bool have_eval = false;
    bool knn_valid = false;
    uint64_t knn_map_version = 0;  // map version of the last kNN evaluation
    // timing
    bool timing = false;
    lio_kernel_timing tm{};
    EventPair ev_main, ev_fin;
    hipEvent_t ev_marks[8] = {};  // kernel start / stop: near, far, plane, reuse (hipExtLaunchKernel)
    lio::FilterBuf filt;                          // scan preprocessing
    float* d_raw = nullptr;                       // raw records / preprocessed records
    int64_t raw_cap = 0;
    float* d_rec = nullptr;
    int64_t rec_cap = 0;
    lio::ImuPose* d_poses = nullptr;
    int64_t poses_cap = 0;
    float seed_scale = 1.0f;  // lio_ctx_set_seed_scale (test hook: < 1 exercises the seeded pass's guard)
    int64_t undist_n = -1;    // feats_undistort of the last lio_scan_preprocess* (records in filt.c); -1: none
    int undist_stride = 0;
    float* d_kf = nullptr;    // lio_scan_keyframe_cloud output (n x 4)
    int64_t kf_cap = 0;
};

extern "C" {

int lio_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* lio_last_error(void) { return lio::last_error().c_str(); }

const char* lio_build_info(void) {
    return "lio_gpu: gfx950 HIP kernels (grid kNN + esti_plane + H^T H reduction, ICP); -ffp-contract=off";
}

int lio_abi_struct_sizes(int64_t* out, int n) {
    const int64_t sz[] = {(int64_t)sizeof(lio_map_params),   (int64_t)sizeof(lio_match_params),
                          (int64_t)sizeof(lio_pose),         (int64_t)sizeof(lio_state),
                          (int64_t)sizeof(lio_ieskf_params), (int64_t)sizeof(lio_ieskf_stats),
                          (int64_t)sizeof(lio_icp_params),   (int64_t)sizeof(lio_icp_result),
                          (int64_t)sizeof(lio_localmap),     (int64_t)sizeof(lio_incremental_stats),
                          (int64_t)sizeof(lio_imu_pose),     (int64_t)sizeof(lio_scan_prep_params),
                          (int64_t)sizeof(lio_cloud_field),  (int64_t)sizeof(lio_kernel_timing)};
    constexpr int kN = (int)(sizeof(sz) / sizeof(sz[0]));
    if (out)
        for (int i = 0; i < n && i < kN; ++i) out[i] = sz[i];
    return kN;
}

int lio_map_create(const lio_map_params* p, lio_map** out) {
    if (!out) return fail(LIO_ERR_ARG, "out is NULL");
    *out = nullptr;
    lio_map_params pp{};
    if (p) pp = *p;
    if (!(pp.cell_size > 0.f)) pp.cell_size = 1.0f;
    if (!(pp.downsample_size > 0.f)) pp.downsample_size = 0.5f;
    int rc = check_device(pp.device);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(pp.device));
    auto* m = new lio_map();
    m->dev = pp.device;
    m->p = pp;
    m->grid.gapped = true;  // per-cell blocks: map_incremental updates in O(points changed)
    if (hipStreamCreateWithFlags(&m->st, hipStreamNonBlocking) != hipSuccess) {
        delete m;
        return fail(LIO_ERR_HIP, "hipStreamCreate failed");
    }
    *out = m;
    return LIO_OK;
}

int lio_map_destroy(lio_map* m) {
    if (!m) return LIO_OK;
    if (m->n_ctx.load() > 0)
        return fail(LIO_ERR_STATE, "lio_map_destroy: h_share_model contexts still use this map (lio_ctx_destroy them first)");
    (void)hipSetDevice(m->dev);
    (void)hipStreamSynchronize(m->st);
    lio::grid_free(m->grid);
    lio::mapupd_free(m->upd);
    if (m->d_xyz) (void)hipFree(m->d_xyz);
    if (m->d_qidx) (void)hipFree(m->d_qidx);
    if (m->d_qd2) (void)hipFree(m->d_qd2);
    (void)hipStreamDestroy(m->st);
    delete m;
    return LIO_OK;
}

int lio_map_set_params(lio_map* m, const lio_map_params* p) {
    if (!m || !p) return fail(LIO_ERR_ARG, "lio_map_set_params: bad arguments");
    if (m->grid.n_ids > 0) return fail(LIO_ERR_STATE, "lio_map_set_params: map already holds points (call before Build)");
    if (p->device != m->dev) return fail(LIO_ERR_ARG, "lio_map_set_params: device cannot change");
    if (p->cell_size > 0.f) m->p.cell_size = p->cell_size;
    if (p->downsample_size > 0.f) m->p.downsample_size = p->downsample_size;
    return LIO_OK;
}

static int map_build_impl(lio_map* m, const float* d_xyz, int64_t n) {
    int rc = lio::grid_build(m->grid, d_xyz, n, m->p.cell_size, m->st);
    if (rc == -5) return fail(LIO_ERR_NOMEM, "grid build: out of device memory");
    if (rc == -1) return fail(LIO_ERR_ARG, "grid build: invalid points (empty, too many, or non-finite)");
    if (rc != 0) return fail(LIO_ERR_HIP, "grid build failed");
    // the map_incremental scratch for a scan of up to 256 k points (C3 131 k, C5 ~30 k undistorted), so the
    // stream's first update allocates nothing; larger scans grow it then
    rc = lio::mapupd_presize(m->upd, (int64_t)1 << 18, m->st);
    if (rc) return fail(rc == -5 ? LIO_ERR_NOMEM : LIO_ERR_HIP, "map update scratch");
    HIP_TRY(hipStreamSynchronize(m->st));
    m->n = m->grid.n;
    ++m->version;
    return LIO_OK;
}

int lio_map_build(lio_map* m, const float* xyz, int64_t n) {
    if (!m || (!xyz && n > 0) || n <= 0) return fail(LIO_ERR_ARG, "lio_map_build: bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    int rc = grow(&m->d_xyz, m->xyz_cap, n, 3);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(m->d_xyz, xyz, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, m->st));
    return map_build_impl(m, m->d_xyz, n);
}

int lio_map_build_device(lio_map* m, const float* d_xyz, int64_t n) {
    if (!m || !d_xyz || n <= 0) return fail(LIO_ERR_ARG, "lio_map_build_device: bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    return map_build_impl(m, d_xyz, n);
}

int64_t lio_map_size(const lio_map* m) { return m ? m->n : 0; }
int64_t lio_map_num_ids(const lio_map* m) { return m ? m->grid.n_ids : 0; }

static int map_by_id_host(lio_map* m, std::vector<float4>& tmp) {
    tmp.resize(m->grid.n_ids);
    if (m->grid.n_ids == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(m->dev));
    HIP_TRY(hipMemcpyAsync(tmp.data(), m->grid.by_id, m->grid.n_ids * sizeof(float4), hipMemcpyDeviceToHost, m->st));
    HIP_TRY(hipStreamSynchronize(m->st));
    return LIO_OK;
}

int lio_map_get_points(lio_map* m, float* xyz_out) {
    if (!m || !xyz_out) return fail(LIO_ERR_ARG, "bad arguments");
    std::vector<float4> tmp;
    int rc = map_by_id_host(m, tmp);
    if (rc) return rc;
    int64_t k = 0;
    for (const float4& p : tmp) {
        if (p.w == 0.f) continue;
        xyz_out[3 * k] = p.x;
        xyz_out[3 * k + 1] = p.y;
        xyz_out[3 * k + 2] = p.z;
        ++k;
    }
    return LIO_OK;
}

int lio_map_get_by_id(lio_map* m, float* xyz_out, uint8_t* alive_out) {
    if (!m) return fail(LIO_ERR_ARG, "bad arguments");
    std::vector<float4> tmp;
    int rc = map_by_id_host(m, tmp);
    if (rc) return rc;
    for (size_t i = 0; i < tmp.size(); ++i) {
        if (xyz_out) {
            xyz_out[3 * i] = tmp[i].x;
            xyz_out[3 * i + 1] = tmp[i].y;
            xyz_out[3 * i + 2] = tmp[i].z;
        }
        if (alive_out) alive_out[i] = tmp[i].w != 0.f;
    }
    return LIO_OK;
}

int lio_map_nearest_search(lio_map* m, const float* q, int64_t n, int k, float max_dist, int32_t* idx, float* d2) {
    if (!m || n < 0 || k < 1 || k > 5 || (n > 0 && (!q || !idx)) || n >= (int64_t)1 << 30 || std::isnan(max_dist))
        return fail(LIO_ERR_ARG, "lio_map_nearest_search: bad arguments (k must be 1..5)");
    if (m->grid.n_ids == 0) return fail(LIO_ERR_STATE, "lio_map_nearest_search: map is empty (call lio_map_build)");
    if (n == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(m->dev));
    int rc = grow(&m->d_xyz, m->xyz_cap, n, 3);
    if (!rc) rc = grow(&m->d_qidx, m->qidx_cap, n * k);
    if (!rc && d2) rc = grow(&m->d_qd2, m->qd2_cap, n * k);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(m->d_xyz, q, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, m->st));
    const lio::GridDev g = lio::grid_view(m->grid);
    const bool unbounded = !(max_dist > 0.f) || std::isinf(max_dist);
    const float bound = unbounded ? INFINITY : max_dist * max_dist;
    const int max_shell = unbounded ? 0x3fffffff : (int)std::ceil(max_dist / g.cell) + 1;
    lio::launch_map_knn(g, m->d_xyz, (int)n, bound, max_shell, k, m->d_qidx, d2 ? m->d_qd2 : nullptr, m->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(idx, m->d_qidx, (size_t)n * k * sizeof(int32_t), hipMemcpyDeviceToHost, m->st));
    if (d2) HIP_TRY(hipMemcpyAsync(d2, m->d_qd2, (size_t)n * k * sizeof(float), hipMemcpyDeviceToHost, m->st));
    HIP_TRY(hipStreamSynchronize(m->st));
    return LIO_OK;
}

int lio_map_gather(lio_map* m, const int32_t* ids, int64_t n, float* xyz_out) {
    if (!m || n < 0 || (n > 0 && (!ids || !xyz_out))) return fail(LIO_ERR_ARG, "lio_map_gather: bad arguments");
    if (n == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(m->dev));
    int rc = grow(&m->d_qidx, m->qidx_cap, n);
    if (!rc) rc = grow(&m->d_xyz, m->xyz_cap, n, 3);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(m->d_qidx, ids, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, m->st));
    lio::map_gather_ids(m->grid, m->d_qidx, n, m->d_xyz, m->st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(xyz_out, m->d_xyz, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost, m->st));
    HIP_TRY(hipStreamSynchronize(m->st));
    return LIO_OK;
}

static int map_status(int rc, const char* what) {
    if (rc == 0) return LIO_OK;
    if (rc == -5) return fail(LIO_ERR_NOMEM, std::string(what) + ": out of device memory");
    if (rc == -1) return fail(LIO_ERR_ARG, std::string(what) + ": invalid points");
    return fail(LIO_ERR_HIP, std::string(what) + " failed");
}

int lio_map_add_device(lio_map* m, const float* d_xyz, int64_t n, int downsample, int64_t* n_added) {
    if (!m || n < 0 || (n > 0 && !d_xyz)) return fail(LIO_ERR_ARG, "lio_map_add: bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    int64_t out[2] = {0, 0};
    if (m->grid.n_ids == 0 && !downsample && n > 0) {  // empty map: a plain add is a build
        int rc = lio_map_build_device(m, d_xyz, n);
        if (n_added) *n_added = n;
        return rc;
    }
    int rc = lio::map_add_device(m->grid, m->upd, d_xyz, n, downsample != 0, m->p.downsample_size, map_slack(m), out,
                                 m->st);
    HIP_TRY(hipStreamSynchronize(m->st));
    m->n = m->grid.n;
    ++m->version;
    if (n_added) *n_added = out[0];
    return map_status(rc, "lio_map_add");
}

int lio_map_add(lio_map* m, const float* xyz, int64_t n, int downsample, int64_t* n_added) {
    if (!m || n < 0 || (n > 0 && !xyz)) return fail(LIO_ERR_ARG, "lio_map_add: bad arguments");
    if (n == 0) {
        if (n_added) *n_added = 0;
        return LIO_OK;
    }
    HIP_TRY(hipSetDevice(m->dev));
    int rc = grow(&m->d_xyz, m->xyz_cap, n, 3);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(m->d_xyz, xyz, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, m->st));
    return lio_map_add_device(m, m->d_xyz, n, downsample, n_added);
}

int lio_map_delete_boxes(lio_map* m, const float* boxes, int nb, int64_t* n_deleted) {
    if (!m || nb < 0 || (nb > 0 && !boxes)) return fail(LIO_ERR_ARG, "lio_map_delete_boxes: bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    int64_t nd = 0;
    int rc = lio::map_delete_boxes(m->grid, m->upd, boxes, nb, map_slack(m), &nd, m->st);
    HIP_TRY(hipStreamSynchronize(m->st));
    m->n = m->grid.n;
    ++m->version;
    if (n_deleted) *n_deleted = nd;
    return map_status(rc, "lio_map_delete_boxes");
}

// lasermap_fov_segment() [U]: float box vertices, MOV_THRESHOLD * DET_RANGE
// trigger distance, mov_dist = max((cube_len - 2*MOV_THRESHOLD*DET_RANGE)*0.5*0.9,
// DET_RANGE*(MOV_THRESHOLD-1)) (double, stored float).
int lio_localmap_update(lio_localmap* lm, const double pos_lid[3], double cube_len, float det_range,
                        float mov_threshold, float boxes_out[18], int* n_boxes) {
    if (!lm || !pos_lid || !boxes_out || !n_boxes) return fail(LIO_ERR_ARG, "lio_localmap_update: bad arguments");
    *n_boxes = 0;
    if (!lm->initialized) {
        for (int i = 0; i < 3; ++i) {
            lm->vertex_min[i] = (float)(pos_lid[i] - cube_len / 2.0);
            lm->vertex_max[i] = (float)(pos_lid[i] + cube_len / 2.0);
        }
        lm->initialized = 1;
        return LIO_OK;
    }
    float dist_to_edge[3][2];
    bool need_move = false;
    for (int i = 0; i < 3; ++i) {
        dist_to_edge[i][0] = (float)std::fabs(pos_lid[i] - lm->vertex_min[i]);
        dist_to_edge[i][1] = (float)std::fabs(pos_lid[i] - lm->vertex_max[i]);
        if (dist_to_edge[i][0] <= mov_threshold * det_range || dist_to_edge[i][1] <= mov_threshold * det_range)
            need_move = true;
    }
    if (!need_move) return LIO_OK;
    lio_localmap nw = *lm;
    const float mov_dist = (float)std::max((cube_len - 2.0 * mov_threshold * det_range) * 0.5 * 0.9,
                                           (double)(det_range * (mov_threshold - 1)));
    for (int i = 0; i < 3; ++i) {
        float bmin[3], bmax[3];
        for (int d = 0; d < 3; ++d) {
            bmin[d] = lm->vertex_min[d];
            bmax[d] = lm->vertex_max[d];
        }
        bool add = false;
        if (dist_to_edge[i][0] <= mov_threshold * det_range) {
            nw.vertex_max[i] -= mov_dist;
            nw.vertex_min[i] -= mov_dist;
            bmin[i] = lm->vertex_max[i] - mov_dist;
            add = true;
        } else if (dist_to_edge[i][1] <= mov_threshold * det_range) {
            nw.vertex_max[i] += mov_dist;
            nw.vertex_min[i] += mov_dist;
            bmax[i] = lm->vertex_min[i] + mov_dist;
            add = true;
        }
        if (add) {
            float* b = boxes_out + 6 * (*n_boxes);
            for (int d = 0; d < 3; ++d) {
                b[d] = bmin[d];
                b[3 + d] = bmax[d];
            }
            ++*n_boxes;
        }
    }
    *lm = nw;
    return LIO_OK;
}

int lio_map_get_grid(lio_map* m, double* out7) {
    if (!m || !out7) return fail(LIO_ERR_ARG, "bad arguments");
    const lio::GridGeom& g = m->grid.geom;
    out7[0] = g.ox;
    out7[1] = g.oy;
    out7[2] = g.oz;
    out7[3] = g.cell;
    out7[4] = g.nx;
    out7[5] = g.ny;
    out7[6] = g.nz;
    return LIO_OK;
}

int lio_map_set_test_limits(lio_map* m, int64_t slot_headroom, int64_t dirty_cells) {
    if (!m || slot_headroom < 0 || dirty_cells < 0) return fail(LIO_ERR_ARG, "lio_map_set_test_limits: bad arguments");
    m->grid.slots_extra = slot_headroom;
    m->upd.dcap_limit = dirty_cells;
    return LIO_OK;
}

int lio_map_get_stats(lio_map* m, int64_t* out8) {
    if (!m || !out8) return fail(LIO_ERR_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    uint32_t bump = 0;
    if (m->grid.bump) {
        HIP_TRY(hipMemcpyAsync(&bump, m->grid.bump, sizeof(bump), hipMemcpyDeviceToHost, m->st));
        HIP_TRY(hipStreamSynchronize(m->st));
    }
    out8[0] = m->grid.rebuilds;
    out8[1] = m->grid.slots_cap;
    out8[2] = bump;
    out8[3] = m->grid.n;
    out8[4] = m->grid.n_ids;
    out8[5] = m->grid.geom.ncells;
    out8[6] = m->upd.h_cnt ? (int64_t)m->upd.h_cnt[9] : 0;  // lio_mapupd.hip kCFlags
    out8[7] = 0;
    return LIO_OK;
}

// =============================================================================
// h_share_model context
// =============================================================================
int lio_ctx_create(lio_map* m, const lio_match_params* p, lio_ctx** out) {
    if (!m || !out) return fail(LIO_ERR_ARG, "bad arguments");
    HIP_TRY(hipSetDevice(m->dev));
    auto* c = new lio_ctx();
    c->map = m;
    ++m->n_ctx;
    if (p)
        c->p = *p;
    else
        c->p = lio_match_params{5.0f, 0.1f, 0.9, 0.9};
    if (hipMalloc(&c->d_sums, 32 * sizeof(double)) != hipSuccess ||
        hipHostMalloc(&c->h_sums, 40 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_sums_dev), c->h_sums, 0) != hipSuccess ||
        hipMalloc(&c->d_nrows, sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&c->d_far_count, sizeof(int)) != hipSuccess ||
        hipMemsetAsync(c->d_far_count, 0, sizeof(int), m->st) != hipSuccess || hipMalloc(&c->d_done, 64) != hipSuccess ||
        hipMemsetAsync(c->d_done, 0, 64, m->st) != hipSuccess) {  // on the map's stream: it does not wait for the null stream
        --m->n_ctx;
        delete c;
        return fail(LIO_ERR_NOMEM, "context allocation failed");
    }
    for (EventPair* e : {&c->ev_main, &c->ev_fin}) {
        (void)hipEventCreate(&e->a);
        (void)hipEventCreate(&e->b);
    }
    for (hipEvent_t& e : c->ev_marks) (void)hipEventCreate(&e);
    *out = c;
    return LIO_OK;
}

int lio_ctx_destroy(lio_ctx* c) {
    if (!c) return LIO_OK;
    (void)hipSetDevice(c->map->dev);
    (void)hipStreamSynchronize(c->map->st);
    void* ptrs[] = {c->d_body,  c->d_nn,    c->d_planes,   c->d_sel,       c->d_partials, c->d_sums,
                    c->d_rows,  c->d_nrows, c->d_far_list, c->d_far_count, c->d_far_d,    c->d_far_id, c->d_done,
                    c->d_d5};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    if (c->h_sums) (void)hipHostFree(c->h_sums);
    for (EventPair* e : {&c->ev_main, &c->ev_fin}) {
        if (e->a) (void)hipEventDestroy(e->a);
        if (e->b) (void)hipEventDestroy(e->b);
    }
    for (hipEvent_t e : c->ev_marks)
        if (e) (void)hipEventDestroy(e);
    lio::filter_free(c->filt);
    for (void* q : {(void*)c->d_raw, (void*)c->d_rec, (void*)c->d_poses, (void*)c->d_kf})
        if (q) (void)hipFree(q);
    --c->map->n_ctx;
    delete c;
    return LIO_OK;
}

static int ctx_reserve(lio_ctx* c, int64_t n) {
    if (n > c->cap || !c->d_body || !c->d_nn || !c->d_planes || !c->d_sel || !c->d_far_list || !c->d_far_d ||
        !c->d_far_id || !c->d_d5) {
        int64_t cap = std::max<int64_t>(n, c->cap + c->cap / 2);
        c->cap = 0;  // a failed reallocation below leaves no buffer that looks usable
        void* ptrs[] = {c->d_body, c->d_nn, c->d_planes, c->d_sel, c->d_far_list, c->d_far_d, c->d_far_id, c->d_d5};
        for (void* q : ptrs)
            if (q) (void)hipFree(q);
        c->d_body = nullptr;
        c->d_nn = nullptr;
        c->d_planes = nullptr;
        c->d_sel = nullptr;
        c->d_far_list = nullptr;
        c->d_far_d = nullptr;
        c->d_far_id = nullptr;
        c->d_d5 = nullptr;
        lio::count_alloc(8);
        if (hipMalloc(&c->d_body, cap * 3 * sizeof(float)) != hipSuccess ||
            hipMalloc(&c->d_nn, cap * 5 * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&c->d_planes, cap * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->d_sel, cap + 64) != hipSuccess ||
            hipMalloc(&c->d_far_list, cap * sizeof(int)) != hipSuccess ||
            hipMalloc(&c->d_far_d, cap * 5 * sizeof(float)) != hipSuccess ||
            hipMalloc(&c->d_far_id, cap * 5 * sizeof(int)) != hipSuccess ||
            hipMalloc(&c->d_d5, cap * sizeof(float)) != hipSuccess)
            return fail(LIO_ERR_NOMEM, "scan buffers: hipMalloc failed");
        c->cap = cap;
    }
    int rc = grow(&c->d_partials, c->part_cap, (int64_t)lio::match_blocks((int)n) * 32 + 32);
    if (rc) return rc;
    c->n = n;
    c->body_ext = nullptr;
    c->have_eval = false;
    c->knn_valid = false;
    return LIO_OK;
}

int lio_scan_set(lio_ctx* c, const float* body, int64_t n) {
    if (!c || n < 0 || (n > 0 && !body) || n >= (int64_t)1 << 30) return fail(LIO_ERR_ARG, "lio_scan_set: bad arguments");
    HIP_TRY(hipSetDevice(c->map->dev));
    int rc = ctx_reserve(c, n);
    if (rc) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(c->d_body, body, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice, c->map->st));
    return LIO_OK;
}

int lio_scan_set_device(lio_ctx* c, const float* d_body, int64_t n) {
    if (!c || n < 0 || (n > 0 && !d_body) || n >= (int64_t)1 << 30) return fail(LIO_ERR_ARG, "lio_scan_set_device: bad arguments");
    HIP_TRY(hipSetDevice(c->map->dev));
    int rc = ctx_reserve(c, n);
    if (rc) return rc;
    if (n)
        HIP_TRY(hipMemcpyAsync(c->d_body, d_body, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToDevice, c->map->st));
    return LIO_OK;
}

int lio_scan_bind_device(lio_ctx* c, const float* d_body, int64_t n) {
    if (!c || n < 0 || (n > 0 && !d_body) || n >= (int64_t)1 << 30) return fail(LIO_ERR_ARG, "lio_scan_bind_device: bad arguments");
    HIP_TRY(hipSetDevice(c->map->dev));
    int rc = ctx_reserve(c, n);
    if (rc) return rc;
    c->body_ext = n ? d_body : nullptr;
    return LIO_OK;
}

static const float* body_ptr(const lio_ctx* c) { return c->body_ext ? c->body_ext : c->d_body; }

static_assert(sizeof(lio_pose) == sizeof(lio::PoseArg), "lio_pose / PoseArg layout");

static lio::MatchArgs make_args(lio_ctx* c, const lio_pose& pose_in) {
    lio::MatchArgs a{};
    const lio_pose pose = filled(pose_in);
    std::memcpy(&a.pose, &pose, sizeof(lio::PoseArg));
    a.grid = lio::grid_view(c->map->grid);
    a.body = body_ptr(c);
    a.map_by_id = c->map->grid.by_id;
    a.nn_idx = c->d_nn;
    a.nn_d5 = c->d_d5;
    a.seed_scale = c->seed_scale;
    {
        const lio_pose pk = filled(c->knn_pose);
        std::memcpy(&a.pose_knn, &pk, sizeof(lio::PoseArg));
        // float affine map body -> world of that pose, [R R_LI | R t_LI + t], from the quaternions the
        // kernels rotate with (never from R / R_LI, which a caller may leave stale)
        double R[9], RL[9];
        quat_to_mat(pk.q, R);
        quat_to_mat(pk.q_LI, RL);
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k)
                a.knn_M[4 * r + k] =
                    (float)(R[3 * r] * RL[k] + R[3 * r + 1] * RL[3 + k] + R[3 * r + 2] * RL[6 + k]);
            a.knn_M[4 * r + 3] =
                (float)(R[3 * r] * pk.t_LI[0] + R[3 * r + 1] * pk.t_LI[1] + R[3 * r + 2] * pk.t_LI[2] + pk.t[r]);
        }
    }
    a.planes = c->d_planes;
    a.sel = c->d_sel;
    a.partials = c->d_partials;
    a.n = (int)c->n;
    // every point with d2 <= range lies within ceil(sqrt(range)/cell)+1 shells
    a.max_shell = (int)std::ceil(std::sqrt((double)c->p.knn_range_sq) / a.grid.cell) + 1;
    a.dbg = nullptr;
    a.sums_out = c->h_sums_dev;
    a.seq_out = reinterpret_cast<unsigned long long*>(c->h_sums_dev + 32);
    a.seq = 0;
    a.far_list = c->d_far_list;
    a.far_count = c->d_far_count;
    a.done_count = c->d_done;
    a.far_d = c->d_far_d;
    a.far_id = c->d_far_id;
    a.range_sq = c->p.knn_range_sq;
    a.plane_thr = c->p.plane_thr;
    a.s_coef = c->p.s_coef;
    a.s_gate = c->p.s_gate;
    return a;
}

static void accum_event(EventPair& e, int64_t& launches, double& ms) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, e.a, e.b) == hipSuccess) {
        ms += t;
        ++launches;
    }
}

// Wait until the evaluation's last block has published sequence number `seq`
// (zero-copy result, no copy / stream-sync round trip).  The GPU stores the
// sums, the number and a checksum of both unordered (lio_match.hip
// publish_host), so a result counts only when the number matches AND the
// sums read after it hash to the checksum; once the stream is idle every word
// has landed, so a stream error, or an idle stream whose words still do not
// match, ends the wait with an error.
static uint64_t mix64(uint64_t z) {  // splitmix64 finaliser, as publish_host
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static bool read_result(const lio_ctx* c, unsigned long long seq, double* sums) {
    const volatile uint64_t* w = reinterpret_cast<const volatile uint64_t*>(c->h_sums);
    if (w[32] != seq) return false;
    uint64_t h = 0, bits[LIO_SUMS_LEN];
    for (int l = 0; l < LIO_SUMS_LEN; ++l) {
        bits[l] = w[l];
        h ^= mix64(bits[l] ^ ((uint64_t)l * 0x9e3779b97f4a7c15ull));
    }
    if ((h ^ mix64(seq)) != w[33]) return false;
    std::memcpy(sums, bits, sizeof(bits));
    return true;
}

static int wait_result(lio_ctx* c, unsigned long long seq, double* sums) {
    for (uint64_t it = 0;; ++it) {
        if (read_result(c, seq, sums)) return LIO_OK;
        if ((it & 255) == 255) {
            const hipError_t e = hipStreamQuery(c->map->st);
            if (e != hipSuccess && e != hipErrorNotReady)
                return fail(LIO_ERR_HIP, std::string("lio_match: ") + hipGetErrorString(e));
            if (e == hipSuccess && !read_result(c, seq, sums))
                return fail(LIO_ERR_HIP, "lio_match: evaluation produced no result");
        }
    }
}

static int match_impl(lio_ctx* c, const lio_pose* pose_in, int redo_knn, double* sums);

int lio_match(lio_ctx* c, const lio_pose* pose_in, int redo_knn, double* sums) {
    if (!c || !pose_in || !sums) return fail(LIO_ERR_ARG, "lio_match: bad arguments");
    return match_impl(c, pose_in, redo_knn, sums);
}

static int match_impl(lio_ctx* c, const lio_pose* pose_in, int redo_knn, double* sums) {
    const lio_pose pose_f = filled(*pose_in);
    const lio_pose* pose = &pose_f;
    if (c->map->grid.n_ids == 0) return fail(LIO_ERR_STATE, "lio_match: map is empty (call lio_map_build)");
    if (!redo_knn && !c->knn_valid) return fail(LIO_ERR_STATE, "lio_match: redo_knn=0 before any kNN evaluation");
    if (!redo_knn && c->knn_map_version != c->map->version)
        return fail(LIO_ERR_STATE, "lio_match: redo_knn=0 but the map changed since this scan's kNN evaluation");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    lio::MatchArgs a = make_args(c, *pose);
    if (c->map->n == 0 && c->n > 0) {
        // every map point deleted (Delete_Point_Boxes): Nearest_Search finds
        // nothing, no point is effective ("No Effective Points!")
        HIP_TRY(hipMemsetAsync(c->d_nn, 0xff, c->n * 5 * sizeof(int32_t), st));
        HIP_TRY(hipMemsetAsync(c->d_sel, 0, c->n, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (c->n == 0 || c->map->n == 0) {
        std::memset(sums, 0, LIO_SUMS_LEN * sizeof(double));
        c->last_pose = *pose;
        c->have_eval = true;
        c->knn_valid = true;
        c->knn_map_version = c->map->version;
        c->knn_pose = *pose;
        return LIO_OK;
    }
    a.seq = ++c->seq;
    // later kNN evaluations of the same scan against the same map start from the previous lists
    a.prior = (redo_knn && c->knn_valid && c->knn_map_version == c->map->version) ? 1 : 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (c->timing) HIP_TRY(hipEventRecord(c->ev_main.a, st));
    lio::launch_h_model(a, redo_knn != 0, st, c->timing ? c->ev_marks : nullptr);
    if (c->timing) HIP_TRY(hipEventRecord(c->ev_main.b, st));
    HIP_TRY(hipGetLastError());
    const auto t1 = std::chrono::steady_clock::now();
    int rc = wait_result(c, a.seq, sums);
    if (rc) return rc;
    const auto t2 = std::chrono::steady_clock::now();
    c->last_launch_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    c->last_wait_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    if (c->timing) {
        HIP_TRY(hipEventSynchronize(c->ev_main.b));
        if (redo_knn) {  // kernel spans (hipExtLaunchKernel events): no launch gaps, as rocprofv3 reports
            const double before = c->tm.near_ms + c->tm.far_ms + c->tm.plane_ms;
            EventPair n{c->ev_marks[0], c->ev_marks[1]}, f{c->ev_marks[2], c->ev_marks[3]},
                p{c->ev_marks[4], c->ev_marks[5]};
            accum_event(n, c->tm.near_launches, c->tm.near_ms);
            if (a.max_shell > 1) accum_event(f, c->tm.far_launches, c->tm.far_ms);
            accum_event(p, c->tm.plane_launches, c->tm.plane_ms);
            c->tm.knn_ms += (c->tm.near_ms + c->tm.far_ms + c->tm.plane_ms) - before;
            ++c->tm.knn_launches;
        } else {
            EventPair r{c->ev_marks[6], c->ev_marks[7]};
            accum_event(r, c->tm.reuse_launches, c->tm.reuse_ms);
        }
    }
    c->last_pose = *pose;
    c->have_eval = true;
    if (redo_knn) {
        c->knn_valid = true;
        c->knn_map_version = c->map->version;
        c->knn_pose = *pose;
    }
    return LIO_OK;
}

int lio_ctx_knn_stats(lio_ctx* c, const lio_pose* pose, double* sums, int32_t* stats3) {
    if (!c || !pose || !sums || !stats3) return fail(LIO_ERR_ARG, "lio_ctx_knn_stats: bad arguments");
    if (c->map->n == 0) return fail(LIO_ERR_STATE, "lio_ctx_knn_stats: map is empty");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    if (c->n == 0) return LIO_OK;
    int* d_dbg = nullptr;
    HIP_TRY(hipMalloc(&d_dbg, c->n * 3 * sizeof(int)));
    lio::MatchArgs a = make_args(c, *pose);
    a.dbg = d_dbg;
    a.seq = ++c->seq;
    lio::launch_h_model(a, true, st);
    hipError_t e2 = hipMemcpyAsync(stats3, d_dbg, c->n * 3 * sizeof(int), hipMemcpyDeviceToHost, st);
    hipError_t e3 = hipStreamSynchronize(st);
    (void)hipFree(d_dbg);
    if (e2 != hipSuccess || e3 != hipSuccess) return fail(LIO_ERR_HIP, "lio_ctx_knn_stats failed");
    int rc = wait_result(c, a.seq, sums);
    if (rc) return rc;
    c->last_pose = *pose;
    c->knn_pose = *pose;
    c->have_eval = true;
    c->knn_valid = true;
    c->knn_map_version = c->map->version;
    return LIO_OK;
}

int lio_ctx_get_knn_pose(lio_ctx* c, lio_pose* out) {
    if (!c || !out) return fail(LIO_ERR_ARG, "bad arguments");
    if (!c->knn_valid) return fail(LIO_ERR_STATE, "lio_ctx_get_knn_pose: no kNN evaluation");
    *out = c->knn_pose;
    return LIO_OK;
}

int lio_map_incremental(lio_ctx* c, const lio_pose* pose, double filter_size_map, lio_incremental_stats* st) {
    if (!c || !pose || !(filter_size_map > 0.0)) return fail(LIO_ERR_ARG, "lio_map_incremental: bad arguments");
    if (c->n > 0 && !c->knn_valid && c->map->n > 0)
        return fail(LIO_ERR_STATE, "lio_map_incremental: no kNN evaluation for this scan (Nearest_Points)");
    if (c->n > 0 && c->map->n > 0 && c->knn_map_version != c->map->version)
        return fail(LIO_ERR_STATE, "lio_map_incremental: the map changed since this scan's kNN evaluation");
    lio_map* m = c->map;
    HIP_TRY(hipSetDevice(m->dev));
    lio::IncrArgs a{};
    const lio_pose pf = filled(*pose);
    std::memcpy(&a.pose, &pf, sizeof(lio::PoseArg));
    const lio_pose pk = filled(c->knn_pose);
    std::memcpy(&a.pose_knn, &pk, sizeof(lio::PoseArg));
    a.body = body_ptr(c);
    a.nn_idx = c->d_nn;
    a.n = (int)c->n;
    a.fs = filter_size_map;
    a.range_sq = c->p.knn_range_sq;
    int64_t out[4] = {0, 0, 0, 0};
    int rc = 0;
    if (m->grid.n_ids == 0) {  // ikdtree.Build on the first scan is the caller's job (lio_map_build)
        return fail(LIO_ERR_STATE, "lio_map_incremental: map is empty (build it from the first scan)");
    }
    rc = lio::map_incremental(m->grid, m->upd, a, m->p.downsample_size, map_slack(m), out, m->st);
    HIP_TRY(hipStreamSynchronize(m->st));
    m->n = m->grid.n;
    ++m->version;
    c->knn_valid = false;  // ids/grid changed
    if (st) {
        st->n_to_add = out[0];
        st->n_no_downsample = out[1];
        st->n_skipped = out[2];
        st->n_added_downsample = out[3];
    }
    return map_status(rc, "lio_map_incremental");
}

int lio_get_knn(lio_ctx* c, int32_t* idx, float* d2) {
    if (!c || !c->have_eval) return fail(LIO_ERR_STATE, "lio_get_knn: no evaluation yet");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    if (c->n == 0) return LIO_OK;
    if (idx) HIP_TRY(hipMemcpyAsync(idx, c->d_nn, c->n * 5 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (d2) {
        float* tmp = nullptr;
        HIP_TRY(hipMalloc(&tmp, c->n * 5 * sizeof(float)));
        lio::launch_debug(make_args(c, c->last_pose), nullptr, tmp, nullptr, st);
        hipError_t e = hipMemcpyAsync(d2, tmp, c->n * 5 * sizeof(float), hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        (void)hipFree(tmp);
        if (e != hipSuccess) return fail(LIO_ERR_HIP, "lio_get_knn copy failed");
    }
    HIP_TRY(hipStreamSynchronize(st));
    return LIO_OK;
}

int lio_get_planes(lio_ctx* c, float* abcd_pd2, uint8_t* sel) {
    if (!c || !c->have_eval) return fail(LIO_ERR_STATE, "lio_get_planes: no evaluation yet");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    if (c->n == 0) return LIO_OK;
    if (sel) HIP_TRY(hipMemcpyAsync(sel, c->d_sel, c->n, hipMemcpyDeviceToHost, st));
    if (abcd_pd2) {
        float* tmp = nullptr;
        HIP_TRY(hipMalloc(&tmp, c->n * 4 * sizeof(float)));
        lio::launch_debug(make_args(c, c->last_pose), nullptr, nullptr, tmp, st);
        hipError_t e = hipMemcpyAsync(abcd_pd2, tmp, c->n * 4 * sizeof(float), hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        (void)hipFree(tmp);
        if (e != hipSuccess) return fail(LIO_ERR_HIP, "lio_get_planes copy failed");
    }
    HIP_TRY(hipStreamSynchronize(st));
    return LIO_OK;
}

int lio_get_world(lio_ctx* c, float* world) {
    if (!c || !world || !c->have_eval) return fail(LIO_ERR_STATE, "lio_get_world: no evaluation yet");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    if (c->n == 0) return LIO_OK;
    float* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, c->n * 3 * sizeof(float)));
    lio::launch_debug(make_args(c, c->last_pose), tmp, nullptr, nullptr, st);
    hipError_t e = hipMemcpyAsync(world, tmp, c->n * 3 * sizeof(float), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    (void)hipFree(tmp);
    if (e != hipSuccess) return fail(LIO_ERR_HIP, "lio_get_world copy failed");
    return LIO_OK;
}

int lio_get_h_rows(lio_ctx* c, double* rows, int64_t max_rows, int64_t* n_rows) {
    if (!c || !n_rows || (max_rows > 0 && !rows)) return fail(LIO_ERR_ARG, "lio_get_h_rows: bad arguments");
    if (!c->have_eval) return fail(LIO_ERR_STATE, "lio_get_h_rows: no evaluation yet");
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    int rc = grow(&c->d_rows, c->rows_cap, std::max<int64_t>(max_rows, 1) * 7);
    if (rc) return rc;
    lio::launch_h_rows(make_args(c, c->last_pose), c->d_rows, max_rows, c->d_nrows, st);
    int64_t nr = 0;
    HIP_TRY(hipMemcpyAsync(&nr, c->d_nrows, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const int64_t ncopy = std::min(nr, max_rows);
    if (ncopy > 0) {
        HIP_TRY(hipMemcpyAsync(rows, c->d_rows, ncopy * 7 * sizeof(double), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    *n_rows = nr;
    return LIO_OK;
}

// =============================================================================
// IESKF
// =============================================================================
static lio::host::State to_host(const lio_state& s) {
    lio::host::State x;
    std::memcpy(x.pos, s.pos, sizeof(x.pos));
    x.rot = {s.rot[0], s.rot[1], s.rot[2], s.rot[3]};
    x.offR = {s.offset_R_L_I[0], s.offset_R_L_I[1], s.offset_R_L_I[2], s.offset_R_L_I[3]};
    std::memcpy(x.offT, s.offset_T_L_I, sizeof(x.offT));
    std::memcpy(x.vel, s.vel, sizeof(x.vel));
    std::memcpy(x.bg, s.bg, sizeof(x.bg));
    std::memcpy(x.ba, s.ba, sizeof(x.ba));
    std::memcpy(x.grav, s.grav, sizeof(x.grav));
    return x;
}
static void from_host(const lio::host::State& x, lio_state& s) {
    std::memcpy(s.pos, x.pos, sizeof(x.pos));
    s.rot[0] = x.rot.w; s.rot[1] = x.rot.x; s.rot[2] = x.rot.y; s.rot[3] = x.rot.z;
    s.offset_R_L_I[0] = x.offR.w; s.offset_R_L_I[1] = x.offR.x; s.offset_R_L_I[2] = x.offR.y; s.offset_R_L_I[3] = x.offR.z;
    std::memcpy(s.offset_T_L_I, x.offT, sizeof(x.offT));
    std::memcpy(s.vel, x.vel, sizeof(x.vel));
    std::memcpy(s.bg, x.bg, sizeof(x.bg));
    std::memcpy(s.ba, x.ba, sizeof(x.ba));
    std::memcpy(s.grav, x.grav, sizeof(x.grav));
}

static lio_pose state_pose(const lio::host::State& s) {  // the pose an evaluation at state s uses
    lio_pose pose;
    lio::host::quat_to_mat(s.rot, pose.R);
    lio::host::quat_to_mat(s.offR, pose.R_LI);
    pose.q[0] = s.rot.w, pose.q[1] = s.rot.x, pose.q[2] = s.rot.y, pose.q[3] = s.rot.z;
    pose.q_LI[0] = s.offR.w, pose.q_LI[1] = s.offR.x, pose.q_LI[2] = s.offR.y, pose.q_LI[3] = s.offR.z;
    std::memcpy(pose.t, s.pos, sizeof(pose.t));
    std::memcpy(pose.t_LI, s.offT, sizeof(pose.t_LI));
    return pose;
}

int lio_ctx_set_seed_scale(lio_ctx* c, float scale) {
    if (!c || !(scale > 0.f && scale <= 1.f)) return fail(LIO_ERR_ARG, "lio_ctx_set_seed_scale: scale in (0, 1]");
    c->seed_scale = scale;
    return LIO_OK;
}

int lio_ieskf_update(lio_ctx* c, lio_state* xs, double* P, const lio_ieskf_params* p, lio_ieskf_stats* st) {
    if (!c || !xs || !P) return fail(LIO_ERR_ARG, "lio_ieskf_update: bad arguments");
    const auto t_call = std::chrono::steady_clock::now();
    lio_ieskf_params pp = p ? *p : lio_ieskf_params{0.001, 3, 0.001};
    lio::host::State x = to_host(*xs);
    lio::host::Mat Pm(P, P + LIO_STATE_DIM * LIO_STATE_DIM);
    int err = LIO_OK;
    double launch_ms = 0.0, wait_ms = 0.0;
    auto hfn = [&](const lio::host::State& s, bool redo, bool want_rows, lio::host::HModel& hm) -> int {
        if (want_rows) {
            const int64_t want = (int64_t)hm.sums[LIO_SUMS_NEFF];
            hm.rows.assign((size_t)std::max<int64_t>(want, 1) * 7, 0.0);
            int64_t nr = 0;
            int rc = lio_get_h_rows(c, hm.rows.data(), want, &nr);
            if (rc) return err = rc;
            hm.rows.resize((size_t)std::min(nr, want) * 7);
            return 0;
        }
        const lio_pose pose = state_pose(s);
        hm.rows.clear();
        c->last_launch_ms = c->last_wait_ms = 0.0;
        int rc = match_impl(c, &pose, redo ? 1 : 0, hm.sums);
        if (rc) return err = rc;
        launch_ms += c->last_launch_ms;
        wait_ms += c->last_wait_ms;
        return 0;
    };
    lio::host::IeskfResult r;
    int rc = lio::host::update_iterated(x, Pm, pp.laser_point_cov, pp.max_iteration, pp.epsi, hfn, r);
    if (rc) return err ? err : fail(LIO_ERR_STATE, "IESKF: singular matrix");
    from_host(x, *xs);
    std::memcpy(P, Pm.data(), sizeof(double) * LIO_STATE_DIM * LIO_STATE_DIM);
    if (st) {
        st->h_evals = r.h_evals;
        st->knn_calls = r.knn_calls;
        st->converged = r.converged;
        st->n_eff = r.n_eff;
        st->res_mean = r.res_mean;
        st->solve_ms = r.solve_ms;
        st->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
        st->launch_ms = launch_ms;
        st->wait_ms = wait_ms;
    }
    return LIO_OK;
}

// =============================================================================
// filters
// =============================================================================
struct lio_filter {
    int dev = 0;
    hipStream_t st = nullptr;
    lio::FilterBuf b;
    float* d_in = nullptr;
    int64_t in_cap = 0;
    float* d_out = nullptr;
    int64_t out_cap = 0;
    int64_t* d_seg = nullptr;
    int64_t seg_cap = 0;
    double* d_T = nullptr;
    int64_t T_cap = 0;
    lio::ImuPose* d_poses = nullptr;
    int64_t poses_cap = 0;
};

static int filter_status(int rc, const char* what) {
    if (rc == 0) return LIO_OK;
    if (rc == -5) return fail(LIO_ERR_NOMEM, std::string(what) + ": out of device memory");
    if (rc == -1) return fail(LIO_ERR_ARG, std::string(what) + ": bad arguments");
    return fail(LIO_ERR_HIP, std::string(what) + " failed");
}

static lio::UndistortEnd undistort_end(const lio_pose* e) {
    lio::UndistortEnd u{};
    if (!e) {
        for (int k = 0; k < 9; ++k) u.R[k] = u.R_LI[k] = (k % 4 == 0) ? 1.0 : 0.0;
        u.q[0] = u.q_LI[0] = 1.0;
        return u;
    }
    const lio_pose f = filled(*e);
    std::memcpy(u.pos, f.t, sizeof(u.pos));
    std::memcpy(u.R, f.R, sizeof(u.R));
    std::memcpy(u.R_LI, f.R_LI, sizeof(u.R_LI));
    std::memcpy(u.t_LI, f.t_LI, sizeof(u.t_LI));
    std::memcpy(u.q, f.q, sizeof(u.q));
    std::memcpy(u.q_LI, f.q_LI, sizeof(u.q_LI));
    return u;
}

static_assert(sizeof(lio_imu_pose) == sizeof(lio::ImuPose), "lio_imu_pose layout");

// The host half of a sweep upload: rows i % every == 0 — Preprocess's point_filter_num drops the others
// by index alone, so they never cross PCIe — and the IMU poses packed into the filter's pinned staging
// buffer, for one DMA each (pageable sources would be staged by the runtime anyway).  *u = rows staged;
// the poses start at byte *pose_off.
static int stage_sweep(lio::FilterBuf& b, const void* rows, int64_t n, size_t row_bytes, int every,
                       const lio_imu_pose* poses, int np, int64_t* u, size_t* pose_off) {
    every = std::max(every, 1);
    *u = (n + every - 1) / every;
    *pose_off = ((size_t)*u * row_bytes + 255) & ~(size_t)255;
    const size_t need = *pose_off + (size_t)np * sizeof(lio_imu_pose);
    if (need > b.stage_bytes || !b.h_stage) {
        if (b.h_stage) (void)hipHostFree(b.h_stage);
        b.h_stage = nullptr;
        const size_t c = std::max(need, b.stage_bytes + b.stage_bytes / 2);
        lio::count_alloc();
        if (hipHostMalloc(&b.h_stage, c) != hipSuccess) {
            b.stage_bytes = 0;
            return fail(LIO_ERR_NOMEM, "sweep staging: hipHostMalloc failed");
        }
        b.stage_bytes = c;
    }
    auto* dst = static_cast<uint8_t*>(b.h_stage);
    const auto* src = static_cast<const uint8_t*>(rows);
    if (every == 1) {
        std::memcpy(dst, src, (size_t)n * row_bytes);
    } else if (row_bytes % 4 == 0 && row_bytes <= 4 * lio::kMaxFields) {
        const int nw = (int)(row_bytes / 4);
        const auto* s = reinterpret_cast<const float*>(rows);
        auto* d = reinterpret_cast<float*>(dst);
        for (int64_t r = 0; r < *u; ++r)
            for (int k = 0; k < nw; ++k) d[r * nw + k] = s[r * every * nw + k];
    } else {
        for (int64_t r = 0; r < *u; ++r) std::memcpy(dst + r * row_bytes, src + r * every * row_bytes, row_bytes);
    }
    if (np) std::memcpy(dst + *pose_off, poses, (size_t)np * sizeof(lio_imu_pose));
    return LIO_OK;
}

// rows i % every == 0 with x*x + y*y + z*z > blind2 (float, left to right: scan_key_kernel's order) copied to
// d in input order; every row is written at the cursor and the cursor advances by the keep flag (no branch
// on the data); sorted: the kept rows' time keys (scan_key_kernel's) never decrease
extern "C++" {  // inside the file's extern "C" block
template <int S>
static int64_t select_rows(const float* __restrict__ raw, int64_t n, int every, float blind2, int tf,
                           float* __restrict__ d, bool& sorted, uint32_t& first_key, uint32_t& last_key) {
    int64_t k = 0;
    uint32_t prev = 0, unsorted = 0, first = 0xffffffffu;
    for (int64_t i = 0; i < n; i += every) {
        const float* q = raw + i * S;
        float r[S];
        for (int f = 0; f < S; ++f) r[f] = q[f];
        const uint32_t keep = (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) > blind2 ? 1u : 0u;
        uint32_t tb;
        std::memcpy(&tb, &r[tf], 4);
        const uint32_t key = (tb & 0x80000000u) ? ~tb : (tb | 0x80000000u);  // scan_key_kernel's time key
        unsorted |= keep & (key < prev ? 1u : 0u);
        first = (keep && k == 0) ? key : first;
        prev = keep ? key : prev;
        for (int f = 0; f < S; ++f) d[k * S + f] = r[f];
        k += keep;
    }
    sorted = unsorted == 0;
    first_key = first;
    last_key = prev;
    return k;
}
}  // extern "C++"

// Float records: Preprocess's whole selection made while packing (the host reads every row here anyway) —
// i % point_filter_num == 0 and x*x + y*y + z*z > blind^2, in float and in that order as the device's
// scan_key_kernel — so the device gets exactly the m selected rows, in input order; *sorted says whether
// their times are non-decreasing (the stable time sort is then the identity and the device skips it).
// Large sweeps are packed by the host pool in up to kStageChunks contiguous pieces, each at its own offset
// of the staging buffer (the upper bound of its rows): the plan lists them, and the caller moves each
// piece with its own DMA to where the concatenation puts it.
constexpr int kStageChunks = lio::kMaxPieces;
struct StagePlan {
    int pieces = 0;
    int64_t src_row[kStageChunks] = {};  // first staging row of the piece
    int64_t rows[kStageChunks] = {};     // its selected rows
};

static int stage_sweep_select(lio::FilterBuf& b, const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                              const lio_imu_pose* poses, int np, int64_t* m, size_t* pose_off, bool* sorted,
                              StagePlan* plan) {
    const int every = std::max(p->point_filter_num, 1);
    const int64_t ub = (n + every - 1) / every;  // candidate rows (i % every == 0)
    *pose_off = ((size_t)ub * stride * sizeof(float) + 255) & ~(size_t)255;
    const size_t need = *pose_off + (size_t)np * sizeof(lio_imu_pose);
    if (need > b.stage_bytes || !b.h_stage) {
        if (b.h_stage) (void)hipHostFree(b.h_stage);
        b.h_stage = nullptr;
        const size_t c = std::max(need, b.stage_bytes + b.stage_bytes / 2);
        lio::count_alloc();
        if (hipHostMalloc(&b.h_stage, c) != hipSuccess) {
            b.stage_bytes = 0;
            return fail(LIO_ERR_NOMEM, "sweep staging: hipHostMalloc failed");
        }
        b.stage_bytes = c;
    }
    const float blind2 = p->blind * p->blind;
    auto* d = static_cast<float*>(b.h_stage);
    const int pieces = ub >= 16384 ? std::min(kStageChunks, lio::HostPool::get().threads()) : 1;
    const int64_t per = (ub + pieces - 1) / pieces;  // candidate rows per piece
    int64_t k[kStageChunks] = {};
    bool srt[kStageChunks] = {};
    uint32_t first[kStageChunks] = {}, last[kStageChunks] = {};
    auto piece = [&](int t) {
        const int64_t c0 = std::min(ub, t * per), c1 = std::min(ub, c0 + per);
        const float* src = raw + c0 * every * stride;
        const int64_t nn = std::min(n - c0 * every, (c1 - c0) * every);  // raw rows of the piece
        float* dst = d + c0 * stride;
        bool s = true;
        switch (stride) {  // the record width as a constant: the row copy unrolls, the loop stays branch-free
            case 4: k[t] = select_rows<4>(src, nn, every, blind2, p->time_field, dst, s, first[t], last[t]); break;
            case 5: k[t] = select_rows<5>(src, nn, every, blind2, p->time_field, dst, s, first[t], last[t]); break;
            case 6: k[t] = select_rows<6>(src, nn, every, blind2, p->time_field, dst, s, first[t], last[t]); break;
            case 7: k[t] = select_rows<7>(src, nn, every, blind2, p->time_field, dst, s, first[t], last[t]); break;
            default: k[t] = select_rows<8>(src, nn, every, blind2, p->time_field, dst, s, first[t], last[t]); break;
        }
        srt[t] = s;
    };
    if (pieces == 1) piece(0);
    else lio::HostPool::get().parallel_for(pieces, piece);
    bool sorted_ = true;
    uint32_t prev = 0;
    bool any = false;
    int64_t total = 0;
    plan->pieces = pieces;
    for (int t = 0; t < pieces; ++t) {
        plan->src_row[t] = std::min(ub, t * per);
        plan->rows[t] = k[t];
        total += k[t];
        if (!k[t]) continue;
        sorted_ = sorted_ && srt[t] && (!any || prev <= first[t]);  // and across the piece boundary
        prev = last[t];
        any = true;
    }
    if (np) std::memcpy(static_cast<uint8_t*>(b.h_stage) + *pose_off, poses, (size_t)np * sizeof(lio_imu_pose));
    *m = total;
    *sorted = sorted_;
    return LIO_OK;
}

// the staging buffer (the pieces with their gaps, then the IMU poses at pose_off) -> d_buf in one DMA; the
// piece table for the device (logical row -> staged row) and the poses' device address
static int upload_staged(const lio::FilterBuf& b, const StagePlan& plan, size_t pose_off, int np, float* d_buf,
                         hipStream_t st, lio::RowPieces* rp, const lio::ImuPose** d_poses) {
    const size_t bytes = pose_off + (size_t)np * sizeof(lio::ImuPose);
    if (bytes) HIP_TRY(hipMemcpyAsync(d_buf, b.h_stage, bytes, hipMemcpyHostToDevice, st));
    rp->n = std::max(plan.pieces, 1);
    uint32_t at = 0;
    for (int t = 0; t < plan.pieces; ++t) {
        rp->start[t] = at;
        rp->src[t] = (uint32_t)plan.src_row[t];
        at += (uint32_t)plan.rows[t];
    }
    *d_poses = reinterpret_cast<const lio::ImuPose*>(reinterpret_cast<const uint8_t*>(d_buf) + pose_off);
    return LIO_OK;
}

int lio_filter_create(int device, lio_filter** out) {
    if (!out) return fail(LIO_ERR_ARG, "out is NULL");
    *out = nullptr;
    int rc = check_device(device);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(device));
    auto* f = new lio_filter();
    f->dev = device;
    if (hipStreamCreateWithFlags(&f->st, hipStreamNonBlocking) != hipSuccess) {
        delete f;
        return fail(LIO_ERR_HIP, "hipStreamCreate failed");
    }
    *out = f;
    return LIO_OK;
}

int lio_filter_destroy(lio_filter* f) {
    if (!f) return LIO_OK;
    (void)hipSetDevice(f->dev);
    (void)hipStreamSynchronize(f->st);
    lio::filter_free(f->b);
    for (void* q : {(void*)f->d_in, (void*)f->d_out, (void*)f->d_seg, (void*)f->d_T, (void*)f->d_poses})
        if (q) (void)hipFree(q);
    (void)hipStreamDestroy(f->st);
    delete f;
    return LIO_OK;
}

int lio_voxel_grid(lio_filter* f, const float* pts, int64_t n, int stride, const float leaf[3], float* out,
                   int64_t* n_out) {
    if (!f || !leaf || !n_out || n < 0 || (n > 0 && (!pts || !out)) || stride < 3 || stride > lio::kMaxFields ||
        !(leaf[0] > 0.f && leaf[1] > 0.f && leaf[2] > 0.f))
        return fail(LIO_ERR_ARG, "lio_voxel_grid: bad arguments");
    *n_out = 0;
    if (n == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(f->dev));
    int rc = grow(&f->d_in, f->in_cap, n * stride);
    if (!rc) rc = grow(&f->d_out, f->out_cap, n * stride);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(f->d_in, pts, (size_t)n * stride * sizeof(float), hipMemcpyHostToDevice, f->st));
    int64_t m = 0;
    rc = lio::voxel_grid(f->b, f->d_in, n, stride, leaf, f->d_out, &m, f->st);
    if (rc) return filter_status(rc, "lio_voxel_grid");
    if (m) HIP_TRY(hipMemcpyAsync(out, f->d_out, (size_t)m * stride * sizeof(float), hipMemcpyDeviceToHost, f->st));
    HIP_TRY(hipStreamSynchronize(f->st));
    *n_out = m;
    return LIO_OK;
}

int lio_submap_voxelize(lio_filter* f, const float* pts, const int64_t* seg_off, int nk, int stride,
                        const double* poses16, float voxel_res, float* out, int64_t* n_out) {
    if (!f || !seg_off || !n_out || nk < 0 || stride < 3 || stride > lio::kMaxFields || !(voxel_res > 0.f) ||
        (nk > 0 && !poses16))
        return fail(LIO_ERR_ARG, "lio_submap_voxelize: bad arguments");
    *n_out = 0;
    const int64_t n = nk > 0 ? seg_off[nk] : 0;
    for (int k = 0; k < nk; ++k)
        if (seg_off[k] < 0 || seg_off[k + 1] < seg_off[k]) return fail(LIO_ERR_ARG, "lio_submap_voxelize: bad segments");
    if (seg_off[0] != 0) return fail(LIO_ERR_ARG, "lio_submap_voxelize: seg_off[0] must be 0");
    if (n == 0) return LIO_OK;
    if (!pts || !out) return fail(LIO_ERR_ARG, "lio_submap_voxelize: bad arguments");
    HIP_TRY(hipSetDevice(f->dev));
    // the loop leg's submaps change size on every loop timer call: the buffers are sized once for a C4-sized
    // submap (2 x 11 keyframes) and grow geometrically past it
    constexpr int64_t kSubmapFloor = (int64_t)1 << 19;
    f->b.min_cap = kSubmapFloor;
    const int64_t nf = std::max(n, kSubmapFloor);
    int rc = grow(&f->d_in, f->in_cap, nf * stride);
    if (!rc) rc = grow(&f->d_out, f->out_cap, 2 * nf * stride);
    if (!rc) rc = grow(&f->d_seg, f->seg_cap, std::max<int64_t>(nk + 1, 64));
    if (!rc) rc = grow(&f->d_T, f->T_cap, 16 * std::max<int64_t>(nk, 64));
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(f->d_in, pts, (size_t)n * stride * sizeof(float), hipMemcpyHostToDevice, f->st));
    HIP_TRY(hipMemcpyAsync(f->d_seg, seg_off, (size_t)(nk + 1) * sizeof(int64_t), hipMemcpyHostToDevice, f->st));
    HIP_TRY(hipMemcpyAsync(f->d_T, poses16, (size_t)nk * 16 * sizeof(double), hipMemcpyHostToDevice, f->st));
    float* d_tf = f->d_out + (size_t)n * stride;  // transformed, concatenated cloud
    rc = lio::transform_segments(f->d_in, n, stride, f->d_seg, nk, f->d_T, d_tf, f->st);
    if (rc) return filter_status(rc, "lio_submap_voxelize");
    const float leaf[3] = {voxel_res, voxel_res, voxel_res};
    int64_t m = 0;
    rc = lio::voxel_grid(f->b, d_tf, n, stride, leaf, f->d_out, &m, f->st);
    if (rc) return filter_status(rc, "lio_submap_voxelize");
    if (m) HIP_TRY(hipMemcpyAsync(out, f->d_out, (size_t)m * stride * sizeof(float), hipMemcpyDeviceToHost, f->st));
    HIP_TRY(hipStreamSynchronize(f->st));
    *n_out = m;
    return LIO_OK;
}

static int prep_args_ok(const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                        const lio_imu_pose* poses, int n_poses) {
    if (!p || n < 0 || (n > 0 && !raw) || stride < 4 || stride > lio::kMaxFields || p->time_field < 3 ||
        p->time_field >= stride || n_poses < 0 || (n_poses > 0 && !poses) || n >= (int64_t)1 << 30)
        return fail(LIO_ERR_ARG, "scan preprocessing: bad arguments");
    return LIO_OK;
}

int lio_preprocess(lio_filter* f, const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                   const lio_imu_pose* poses, int n_poses, const lio_pose* end, float* out, int64_t* n_out) {
    if (!f || !n_out || (n > 0 && !out)) return fail(LIO_ERR_ARG, "lio_preprocess: bad arguments");
    int rc = prep_args_ok(raw, n, stride, p, poses, n_poses);
    if (rc) return rc;
    *n_out = 0;
    if (n == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(f->dev));
    hipStream_t st = f->st;
    lio::ScanPrepParams sp{p->point_filter_num, p->blind, p->filter_size_surf, p->time_field};
    int64_t rows = n;
    size_t pose_off = 0;
    StagePlan plan;
    bool sorted = false;
    rc = stage_sweep_select(f->b, raw, n, stride, p, poses, n_poses, &rows, &pose_off, &sorted, &plan);
    if (rc) return rc;
    const int presel = sorted ? 1 : 0;
    if (rows == 0) return LIO_OK;
    const size_t staged = pose_off + (size_t)n_poses * sizeof(lio::ImuPose);
    rc = grow(&f->d_in, f->in_cap, (int64_t)((staged + 3) / 4) + 1);
    if (!rc) rc = grow(&f->d_out, f->out_cap, rows * stride);
    if (rc) return rc;
    lio::RowPieces rp;
    const lio::ImuPose* d_poses = f->d_poses;
    rc = upload_staged(f->b, plan, pose_off, n_poses, f->d_in, st, &rp, &d_poses);
    if (rc) return rc;
    int64_t m = 0;
    rc = 2;
    for (int attempt = 0; attempt < 2 && rc == 2; ++attempt) {  // 2: the voxel key width was learnt too narrow
        rc = lio::scan_preprocess_enqueue(f->b, f->d_in, rows, stride, sp, d_poses, n_poses, undistort_end(end),
                                          f->d_out, st, presel, nullptr, nullptr, rp);
        if (!rc) rc = lio::scan_preprocess_finish(f->b, stride, f->d_out, &m, nullptr, st);
    }
    if (rc == 2) rc = -2;
    if (rc < 0) {
        (void)hipStreamSynchronize(st);  // the staging buffer is reused by the next call
        return filter_status(rc, "lio_preprocess");
    }
    if (m) HIP_TRY(hipMemcpyAsync(out, f->d_out, (size_t)m * stride * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *n_out = m;
    return LIO_OK;
}

// LIO_PREP_PROFILE=1 (diagnostics): host-side phases of every lio_scan_preprocess on stderr
static bool prep_profile() {
    static const bool on = std::getenv("LIO_PREP_PROFILE") != nullptr;
    return on;
}
static double prep_us(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

// the device half shared by lio_scan_preprocess and lio_scan_preprocess_cloud2: c->d_raw holds `rows`
// records; every stage is queued, the scan buffers set up behind it, and the host waits once
static int scan_prep_device(lio_ctx* c, int64_t rows, int stride, const lio::ScanPrepParams& sp, int n_poses,
                            const lio_pose* end, int64_t* n_down, const char* what, int presel = -1,
                            const lio::ImuPose* d_poses = nullptr, const lio::RowPieces& rp = lio::RowPieces{}) {
    if (!d_poses) d_poses = c->d_poses;
    hipStream_t st = c->map->st;
    c->undist_n = -1;
    auto bail = [&](int r) {
        (void)hipStreamSynchronize(st);  // nothing queued may outlive the call (the staging buffer is reused)
        return r;
    };
    int rc = ctx_reserve(c, rows);  // sized for the row bound; c->n set to the count below
    if (rc) return bail(rc);
    int64_t m = 0, mu = 0;
    rc = 2;
    for (int attempt = 0; attempt < 2 && rc == 2; ++attempt) {  // 2: the voxel key width was learnt too narrow
        const bool vox = sp.leaf > 0.f;  // the centroid pass writes the scan's xyz and flags itself
        rc = lio::scan_preprocess_enqueue(c->filt, c->d_raw, rows, stride, sp, d_poses, n_poses,
                                          undistort_end(end), c->d_rec, st, presel, vox ? c->d_body : nullptr,
                                          vox ? c->d_sel : nullptr, rp);
        if (rc) return bail(filter_status(rc, what));
        if (!vox) rc = lio::records_to_xyz_sel(c->d_rec, rows, stride, c->d_body, c->d_sel, st);
        if (rc) return bail(filter_status(rc, what));
        const auto tw = std::chrono::steady_clock::now();
        rc = lio::scan_preprocess_finish(c->filt, stride, c->d_rec, &m, &mu, st);
        if (prep_profile())
            std::fprintf(stderr, "prep_profile wait_us %.1f attempt %d\n", prep_us(tw, std::chrono::steady_clock::now()),
                         attempt);
    }
    if (rc == 2) rc = -2;
    if (rc < 0) return bail(filter_status(rc, what));
    if (rc == 1) {  // VoxelGrid index overflow: the output is the undistorted input, its xyz again
        rc = lio::records_to_xyz_sel(c->d_rec, m, stride, c->d_body, c->d_sel, st);
        if (rc) return bail(filter_status(rc, what));
        HIP_TRY(hipStreamSynchronize(st));
    }
    c->n = m;
    c->undist_n = mu;
    c->undist_stride = stride;
    if (n_down) *n_down = m;
    return LIO_OK;
}

int lio_scan_preprocess(lio_ctx* c, const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                        const lio_imu_pose* poses, int n_poses, const lio_pose* end, int64_t* n_down) {
    if (!c) return fail(LIO_ERR_ARG, "lio_scan_preprocess: NULL ctx");
    int rc = prep_args_ok(raw, n, stride, p, poses, n_poses);
    if (rc) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    lio::ScanPrepParams sp{p->point_filter_num, p->blind, p->filter_size_surf, p->time_field};
    int64_t rows = n;
    size_t pose_off = 0;
    StagePlan plan;
    bool sorted = false;
    rc = stage_sweep_select(c->filt, raw, n, stride, p, poses, n_poses, &rows, &pose_off, &sorted, &plan);
    if (rc) return rc;
    const int presel = sorted ? 1 : 0;
    const auto t1 = std::chrono::steady_clock::now();
    // staged: the pieces (with their gaps) and the poses behind them in one DMA into d_raw
    const size_t staged = pose_off + (size_t)n_poses * sizeof(lio::ImuPose);
    rc = grow(&c->d_raw, c->raw_cap, (int64_t)((staged + 3) / 4) + 1);
    if (!rc) rc = grow(&c->d_rec, c->rec_cap, std::max<int64_t>(rows, 1) * stride);
    if (rc) return rc;
    lio::RowPieces rp;
    const lio::ImuPose* d_poses = c->d_poses;
    rc = upload_staged(c->filt, plan, pose_off, n_poses, c->d_raw, st, &rp, &d_poses);
    if (rc) return rc;
    const auto t2 = std::chrono::steady_clock::now();
    rc = scan_prep_device(c, rows, stride, sp, n_poses, end, n_down, "lio_scan_preprocess", presel, d_poses, rp);
    if (prep_profile()) {
        const auto t3 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "prep_profile rows %lld presel %d stage_us %.1f upload_enqueue_us %.1f device_us %.1f total_us %.1f\n",
                     (long long)rows, presel, prep_us(t0, t1), prep_us(t1, t2), prep_us(t2, t3), prep_us(t0, t3));
    }
    return rc;
}

int lio_scan_get_undistorted(lio_ctx* c, float* out, int64_t cap_points, int64_t* n_points, int* stride) {
    if (!c || !n_points) return fail(LIO_ERR_ARG, "lio_scan_get_undistorted: bad arguments");
    if (c->undist_n < 0) return fail(LIO_ERR_STATE, "lio_scan_get_undistorted: no lio_scan_preprocess* on this ctx");
    *n_points = c->undist_n;
    if (stride) *stride = c->undist_stride;
    if (!out || c->undist_n == 0) return LIO_OK;
    if (cap_points < c->undist_n) return fail(LIO_ERR_ARG, "lio_scan_get_undistorted: out too small");
    HIP_TRY(hipSetDevice(c->map->dev));
    HIP_TRY(hipMemcpyAsync(out, c->filt.c, (size_t)c->undist_n * c->undist_stride * sizeof(float),
                           hipMemcpyDeviceToHost, c->map->st));
    HIP_TRY(hipStreamSynchronize(c->map->st));
    return LIO_OK;
}

int lio_scan_keyframe_cloud(lio_ctx* c, const lio_pose* pose, const double* T16, float* out, int64_t cap_points,
                            int64_t* n_points) {
    if (!c || !pose || !T16 || !n_points) return fail(LIO_ERR_ARG, "lio_scan_keyframe_cloud: bad arguments");
    if (c->undist_n < 0) return fail(LIO_ERR_STATE, "lio_scan_keyframe_cloud: no lio_scan_preprocess* on this ctx");
    *n_points = c->undist_n;
    if (!out || c->undist_n == 0) return LIO_OK;
    if (cap_points < c->undist_n) return fail(LIO_ERR_ARG, "lio_scan_keyframe_cloud: out too small");
    HIP_TRY(hipSetDevice(c->map->dev));
    int rc = grow(&c->d_kf, c->kf_cap, c->undist_n * 4);
    if (rc) return rc;
    lio::PoseArg ps;
    const lio_pose pf = filled(*pose);  // matrix-only callers: q / q_LI derived from R / R_LI (body_to_world rotates with them)
    std::memcpy(&ps, &pf, sizeof(ps));
    if (lio::keyframe_cloud(c->filt.c, c->undist_n, c->undist_stride, ps, T16, c->d_kf, c->map->st))
        return fail(LIO_ERR_HIP, "keyframe cloud kernel failed");
    HIP_TRY(hipMemcpyAsync(out, c->d_kf, (size_t)c->undist_n * 4 * sizeof(float), hipMemcpyDeviceToHost, c->map->st));
    HIP_TRY(hipStreamSynchronize(c->map->st));
    return LIO_OK;
}

// =============================================================================
// wire / disk formats
// =============================================================================
static_assert(sizeof(lio_cloud_field) == sizeof(lio::CloudField), "lio_cloud_field layout");

int lio_cloud2_decode(lio_filter* f, const uint8_t* data, int64_t n_points, int32_t point_step, int is_bigendian,
                      const lio_cloud_field* fields, int n_fields, float* out) {
    if (!f || n_points < 0 || (n_points > 0 && (!data || !out)) || point_step <= 0 || !fields || n_fields < 1 ||
        n_fields > lio::kMaxFields)
        return fail(LIO_ERR_ARG, "lio_cloud2_decode: bad arguments");
    for (int k = 0; k < n_fields; ++k) {
        const int dt = fields[k].datatype;
        const int size = dt <= 2 ? 1 : dt <= 4 ? 2 : dt <= 7 ? 4 : 8;
        if (dt < 0 || dt > 8 || (dt && (fields[k].offset < 0 || fields[k].offset + size > point_step)))
            return fail(LIO_ERR_ARG, "lio_cloud2_decode: field outside the record");
    }
    if (n_points == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(f->dev));
    const int64_t bytes = n_points * point_step;
    int rc = grow(&f->d_in, f->in_cap, (bytes + 3) / 4);
    if (!rc) rc = grow(&f->d_out, f->out_cap, n_points * n_fields);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(f->d_in, data, (size_t)bytes, hipMemcpyHostToDevice, f->st));
    rc = lio::cloud_decode(reinterpret_cast<const uint8_t*>(f->d_in), n_points, point_step, is_bigendian != 0,
                           reinterpret_cast<const lio::CloudField*>(fields), n_fields, f->d_out, f->st);
    if (rc) return filter_status(rc, "lio_cloud2_decode");
    HIP_TRY(hipMemcpyAsync(out, f->d_out, (size_t)n_points * n_fields * sizeof(float), hipMemcpyDeviceToHost, f->st));
    HIP_TRY(hipStreamSynchronize(f->st));
    return LIO_OK;
}

int lio_cloud2_encode(lio_filter* f, const float* rec, int64_t n, int stride, const lio_cloud_field* fields,
                      int n_fields, int32_t point_step, uint8_t* data) {
    if (!f || n < 0 || (n > 0 && (!rec || !data)) || stride < 1 || !fields || n_fields < 1 ||
        n_fields > lio::kMaxFields || point_step <= 0)
        return fail(LIO_ERR_ARG, "lio_cloud2_encode: bad arguments");
    for (int k = 0; k < n_fields; ++k)
        if (fields[k].datatype == 7 && (fields[k].offset < 0 || fields[k].offset + 4 > point_step))
            return fail(LIO_ERR_ARG, "lio_cloud2_encode: field outside the record");
    if (n == 0) return LIO_OK;
    HIP_TRY(hipSetDevice(f->dev));
    const int64_t bytes = n * point_step;
    int rc = grow(&f->d_in, f->in_cap, n * stride);
    if (!rc) rc = grow(&f->d_out, f->out_cap, (bytes + 3) / 4);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(f->d_in, rec, (size_t)n * stride * sizeof(float), hipMemcpyHostToDevice, f->st));
    rc = lio::cloud_encode(f->d_in, n, stride, point_step, reinterpret_cast<const lio::CloudField*>(fields), n_fields,
                           reinterpret_cast<uint8_t*>(f->d_out), f->st);
    if (rc) return filter_status(rc, "lio_cloud2_encode");
    HIP_TRY(hipMemcpyAsync(data, f->d_out, (size_t)bytes, hipMemcpyDeviceToHost, f->st));
    HIP_TRY(hipStreamSynchronize(f->st));
    return LIO_OK;
}

int lio_scan_preprocess_cloud2(lio_ctx* c, const uint8_t* data, int64_t n_points, int32_t point_step,
                               int is_bigendian, const lio_cloud_field fields[5], const lio_scan_prep_params* p,
                               const lio_imu_pose* poses, int n_poses, const lio_pose* end, int64_t* n_down) {
    if (!c || !fields || point_step <= 0 || n_points < 0 || (n_points > 0 && !data))
        return fail(LIO_ERR_ARG, "lio_scan_preprocess_cloud2: bad arguments");
    lio_scan_prep_params pp = p ? *p : lio_scan_prep_params{1, 0.f, 0.f, 4};
    pp.time_field = 4;
    int rc = prep_args_ok(nullptr, 0, 5, &pp, poses, n_poses);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->map->dev));
    hipStream_t st = c->map->st;
    lio::ScanPrepParams sp{pp.point_filter_num, pp.blind, pp.filter_size_surf, 4};
    int64_t rows = n_points;
    size_t pose_off = 0;
    // the records Preprocess keeps by index, still packed
    rc = stage_sweep(c->filt, data, n_points, (size_t)point_step, pp.point_filter_num, poses, n_poses, &rows, &pose_off);
    if (rc) return rc;
    sp.point_filter_num = 1;
    const int64_t bytes = rows * point_step;
    rc = grow(&c->d_rec, c->rec_cap, std::max<int64_t>((bytes + 3) / 4, rows * 5 + 1));  // staging for the bytes
    if (!rc) rc = grow(&c->d_raw, c->raw_cap, std::max<int64_t>(rows, 1) * 5);
    if (!rc && n_poses) rc = grow(&c->d_poses, c->poses_cap, n_poses);
    if (rc) return rc;
    const auto* stage = static_cast<const uint8_t*>(c->filt.h_stage);
    if (rows)
        HIP_TRY(hipMemcpyAsync(c->d_rec, stage, (size_t)bytes, hipMemcpyHostToDevice, st));
    if (n_poses)
        HIP_TRY(hipMemcpyAsync(c->d_poses, stage + pose_off,
                               (size_t)n_poses * sizeof(lio::ImuPose), hipMemcpyHostToDevice, st));
    rc = lio::cloud_decode(reinterpret_cast<const uint8_t*>(c->d_rec), rows, point_step, is_bigendian != 0,
                           reinterpret_cast<const lio::CloudField*>(fields), 5, c->d_raw, st);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return filter_status(rc, "lio_scan_preprocess_cloud2");
    }
    return scan_prep_device(c, rows, 5, sp, n_poses, end, n_down, "lio_scan_preprocess_cloud2");
}

int lio_pcd_write_binary(const char* path, const float* rec, int64_t n, int stride, const char* const* names) {
    if (!path || n < 0 || (n > 0 && !rec) || stride < 1 || stride > 16 || !names)
        return fail(LIO_ERR_ARG, "lio_pcd_write_binary: bad arguments");
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return fail(LIO_ERR_ARG, std::string("lio_pcd_write_binary: cannot open ") + path);
    std::string h = "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS";
    for (int k = 0; k < stride; ++k) h += std::string(" ") + names[k];
    h += "\nSIZE";
    for (int k = 0; k < stride; ++k) h += " 4";
    h += "\nTYPE";
    for (int k = 0; k < stride; ++k) h += " F";
    h += "\nCOUNT";
    for (int k = 0; k < stride; ++k) h += " 1";
    h += "\nWIDTH " + std::to_string(n) + "\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS " + std::to_string(n) +
         "\nDATA binary\n";
    bool ok = std::fwrite(h.data(), 1, h.size(), fp) == h.size();
    if (ok && n) ok = std::fwrite(rec, sizeof(float) * stride, (size_t)n, fp) == (size_t)n;
    ok = (std::fclose(fp) == 0) && ok;
    return ok ? LIO_OK : fail(LIO_ERR_ARG, "lio_pcd_write_binary: write failed");
}

namespace {
struct PcdHeader {
    std::vector<std::string> names;
    std::vector<int> sizes, counts;
    std::vector<char> types;
    int64_t points = 0;
    std::string data;
    long data_pos = 0;
};

int pcd_parse(FILE* fp, PcdHeader& h) {
    char line[4096];
    while (std::fgets(line, sizeof(line), fp)) {
        std::string l(line);
        while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
        if (l.empty() || l[0] == '#') continue;
        std::vector<std::string> tok;
        size_t a = 0;
        while (a < l.size()) {
            size_t b = l.find_first_of(" \t", a);
            if (b == std::string::npos) b = l.size();
            if (b > a) tok.push_back(l.substr(a, b - a));
            a = b + 1;
        }
        if (tok.empty()) continue;
        const std::string& k = tok[0];
        if (k == "FIELDS") h.names.assign(tok.begin() + 1, tok.end());
        else if (k == "SIZE") for (size_t i = 1; i < tok.size(); ++i) h.sizes.push_back(std::atoi(tok[i].c_str()));
        else if (k == "TYPE") for (size_t i = 1; i < tok.size(); ++i) h.types.push_back(tok[i][0]);
        else if (k == "COUNT") for (size_t i = 1; i < tok.size(); ++i) h.counts.push_back(std::atoi(tok[i].c_str()));
        else if (k == "POINTS" && tok.size() > 1) h.points = std::atoll(tok[1].c_str());
        else if (k == "DATA" && tok.size() > 1) {
            h.data = tok[1];
            h.data_pos = std::ftell(fp);
            break;
        }
    }
    if (h.counts.empty()) h.counts.assign(h.names.size(), 1);
    if (h.data.empty() || h.names.size() != h.sizes.size() || h.names.size() != h.types.size() ||
        h.names.size() != h.counts.size())
        return -1;
    return 0;
}

int pcd_datatype(char t, int size) {
    if (t == 'F') return size == 4 ? 7 : size == 8 ? 8 : 0;
    if (t == 'I') return size == 1 ? 1 : size == 2 ? 3 : size == 4 ? 5 : 0;
    if (t == 'U') return size == 1 ? 2 : size == 2 ? 4 : size == 4 ? 6 : 0;
    return 0;
}
}  // namespace

int lio_pcd_read(lio_filter* f, const char* path, const char* const* want, int n_want, float* out, int64_t cap,
                 int64_t* n_points) {
    if (!path || !n_points || (out && (!f || !want || n_want < 1 || n_want > lio::kMaxFields)))
        return fail(LIO_ERR_ARG, "lio_pcd_read: bad arguments");
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(LIO_ERR_ARG, std::string("lio_pcd_read: cannot open ") + path);
    PcdHeader h;
    if (pcd_parse(fp, h)) {
        std::fclose(fp);
        return fail(LIO_ERR_ARG, "lio_pcd_read: malformed header");
    }
    *n_points = h.points;
    if (!out) {
        std::fclose(fp);
        return LIO_OK;
    }
    if (h.points > cap) {
        std::fclose(fp);
        return fail(LIO_ERR_ARG, "lio_pcd_read: out too small");
    }
    // column layout of one record
    std::vector<int> off(h.names.size());
    int step = 0;
    for (size_t k = 0; k < h.names.size(); ++k) {
        off[k] = step;
        step += h.sizes[k] * h.counts[k];
    }
    std::vector<lio::CloudField> fl(n_want, lio::CloudField{0, 0, 1.f});
    std::vector<int> col(n_want, -1);
    for (int w = 0; w < n_want; ++w)
        for (size_t k = 0; k < h.names.size(); ++k)
            if (h.names[k] == want[w]) {
                fl[w] = lio::CloudField{off[k], pcd_datatype(h.types[k], h.sizes[k]), 1.f};
                col[w] = (int)k;
            }
    int rc = LIO_OK;
    if (h.data == "binary") {
        std::vector<uint8_t> buf((size_t)h.points * step);
        const bool ok = h.points == 0 || std::fread(buf.data(), (size_t)step, (size_t)h.points, fp) == (size_t)h.points;
        std::fclose(fp);
        if (!ok) return fail(LIO_ERR_ARG, "lio_pcd_read: truncated data");
        rc = lio_cloud2_decode(f, buf.data(), h.points, step, 0, reinterpret_cast<const lio_cloud_field*>(fl.data()),
                               n_want, out);
    } else if (h.data == "ascii") {
        // one record per line, COUNT values per field, parsed as float (strtof)
        std::vector<int> first(h.names.size());
        int nv = 0;
        for (size_t k = 0; k < h.names.size(); ++k) {
            first[k] = nv;
            nv += h.counts[k];
        }
        char line[1 << 16];
        int64_t i = 0;
        while (i < h.points && std::fgets(line, sizeof(line), fp)) {
            std::vector<float> v;
            char* p = line;
            char* e = nullptr;
            for (int t = 0; t < nv; ++t) {
                const float x = std::strtof(p, &e);
                if (e == p) break;
                v.push_back(x);
                p = e;
            }
            if ((int)v.size() < nv) continue;
            for (int w = 0; w < n_want; ++w) out[i * n_want + w] = col[w] >= 0 ? v[first[col[w]]] : 0.f;
            ++i;
        }
        std::fclose(fp);
        if (i != h.points) return fail(LIO_ERR_ARG, "lio_pcd_read: truncated ascii data");
    } else {
        std::fclose(fp);
        return fail(LIO_ERR_ARG, "lio_pcd_read: DATA " + h.data + " unsupported (ascii | binary)");
    }
    return rc;
}

int lio_map_build_pcd(lio_map* m, const char* path) {
    if (!m || !path) return fail(LIO_ERR_ARG, "lio_map_build_pcd: bad arguments");
    int64_t n = 0;
    int rc = lio_pcd_read(nullptr, path, nullptr, 0, nullptr, 0, &n);
    if (rc) return rc;
    if (n <= 0) return fail(LIO_ERR_ARG, "lio_map_build_pcd: empty cloud");
    lio_filter* f = nullptr;
    rc = lio_filter_create(m->dev, &f);
    if (rc) return rc;
    std::vector<float> xyz((size_t)n * 3);
    const char* want[3] = {"x", "y", "z"};
    rc = lio_pcd_read(f, path, want, 3, xyz.data(), n, &n);
    lio_filter_destroy(f);
    if (rc) return rc;
    return lio_map_build(m, xyz.data(), n);
}

// =============================================================================
// timing
// =============================================================================
int lio_ctx_set_timing(lio_ctx* c, int enable) {
    if (!c) return fail(LIO_ERR_ARG, "NULL ctx");
    c->timing = enable != 0;
    return LIO_OK;
}
int lio_ctx_get_timing(lio_ctx* c, lio_kernel_timing* out) {
    if (!c || !out) return fail(LIO_ERR_ARG, "bad arguments");
    *out = c->tm;
    return LIO_OK;
}
int lio_ctx_reset_timing(lio_ctx* c) {
    if (!c) return fail(LIO_ERR_ARG, "NULL ctx");
    c->tm = lio_kernel_timing{};
    return LIO_OK;
}

}  // extern "C"
