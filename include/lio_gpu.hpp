// lio_gpu.hpp — C++ host-side mirror of the reference interfaces over the
// C-ABI in lio_gpu.h (header-only; link liblio_gpu.so).
//
// What a FAST-LIO-SAM maintainer swaps in, under the reference's own names:
//   * KdTreeGPU<PointType>   ~ ikd-Tree `KD_TREE<PointType>` [U: ikd_Tree.h]:
//       Build, Nearest_Search (single point and batch), Add_Points,
//       Delete_Point_Boxes, size, validnum, flatten, set_downsample_param
//   * ScanMatcherGPU          ~ laserMapping.cpp h_share_model +
//       kf.update_iterated_dyn_share_modified(LASER_POINT_COV, solve_time)
//       + map_incremental() + lasermap_fov_segment() [U]
//   * LoopClosureICP          ~ LoopClosure::icpAlignment
//       (fast_lio_sam/src/loop_closure.cpp:69-92, loop_closure.h:31-37)
//   * VoxelGrid<PointT>, submap_voxelize, preprocess_scan, savePCDFileBinary,
//     loadPCDFile ~ pcl::VoxelGrid, setSrcAndDstCloud's transformPcd +
//     voxelizePcd, Preprocess + UndistortPcl, pcl::io PCD I/O
// PointType is any struct with float members x, y, z (pcl::PointXYZI,
// pcl::PointXYZINormal, ...).  Errors throw lio_gpu::Error carrying
// lio_last_error(); there is no CPU fallback behind any call.
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "lio_gpu.h"

namespace lio_gpu {

struct Error : std::runtime_error {
    int code;
    Error(int rc, const std::string& what) : std::runtime_error(what), code(rc) {}
};

inline void check(int rc, const char* where) {
    if (rc != LIO_OK) throw Error(rc, std::string(where) + ": " + lio_last_error());
}

// ikd-Tree's BoxPointType (vertex_min / vertex_max), min <= p < max
struct BoxPointType {
    float vertex_min[3];
    float vertex_max[3];
};

template <typename P>
std::vector<float> packed_xyz(const std::vector<P>& pts) {
    std::vector<float> xyz(pts.size() * 3);
    for (size_t i = 0; i < pts.size(); ++i) {
        xyz[3 * i] = pts[i].x;
        xyz[3 * i + 1] = pts[i].y;
        xyz[3 * i + 2] = pts[i].z;
    }
    return xyz;
}

// floats per record of a POD point type: 3..8 floats, x, y, z first
template <typename PointT>
constexpr int float_stride() {
    static_assert(sizeof(PointT) % sizeof(float) == 0 && sizeof(PointT) >= 3 * sizeof(float) &&
                      sizeof(PointT) <= 8 * sizeof(float),
                  "PointT must be 3..8 floats (x, y, z first)");
    return (int)(sizeof(PointT) / sizeof(float));
}

// Eigen::Quaterniond::toRotationMatrix for (w, x, y, z), row-major
inline void quat_to_rot(const double q[4], double R[9]) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz), R[1] = txy - twz, R[2] = txz + twy;
    R[3] = txy + twz, R[4] = 1 - (txx + tzz), R[5] = tyz - twx;
    R[6] = txz - twy, R[7] = tyz + twx, R[8] = 1 - (txx + tyy);
}

// the parts of state_ikfom the measurement model reads
inline lio_pose pose_of(const lio_state& x) {
    lio_pose p{};
    quat_to_rot(x.rot, p.R);
    quat_to_rot(x.offset_R_L_I, p.R_LI);
    for (int k = 0; k < 4; ++k) {
        p.q[k] = x.rot[k];
        p.q_LI[k] = x.offset_R_L_I[k];
    }
    for (int k = 0; k < 3; ++k) {
        p.t[k] = x.pos[k];
        p.t_LI[k] = x.offset_T_L_I[k];
    }
    return p;
}

// ---------------------------------------------------------------------------
// KD_TREE<PointType> surface used by laserMapping.cpp, on the device grid.
// Ids are insertion order; deleted points stay as tombstoned ids.
template <typename PointType>
class KdTreeGPU {
public:
    using PointVector = std::vector<PointType>;

    explicit KdTreeGPU(float cell_size = 1.0f, float downsample_size = 0.5f, int device = 0)
        : cell_(cell_size), dev_(device) {
        lio_map_params p{cell_size, downsample_size, device, 0};
        check(lio_map_create(&p, &m_), "lio_map_create");
    }
    ~KdTreeGPU() { lio_map_destroy(m_); }
    KdTreeGPU(const KdTreeGPU&) = delete;
    KdTreeGPU& operator=(const KdTreeGPU&) = delete;

    // ikdtree.set_downsample_param(filter_size_map_min): changes the map's
    // parameters in place (ScanMatcherGPU objects built on this tree stay
    // valid); call before Build, as laserMapping does
    void set_downsample_param(float ds) {
        lio_map_params p{0.f, ds, dev_, 0};
        check(lio_map_set_params(m_, &p), "set_downsample_param");
    }

    void Build(const PointVector& pts) {
        const std::vector<float> xyz = packed_xyz(pts);
        check(lio_map_build(m_, xyz.data(), (int64_t)pts.size()), "Build");
    }

    // single query, as h_share_model calls it (k = 5, max_dist = INFINITY);
    // prefer the batch form or ScanMatcherGPU on hot loops
    void Nearest_Search(const PointType& point, int k_nearest, PointVector& Nearest_Points,
                        std::vector<float>& Point_Distance, double max_dist = INFINITY) {
        std::vector<int32_t> ids;
        Nearest_Search_Batch(PointVector{point}, k_nearest, ids, Point_Distance, max_dist);
        resolve(ids, Nearest_Points);
        size_t found = 0;
        while (found < ids.size() && ids[found] >= 0) ++found;
        Point_Distance.resize(found);
    }

    // batch: ids (n*k, -1 where fewer exist) and sq-distances (n*k, +inf where missing)
    void Nearest_Search_Batch(const PointVector& q, int k_nearest, std::vector<int32_t>& ids,
                              std::vector<float>& sq_dist, double max_dist = INFINITY) {
        const std::vector<float> xyz = packed_xyz(q);
        ids.resize(q.size() * k_nearest);
        sq_dist.resize(q.size() * k_nearest);
        check(lio_map_nearest_search(m_, xyz.data(), (int64_t)q.size(), k_nearest, (float)max_dist, ids.data(),
                                     sq_dist.data()),
              "Nearest_Search");
    }

    // ikdtree.Add_Points(PointToAdd, downsample_on): the reference's return value
    int Add_Points(const PointVector& pts, bool downsample_on) {
        const std::vector<float> xyz = packed_xyz(pts);
        int64_t n = 0;
        check(lio_map_add(m_, xyz.data(), (int64_t)pts.size(), downsample_on ? 1 : 0, &n), "Add_Points");
        return (int)n;
    }

    int Delete_Point_Boxes(const std::vector<BoxPointType>& boxes) {
        std::vector<float> b(boxes.size() * 6);
        for (size_t i = 0; i < boxes.size(); ++i)
            for (int d = 0; d < 3; ++d) {
                b[6 * i + d] = boxes[i].vertex_min[d];
                b[6 * i + 3 + d] = boxes[i].vertex_max[d];
            }
        int64_t n = 0;
        check(lio_map_delete_boxes(m_, b.data(), (int)boxes.size(), &n), "Delete_Point_Boxes");
        return (int)n;
    }

    int size() const { return (int)lio_map_num_ids(m_); }   // ikd-Tree size(): nodes incl. deleted
    int validnum() const { return (int)lio_map_size(m_); }  // alive points

    // ikdtree.flatten(Root_Node, PCL_Storage, NOT_RECORD): the alive points (id order)
    void flatten(PointVector& storage) {
        std::vector<float> xyz;
        std::vector<uint8_t> alive;
        by_id(xyz, alive);
        storage.clear();
        for (size_t i = 0; i < alive.size(); ++i)
            if (alive[i]) storage.push_back(make_point(&xyz[3 * i]));
    }

    // every id's coordinates + alive flag (kNN ids index this)
    void by_id(std::vector<float>& xyz, std::vector<uint8_t>& alive) {
        const int64_t n = lio_map_num_ids(m_);
        xyz.resize((size_t)n * 3);
        alive.resize((size_t)n);
        check(lio_map_get_by_id(m_, xyz.data(), alive.data()), "by_id");
    }

    // ids -> points (Nearest_Points), skipping -1
    void resolve(const std::vector<int32_t>& ids, PointVector& out) {
        std::vector<int32_t> valid;
        for (int32_t id : ids)
            if (id >= 0) valid.push_back(id);
        std::vector<float> xyz(valid.size() * 3);
        check(lio_map_gather(m_, valid.data(), (int64_t)valid.size(), xyz.data()), "resolve");
        out.clear();
        for (size_t i = 0; i < valid.size(); ++i) out.push_back(make_point(&xyz[3 * i]));
    }

    lio_map* handle() { return m_; }

private:
    static PointType make_point(const float* p) {
        PointType q{};
        q.x = p[0];
        q.y = p[1];
        q.z = p[2];
        return q;
    }
    lio_map* m_ = nullptr;
    float cell_ = 1.0f;
    int dev_ = 0;
};

// ---------------------------------------------------------------------------
// h_share_model + IESKF update + map maintenance for one map.
class ScanMatcherGPU {
public:
    template <typename P>
    explicit ScanMatcherGPU(KdTreeGPU<P>& tree, const lio_match_params& p = defaults()) {
        check(lio_ctx_create(tree.handle(), &p, &c_), "lio_ctx_create");
    }
    ~ScanMatcherGPU() { lio_ctx_destroy(c_); }
    ScanMatcherGPU(const ScanMatcherGPU&) = delete;
    ScanMatcherGPU& operator=(const ScanMatcherGPU&) = delete;

    static lio_match_params defaults() { return lio_match_params{5.0f, 0.1f, 0.9, 0.9}; }

    // feats_down_body
    template <typename P>
    void set_scan(const std::vector<P>& feats_down_body) {
        const std::vector<float> xyz = packed_xyz(feats_down_body);
        check(lio_scan_set(c_, xyz.data(), (int64_t)feats_down_body.size()), "set_scan");
    }

    // raw scan -> Preprocess + UndistortPcl + downSizeFilterSurf -> feats_down_body on the device
    template <typename PointT>
    int64_t set_scan_raw(const std::vector<PointT>& raw, const lio_scan_prep_params& params,
                         const std::vector<lio_imu_pose>& imu_poses, const lio_state& end_state) {
        const lio_pose end = pose_of(end_state);
        int64_t n = 0;
        check(lio_scan_preprocess(c_, reinterpret_cast<const float*>(raw.data()), (int64_t)raw.size(),
                                  float_stride<PointT>(), &params, imu_poses.data(), (int)imu_poses.size(), &end, &n),
              "set_scan_raw");
        return n;
    }

    // the same from float records (n x stride, the time offset at params.time_field) and the scan-end pose
    int64_t set_scan_raw(const float* raw, int64_t n, int stride, const lio_scan_prep_params& params,
                         const lio_imu_pose* imu_poses, int n_poses, const lio_pose& end) {
        int64_t m = 0;
        check(lio_scan_preprocess(c_, raw, n, stride, &params, imu_poses, n_poses, &end, &m), "set_scan_raw");
        return m;
    }

    // feats_undistort of the last set_scan_raw (n x *stride records, before downSizeFilterSurf)
    std::vector<float> undistorted(int* stride = nullptr) {
        int64_t n = 0;
        int w = 0;
        check(lio_scan_get_undistorted(c_, nullptr, 0, &n, &w), "undistorted");
        std::vector<float> out((size_t)n * (size_t)std::max(w, 1));
        check(lio_scan_get_undistorted(c_, out.data(), n, &n, &w), "undistorted");
        if (stride) *stride = w;
        return out;
    }

    // fast_lio_sam's keyframe cloud from FAST-LIO's /cloud_registered, built on the device: T16 (row-major)
    // * pointBodyToWorld(x, feats_undistort), intensity kept — PosePcd::pcd_ with T16 = pose_eig_.inverse()
    // (pose_pcd.hpp:22-42)
    template <typename PointXYZI_T>
    std::vector<PointXYZI_T> keyframe_cloud(const lio_state& x, const double T16[16]) {
        static_assert(sizeof(PointXYZI_T) == 4 * sizeof(float), "keyframe_cloud: x, y, z, intensity records");
        const lio_pose p = pose_of(x);
        int64_t n = 0;
        check(lio_scan_keyframe_cloud(c_, &p, T16, nullptr, 0, &n), "keyframe_cloud");
        std::vector<PointXYZI_T> out((size_t)n);
        check(lio_scan_keyframe_cloud(c_, &p, T16, reinterpret_cast<float*>(out.data()), n, &n), "keyframe_cloud");
        return out;
    }

    // kf.update_iterated_dyn_share_modified(LASER_POINT_COV, solve_H_time): x, P (23x23 row-major) in place
    lio_ieskf_stats update_iterated_dyn_share_modified(lio_state& x, double* P, double laser_point_cov = 0.001,
                                                       int max_iteration = 3, double epsi = 0.001) {
        lio_ieskf_params ip{laser_point_cov, max_iteration, epsi};
        lio_ieskf_stats st{};
        check(lio_ieskf_update(c_, &x, P, &ip, &st), "update_iterated_dyn_share_modified");
        return st;
    }

    // one h_share_model evaluation: sums[LIO_SUMS_LEN] (H^T H, H^T h, effct_feat_num, ...)
    void h_share_model(const lio_state& x, bool converge, double* sums) {
        const lio_pose p = pose_of(x);
        check(lio_match(c_, &p, converge ? 1 : 0, sums), "h_share_model");
    }

    // map_incremental() after the update, with the final state
    lio_incremental_stats map_incremental(const lio_state& x, double filter_size_map) {
        const lio_pose p = pose_of(x);
        lio_incremental_stats st{};
        check(lio_map_incremental(c_, &p, filter_size_map, &st), "map_incremental");
        return st;
    }

    // Nearest_Points ids + sq-distances of the last kNN evaluation (n*5)
    void nearest_points(std::vector<int32_t>& ids, std::vector<float>& sq_dist, int64_t n) {
        ids.resize((size_t)n * 5);
        sq_dist.resize((size_t)n * 5);
        check(lio_get_knn(c_, ids.data(), sq_dist.data()), "nearest_points");
    }

    lio_ctx* handle() { return c_; }

private:
    lio_ctx* c_ = nullptr;
};

// lasermap_fov_segment(): boxes to pass to Delete_Point_Boxes
class LocalMap {
public:
    std::vector<BoxPointType> segment(const double pos_lid[3], double cube_len = 1000.0, float det_range = 300.f,
                                      float mov_threshold = 1.5f) {
        float b[18];
        int nb = 0;
        check(lio_localmap_update(&lm_, pos_lid, cube_len, det_range, mov_threshold, b, &nb), "lasermap_fov_segment");
        std::vector<BoxPointType> out((size_t)nb);
        for (int i = 0; i < nb; ++i)
            for (int d = 0; d < 3; ++d) {
                out[i].vertex_min[d] = b[6 * i + d];
                out[i].vertex_max[d] = b[6 * i + 3 + d];
            }
        return out;
    }
    const lio_localmap& state() const { return lm_; }

private:
    lio_localmap lm_{};
};

// ---------------------------------------------------------------------------
// Filters and formats.  PointT: a POD of 3..8 floats starting with x, y, z
// (every float field is averaged / carried, as PCL does with downsample_all_data_).
class FilterGPU {  // device + scratch shared by the filters below
public:
    explicit FilterGPU(int device = 0) { check(lio_filter_create(device, &f_), "lio_filter_create"); }
    ~FilterGPU() { lio_filter_destroy(f_); }
    FilterGPU(const FilterGPU&) = delete;
    FilterGPU& operator=(const FilterGPU&) = delete;
    lio_filter* handle() { return f_; }
    // host scratch kept across calls (submap_voxelize: the concatenated keyframes and the filter's output), so a
    // loop timer's calls touch no fresh pages once the largest submap has been seen
    std::vector<float>& scratch(int i) { return scratch_[i]; }

private:
    lio_filter* f_ = nullptr;
    std::vector<float> scratch_[2];
};

// grow a scratch vector to at least n elements, never shrinking it (no zero-fill of reused capacity)
inline float* scratch_at_least(std::vector<float>& v, size_t n) {
    if (v.size() < n) v.resize(std::max(n, v.size() + v.size() / 2));
    return v.data();
}

// pcl::VoxelGrid<PointT>: setLeafSize / setInputCloud / filter (FAST-LIO downSizeFilterSurf,
// utilities.hpp voxelizePcd)
template <typename PointT>
class VoxelGrid {
public:
    explicit VoxelGrid(FilterGPU& f) : f_(f) {}
    void setLeafSize(float lx, float ly, float lz) { leaf_[0] = lx, leaf_[1] = ly, leaf_[2] = lz; }
    void setInputCloud(const std::vector<PointT>* cloud) { in_ = cloud; }
    void filter(std::vector<PointT>& out) {
        if (!in_) throw Error(LIO_ERR_ARG, "VoxelGrid: no input cloud");
        out.resize(in_->size());
        int64_t n = 0;
        check(lio_voxel_grid(f_.handle(), reinterpret_cast<const float*>(in_->data()), (int64_t)in_->size(),
                             float_stride<PointT>(), leaf_, reinterpret_cast<float*>(out.data()), &n),
              "VoxelGrid::filter");
        out.resize((size_t)n);
    }

private:
    FilterGPU& f_;
    const std::vector<PointT>* in_ = nullptr;
    float leaf_[3] = {0.5f, 0.5f, 0.5f};
};

// one side of LoopClosure::setSrcAndDstCloud (loop_closure.cpp:42-67): transformPcd of each
// keyframe cloud by its corrected pose (row-major double 4x4), concatenated, voxelizePcd
template <typename PointT>
std::vector<PointT> submap_voxelize(FilterGPU& f, const std::vector<const std::vector<PointT>*>& clouds,
                                    const std::vector<const double*>& poses16, float voxel_res) {
    if (clouds.size() != poses16.size()) throw Error(LIO_ERR_ARG, "submap_voxelize: clouds / poses mismatch");
    constexpr int S = float_stride<PointT>();
    std::vector<int64_t> off{0};
    std::vector<double> T;
    for (size_t k = 0; k < clouds.size(); ++k) {
        off.push_back(off.back() + (int64_t)clouds[k]->size());
        T.insert(T.end(), poses16[k], poses16[k] + 16);
    }
    const size_t n_all = (size_t)off.back();
    // concatenated into reused host memory, sized at least for a C4-sized submap (2^19 points) from the first call
    const size_t n_cap = std::max(n_all, (size_t)1 << 19) * S + 1;
    float* all = scratch_at_least(f.scratch(0), n_cap);
    for (size_t k = 0; k < clouds.size(); ++k)
        if (!clouds[k]->empty())
            std::memcpy(all + (size_t)off[k] * S, clouds[k]->data(), clouds[k]->size() * sizeof(PointT));
    float* res = scratch_at_least(f.scratch(1), n_cap);
    int64_t n = 0;
    check(lio_submap_voxelize(f.handle(), all, off.data(), (int)clouds.size(), S, T.data(), voxel_res, res, &n),
          "submap_voxelize");
    std::vector<PointT> out((size_t)n);
    if (n) std::memcpy(out.data(), res, (size_t)n * sizeof(PointT));
    return out;
}

// Preprocess + UndistortPcl + downSizeFilterSurf of one raw scan; the record's time offset [ms]
// sits at float index params.time_field (FAST-LIO keeps it in `curvature`)
template <typename PointT>
std::vector<PointT> preprocess_scan(FilterGPU& f, const std::vector<PointT>& raw, const lio_scan_prep_params& params,
                                    const std::vector<lio_imu_pose>& imu_poses, const lio_state& end_state) {
    const lio_pose end = pose_of(end_state);
    std::vector<PointT> out(raw.size());
    int64_t n = 0;
    check(lio_preprocess(f.handle(), reinterpret_cast<const float*>(raw.data()), (int64_t)raw.size(),
                         float_stride<PointT>(), &params, imu_poses.data(), (int)imu_poses.size(), &end,
                         reinterpret_cast<float*>(out.data()), &n),
          "preprocess_scan");
    out.resize((size_t)n);
    return out;
}

// pcl::io::savePCDFileBinary of the float fields `names` (one per float of PointT)
template <typename PointT>
void savePCDFileBinary(const std::string& path, const std::vector<PointT>& cloud, const std::vector<std::string>& names) {
    if ((int)names.size() != float_stride<PointT>()) throw Error(LIO_ERR_ARG, "savePCDFileBinary: one name per field");
    std::vector<const char*> nm;
    for (const auto& s : names) nm.push_back(s.c_str());
    check(lio_pcd_write_binary(path.c_str(), reinterpret_cast<const float*>(cloud.data()), (int64_t)cloud.size(),
                               float_stride<PointT>(), nm.data()),
          "savePCDFileBinary");
}

// PCD reader (ascii / binary): the fields `names`, in order, into PointT (absent fields read 0)
template <typename PointT>
std::vector<PointT> loadPCDFile(FilterGPU& f, const std::string& path, const std::vector<std::string>& names) {
    if ((int)names.size() != float_stride<PointT>()) throw Error(LIO_ERR_ARG, "loadPCDFile: one name per field");
    std::vector<const char*> nm;
    for (const auto& s : names) nm.push_back(s.c_str());
    int64_t n = 0;
    check(lio_pcd_read(f.handle(), path.c_str(), nm.data(), (int)nm.size(), nullptr, 0, &n), "loadPCDFile");
    std::vector<PointT> out((size_t)n);
    check(lio_pcd_read(f.handle(), path.c_str(), nm.data(), (int)nm.size(), reinterpret_cast<float*>(out.data()), n,
                       &n),
          "loadPCDFile");
    return out;
}

// ---------------------------------------------------------------------------
// LoopClosure::icpAlignment (loop_closure.cpp:69-92) with the reference's ICP
// settings (loop_closure.cpp:6-11) and LoopClosureConfig fields.
struct LoopClosureConfig {  // loop_closure.h:21-29, values from fast_lio_sam.cpp:64-80 + config.yaml
    int num_submap_keyframes_ = 5;
    double voxel_res_ = 0.3;
    double loop_detection_radius_ = 35.0;
    double loop_detection_timediff_threshold_ = 30.0;
    double icp_score_threshold_ = 1.5;
    double icp_max_corr_dist_ = 52.5;  // 1.5 * loop_detection_radius_ (fast_lio_sam.cpp:73)
};

struct RegistrationOutput {  // loop_closure.h:31-37
    bool is_valid_ = false;
    bool is_converged_ = false;
    double score_ = 1.7976931348623157e308;
    double pose_between_eig_[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};  // row-major
};

class LoopClosureICP {
public:
    // umeyama: LIO_ICP_UMEYAMA_DEFAULT = PCL's float Umeyama in the Eigen 3.3 order (the reference's arithmetic,
    // loop_closure.h:42); LIO_ICP_UMEYAMA_DOUBLE opts into the double statistics (outside the 1e-5 bar)
    explicit LoopClosureICP(const LoopClosureConfig& cfg = {}, int device = 0, float cell_size = 1.0f,
                            int umeyama = LIO_ICP_UMEYAMA_DEFAULT) {
        lio_icp_params p{cfg.icp_max_corr_dist_, 0.01, 0.01, 50, 0.0, cfg.icp_score_threshold_, cell_size, device, umeyama};
        check(lio_icp_create(&p, &h_), "lio_icp_create");
    }
    ~LoopClosureICP() { lio_icp_destroy(h_); }
    LoopClosureICP(const LoopClosureICP&) = delete;
    LoopClosureICP& operator=(const LoopClosureICP&) = delete;

    template <typename P>
    RegistrationOutput icpAlignment(const std::vector<P>& src, const std::vector<P>& dst,
                                    std::vector<float>* aligned_xyz = nullptr) {
        const std::vector<float> s = packed_xyz(src), d = packed_xyz(dst);
        check(lio_icp_set_source(h_, s.data(), (int64_t)src.size()), "setInputSource");
        check(lio_icp_set_target(h_, d.data(), (int64_t)dst.size()), "setInputTarget");
        if (aligned_xyz) aligned_xyz->resize(s.size());
        lio_icp_result r{};
        check(lio_icp_align(h_, nullptr, &r, aligned_xyz ? aligned_xyz->data() : nullptr), "align");
        RegistrationOutput out;
        out.score_ = r.score;
        if (r.is_valid) {
            out.is_valid_ = out.is_converged_ = true;
            for (int k = 0; k < 16; ++k) out.pose_between_eig_[k] = r.T[k];
        }
        last_ = r;
        return out;
    }
    const lio_icp_result& last() const { return last_; }
    lio_icp* handle() { return h_; }

private:
    lio_icp* h_ = nullptr;
    lio_icp_result last_{};
};

// LoopClosure's ICP served by several GPUs from one process (lio_icp_group):
// the source sharded, the per-iteration records (and, in the default PCL float
// mode, the accepted correspondence ids) all-gathered over RCCL; results
// bit-identical to LoopClosureICP.  devices empty => 0 .. n_gpus-1.
class LoopClosureICPGroup {
public:
    LoopClosureICPGroup(const LoopClosureConfig& cfg, int n_gpus, const std::vector<int>& devices = {},
                        float cell_size = 1.0f, int umeyama = LIO_ICP_UMEYAMA_DEFAULT) {
        lio_icp_params p{cfg.icp_max_corr_dist_, 0.01, 0.01, 50, 0.0, cfg.icp_score_threshold_, cell_size,
                         devices.empty() ? 0 : devices[0], umeyama};
        check(lio_icp_group_create(&p, n_gpus, devices.empty() ? nullptr : devices.data(), &g_), "lio_icp_group_create");
    }
    ~LoopClosureICPGroup() { lio_icp_group_destroy(g_); }
    LoopClosureICPGroup(const LoopClosureICPGroup&) = delete;
    LoopClosureICPGroup& operator=(const LoopClosureICPGroup&) = delete;

    template <typename P>
    RegistrationOutput icpAlignment(const std::vector<P>& src, const std::vector<P>& dst,
                                    std::vector<float>* aligned_xyz = nullptr) {
        const std::vector<float> s = packed_xyz(src), d = packed_xyz(dst);
        check(lio_icp_group_set_source(g_, s.data(), (int64_t)src.size()), "setInputSource");
        check(lio_icp_group_set_target(g_, d.data(), (int64_t)dst.size()), "setInputTarget");
        if (aligned_xyz) aligned_xyz->resize(s.size());
        lio_icp_result r{};
        check(lio_icp_group_align(g_, nullptr, &r, aligned_xyz ? aligned_xyz->data() : nullptr), "align");
        RegistrationOutput out;
        out.score_ = r.score;
        if (r.is_valid) {
            out.is_valid_ = out.is_converged_ = true;
            for (int k = 0; k < 16; ++k) out.pose_between_eig_[k] = r.T[k];
        }
        last_ = r;
        return out;
    }
    const lio_icp_result& last() const { return last_; }
    bool uses_rccl() const { return lio_icp_group_uses_rccl(g_) != 0; }

private:
    lio_icp_group* g_ = nullptr;
    lio_icp_result last_{};
};

// ---------------------------------------------------------------------------
// fast_lio_sam's keyframe and loop leg (pose_pcd.hpp, loop_closure.h / .cpp) and the C5 stream that feeds
// it (FAST-LIO's per-sweep front end [U] + fast_lio_sam.cpp:367-573,682-730): the C++ form of
// lio_gpu/pipeline.py, for a maintainer who drives the path without Python.
struct PointXYZI {  // pcl::PointXYZI's float fields (x, y, z, intensity)
    float x, y, z, intensity;
};

struct PosePcd {  // pose_pcd.hpp:7-19
    std::vector<PointXYZI> pcd_;
    double pose_eig_[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};            // row-major
    double pose_corrected_eig_[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};  // row-major
    double timestamp_ = 0.0;
    int idx_ = 0;
    bool processed_ = false;
};

// pose_pcd.hpp:26-36: /Odometry's orientation through tf::Matrix3x3(q) (setRotation: s = 2 / |q|^2) and the
// position -> pose_eig_ (row-major)
inline void odom_matrix(const lio_state& x, double T[16]) {
    const double w = x.rot[0], qx = x.rot[1], qy = x.rot[2], qz = x.rot[3];
    const double d = qx * qx + qy * qy + qz * qz + w * w, s = 2.0 / d;
    const double xs = qx * s, ys = qy * s, zs = qz * s;
    const double wx = w * xs, wy = w * ys, wz = w * zs;
    const double xx = qx * xs, xy = qx * ys, xz = qx * zs;
    const double yy = qy * ys, yz = qy * zs, zz = qz * zs;
    const double R[9] = {1.0 - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0 - (xx + zz), yz - wx,
                         xz - wy, yz + wx, 1.0 - (xx + yy)};
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = R[3 * r + c];
        T[4 * r + 3] = x.pos[r];
    }
    T[12] = T[13] = T[14] = 0.0;
    T[15] = 1.0;
}

// Matrix4d::inverse() (pose_eig_.inverse(), pose_pcd.hpp:39) as an x86-64 build of Eigen 3.3 evaluates it:
// Architecture::Target is SSE (SSE2 is on by default), so compute_inverse_size4<SSE, double> (Inverse_SSE.h,
// the "divide and conquer" 2x2-block inverse) runs on the column-major storage — restated here op for op
// (packet lanes as scalars, no FMA), bit-identical to lio_gpu.pipeline.eigen_inverse4 on the Python side.
// m, inv: row-major.  Restated from Eigen's published algorithm; a binary of the reference is not available to
// pin it.
inline void inverse4(const double m[16], double inv[16]) {
    double s[16];  // Eigen's column-major storage: s[k] = M(k % 4, k / 4)
    for (int k = 0; k < 16; ++k) s[k] = m[4 * (k % 4) + k / 4];
    const double A1[2] = {s[0], s[1]}, B1[2] = {s[2], s[3]}, A2[2] = {s[4], s[5]}, B2[2] = {s[6], s[7]};
    const double C1[2] = {s[8], s[9]}, D1[2] = {s[10], s[11]}, C2[2] = {s[12], s[13]}, D2[2] = {s[14], s[15]};
    const double dA = A1[0] * A2[1] - A1[1] * A2[0], dB = B1[0] * B2[1] - B1[1] * B2[0];
    const double AB1[2] = {B1[0] * A2[1] - B2[0] * A1[1], B1[1] * A2[1] - B2[1] * A1[1]};  // A# B
    const double AB2[2] = {B2[0] * A1[0] - B1[0] * A2[0], B2[1] * A1[0] - B1[1] * A2[0]};
    const double dC = C1[0] * C2[1] - C1[1] * C2[0], dD = D1[0] * D2[1] - D1[1] * D2[0];
    const double DC1[2] = {C1[0] * D2[1] - C2[0] * D1[1], C1[1] * D2[1] - C2[1] * D1[1]};  // D# C
    const double DC2[2] = {C2[0] * D1[0] - C1[0] * D2[0], C2[1] * D1[0] - C1[1] * D2[0]};
    const double rd = (AB1[0] * DC1[0] + AB2[0] * DC1[1]) + (AB1[1] * DC2[0] + AB2[1] * DC2[1]);  // tr(A#B D#C)
    double iD1[2] = {AB1[0] * C1[0] + AB2[0] * C1[1], AB1[1] * C1[0] + AB2[1] * C1[1]};  // C A# B
    double iD2[2] = {AB1[0] * C2[0] + AB2[0] * C2[1], AB1[1] * C2[0] + AB2[1] * C2[1]};
    double iA1[2] = {DC1[0] * B1[0] + DC2[0] * B1[1], DC1[1] * B1[0] + DC2[1] * B1[1]};  // B D# C
    double iA2[2] = {DC1[0] * B2[0] + DC2[0] * B2[1], DC1[1] * B2[0] + DC2[1] * B2[1]};
    for (int k = 0; k < 2; ++k) {
        iD1[k] = D1[k] * dA - iD1[k];
        iD2[k] = D2[k] * dA - iD2[k];
        iA1[k] = A1[k] * dD - iA1[k];
        iA2[k] = A2[k] * dD - iA2[k];
    }
    const double d1 = dA * dD, d2 = dB * dC;
    double iB1[2] = {D1[0] * AB2[1] - D1[1] * AB2[0], D1[1] * AB1[0] - D1[0] * AB1[1]};  // D (A# B)#
    double iB2[2] = {D2[0] * AB2[1] - D2[1] * AB2[0], D2[1] * AB1[0] - D2[0] * AB1[1]};
    const double det = (d1 + d2) - rd;
    if (!(std::fabs(det) > 0.0)) throw Error(LIO_ERR_ARG, "inverse4: singular pose");
    double iC1[2] = {A1[0] * DC2[1] - A1[1] * DC2[0], A1[1] * DC1[0] - A1[0] * DC1[1]};  // A (D# C)#
    double iC2[2] = {A2[0] * DC2[1] - A2[1] * DC2[0], A2[1] * DC1[0] - A2[0] * DC1[1]};
    const double r = 1.0 / det;
    for (int k = 0; k < 2; ++k) {
        iB1[k] = C1[k] * dB - iB1[k];
        iB2[k] = C2[k] * dB - iB2[k];
        iC1[k] = B1[k] * dC - iC1[k];
        iC2[k] = B2[k] * dC - iC2[k];
    }
    double o[16];  // the packets written times (r, -r) / (-r, r)
    auto put = [&](int k, const double* X1, const double* X2) {
        o[k] = X2[1] * r;
        o[k + 1] = -(X1[1] * r);
        o[k + 4] = -(X2[0] * r);
        o[k + 5] = X1[0] * r;
    };
    put(0, iA1, iA2);
    put(2, iB1, iB2);
    put(8, iC1, iC2);
    put(10, iD1, iD2);
    for (int k = 0; k < 16; ++k) inv[4 * (k % 4) + k / 4] = o[k];
}

// loop_closure.cpp:18-40 (host logic): among keyframes[0 .. size-2] the closest (translation of
// pose_corrected_eig_) within loop_detection_radius_ and more than loop_detection_timediff_threshold_ older;
// its idx_, or -1
inline int fetch_closest_keyframe_idx(const LoopClosureConfig& config, const PosePcd& query_keyframe,
                                      const std::vector<PosePcd>& keyframes) {
    const double radi = config.loop_detection_radius_;
    double shortest = radi * 3.0;
    int closest = -1;
    const double* q = query_keyframe.pose_corrected_eig_;
    for (size_t i = 0; i + 1 < keyframes.size(); ++i) {
        const double* p = keyframes[i].pose_corrected_eig_;
        const double dx = p[3] - q[3], dy = p[7] - q[7], dz = p[11] - q[11];
        const double d = std::sqrt(dx * dx + dy * dy + dz * dz);
        if (radi > d && config.loop_detection_timediff_threshold_ < query_keyframe.timestamp_ - keyframes[i].timestamp_ &&
            d < shortest) {
            shortest = d;
            closest = keyframes[i].idx_;
        }
    }
    return closest;
}

// LoopClosure (loop_closure.h:39-70): the loop leg with the GPU submap assembly and ICP behind it
class LoopClosure {
public:
    explicit LoopClosure(const LoopClosureConfig& config, int device = 0, int umeyama = LIO_ICP_UMEYAMA_DEFAULT)
        : config_(config), f_(device), icp_(config, device, 1.0f, umeyama) {}

    int fetchClosestKeyframeIdx(const PosePcd& query_keyframe, const std::vector<PosePcd>& keyframes) const {
        return fetch_closest_keyframe_idx(config_, query_keyframe, keyframes);
    }

    // loop_closure.cpp:42-67: per side, transformPcd of keyframes [idx - range, idx + range] (never the newest:
    // i < size - 1) by pose_corrected_eig_, concatenated, voxelizePcd(voxel_res) — on the GPU
    std::pair<std::vector<PointXYZI>, std::vector<PointXYZI>> setSrcAndDstCloud(const std::vector<PosePcd>& keyframes,
                                                                                int src_idx, int dst_idx,
                                                                                int submap_range, double voxel_res) {
        auto side = [&](int center) {
            std::vector<const std::vector<PointXYZI>*> clouds;
            std::vector<const double*> poses;
            for (int i = center - submap_range; i <= center + submap_range; ++i)
                if (i >= 0 && i + 1 < (int)keyframes.size()) {
                    clouds.push_back(&keyframes[(size_t)i].pcd_);
                    poses.push_back(keyframes[(size_t)i].pose_corrected_eig_);
                }
            return clouds.empty() ? std::vector<PointXYZI>{} : submap_voxelize(f_, clouds, poses, (float)voxel_res);
        };
        return {side(src_idx), side(dst_idx)};
    }

    // loop_closure.cpp:69-92
    RegistrationOutput icpAlignment(const std::vector<PointXYZI>& src, const std::vector<PointXYZI>& dst) {
        return icp_.icpAlignment(src, dst, &aligned_);
    }

    // Node start-up (no counterpart in the reference): one small submap and alignment through every stage, so
    // the device buffers (their C4-sized floors), the kernels' code objects and the sort scratch exist before
    // the first loopTimerFunc call — which otherwise pays ~65 ms for them.  Results are discarded.
    void prewarm() {
        std::vector<PointXYZI> a, b;
        for (int i = 0; i < 100; ++i)  // past the voxel filter's one-block size: the large-input path warmed too
            for (int j = 0; j < 100; ++j)
                for (int k = 0; k < 4; ++k) {  // a 100 m x 100 m x 18 m lattice (a submap's extent), b shifted 5 cm
                    const float x = 1.0f * (float)i, y = 1.0f * (float)j, z = 6.0f * (float)k;
                    a.push_back({x, y, z, 0.f});
                    b.push_back({x + 0.05f, y - 0.03f, z + 0.02f, 0.f});
                }
        const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        std::vector<const double*> poses{I};
        std::vector<const std::vector<PointXYZI>*> ca{&a}, cb{&b};
        const auto sa = submap_voxelize(f_, ca, poses, (float)config_.voxel_res_);
        const auto sb = submap_voxelize(f_, cb, poses, (float)config_.voxel_res_);
        icpAlignment(sa, sb);
        aligned_.clear();
    }

    // loop_closure.cpp:95-126 (submap_range < 0: num_submap_keyframes_)
    RegistrationOutput performLoopClosure(const PosePcd& query_keyframe, const std::vector<PosePcd>& keyframes,
                                          int closest_keyframe_idx, int submap_range = -1) {
        closest_keyframe_idx_ = closest_keyframe_idx;
        if (closest_keyframe_idx < 0) return RegistrationOutput{};
        const int rng = submap_range < 0 ? config_.num_submap_keyframes_ : submap_range;
        auto sd = setSrcAndDstCloud(keyframes, query_keyframe.idx_, closest_keyframe_idx, rng, config_.voxel_res_);
        src_cloud_ = std::move(sd.first);
        dst_cloud_ = std::move(sd.second);
        return icpAlignment(src_cloud_, dst_cloud_);
    }
    RegistrationOutput performLoopClosure(const PosePcd& query_keyframe, const std::vector<PosePcd>& keyframes) {
        return performLoopClosure(query_keyframe, keyframes, fetchClosestKeyframeIdx(query_keyframe, keyframes));
    }

    const std::vector<PointXYZI>& getSourceCloud() const { return src_cloud_; }
    const std::vector<PointXYZI>& getTargetCloud() const { return dst_cloud_; }
    const std::vector<float>& getFinalAlignedCloud() const { return aligned_; }  // xyz of the aligned source
    int getClosestKeyframeidx() const { return closest_keyframe_idx_; }
    const lio_icp_result& last_result() const { return icp_.last(); }
    const LoopClosureConfig& config() const { return config_; }

private:
    LoopClosureConfig config_;
    FilterGPU f_;
    LoopClosureICP icp_;
    int closest_keyframe_idx_ = -1;
    std::vector<PointXYZI> src_cloud_, dst_cloud_;
    std::vector<float> aligned_;
};

// One sensor stream through the GPU front end plus the loop leg (lio_gpu/pipeline.py FastLioSamStream):
// per sweep Preprocess + UndistortPcl + downSizeFilterSurf -> IESKF update -> map_incremental -> keyframe
// (every processed sweep: keyframe_threshold is 0 in config.yaml); loop() runs loopTimerFunc's work on the
// newest keyframe.  Stage times are host wall times (ms).
struct SweepResult {
    lio_state x{};
    std::vector<double> P;  // 23 x 23 row-major
    lio_ieskf_stats stats{};
    lio_incremental_stats incremental{};
    int64_t n_down = 0, n_undistorted = 0;
    double ms_preprocess = 0, ms_update = 0, ms_map_incremental = 0, ms_keyframe = 0;
};

class FastLioSamStream {
public:
    template <typename P>
    FastLioSamStream(KdTreeGPU<P>& tree, const LoopClosureConfig& config = {}, double filter_size_map = 0.5,
                     int max_iteration = 3, int point_filter_num = 4, float blind = 2.0f, float filter_size_surf = 0.5f,
                     int device = 0)
        : sm_(tree), lc_(config, device), fs_map_(filter_size_map), max_iter_(max_iteration),
          prep_{point_filter_num, blind, filter_size_surf, 4} {
        lc_.prewarm();  // node start-up: the loop leg's first loopTimerFunc call is not the one to size its buffers
    }

    // one raw sweep (n float records of `stride`, the time offset [ms] at field 4), its IMU poses and the
    // scan-end pose; init / P0 the propagated state and covariance
    SweepResult process(const float* raw, int64_t n, int stride, const std::vector<lio_imu_pose>& imu_poses,
                        const lio_pose& end, const lio_state& init, const double* P0, double timestamp) {
        using clk = std::chrono::steady_clock;
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        SweepResult r;
        const auto t0 = clk::now();
        r.n_down = sm_.set_scan_raw(raw, n, stride, prep_, imu_poses.data(), (int)imu_poses.size(), end);
        const auto t1 = clk::now();
        r.x = init;
        r.P.assign(P0, P0 + 23 * 23);
        r.stats = sm_.update_iterated_dyn_share_modified(r.x, r.P.data(), 0.001, max_iter_, 0.001);
        const auto t2 = clk::now();
        r.incremental = sm_.map_incremental(r.x, fs_map_);
        const auto t3 = clk::now();
        PosePcd kf;
        odom_matrix(r.x, kf.pose_eig_);
        double inv[16];
        inverse4(kf.pose_eig_, inv);
        kf.pcd_ = sm_.keyframe_cloud<PointXYZI>(r.x, inv);
        std::copy(kf.pose_eig_, kf.pose_eig_ + 16, kf.pose_corrected_eig_);
        kf.timestamp_ = timestamp;
        kf.idx_ = (int)keyframes_.size();
        r.n_undistorted = (int64_t)kf.pcd_.size();
        keyframes_.push_back(std::move(kf));
        const auto t4 = clk::now();
        r.ms_preprocess = ms(t0, t1);
        r.ms_update = ms(t1, t2);
        r.ms_map_incremental = ms(t2, t3);
        r.ms_keyframe = ms(t3, t4);
        return r;
    }

    // loopTimerFunc's work on the newest keyframe: the closest index (-1: none) and the registration
    int loop(RegistrationOutput* out, int submap_range = -1) {
        *out = RegistrationOutput{};
        if (keyframes_.empty()) return -1;
        const PosePcd& q = keyframes_.back();
        const int idx = lc_.fetchClosestKeyframeIdx(q, keyframes_);
        if (idx >= 0) *out = lc_.performLoopClosure(q, keyframes_, idx, submap_range);
        return idx;
    }

    const std::vector<PosePcd>& keyframes() const { return keyframes_; }
    ScanMatcherGPU& matcher() { return sm_; }
    LoopClosure& loop_closure() { return lc_; }

private:
    ScanMatcherGPU sm_;
    LoopClosure lc_;
    double fs_map_;
    int max_iter_;
    lio_scan_prep_params prep_;
    std::vector<PosePcd> keyframes_;
};

}  // namespace lio_gpu
