// lio_filter.hpp — point-cloud filters (lio_filter.hip): PCL VoxelGrid,
// transformPcd, FAST-LIO scan preprocessing / undistortion.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lio {

constexpr int kMaxFields = 8;  // floats per point record (x, y, z, + up to 5 attributes)

struct VoxelGeom {
    float inv[3];
    int min_b[3];
    int mul[3];
    int overflow;
    int empty;
    int key_bits;  // bits of the largest voxel index (div_b.x * div_b.y * div_b.z - 1)
};

// One IMUpose entry (FAST-LIO set_pose6d [U]): offset_time [s] from the scan
// start, acc (world, gravity added), gyr (bias removed), vel, pos, rot (row-major).
struct ImuPose {
    double offset_time;
    double acc[3], gyr[3], vel[3], pos[3], rot[9];
};

// State at the scan end (after the last predict): rot/pos of the IMU and the
// LiDAR-IMU extrinsic, row-major rotation matrices.
struct UndistortEnd {
    double pos[3];
    double R[9];
    double R_LI[9];
    double t_LI[3];
    double q[4];     // rot as Eigen::Quaternion<double> (w, x, y, z): the SO3 products use it
    double q_LI[4];  // offset_R_L_I
};

// Where the host packed the selected rows: logical row i of piece t (start[t] <= i < start[t + 1]) lives at
// staged row src[t] + (i - start[t]) (the pieces were packed in parallel, each at its own offset, and go
// to the device in one DMA with the gaps).  n = 1, start = src = 0: rows in place.
constexpr int kMaxPieces = 8;
struct RowPieces {
    int n = 1;
    uint32_t start[kMaxPieces] = {};
    uint32_t src[kMaxPieces] = {};
};

struct ScanPrepParams {
    int point_filter_num;  // keep every n-th input point (Preprocess, kitti.launch:6)
    float blind;           // drop points with |p| <= blind (kitti.yaml:13)
    float leaf;            // filter_size_surf (kitti.launch:9); 0 = no downsample
    int time_field;        // index of the per-point time offset [ms] (FAST-LIO's curvature)
};

struct FilterBuf {
    uint32_t *keys = nullptr, *keys_alt = nullptr, *vals = nullptr, *vals_alt = nullptr;
    uint32_t *head = nullptr, *vid = nullptr;
    int64_t cap = 0;
    int64_t min_cap = 0;     // capacity floor (the loop leg's submaps: sized once, lio_submap_voxelize)
    float* part = nullptr;
    VoxelGeom* geom = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int* h_small = nullptr;  // pinned, host-mapped: [0] voxel count, [1..] VoxelGeom, [kHostSel] selected count,
    int* d_small = nullptr;  //   [kHostFlags] flags (bit 0: a voxel key past vox_bits); d_small = the device view
    uint32_t* cnt = nullptr; // device: [0] scan_preprocess's selected count, [1] minmax_geom_kernel's ticket
    int vox_bits = 32;       // voxel-key bits the next voxel sort assumes (learnt, checked on the device)
    float* a = nullptr;      // staging records
    int64_t a_cap = 0;
    float* c = nullptr;
    int64_t c_cap = 0;
    void* aux = nullptr;     // caller-side scratch (host API uploads)
    size_t aux_bytes = 0;
    void* h_stage = nullptr; // pinned host staging of the sweep uploads (lio_capi stage_sweep)
    size_t stage_bytes = 0;
    int64_t prep_n = 0;      // row bound of the last scan_preprocess_enqueue (0: nothing pending)
    int64_t prep_sel = -1;   // its selected count when the host selected the rows (-1: on the device)
    bool prep_leaf = false;
};
constexpr int kHostSel = 16, kHostFlags = 17;

void filter_free(FilterBuf& b);
// d_out capacity: n * stride floats.  Synchronises the stream (output count).
int voxel_grid(FilterBuf& b, const float* d_in, int64_t n, int stride, const float leaf[3], float* d_out,
               int64_t* n_out, hipStream_t st);
// points of segment s ([seg_off[s], seg_off[s+1]), nseg segments, seg_off[nseg] = n) through T16[s]
int transform_segments(const float* d_in, int64_t n, int stride, const int64_t* d_seg_off, int nseg,
                       const double* d_T16, float* d_out, hipStream_t st);
// selection -> stable sort by time -> undistortion (np >= 2 poses) -> voxel grid.  The undistorted,
// time-sorted records before the voxel grid (FAST-LIO feats_undistort) stay in b.c, *n_undist of them,
// until the next call on b.
int scan_preprocess(FilterBuf& b, const float* d_raw, int64_t n, int stride, const ScanPrepParams& p,
                    const ImuPose* d_poses, int np, const UndistortEnd& end, float* d_out, int64_t* n_out,
                    hipStream_t st, int64_t* n_undist = nullptr);
// The same in two halves, one host wait: _enqueue queues every stage (d_out and the ctx buffers sized
// for the row bound n; rows past the count are scratch), _finish waits for the stream and reads the
// counts.  _finish returns 1 when VoxelGrid's index overflow replaced the output by its input: that
// copy is queued, not waited on, and the caller's follow-up work on d_out must be queued again.
// presel >= 0: the n rows are already Preprocess's selection, in input order (the host packed them), and
// presel = 1 says their times are non-decreasing — the stable time sort is then the identity and is skipped.
// _finish returns 2 when the learnt voxel-key width was too narrow: the caller enqueues again (same input).
// xyz / sel (optional, leaf > 0): the output's packed xyz and zeroed selection flags written by the
// centroid pass (rows past the voxel count untouched)
int scan_preprocess_enqueue(FilterBuf& b, const float* d_raw, int64_t n, int stride, const ScanPrepParams& p,
                            const ImuPose* d_poses, int np, const UndistortEnd& end, float* d_out, hipStream_t st,
                            int presel = -1, float* xyz = nullptr, uint8_t* sel = nullptr,
                            const RowPieces& pieces = RowPieces{});
int scan_preprocess_finish(FilterBuf& b, int stride, float* d_out, int64_t* n_out, int64_t* n_undist, hipStream_t st);
// records -> packed xyz, and sel[0 .. n) = 0 (the scan's selection flags) in the same pass
int records_to_xyz_sel(const float* d_rec, int64_t n, int stride, float* d_xyz, uint8_t* sel, hipStream_t st);

int records_to_xyz(const float* d_rec, int64_t n, int stride, float* d_xyz, hipStream_t st);

// d_out (n x 4: x, y, z, intensity) = T16 (row-major, double) * pointBodyToWorld(ps, record xyz) — the
// keyframe cloud fast_lio_sam builds from /cloud_registered (lio_scan_keyframe_cloud)
int keyframe_cloud(const float* d_rec, int64_t n, int stride, const PoseArg& ps, const double* T16, float* d_out,
                   hipStream_t st);

// One output column of a packed point record (sensor_msgs/PointField or a PCD field):
// byte offset, PointField datatype (1..8, 0 = absent -> 0), scale (e.g. time unit -> ms).
struct CloudField {
    int32_t offset;
    int32_t datatype;
    float scale;
};
int cloud_decode(const uint8_t* d_data, int64_t n, int point_step, bool big_endian, const CloudField* fields, int nf,
                 float* d_out, hipStream_t st);
int cloud_encode(const float* d_rec, int64_t n, int stride, int point_step, const CloudField* fields, int nf,
                 uint8_t* d_data, hipStream_t st);

}  // namespace lio
