/*
 * lio_gpu.h — C-ABI of the MI355X (gfx950) scan-matching hot path.
 *
 * Drop-in boundary for the reference's hot path:
 *
 *  B-front: FAST-LIO's measurement model `void h_share_model(state_ikfom&,
 *    esekfom::dyn_share_datastruct<double>&)` plus the ikd-Tree it queries
 *    (upstream hku-mars FAST_LIO src/laserMapping.cpp + include/ikd-Tree; the
 *    Kodifly fork is an empty submodule in the reference: .gitmodules:1-3,
 *    launched by fast_lio_sam/launch/run.launch:20-46).  The host IESKF keeps
 *    its 23-dim state; one lio_match() per h-evaluation replaces the per-point
 *    OpenMP loop, and lio_ieskf_update() is the complete
 *    `kf.update_iterated_dyn_share_modified(LASER_POINT_COV, solve_H_time)`.
 *  B-loop: `RegistrationOutput LoopClosure::icpAlignment(src, dst)`
 *    (/root/reference/fast_lio_sam/src/loop_closure.cpp:69-92, declared at
 *    include/loop_closure.h:59-60) — replaced whole by lio_icp_align().
 *
 * Conventions: every call returns int status (LIO_OK = 0, < 0 on error;
 * lio_last_error() gives text).  Host buffers are caller-owned and copied in;
 * handles own device memory; one HIP stream per handle; a handle is not
 * thread-safe, distinct handles may be used concurrently.  No torch types.
 * There is no CPU fallback: without a gfx950 device every compute entry point
 * fails with LIO_ERR_NODEV.
 */
#ifndef LIO_GPU_H
#define LIO_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIO_OK 0
#define LIO_ERR_ARG (-1)
#define LIO_ERR_HIP (-2)
#define LIO_ERR_NODEV (-3)
#define LIO_ERR_STATE (-4)
#define LIO_ERR_NOMEM (-5)

#define LIO_NUM_MATCH_POINTS 5 /* NUM_MATCH_POINTS [U: FAST-LIO common_lib.h] */
#define LIO_STATE_DIM 23       /* state_ikfom DOF [U: FAST-LIO use-ikfom.hpp] */

/* Layout of the per-h-evaluation reduction returned by lio_match() (doubles):
 * H^T H upper triangle of the 6 non-zero columns (extrinsic_est_en = false,
 * kitti.yaml:22) row-major i<=j, H^T h, effct_feat_num, total_residual, h^T h. */
#define LIO_SUMS_HTH 0
#define LIO_SUMS_HTh 21
#define LIO_SUMS_NEFF 27
#define LIO_SUMS_RES 28
#define LIO_SUMS_HH 29
#define LIO_SUMS_LEN 32

/* ------------------------------------------------------------------ device */
int lio_device_count(void);
const char* lio_last_error(void);
const char* lio_build_info(void);
/* Diagnostics (no device needed): device / pinned allocations the library's growth paths (loop ICP, grids,
 * filters, scan buffers) have made in this process.  A warm loop-closure sequence adds none (bench.py
 * loop_sequence).                                                                                  */
int64_t lio_alloc_count(void);
/* ABI guard (no device needed): sizeof of the public structs, in the order map_params, match_params, pose,
 * state, ieskf_params, ieskf_stats, icp_params, icp_result, localmap, incremental_stats, imu_pose,
 * scan_prep_params, cloud_field, kernel_timing — the first min(n, count) into out; returns the count.
 * A binding built against another header version must refuse the library (an output struct of the wrong
 * size is a buffer overrun: round 4's A/B of a round-2 build segfaulted at exit that way).           */
int lio_abi_struct_sizes(int64_t* out, int n);

/* -------------------------------------------------------------------- map
 * Replaces `KD_TREE<PointType> ikdtree` [U: ikd-Tree ikd_Tree.h]: a dense
 * uniform grid in HBM (points float4 sorted by cell, u32 cell offsets).
 * kNN results are exact; point ids are insertion order (0..size-1).       */
typedef struct lio_map lio_map;

typedef struct lio_map_params {
    float cell_size;        /* grid cell edge [m]; 0 => 1.0                          */
    float downsample_size;  /* filter_size_map (kitti.launch:10) for lio_map_add    */
    int device;             /* HIP device ordinal                                   */
    int reserved;
} lio_map_params;

int lio_map_create(const lio_map_params* p, lio_map** out);
/* Refuses (LIO_ERR_STATE) while lio_ctx handles created on m are alive.    */
int lio_map_destroy(lio_map* m);
/* ikdtree.set_downsample_param(filter_size_map_min) [U: laserMapping.cpp
 * main(), before Build]: changes cell_size / downsample_size in place (a
 * value <= 0 keeps the current one); only while the map holds no points, so
 * every lio_ctx already created on m stays valid.  device must not change. */
int lio_map_set_params(lio_map* m, const lio_map_params* p);
/* ikdtree.Build(points) [U]: replaces the content. xyz: n*3 float, host.   */
int lio_map_build(lio_map* m, const float* xyz, int64_t n);
/* same, xyz already resident in device memory (e.g. a torch tensor).       */
int lio_map_build_device(lio_map* m, const float* d_xyz, int64_t n);
/* ikdtree.size() [U]: alive points                                        */
int64_t lio_map_size(const lio_map* m);
/* ids ever inserted (alive + deleted); kNN ids index this space            */
int64_t lio_map_num_ids(const lio_map* m);
/* copies the alive map points (id order) to host, lio_map_size()*3 float   */
int lio_map_get_points(lio_map* m, float* xyz_out);
/* every id: xyz (num_ids*3, may be NULL) and alive flags (num_ids, may be NULL) */
int lio_map_get_by_id(lio_map* m, float* xyz_out, uint8_t* alive_out);
/* ikd-Tree Nearest_Search(point, k, Nearest_Points, Point_Distance, max_dist)
 * [U: ikd-Tree ikd_Tree.h; FAST-LIO laserMapping.cpp h_share_model calls it
 * with k = NUM_MATCH_POINTS = 5, max_dist = INFINITY] for a batch of n query
 * points q (n*3 float): the k <= 5 nearest alive map points in ascending
 * (sq-distance, id) order with sq-distance <= max_dist^2 (max_dist <= 0 or
 * INFINITY: unbounded).  idx (n*k, map ids = insertion order, -1 where fewer
 * exist), d2 (n*k, optional, INFINITY where missing).                      */
int lio_map_nearest_search(lio_map* m, const float* q, int64_t n, int k, float max_dist, int32_t* idx, float* d2);
/* Coordinates of map ids (Nearest_Points from lio_map_nearest_search /
 * lio_get_knn ids): xyz_out n*3; ids < 0 or unknown give NaN.             */
int lio_map_gather(lio_map* m, const int32_t* ids, int64_t n, float* xyz_out);

/* ---- incremental maintenance ----
 * ikdtree.Add_Points(PointToAdd, downsample_on) [U]: with downsample, per
 * point (in order) the filter_size_map voxel [floor(p/ds)*ds, +ds) keeps only
 * the point nearest its centre (Search_by_range + Delete_by_range +
 * Add_by_point).  n_added (may be NULL): the reference's return value (the
 * number of Add_by_point calls; n for downsample = 0).                      */
int lio_map_add(lio_map* m, const float* xyz, int64_t n, int downsample, int64_t* n_added);
int lio_map_add_device(lio_map* m, const float* d_xyz, int64_t n, int downsample, int64_t* n_added);
/* ikdtree.Delete_Point_Boxes(cub_needrm) [U]: boxes nb x 6 floats
 * (min x y z, max x y z), a point is inside when min <= p < max.           */
int lio_map_delete_boxes(lio_map* m, const float* boxes, int nb, int64_t* n_deleted);

/* lasermap_fov_segment() [U] (FAST-LIO laserMapping.cpp): host helper that
 * keeps the local map cube around the LiDAR and returns the boxes to delete
 * (pass them to lio_map_delete_boxes).  pos_lid = pos + rot * offset_T_L_I.  */
typedef struct lio_localmap {
    float vertex_min[3], vertex_max[3];
    int initialized;
} lio_localmap;
int lio_localmap_update(lio_localmap* lm, const double pos_lid[3], double cube_len, float det_range,
                        float mov_threshold, float boxes_out[18], int* n_boxes);
/* grid geometry: origin[3], cell, dims[3] (as doubles)                     */
int lio_map_get_grid(lio_map* m, double* out7);
/* diagnostics: out8 = [full grid rebuilds so far, slot pool capacity, slots handed out (device bump),
 * alive points, ids, grid cells, flags of the last update (1 outside the grid, 2 pool exhausted,
 * 4 tombstone cell list full: each forces a rebuild), reserved]                                  */
int lio_map_get_stats(lio_map* m, int64_t* out8);
/* Test hook: cap the slot pool at (slots in use after the last rebuild + slot_headroom) and the per-update
 * list of cells holding tombstones at dirty_cells (0: no cap), so that the pool-exhausted (flag 2) and
 * list-full (flag 4) recovery paths run on small maps.                                          */
int lio_map_set_test_limits(lio_map* m, int64_t slot_headroom, int64_t dirty_cells);

/* ------------------------------------------------------------ h-model ctx */
typedef struct lio_ctx lio_ctx;

typedef struct lio_match_params {
    float knn_range_sq; /* 5.0: gate `sqdist[4] > 5` rejects; bounded-search radius^2 */
    float plane_thr;    /* 0.1f: esti_plane(pabcd, points_near, 0.1f)                  */
    double s_coef;      /* 0.9: s = 1 - 0.9*|pd2|/sqrt(|p_body|)                        */
    double s_gate;      /* 0.9: keep if s > 0.9                                         */
} lio_match_params;

/* The parts of state_ikfom the measurement model reads:
 *   p_world = rot * (offset_R_L_I * p_body + t_LI) + t.
 * q / q_LI are state_ikfom's rot / offset_R_L_I (MTK::SO3 = Eigen::Quaternion
 * <double>, stored (w, x, y, z)); the kernels evaluate every `SO3 * v` from
 * them exactly as Eigen's QuaternionBase::_transformVector does.  R / R_LI are
 * the same rotations as row-major matrices.  A caller holding only matrices
 * leaves q (q_LI) all zero: it is then derived from R (R_LI) with Eigen's
 * Matrix3 -> Quaternion conversion.  A non-zero q takes precedence: R / R_LI
 * are then not read by any computation (so a stale R cannot disagree with
 * the kernels' rotation).                                                   */
typedef struct lio_pose {
    double R[9];
    double t[3];
    double R_LI[9];
    double t_LI[3];
    double q[4];
    double q_LI[4];
} lio_pose;

int lio_ctx_create(lio_map* m, const lio_match_params* p, lio_ctx** out);
int lio_ctx_destroy(lio_ctx* c);
/* feats_down_body (n*3 float, LiDAR frame), host / device pointer.         */
int lio_scan_set(lio_ctx* c, const float* body_xyz, int64_t n);
int lio_scan_set_device(lio_ctx* c, const float* d_body_xyz, int64_t n);
/* same without a copy: the ctx reads the caller's device buffer, which must stay valid and
 * unchanged until the next lio_scan_* call on this ctx.                                       */
int lio_scan_bind_device(lio_ctx* c, const float* d_body, int64_t n);
/* One h_share_model evaluation [U]. redo_knn = ekfom_data.converge.
 * sums: LIO_SUMS_LEN doubles (see layout above).                           */
int lio_match(lio_ctx* c, const lio_pose* pose, int redo_knn, double* sums);
/* Debug getters (not on the timed path):
 *   Nearest_Points ids + sq-distances (n*5, -1 / +inf where fewer than 5),
 *   normvec (a,b,c,pd2 for selected points) + point_selected_surf,
 *   feats_down_world for the pose of the last lio_match.                    */
int lio_get_knn(lio_ctx* c, int32_t* idx, float* d2);
int lio_get_planes(lio_ctx* c, float* abcd_pd2, uint8_t* sel);
int lio_get_world(lio_ctx* c, float* world);
/* ekfom_data.h_x rows (6 non-zero columns) + h of the selected points, in
 * point order, for the dof < 23 branch of the IESKF: rows = 7 doubles each. */
int lio_get_h_rows(lio_ctx* c, double* rows, int64_t max_rows, int64_t* n_rows);
/* Diagnostics: one kNN evaluation (same results as lio_match(redo_knn=1))
 * that also reports, per point, {cells scanned, map points scanned, last
 * shell visited} (stats3: n*3 int32).                                     */
int lio_ctx_knn_stats(lio_ctx* c, const lio_pose* pose, double* sums, int32_t* stats3);

/* ------------------------------------------------------------------ IESKF */
typedef struct lio_state { /* state_ikfom [U], quaternions are (w, x, y, z) */
    double pos[3];
    double rot[4];
    double offset_R_L_I[4];
    double offset_T_L_I[3];
    double vel[3];
    double bg[3];
    double ba[3];
    double grav[3];
} lio_state;

typedef struct lio_ieskf_params {
    double laser_point_cov; /* LASER_POINT_COV = 0.001 [U]                  */
    int max_iteration;      /* NUM_MAX_ITERATIONS = max_iteration = 3 (kitti.launch:8) */
    double epsi;            /* convergence limit per state dim = 0.001 [U]  */
} lio_ieskf_params;

typedef struct lio_ieskf_stats {
    int h_evals;    /* h_share_model calls                               */
    int knn_calls;  /* of which redid the kNN (ekfom_data.converge)      */
    int converged;  /* exited through t > 1 (1) or the iteration cap (0) */
    int n_eff;      /* effct_feat_num of the last evaluation             */
    double res_mean;/* res_mean_last                                     */
    double solve_ms;/* host time in the 23-dim algebra                   */
    double wall_ms; /* host wall time of the whole call                  */
    double launch_ms;/* host time enqueueing the evaluations' kernels     */
    double wait_ms; /* host time waiting for the evaluations' results    */
} lio_ieskf_stats;

/* esekf::update_iterated_dyn_share_modified(R, solve_time) [U IKFoM];
 * x and P (23x23 row-major) are updated in place.  Default: the host loop
 * (one h-evaluation launch + one zero-copy result per iteration, 23-dim
 * algebra on the host).                                                     */
int lio_ieskf_update(lio_ctx* c, lio_state* x, double* P, const lio_ieskf_params* p, lio_ieskf_stats* st);
/* Test hook: the seeded kNN pass's bound (later kNN evaluations of a scan) is
 * multiplied by scale in (0, 1]; < 1 shrinks it below the true 5th distance so
 * the not-full guard (whole-box far search) is exercised.  Default 1.        */
int lio_ctx_set_seed_scale(lio_ctx* c, float scale);

/* ---------------------------------------------------------------- loop ICP */
typedef struct lio_icp lio_icp;

typedef struct lio_icp_params {
    double max_corr_dist;   /* icp_max_corr_dist_ = 1.5 * loop_detection_radius (fast_lio_sam.cpp:73) */
    double trans_eps;       /* setTransformationEpsilon(0.01)   loop_closure.cpp:8  */
    double fitness_eps;     /* setEuclideanFitnessEpsilon(0.01) loop_closure.cpp:9  */
    int max_iter;           /* setMaximumIterations(50)         loop_closure.cpp:10 */
    double rot_eps;         /* 0 => PCL default 1 - trans_eps                        */
    double score_threshold; /* icp_score_threshold (config.yaml:16)                   */
    float cell_size;        /* target grid cell [m]; 0 => 1.0                        */
    int device;
    /* How TransformationEstimationSVD's Umeyama step is evaluated (LIO_ICP_UMEYAMA_*).
     * 0 (LIO_ICP_UMEYAMA_DEFAULT, a zero-initialised struct) = 2: the reference's arithmetic.
     * 1..3: PCL float modes — TransformationEstimationSVD<PointXYZI, PointXYZI, float>'s pcl::umeyama
     *    (loop_closure.h:42, aligned at loop_closure.cpp:81) restated in float with the float summation
     *    order of a given PCL/Eigen build (parity with a real PCL build unpinned: no PCL here):
     *    1 sequential-order restatement: means and sigma's depth as single sequential chains;
     *    2 Eigen 3.3 model (32 KiB L1): sequential means, sigma by Eigen's GEMM — depth blocked by
     *      kc = 680, res += alpha * block sum — THE DEFAULT;
     *    3 as 2 with a 48 KiB L1 (kc = 1016).
     *    The sequential float chains are evaluated in parallel and verified bit-exact on the GPU
     *    (lio_seqsum: predicted binades, event replay, full verification; serial kernel fallback);
     *    float JacobiSVD on the host.  Sharded (world > 1): every rank's accepted correspondence ids
     *    ride the records' all-gather and every rank evaluates the float chains over the whole
     *    source, so the transform is the one-rank transform bit for bit.
     * -1 (LIO_ICP_UMEYAMA_DOUBLE, opt-in): the statistics in double about a fixed centre — faster, but
     *    1.2-1.9e-4 from PCL's float arithmetic at C4 (outside the 1e-5 parity bar).      */
    int umeyama_float;
} lio_icp_params;
#define LIO_ICP_UMEYAMA_DEFAULT 0
#define LIO_ICP_UMEYAMA_PCL_SEQ 1
#define LIO_ICP_UMEYAMA_PCL_GEMM32 2
#define LIO_ICP_UMEYAMA_PCL_GEMM48 3
#define LIO_ICP_UMEYAMA_DOUBLE (-1)

typedef struct lio_icp_result {  /* RegistrationOutput (loop_closure.h:21-27) + diagnostics */
    int is_valid;
    int is_converged;
    double score;          /* getFitnessScore()                         */
    float T[16];           /* getFinalTransformation(), row-major        */
    int iterations;
    int state;             /* convergence state: 0 none, 1 iter, 2 transform, 3 abs mse, 4 rel mse, 5 no corr */
    double last_mse;
    int64_t last_corr;
} lio_icp_result;

/* Exchange hook for sharded ICP (one process per GPU): all-gather `n` doubles
 * from every rank into recv (world*n, rank order).  NULL => single rank.   */
typedef int (*lio_allgather_fn)(const double* send, int64_t n, double* recv, void* user);

int lio_icp_create(const lio_icp_params* p, lio_icp** out);
int lio_icp_destroy(lio_icp* h);
int lio_icp_set_target(lio_icp* h, const float* xyz, int64_t n);         /* setInputTarget */
int lio_icp_set_source(lio_icp* h, const float* xyz, int64_t n);         /* setInputSource */
/* Shard the source's fixed 4096-point blocks over `world` ranks.          */
int lio_icp_set_shard(lio_icp* h, int rank, int world, lio_allgather_fn fn, void* user);
/* Host-only helpers of the sharded path (no device needed): the contiguous
 * source range a rank owns (whole 4096-point records), and the rank-order
 * combination of all-gathered records into the 17 Umeyama statistics
 * [n, sum p(3), sum q(3), sum q p^T(9), sum d2].  recv = world slots of
 * ceil(records/world)*20 doubles, as lio_allgather_fn delivers them.       */
int lio_icp_shard_range(int64_t n_source, int rank, int world, int64_t* begin, int64_t* count);
int lio_icp_combine(const double* recv, int64_t n_source, int world, double* out17);
/* Host mirrors of the sharded float chains' exchange (no device; the kernels run the same code):
 * lio_seq_shard_offsets — every rank's block-sum message (rank r at recv + r * stride: [0] the window's
 * element count, then per chain c at 8 + 2 c nb_slot its 1024-element blocks' (double sum, sum |x|)) -> rank
 * `rank`'s starting prefix, drift variance and the common floor of chains 0 .. nch-1, its first global index
 * and the total (gbase_nglobal[2]); lio_seq_shard_merge — every rank's event message (header: [0] n, [1] overflow bits,
 * [2 + c] increment total, [11 + c] event count, [20 + c] first element; at 32 + 2 slot c the events:
 * increment prefix bits, then position | value bits << 32) -> chain `chain`'s global lists (pos, P, x) and
 * nev_ptot_bad = {events, longest list, problems (1 own overflow, 2 over the slot, 4 over evs)}.          */
int lio_seq_shard_offsets(const double* recv, int64_t stride, int64_t nb_slot, int rank, int world, int nch,
                          double* off0, double* var0, int32_t* floor_e, int64_t* gbase_nglobal);
int lio_seq_shard_merge(const double* recv, int64_t stride, int world, int slot, int chain, int64_t evs,
                        int32_t* pos, uint64_t* P, float* x, int32_t* nev_ptot_bad, uint64_t* ptot, float* x0);
/* Host half of the float fidelity modes (no device needed): sums16 = the float sums the GPU
 * returns per pass [sum src xyz(3), sum tgt xyz(3), count (uint32 bits), sigma accumulator (9,
 * row-major target x source): unscaled for order 1] -> the incremental transform (row-major 4x4
 * float) through the float JacobiSVD (pcl::umeyama(src, dst, false) [U], Eigen 3.3 Umeyama.h).  */
int lio_icp_umeyama_pcl_float(const float* sums16, float* T16);
/* As above for summation order `order` (lio_icp_params.umeyama_float 1..3: orders 2 / 3 return sigma
 * already scaled by 1/n, as Eigen's GEMM leaves it).                                            */
int lio_icp_umeyama_pcl_float_order(const float* sums16, int order, float* T16);
/* Diagnostics of the float fidelity modes: out4 = [verification re-passes, serial fallbacks, events of
 * the last pass (max over chains), passes run] since the handle was created.  Test hook: flags bit 0
 * makes the first seqsum pass skip its grid-coarsening event rule (verification then fails and the
 * re-pass path runs); flags & 4 reports a compaction look-back time-out on every pass (the pass then
 * re-compacts on the serial kernels and clears the flag); evcap > 0 caps the events per chain
 * (overflow -> the serial fallback).                                                              */
int lio_icp_get_fidelity_stats(lio_icp* h, int64_t* out4);
int lio_icp_set_fidelity_debug(lio_icp* h, int flags, int64_t evcap);
/* Test hook: sequential float sums of 6 interleaved chains (x: n x 6 host floats) on `device` through
 * the seqsum path — sums6[c] = fl(...fl(x[0][c] + x[1][c]) ... + x[n-1][c]); passes_out = passes used
 * (-1: the serial kernel was needed).                                                             */
int lio_seqsum6(int device, const float* x, int64_t n, int flags, float* sums6, int* passes_out);
/* Device-side exchange (the form to use with RCCL): per pass the statistics kernel writes this rank's
 * records into a DEVICE send buffer, `fn` enqueues the all-gather of n doubles per rank into the
 * device recv buffer (world * n, rank order) ordered on `stream` (RCCL in-stream, or a collective on
 * torch.cuda.ExternalStream(stream)), the handle enqueues the record-order sum behind it and reads 17
 * doubles back: one host wait per pass, no host copies of the records.  Buffers: the handle's own,
 * or the caller's (lio_icp_set_exchange_buffers, e.g. tensors a collective library registered);
 * capacity lio_icp_exchange_len(n_source, world) doubles per rank.  The n of a call may be less than
 * the capacity and differs between the calls of a pass, the same on every rank: the records (double
 * statistics, fitness passes); in the PCL float modes (the default) three all-gathers per pass — the
 * records followed by the window's chain totals, the window's float-chain event lists (and its first
 * pairs), the window's GEMM depth blocks (lio_icp_host.cpp, lio_seqsum.hpp); recv holds rank r at r * n. */
typedef int (*lio_allgather_dev_fn)(const double* d_send, int64_t n, double* d_recv, void* stream, void* user);
int lio_icp_set_shard_device(lio_icp* h, int rank, int world, lio_allgather_dev_fn fn, void* user);
int lio_icp_exchange_len(int64_t n_source, int world, int64_t* n_per_rank);
int lio_icp_set_exchange_buffers(lio_icp* h, double* d_send, double* d_recv, int64_t n_per_rank);
/* Multi-process exchanges in C++ (no callback into the caller per pass; lio_icp_mp.cpp):
 *  RCCL: rank 0 calls lio_rccl_unique_id, the caller broadcasts the 128 bytes to every rank ONCE (e.g. over
 *  torch.distributed), then every rank calls lio_icp_set_shard_rccl (collective: ncclCommInitRank on the
 *  handle's device); per pass ncclAllGather is enqueued on the handle's stream and the records are summed in
 *  record order behind it.  The communicator is owned by the handle.                                       */
int lio_rccl_unique_id(uint8_t* id128);
int lio_icp_set_shard_rccl(lio_icp* h, int rank, int world, const uint8_t* id128);
/*  Shared memory (ranks on one node without RCCL, e.g. several ranks on one GPU): `name` = a POSIX shm name
 *  ("/..."), rank 0 opens first (the caller orders it, e.g. a barrier), max_source_points sizes the segment.
 *  The bare primitive (host only, no device): lio_shm_exchange_* — n doubles from every rank, rank order.  */
int lio_icp_set_shard_shm(lio_icp* h, int rank, int world, const char* name, int64_t max_source_points);
int lio_shm_exchange_open(const char* name, int rank, int world, int64_t n_per_rank, void** out);
int lio_shm_exchange_allgather(void* ex, const double* send, int64_t n, double* recv);
int lio_shm_exchange_close(void* ex);
/* barrier timeout of an exchange (default 60 s; tests shorten it).  A timed-out barrier POISONS the
 * segment: every later all-gather on it, on every rank, fails (the arrival count is no longer exact).   */
int lio_shm_exchange_set_timeout(void* ex, double seconds);
/* align(guess) + getFitnessScore() + is_valid decision (loop_closure.cpp:81-90).
 * aligned_opt (n*3, this rank's shard only when sharded) may be NULL.      */
int lio_icp_align(lio_icp* h, const float* guess16, lio_icp_result* out, float* aligned_opt);
/* Diagnostics: the 1-NN of the last pass (after lio_icp_align: the
 * getFitnessScore pass) per source point of this rank's shard: target index
 * (input order of lio_icp_set_target) and float squared distance.          */
int lio_icp_get_correspondences(lio_icp* h, int32_t* ids, float* d2);
/* Single-process multi-GPU loop ICP for a C++ host: one
 * lio_icp per device (devices NULL => 0 .. n_gpus-1), the source sharded in
 * 4096-point records, the target replicated; per iteration the ranks' records
 * are all-gathered over RCCL (ncclCommInitAll + ncclAllGather; librccl is
 * opened at creation) and summed in record order, so the transform is
 * bit-identical to one GPU.  LIO_ICP_EXCHANGE=host (or the same device listed
 * twice) swaps the records through host memory instead.  A failed rank aborts
 * the group (recreate it).  Replaces LoopClosure's ICP instance
 * (loop_closure.cpp:3-14) when several GPUs serve the loop-closure thread.  */
typedef struct lio_icp_group lio_icp_group;
int lio_icp_group_create(const lio_icp_params* p, int n_gpus, const int* devices, lio_icp_group** out);
int lio_icp_group_destroy(lio_icp_group* g);
int lio_icp_group_size(const lio_icp_group* g);
int lio_icp_group_uses_rccl(const lio_icp_group* g);
int lio_icp_group_set_target(lio_icp_group* g, const float* xyz, int64_t n);
int lio_icp_group_set_source(lio_icp_group* g, const float* xyz, int64_t n);
/* as lio_icp_align; aligned_opt is the whole n*3 cloud (each rank fills its shard) */
int lio_icp_group_align(lio_icp_group* g, const float* guess16, lio_icp_result* out, float* aligned_opt);
/* One-shot form (SURVEY §8(b) signature): n_gpus <= 1 runs on p->device, n_gpus > 1 on devices
 * p->device .. p->device + n_gpus - 1 through lio_icp_group.                                     */
int icp_align(const float* src_xyz, int64_t ns, const float* dst_xyz, int64_t nd, const lio_icp_params* p,
              int n_gpus, float* T_out, double* fitness, int* converged, int* iters, float* aligned_xyz_opt);

/* FAST-LIO map_incremental() [U] for the ctx's current scan: world points
 * with the final pose, Nearest_Points from the ctx's last kNN evaluation
 * (lio_match / lio_ieskf_update with redo), PointToAdd / PointNoNeedDownsample
 * classification on filter_size_map (double, as laserMapping), then
 * Add_Points(PointToAdd, true) and Add_Points(PointNoNeedDownsample, false)
 * on the ctx's map.  Invalidates the ctx's kNN lists.                      */
typedef struct lio_incremental_stats {
    int64_t n_to_add;           /* PointToAdd.size()                          */
    int64_t n_no_downsample;    /* PointNoNeedDownsample.size()               */
    int64_t n_skipped;          /* points not added                           */
    int64_t n_added_downsample; /* Add_Points(PointToAdd, true) return value  */
} lio_incremental_stats;
int lio_map_incremental(lio_ctx* c, const lio_pose* pose, double filter_size_map, lio_incremental_stats* st);
/* pose of the ctx's last kNN evaluation (the pose Nearest_Points belong to) */
int lio_ctx_get_knn_pose(lio_ctx* c, lio_pose* out);

/* ------------------------------------------ filters */
typedef struct lio_filter lio_filter;
int lio_filter_create(int device, lio_filter** out);
int lio_filter_destroy(lio_filter* f);

/* pcl::VoxelGrid<PointT>::filter, PCL 1.10 applyFilter [U] (FAST-LIO downSizeFilterSurf,
 * voxelizePcd utilities.hpp:161-183): pts is n x stride floats (x, y, z first; stride 3..8);
 * every field is averaged per voxel (downsample_all_data_ = true), summed in input order inside
 * a voxel (PCL's std::sort order there is unspecified); output in voxel-index order (out capacity
 * n x stride); non-finite points are dropped; index overflow returns the input unchanged (as PCL). */
int lio_voxel_grid(lio_filter* f, const float* pts, int64_t n, int stride, const float leaf[3], float* out,
                   int64_t* n_out);

/* One side of LoopClosure::setSrcAndDstCloud (loop_closure.cpp:42-67): the nk keyframe clouds
 * (segments [seg_off[k], seg_off[k+1]) of pts) each through transformPcd(cloud, pose_k)
 * (utilities.hpp:132-143: pcl::transformPointCloud with a double 4x4, row-major poses16[16k..]),
 * concatenated in order, then voxelizePcd(voxel_res). */
int lio_submap_voxelize(lio_filter* f, const float* pts, const int64_t* seg_off, int nk, int stride,
                        const double* poses16, float voxel_res, float* out, int64_t* n_out);

/* FAST-LIO front-end preprocessing of one raw scan [U]: Preprocess selection (every
 * point_filter_num-th point with |p| > blind), ImuProcess::UndistortPcl (sort by the per-point
 * time offset in ms, field time_field; backward propagation through the IMU poses of the scan
 * to the scan-end state `end`), then downSizeFilterSurf (VoxelGrid, filter_size_surf; 0 = off). */
typedef struct lio_imu_pose {  /* set_pose6d: offset from scan start [s], acc, gyr, vel, pos, rot */
    double offset_time;
    double acc[3], gyr[3], vel[3], pos[3];
    double rot[9];
} lio_imu_pose;
typedef struct lio_scan_prep_params {
    int point_filter_num;   /* kitti.launch:6 = 4 */
    float blind;            /* kitti.yaml:13 = 2 */
    float filter_size_surf; /* kitti.launch:9 = 0.5 */
    int time_field;         /* index of the time offset [ms] in a record (FAST-LIO's curvature) */
} lio_scan_prep_params;
/* to host memory: out capacity n x stride, *n_out records (x, y, z, ... averaged)            */
int lio_preprocess(lio_filter* f, const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                   const lio_imu_pose* poses, int n_poses, const lio_pose* end, float* out, int64_t* n_out);
/* straight into the ctx's scan (feats_down_body) without a host round trip; *n_down points */
int lio_scan_preprocess(lio_ctx* c, const float* raw, int64_t n, int stride, const lio_scan_prep_params* p,
                        const lio_imu_pose* poses, int n_poses, const lio_pose* end, int64_t* n_down);

/* feats_undistort of the ctx's last lio_scan_preprocess*: the undistorted, time-sorted records
 * before downSizeFilterSurf — what FAST-LIO publishes on /cloud_registered with dense_publish_en
 * (kitti.yaml:31), transformed to the world frame, and what fast_lio_sam keeps per keyframe
 * (pose_pcd.hpp:37-39).  *n_points (and *stride) always set; out (cap_points records) optional.    */
int lio_scan_get_undistorted(lio_ctx* c, float* out, int64_t cap_points, int64_t* n_points, int* stride);
/* The keyframe cloud fast_lio_sam builds from FAST-LIO's /cloud_registered, on the device: out (n x 4:
 * x, y, z, intensity) = T16 * pointBodyToWorld(pose, feats_undistort), T16 row-major double — pass
 * pose_eig_.inverse() for PosePcd::pcd_ (pose_pcd.hpp:22-42; utilities.hpp:132-143 transformPcd order).
 * out = NULL: count only.                                                                          */
int lio_scan_keyframe_cloud(lio_ctx* c, const lio_pose* pose, const double* T16, float* out, int64_t cap_points,
                            int64_t* n_points);

/* ------------------------------------------- wire / disk formats (§8(f) row 4) */
/* One output column of a packed point record: byte offset, sensor_msgs/PointField datatype
 * (INT8 1, UINT8 2, INT16 3, UINT16 4, INT32 5, UINT32 6, FLOAT32 7, FLOAT64 8; 0 = absent -> 0)
 * and a scale (1 = exact; e.g. a time unit -> ms as FAST-LIO's time_unit_scale).                 */
typedef struct lio_cloud_field {
    int32_t offset;
    int32_t datatype;
    float scale;
} lio_cloud_field;
/* sensor_msgs/PointCloud2 data (n_points records of point_step bytes) -> float records with one
 * column per field (pcl::fromROSMsg's field copy; other datatypes are converted to float).     */
int lio_cloud2_decode(lio_filter* f, const uint8_t* data, int64_t n_points, int32_t point_step, int is_bigendian,
                      const lio_cloud_field* fields, int n_fields, float* out);
/* float records -> little-endian FLOAT32 fields at the given offsets, other bytes zero
 * (pcl::toROSMsg of PointXYZI: x 0, y 4, z 8, intensity 16, point_step 32).                   */
int lio_cloud2_encode(lio_filter* f, const float* rec, int64_t n, int stride, const lio_cloud_field* fields,
                      int n_fields, int32_t point_step, uint8_t* data);
/* lio_scan_preprocess straight from the PointCloud2 bytes of a raw scan; fields[5] = x, y, z,
 * intensity, time (scaled to ms): one upload, decode + preprocessing on the device.            */
int lio_scan_preprocess_cloud2(lio_ctx* c, const uint8_t* data, int64_t n_points, int32_t point_step,
                               int is_bigendian, const lio_cloud_field fields[5], const lio_scan_prep_params* p,
                               const lio_imu_pose* poses, int n_poses, const lio_pose* end, int64_t* n_down);
/* pcl::io::savePCDFileBinary (fast_lio_sam.cpp:925-932): header + packed float32 fields.       */
int lio_pcd_write_binary(const char* path, const float* rec, int64_t n, int stride, const char* const* names);
/* PCD v0.7 reader (DATA ascii | binary): POINTS and the float columns named in `want`
 * (absent fields read 0).  out == NULL returns the point count only.                           */
int lio_pcd_read(lio_filter* f, const char* path, const char* const* want, int n_want, float* out, int64_t cap,
                 int64_t* n_points);
/* a saved map (x y z of a PCD file) straight into the GPU grid (ikdtree.Build)                   */
int lio_map_build_pcd(lio_map* m, const char* path);

/* ----------------------------------------------------------------- timing */
typedef struct lio_kernel_timing {
    int64_t knn_launches;   double knn_ms;     /* kNN h-evaluation: near + far + plane kernels  */
    int64_t reuse_launches; double reuse_ms;   /* converge=false re-evaluation kernel         */
    int64_t icp_launches;   double icp_ms;     /* ICP correspondence + statistics kernels     */
    int64_t near_launches;  double near_ms;    /* kNN near pass (inside knn_ms)                */
    int64_t far_launches;   double far_ms;     /* kNN far pass (inside knn_ms)                 */
    int64_t plane_launches; double plane_ms;   /* plane / H / reduction pass (inside knn_ms)   */
    int64_t icp_nn_launches; double icp_nn_ms; /* ICP correspondence kernel alone (inside icp_ms) */
} lio_kernel_timing;

/* When enabled, every front-end kernel is launched with hipExtLaunchKernel's
 * start / stop events — the kernel's own execution span, as rocprofv3 reports
 * it (no launch gaps) — and the spans accumulate here (knn_ms = near + far +
 * plane).  The ICP handle brackets its pass (both kernels) with events, and its
 * correspondence kernel alone (icp_nn_ms).                                    */
int lio_ctx_set_timing(lio_ctx* c, int enable);
int lio_ctx_get_timing(lio_ctx* c, lio_kernel_timing* out);
int lio_ctx_reset_timing(lio_ctx* c);
int lio_icp_set_timing(lio_icp* h, int enable);
int lio_icp_get_timing(lio_icp* h, lio_kernel_timing* out);

#ifdef __cplusplus
}
#endif
#endif /* LIO_GPU_H */
