// lio_mapupd.hpp — incremental map maintenance (lio_mapupd.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lio_kernels.hpp"

namespace lio {

// Scratch owned by a map handle (sized for the largest call so far).
struct MapUpdBuf {
    unsigned long long* f64 = nullptr;    // packed class flags (map_incremental)
    unsigned long long* pos64 = nullptr;  // their exclusive scan
    uint32_t* add_flag = nullptr;         // survivor of the downsampled add, per offered point
    uint32_t* pos = nullptr;              // its exclusive scan (survivor ids)
    uint8_t* cls = nullptr;               // per point class
    float* world = nullptr;               // n*3 world points (map_incremental)
    float* xyz_a = nullptr;               // PointToAdd
    float* xyz_b = nullptr;               // PointNoNeedDownsample
    int* pending = nullptr;               // points queued for the unbounded kNN
    uint32_t* skey = nullptr;             // voxel grouping: (table slot, input index) pairs, and the
    uint32_t* sval = nullptr;             // stable sort's output (each voxel's points contiguous,
    uint32_t* skey2 = nullptr;            // in input order)
    uint32_t* sval2 = nullptr;
    float4* xs = nullptr;                 // the offered points in that sorted order (x, y, z, -)
    uint32_t* vlist = nullptr;            // voxels touched
    uint32_t* dlist = nullptr;            // grid cells holding tombstones
    uint32_t* tmp_cell = nullptr;         // grid insert scratch
    uint32_t* tmp_rank = nullptr;
    uint32_t* tlist = nullptr;
    unsigned long long* hkey = nullptr;   // voxel table: keys (all ones = empty) ...
    int* hhead = nullptr;                 // ... and the voxel's first sorted entry / run list head (-1), clean
                                          // between calls
    int* hend = nullptr;                  // one past the voxel's last sorted entry
    uint32_t* vnruns = nullptr;           // grouped update: runs per voxel slot (zero between calls)
    uint4* runs = nullptr;                // grouped update: run records {first sorted position, count, next}
    uint32_t* blk = nullptr;              // grouped update: survivors | no-need points per sort block
    int64_t blk_cap = 0;
    uint32_t hcap = 0;
    int hbits = 0;                        // log2(hcap)
    int64_t cap = 0;
    int64_t dcap_limit = 0;               // test hook (lio_map_set_test_limits): tombstone cell list length (0: cap * 27)
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    uint32_t* cnt = nullptr;    // per-call counters (lio_mapupd.hip kC*)
    uint32_t* h_cnt = nullptr;  // pinned copy
    float* boxes = nullptr;
    int boxes_cap = 0;
};

// map_incremental inputs (per scan)
struct IncrArgs {
    PoseArg pose;      // final state (pointBodyToWorld)
    PoseArg pose_knn;  // pose of the last kNN evaluation (Nearest_Points)
    const float* body;
    const int32_t* nn_idx;  // n*5, -1 = none within range
    int n;
    double fs;        // filter_size_map_min (double, laserMapping)
    float range_sq;   // kNN range of the lists
    // filled by map_incremental()
    GridDev grid;
    const float4* map_by_id;
    int64_t map_alive;
    float* world;
    uint8_t* cls;
    int* pending;
    int* pending_count;
};

void mapupd_free(MapUpdBuf& u);
// scratch for updates of up to n offered points, allocated ahead of the first one
int mapupd_presize(MapUpdBuf& u, int64_t n, hipStream_t st);
int map_add_device(GridBuf& g, MapUpdBuf& u, const float* d_xyz, int64_t n, bool downsample, float ds, float slack,
                   int64_t out[2], hipStream_t st);
int map_delete_boxes(GridBuf& g, MapUpdBuf& u, const float* boxes, int nb, float slack, int64_t* n_deleted,
                     hipStream_t st);
int map_incremental(GridBuf& g, MapUpdBuf& u, IncrArgs a, float ds, float slack, int64_t out[4], hipStream_t st);
// xyz of map ids (Nearest_Points from ids): ids < 0 or >= n_ids -> NaN
void map_gather_ids(const GridBuf& g, const int32_t* d_ids, int64_t n, float* d_xyz, hipStream_t st);

}  // namespace lio
