// lio_kernels.hpp — kernel argument blocks and launcher declarations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lio_dev.hpp"

namespace lio {

struct MatchArgs {
    PoseArg pose;
    GridDev grid;
    const float* body;        // n*3 feats_down_body
    const float4* map_by_id;  // map points in id order (neighbour coordinates)
    int32_t* nn_idx;          // n*5 Nearest_Points ids
    float* nn_d5;             // n: 5th neighbour d2 of the last kNN (+inf when fewer than 5; seeds the next one)
    float4* planes;           // n plane (a,b,c,d) cache
    uint8_t* sel;             // n point_selected_surf
    double* partials;         // nblocks*32
    double* sums_out;         // 32 sums (host-mapped)
    unsigned long long* seq_out;  // written with `seq` after sums_out (host-mapped)
    unsigned long long seq;
    int* dbg;                 // optional n*3 search statistics (diagnostics only)
    int* far_list;            // n: points queued for the far pass
    int* far_count;           // queue length (reset to 0 by plane_kernel)
    unsigned* done_count;     // blocks of plane/reuse finished (0 between launches; the last block resets it)
    float* far_d;             // n*5 their near-pass lists
    int* far_id;
    int n;
    int max_shell;
    int prior;                // 1: nn_idx holds this scan's previous lists against the unchanged map (seeded near pass)
    float range_sq;
    float plane_thr;
    double s_coef;
    double s_gate;
    PoseArg pose_knn;         // pose of the previous kNN evaluation (seeded near pass: w_old)
    float knn_M[12];          // the same as one float affine map body -> world (row-major 3x4): the seeded
                              // pass's displacement bound (error covered by a margin)
    float seed_scale;         // seeded bound factor: 1 (lio_ctx_set_seed_scale < 1 forces the not-full guard: tests)
};

// marks (optional, timing): 8 events, start / stop of near, far, plane (redo) or reuse (marks[6..7]),
// recorded by hipExtLaunchKernel at each kernel's own start and end.  Returns the plane / reuse grid.
int launch_h_model(const MatchArgs& a, bool redo, hipStream_t st, hipEvent_t* marks = nullptr);
void launch_debug(const MatchArgs& a, float* world, float* d2, float* abcd_pd2, hipStream_t st);
void launch_h_rows(const MatchArgs& a, double* rows, int64_t max_rows, int64_t* n_rows, hipStream_t st);
int match_blocks(int n);
// batch Nearest_Search: k <= 5 neighbours per query within d2 <= bound (INFINITY: unbounded)
void launch_map_knn(const GridDev& g, const float* q, int n, float bound, int max_shell, int k, int32_t* idx,
                    float* d2, hipStream_t st);

// --------------------------------------------------------------- grid build
struct GridGeom {
    float ox, oy, oz, cell;
    int nx, ny, nz;
    uint32_t ncells;
};

// Device buffers owned by a grid (map or ICP target).
//   by_id[id]   (x, y, z, alive 1/0) for every id ever inserted (ids are
//               insertion order; deleted ids stay as tombstones)
//   dense grids (ICP target / source binning): pts[j] sorted by (cell, id),
//               start[c] CSR offsets (ncells + 1): a row of cells is one range
//   gapped grids (the front-end map, `gapped`): each cell owns a block of slots
//               [rng[c].x, lim[c]) of which [rng[c].x, rng[c].y) are live,
//               (cell, id)-sorted; inserts fill a block's spare room or move the
//               cell to a bigger block bump-allocated at the end of pts, deletes
//               compact the block in place — O(points changed) per update, the
//               whole map is re-laid only when the slot pool runs out.
struct GridBuf {
    float4* pts = nullptr;      // points grouped by cell
    uint32_t* ckeys = nullptr;  // dense grids: cell of pts[j]
    float4* by_id = nullptr;    // id order
    uint32_t* start = nullptr;  // ncells + 1 (+ histogram scratch)
    int64_t n = 0, cap = 0;     // alive entries / entry capacity (sort scratch, dense pts)
    int64_t n_ids = 0, id_cap = 0;
    uint32_t cells_cap = 0;
    GridGeom geom{};
    // gapped (map) grids
    bool gapped = false;
    uint2* rng = nullptr;        // ncells: live slots of each cell
    uint32_t* lim = nullptr;     // ncells + 1: end of each cell's block
    uint32_t* addc = nullptr;    // ncells: per-cell insert counter (zero between updates)
    uint8_t* dirty = nullptr;    // ncells: cell holds deleted entries this update (zero between updates)
    uint32_t* bump = nullptr;    // device: next free slot of the pool
    int64_t slots_cap = 0;       // pts capacity in slots
    int64_t slots_used = 0;      // bump value after the last rebuild (host view; the pool's live share)
    int64_t rebuilds = 0;        // full rebuilds so far (diagnostics: lio_map_get_stats)
    int64_t slots_extra = 0;     // test hook (lio_map_set_test_limits): usable pool = slots_used + this (0: all)
    int64_t min_entries = 0;     // capacity floors (the loop ICP's grids: sized once for its largest submaps)
    uint32_t min_cells = 0;
    // temporaries
    uint32_t* keys = nullptr;
    uint32_t* keys_alt = nullptr;
    uint32_t* vals = nullptr;
    uint32_t* vals_alt = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    float* aabb = nullptr;       // device 6 floats
    float* aabb_host = nullptr;  // pinned 6 floats
    float* xyz = nullptr;        // staging for host input, cap*3
};

// Build grid from device xyz (n*3), ids 0..n-1.  Synchronises the stream (AABB, pool size).
int grid_build(GridBuf& g, const float* d_xyz, int64_t n, float cell, hipStream_t st);
// Full rebuild over the alive ids of by_id; geometry = AABB + slack (+1-cell pad).
int grid_rebuild(GridBuf& g, float cell, float slack, hipStream_t st);
// Grow by_id to hold n_ids ids (contents kept).
int grid_reserve_ids(GridBuf& g, int64_t n_ids, hipStream_t st);
void grid_free(GridBuf& g);
GridDev grid_view(const GridBuf& g);

// Gapped-grid maintenance, enqueued without host synchronisation (counts live on the device):
//   compact the cells listed in dlist[0 .. *d_ndirty) (entries marked dead: id bits kNone), clearing
//   their dirty flags; then insert the ids [id0, id0 + *d_nnew) of by_id: per-cell ranks by atomics,
//   one lane per touched cell grows its block (a bigger one from the pool when full), one lane per
//   point writes it.  flags[0] |= 1: a point outside the grid, flags[0] |= 2: the pool ran out — the
//   caller then rebuilds (by_id is complete either way).  Scratch: n_max entries in tmp_cell /
//   tmp_rank / tlist (n_max >= the number of new ids and of dirty cells).
struct GridInsertScratch {
    uint32_t* tmp_cell;  // n_max
    uint32_t* tmp_rank;  // n_max
    uint32_t* tlist;     // n_max: touched cells
    uint32_t* d_ntouch;  // counter
};
void grid_compact_cells(GridBuf& g, const uint32_t* dlist, const uint32_t* d_ndirty, uint32_t dcap, int n_max,
                        hipStream_t st);
void grid_insert_ids(GridBuf& g, int64_t id0, const uint32_t* d_nnew, int n_max, GridInsertScratch s,
                     uint32_t* flags, hipStream_t st);

// ---------------------------------------------------------------------- ICP
struct IcpArgs {
    GridDev grid;
    const float4* tgt_by_id;
    float* cur;          // n*3 incrementally transformed source (this rank's shard): written by the correspondence
                         // kernel for the statistics / compaction of the same pass
    const float* src;    // n*3 original source
    float* thist;        // the transforms applied before this pass (nT x 16 floats): the correspondence kernel
                         // rebuilds its current point from the binned source point with them (no per-pass
                         // gather of cur) and appends this pass's T
    int nT;
    int n;               // points in this shard
    int apply_T;         // apply T (float 4x4 row-major) to cur before the NN (incremental transform)
    float T[16];
    double c0[3];        // accumulation centre
    double max_d2;       // correspondence rejection (d2 > max_d2 => skip)
    int fitness;         // 1: fitness pass (src with T, unbounded, sum d2 only)
    int prior;           // 1: nn_id holds this alignment's previous correspondences (a starting bound)
    int r0;              // first bound box: the tile's cells grown by r0 target cells
    float* nn_d2;        // per point: 1-NN squared distance (n)
    int* nn_id;          //            1-NN target id
    const float4* qpts;  // source binned by tile cell: (x, y, z, local index bits), cell order
    const uint2* tiles;  // (first entry in qpts, query count <= kIcpTileQ) per tile
    const uint32_t* order;  // optional tile visit order (heaviest first, from the previous pass's costs)
    uint32_t* tile_cost;    // per tile: candidates scanned in this pass
    unsigned long long* dbg;  // optional counters (diagnostics): candidates, rings, tiles, lanes, tested
};

constexpr int kIcpSuper = 4096;    // points per exchanged partial (shard granule)
constexpr int kIcpStride = 20;     // doubles per record (17 statistics, padded)

constexpr int kIcpTileQ = 64;     // queries per tile (one wave)

// tiles of <= kIcpTileQ queries per non-empty cell of the source grid `q`
// (ceil(count / 64) tiles per cell, sizes balanced), in cell order.  Returns
// the tile count (synchronises the stream once).  tiles: capacity n + n / 64 + 1.
int icp_build_tiles(const GridBuf& q, uint2* tiles, uint32_t* scratch, void*& tmp, size_t& tmp_bytes, hipStream_t st);
void launch_icp_tiles(const IcpArgs& a, int ntiles, hipStream_t st);
// tile order for the next pass: descending log2(cost) buckets (one block)
// one record per 4096 points; with `order`, the next pass's tile order from a.tile_cost in the same launch
// With cp.pairs set (the PCL float modes' correspondence passes), the same launch compacts the accepted pairs
// in source order into cp.pairs (column-major, cp.cap per column: cur xyz, target xyz) — one record block per
// 4096 points, the records' counts chained by a look-back (cp.st / cp.ticket / cp.epoch as pcl_compact_kernel's),
// the total into *cp.d_n; a look-back time-out sets cp.ticket[1].
struct IcpCompact {
    float* pairs = nullptr;
    int64_t cap = 0;
    unsigned long long* st = nullptr;
    uint32_t* ticket = nullptr;
    uint32_t epoch = 0;
    uint32_t* d_n = nullptr;
};
void launch_icp_stats(const IcpArgs& a, double* super, hipStream_t st, uint32_t* order = nullptr, int ntiles = 0,
                      const IcpCompact* cp = nullptr);
// the all-gathered records (rank r's records from recv + r * rank_stride doubles) summed in global record
// order, one thread per statistic (the order of lio_icp_combine: bit-identical) -> out17 (host-mapped)
void launch_icp_combine(const double* recv, int64_t nsup, int world, int64_t rank_stride, double* out17, hipStream_t st);
// PCL-order fidelity mode: out16[0..5] float sums (src, tgt), [6] count bits, [7..15] sigma accumulator
// (row-major target x source) — serial float chains (one block); pairs: n * 6 floats scratch
void launch_icp_pcl_stats(const IcpArgs& a, float* pairs, int64_t cap, float* out16, hipStream_t st);
// the serial means alone (out16[0..6]; pairs compacted as a by-product): the fidelity orders' fallback
void launch_icp_pcl_means_serial(const IcpArgs& a, float* pairs, int64_t cap, float* out16, hipStream_t st);
// the same over pairs compacted already (*d_n of them), and order 1's serial sigma over them (out16[6] = n)
void launch_icp_pcl_means_pairs(const float* pairs, int64_t cap, const uint32_t* d_n, float* out16, hipStream_t st);
void launch_icp_pcl_sigma_serial(const float* pairs, int64_t cap, float* out16, hipStream_t st);

}  // namespace lio
