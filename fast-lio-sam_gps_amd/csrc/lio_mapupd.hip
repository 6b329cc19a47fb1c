// lio_mapupd.hip — incremental map maintenance on gfx950:
//
//   map_add      ikd-Tree Add_Points(PointToAdd, downsample_on) [U]
//   map_delete   ikd-Tree Delete_Point_Boxes(cub_needrm) [U]
//   incremental  FAST-LIO map_incremental() [U] over a ctx's scan
//
// Add_Points processes its points one after another; the only coupling
// between points is through their downsample voxel, so the GPU sorts the
// points by voxel (stable: input order inside a voxel) and one lane replays
// each voxel's sequence against the map points already in that voxel
// (found through the grid).  Survivors are appended to the id-order array,
// replaced points become tombstones, and the cell-sorted grid is merged
// (lio_grid.hip: grid_update), never fully re-sorted.
// Semantics restated in oracle/lio_oracle.cpp (DynMap, map_incremental).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "lio_kernels.hpp"
#include "lio_mapupd.hpp"

namespace lio {

namespace {

constexpr int kVoxBits = 21;
constexpr int kVoxOff = 1 << 20;

__device__ __forceinline__ float calc_dist(float ax, float ay, float az, float bx, float by, float bz) {
    return sqdist3(ax, ay, az, bx, by, bz);
}
__device__ __forceinline__ bool same_point(float ax, float ay, float az, float bx, float by, float bz) {
    return fabsf(ax - bx) < 1e-6f && fabsf(ay - by) < 1e-6f && fabsf(az - bz) < 1e-6f;
}

struct VoxBox {
    float lo[3], hi[3], mid[3];
};

// Add_Points box: [floor(p/ds)*ds, +ds) (float), centre min + (max-min)/2.0 (double -> float)
__device__ __forceinline__ VoxBox vox_box(float x, float y, float z, float ds) {
    VoxBox b;
    const float p[3] = {x, y, z};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        b.lo[d] = floorf(p[d] / ds) * ds;
        b.hi[d] = b.lo[d] + ds;
        b.mid[d] = (float)((double)b.lo[d] + (double)(b.hi[d] - b.lo[d]) / 2.0);
    }
    return b;
}
__device__ __forceinline__ bool in_box(const VoxBox& b, float x, float y, float z) {
    return b.lo[0] <= x && b.hi[0] > x && b.lo[1] <= y && b.hi[1] > y && b.lo[2] <= z && b.hi[2] > z;
}

__global__ void voxel_key_kernel(const float* __restrict__ xyz, int n, float ds, uint64_t* __restrict__ keys,
                                 uint32_t* __restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = 0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float f = floorf(xyz[3 * i + d] / ds);
        const int v = (int)fminf(fmaxf(f, (float)-kVoxOff), (float)(kVoxOff - 1));
        k = (k << kVoxBits) | (uint64_t)(uint32_t)(v + kVoxOff);
    }
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

// One wave per voxel run of the sorted keys: replay Add_Points' sequence for
// the run's points against the alive map points in the voxel.
//   S := map points in the box; for each new point q (input order):
//     winner = q unless some s in S has calc_dist(s, mid) < calc_dist(q, mid)
//     if |S| > 1 or same_point(q, winner): S := {winner}, counter++
// The 64 lanes stride the box's cells (count + first nearest-to-centre point
// in visit order = a min over (d, visit index)), lane 0 replays the run's few
// new points, and the lanes stride again to write the tombstones
// (by_id[id].w = 0 and the entry's survivor flag) of replaced map points.
// add_flag[i] marks the new point that survives (at most one per voxel).
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ void __launch_bounds__(256) voxel_resolve_kernel(const uint64_t* __restrict__ skeys,
                                                           const uint32_t* __restrict__ svals, int n,
                                                           const float* __restrict__ xyz, float ds, GridDev g,
                                                           int grid_n, float4* __restrict__ by_id,
                                                           uint32_t* __restrict__ entry_alive,
                                                           uint8_t* __restrict__ add_flag, int* __restrict__ trig_out,
                                                           int* __restrict__ dead_out) {
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);  // one sorted position per wave
    if (j >= n) return;
    const uint64_t key = skeys[j];
    if (j > 0 && skeys[j - 1] == key) {  // not a run head (wave-uniform)
        if (lane == 0) trig_out[j] = dead_out[j] = 0;
        return;
    }
    const int i0 = (int)svals[j];
    const VoxBox b = vox_box(xyz[3 * i0], xyz[3 * i0 + 1], xyz[3 * i0 + 2], ds);
    // ---- map points in the box: a point p with lo <= p < hi has its (clamped) cell
    // between the cells of lo and of the largest float below hi — the build's
    // cell assignment is monotone in each coordinate — so no margin is needed
    int x0 = 0, x1 = -1, y0 = 0, y1 = -1, z0 = 0, z1 = -1;
    if (grid_n > 0) {
        x0 = min(max(cell_coord(b.lo[0], g.ox, g.inv_cell), 0), g.nx - 1);
        x1 = min(max(cell_coord(nextafterf(b.hi[0], -INFINITY), g.ox, g.inv_cell), 0), g.nx - 1);
        y0 = min(max(cell_coord(b.lo[1], g.oy, g.inv_cell), 0), g.ny - 1);
        y1 = min(max(cell_coord(nextafterf(b.hi[1], -INFINITY), g.oy, g.inv_cell), 0), g.ny - 1);
        z0 = min(max(cell_coord(b.lo[2], g.oz, g.inv_cell), 0), g.nz - 1);
        z1 = min(max(cell_coord(nextafterf(b.hi[2], -INFINITY), g.oz, g.inv_cell), 0), g.nz - 1);
    }
    // one pass over the box's cells: count, first nearest-to-centre point in visit order (a min over
    // (d, visit index)), and each lane keeps its own in-box entries (up to kRec) for the tombstones,
    // so the cells are walked again only when some lane saw more (rare: a voxel holds a few points)
    constexpr int kRec = 2;
    int cnt_e = 0;
    unsigned long long best = ~0ull, lbest = ~0ull;  // (float bits of d, visit index)
    int lb_id = -1;
    float lbx = 0.f, lby = 0.f, lbz = 0.f;
    uint32_t rk[kRec] = {0u, 0u};
    int rid[kRec] = {-1, -1};
    bool ovf = false;
    uint32_t visit = 0;
    for (int z = z0; z <= z1; ++z)
        for (int y = y0; y <= y1; ++y)
            for (int x = x0; x <= x1; ++x) {
                const uint32_t c = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x;
                const uint32_t cb = g.start[c], ce = g.start[c + 1];
                for (uint32_t k = cb + (uint32_t)lane; k < ce; k += 64) {
                    const float4 p = g.pts[k];
                    if (!in_box(b, p.x, p.y, p.z)) continue;
                    const int id = __float_as_int(p.w);
                    if (cnt_e < kRec) {
                        rk[cnt_e == 0 ? 0 : 1] = k;
                        rid[cnt_e == 0 ? 0 : 1] = id;
                    } else {
                        ovf = true;
                    }
                    ++cnt_e;
                    const float t = calc_dist(p.x, p.y, p.z, b.mid[0], b.mid[1], b.mid[2]);
                    const unsigned long long kk = ((unsigned long long)__float_as_uint(t) << 32) | (visit + (k - cb));
                    if (kk < lbest) {
                        lbest = kk;
                        lb_id = id;
                        lbx = p.x;
                        lby = p.y;
                        lbz = p.z;
                    }
                }
                visit += ce - cb;
            }
    const int my_cnt = cnt_e;
    cnt_e = wave_sum_i32(cnt_e);
    best = wave_min_u64(lbest);
    const bool any_ovf = __any(ovf);
    // best's entry: from the lane that holds it (visit indices are unique: exactly one lane)
    int best_id = -1;
    float bx = 0.f, by = 0.f, bz = 0.f, best_d = INFINITY;
    if (cnt_e > 0) {
        best_d = __uint_as_float((uint32_t)(best >> 32));
        const uint64_t wm = __ballot(lbest == best);
        const int wl = __ffsll((unsigned long long)wm) - 1;
        best_id = __builtin_amdgcn_readlane(lb_id, wl);
        bx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbx), wl));
        by = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lby), wl));
        bz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbz), wl));
    }
    // ---- replay the run: the lanes load 64 of its points at a time (the run is
    // a prefix of the chunk: keys are sorted), every lane replays them in order
    // from the broadcast values (wave-uniform state)
    int surv_new = -1;
    float sx = bx, sy = by, sz = bz, sd = best_d;
    int triggers = 0;
    bool first = true;
    for (int k = j;; k += 64) {
        const int kk = k + lane;
        const bool in = kk < n && skeys[kk] == key;
        const int m = __popcll(__ballot(in));
        int il = 0;
        float lx = 0.f, ly = 0.f, lz = 0.f;
        if (in) {
            il = (int)svals[kk];
            lx = xyz[3 * il];
            ly = xyz[3 * il + 1];
            lz = xyz[3 * il + 2];
        }
        for (int l = 0; l < m; ++l) {
            const int i = __builtin_amdgcn_readlane(il, l);
            const float qx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lx), l));
            const float qy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ly), l));
            const float qz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lz), l));
            const float qd = calc_dist(qx, qy, qz, b.mid[0], b.mid[1], b.mid[2]);
            const int size_s = first ? cnt_e : 1;
            const bool q_wins = size_s == 0 || !(sd < qd);
            if (size_s > 1 || q_wins || same_point(qx, qy, qz, sx, sy, sz)) {
                ++triggers;
                if (q_wins) {
                    surv_new = i;
                    sx = qx;
                    sy = qy;
                    sz = qz;
                    sd = qd;
                }
            }
            first = false;
        }
        if (m < 64) break;
    }
    // ---- tombstones: every map point of the box except a surviving map point
    int dead = 0;
    if (cnt_e > 0 && (surv_new >= 0 || cnt_e > 1) && !any_ovf) {  // from the lanes' own records
#pragma unroll
        for (int r = 0; r < kRec; ++r) {
            if (r >= my_cnt) break;
            const int id = rid[r];
            if (surv_new < 0 && id == best_id) continue;
            by_id[id].w = 0.f;
            entry_alive[rk[r]] = 0u;
            ++dead;
        }
        dead = wave_sum_i32(dead);
    } else if (cnt_e > 0 && (surv_new >= 0 || cnt_e > 1)) {
        for (int z = z0; z <= z1; ++z)
            for (int y = y0; y <= y1; ++y)
                for (int x = x0; x <= x1; ++x) {
                    const uint32_t c = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x;
                    for (uint32_t k = g.start[c] + (uint32_t)lane; k < g.start[c + 1]; k += 64) {
                        const float4 p = g.pts[k];
                        if (!in_box(b, p.x, p.y, p.z)) continue;
                        const int id = __float_as_int(p.w);
                        if (surv_new < 0 && id == best_id) continue;
                        by_id[id].w = 0.f;
                        entry_alive[k] = 0u;
                        ++dead;
                    }
                }
        dead = wave_sum_i32(dead);
    }
    if (lane == 0) {  // per-run counts, summed by a reduction (no contended atomics)
        if (surv_new >= 0) add_flag[surv_new] = 1;
        trig_out[j] = triggers;
        dead_out[j] = dead;
    }
}

// append the flagged points (pos = exclusive scan of the flags) as ids id0 + pos
__global__ void append_flagged_kernel(const float* __restrict__ xyz, const uint8_t* __restrict__ flag,
                                      const uint32_t* __restrict__ pos, int n, int64_t id0,
                                      float4* __restrict__ by_id) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    by_id[id0 + pos[i]] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.f);
}

__global__ void append_all_kernel(const float* __restrict__ xyz, int n, int64_t id0, float4* __restrict__ by_id) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    by_id[id0 + i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.f);
}

__global__ void u8_to_u32_kernel(const uint8_t* __restrict__ f, int n, uint32_t* __restrict__ o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) o[i] = i < n ? (uint32_t)f[i] : 0u;
}

// Delete_Point_Boxes: alive ids inside any box (min <= x < max) -> tombstones
__global__ void delete_boxes_kernel(float4* __restrict__ by_id, int64_t n, const float* __restrict__ boxes, int nb,
                                    int* __restrict__ counter) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int hit = 0;
    if (i < n) {
        const float4 p = by_id[i];
        if (p.w != 0.f) {
            for (int k = 0; k < nb; ++k) {
                const float* bx = boxes + 6 * k;
                if (bx[0] <= p.x && bx[3] > p.x && bx[1] <= p.y && bx[4] > p.y && bx[2] <= p.z && bx[5] > p.z) {
                    by_id[i].w = 0.f;
                    hit = 1;
                    break;
                }
            }
        }
    }
    // per-block count (summed by a reduction: no contended atomics)
    __shared__ int s_cnt[4];
    const unsigned long long m = __ballot(hit);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) counter[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

// ---- map_incremental ---------------------------------------------------------
enum : uint8_t { kSkip = 0, kToAdd = 1, kNoNeed = 2 };

// FAST-LIO map_incremental() classification of one point given its nearest
// points (ascending, nf >= 1 of them).  The reference's list holds
// min(5, map size) points and its re-add loop only runs when it holds 5; list
// entries beyond the ones given here cannot pass the voxel-centre test
// (incr_classify_kernel checks that), so the loop runs over the nf given.
__device__ __forceinline__ uint8_t classify(const IncrArgs& a, float wx, float wy, float wz, const int* nn, int nf) {
    const double fs = a.fs;
    const float mx = (float)(floor((double)wx / fs) * fs + 0.5 * fs);
    const float my = (float)(floor((double)wy / fs) * fs + 0.5 * fs);
    const float mz = (float)(floor((double)wz / fs) * fs + 0.5 * fs);
    const float dist = calc_dist(wx, wy, wz, mx, my, mz);
    const float4 n0 = a.map_by_id[nn[0]];
    if (fabsf(n0.x - mx) > 0.5 * fs && fabsf(n0.y - my) > 0.5 * fs && fabsf(n0.z - mz) > 0.5 * fs) return kNoNeed;
    if (a.map_alive >= 5) {
        for (int j = 0; j < nf; ++j) {
            const float4 q = a.map_by_id[nn[j]];
            if (calc_dist(q.x, q.y, q.z, mx, my, mz) < dist) return kSkip;
        }
    }
    return kToAdd;
}

// Pass 1, lane = point: world point (final pose), classification from the
// bounded kNN lists of the last evaluation.  A bounded list equals the
// reference's unbounded 5-NN when it is full; when it is partial, the missing
// neighbours lie beyond sqrt(range) of the kNN-pose point and cannot beat the
// voxel-centre test unless the pose moved by ~sqrt(range) - 2 * half-diagonal
// (checked); otherwise (and for empty lists) the point is queued for an
// unbounded 5-NN.
__global__ void incr_classify_kernel(IncrArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
    float wx, wy, wz;
    body_to_world(a.pose, bx, by, bz, wx, wy, wz);
    a.world[3 * i] = wx;
    a.world[3 * i + 1] = wy;
    a.world[3 * i + 2] = wz;
    if (a.map_alive == 0) {
        a.cls[i] = kToAdd;
        return;
    }
    int nn[5];
    int nf = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        nn[j] = a.nn_idx[5 * i + j];
        nf += nn[j] >= 0;
    }
    bool exact = nf >= (a.map_alive < 5 ? (int)a.map_alive : 5);
    if (!exact && nf > 0) {
        float kx, ky, kz;
        body_to_world(a.pose_knn, bx, by, bz, kx, ky, kz);
        const float delta = sqrtf(sqdist3(wx, wy, wz, kx, ky, kz));
        const float hd = 0.8660254f * (float)a.fs;  // half diagonal of the voxel
        exact = sqrtf(a.range_sq) - delta - 2.f * hd > 1e-3f;
    }
    if (!exact) {
        a.cls[i] = kSkip;
        a.pending[atomicAdd(a.pending_count, 1)] = i;
        return;
    }
    a.cls[i] = classify(a, wx, wy, wz, nn, nf);
}

// Pass 2: queued points, 8 lanes each: unbounded 5-NN at the kNN-pose point
// (ikd-Tree Nearest_Search with max_dist = INF), then the classification.
__global__ void __launch_bounds__(256) incr_pending_kernel(IncrArgs a) {
    constexpr int G = 8;
    const int sub = threadIdx.x % G;
    const int cnt = *a.pending_count;
    for (int f = blockIdx.x * (256 / G) + threadIdx.x / G; f < cnt; f += gridDim.x * (256 / G)) {
        const int i = a.pending[f];
        float kx, ky, kz;
        body_to_world(a.pose_knn, a.body[3 * i], a.body[3 * i + 1], a.body[3 * i + 2], kx, ky, kz);
        TopK<5> tk;
        tk.init(INFINITY);
        group_knn_exact<5, G>(a.grid, kx, ky, kz, 0x3fffffff, sub, tk);
        if (sub == 0) {
            int nn[5];
            int nf = 0;
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                nn[j] = tk.id(j) == kNone ? -1 : tk.id(j);
                nf += nn[j] >= 0;
            }
            a.cls[i] = classify(a, a.world[3 * i], a.world[3 * i + 1], a.world[3 * i + 2], nn, nf);
        }
    }
}

// class flags for the two compactions (slot n = 0 for the scan totals)
__global__ void incr_flags_kernel(const uint8_t* __restrict__ cls, int n, uint32_t* __restrict__ f_add,
                                  uint32_t* __restrict__ f_nn) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint8_t c = i < n ? cls[i] : kSkip;
    f_add[i] = c == kToAdd;
    f_nn[i] = c == kNoNeed;
}

__global__ void incr_scatter_kernel(const float* __restrict__ world, const uint8_t* __restrict__ cls, int n,
                                    const uint32_t* __restrict__ p_add, const uint32_t* __restrict__ p_nn,
                                    float* __restrict__ o_add, float* __restrict__ o_nn) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t c = cls[i];
    float* o = c == kToAdd ? o_add + 3 * (size_t)p_add[i] : (c == kNoNeed ? o_nn + 3 * (size_t)p_nn[i] : nullptr);
    if (!o) return;
    o[0] = world[3 * i];
    o[1] = world[3 * i + 1];
    o[2] = world[3 * i + 2];
}

#define UPD_CHK(x)                            \
    do {                                      \
        if ((x) != hipSuccess) return -2;     \
    } while (0)

template <class T>
int ensure_buf(T** p, int64_t& cap, int64_t need) {
    if (need <= cap && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const int64_t c = std::max<int64_t>(need, cap + cap / 2);
    if (hipMalloc(p, (size_t)c * sizeof(T)) != hipSuccess) {
        cap = 0;
        return -5;
    }
    cap = c;
    return 0;
}

// sort / scan scratch: grown geometrically (with a 1 MiB floor), so scans of varying size do not
// re-allocate (hipFree synchronises the device) on every call that needs a little more
int ensure_tmp(MapUpdBuf& u, size_t need) {
    if (need <= u.tmp_bytes && u.tmp) return 0;
    if (u.tmp) (void)hipFree(u.tmp);
    u.tmp = nullptr;
    const size_t c = std::max(std::max(need, u.tmp_bytes + u.tmp_bytes / 2), (size_t)1 << 20);
    if (hipMalloc(&u.tmp, c) != hipSuccess) {
        u.tmp_bytes = 0;
        return -5;
    }
    u.tmp_bytes = c;
    return 0;
}

int ensure_pts(MapUpdBuf& u, int64_t n) {
    if (n <= u.cap && u.keys) return 0;
    const int64_t c = std::max<int64_t>(n, u.cap + u.cap / 2);
    void* bufs[] = {u.keys, u.keys_alt, u.vals, u.vals_alt, u.flag, u.pos, u.flag2, u.pos2, u.cls, u.world,
                    u.xyz_a, u.xyz_b, u.pending};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    UPD_CHK(hipMalloc(&u.keys, c * sizeof(uint64_t)));
    UPD_CHK(hipMalloc(&u.keys_alt, c * sizeof(uint64_t)));
    UPD_CHK(hipMalloc(&u.vals, c * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.vals_alt, c * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.flag, (c + 1) * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.pos, (c + 1) * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.flag2, (c + 1) * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.pos2, (c + 1) * sizeof(uint32_t)));
    UPD_CHK(hipMalloc(&u.cls, c + 64));
    UPD_CHK(hipMalloc(&u.world, c * 3 * sizeof(float)));
    UPD_CHK(hipMalloc(&u.xyz_a, c * 3 * sizeof(float)));
    UPD_CHK(hipMalloc(&u.xyz_b, c * 3 * sizeof(float)));
    UPD_CHK(hipMalloc(&u.pending, c * sizeof(int)));
    u.cap = c;
    return 0;
}

int ensure_small(MapUpdBuf& u) {
    if (!u.d_small) UPD_CHK(hipMalloc(&u.d_small, 64 * sizeof(int)));
    if (!u.h_small) UPD_CHK(hipHostMalloc(&u.h_small, 64 * sizeof(int)));
    return 0;
}

int exclusive_scan(MapUpdBuf& u, const uint32_t* in, uint32_t* out, int n1, hipStream_t st) {
    size_t bytes = 0;
    UPD_CHK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n1, st));
    if (ensure_tmp(u, bytes)) return -5;
    bytes = u.tmp_bytes;
    UPD_CHK(hipcub::DeviceScan::ExclusiveSum(u.tmp, bytes, in, out, n1, st));
    return 0;
}

// Downsampled add of n device points (xyz): voxel sort + resolve; survivors'
// flags in u.cls[0..n) (as u8), their count -> *n_surv (host), triggers /
// tombstones -> counters.  Does not touch by_id beyond the tombstones.
int resolve_downsample(GridBuf& g, MapUpdBuf& u, const float* xyz, int n, float ds, int64_t extra_ids,
                       hipStream_t st) {
    const int nb = (n + 255) / 256;
    voxel_key_kernel<<<nb, 256, 0, st>>>(xyz, n, ds, u.keys, u.vals);
    size_t bytes = 0;
    UPD_CHK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, u.keys, u.keys_alt, u.vals, u.vals_alt, n, 0,
                                               3 * kVoxBits, st));
    if (ensure_tmp(u, bytes)) return -5;
    bytes = u.tmp_bytes;
    UPD_CHK(hipcub::DeviceRadixSort::SortPairs(u.tmp, bytes, u.keys, u.keys_alt, u.vals, u.vals_alt, n, 0,
                                               3 * kVoxBits, st));
    UPD_CHK(hipMemsetAsync(u.cls, 0, n, st));
    // survivor flags of the cell-sorted entries, cleared by the resolve kernel for the
    // entries it replaces (grid_update then skips its by_id gather)
    int rc = grid_reserve_entries(g, g.n_ids + n + extra_ids, st);  // no re-allocation before grid_update
    if (rc) return rc;
    UPD_CHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.flag), 1, (size_t)g.n, st));
    UPD_CHK(hipMemsetAsync(g.flag + g.n, 0, sizeof(uint32_t), st));
    g.flags_ready = true;
    int* trig = reinterpret_cast<int*>(u.pos2);  // n + n ints of scratch (pos2 / flag2 free here)
    int* dead = reinterpret_cast<int*>(u.flag2);
    voxel_resolve_kernel<<<(n + 3) / 4, 256, 0, st>>>(u.keys_alt, u.vals_alt, n, xyz, ds, grid_view(g), (int)g.n,
                                                     g.by_id, g.flag, u.cls, trig, dead);
    size_t rbytes = 0;
    UPD_CHK(hipcub::DeviceReduce::Sum(nullptr, rbytes, trig, u.d_small, n, st));
    if (ensure_tmp(u, rbytes)) return -5;
    rbytes = u.tmp_bytes;
    UPD_CHK(hipcub::DeviceReduce::Sum(u.tmp, rbytes, trig, u.d_small, n, st));
    rbytes = u.tmp_bytes;
    UPD_CHK(hipcub::DeviceReduce::Sum(u.tmp, rbytes, dead, u.d_small + 1, n, st));
    return 0;
}

}  // namespace

void mapupd_free(MapUpdBuf& u) {
    void* bufs[] = {u.keys, u.keys_alt, u.vals, u.vals_alt, u.flag, u.pos, u.flag2, u.pos2, u.cls, u.world,
                    u.xyz_a, u.xyz_b, u.pending, u.tmp, u.d_small, u.boxes};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (u.h_small) (void)hipHostFree(u.h_small);
    u = MapUpdBuf{};
}

// Add_Points(xyz[0..n), downsample) for device points; out: [triggers/added, tombstones]
int map_add_device(GridBuf& g, MapUpdBuf& u, const float* d_xyz, int64_t n64, bool downsample, float ds,
                   float slack, int64_t out[2], hipStream_t st) {
    out[0] = out[1] = 0;
    if (n64 <= 0) return 0;
    if (n64 >= (int64_t)1 << 30) return -1;
    const int n = (int)n64;
    if (ensure_pts(u, n) || ensure_small(u)) return -5;
    const int64_t id0 = g.n_ids;
    if (!downsample) {
        int rc = grid_reserve_ids(g, id0 + n, st);
        if (rc) return rc;
        append_all_kernel<<<(n + 255) / 256, 256, 0, st>>>(d_xyz, n, id0, g.by_id);
        g.n_ids = id0 + n;
        out[0] = n;
        return grid_update(g, id0, false, slack, st);
    }
    UPD_CHK(hipMemsetAsync(u.d_small, 0, 4 * sizeof(int), st));
    int rc = resolve_downsample(g, u, d_xyz, n, ds, 0, st);
    if (rc) return rc;
    u8_to_u32_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(u.cls, n, u.flag);
    rc = exclusive_scan(u, u.flag, u.pos, n + 1, st);
    if (rc) return rc;
    UPD_CHK(hipMemcpyAsync(u.h_small, u.d_small, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    UPD_CHK(hipMemcpyAsync(u.h_small + 2, u.pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    UPD_CHK(hipStreamSynchronize(st));
    const int64_t n_surv = (uint32_t)u.h_small[2];
    out[0] = u.h_small[0];
    out[1] = u.h_small[1];
    rc = grid_reserve_ids(g, id0 + n_surv, st);
    if (rc) return rc;
    append_flagged_kernel<<<(n + 255) / 256, 256, 0, st>>>(d_xyz, u.cls, u.pos, n, id0, g.by_id);
    g.n_ids = id0 + n_surv;
    return grid_update(g, id0, out[1] > 0, slack, st);
}

int map_delete_boxes(GridBuf& g, MapUpdBuf& u, const float* boxes, int nb, float slack, int64_t* n_deleted,
                     hipStream_t st) {
    *n_deleted = 0;
    g.flags_ready = false;  // tombstones come from the alive bits here
    if (nb <= 0 || g.n_ids == 0) return 0;
    if (ensure_small(u)) return -5;
    if (!u.boxes || nb > u.boxes_cap) {
        if (u.boxes) (void)hipFree(u.boxes);
        UPD_CHK(hipMalloc(&u.boxes, (size_t)nb * 6 * sizeof(float)));
        u.boxes_cap = nb;
    }
    UPD_CHK(hipMemcpyAsync(u.boxes, boxes, (size_t)nb * 6 * sizeof(float), hipMemcpyHostToDevice, st));
    const int nblk = (int)((g.n_ids + 255) / 256);
    if (ensure_pts(u, nblk)) return -5;
    int* cnt = reinterpret_cast<int*>(u.flag2);
    delete_boxes_kernel<<<nblk, 256, 0, st>>>(g.by_id, g.n_ids, u.boxes, nb, cnt);
    size_t bytes = 0;
    UPD_CHK(hipcub::DeviceReduce::Sum(nullptr, bytes, cnt, u.d_small, nblk, st));
    if (ensure_tmp(u, bytes)) return -5;
    bytes = u.tmp_bytes;
    UPD_CHK(hipcub::DeviceReduce::Sum(u.tmp, bytes, cnt, u.d_small, nblk, st));
    UPD_CHK(hipMemcpyAsync(u.h_small, u.d_small, sizeof(int), hipMemcpyDeviceToHost, st));
    UPD_CHK(hipStreamSynchronize(st));
    *n_deleted = u.h_small[0];
    if (*n_deleted == 0) return 0;
    return grid_update(g, g.n_ids, true, slack, st);
}

// map_incremental(): classification (+ unbounded 5-NN for queued points), then
// Add_Points(PointToAdd, true) and Add_Points(PointNoNeedDownsample, false)
// with one grid merge.  out: [to_add, no_need, skipped, added_by_downsample_call]
int map_incremental(GridBuf& g, MapUpdBuf& u, IncrArgs a, float ds, float slack, int64_t out[4], hipStream_t st) {
    for (int k = 0; k < 4; ++k) out[k] = 0;
    const int n = a.n;
    if (n <= 0) return 0;
    if (ensure_pts(u, n) || ensure_small(u)) return -5;
    a.grid = grid_view(g);
    a.map_by_id = g.by_id;
    a.map_alive = g.n;
    a.world = u.world;
    a.cls = u.cls;
    a.pending = u.pending;
    a.pending_count = u.d_small + 8;
    UPD_CHK(hipMemsetAsync(u.d_small, 0, 16 * sizeof(int), st));
    const int nb = (n + 255) / 256;
    incr_classify_kernel<<<nb, 256, 0, st>>>(a);
    incr_pending_kernel<<<128, 256, 0, st>>>(a);
    incr_flags_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(u.cls, n, u.flag, u.flag2);
    int rc = exclusive_scan(u, u.flag, u.pos, n + 1, st);
    if (rc) return rc;
    rc = exclusive_scan(u, u.flag2, u.pos2, n + 1, st);
    if (rc) return rc;
    incr_scatter_kernel<<<nb, 256, 0, st>>>(u.world, u.cls, n, u.pos, u.pos2, u.xyz_a, u.xyz_b);
    UPD_CHK(hipMemcpyAsync(u.h_small + 2, u.pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    UPD_CHK(hipMemcpyAsync(u.h_small + 3, u.pos2 + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    UPD_CHK(hipStreamSynchronize(st));
    const int n_add = (int)(uint32_t)u.h_small[2], n_nn = (int)(uint32_t)u.h_small[3];
    out[0] = n_add;
    out[1] = n_nn;
    out[2] = n - n_add - n_nn;
    const int64_t id0 = g.n_ids;
    int64_t n_surv = 0, dead = 0;
    if (n_add > 0) {
        rc = resolve_downsample(g, u, u.xyz_a, n_add, ds, n_nn, st);  // cls reused as survivor flags
        if (rc) return rc;
        u8_to_u32_kernel<<<(n_add + 1 + 255) / 256, 256, 0, st>>>(u.cls, n_add, u.flag);
        rc = exclusive_scan(u, u.flag, u.pos, n_add + 1, st);
        if (rc) return rc;
        UPD_CHK(hipMemcpyAsync(u.h_small, u.d_small, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        UPD_CHK(hipMemcpyAsync(u.h_small + 2, u.pos + n_add, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        UPD_CHK(hipStreamSynchronize(st));
        out[3] = u.h_small[0];
        dead = u.h_small[1];
        n_surv = (uint32_t)u.h_small[2];
    }
    rc = grid_reserve_ids(g, id0 + n_surv + n_nn, st);
    if (rc) return rc;
    if (n_surv > 0) append_flagged_kernel<<<(n_add + 255) / 256, 256, 0, st>>>(u.xyz_a, u.cls, u.pos, n_add, id0, g.by_id);
    if (n_nn > 0) append_all_kernel<<<(n_nn + 255) / 256, 256, 0, st>>>(u.xyz_b, n_nn, id0 + n_surv, g.by_id);
    g.n_ids = id0 + n_surv + n_nn;
    return grid_update(g, id0, dead > 0, slack, st);
}

namespace {
__global__ void gather_ids_kernel(const float4* __restrict__ by_id, int64_t n_ids, const int32_t* __restrict__ ids,
                                  int64_t n, float* __restrict__ xyz) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t id = ids[i];
    float4 p = make_float4(NAN, NAN, NAN, 0.f);
    if (id >= 0 && id < n_ids) p = by_id[id];
    xyz[3 * i] = p.x;
    xyz[3 * i + 1] = p.y;
    xyz[3 * i + 2] = p.z;
}
}  // namespace

void map_gather_ids(const GridBuf& g, const int32_t* d_ids, int64_t n, float* d_xyz, hipStream_t st) {
    if (n <= 0) return;
    gather_ids_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(g.by_id, g.n_ids, d_ids, n, d_xyz);
}

}  // namespace lio
