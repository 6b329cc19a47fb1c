// lio_grid.hip — dense uniform grid build on gfx950 (the ikd-Tree Build [U]
// replacement): AABB reduction -> linear cell keys -> radix sort (key, id)
// -> cell histogram + exclusive scan -> float4 gather (sorted + id order).
// Layout rationale: the kNN reads a query's neighbour cells as short runs of
// contiguous 16-B points; x is the fastest grid axis so a 3-cell row is one
// contiguous run of the sorted array and one or two cache lines of start[].
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "lio_kernels.hpp"

namespace lio {

// AABB (+ alive count) over the alive entries of the id-order array.
__global__ void aabb_partial_kernel(const float4* __restrict__ by_id, int64_t n, float* __restrict__ part,
                                    uint32_t* __restrict__ alive_count) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t cnt = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 p = by_id[i];
        if (p.w == 0.f) continue;
        ++cnt;
        lo[0] = fminf(lo[0], p.x);
        lo[1] = fminf(lo[1], p.y);
        lo[2] = fminf(lo[2], p.z);
        hi[0] = fmaxf(hi[0], p.x);
        hi[1] = fmaxf(hi[1], p.y);
        hi[2] = fmaxf(hi[2], p.z);
    }
    __shared__ float s[6][256];
    __shared__ uint32_t sc;
    if (threadIdx.x == 0) sc = 0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        s[d][threadIdx.x] = lo[d];
        s[3 + d][threadIdx.x] = hi[d];
    }
    __syncthreads();
    if (cnt) atomicAdd(&sc, cnt);
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                s[d][threadIdx.x] = fminf(s[d][threadIdx.x], s[d][threadIdx.x + w]);
                s[3 + d][threadIdx.x] = fmaxf(s[3 + d][threadIdx.x], s[3 + d][threadIdx.x + w]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
    if (threadIdx.x == 0 && sc) atomicAdd(alive_count, sc);
}

// min/max over the block partials: 256 threads stride the partials, then an
// LDS tree (min/max are order-independent, so this is exact)
__global__ void __launch_bounds__(256) aabb_final_kernel(const float* __restrict__ part, int nb,
                                                         float* __restrict__ out) {
    __shared__ float s[6][256];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int b = threadIdx.x; b < nb; b += 256) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = fminf(lo[d], part[b * 6 + d]);
            hi[d] = fmaxf(hi[d], part[b * 6 + 3 + d]);
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        s[d][threadIdx.x] = lo[d];
        s[3 + d][threadIdx.x] = hi[d];
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                s[d][threadIdx.x] = fminf(s[d][threadIdx.x], s[d][threadIdx.x + w]);
                s[3 + d][threadIdx.x] = fmaxf(s[3 + d][threadIdx.x], s[3 + d][threadIdx.x + w]);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 6) out[threadIdx.x] = s[threadIdx.x][0];
}

// cell index of a point, clamped into the grid (build assignment); *out is set
// when the unclamped index leaves the grid (a point the geometry cannot hold)
__device__ __forceinline__ uint32_t cell_key_of(const GridGeom& g, float inv, float x, float y, float z,
                                                int* out = nullptr) {
    int cx = cell_coord(x, g.ox, inv);
    int cy = cell_coord(y, g.oy, inv);
    int cz = cell_coord(z, g.oz, inv);
    if (out && ((unsigned)cx >= (unsigned)g.nx || (unsigned)cy >= (unsigned)g.ny || (unsigned)cz >= (unsigned)g.nz))
        *out = 1;
    cx = min(max(cx, 0), g.nx - 1);
    cy = min(max(cy, 0), g.ny - 1);
    cz = min(max(cz, 0), g.nz - 1);
    return ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx;
}

__global__ void init_by_id_kernel(const float* __restrict__ xyz, int64_t n, float4* __restrict__ by_id) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    by_id[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.f);
}

// keys of every id; dead ids get the sentinel ncells (sorted past the table)
__global__ void cell_key_kernel(const float4* __restrict__ by_id, int64_t n, GridGeom g, uint32_t* __restrict__ keys,
                                uint32_t* __restrict__ vals, uint32_t* __restrict__ counts) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = by_id[i];
    uint32_t k = g.ncells;
    if (p.w != 0.f) {
        k = cell_key_of(g, 1.0f / g.cell, p.x, p.y, p.z);
        atomicAdd(&counts[k], 1u);
    }
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

__global__ void gather_kernel(const float4* __restrict__ by_id, int64_t n, const uint32_t* __restrict__ sorted_ids,
                              const uint32_t* __restrict__ sorted_keys, float4* __restrict__ pts,
                              uint32_t* __restrict__ ckeys) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t id = sorted_ids[j];
    const float4 p = by_id[id];
    pts[j] = make_float4(p.x, p.y, p.z, __int_as_float((int)id));
    ckeys[j] = sorted_keys[j];
}

// ---- incremental maintenance (merge path) ----------------------------------
// keys of the appended ids [id0, id0+n): all alive; flags points outside the grid
__global__ void new_key_kernel(const float4* __restrict__ by_id, int64_t id0, int64_t n, GridGeom g,
                               uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, int* __restrict__ outside) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float4 p = by_id[id0 + k];
    keys[k] = cell_key_of(g, 1.0f / g.cell, p.x, p.y, p.z, outside);
    vals[k] = (uint32_t)(id0 + k);
}

// survivor flags of the current cell-sorted entries (slot n = 0 for the scan total)
__global__ void alive_flag_kernel(const float4* __restrict__ pts, const float4* __restrict__ by_id, int64_t n,
                                  uint32_t* __restrict__ flag) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j > n) return;
    flag[j] = j < n ? (by_id[__float_as_int(pts[j].w)].w != 0.f ? 1u : 0u) : 0u;
}

__device__ __forceinline__ int64_t lower_bound_u32(const uint32_t* a, int64_t n, uint32_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// old entry j -> its compacted rank + the number of new entries in earlier
// cells (ties: old ids are smaller than every appended id, so old first)
__global__ void merge_old_kernel(const float4* __restrict__ pts, const uint32_t* __restrict__ ckeys, int64_t n_old,
                                 const uint32_t* __restrict__ pos, const uint32_t* __restrict__ new_keys, int64_t n_new,
                                 float4* __restrict__ pts_out, uint32_t* __restrict__ ckeys_out) {
    const int64_t j0 = blockIdx.x * (int64_t)blockDim.x, j = j0 + threadIdx.x;
    // the block's entries are cell-sorted: their cells' new keys form one narrow window of new_keys
    __shared__ int64_t s_lo, s_hi;
    if (threadIdx.x == 0) s_lo = lower_bound_u32(new_keys, n_new, ckeys[j0]);
    if (threadIdx.x == 1) s_hi = lower_bound_u32(new_keys, n_new, ckeys[min(j0 + (int64_t)blockDim.x, n_old) - 1] + 1u);
    __syncthreads();
    if (j >= n_old) return;
    if (pos && pos[j + 1] == pos[j]) return;  // deleted
    const uint32_t c = ckeys[j];
    const int64_t lo = s_lo;
    const int64_t o = (pos ? (int64_t)pos[j] : j) + lo + lower_bound_u32(new_keys + lo, s_hi - lo, c);
    pts_out[o] = pts[j];
    ckeys_out[o] = c;
}

// new entry k (sorted) -> k + the number of surviving old entries in cells <= its cell
__global__ void merge_new_kernel(const float4* __restrict__ by_id, const uint32_t* __restrict__ new_keys,
                                 const uint32_t* __restrict__ new_ids, int64_t n_new,
                                 const uint32_t* __restrict__ ckeys, int64_t n_old, const uint32_t* __restrict__ pos,
                                 float4* __restrict__ pts_out, uint32_t* __restrict__ ckeys_out) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= n_new) return;
    const uint32_t c = new_keys[k];
    const int64_t u = c == 0xffffffffu ? n_old : lower_bound_u32(ckeys, n_old, c + 1);
    const int64_t o = k + (pos ? (int64_t)pos[u] : u);
    const uint32_t id = new_ids[k];
    const float4 p = by_id[id];
    pts_out[o] = make_float4(p.x, p.y, p.z, __int_as_float((int)id));
    ckeys_out[o] = c;
}

// incremental cell table after a merge, in place: cell c starts after the surviving old entries of
// earlier cells (pos[start_old[c]], or start_old[c] with no deletions) and the new entries of
// earlier cells (lower bound of c in the sorted new keys).  Slot ncells gives the new total.
// Replaces a clear + run count + scan over all cells.
__global__ void start_update_kernel(uint32_t* __restrict__ start, uint32_t nc1, const uint32_t* __restrict__ pos,
                                    const uint32_t* __restrict__ new_keys, int64_t n_new) {
    const uint32_t c0 = blockIdx.x * 256u, c = c0 + threadIdx.x;
    // the block's cells share a narrow window of the new keys: bound it once per block
    __shared__ int64_t s_lo, s_hi;
    if (threadIdx.x == 0) s_lo = lower_bound_u32(new_keys, n_new, c0);
    if (threadIdx.x == 1) s_hi = lower_bound_u32(new_keys, n_new, c0 + 256u);
    __syncthreads();
    if (c >= nc1) return;
    const int64_t lo = s_lo;
    const uint32_t so = start[c];
    start[c] = (pos ? pos[so] : so) + (uint32_t)(lo + lower_bound_u32(new_keys + lo, s_hi - lo, c));
}

#define HIPCHK(x)                                                               \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "lio_grid: %s -> %s\n", #x, hipGetErrorString(e_)); \
            return -2;                                                          \
        }                                                                       \
    } while (0)

// scratch grown geometrically (1 MiB floor): no re-allocation (a device-wide sync) per slightly larger call
static int ensure(void** p, size_t& cap_bytes, size_t need) {
    if (need <= cap_bytes && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const size_t c = std::max(std::max(need, cap_bytes + cap_bytes / 2), (size_t)1 << 20);
    if (hipMalloc(p, c) != hipSuccess) {
        cap_bytes = 0;
        return -5;
    }
    cap_bytes = c;
    return 0;
}

void grid_free(GridBuf& g) {
    void* ptrs[] = {g.pts, g.by_id, g.start, g.keys, g.keys_alt, g.vals, g.vals_alt, g.tmp, g.aabb, g.xyz,
                    g.ckeys, g.pts_alt, g.ckeys_alt, g.flag, g.pos};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (g.aabb_host) (void)hipHostFree(g.aabb_host);
    g = GridBuf{};
}

GridDev grid_view(const GridBuf& g) {
    GridDev v;
    v.pts = g.pts;
    v.start = g.start;
    v.ox = g.geom.ox;
    v.oy = g.geom.oy;
    v.oz = g.geom.oz;
    v.cell = g.geom.cell;
    v.inv_cell = 1.0f / g.geom.cell;
    // assignment uses floorf((v - o) * inv): error << 1e-3 m for |v| < 1e4 m
    v.margin = 1e-3f + 1e-4f * g.geom.cell;
    v.nx = g.geom.nx;
    v.ny = g.geom.ny;
    v.nz = g.geom.nz;
    return v;
}

int grid_reserve_ids(GridBuf& g, int64_t n_ids, hipStream_t st) {
    if (n_ids <= g.id_cap && g.by_id) return 0;
    const int64_t cap = std::max<int64_t>(n_ids, g.id_cap + g.id_cap / 2);
    float4* nb = nullptr;
    HIPCHK(hipMalloc(&nb, cap * sizeof(float4)));
    if (g.by_id) {
        if (g.n_ids) HIPCHK(hipMemcpyAsync(nb, g.by_id, g.n_ids * sizeof(float4), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        HIPCHK(hipFree(g.by_id));
    }
    g.by_id = nb;
    g.id_cap = cap;
    return 0;
}

// per-entry buffers (cell-sorted arrays, sort scratch) for n ids; the live
// cell-sorted entries (pts, ckeys: g.n of them) are carried over
static int reserve_entries(GridBuf& g, int64_t n, hipStream_t st) {
    if (n <= g.cap && g.pts) return 0;
    const int64_t cap = std::max<int64_t>(n, g.cap + g.cap / 2);
    float4* pts = nullptr;
    uint32_t* ck = nullptr;
    HIPCHK(hipMalloc(&pts, cap * sizeof(float4)));
    HIPCHK(hipMalloc(&ck, cap * sizeof(uint32_t)));
    if (g.pts && g.n > 0) {
        HIPCHK(hipMemcpyAsync(pts, g.pts, g.n * sizeof(float4), hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(ck, g.ckeys, g.n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    void* bufs[] = {g.pts, g.keys, g.keys_alt, g.vals, g.vals_alt, g.ckeys, g.pts_alt, g.ckeys_alt, g.flag, g.pos};
    for (void* p : bufs)
        if (p) HIPCHK(hipFree(p));
    g.pts = pts;
    g.ckeys = ck;
    HIPCHK(hipMalloc(&g.pts_alt, cap * sizeof(float4)));
    HIPCHK(hipMalloc(&g.keys, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.keys_alt, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.vals, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.vals_alt, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.ckeys_alt, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.flag, (cap + 1) * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.pos, (cap + 1) * sizeof(uint32_t)));
    g.cap = cap;
    return 0;
}

static int reserve_cells(GridBuf& g, uint32_t nc1) {
    if (nc1 <= g.cells_cap && g.start) return 0;
    if (g.start) HIPCHK(hipFree(g.start));
    const uint32_t cap = std::max<uint32_t>(nc1, g.cells_cap + g.cells_cap / 2);
    HIPCHK(hipMalloc(&g.start, 2 * (size_t)cap * sizeof(uint32_t)));  // + histogram scratch
    g.cells_cap = cap;
    return 0;
}

int grid_build(GridBuf& g, const float* d_xyz, int64_t n, float cell, hipStream_t st) {
    if (n <= 0 || n >= (int64_t)0x7fffffff) return -1;
    g.n_ids = 0;
    // 1.5x headroom: the first map_incremental calls append without re-allocating (and copying) the map
    const int64_t room = n + n / 2;
    int rc = grid_reserve_ids(g, room, st);
    if (rc) return rc;
    rc = reserve_entries(g, room, st);
    if (rc) return rc;
    init_by_id_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(d_xyz, n, g.by_id);
    g.n_ids = n;
    return grid_rebuild(g, cell, 0.f, st);
}

int grid_rebuild(GridBuf& g, float cell, float slack, hipStream_t st) {
    const int64_t n_ids = g.n_ids;
    if (!(cell > 0.f)) cell = 1.0f;
    int rc = reserve_entries(g, std::max<int64_t>(n_ids, 1), st);
    if (rc) return rc;
    if (!g.aabb) HIPCHK(hipMalloc(&g.aabb, 6 * 1024 * sizeof(float) + 64));
    if (!g.aabb_host) HIPCHK(hipHostMalloc(&g.aabb_host, 64));
    // ---- AABB + alive count
    const int nbA = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n_ids + 255) / 256));
    float* part = g.aabb + 8;
    uint32_t* d_cnt = reinterpret_cast<uint32_t*>(g.aabb + 6);
    HIPCHK(hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), st));
    if (n_ids) aabb_partial_kernel<<<nbA, 256, 0, st>>>(g.by_id, n_ids, part, d_cnt);
    aabb_final_kernel<<<1, 256, 0, st>>>(part, n_ids ? nbA : 0, g.aabb);
    HIPCHK(hipMemcpyAsync(g.aabb_host, g.aabb, 7 * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const float* bb = g.aabb_host;
    uint32_t n_alive = 0;
    std::memcpy(&n_alive, bb + 6, sizeof(uint32_t));
    GridGeom geo;
    if (n_alive == 0) {  // empty map: one empty cell
        geo = GridGeom{0.f, 0.f, 0.f, cell, 1, 1, 1, 1u};
    } else {
        for (int d = 0; d < 6; ++d)
            if (!std::isfinite(bb[d])) return -1;
        // geometry: slack + 1-cell pad on every side; grow the cell if the table would exceed 2^29 cells
        for (;;) {
            double o[3], ext[3];
            for (int d = 0; d < 3; ++d) {
                o[d] = std::floor(((double)bb[d] - slack) / cell) * cell - cell;
                ext[d] = (double)bb[3 + d] + slack - o[d];
            }
            double nx = std::floor(ext[0] / cell) + 2, ny = std::floor(ext[1] / cell) + 2,
                   nz = std::floor(ext[2] / cell) + 2;
            if (nx * ny * nz <= (double)(1u << 29)) {
                geo.ox = (float)o[0];
                geo.oy = (float)o[1];
                geo.oz = (float)o[2];
                geo.cell = cell;
                geo.nx = (int)nx;
                geo.ny = (int)ny;
                geo.nz = (int)nz;
                geo.ncells = (uint32_t)(nx * ny * nz);
                break;
            }
            cell *= 2.f;
        }
    }
    g.geom = geo;
    const uint32_t nc1 = geo.ncells + 1;
    rc = reserve_cells(g, nc1);
    if (rc) return rc;
    uint32_t* counts = g.start + g.cells_cap;
    HIPCHK(hipMemsetAsync(counts, 0, (size_t)nc1 * sizeof(uint32_t), st));
    const int nb = (int)std::max<int64_t>(1, (n_ids + 255) / 256);
    if (n_ids) cell_key_kernel<<<nb, 256, 0, st>>>(g.by_id, n_ids, geo, g.keys, g.vals, counts);
    // ---- sort (key, id): stable, so ids ascend inside a cell; dead ids (key ncells) last
    int bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) <= (uint64_t)geo.ncells) ++bits;
    size_t sort_bytes = 0, scan_bytes = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, g.keys, g.keys_alt, g.vals, g.vals_alt,
                                              (int)std::max<int64_t>(n_ids, 1), 0, bits, st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, counts, g.start, (int)nc1, st));
    size_t need = std::max(sort_bytes, scan_bytes);
    if (ensure(&g.tmp, g.tmp_bytes, need) != 0) return -5;
    size_t tb = g.tmp_bytes;
    if (n_ids)
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(g.tmp, tb, g.keys, g.keys_alt, g.vals, g.vals_alt, (int)n_ids, 0,
                                                  bits, st));
    tb = g.tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(g.tmp, tb, counts, g.start, (int)nc1, st));
    if (n_alive)
        gather_kernel<<<(int)((n_alive + 255) / 256), 256, 0, st>>>(g.by_id, n_alive, g.vals_alt, g.keys_alt, g.pts,
                                                                    g.ckeys);
    HIPCHK(hipGetLastError());
    g.n = n_alive;
    return 0;
}

// Incremental update after ids [id0, n_ids) were appended to by_id (alive) and
// (when `deleted`) some earlier ids were marked dead: surviving entries and
// the new ones are merged in cell order (no full sort), start[] recounted.
// Falls back to grid_rebuild (geometry + slack) when a new point lies outside
// the grid.  Synchronises the stream once.
int grid_reserve_entries(GridBuf& g, int64_t n, hipStream_t st) { return reserve_entries(g, std::max<int64_t>(n, 1), st); }

int grid_update(GridBuf& g, int64_t id0, bool deleted, float slack, hipStream_t st) {
    const int64_t n_new = g.n_ids - id0, n_old = g.n;
    if (n_new < 0) return -1;
    if (g.flags_ready && g.cap < g.n_ids) return -1;  // the caller reserved the entries first
    int rc = reserve_entries(g, std::max<int64_t>(g.n_ids, 1), st);
    if (rc) return rc;
    int* d_out = reinterpret_cast<int*>(g.aabb + 7);  // outside flag
    HIPCHK(hipMemsetAsync(d_out, 0, sizeof(int), st));
    uint32_t* nkeys = g.keys_alt;  // sorted new (key, id)
    uint32_t* nids = g.vals_alt;
    if (n_new > 0) {
        new_key_kernel<<<(int)((n_new + 255) / 256), 256, 0, st>>>(g.by_id, id0, n_new, g.geom, g.keys, g.vals, d_out);
        size_t sort_bytes = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, g.keys, g.keys_alt, g.vals, g.vals_alt,
                                                  (int)n_new, 0, 32, st));
        if (ensure(&g.tmp, g.tmp_bytes, sort_bytes) != 0) return -5;
        size_t tb = g.tmp_bytes;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(g.tmp, tb, g.keys, g.keys_alt, g.vals, g.vals_alt, (int)n_new, 0,
                                                  32, st));
    }
    uint32_t* pos = nullptr;
    if (deleted && n_old > 0) {
        if (!g.flags_ready)  // survivor flags from the alive bits (else set by the caller's kernels)
            alive_flag_kernel<<<(int)((n_old + 1 + 255) / 256), 256, 0, st>>>(g.pts, g.by_id, n_old, g.flag);
        size_t scan_bytes = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, g.flag, g.pos, (int)(n_old + 1), st));
        if (ensure(&g.tmp, g.tmp_bytes, scan_bytes) != 0) return -5;
        size_t tb = g.tmp_bytes;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(g.tmp, tb, g.flag, g.pos, (int)(n_old + 1), st));
        pos = g.pos;
        HIPCHK(hipMemcpyAsync(g.aabb_host + 8, g.pos + n_old, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipMemcpyAsync(g.aabb_host + 7, d_out, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    int outside = 0;
    std::memcpy(&outside, g.aabb_host + 7, sizeof(int));
    g.flags_ready = false;
    if (outside || g.n == 0) return grid_rebuild(g, g.geom.cell, slack, st);
    uint32_t kept = (uint32_t)n_old;
    if (pos) std::memcpy(&kept, g.aabb_host + 8, sizeof(uint32_t));
    if (n_old > 0)
        merge_old_kernel<<<(int)((n_old + 255) / 256), 256, 0, st>>>(g.pts, g.ckeys, n_old, pos, nkeys, n_new,
                                                                     g.pts_alt, g.ckeys_alt);
    if (n_new > 0)
        merge_new_kernel<<<(int)((n_new + 255) / 256), 256, 0, st>>>(g.by_id, nkeys, nids, n_new, g.ckeys, n_old,
                                                                     pos, g.pts_alt, g.ckeys_alt);
    std::swap(g.pts, g.pts_alt);
    std::swap(g.ckeys, g.ckeys_alt);
    g.n = (int64_t)kept + n_new;
    const uint32_t nc1 = g.geom.ncells + 1;
    start_update_kernel<<<(int)((nc1 + 255) / 256), 256, 0, st>>>(g.start, nc1, pos, nkeys, n_new);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace lio
