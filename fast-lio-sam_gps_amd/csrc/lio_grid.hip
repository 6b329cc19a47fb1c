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

#include "lio_error.hpp"
#include "lio_grid_dev.hpp"
#include "lio_kernels.hpp"

namespace lio {

// AABB (+ alive count) over the alive entries of the id-order array.
__global__ void aabb_partial_kernel(const float4* __restrict__ by_id, int64_t n, float* __restrict__ part) {
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
    __syncthreads();  // sc complete
    // partial = 6 floats + the alive count (8-word stride): no same-address device atomics (1024 blocks
    // adding to one counter serialise at the memory-side atomic unit)
    if (threadIdx.x < 6) part[blockIdx.x * 8 + threadIdx.x] = s[threadIdx.x][0];
    if (threadIdx.x == 0) part[blockIdx.x * 8 + 6] = __uint_as_float(sc);
}

// min/max over the block partials: 256 threads stride the partials, then an
// LDS tree (min/max are order-independent, so this is exact)
// out[0..5] = AABB, out[6] = alive count (uint bits)
__global__ void __launch_bounds__(256) aabb_final_kernel(const float* __restrict__ part, int nb,
                                                         float* __restrict__ out) {
    __shared__ float s[6][256];
    __shared__ uint32_t s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t cnt = 0;
    for (int b = threadIdx.x; b < nb; b += 256) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = fminf(lo[d], part[b * 8 + d]);
            hi[d] = fmaxf(hi[d], part[b * 8 + 3 + d]);
        }
        cnt += __float_as_uint(part[b * 8 + 6]);
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
    if (cnt) atomicAdd(&s_cnt, cnt);  // LDS
    __syncthreads();
    if (threadIdx.x < 6) out[threadIdx.x] = s[threadIdx.x][0];
    if (threadIdx.x == 0) out[6] = __uint_as_float(s_cnt);
}

__global__ void init_by_id_kernel(const float* __restrict__ xyz, int64_t n, float4* __restrict__ by_id) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    by_id[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 1.f);
}

// keys of every id; dead ids get the sentinel ncells (sorted past the table)
__global__ void cell_key_kernel(const float4* __restrict__ by_id, int64_t n, GridGeom g, uint32_t* __restrict__ keys,
                                uint32_t* __restrict__ vals) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = by_id[i];
    uint32_t k = g.ncells;
    if (p.w != 0.f) k = cell_key_of(g, 1.0f / g.cell, p.x, p.y, p.z);
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

// per-cell counts from the SORTED keys: a wave's lanes hold runs of equal keys; the first lane of each run
// (inside the wave) adds the run's length — one device atomic per run piece instead of one per point
// (spatially ordered clouds put whole waves on one cell, which serialised the per-point adds)
__global__ void sorted_counts_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t ncells,
                                     uint32_t* __restrict__ counts) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t k = j < n ? keys[j] : ncells;
    const uint32_t prev = (j > 0 && j < n) ? keys[j - 1] : ~k;
    const bool head = lane == 0 || k != prev;
    const uint64_t heads = __ballot(head);
    const uint64_t above = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
    const int next = above ? __ffsll((unsigned long long)above) - 1 : 64;
    if (head && j < n && k < ncells) atomicAdd(&counts[k], (uint32_t)(next - lane));
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

// ---- gapped (map) grids -------------------------------------------------------
// block capacity of a cell holding `cnt` points at a (re)build: room for a few more (a 1 m cell of a
// 0.5 m-downsampled map holds at most 8 downsampled points, map_incremental adds a handful per scan)
__device__ __forceinline__ uint32_t cell_capacity(uint32_t cnt) { return cnt ? cnt + max(4u, cnt >> 2) : 0u; }

// lim[c] = capacity of cell c (counts: the dense CSR start[]); lim[ncells] = 0 for the scan total
__global__ void cap_kernel(const uint32_t* __restrict__ start, uint32_t nc, uint32_t* __restrict__ lim) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c > nc) return;
    lim[c] = c < nc ? cell_capacity(start[c + 1] - start[c]) : 0u;
}

// gbase = exclusive scan of the capacities: rng[c] = {gbase[c], gbase[c] + count}, lim[c] = gbase[c + 1]
__global__ void rng_kernel(const uint32_t* __restrict__ start, const uint32_t* __restrict__ gbase, uint32_t nc,
                           uint2* __restrict__ rng, uint32_t* __restrict__ lim, uint32_t* __restrict__ bump) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c >= nc) {
        if (c == nc) *bump = gbase[nc];
        return;
    }
    const uint32_t b = gbase[c];
    rng[c] = make_uint2(b, b + (start[c + 1] - start[c]));
    lim[c] = gbase[c + 1];
}

// sorted entry j of cell ck -> slot gbase[ck] + (j - start[ck]) (rank inside the cell kept: id order)
__global__ void gather_gapped_kernel(const float4* __restrict__ by_id, int64_t n, const uint32_t* __restrict__ sorted_ids,
                                     const uint32_t* __restrict__ sorted_keys, const uint32_t* __restrict__ start,
                                     const uint2* __restrict__ rng, float4* __restrict__ pts) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t id = sorted_ids[j], ck = sorted_keys[j];
    const float4 p = by_id[id];
    pts[rng[ck].x + (uint32_t)(j - start[ck])] = make_float4(p.x, p.y, p.z, __int_as_float((int)id));
}

// one WAVE per listed cell (grid-stride): lio_grid_dev.hpp compact_cell_wave
__global__ void __launch_bounds__(256) compact_cells_kernel(float4* __restrict__ pts, uint2* __restrict__ rng,
                                                            uint8_t* __restrict__ dirty, const uint32_t* __restrict__ dlist,
                                                            const uint32_t* __restrict__ d_ndirty, uint32_t dcap) {
    const uint32_t nd = min(*d_ndirty, dcap);
    for (uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6); k < nd; k += gridDim.x * 4u)  // wave-uniform
        compact_cell_wave(pts, rng, dirty, dlist[k]);
}

// new id j (0 <= j < *d_nnew): its cell and its rank among this update's points of that cell
__global__ void insert_rank_kernel(const float4* __restrict__ by_id, int64_t id0, const uint32_t* __restrict__ d_nnew,
                                   GridGeom g, uint32_t* __restrict__ addc, uint32_t* __restrict__ tmp_cell,
                                   uint32_t* __restrict__ tmp_rank, uint32_t* __restrict__ tlist,
                                   uint32_t* __restrict__ d_ntouch, uint32_t* __restrict__ flags) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = j < *d_nnew;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (act) p = by_id[id0 + j];
    insert_rank_point(act, j, p.x, p.y, p.z, g, addc, tmp_cell, tmp_rank, tlist, d_ntouch, flags);
}

// one lane per touched cell: room for its new points (a bigger block from the pool when the cell's is
// full: the live points move, the old block is left behind); addc[c] becomes the first new slot
__global__ void insert_alloc_kernel(float4* __restrict__ pts, uint2* __restrict__ rng, uint32_t* __restrict__ lim,
                                    uint32_t* __restrict__ addc, const uint32_t* __restrict__ tlist,
                                    const uint32_t* __restrict__ d_ntouch, uint32_t* __restrict__ bump,
                                    uint32_t slots_cap, uint32_t* __restrict__ flags) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= *d_ntouch) return;
    const uint32_t c = tlist[k];
    const uint32_t add = addc[c];
    uint2 r = rng[c];
    const uint32_t live = r.y - r.x;
    if (r.y + add > lim[c]) {
        const uint32_t cap = max(8u, 2u * (live + add));
        const uint32_t base = atomicAdd(bump, cap);
        if ((uint64_t)base + cap > (uint64_t)slots_cap) {  // pool exhausted: the caller rebuilds
            atomicOr(flags, 2u);
            addc[c] = 0xffffffffu;
            return;
        }
        for (uint32_t j0 = 0; j0 < live; j0 += 4) {  // four loads in flight (the new block is disjoint)
            float4 p4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) p4[u] = pts[r.x + min(j0 + (uint32_t)u, live - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j0 + (uint32_t)u < live) pts[base + j0 + (uint32_t)u] = p4[u];
        }
        r = make_uint2(base, base + live);
        lim[c] = base + cap;
    }
    addc[c] = r.y;
    rng[c] = make_uint2(r.x, r.y + add);
}

__global__ void insert_write_kernel(const float4* __restrict__ by_id, int64_t id0, const uint32_t* __restrict__ d_nnew,
                                    const uint32_t* __restrict__ tmp_cell, const uint32_t* __restrict__ tmp_rank,
                                    const uint32_t* __restrict__ addc, float4* __restrict__ pts) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *d_nnew) return;
    const uint32_t base = addc[tmp_cell[j]];
    if (base == 0xffffffffu) return;
    const uint32_t id = (uint32_t)(id0 + j);
    const float4 p = by_id[id];
    pts[base + tmp_rank[j]] = make_float4(p.x, p.y, p.z, __int_as_float((int)id));
}

__global__ void insert_clear_kernel(uint32_t* __restrict__ addc, const uint32_t* __restrict__ tlist,
                                    const uint32_t* __restrict__ d_ntouch) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < *d_ntouch) addc[tlist[k]] = 0u;
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
    count_alloc();
    if (hipMalloc(p, c) != hipSuccess) {
        cap_bytes = 0;
        return -5;
    }
    cap_bytes = c;
    return 0;
}

void grid_free(GridBuf& g) {
    void* ptrs[] = {g.pts, g.by_id, g.start, g.keys, g.keys_alt, g.vals, g.vals_alt, g.tmp, g.aabb, g.xyz,
                    g.ckeys, g.rng, g.lim, g.addc, g.dirty, g.bump};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (g.aabb_host) (void)hipHostFree(g.aabb_host);
    const bool gapped = g.gapped;
    g = GridBuf{};
    g.gapped = gapped;
}

GridDev grid_view(const GridBuf& g) {
    GridDev v;
    v.pts = g.pts;
    v.start = g.start;
    v.rng = g.rng;
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
    const int64_t cap = std::max<int64_t>(std::max<int64_t>(n_ids, g.id_cap + g.id_cap / 2), g.min_entries);
    float4* nb = nullptr;
    count_alloc();
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

// per-entry buffers for n ids: the (key, id) sort scratch, and for dense grids the cell-sorted
// arrays (gapped grids keep their points in the slot pool, reserve_slots)
static int reserve_entries(GridBuf& g, int64_t n) {
    if (n <= g.cap && g.keys) return 0;
    const int64_t cap = std::max<int64_t>(std::max<int64_t>(n, g.cap + g.cap / 2), g.min_entries);
    count_alloc(g.gapped ? 4 : 6);
    void* bufs[] = {g.keys, g.keys_alt, g.vals, g.vals_alt};
    for (void* p : bufs)
        if (p) HIPCHK(hipFree(p));
    HIPCHK(hipMalloc(&g.keys, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.keys_alt, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.vals, cap * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g.vals_alt, cap * sizeof(uint32_t)));
    if (!g.gapped) {
        if (g.pts) HIPCHK(hipFree(g.pts));
        if (g.ckeys) HIPCHK(hipFree(g.ckeys));
        g.pts = nullptr;
        g.ckeys = nullptr;
        HIPCHK(hipMalloc(&g.pts, cap * sizeof(float4)));
        HIPCHK(hipMalloc(&g.ckeys, cap * sizeof(uint32_t)));
    }
    g.cap = cap;
    return 0;
}

// gapped grids: the slot pool (contents are rewritten by the rebuild that asks for it)
static int reserve_slots(GridBuf& g, int64_t slots) {
    if (slots <= g.slots_cap && g.pts) return 0;
    if (slots >= (int64_t)0xffffffffu) return -1;
    if (g.pts) HIPCHK(hipFree(g.pts));
    g.pts = nullptr;
    g.slots_cap = 0;
    count_alloc();
    HIPCHK(hipMalloc(&g.pts, (size_t)slots * sizeof(float4)));
    g.slots_cap = slots;
    return 0;
}

static int reserve_cells(GridBuf& g, uint32_t nc1) {
    if (nc1 <= g.cells_cap && g.start) return 0;
    void* bufs[] = {g.start, g.rng, g.lim, g.addc, g.dirty};
    for (void* p : bufs)
        if (p) HIPCHK(hipFree(p));
    g.start = nullptr;
    g.rng = nullptr;
    g.lim = nullptr;
    g.addc = nullptr;
    g.dirty = nullptr;
    const uint32_t cap = std::max<uint32_t>(std::max<uint32_t>(nc1, g.cells_cap + g.cells_cap / 2), g.min_cells);
    count_alloc(g.gapped ? 5 : 1);
    HIPCHK(hipMalloc(&g.start, 2 * (size_t)cap * sizeof(uint32_t)));  // + histogram scratch
    if (g.gapped) {
        HIPCHK(hipMalloc(&g.rng, (size_t)cap * sizeof(uint2)));
        HIPCHK(hipMalloc(&g.lim, (size_t)cap * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&g.addc, (size_t)cap * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&g.dirty, (size_t)cap + 4));  // + 4: flagged through 32-bit words
        if (!g.bump) HIPCHK(hipMalloc(&g.bump, sizeof(uint32_t)));
    }
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
    rc = reserve_entries(g, room);
    if (rc) return rc;
    init_by_id_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(d_xyz, n, g.by_id);
    g.n_ids = n;
    return grid_rebuild(g, cell, 0.f, st);
}

int grid_rebuild(GridBuf& g, float cell, float slack, hipStream_t st) {
    const int64_t n_ids = g.n_ids;
    ++g.rebuilds;
    if (!(cell > 0.f)) cell = 1.0f;
    int rc = reserve_entries(g, std::max<int64_t>(n_ids, 1));
    if (rc) return rc;
    if (!g.aabb) HIPCHK(hipMalloc(&g.aabb, 8 * 1024 * sizeof(float) + 64));  // result + 8-word partials
    if (!g.aabb_host) HIPCHK(hipHostMalloc(&g.aabb_host, 64));
    // ---- AABB + alive count
    const int nbA = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n_ids + 255) / 256));
    float* part = g.aabb + 8;
    if (n_ids) aabb_partial_kernel<<<nbA, 256, 0, st>>>(g.by_id, n_ids, part);
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
    if (n_ids) cell_key_kernel<<<nb, 256, 0, st>>>(g.by_id, n_ids, geo, g.keys, g.vals);
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
    if (n_ids) {
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(g.tmp, tb, g.keys, g.keys_alt, g.vals, g.vals_alt, (int)n_ids, 0,
                                                  bits, st));
        sorted_counts_kernel<<<nb, 256, 0, st>>>(g.keys_alt, n_ids, geo.ncells, counts);
    }
    tb = g.tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(g.tmp, tb, counts, g.start, (int)nc1, st));
    if (!g.gapped) {
        if (n_alive)
            gather_kernel<<<(int)((n_alive + 255) / 256), 256, 0, st>>>(g.by_id, n_alive, g.vals_alt, g.keys_alt,
                                                                        g.pts, g.ckeys);
        HIPCHK(hipGetLastError());
        g.n = n_alive;
        return 0;
    }
    // gapped: block capacities -> block bases (scan into the histogram scratch, free after the dense scan)
    uint32_t* gbase = counts;
    const int nbc = (int)((nc1 + 255) / 256);
    cap_kernel<<<nbc, 256, 0, st>>>(g.start, geo.ncells, g.lim);
    tb = g.tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(g.tmp, tb, g.lim, gbase, (int)nc1, st));
    rng_kernel<<<nbc, 256, 0, st>>>(g.start, gbase, geo.ncells, g.rng, g.lim, g.bump);
    HIPCHK(hipMemsetAsync(g.addc, 0, (size_t)geo.ncells * sizeof(uint32_t), st));
    HIPCHK(hipMemsetAsync(g.dirty, 0, (size_t)geo.ncells, st));
    uint32_t used = 0;
    HIPCHK(hipMemcpyAsync(g.aabb_host + 9, gbase + geo.ncells, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(&used, g.aabb_host + 9, sizeof(uint32_t));
    // pool: the blocks + room for the cells that will outgrow theirs before the next rebuild
    const int64_t pool = (int64_t)used + std::max<int64_t>((int64_t)1 << 20, (int64_t)used / 2);
    rc = reserve_slots(g, pool);
    if (rc) return rc;
    if (n_alive)
        gather_gapped_kernel<<<(int)((n_alive + 255) / 256), 256, 0, st>>>(g.by_id, n_alive, g.vals_alt, g.keys_alt,
                                                                           g.start, g.rng, g.pts);
    HIPCHK(hipGetLastError());
    g.slots_used = used;
    g.n = n_alive;
    return 0;
}

void grid_compact_cells(GridBuf& g, const uint32_t* dlist, const uint32_t* d_ndirty, uint32_t dcap, int n_max,
                        hipStream_t st) {
    if (n_max <= 0) return;
    compact_cells_kernel<<<std::min(2048, (n_max + 3) / 4), 256, 0, st>>>(g.pts, g.rng, g.dirty, dlist, d_ndirty, dcap);
}

void grid_insert_ids(GridBuf& g, int64_t id0, const uint32_t* d_nnew, int n_max, GridInsertScratch s,
                     uint32_t* flags, hipStream_t st) {
    if (n_max <= 0) return;
    const int nb = (n_max + 255) / 256;
    (void)hipMemsetAsync(s.d_ntouch, 0, sizeof(uint32_t), st);
    insert_rank_kernel<<<nb, 256, 0, st>>>(g.by_id, id0, d_nnew, g.geom, g.addc, s.tmp_cell, s.tmp_rank, s.tlist,
                                           s.d_ntouch, flags);
    grid_insert_finish(g, id0, d_nnew, n_max, s, flags, st);
}

void grid_insert_finish(GridBuf& g, int64_t id0, const uint32_t* d_nnew, int n_max, GridInsertScratch s,
                        uint32_t* flags, hipStream_t st) {
    if (n_max <= 0) return;
    const int nb = (n_max + 255) / 256;
    const int64_t usable = g.slots_extra > 0 ? std::min<int64_t>(g.slots_cap, g.slots_used + g.slots_extra) : g.slots_cap;
    insert_alloc_kernel<<<nb, 256, 0, st>>>(g.pts, g.rng, g.lim, g.addc, s.tlist, s.d_ntouch, g.bump,
                                            (uint32_t)std::min<int64_t>(usable, 0xffffffffll), flags);
    insert_write_kernel<<<nb, 256, 0, st>>>(g.by_id, id0, d_nnew, s.tmp_cell, s.tmp_rank, g.addc, g.pts);
    insert_clear_kernel<<<nb, 256, 0, st>>>(g.addc, s.tlist, s.d_ntouch);
}

}  // namespace lio
