// lio_grid.hip — dense uniform grid build on gfx950 (the ikd-Tree Build [U]
// replacement): AABB reduction -> linear cell keys -> radix sort (key, id)
// -> cell histogram + exclusive scan -> float4 gather (sorted + id order).
// Layout rationale: the kNN reads a query's neighbour cells as short runs of
// contiguous 16-B points; x is the fastest grid axis so a 3-cell row is one
// contiguous run of the sorted array and one or two cache lines of start[].
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstdio>

#include "lio_kernels.hpp"

namespace lio {

__global__ void aabb_partial_kernel(const float* __restrict__ xyz, int64_t n, float* __restrict__ part) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            float v = xyz[3 * i + d];
            lo[d] = fminf(lo[d], v);
            hi[d] = fmaxf(hi[d], v);
        }
    }
    __shared__ float s[6][256];
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
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
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

__global__ void cell_key_kernel(const float* __restrict__ xyz, int64_t n, GridGeom g, uint32_t* __restrict__ keys,
                                uint32_t* __restrict__ vals, uint32_t* __restrict__ counts) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float inv = 1.0f / g.cell;
    int cx = cell_coord(xyz[3 * i], g.ox, inv);
    int cy = cell_coord(xyz[3 * i + 1], g.oy, inv);
    int cz = cell_coord(xyz[3 * i + 2], g.oz, inv);
    cx = min(max(cx, 0), g.nx - 1);
    cy = min(max(cy, 0), g.ny - 1);
    cz = min(max(cz, 0), g.nz - 1);
    const uint32_t k = ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx;
    keys[i] = k;
    vals[i] = (uint32_t)i;
    atomicAdd(&counts[k], 1u);
}

__global__ void gather_kernel(const float* __restrict__ xyz, int64_t n, const uint32_t* __restrict__ sorted_ids,
                              float4* __restrict__ pts, float4* __restrict__ by_id) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t id = sorted_ids[j];
    pts[j] = make_float4(xyz[3 * (size_t)id], xyz[3 * (size_t)id + 1], xyz[3 * (size_t)id + 2], __int_as_float((int)id));
    by_id[j] = make_float4(xyz[3 * j], xyz[3 * j + 1], xyz[3 * j + 2], __int_as_float((int)j));
}

#define HIPCHK(x)                                                               \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "lio_grid: %s -> %s\n", #x, hipGetErrorString(e_)); \
            return -2;                                                          \
        }                                                                       \
    } while (0)

static int ensure(void** p, size_t& cap_bytes, size_t need) {
    if (need <= cap_bytes && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    if (hipMalloc(p, need) != hipSuccess) {
        cap_bytes = 0;
        return -5;
    }
    cap_bytes = need;
    return 0;
}

void grid_free(GridBuf& g) {
    void* ptrs[] = {g.pts, g.by_id, g.start, g.keys, g.keys_alt, g.vals, g.vals_alt, g.tmp, g.aabb, g.xyz};
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

int grid_build(GridBuf& g, const float* d_xyz, int64_t n, float cell, hipStream_t st) {
    if (n <= 0 || n >= (int64_t)0x7fffffff) return -1;
    if (!(cell > 0.f)) cell = 1.0f;
    // ---- buffers sized by n
    if (n > g.cap) {
        int64_t cap = std::max<int64_t>(n, g.cap + g.cap / 2);
        void* bufs[] = {g.pts, g.by_id, g.keys, g.keys_alt, g.vals, g.vals_alt};
        for (void* p : bufs)
            if (p) HIPCHK(hipFree(p));
        HIPCHK(hipMalloc(&g.pts, cap * sizeof(float4)));
        HIPCHK(hipMalloc(&g.by_id, cap * sizeof(float4)));
        HIPCHK(hipMalloc(&g.keys, cap * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&g.keys_alt, cap * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&g.vals, cap * sizeof(uint32_t)));
        HIPCHK(hipMalloc(&g.vals_alt, cap * sizeof(uint32_t)));
        g.cap = cap;
    }
    if (!g.aabb) HIPCHK(hipMalloc(&g.aabb, 6 * 1024 * sizeof(float) + 64));
    if (!g.aabb_host) HIPCHK(hipHostMalloc(&g.aabb_host, 64));
    // ---- AABB
    const int nbA = (int)std::min<int64_t>(1024, (n + 255) / 256);
    float* part = g.aabb + 8;
    aabb_partial_kernel<<<nbA, 256, 0, st>>>(d_xyz, n, part);
    aabb_final_kernel<<<1, 256, 0, st>>>(part, nbA, g.aabb);
    HIPCHK(hipMemcpyAsync(g.aabb_host, g.aabb, 6 * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const float* bb = g.aabb_host;
    for (int d = 0; d < 6; ++d)
        if (!std::isfinite(bb[d])) return -1;
    // ---- geometry: 1-cell pad on every side; grow the cell if the table would exceed 2^29 cells
    GridGeom geo;
    for (;;) {
        double o[3], ext[3];
        for (int d = 0; d < 3; ++d) {
            o[d] = std::floor((double)bb[d] / cell) * cell - cell;
            ext[d] = (double)bb[3 + d] - o[d];
        }
        double nx = std::floor(ext[0] / cell) + 2, ny = std::floor(ext[1] / cell) + 2, nz = std::floor(ext[2] / cell) + 2;
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
    g.geom = geo;
    g.n = n;
    // ---- cell table (+ histogram scratch after it)
    const uint32_t nc1 = geo.ncells + 1;
    if (nc1 > g.cells_cap || !g.start) {
        if (g.start) HIPCHK(hipFree(g.start));
        uint32_t cap = std::max<uint32_t>(nc1, g.cells_cap + g.cells_cap / 2);
        HIPCHK(hipMalloc(&g.start, 2 * (size_t)cap * sizeof(uint32_t)));
        g.cells_cap = cap;
    }
    uint32_t* counts = g.start + g.cells_cap;
    HIPCHK(hipMemsetAsync(counts, 0, (size_t)nc1 * sizeof(uint32_t), st));
    const int nb = (int)((n + 255) / 256);
    cell_key_kernel<<<nb, 256, 0, st>>>(d_xyz, n, geo, g.keys, g.vals, counts);
    // ---- sort (key, id): stable, so ids ascend inside a cell
    int bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)geo.ncells) ++bits;
    size_t sort_bytes = 0, scan_bytes = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, g.keys, g.keys_alt, g.vals, g.vals_alt, (int)n, 0,
                                              bits, st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, counts, g.start, (int)nc1, st));
    size_t need = std::max(sort_bytes, scan_bytes);
    if (ensure(&g.tmp, g.tmp_bytes, need) != 0) return -5;
    size_t tb = g.tmp_bytes;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(g.tmp, tb, g.keys, g.keys_alt, g.vals, g.vals_alt, (int)n, 0, bits, st));
    tb = g.tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(g.tmp, tb, counts, g.start, (int)nc1, st));
    gather_kernel<<<nb, 256, 0, st>>>(d_xyz, n, g.vals_alt, g.pts, g.by_id);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // namespace lio
