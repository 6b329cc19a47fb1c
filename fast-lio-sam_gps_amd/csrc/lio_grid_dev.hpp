// lio_grid_dev.hpp — device pieces of the gapped-grid maintenance shared by lio_grid.hip's kernels and
// the fused map-update kernel of lio_mapupd.hip (one translation unit each: no relocatable device code).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lio_kernels.hpp"

namespace lio {

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

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set lanes of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One WAVE compacts listed cell c: drop the entries marked dead (id bits kNone), keep the order (64
// entries at a time: ballot + mbcnt give each survivor its slot), clear the cell's dirty byte.
__device__ __forceinline__ void compact_cell_wave(float4* __restrict__ pts, uint2* __restrict__ rng,
                                                  uint8_t* __restrict__ dirty, uint32_t c) {
    const int lane = threadIdx.x & 63;
    const uint2 r = rng[c];
    uint32_t o = r.x;
    for (uint32_t j0 = r.x; j0 < r.y; j0 += 64u) {
        const uint32_t j = j0 + (uint32_t)lane;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < r.y) p = pts[j];
        const bool keep = j < r.y && __float_as_int(p.w) != kNone;
        const uint64_t m = __ballot(keep);
        // every lane has its entry in registers before any store: slots below j0 + 64 only
        __builtin_amdgcn_wave_barrier();
        if (keep && o + lane_rank(m) != j) pts[o + lane_rank(m)] = p;
        o += (uint32_t)__popcll(m);
    }
    if (lane == 0) {
        rng[c].y = o;
        dirty[c] = 0;
    }
}

// Insert rank of new id j (point p) in its cell: tmp_cell[j] = cell, tmp_rank[j] = rank among this
// update's points of the cell (addc[c] counts them); the first point of a cell lists it in tlist.
// Called by the whole wave (`act`: this lane has a point); the wave's newly touched cells are listed
// with one counter add (thousands of lanes adding to one counter serialise at the atomic unit).
__device__ __forceinline__ void insert_rank_point(bool act, uint32_t j, float x, float y, float z, const GridGeom& g,
                                                  uint32_t* __restrict__ addc, uint32_t* __restrict__ tmp_cell,
                                                  uint32_t* __restrict__ tmp_rank, uint32_t* __restrict__ tlist,
                                                  uint32_t* __restrict__ d_ntouch, uint32_t* __restrict__ flags) {
    uint32_t c = 0, r = 1;
    if (act) {
        int out = 0;
        c = cell_key_of(g, 1.0f / g.cell, x, y, z, &out);
        if (out) atomicOr(flags, 1u);
        r = atomicAdd(&addc[c], 1u);
        tmp_cell[j] = c;
        tmp_rank[j] = r;
    }
    const uint64_t m = __ballot(r == 0);
    if (r == 0) {
        const int leader = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(d_ntouch, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader, 64);
        tlist[base + lane_rank(m)] = c;
    }
}

// after the fused update kernel: grow the touched cells' blocks, write the new ids, clear addc
// (lio_grid.hip; d_nnew / d_ntouch live on the device)
void grid_insert_finish(GridBuf& g, int64_t id0, const uint32_t* d_nnew, int n_max, GridInsertScratch s,
                        uint32_t* flags, hipStream_t st);

}  // namespace lio
