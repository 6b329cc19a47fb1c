// lio_dev.hpp — device-side primitives shared by the gfx950 kernels.
//
//   * GridDev: the map / ICP target as a dense uniform grid in HBM
//       pts[]   float4 (x, y, z, id-bits) sorted by linear cell index, id order
//               inside a cell (16-B aligned: one global_load_dwordx4 per point)
//       start[] u32 cell offsets, ncells+1 (count = start[c+1]-start[c])
//   * grid_knn<K>: exact K nearest neighbours under the total order (d2, id),
//     d2 = float ((dx*dx + dy*dy) + dz*dz) (ikd-Tree calc_dist [U]), restricted
//     to d2 <= bound.  Cells are visited shell by shell (Chebyshev rings around
//     the query's cell), each cell/row pruned by its box distance against the
//     current K-th best, and the walk stops once the K-th best lies inside the
//     radius the finished shells guarantee.
//   * esti_plane_dev: FAST-LIO esti_plane<float> [U] — Eigen ColPivHouseholderQR
//     restated in registers, same float operation order as the oracle.
//
// Compiled with -ffp-contract=off: no FMA contraction, so float/double results
// are bit-identical to the CPU restatement wherever the operation order is.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lio {

constexpr int kNone = 0x7fffffff;

struct GridDev {
    const float4* pts;      // sorted by cell
    const uint32_t* start;  // ncells + 1
    float ox, oy, oz;       // grid origin (min corner)
    float cell, inv_cell;
    float margin;           // conservative slack for cell assignment rounding
    int nx, ny, nz;
};

struct PoseArg {  // lio_pose
    double R[9];
    double t[3];
    double RLI[9];
    double tLI[3];
};

__device__ __forceinline__ float sqdist3(float ax, float ay, float az, float bx, float by, float bz) {
    float dx = ax - bx;
    float dy = ay - by;
    float dz = az - bz;
    return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ bool lexless(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}

// world = R*(R_LI*p + t_LI) + t in double, stored as float  (h_share_model [U])
__device__ __forceinline__ void body_to_world(const PoseArg& ps, float bx, float by, float bz, float& wx,
                                              float& wy, float& wz) {
    double b0 = bx, b1 = by, b2 = bz;
    double p0 = ((ps.RLI[0] * b0 + ps.RLI[1] * b1) + ps.RLI[2] * b2) + ps.tLI[0];
    double p1 = ((ps.RLI[3] * b0 + ps.RLI[4] * b1) + ps.RLI[5] * b2) + ps.tLI[1];
    double p2 = ((ps.RLI[6] * b0 + ps.RLI[7] * b1) + ps.RLI[8] * b2) + ps.tLI[2];
    wx = (float)(((ps.R[0] * p0 + ps.R[1] * p1) + ps.R[2] * p2) + ps.t[0]);
    wy = (float)(((ps.R[3] * p0 + ps.R[4] * p1) + ps.R[5] * p2) + ps.t[1]);
    wz = (float)(((ps.R[6] * p0 + ps.R[7] * p1) + ps.R[8] * p2) + ps.t[2]);
}

// Sorted top-K list in registers.  Unfilled slots hold (bound, kNone) so the
// acceptance test `lexless(d, id, d[K-1], id[K-1])` is exactly "d2 <= bound".
template <int K>
struct TopK {
    float d[K];
    int id[K];
    __device__ __forceinline__ void init(float bound) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            d[j] = bound;
            id[j] = kNone;
        }
    }
    __device__ __forceinline__ void push(float dc, int ic) {
        if (!lexless(dc, ic, d[K - 1], id[K - 1])) return;
        d[K - 1] = dc;
        id[K - 1] = ic;
#pragma unroll
        for (int j = K - 1; j > 0; --j) {
            if (lexless(d[j], id[j], d[j - 1], id[j - 1])) {
                float td = d[j];
                d[j] = d[j - 1];
                d[j - 1] = td;
                int ti = id[j];
                id[j] = id[j - 1];
                id[j - 1] = ti;
            }
        }
    }
    __device__ __forceinline__ float worst() const { return d[K - 1]; }
};

__device__ __forceinline__ int cell_coord(float v, float o, float inv) {
    float f = floorf((v - o) * inv);
    f = fminf(fmaxf(f, -1.0e9f), 1.0e9f);
    return (int)f;
}

// squared distance from q to the closed interval [lo, hi] on one axis
__device__ __forceinline__ float axis_gap(float q, float lo, float hi) {
    float g = fmaxf(fmaxf(lo - q, q - hi), 0.f);
    return g * g;
}

// Scan the points of one cell into the top-K list.
template <int K>
__device__ __forceinline__ void scan_cell(const GridDev& g, uint32_t c, float qx, float qy, float qz,
                                          TopK<K>& tk) {
    uint32_t b = g.start[c];
    uint32_t e = g.start[c + 1];
    for (uint32_t j = b; j < e; ++j) {
        float4 p = g.pts[j];
        float d = sqdist3(qx, qy, qz, p.x, p.y, p.z);
        tk.push(d, __float_as_int(p.w));
    }
}

// Exact bounded K-NN.  Shells 0..max_shell around the query's cell (clipped to
// the grid).  Returns true when the list is provably final: the K-th best lies
// inside the radius the visited shells guarantee, or the whole grid was
// visited.  false => cells beyond max_shell could still hold a better point.
// Shell walk from shell s_first on (own = distance from q to its own cell's
// faces, shrunk by the margin).
template <int K>
__device__ bool grid_knn_from(const GridDev& g, float qx, float qy, float qz, int cx, int cy, int cz, float own,
                              int s_first, int max_shell, TopK<K>& tk) {
    // first shell that can touch the grid at all
    int s0 = s_first;
    s0 = max(s0, max(-cx, cx - (g.nx - 1)));
    s0 = max(s0, max(-cy, cy - (g.ny - 1)));
    s0 = max(s0, max(-cz, cz - (g.nz - 1)));
    int smax_grid = max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
    const int smax = min(max_shell, smax_grid);
    const float cs = g.cell, m = g.margin;
    int s = s0;
    for (; s <= smax; ++s) {
        const int z0 = max(cz - s, 0), z1 = min(cz + s, g.nz - 1);
        const int y0 = max(cy - s, 0), y1 = min(cy + s, g.ny - 1);
        const int x0 = max(cx - s, 0), x1 = min(cx + s, g.nx - 1);
        for (int z = z0; z <= z1; ++z) {
            const float zl = g.oz + (float)z * cs - m;
            const float gz = axis_gap(qz, zl, zl + cs + 2.f * m);
            if (gz * 0.999999f > tk.worst()) continue;
            const bool zb = (z == cz - s) || (z == cz + s);
            for (int y = y0; y <= y1; ++y) {
                const float yl = g.oy + (float)y * cs - m;
                const float gyz = gz + axis_gap(qy, yl, yl + cs + 2.f * m);
                if (gyz * 0.999999f > tk.worst()) continue;
                const bool full = zb || (y == cy - s) || (y == cy + s);
                const uint32_t rowbase = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx;
                if (full) {
                    for (int x = x0; x <= x1; ++x) {
                        const float xl = g.ox + (float)x * cs - m;
                        const float bd = gyz + axis_gap(qx, xl, xl + cs + 2.f * m);
                        if (bd * 0.999999f > tk.worst()) continue;
                        scan_cell<K>(g, rowbase + (uint32_t)x, qx, qy, qz, tk);
                    }
                } else {
#pragma unroll
                    for (int side = 0; side < 2; ++side) {
                        const int x = side ? cx + s : cx - s;
                        if (x < x0 || x > x1) continue;
                        const float xl = g.ox + (float)x * cs - m;
                        const float bd = gyz + axis_gap(qx, xl, xl + cs + 2.f * m);
                        if (bd * 0.999999f > tk.worst()) continue;
                        scan_cell<K>(g, rowbase + (uint32_t)x, qx, qy, qz, tk);
                    }
                }
            }
        }
        // every unvisited cell is farther than the radius the shells <= s guarantee
        const float gr = own + (float)s * cs;
        if (gr > 0.f && tk.worst() < gr * gr * 0.999999f) return true;
    }
    return smax == smax_grid;
}

template <int K>
__device__ bool grid_knn_exact(const GridDev& g, float qx, float qy, float qz, int max_shell, TopK<K>& tk) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    // distance from q to the faces of its own cell (shrunk by the margin)
    const float lox = g.ox + (float)cx * g.cell, loy = g.oy + (float)cy * g.cell, loz = g.oz + (float)cz * g.cell;
    float own = fminf(fminf(qx - lox, lox + g.cell - qx), fminf(qy - loy, loy + g.cell - qy));
    own = fminf(own, fminf(qz - loz, loz + g.cell - qz)) - g.margin;
    return grid_knn_from<K>(g, qx, qy, qz, cx, cy, cz, own, 0, max_shell, tk);
}

// ----------------------------------------------------------------------------
// Cooperative variant: G consecutive lanes (an aligned group inside the wave)
// search for ONE query.  Control flow is uniform inside the group; each cell's
// points are split lane-strided (one coalesced G*16-B load per step), every
// lane keeps a private top-K, the pruning bound is the group minimum of the
// private K-th bests (>= the group's true K-th best, so pruning stays exact),
// and a butterfly merge leaves the exact group top-K in every lane.
// ----------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ float group_min(float v) {
#pragma unroll
    for (int off = 1; off < G; off <<= 1) v = fminf(v, __shfl_xor(v, off, 64));
    return v;
}

template <int K, int G>
__device__ __forceinline__ void group_merge(TopK<K>& tk) {
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
        float od[K];
        int oi[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            od[j] = __shfl_xor(tk.d[j], off, 64);
            oi[j] = __shfl_xor(tk.id[j], off, 64);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) tk.push(od[j], oi[j]);
    }
}

template <int K, int G>
__device__ __forceinline__ void scan_cell_group(const GridDev& g, uint32_t c, float qx, float qy, float qz, int sub,
                                                TopK<K>& tk) {
    const uint32_t b = g.start[c];
    const uint32_t e = g.start[c + 1];
    for (uint32_t j = b + (uint32_t)sub; j < e; j += G) {
        const float4 p = g.pts[j];
        tk.push(sqdist3(qx, qy, qz, p.x, p.y, p.z), __float_as_int(p.w));
    }
}

// Returns true when the merged list is provably final (see grid_knn_exact).
template <int K, int G>
__device__ bool group_knn_exact(const GridDev& g, float qx, float qy, float qz, int max_shell, int sub,
                                TopK<K>& tk) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    const float lox = g.ox + (float)cx * g.cell, loy = g.oy + (float)cy * g.cell, loz = g.oz + (float)cz * g.cell;
    float own = fminf(fminf(qx - lox, lox + g.cell - qx), fminf(qy - loy, loy + g.cell - qy));
    own = fminf(own, fminf(qz - loz, loz + g.cell - qz)) - g.margin;
    int s0 = 0;
    s0 = max(s0, max(-cx, cx - (g.nx - 1)));
    s0 = max(s0, max(-cy, cy - (g.ny - 1)));
    s0 = max(s0, max(-cz, cz - (g.nz - 1)));
    const int smax_grid = max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
    const int smax = min(max_shell, smax_grid);
    const float cs = g.cell, m = g.margin;
    float bound = group_min<G>(tk.worst());  // group-uniform pruning bound
    bool done = false;
    for (int s = s0; s <= smax && !done; ++s) {
        if (s > s0 && sub != 0) {
            // after the merge every lane holds the group list; keep it in lane 0
            // only and re-seed the others with its K-th entry as filler: fillers
            // are never re-inserted (push rejects equal keys), so the next merge
            // sees each candidate once, and every lane prunes with the tight bound
#pragma unroll
            for (int j = 0; j < K - 1; ++j) {
                tk.d[j] = tk.d[K - 1];
                tk.id[j] = tk.id[K - 1];
            }
        }
        const int z0 = max(cz - s, 0), z1 = min(cz + s, g.nz - 1);
        const int y0 = max(cy - s, 0), y1 = min(cy + s, g.ny - 1);
        const int x0 = max(cx - s, 0), x1 = min(cx + s, g.nx - 1);
        for (int z = z0; z <= z1; ++z) {
            const float zl = g.oz + (float)z * cs - m;
            const float gz = axis_gap(qz, zl, zl + cs + 2.f * m);
            if (gz * 0.999999f > bound) continue;
            const bool zb = (z == cz - s) || (z == cz + s);
            for (int y = y0; y <= y1; ++y) {
                const float yl = g.oy + (float)y * cs - m;
                const float gyz = gz + axis_gap(qy, yl, yl + cs + 2.f * m);
                if (gyz * 0.999999f > bound) continue;
                const bool full = zb || (y == cy - s) || (y == cy + s);
                const uint32_t rowbase = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx;
                const int step = full ? 1 : 2 * s;
                for (int x = full ? x0 : cx - s; x <= (full ? x1 : cx + s); x += (step > 0 ? step : 1)) {
                    if (x < x0 || x > x1) continue;
                    const float xl = g.ox + (float)x * cs - m;
                    const float bd = gyz + axis_gap(qx, xl, xl + cs + 2.f * m);
                    if (bd * 0.999999f > bound) continue;
                    scan_cell_group<K, G>(g, rowbase + (uint32_t)x, qx, qy, qz, sub, tk);
                    bound = group_min<G>(tk.worst());
                }
            }
        }
        group_merge<K, G>(tk);  // every lane now holds the exact top-K so far
        bound = tk.worst();
        const float gr = own + (float)s * cs;
        if (gr > 0.f && bound < gr * gr * 0.999999f) done = true;
    }
    return done || smax == smax_grid;
}

// Scan one cell sequentially, four independent point loads in flight.
template <int K>
__device__ __forceinline__ void scan_cell_seq(const GridDev& g, uint32_t c, float qx, float qy, float qz,
                                              TopK<K>& tk) {
    const uint32_t b = g.start[c];
    const uint32_t e = g.start[c + 1];
    uint32_t j = b;
    for (; j + 4 <= e; j += 4) {
        const float4 p0 = g.pts[j], p1 = g.pts[j + 1], p2 = g.pts[j + 2], p3 = g.pts[j + 3];
        tk.push(sqdist3(qx, qy, qz, p0.x, p0.y, p0.z), __float_as_int(p0.w));
        tk.push(sqdist3(qx, qy, qz, p1.x, p1.y, p1.z), __float_as_int(p1.w));
        tk.push(sqdist3(qx, qy, qz, p2.x, p2.y, p2.z), __float_as_int(p2.w));
        tk.push(sqdist3(qx, qy, qz, p3.x, p3.y, p3.z), __float_as_int(p3.w));
    }
    for (; j < e; ++j) {
        const float4 p = g.pts[j];
        tk.push(sqdist3(qx, qy, qz, p.x, p.y, p.z), __float_as_int(p.w));
    }
}

// Scan up to 4 cells (cl[u] == 0xffffffff: unused) as ONE concatenated range:
// the 8 start[] loads issue together, then 8 point loads at a time, so a lane
// pays ~2 dependent memory round trips instead of 2 per cell plus 1 per point.
template <int K>
__device__ __forceinline__ void scan_cells_flat4(const GridDev& g, const uint32_t cl[4], float qx, float qy, float qz,
                                                 TopK<K>& tk) {
    uint32_t b[4], n[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const bool ok = cl[u] != 0xffffffffu;
        const uint32_t c = ok ? cl[u] : 0u;
        const uint32_t s0 = g.start[c], s1 = g.start[c + 1];
        b[u] = s0;
        n[u] = ok ? s1 - s0 : 0u;
    }
    const uint32_t p1 = n[0], p2 = p1 + n[1], p3 = p2 + n[2], tot = p3 + n[3];
    for (uint32_t t = 0; t < tot; t += 8) {
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t tt = t + (uint32_t)u;
            const uint32_t addr = tt < p1 ? b[0] + tt : (tt < p2 ? b[1] + (tt - p1) : (tt < p3 ? b[2] + (tt - p2) : b[3] + (tt - p3)));
            pp[u] = tt < tot ? g.pts[addr] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (t + (uint32_t)u < tot) tk.push(sqdist3(qx, qy, qz, pp[u].x, pp[u].y, pp[u].z), __float_as_int(pp[u].w));
    }
}

// Lane-strided scan of one cell by the whole group, 4 loads per lane in flight.
template <int K, int G>
__device__ __forceinline__ void scan_cell_group4(const GridDev& g, uint32_t c, float qx, float qy, float qz, int sub,
                                                 TopK<K>& tk) {
    const uint32_t b = g.start[c];
    const uint32_t e = g.start[c + 1];
    for (uint32_t j = b + (uint32_t)sub; j < e; j += 4 * G) {
        float4 pp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t jj = j + (uint32_t)(u * G);
            pp[u] = jj < e ? g.pts[jj] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (j + (uint32_t)(u * G) < e) tk.push(sqdist3(qx, qy, qz, pp[u].x, pp[u].y, pp[u].z), __float_as_int(pp[u].w));
    }
}

// k-th cell (0 <= k < 24 s^2 + 2) of the Chebyshev shell s >= 1: the two z
// faces, then the two y faces of the inner z slices, then the two x cells of
// every inner (z, y) row.
__device__ __forceinline__ void shell_offset(int s, int k, int& dx, int& dy, int& dz) {
    const int w = 2 * s + 1, w2 = w * w, wm = 2 * s - 1;
    const int nzf = 2 * w2, nyf = 2 * wm * w;
    if (k < nzf) {
        const int f = k >= w2;
        const int r = k - f * w2;
        const int ry = r / w;
        dz = f ? s : -s;
        dy = ry - s;
        dx = r - ry * w - s;
    } else if (k < nzf + nyf) {
        const int kk = k - nzf;
        const int zi = kk / (2 * w);
        const int r = kk - zi * 2 * w;
        dz = zi - (s - 1);
        dy = r >= w ? s : -s;
        dx = (r >= w ? r - w : r) - s;
    } else {
        const int kk = k - nzf - nyf;
        const int idx = kk >> 1;
        const int zi = idx / wm;
        dz = zi - (s - 1);
        dy = idx - zi * wm - (s - 1);
        dx = (kk & 1) ? s : -s;
    }
}

// Split variant for short searches (front-end kNN, ICP near pass): shell 0
// (the query's own cell) is scanned lane-strided by the whole group; for every
// later shell the G lanes take disjoint subsets of the shell's cells, each
// lane pruning and scanning its own cells (so the per-query cell enumeration
// is not replicated G times).  Lists are merged after every shell, which keeps
// the pruning bound exact and group-uniform.  Same result contract as
// grid_knn_exact.
struct SearchStats {  // diagnostics (lio_ctx_knn_stats), per lane
    int cells, points, shell;
};

template <int K, int G>
__device__ bool group_knn_split(const GridDev& g, float qx, float qy, float qz, int max_shell, int sub,
                                TopK<K>& tk, SearchStats* dbg = nullptr) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    const float lox = g.ox + (float)cx * g.cell, loy = g.oy + (float)cy * g.cell, loz = g.oz + (float)cz * g.cell;
    float own = fminf(fminf(qx - lox, lox + g.cell - qx), fminf(qy - loy, loy + g.cell - qy));
    own = fminf(own, fminf(qz - loz, loz + g.cell - qz)) - g.margin;
    int s0 = 0;
    s0 = max(s0, max(-cx, cx - (g.nx - 1)));
    s0 = max(s0, max(-cy, cy - (g.ny - 1)));
    s0 = max(s0, max(-cz, cz - (g.nz - 1)));
    const int smax_grid = max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
    const int smax = min(max_shell, smax_grid);
    const float cs = g.cell, m = g.margin;
    float bound = group_min<G>(tk.worst());
    bool done = false;
    for (int s = s0; s <= smax && !done; ++s) {
        if (s > s0 && sub != 0) {  // re-seed non-leader lanes (see group_knn_exact)
#pragma unroll
            for (int j = 0; j < K - 1; ++j) {
                tk.d[j] = tk.d[K - 1];
                tk.id[j] = tk.id[K - 1];
            }
        }
        if (dbg) dbg->shell = s;
        if (s == 0) {
            const uint32_t c0 = ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx;
            if (dbg && sub == 0) {
                dbg->cells += 1;
                dbg->points += (int)(g.start[c0 + 1] - g.start[c0]);
            }
            scan_cell_group4<K, G>(g, c0, qx, qy, qz, sub, tk);
        } else {
            const int ncell = 24 * s * s + 2;
            for (int k0 = sub; k0 < ncell; k0 += 4 * G) {  // chunks of 4 cells per lane
                uint32_t cl[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    cl[u] = 0xffffffffu;
                    const int k = k0 + u * G;
                    if (k >= ncell) continue;
                    int dx, dy, dz;
                    shell_offset(s, k, dx, dy, dz);
                    const int x = cx + dx, y = cy + dy, z = cz + dz;
                    if ((unsigned)x >= (unsigned)g.nx || (unsigned)y >= (unsigned)g.ny || (unsigned)z >= (unsigned)g.nz)
                        continue;
                    const float xl = g.ox + (float)x * cs - m, yl = g.oy + (float)y * cs - m,
                                zl = g.oz + (float)z * cs - m;
                    const float bd = axis_gap(qx, xl, xl + cs + 2.f * m) + axis_gap(qy, yl, yl + cs + 2.f * m) +
                                     axis_gap(qz, zl, zl + cs + 2.f * m);
                    if (bd * 0.999999f > fminf(bound, tk.worst())) continue;
                    cl[u] = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x;
                    if (dbg) {
                        dbg->cells += 1;
                        dbg->points += (int)(g.start[cl[u] + 1] - g.start[cl[u]]);
                    }
                }
                scan_cells_flat4<K>(g, cl, qx, qy, qz, tk);
            }
        }
        group_merge<K, G>(tk);
        bound = tk.worst();
        const float gr = own + (float)s * cs;
        if (gr > 0.f && bound < gr * gr * 0.999999f) done = true;
    }
    return done || smax == smax_grid;
}

// ----------------------------------------------------------------------------
// One lane = one query, built for memory-level parallelism rather than for
// lanes cooperating on a query:
//   1. own cell: one start[] pair, then its points 8 loads at a time;
//   2. the 26 neighbours as 9 x-rows (dy, dz in {-1,0,1}): rows and their end
//      cells are pruned against the own-cell bound WITHOUT memory access, the
//      start[] values of all surviving rows are loaded in one batch, and the
//      surviving row ranges (each contiguous in the cell-sorted point array;
//      the centre row splits around the own cell => <= 10 ranges) are scanned
//      as ONE flat stream, software pipelined: batch t+1's 8 loads are in
//      flight while batch t is pushed;
//   3. only if the radius guaranteed by shells 0-1 does not cover the K-th
//      best (sparse maps) the generic shell walk continues from shell 2.
// Exactness contract identical to grid_knn_exact.
// ----------------------------------------------------------------------------
constexpr int kFlatRanges = 10;

template <int K>
__device__ __forceinline__ void flat_stream_scan(const GridDev& g, const uint32_t (&b)[kFlatRanges],
                                                 const uint32_t (&n)[kFlatRanges], float qx, float qy, float qz,
                                                 TopK<K>& tk) {
    uint32_t P[kFlatRanges];  // exclusive prefix of range lengths
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kFlatRanges; ++k) {
        P[k] = tot;
        tot += n[k];
    }
    auto addr_of = [&](uint32_t tt) {
        uint32_t a = b[0] + tt;
#pragma unroll
        for (int k = 1; k < kFlatRanges; ++k)
            if (n[k] != 0u && tt >= P[k]) a = b[k] + (tt - P[k]);
        return a;
    };
    float4 cur[8], nxt[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) cur[u] = (uint32_t)u < tot ? g.pts[addr_of((uint32_t)u)] : make_float4(0, 0, 0, 0);
    for (uint32_t t = 0; t < tot; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t tt = t + 8u + (uint32_t)u;
            nxt[u] = tt < tot ? g.pts[addr_of(tt)] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (t + (uint32_t)u < tot) tk.push(sqdist3(qx, qy, qz, cur[u].x, cur[u].y, cur[u].z), __float_as_int(cur[u].w));
#pragma unroll
        for (int u = 0; u < 8; ++u) cur[u] = nxt[u];
    }
}

template <int K>
__device__ bool lane_knn_exact(const GridDev& g, float qx, float qy, float qz, int max_shell, TopK<K>& tk) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    const bool inside = (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny && (unsigned)cz < (unsigned)g.nz;
    if (!inside || max_shell < 1) return grid_knn_exact<K>(g, qx, qy, qz, max_shell, tk);
    const float cs = g.cell, m = g.margin;
    const float lox = g.ox + (float)cx * cs, loy = g.oy + (float)cy * cs, loz = g.oz + (float)cz * cs;
    float own = fminf(fminf(qx - lox, lox + cs - qx), fminf(qy - loy, loy + cs - qy));
    own = fminf(own, fminf(qz - loz, loz + cs - qz)) - m;
    const uint32_t nx = (uint32_t)g.nx, ny = (uint32_t)g.ny;
    // ---- shell 0
    {
        uint32_t b[kFlatRanges], n[kFlatRanges];
        const uint32_t c0 = ((uint32_t)cz * ny + (uint32_t)cy) * nx + (uint32_t)cx;
        b[0] = g.start[c0];
        n[0] = g.start[c0 + 1] - b[0];
#pragma unroll
        for (int k = 1; k < kFlatRanges; ++k) b[k] = n[k] = 0u;
        flat_stream_scan<K>(g, b, n, qx, qy, qz, tk);
    }
    if (own > 0.f && tk.worst() < own * own * 0.999999f) return true;
    // ---- shell 1 as 9 x-rows; per-axis gaps of the neighbour slabs
    const float gxl = axis_gap(qx, lox - cs - m, lox + m), gxh = axis_gap(qx, lox + cs - m, lox + 2.f * cs + m);
    float gyv[3], gzv[3];
    gyv[0] = axis_gap(qy, loy - cs - m, loy + m);
    gyv[1] = 0.f;
    gyv[2] = axis_gap(qy, loy + cs - m, loy + 2.f * cs + m);
    gzv[0] = axis_gap(qz, loz - cs - m, loz + m);
    gzv[1] = 0.f;
    gzv[2] = axis_gap(qz, loz + cs - m, loz + 2.f * cs + m);
    const float w = tk.worst();
    const bool xl_ok = cx > 0, xh_ok = cx + 1 < g.nx;
    uint32_t lo_i[kFlatRanges], hi_i[kFlatRanges];  // cell index ranges [lo, hi) to load
    int r = 0;
#pragma unroll
    for (int dz = 0; dz < 3; ++dz) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int z = cz + dz - 1, y = cy + dy - 1;
            const float gyz = gzv[dz] + gyv[dy];
            const bool row_ok = (unsigned)z < (unsigned)g.nz && (unsigned)y < (unsigned)g.ny && gyz * 0.999999f <= w;
            const uint32_t rb = ((uint32_t)max(z, 0) * ny + (uint32_t)max(y, 0)) * nx;
            const bool use_l = row_ok && xl_ok && (gyz + gxl) * 0.999999f <= w;
            const bool use_h = row_ok && xh_ok && (gyz + gxh) * 0.999999f <= w;
            if (dz == 1 && dy == 1) {  // centre row: the two side cells only
                lo_i[r] = rb + (uint32_t)cx - 1u;
                hi_i[r] = use_l ? rb + (uint32_t)cx : lo_i[r];
                ++r;
                lo_i[r] = rb + (uint32_t)cx + 1u;
                hi_i[r] = use_h ? rb + (uint32_t)cx + 2u : lo_i[r];
                ++r;
            } else {
                const bool use_c = row_ok;
                const uint32_t a = rb + (uint32_t)cx - (use_l ? 1u : 0u);
                const uint32_t e = rb + (uint32_t)cx + 1u + (use_h ? 1u : 0u);
                lo_i[r] = use_c ? a : 0u;
                hi_i[r] = use_c ? e : 0u;
                ++r;
            }
        }
    }
    uint32_t b[kFlatRanges], n[kFlatRanges];
#pragma unroll
    for (int k = 0; k < kFlatRanges; ++k) {
        const bool nz = hi_i[k] > lo_i[k];
        const uint32_t s0 = nz ? g.start[lo_i[k]] : 0u;
        const uint32_t s1 = nz ? g.start[hi_i[k]] : 0u;
        b[k] = s0;
        n[k] = s1 - s0;
    }
    flat_stream_scan<K>(g, b, n, qx, qy, qz, tk);
    const float gr = own + cs;
    if (gr > 0.f && tk.worst() < gr * gr * 0.999999f) return true;
    if (max_shell < 2) return false;
    return grid_knn_from<K>(g, qx, qy, qz, cx, cy, cz, own, 2, max_shell, tk);
}

// XCD-aware block order: the hardware deals blocks round-robin over the 8 XCDs
// (block b -> XCD b % 8, MI355X_MICROARCH.md); remap so every XCD works on one
// contiguous range of logical blocks — spatially coherent queries share that
// XCD's L2.  A bijection for any grid size; placement affects speed only.
__device__ __forceinline__ int xcd_block(int b, int nb) {
    const int q = nb >> 3, r = nb & 7;
    const int x = b & 7, slot = b >> 3;
    return x * q + min(x, r) + slot;
}

// ----------------------------------------------------------------------------
// esti_plane<float> [U] — A(5x3) n = -1 by Eigen ColPivHouseholderQR, same
// operation order as oracle/lio_oracle.cpp::esti_plane (statically indexed so
// everything stays in VGPRs).
// ----------------------------------------------------------------------------
__device__ __forceinline__ void swap_f(float& a, float& b) {
    float t = a;
    a = b;
    b = t;
}

__device__ __forceinline__ bool esti_plane_dev(const float P[5][3], float thr, float out[4]) {
    float A[3][5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        A[0][j] = P[j][0];
        A[1][j] = P[j][1];
        A[2][j] = P[j][2];
    }
    float cnU[3], cnD[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) s += A[k][i] * A[k][i];
        cnD[k] = sqrtf(s);
        cnU[k] = cnD[k];
    }
    float mx = cnU[0];
    if (cnU[1] > mx) mx = cnU[1];
    if (cnU[2] > mx) mx = cnU[2];
    const float eps = 1.1920928955078125e-07f;  // FLT_EPSILON
    const float th_help = ((mx * eps) * (mx * eps)) / 5.0f;
    const float ndt = sqrtf(eps);
    int nzp = 3;
    int tr[3];
    float hc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        int bi = k;
        float bn = cnU[k];
#pragma unroll
        for (int j = k + 1; j < 3; ++j)
            if (cnU[j] > bn) {
                bn = cnU[j];
                bi = j;
            }
        float bsq = bn * bn;
        if (nzp == 3 && bsq < th_help * (float)(5 - k)) nzp = k;
        tr[k] = bi;
#pragma unroll
        for (int j = k + 1; j < 3; ++j) {
            if (bi == j) {
#pragma unroll
                for (int i = 0; i < 5; ++i) swap_f(A[k][i], A[j][i]);
                swap_f(cnU[k], cnU[j]);
                swap_f(cnD[k], cnD[j]);
            }
        }
        float c0 = A[k][k];
        float tsq = 0.f;
#pragma unroll
        for (int i = k + 1; i < 5; ++i) tsq += A[k][i] * A[k][i];
        float beta, tau;
        if (tsq <= 1.17549435e-38f) {  // FLT_MIN
            tau = 0.f;
            beta = c0;
#pragma unroll
            for (int i = k + 1; i < 5; ++i) A[k][i] = 0.f;
        } else {
            beta = sqrtf(c0 * c0 + tsq);
            if (c0 >= 0.f) beta = -beta;
            float den = c0 - beta;
#pragma unroll
            for (int i = k + 1; i < 5; ++i) A[k][i] = A[k][i] / den;
            tau = (beta - c0) / beta;
        }
        A[k][k] = beta;
        hc[k] = tau;
        if (tau != 0.f) {
#pragma unroll
            for (int j = k + 1; j < 3; ++j) {
                float tmp = 0.f;
#pragma unroll
                for (int i = k + 1; i < 5; ++i) tmp += A[k][i] * A[j][i];
                tmp += A[j][k];
                A[j][k] -= tau * tmp;
#pragma unroll
                for (int i = k + 1; i < 5; ++i) A[j][i] -= (tau * A[k][i]) * tmp;
            }
        }
#pragma unroll
        for (int j = k + 1; j < 3; ++j) {
            if (cnU[j] != 0.f) {
                float temp = fabsf(A[j][k]) / cnU[j];
                temp = (1.f + temp) * (1.f - temp);
                temp = temp < 0.f ? 0.f : temp;
                float r = cnU[j] / cnD[j];
                float temp2 = temp * (r * r);
                if (temp2 <= ndt) {
                    float s = 0.f;
#pragma unroll
                    for (int i = k + 1; i < 5; ++i) s += A[j][i] * A[j][i];
                    cnD[j] = sqrtf(s);
                    cnU[j] = cnD[j];
                } else {
                    cnU[j] *= sqrtf(temp);
                }
            }
        }
    }
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if (nzp > 0) {
        float c[5] = {-1.f, -1.f, -1.f, -1.f, -1.f};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k < nzp && hc[k] != 0.f) {
                float tmp = 0.f;
#pragma unroll
                for (int i = k + 1; i < 5; ++i) tmp += A[k][i] * c[i];
                tmp += c[k];
                c[k] -= hc[k] * tmp;
#pragma unroll
                for (int i = k + 1; i < 5; ++i) c[i] -= (hc[k] * A[k][i]) * tmp;
            }
        }
#pragma unroll
        for (int i = 2; i >= 0; --i) {
            if (i < nzp && c[i] != 0.f) {
                c[i] /= A[i][i];
#pragma unroll
                for (int j = 0; j < i; ++j) c[j] -= c[i] * A[i][j];
            }
        }
        // column permutation from the transpositions
        int p0 = 0, p1 = 1, p2 = 2;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            int t = tr[k];
            int a = (k == 0) ? p0 : (k == 1 ? p1 : p2);
            int b = (t == 0) ? p0 : (t == 1 ? p1 : p2);
            if (k == 0) p0 = b; else if (k == 1) p1 = b; else p2 = b;
            if (t == 0) p0 = a; else if (t == 1) p1 = a; else p2 = a;
        }
        const float v0 = 0 < nzp ? c[0] : 0.f;
        const float v1 = 1 < nzp ? c[1] : 0.f;
        const float v2 = 2 < nzp ? c[2] : 0.f;
        // x[perm[i]] = v_i
        x0 = (p0 == 0) ? v0 : ((p1 == 0) ? v1 : v2);
        x1 = (p0 == 1) ? v0 : ((p1 == 1) ? v1 : v2);
        x2 = (p0 == 2) ? v0 : ((p1 == 2) ? v1 : v2);
    }
    float n = sqrtf((x0 * x0 + x1 * x1) + x2 * x2);
    out[0] = x0 / n;
    out[1] = x1 / n;
    out[2] = x2 / n;
    out[3] = (float)(1.0 / (double)n);
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        float r = ((out[0] * P[j][0] + out[1] * P[j][1]) + out[2] * P[j][2]) + out[3];
        if (fabsf(r) > thr) ok = false;
    }
    return ok;
}

// H row, extrinsic_est_en = false: J = [n, (R_LI p + t_LI) x (R^T n)]  [U]
__device__ __forceinline__ void h_row(const PoseArg& ps, float bx, float by, float bz, float na, float nb,
                                      float nc, double J[6]) {
    double b0 = bx, b1 = by, b2 = bz;
    double p0 = ((ps.RLI[0] * b0 + ps.RLI[1] * b1) + ps.RLI[2] * b2) + ps.tLI[0];
    double p1 = ((ps.RLI[3] * b0 + ps.RLI[4] * b1) + ps.RLI[5] * b2) + ps.tLI[1];
    double p2 = ((ps.RLI[6] * b0 + ps.RLI[7] * b1) + ps.RLI[8] * b2) + ps.tLI[2];
    double n0 = na, n1 = nb, n2 = nc;
    double C0 = (ps.R[0] * n0 + ps.R[3] * n1) + ps.R[6] * n2;
    double C1 = (ps.R[1] * n0 + ps.R[4] * n1) + ps.R[7] * n2;
    double C2 = (ps.R[2] * n0 + ps.R[5] * n1) + ps.R[8] * n2;
    J[0] = n0;
    J[1] = n1;
    J[2] = n2;
    J[3] = p1 * C2 - p2 * C1;
    J[4] = p2 * C0 - p0 * C2;
    J[5] = p0 * C1 - p1 * C0;
}

}  // namespace lio
