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
template <int K>
__device__ bool grid_knn_exact(const GridDev& g, float qx, float qy, float qz, int max_shell, TopK<K>& tk) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    // distance from q to the faces of its own cell (shrunk by the margin)
    const float lox = g.ox + (float)cx * g.cell, loy = g.oy + (float)cy * g.cell, loz = g.oz + (float)cz * g.cell;
    float own = fminf(fminf(qx - lox, lox + g.cell - qx), fminf(qy - loy, loy + g.cell - qy));
    own = fminf(own, fminf(qz - loz, loz + g.cell - qz)) - g.margin;
    // first shell that can touch the grid at all
    int s0 = 0;
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
