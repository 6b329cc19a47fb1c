// lio_dev.hpp — device-side primitives shared by the gfx950 kernels.
//
//   * GridDev: the map / ICP target as a dense uniform grid in HBM
//       pts[]   float4 (x, y, z, id-bits) sorted by linear cell index, id order
//               inside a cell (16-B aligned: one global_load_dwordx4 per point)
//       start[] u32 cell offsets, ncells+1 (count = start[c+1]-start[c])
//   * exact K nearest neighbours under the total order (d2, id),
//     d2 = float ((dx*dx + dy*dy) + dz*dz) (ikd-Tree calc_dist [U]), restricted
//     to d2 <= bound.  Cells are visited shell by shell (Chebyshev rings around
//     the query's cell), each cell pruned by its box distance against the
//     current K-th best, and the walk stops once the K-th best lies inside the
//     radius the finished shells guarantee:
//       group_knn_near      8 lanes per query, shells 0-1 (the common case)
//       block_knn_box_flat  a block per query, the rest of its search box
//                           (the sparse tail, ~0.4% of a dense scan)
//       group_knn_exact     8 lanes per query, any number of shells
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
    const float4* pts;      // points grouped by cell
    const uint32_t* start;  // dense grids (ICP): ncells + 1 CSR offsets, a row of cells one contiguous range
    const uint2* rng;       // map grids: per cell its live slots [x, y) (gapped CSR: blocks with spare room)
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
    double q[4];    // state rot as MTK::SO3 = Eigen::Quaternion<double>, (w, x, y, z)
    double qLI[4];  // offset_R_L_I
};

// `Eigen::Quaternion<double> * Vector3d` as Eigen 3.3 evaluates it
// (QuaternionBase::_transformVector, Geometry/Quaternion.h):
//   uv = q.vec().cross(v); uv += uv; return v + q.w() * uv + q.vec().cross(uv);
// conj: by q.conjugate() (vec negated).  Same operation order as the oracle's quat_rotate.
__device__ __forceinline__ void quat_rotate(const double* q, bool conj, double v0, double v1, double v2,
                                            double& o0, double& o1, double& o2) {
    const double w = q[0];
    const double x = conj ? -q[1] : q[1], y = conj ? -q[2] : q[2], z = conj ? -q[3] : q[3];
    double u0 = y * v2 - z * v1;
    double u1 = z * v0 - x * v2;
    double u2 = x * v1 - y * v0;
    u0 += u0;
    u1 += u1;
    u2 += u2;
    const double c0 = y * u2 - z * u1;
    const double c1 = z * u0 - x * u2;
    const double c2 = x * u1 - y * u0;
    o0 = (v0 + w * u0) + c0;
    o1 = (v1 + w * u1) + c1;
    o2 = (v2 + w * u2) + c2;
}

__device__ __forceinline__ float sqdist3(float ax, float ay, float az, float bx, float by, float bz) {
    float dx = ax - bx;
    float dy = ay - by;
    float dz = az - bz;
    return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ bool lexless(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}

// pointBodyToWorld / h_share_model [U]: p_global = s.rot * (s.offset_R_L_I * p_body + s.offset_T_L_I)
// + s.pos in double (both SO3 products through quat_rotate), stored as float
__device__ __forceinline__ void body_to_world(const PoseArg& ps, float bx, float by, float bz, float& wx,
                                              float& wy, float& wz) {
    double a0, a1, a2, w0, w1, w2;
    quat_rotate(ps.qLI, false, bx, by, bz, a0, a1, a2);
    quat_rotate(ps.q, false, a0 + ps.tLI[0], a1 + ps.tLI[1], a2 + ps.tLI[2], w0, w1, w2);
    wx = (float)(w0 + ps.t[0]);
    wy = (float)(w1 + ps.t[1]);
    wz = (float)(w2 + ps.t[2]);
}

// Sorted top-K list in registers.  Each entry is one 64-bit key
// (float bits of d2) << 32 | id: d2 >= +0, so the float bits order like the
// values and ONE unsigned compare is the (d2, id) total order of the
// reference's tie-free kNN.  Unfilled slots hold (bound, kNone), so the
// acceptance test `key < k[K-1]` is exactly "d2 <= bound".
__device__ __forceinline__ uint64_t knn_key(float d, int id) {
    return ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)id;
}

// Keys as f64: knn_key(d2, id) with 0 <= d2 <= +inf float is the bit pattern of a positive, finite
// double (exponent <= 0x7f8) whose numeric order is the key order, so v_min_f64 / v_max_f64 order
// keys in one instruction each (instead of a 64-bit compare and two selects).  Inline asm: clang's
// fmin/fmax add sNaN canonicalisation that keys never need.  d2 = 0 gives an f64 denormal, kept by
// the default FP64 denormal mode (tested: exact zero-distance ties, tests/test_gpu_icp.py).
__device__ __forceinline__ uint64_t key_min(uint64_t a, uint64_t b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(__longlong_as_double((long long)a)), "v"(__longlong_as_double((long long)b)));
    return (uint64_t)__double_as_longlong(r);
}
__device__ __forceinline__ uint64_t key_max(uint64_t a, uint64_t b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(__longlong_as_double((long long)a)), "v"(__longlong_as_double((long long)b)));
    return (uint64_t)__double_as_longlong(r);
}

typedef float f2v __attribute__((ext_vector_type(2)));

// two candidates' squared distances with packed FP32 (v_pk_add_f32 / v_pk_mul_f32): per element
// exactly sqdist3's ((dx*dx + dy*dy) + dz*dz) (no FMA: -ffp-contract=off)
__device__ __forceinline__ void sqdist3_x2(float qx, float qy, float qz, const float4& a, const float4& b, float& da,
                                           float& db) {
    const f2v dx = f2v{qx, qx} - f2v{a.x, b.x}, dy = f2v{qy, qy} - f2v{a.y, b.y}, dz = f2v{qz, qz} - f2v{a.z, b.z};
    const f2v d = (dx * dx + dy * dy) + dz * dz;
    da = d.x;
    db = d.y;
}

// a bitonic 5-list sorted in place (5 comparators suffice for bitonic inputs, 0-1 principle)
__device__ __forceinline__ void sort_bitonic5(uint64_t (&v)[5]) {
    auto cx = [&](int i, int j) {
        const uint64_t x = v[i], y = v[j];
        v[i] = key_min(x, y);
        v[j] = key_max(x, y);
    };
    cx(0, 4);
    cx(1, 3);
    cx(1, 4);
    cx(2, 4);
    cx(3, 4);
}

template <int K>
struct TopK {
    uint64_t k[K];
    __device__ __forceinline__ void init(float bound) {
#pragma unroll
        for (int j = 0; j < K; ++j) k[j] = knn_key(bound, kNone);
    }
    __device__ __forceinline__ float d(int j) const { return __uint_as_float((uint32_t)(k[j] >> 32)); }
    __device__ __forceinline__ int id(int j) const { return (int)(uint32_t)k[j]; }
    __device__ __forceinline__ float worst() const { return d(K - 1); }
    // insertion: entry j takes k[j-1] if x sorts before it, else x if x sorts
    // before k[j] (old values throughout), one compare per slot
    // (old values throughout: k[j] <- min(k[j], max(k[j-1], x)), k[0] <- min(k[0], x) is the sorted
    // insertion of x dropping the largest; min / max as f64, no compares or selects)
    __device__ __forceinline__ void push(float dc, int ic) {
        const uint64_t x = knn_key(dc, ic);
        if (!(x < k[K - 1])) return;
#pragma unroll
        for (int j = K - 1; j > 0; --j) k[j] = key_min(k[j], key_max(k[j - 1], x));
        k[0] = key_min(k[0], x);
    }
    // two candidates at once (K = 5): order them (one comparator), keep the 5 smallest of the two
    // sorted lists — min(a[j], b[4 - j]) touches a[3], a[4] only, a bitonic sequence — and sort that
    // (5 comparators): 14 min / max instead of up to 2 x 9 for two single insertions; same list
    __device__ __forceinline__ void push2(uint64_t b0, uint64_t b1) {
        static_assert(K == 5, "push2: K = 5");
        const uint64_t lo = key_min(b0, b1);
        if (!(lo < k[K - 1])) return;
        const uint64_t hi = key_max(b0, b1);
        k[4] = key_min(k[4], lo);
        k[3] = key_min(k[3], hi);
        sort_bitonic5(k);
    }
    // every slot := the K-th entry (a filler that is never re-inserted)
    __device__ __forceinline__ void fill_with_worst() {
#pragma unroll
        for (int j = 0; j < K - 1; ++j) k[j] = k[K - 1];
    }
};

struct SearchStats {  // diagnostics (lio_ctx_knn_stats), per lane
    int cells, points, shell;
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

// ----------------------------------------------------------------------------
// Cooperative variant: G consecutive lanes (an aligned group inside the wave)
// search for ONE query.  Control flow is uniform inside the group; each cell's
// points are split lane-strided (one coalesced G*16-B load per step), every
// lane keeps a private top-K, the pruning bound is the group minimum of the
// private K-th bests (>= the group's true K-th best, so pruning stays exact),
// and a butterfly merge leaves the exact group top-K in every lane.
// ----------------------------------------------------------------------------
// Exchange with the partner lane of butterfly round `off` inside aligned
// groups of 8: DPP lane permutations on the VALU (no LDS round trip).  Round
// 1 and 2 are xor 1 / xor 2 (quad_perm); round 4 pairs lane i with 7 - i
// (row_half_mirror) — a different matching than xor 4, equally valid for
// butterfly min / merge since after rounds 1-2 all lanes of a quad agree.
// Other offsets (groups wider than 8) fall back to ds_bpermute.
template <int OFF>
__device__ __forceinline__ uint32_t partner_u32(uint32_t v) {
    if constexpr (OFF == 1) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xb1, 0xf, 0xf, false);
    else if constexpr (OFF == 2) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4e, 0xf, 0xf, false);
    else if constexpr (OFF == 4) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xf, 0xf, false);
    else return (uint32_t)__shfl_xor((int)v, OFF, 64);
}
template <int OFF>
__device__ __forceinline__ float partner_f(float v) {
    return __uint_as_float(partner_u32<OFF>(__float_as_uint(v)));
}

template <int G, int OFF = 1>
__device__ __forceinline__ float group_min(float v) {
    if constexpr (OFF >= G) {
        return v;
    } else {
        v = fminf(v, partner_f<OFF>(v));
        return group_min<G, 2 * OFF>(v);
    }
}

// Sort a bitonic (non-decreasing, then non-increasing) list in place.
template <int K>
__device__ __forceinline__ void cmpx(uint64_t (&v)[K], int i, int j) {
    const uint64_t a = v[i], b = v[j];
    v[i] = key_min(a, b);
    v[j] = key_max(a, b);
}
template <int K>
__device__ __forceinline__ void sort_bitonic(uint64_t (&v)[K]) {
    static_assert(K == 1 || K == 5, "sort_bitonic: K = 1 or 5");
    if constexpr (K == 5) {  // 5 comparators suffice for bitonic inputs (0-1 principle)
        cmpx(v, 0, 4);
        cmpx(v, 1, 3);
        cmpx(v, 1, 4);
        cmpx(v, 2, 4);
        cmpx(v, 3, 4);
    }
}

// Butterfly merge over the G lanes of a group: per round the K smallest of
// the two (disjoint) sorted lists are min(a[j], b[K-1-j]) — a bitonic
// sequence — then sorted.  Afterwards every lane holds the group's top-K.
template <int K, int G, int OFF = 1>
__device__ __forceinline__ void group_merge(TopK<K>& tk) {
    if constexpr (OFF < G) {
        uint64_t c[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t lo = partner_u32<OFF>((uint32_t)tk.k[K - 1 - j]);
            const uint32_t hi = partner_u32<OFF>((uint32_t)(tk.k[K - 1 - j] >> 32));
            const uint64_t b = ((uint64_t)hi << 32) | lo;
            c[j] = key_min(b, tk.k[j]);
        }
        sort_bitonic<K>(c);
#pragma unroll
        for (int j = 0; j < K; ++j) tk.k[j] = c[j];
        group_merge<K, G, 2 * OFF>(tk);
    }
}

template <int K, int G>
__device__ __forceinline__ void scan_cell_group(const GridDev& g, uint32_t c, float qx, float qy, float qz, int sub,
                                                TopK<K>& tk) {
    const uint2 r = g.rng[c];
    const uint32_t b = r.x, e = r.y;
    for (uint32_t j = b + (uint32_t)sub; j < e; j += G) {
        const float4 p = g.pts[j];
        tk.push(sqdist3(qx, qy, qz, p.x, p.y, p.z), __float_as_int(p.w));
    }
}

// Lane-strided scan of one cell by the group, four loads in flight per lane
// (the addresses clamped to the cell's last point; only real ones pushed).
template <int K, int G, int U = 4>
__device__ __forceinline__ void scan_cell_group2(const GridDev& g, uint32_t c, float qx, float qy, float qz, int sub,
                                                 TopK<K>& tk) {
    const uint2 r = g.rng[c];
    const uint32_t b = r.x, e = r.y;
    for (uint32_t j = b + (uint32_t)sub; j < e; j += U * G) {
        float4 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = g.pts[min(j + (uint32_t)(u * G), e - 1)];
#pragma unroll
        for (int u = 0; u < U; u += 2) {
            float d0, d1;
            sqdist3_x2(qx, qy, qz, p[u], p[u + 1], d0, d1);
            const bool in0 = j + (uint32_t)(u * G) < e, in1 = j + (uint32_t)((u + 1) * G) < e;
            if constexpr (K == 5) {  // pairwise insertion; slots past the cell: (+inf, kNone) keys
                tk.push2(knn_key(in0 ? d0 : INFINITY, in0 ? __float_as_int(p[u].w) : kNone),
                         knn_key(in1 ? d1 : INFINITY, in1 ? __float_as_int(p[u + 1].w) : kNone));
            } else {
                if (in0) tk.push(d0, __float_as_int(p[u].w));
                if (in1) tk.push(d1, __float_as_int(p[u + 1].w));
            }
        }
    }
}

// Returns true when the merged list is provably final: the K-th best lies
// inside the radius the visited shells guarantee, or the whole grid was
// visited; false => cells beyond max_shell could still hold a better point.
// s_first > 0 resumes the walk (lists may already be merged across the group:
// re-seeding is then needed before the first shell too, and is a no-op on
// lists that are identical fillers).
template <int K, int G>
__device__ bool group_knn_exact_from(const GridDev& g, float qx, float qy, float qz, int s_first, int max_shell,
                                     int sub, TopK<K>& tk) {
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    const float lox = g.ox + (float)cx * g.cell, loy = g.oy + (float)cy * g.cell, loz = g.oz + (float)cz * g.cell;
    float own = fminf(fminf(qx - lox, lox + g.cell - qx), fminf(qy - loy, loy + g.cell - qy));
    own = fminf(own, fminf(qz - loz, loz + g.cell - qz)) - g.margin;
    int s0 = s_first;
    s0 = max(s0, max(-cx, cx - (g.nx - 1)));
    s0 = max(s0, max(-cy, cy - (g.ny - 1)));
    s0 = max(s0, max(-cz, cz - (g.nz - 1)));
    const int smax_grid = max(max(max(cx, g.nx - 1 - cx), max(cy, g.ny - 1 - cy)), max(cz, g.nz - 1 - cz));
    const int smax = min(max_shell, smax_grid);
    const float cs = g.cell, m = g.margin;
    float bound = group_min<G>(tk.worst());  // group-uniform pruning bound
    bool done = false;
    for (int s = s0; s <= smax && !done; ++s) {
        if (sub != 0) {
            // after the merge every lane holds the group list; keep it in lane 0
            // only and re-seed the others with its K-th entry f as filler: push
            // accepts only keys < f, so every real candidate lives in exactly one
            // lane, copies of f can only fill the tail of a merged list (lane 0
            // holds K entries <= f), and every lane prunes with the tight bound
                tk.fill_with_worst();
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

template <int K, int G>
__device__ bool group_knn_exact(const GridDev& g, float qx, float qy, float qz, int max_shell, int sub,
                                TopK<K>& tk) {
    return group_knn_exact_from<K, G>(g, qx, qy, qz, 0, max_shell, sub, tk);
}

// Scan one cell sequentially, four independent point loads in flight.
template <int K>
__device__ __forceinline__ void scan_cell_seq(const GridDev& g, uint32_t c, float qx, float qy, float qz,
                                              TopK<K>& tk) {
    const uint2 r = g.rng[c];
    const uint32_t b = r.x, e = r.y;
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

// Shell 1 of the 3x3x3 block, load-balanced over an aligned group of G = 8
// lanes.  Lane `sub` owns cells 4*sub .. 4*sub+3 of the block (their ranges
// preloaded by shell1_ranges), drops those the (merged, group-uniform) K-th
// best rules out by box distance, a group prefix sum
// concatenates the ranges into a slot table in LDS (lds[0..32) range starts,
// lds[32..65) offsets), and the G lanes then stride the concatenated points,
// two loads in flight per lane.  The work per group is ceil(points / G)
// steps whatever the cells' sizes, instead of the largest cell of each lane.
// Shell-1 ranges of lane `sub` (cells CPL*sub .. CPL*sub+CPL-1 of the 3x3x3 block),
// loaded before the own cell is scanned so their latency overlaps it.
template <int G>
constexpr int shell1_cpl() {  // cells of the 3x3x3 block per lane
    return (27 + G - 1) / G;
}

template <int G, bool OWN = false>  // OWN: the own cell (k = 13) is a range too
__device__ __forceinline__ void shell1_ranges(const GridDev& g, int cx, int cy, int cz, int sub,
                                              uint32_t* b4, uint32_t* n4) {
    constexpr int CPL = shell1_cpl<G>();
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int k = CPL * sub + j;
        const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
        const int x = cx + dx, y = cy + dy, z = cz + dz;
        const bool ok = k < 27 && (OWN || k != 13) && (unsigned)x < (unsigned)g.nx && (unsigned)y < (unsigned)g.ny &&
                        (unsigned)z < (unsigned)g.nz;
        uint32_t b = 0, e = 0;
        if (ok) {
            const uint32_t c = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x;
            const uint2 r = g.rng[c];
            b = r.x;
            e = r.y;
        }
        b4[j] = b;
        n4[j] = e - b;
    }
}

// The pruned shell-1 ranges of a group's query, concatenated into the
// group's LDS slot table (lds[0..32) range starts, lds[32..65) offsets);
// returns NR << 24 | T: the non-empty ranges and the total point count (group-uniform).
template <int K, int G>
__device__ __forceinline__ uint32_t shell1_table(const GridDev& g, float qx, float qy, float qz, float lox, float loy,
                                                 float loz, int sub, uint32_t* lds, uint32_t* b4, uint32_t* n4,
                                                 float bound, SearchStats* dbg) {
    constexpr int CPL = shell1_cpl<G>();
    static_assert(CPL * G == 32, "shell1_table: slot table = 32 range starts + 33 offsets");
    const float cs = g.cell, m = g.margin, w = cs + 2.f * m;
    // prune the preloaded ranges against the bound; count points and non-empty ranges in one
    // packed word (ranges << 24 | points) so one group prefix sum gives both
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        const int k = CPL * sub + j;
        const int dx = k % 3 - 1, dy = (k / 3) % 3 - 1, dz = k / 9 - 1;
        const float xl = lox + (float)dx * cs - m, yl = loy + (float)dy * cs - m, zl = loz + (float)dz * cs - m;
        const float bd = (axis_gap(qx, xl, xl + w) + axis_gap(qy, yl, yl + w)) + axis_gap(qz, zl, zl + w);
        if (bd * 0.999999f > bound) n4[j] = 0;
        if (dbg && n4[j]) dbg->cells += 1;
        packed += n4[j] + (n4[j] ? (1u << 24) : 0u);
    }
    uint32_t incl = packed, tot;
    if constexpr (G == 8) {  // DPP row shifts (lanes from the neighbouring group are masked by sub >= off)
        uint32_t v = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xf, 0xf, false);  // row_shr:1
        if (sub >= 1) incl += v;
        v = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xf, 0xf, false);  // row_shr:2
        if (sub >= 2) incl += v;
        v = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xf, 0xf, false);  // row_shr:4
        if (sub >= 4) incl += v;
        uint32_t t = packed;  // group total by butterfly (integer: order-free)
        t += partner_u32<1>(t);
        t += partner_u32<2>(t);
        t += partner_u32<4>(t);
        tot = t;
    } else {
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const uint32_t v = __shfl_up(incl, off, G);
            if (sub >= off) incl += v;
        }
        tot = __shfl(incl, G - 1, G);
    }
    const uint32_t T = tot & 0xffffffu, NR = tot >> 24;
    // compacted slot table: only the non-empty ranges, so the lanes' slot walks never step
    // through pruned or empty cells (each step is a dependent LDS read)
    const uint32_t excl = incl - packed;
    uint32_t o = excl & 0xffffffu, slot = excl >> 24;
    uint32_t* s_b = lds;
    uint32_t* s_off = lds + CPL * G;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
        if (n4[j]) {
            s_b[slot] = b4[j];
            s_off[slot] = o;
            ++slot;
        }
        o += n4[j];
    }
    if (sub == G - 1) s_off[NR] = T;
    if (dbg && sub == 0) dbg->points += (int)T;
    return tot;  // NR << 24 | T
}

// Lane `r` of `L` lanes strides the concatenated table [0, T) (U loads in
// flight per lane: the slot walk first, then the loads, then the pushes) and
// pushes every point into its private list.
template <int K, int U = 4>
__device__ __forceinline__ void scan_table_strided(const GridDev& g, float qx, float qy, float qz, const uint32_t* lds,
                                                   uint32_t T, uint32_t NR, uint32_t r, uint32_t L, TopK<K>& tk) {
    (void)NR;
    const uint32_t* s_b = lds;
    const uint32_t* s_off = lds + 32;
    int sl = 0;
    uint32_t lo = 0, hi = s_off[1], sb = s_b[0];
    for (uint32_t t = r; t < T; t += U * L) {
        uint32_t src[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t tu = min(t + (uint32_t)u * L, T - 1);  // clamped: a valid address, pushed only if < T
            while (tu >= hi) {
                lo = hi;
                hi = s_off[++sl + 1];
                sb = s_b[sl];
            }
            src[u] = sb + (tu - lo);
        }
        float4 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = g.pts[src[u]];
        static_assert(U % 2 == 0, "scan_table_strided: pairs of loads");
#pragma unroll
        for (int u = 0; u < U; u += 2) {
            float d0, d1;
            sqdist3_x2(qx, qy, qz, p[u], p[u + 1], d0, d1);
            // slots past the end: (+inf, kNone) keys, never below a list entry (not NaN patterns, which
            // v_min / v_max_f64 would drop)
            const bool in0 = t + (uint32_t)u * L < T, in1 = t + (uint32_t)(u + 1) * L < T;
            tk.push2(knn_key(in0 ? d0 : INFINITY, in0 ? __float_as_int(p[u].w) : kNone),
                     knn_key(in1 ? d1 : INFINITY, in1 ? __float_as_int(p[u + 1].w) : kNone));
        }
    }
}

template <int K, int G, int U = 4>
__device__ __forceinline__ void scan_shell1_flat(const GridDev& g, float qx, float qy, float qz, int cx, int cy,
                                                 int cz, float lox, float loy, float loz, int sub, uint32_t* lds,
                                                 uint32_t* b4, uint32_t* n4, TopK<K>& tk, SearchStats* dbg) {
    (void)cx, (void)cy, (void)cz;
    const uint32_t TP = shell1_table<K, G>(g, qx, qy, qz, lox, loy, loz, sub, lds, b4, n4, tk.worst(), dbg);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    scan_table_strided<K, U>(g, qx, qy, qz, lds, TP & 0xffffffu, TP >> 24, (uint32_t)sub, (uint32_t)G, tk);
}

// Lean group walk for dense maps (front-end kNN, ICP near pass), written for
// occupancy (no per-lane arrays): the own cell lane-strided by the whole group,
// merge; then the shell-1 cells of the 3x3x3 block (ranges loaded during the
// own-cell scan) pruned against the merged K-th best, concatenated through the
// group's LDS slot table and strided by the lanes (scan_shell1_flat); merge.
// Shells >= 2 (sparse neighbourhoods) continue with the generic walk, or are
// left to the far pass when max_shell < 2.  Same result contract as
// group_knn_exact_from.  TAIL = false (front-end near pass): no generic walk
// at all — queries outside the grid or unresolved after shell 1 return false
// with their partial list and go to the far pass.
template <int K, int G, bool TAIL = true, int U = 4, int UO = 4>  // UO: loads in flight in the own-cell scan
__device__ bool group_knn_near(const GridDev& g, float qx, float qy, float qz, int cx, int cy, int cz, int max_shell,
                               int sub, TopK<K>& tk, SearchStats* dbg, uint32_t* lds) {
    const bool inside = (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny && (unsigned)cz < (unsigned)g.nz;
    if (!inside || max_shell < 1) {
        if constexpr (TAIL) return group_knn_exact_from<K, G>(g, qx, qy, qz, 0, max_shell, sub, tk);
        return false;
    }
    const float cs = g.cell, m = g.margin;
    const float lox = g.ox + (float)cx * cs, loy = g.oy + (float)cy * cs, loz = g.oz + (float)cz * cs;
    float own = fminf(fminf(qx - lox, lox + cs - qx), fminf(qy - loy, loy + cs - qy));
    own = fminf(own, fminf(qz - loz, loz + cs - qz)) - m;
    const uint32_t nx = (uint32_t)g.nx, nxy = (uint32_t)g.nx * (uint32_t)g.ny;
    const uint32_t c0 = (uint32_t)cz * nxy + (uint32_t)cy * nx + (uint32_t)cx;
    uint32_t b4[shell1_cpl<G>()], n4[shell1_cpl<G>()];
    shell1_ranges<G>(g, cx, cy, cz, sub, b4, n4);  // in flight during the own-cell scan
    scan_cell_group2<K, G, UO>(g, c0, qx, qy, qz, sub, tk);
    group_merge<K, G>(tk);
    if (dbg) dbg->shell = 0;
    if (own > 0.f && tk.worst() < own * own * 0.999999f) return true;
    if (sub != 0) {  // re-seed non-leader lanes (see group_knn_exact_from)
        tk.fill_with_worst();
    }
    scan_shell1_flat<K, G, U>(g, qx, qy, qz, cx, cy, cz, lox, loy, loz, sub, lds, b4, n4, tk, dbg);
    group_merge<K, G>(tk);
    if (dbg) dbg->shell = 1;
    const float gr = own + cs;
    if (gr > 0.f && tk.worst() < gr * gr * 0.999999f) return true;
    if (!TAIL || max_shell < 2) return false;
    if (dbg) dbg->shell = 2;
    return group_knn_exact_from<K, G>(g, qx, qy, qz, 2, max_shell, sub, tk);
}

// Near pass seeded by the query's previous kNN (the second and later kNN
// evaluations of a scan, map unchanged since): the previous 5th-neighbour
// distance d5 (at the previous world position w_old) and the query's
// displacement bound the answer by the triangle inequality — every previous
// neighbour lies within sqrt(d5) + |w - w_old| of w — so no neighbour has to be
// re-gathered.  bound = that radius squared (plus margins for float rounding and
// for w_old from a float affine map),
// capped at the gate; every lane starts with (bound, kNone) as filler (push
// keeps every key with d2 <= bound), the 27 cells of the 3x3x3 block are pruned
// against it and scanned in ONE flat pass, and one merge gives the list.  A
// list that is not full (impossible for a valid bound, kept as a guard) is
// reset to range fillers and returns -1: the far pass then searches the whole
// box, the 3x3x3 block included.  Returns 1 when final, 0 when the far pass
// must search the box outside the block (group_knn_near's false).
// The seeded pass's bound for query q (float throughout: w_old may come from a float affine map,
// ~1e-5 m off at 100 m, and every step rounds, so the radius gets an absolute + relative margin and
// the square a relative one); range_sq when the previous list was not full or q is outside the grid.
__device__ __forceinline__ float seeded_bound(bool inside, float d5prev, float wox, float woy, float woz, float qx,
                                             float qy, float qz, float range_sq, float scale) {
    float bound = range_sq;
    if (inside && d5prev <= range_sq) {  // the previous list was full
        const float dx = qx - wox, dy = qy - woy, dz = qz - woz;
        const float eps = 1e-4f + 1e-6f * ((fabsf(qx) + fabsf(qy)) + fabsf(qz));
        const float r = (sqrtf(d5prev) + sqrtf((dx * dx + dy * dy) + dz * dz)) + eps;
        const float b = r * r * (1.0f + 1e-5f);
        if (b < range_sq) bound = b * scale;  // scale: 1 (< 1 tests the guard)
    }
    return bound;
}

// (cx, cy, cz) = the query's cell, bound = seeded_bound(...): computed once per query by the caller
template <int K, int G, int U = 4>
__device__ int group_knn_seeded(const GridDev& g, float bound, int cx, int cy, int cz, float qx, float qy, float qz,
                                 float range_sq, int sub, TopK<K>& tk, uint32_t* lds) {
    static_assert(K == 5, "group_knn_seeded: K = 5");
    const bool inside = (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny && (unsigned)cz < (unsigned)g.nz;
    tk.init(bound);
    if (!inside) return 0;  // the far pass scans the whole box from range fillers
    uint32_t b4[shell1_cpl<G>()], n4[shell1_cpl<G>()];
    shell1_ranges<G, true>(g, cx, cy, cz, sub, b4, n4);
    const float cs = g.cell, m = g.margin;
    const float lox = g.ox + (float)cx * cs, loy = g.oy + (float)cy * cs, loz = g.oz + (float)cz * cs;
    float own = fminf(fminf(qx - lox, lox + cs - qx), fminf(qy - loy, loy + cs - qy));
    own = fminf(own, fminf(qz - loz, loz + cs - qz)) - m;
    const uint32_t TP = shell1_table<K, G>(g, qx, qy, qz, lox, loy, loz, sub, lds, b4, n4, tk.worst(), nullptr);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    scan_table_strided<K, U>(g, qx, qy, qz, lds, TP & 0xffffffu, TP >> 24, (uint32_t)sub, (uint32_t)G, tk);
    group_merge<K, G>(tk);
    if (tk.id(K - 1) == kNone && bound < range_sq) {  // guard: not full under a finite bound
        tk.init(range_sq);
        return -1;
    }
    const float gr = own + cs;
    return (gr > 0.f && tk.worst() < gr * gr * 0.999999f) ? 1 : 0;
}

// Far pass with a whole block (NT lanes) per query: the box cells outside
// the 3x3x3 block are judged one per lane per round of NT, the kept cells'
// ranges concatenated by a block prefix sum (slot table in LDS: s_b[NT],
// s_off[NT+1]), every lane takes a contiguous chunk of the concatenation
// (one binary search, then sequential, four loads in flight), and the lists
// are merged per wave (butterfly) and across waves (thread 0).  The result is
// in thread 0.  Exact: every point with d2 <= K-th best lies in
// the box, because the grid build's cell assignment (cell_coord, clamped) is
// monotone in each coordinate.  Must be called
// by all NT threads of the block (it synchronises the block).
template <int K, int NT>
__device__ void block_knn_box_flat(const GridDev& g, float qx, float qy, float qz, uint32_t* s_b, uint32_t* s_off,
                                   uint32_t* s_w, uint64_t* s_lists, TopK<K>& tk, bool whole = false) {
    static_assert(NT % 64 == 0 && NT <= 1024, "block_knn_box_flat: NT = multiple of 64");
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cx = cell_coord(qx, g.ox, g.inv_cell);
    const int cy = cell_coord(qy, g.oy, g.inv_cell);
    const int cz = cell_coord(qz, g.oz, g.inv_cell);
    // the near pass covered the 3x3x3 block only for queries whose cell lies in the grid
    // (whole: the near pass left the block unfinished, scan it too)
    const bool near_done = !whole && (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny &&
                           (unsigned)cz < (unsigned)g.nz;
    const float r = sqrtf(tk.worst()) + 2.f * g.margin;
    const int x0 = max(cell_coord(qx - r, g.ox, g.inv_cell), 0), x1 = min(cell_coord(qx + r, g.ox, g.inv_cell), g.nx - 1);
    const int y0 = max(cell_coord(qy - r, g.oy, g.inv_cell), 0), y1 = min(cell_coord(qy + r, g.oy, g.inv_cell), g.ny - 1);
    const int z0 = max(cell_coord(qz - r, g.oz, g.inv_cell), 0), z1 = min(cell_coord(qz + r, g.oz, g.inv_cell), g.nz - 1);
    if (x0 > x1 || y0 > y1 || z0 > z1) return;  // block-uniform
    if (tid != 0) tk.fill_with_worst();
    const float cs = g.cell, m = g.margin, w = cs + 2.f * m;
    const float bound = tk.worst();
    const int wx = x1 - x0 + 1, wxy = wx * (y1 - y0 + 1), nbox = wxy * (z1 - z0 + 1);
    for (int base = 0; base < nbox; base += NT) {
        const int k = base + tid;
        uint32_t b = 0, n = 0;
        if (k < nbox) {
            const int z = z0 + k / wxy, kk = k % wxy;
            const int y = y0 + kk / wx, x = x0 + kk % wx;
            if (!(near_done && abs(x - cx) <= 1 && abs(y - cy) <= 1 && abs(z - cz) <= 1)) {  // block: near pass
                const float xl = g.ox + (float)x * cs - m, yl = g.oy + (float)y * cs - m, zl = g.oz + (float)z * cs - m;
                const float bd = (axis_gap(qx, xl, xl + w) + axis_gap(qy, yl, yl + w)) + axis_gap(qz, zl, zl + w);
                if (!(bd * 0.999999f > bound)) {
                    const uint32_t c = ((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x;
                    const uint2 rc = g.rng[c];
                    b = rc.x;
                    n = rc.y - rc.x;
                }
            }
        }
        uint32_t incl = n;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(incl, off, 64);
            if (lane >= off) incl += v;
        }
        if (lane == 63) s_w[wid] = incl;
        __syncthreads();  // also: the previous round's readers are done
        uint32_t wbase = 0, T = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            const uint32_t v = s_w[q];
            wbase += q < wid ? v : 0u;
            T += v;
        }
        s_b[tid] = b;
        s_off[tid] = wbase + incl - n;
        if (tid == 0) s_off[NT] = T;
        __syncthreads();
        if (T == 0) continue;  // block-uniform
        // contiguous chunk [c0, c1) of the concatenation per lane
        const uint32_t chunk = (T + NT - 1) / NT;
        const uint32_t c0 = min((uint32_t)tid * chunk, T), c1 = min(c0 + chunk, T);
        if (c0 < c1) {
            int lo = 0, hi = NT;  // last slot with s_off[slot] <= c0
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_off[mid] <= c0) lo = mid;
                else hi = mid;
            }
            int sl = lo;
            uint32_t so = s_off[sl], se = s_off[sl + 1], sb = s_b[sl];
            for (uint32_t t = c0; t < c1; t += 4) {
                float4 pp[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t tt = t + (uint32_t)u;
                    pp[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (tt < c1) {
                        while (tt >= se) {
                            ++sl;
                            so = se;
                            se = s_off[sl + 1];
                            sb = s_b[sl];
                        }
                        pp[u] = g.pts[sb + (tt - so)];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (t + (uint32_t)u < c1) {
                        const float d = sqdist3(qx, qy, qz, pp[u].x, pp[u].y, pp[u].z);
                        tk.push(d, __float_as_int(pp[u].w));
                    }
            }
        }
    }
    group_merge<K, 64>(tk);
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < K; ++j) s_lists[wid * K + j] = tk.k[j];
    __syncthreads();
    if (tid == 0)
        for (int q = 1; q < NW; ++q)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint64_t v = s_lists[q * K + j];
                tk.push(__uint_as_float((uint32_t)(v >> 32)), (int)(uint32_t)v);
            }
    __syncthreads();  // s_lists / slot tables free for the caller's next query
}

// Wave64 sum of a double with DPP row operations (no LDS round trips):
// quad swaps, row_shr 4/8, row_bcast 15/31 leave the total in lane 63.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const int rlo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xf, false);
    const int rhi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROWMASK, 0xf, false);
    return __hiloint2double(rhi, rlo);
}
__device__ __forceinline__ double wave_sum_to_lane63(double v) {
    v += dpp_d<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_d<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_d<0x114, 0xf>(v);  // row_shr:4
    v += dpp_d<0x118, 0xf>(v);  // row_shr:8
    v += dpp_d<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp_d<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;                   // lane 63 holds the wave total
}

// Wave sum of 32 per-lane doubles by recursive halving: at each step a lane
// keeps half of its remaining values and adds the partner's copy of that half
// (the partner keeps the other half), so 32 values take 16+8+4+2+1 exchanges
// and adds instead of 32 x 6 (wave_sum_to_lane63 per value).  Partners:
// row_mirror (lane bit 3 decides the half), row_half_mirror (bit 2), quad_perm
// xor 2 (bit 1), xor 1 (bit 0), xor 16 (bit 4; a mirror partner flips the
// lower bits too, so the mirrors go first, while every partner pair still
// holds the same index set), then xor 32.  Returns, in lane l < 32, the wave
// total of value wave_sum32_index(l) (a fixed order: deterministic).
template <int CTRL, int BIT, int H>
__device__ __forceinline__ void halve_step(double (&v)[32], int lane) {
    const bool up = (lane >> BIT) & 1;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const double send = up ? v[j] : v[j + H];
        const double keep = up ? v[j + H] : v[j];
        v[j] = keep + dpp_d<CTRL, 0xf>(send);
    }
}

__device__ __forceinline__ int wave_sum32_index(int lane) {
    return ((lane >> 3) & 1) * 16 + ((lane >> 2) & 1) * 8 + ((lane >> 1) & 1) * 4 + (lane & 1) * 2 + ((lane >> 4) & 1);
}

__device__ __forceinline__ double wave_sum32(double (&v)[32], int lane) {
    halve_step<0x140, 3, 16>(v, lane);  // row_mirror
    halve_step<0x141, 2, 8>(v, lane);   // row_half_mirror
    halve_step<0x4e, 1, 4>(v, lane);    // quad_perm [2,3,0,1]
    halve_step<0xb1, 0, 2>(v, lane);    // quad_perm [1,0,3,2]
    const bool up = (lane >> 4) & 1;
    const double send = up ? v[0] : v[1];
    const double keep = up ? v[1] : v[0];
    const double t = keep + __shfl_xor(send, 16, 64);
    return t + __shfl_xor(t, 32, 64);
}

// ----------------------------------------------------------------------------
// Wave-level helpers shared by the tile kernels (ICP 1-NN, lio_icp.hip; the cell-grouped kNN near pass,
// lio_match.hip): LDS hand-off inside one wave, DPP reductions / scans, (d2, id) keys as f64.
// ----------------------------------------------------------------------------
// LDS handoff between the lanes of ONE wave (each wave owns its staging area)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (d2, id) keys minimised as f64: lio_dev.hpp key_min (one v_min_f64 instead of compare + two selects)
__device__ __forceinline__ double key_min_d(double a, double b) {
    return __longlong_as_double((long long)key_min((uint64_t)__double_as_longlong(a), (uint64_t)__double_as_longlong(b)));
}
__device__ __forceinline__ double key_of(float d2, uint32_t id) {
    return __longlong_as_double((long long)(((uint64_t)__float_as_uint(d2) << 32) | id));
}

// key (d[H], id[H]) of element H of a candidate pair in one v_pk_mov_b32: low word from the
// id pair, high word from the packed distance pair (no register shuffling)
template <int H>
__device__ __forceinline__ double key_pk(uint32_t id0, uint32_t id1, f2v d) {
    const double ids = __longlong_as_double((long long)(((uint64_t)id1 << 32) | id0));
    double k;
    if constexpr (H == 0)
        asm("v_pk_mov_b32 %0, %1, %2 op_sel:[0,0]" : "=v"(k) : "v"(ids), "v"(d));
    else
        asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,1]" : "=v"(k) : "v"(ids), "v"(d));
    return k;
}

// wave maximum of non-negative floats (as integers: same order), wave-uniform: DPP inside
// each row of 16 (quad swaps, half-row and row mirrors), then the four row maxima by readlane
// — no LDS permutes on the per-chunk path
__device__ __forceinline__ float wave_max_nonneg(float v) {
    uint32_t u = __float_as_uint(v);
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp((int)u, (int)u, 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp((int)u, (int)u, 0x4e, 0xf, 0xf, false));   // quad_perm 2,3,0,1
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp((int)u, (int)u, 0x141, 0xf, 0xf, false));  // row_half_mirror
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp((int)u, (int)u, 0x140, 0xf, 0xf, false));  // row_mirror
    const uint32_t m = max(max((uint32_t)__builtin_amdgcn_readlane((int)u, 0), (uint32_t)__builtin_amdgcn_readlane((int)u, 16)),
                           max((uint32_t)__builtin_amdgcn_readlane((int)u, 32), (uint32_t)__builtin_amdgcn_readlane((int)u, 48)));
    return __uint_as_float(m);
}

// wave-uniform values to SGPRs (the compiler cannot see that a butterfly
// result is uniform; keeping the box arithmetic scalar frees VGPRs)
__device__ __forceinline__ float uni_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ uint32_t uni_u(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// wave min / max of floats (any sign) by DPP inside each row of 16, then the four row
// results by readlane: wave-uniform, no LDS permutes
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, 0xf, 0xf, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_ext_dpp(float v) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
    v = op(v, dpp_f<0xb1>(v));   // quad_perm 1,0,3,2
    v = op(v, dpp_f<0x4e>(v));   // quad_perm 2,3,0,1
    v = op(v, dpp_f<0x141>(v));  // row_half_mirror
    v = op(v, dpp_f<0x140>(v));  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return uni_f(op(op(r0, r1), op(r2, r3)));
}

// inclusive prefix sum over the wave: DPP row shifts inside rows of 16, then row_bcast:15 /
// row_bcast:31 carry the row totals forward (rows 1, 3 then rows 2, 3)
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
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

// H row, extrinsic_est_en = false [U]: point_this = offset_R_L_I * p + offset_T_L_I,
// C = s.rot.conjugate() * n (quat_rotate), A = skew(point_this) * C:
// J = [n, p1 C2 - p2 C1, p2 C0 - p0 C2, p0 C1 - p1 C0]
__device__ __forceinline__ void h_row(const PoseArg& ps, float bx, float by, float bz, float na, float nb,
                                      float nc, double J[6]) {
    double a0, a1, a2;
    quat_rotate(ps.qLI, false, bx, by, bz, a0, a1, a2);
    const double p0 = a0 + ps.tLI[0], p1 = a1 + ps.tLI[1], p2 = a2 + ps.tLI[2];
    double n0 = na, n1 = nb, n2 = nc;
    double C0, C1, C2;
    quat_rotate(ps.q, true, n0, n1, n2, C0, C1, C2);
    J[0] = n0;
    J[1] = n1;
    J[2] = n2;
    J[3] = p1 * C2 - p2 * C1;
    J[4] = p2 * C0 - p0 * C2;
    J[5] = p0 * C1 - p1 * C0;
}

// ---------------------------------------------------------------------------------------------------------------
// Decoupled look-back (one pass scans: compaction offsets, event offsets).  Block b (its logical id from a ticket,
// so every predecessor was scheduled first) publishes a status word epoch << 34 | flag << 32 | value (flag 1: its
// aggregate, 2: its inclusive prefix; epoch: the launch's, so no memset between launches), looks back over its
// predecessors' words and publishes its inclusive prefix.  The look-back reads 64 predecessors per round with one
// wave (lane l: block j - l) and stops at the nearest inclusive word; a window holding a word of an older epoch
// (not yet published) is read again.  Words are 8-B agent-scope relaxed atomics (sc1) on both sides
// (MI355X_MICROARCH.md, hand-off table row 1: one lane per workgroup stores, the poller loads sc1).
typedef __attribute__((address_space(1))) unsigned long long lb_gu64;

__device__ __forceinline__ unsigned long long lb_word(uint32_t epoch, uint32_t flag, uint32_t v) {
    return ((unsigned long long)epoch << 34) | ((unsigned long long)flag << 32) | v;
}
__device__ __forceinline__ void lb_store(unsigned long long* st, int b, unsigned long long w) {
    __hip_atomic_store((lb_gu64*)(st + b), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* st, int j) {
    return __hip_atomic_load((lb_gu64*)(st + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The exclusive prefix of block b (all 64 lanes of the calling wave; b > 0, its aggregate already published).
// 64-bit second values ride along: aggregate / inclusive in agg64[j] / inc64[j], stored before the word that
// announces them (store, s_waitcnt vmcnt(0), word) and loaded after it (the load's address depends on the flag).
// time bound: a safety valve only (sets *timeout after 20 ms of wall_clock64's 100 MHz), every predecessor publishes
// before it looks back itself.
template <bool WITH64>
__device__ inline uint32_t lookback_excl(const unsigned long long* st, const unsigned long long* agg64,
                                         const unsigned long long* inc64, int b, uint32_t epoch, uint64_t& ex64,
                                         bool& timeout) {
    const int lane = threadIdx.x & 63;
    uint32_t acc = 0;
    uint64_t acc64 = 0;
    timeout = false;
    const uint64_t t0 = wall_clock64();
    for (int j = b - 1; j >= 0;) {
        const int idx = j - lane;
        unsigned long long w = idx >= 0 ? lb_load(st, idx) : lb_word(epoch, 2u, 0u);
        const bool valid = (uint32_t)(w >> 34) == epoch;
        const uint32_t flag = (uint32_t)(w >> 32) & 3u;
        const uint64_t incl = __ballot(valid && flag == 2u);
        const uint64_t inval = __ballot(!valid);
        const int fi = incl ? __builtin_ctzll(incl) : 64;   // nearest inclusive word
        const int fv = inval ? __builtin_ctzll(inval) : 64; // nearest unpublished word
        if (fv < fi) {  // a word before the nearest inclusive one is not published yet: read the window again
            if (wall_clock64() - t0 > 2000000ull) {
                timeout = true;
                break;
            }
            continue;
        }
        const int last = fi < 64 ? fi : 63;  // lanes 0 .. last contribute
        const bool take = lane <= last;
        uint32_t v = take ? (uint32_t)w : 0u;
        uint64_t v64 = 0;
        if constexpr (WITH64) {
            if (take && idx >= 0) v64 = lb_load(flag == 2u ? inc64 : agg64, idx);
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            v += __shfl_xor(v, d, 64);
            if constexpr (WITH64) v64 += __shfl_xor(v64, d, 64);
        }
        acc += v;
        acc64 += v64;
        if (fi < 64) break;
        j -= 64;
    }
    ex64 = acc64;
    return acc;
}

}  // namespace lio
