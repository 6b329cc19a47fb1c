// lio_match.hip — FAST-LIO h_share_model on gfx950.
//
// Per h-evaluation:
//
//   ekfom_data.converge == true (redo the kNN):
//     knn_near_kernel  512 threads = 64 points, 8 lanes per point:
//       body->world (double, stored float) -> exact grid 5-NN over shells 0-1,
//       cell points scanned lane-strided (coalesced), private top-5 lists
//       merged by a shuffle butterfly; unresolved points -> far queue
//     knn_far_kernel   one block per queued point, the rest of its search box
//     plane_kernel     lane = point: gate (found == 5 && d2[4] <= 5) ->
//       esti_plane (QR, registers) -> pd2, s-gate -> H row (double) ->
//       30-value DPP wave reduction -> block partial
//     writes: nn_idx[5] (20 B), plane abcd (16 B), sel (1 B)
//   ekfom_data.converge == false: h_model_reuse_kernel, lane = point
//     body->world -> cached plane -> pd2, s-gate -> H row -> block partial
//   the last block of plane/reuse to finish (agent-scope counter) sums the
//     block partials in a fixed order (deterministic) into host-mapped memory
//     + a sequence number (zero-copy result, no finalize launch)
//
// The per-point dense H (effct x 12 doubles) of the reference is never
// materialised: the IESKF only consumes H^T H and H^T h.
#include <hip/hip_ext.h>

#include "lio_dev.hpp"
#include "lio_kernels.hpp"

#include <algorithm>

namespace lio {

constexpr int kBlock = 256;  // partial-slot granule (the plane / reuse grids below never exceed n / 256 blocks)
constexpr int kPlaneBlock = 512;  // plane pass: 512 threads, 1 point per lane
constexpr int kReuseBlock = 512;  // reuse pass: 512 threads, 2 points per lane
constexpr int kReusePpl = 2;
constexpr int kNearBlock = 256;   // near pass: 32 queries per block

constexpr int kGroup = 8;   // lanes cooperating on one query's kNN
constexpr int kFarBlock = 128;  // threads per far query (64 / 256 / 512 measured slower)
constexpr int kFarBlocks = 1024;  // blocks striding the far queue (one query per block)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// pd2 / s-gate / H row of one selected point (h_share_model [U])
__device__ __forceinline__ bool residual_row(const MatchArgs& a, const PoseArg& ps, float bx, float by, float bz, float wx, float wy,
                                             float wz, const float4& pl, double J[6], double& h, double& res) {
    const float pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
    const double b0 = bx, b1 = by, b2 = bz;
    const double pn = sqrt((b0 * b0 + b1 * b1) + b2 * b2);
    const float s = (float)(1.0 - a.s_coef * (double)fabsf(pd2) / sqrt(pn));
    if (!((double)s > a.s_gate)) return false;
    h_row(ps, bx, by, bz, pl.x, pl.y, pl.z, J);
    h = -(double)pd2;
    res = (double)fabsf(pd2);
    return true;
}

// ekfom_data.converge == true, pass 1: 512 threads = 64 queries, 8 lanes per
// query run the exact 5-NN over shells 0-1 cooperatively (group_knn_near).
// Queries whose 5th neighbour is not yet provably final (sparse
// neighbourhoods, ~0.4% of a dense scan) are queued, with their list, for
// the wave-per-query far pass instead of holding their wave: a kernel runs as
// long as its slowest wave.  Written for 8 waves/SIMD (<= 64 VGPRs).
// U / UO: loads in flight in the seeded table scan / own-cell scan (2 keeps the kernel at <= 64 VGPRs
// without scratch).
template <bool DBG, bool SEEDED, int U, int NB, int UO>
__global__ void __launch_bounds__(NB) __attribute__((amdgpu_waves_per_eu(8, 8))) knn_near_kernel(MatchArgs a) {
    const PoseArg& ps = a.pose;
    constexpr int G = kGroup;
    constexpr int QPB = NB / G;  // 64 queries per block
    __shared__ uint32_t s_tab[QPB][72];      // per-group shell-1 slot table
    __shared__ float s_q[4][QPB];            // per query: world point (and the seeded pass's bound)
    __shared__ int s_c[3][QPB];              //            its cell
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int sub = threadIdx.x % G;
    const int q = threadIdx.x / G;
    const int i = blk * QPB + q;
    // the per-query transforms once per query, not once per lane of its group: wave 0, lane = query
    if (threadIdx.x < QPB) {
        const int iq = blk * QPB + (int)threadIdx.x;
        if (iq < a.n) {
            const float bx = a.body[3 * iq], by = a.body[3 * iq + 1], bz = a.body[3 * iq + 2];
            float wx, wy, wz;
            body_to_world(ps, bx, by, bz, wx, wy, wz);
            s_q[0][threadIdx.x] = wx;
            s_q[1][threadIdx.x] = wy;
            s_q[2][threadIdx.x] = wz;
            const int cx = cell_coord(wx, a.grid.ox, a.grid.inv_cell);
            const int cy = cell_coord(wy, a.grid.oy, a.grid.inv_cell);
            const int cz = cell_coord(wz, a.grid.oz, a.grid.inv_cell);
            s_c[0][threadIdx.x] = cx;
            s_c[1][threadIdx.x] = cy;
            s_c[2][threadIdx.x] = cz;
            if constexpr (SEEDED) {
                // float affine map of the previous kNN pose: w_old within ~1e-5 m, covered by the bound's margin
                const float* M = a.knn_M;
                const float wox = ((M[0] * bx + M[1] * by) + M[2] * bz) + M[3];
                const float woy = ((M[4] * bx + M[5] * by) + M[6] * bz) + M[7];
                const float woz = ((M[8] * bx + M[9] * by) + M[10] * bz) + M[11];
                const bool inside = (unsigned)cx < (unsigned)a.grid.nx && (unsigned)cy < (unsigned)a.grid.ny &&
                                    (unsigned)cz < (unsigned)a.grid.nz;
                s_q[3][threadIdx.x] = seeded_bound(inside, a.nn_d5[iq], wox, woy, woz, wx, wy, wz, a.range_sq, a.seed_scale);
            }
        }
    }
    __syncthreads();
    if (i >= a.n) return;
    const float wx = s_q[0][q], wy = s_q[1][q], wz = s_q[2][q];
    TopK<5> tk;
    tk.init(a.range_sq);
    SearchStats st{0, 0, 0};
    bool done, whole = false;
    if constexpr (SEEDED) {  // this scan's previous kNN against the same map: the triangle bound (no re-gathers)
        const int r = group_knn_seeded<5, G, U>(a.grid, s_q[3][q], s_c[0][q], s_c[1][q], s_c[2][q], wx, wy, wz, a.range_sq, sub,
                                                tk, s_tab[threadIdx.x / G]);
        done = r > 0;
        whole = r < 0;
    } else {
        done = group_knn_near<5, G, false, U, UO>(a.grid, wx, wy, wz, s_c[0][q], s_c[1][q], s_c[2][q], 1, sub, tk,
                                              DBG ? &st : nullptr, s_tab[threadIdx.x / G]);
    }
    const bool far = !done && a.max_shell > 1;
    if constexpr (DBG) {
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            st.cells += __shfl_xor(st.cells, off, 64);
            st.points += __shfl_xor(st.points, off, 64);
        }
        if (sub == 0) {
            a.dbg[3 * (size_t)i] = st.cells;
            a.dbg[3 * (size_t)i + 1] = st.points;
            a.dbg[3 * (size_t)i + 2] = far ? 2 : st.shell;
        }
    }
    if (far) {
        if (sub == 0) {
            const int slot = atomicAdd(a.far_count, 1);
            a.far_list[slot] = whole ? (int)((unsigned)i | 0x80000000u) : i;  // sign bit: search the block too
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                a.far_d[5 * (size_t)slot + j] = tk.d(j);
                a.far_id[5 * (size_t)slot + j] = tk.id(j);
            }
        }
        return;
    }
#pragma unroll
    for (int js = 0; js < 5; js += G) {
        const int jj = js + sub;
        if (jj < 5) {
            int v = tk.id(0);
#pragma unroll
            for (int j = 1; j < 5; ++j)
                if (jj == j) v = tk.id(j);
            a.nn_idx[5 * (size_t)i + jj] = v == kNone ? -1 : v;
        }
    }
    if (sub == 5) a.nn_d5[i] = tk.id(4) == kNone ? INFINITY : tk.d(4);
}

// ----------------------------------------------------------------------------
// Cell-grouped near pass (opt-in A/B, LIO_KNN_NEAR=cell; VERDICT r04 next #5 — bit-identical but 12x slower
// than the per-query pass at C3/C2, DESIGN §4: the wave tests every point of the union, which the per-query
// box pruning never touches).  A C3 Livox scan puts its 131 k queries in ~2.2 k
// map cells (median 8, p90 100 queries per 1 m cell), so queries of one cell share their 27-cell candidate set:
//   knn_group_kernel  once per scan (the first kNN evaluation): each block of 1024 consecutive queries sorted
//                     by world cell (bitonic, LDS) -> perm; 64 consecutive entries of perm = one wave's queries
//                     (~3 distinct cells per wave at C3)
//   knn_cell_kernel   one wave per 64 grouped queries, lane = query: the union of the wave's 3x3x3 blocks
//                     (each cell once: a head cell's neighbour inside an earlier head's block is skipped),
//                     own cells first, streamed through LDS in chunks of 256 with the ICP staging filter (a
//                     point farther from the wave's query box than every lane's current 5th best cannot
//                     enter any list), every lane testing every survivor (packed FP32 distances, TopK<5>
//                     under the (d2, id) total order: the list does not depend on the arrival order)
// The result contract is group_knn_near's / group_knn_seeded's: a query whose 5th best lies inside its block
// (worst < (own + cell)^2) is final — its list is then the exact top-5 whatever extra cells the wave added —
// and the others go to the far pass with their list, which is the exact top-5 over a superset of the block
// (points of other lanes' blocks included: the far pass skips keys already in the list, DEDUP).  The
// grouping only shapes the work: every lane transforms its own query with the current pose.
// ----------------------------------------------------------------------------
constexpr int kGroupSort = 1024;  // queries sorted per block
constexpr int kCellBlock = 256;   // near pass: 4 waves of 64 grouped queries
constexpr int kCellCh = 256;      // candidates staged per LDS round (per wave)

__global__ void __launch_bounds__(kGroupSort) knn_group_kernel(MatchArgs a) {
    __shared__ uint64_t s[kGroupSort];
    const int tid = threadIdx.x;
    const int base = blockIdx.x * kGroupSort;
    const int i = base + tid;
    uint64_t key = ~0ull;  // pads sort last
    if (i < a.n) {
        float wx, wy, wz;
        body_to_world(a.pose, a.body[3 * i], a.body[3 * i + 1], a.body[3 * i + 2], wx, wy, wz);
        const GridDev& g = a.grid;
        const int cx = cell_coord(wx, g.ox, g.inv_cell), cy = cell_coord(wy, g.oy, g.inv_cell),
                  cz = cell_coord(wz, g.oz, g.inv_cell);
        const bool inside = (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny && (unsigned)cz < (unsigned)g.nz;
        const uint32_t lin = inside ? ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx
                                    : 0xfffffffeu;
        key = ((uint64_t)lin << 32) | (uint32_t)tid;
    }
    s[tid] = key;
    __syncthreads();
    for (int k = 2; k <= kGroupSort; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int p = tid ^ j;
            if (p > tid) {
                const uint64_t x = s[tid], y = s[p];
                if ((x > y) == ((tid & k) == 0)) {
                    s[tid] = y;
                    s[p] = x;
                }
            }
            __syncthreads();
        }
    if (i < a.n) a.perm[i] = base + (int)(uint32_t)s[tid];
}

struct alignas(16) CellLds {
    float x[kCellCh], y[kCellCh], z[kCellCh];  // staged candidates (structure of arrays)
    uint32_t id[kCellCh];
    uint32_t b[64];                            // this round's cell ranges: start, exclusive prefix (+ total)
    uint32_t off[65];
    int hx[64], hy[64], hz[64];                // the wave's distinct query cells (heads)
};

// One round: every lane contributes one cell range [b, b + n); the concatenation streams through LDS in
// chunks of kCellCh, those farther from the wave's query box qb than every accepting lane's 5th best dropped
// (margin 1e-5 for the rounding of the gap and of d2), the survivors compacted (ballot + mbcnt) and tested by
// every lane.
__device__ __forceinline__ void cell_scan_round(const GridDev& g, CellLds& L, uint32_t b, uint32_t n, bool take,
                                                float qx, float qy, float qz, const float (&qb)[6], TopK<5>& tk) {
    const int lane = threadIdx.x & 63;
    const uint32_t incl = wave_incl_scan_dpp(n);
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (T == 0) return;  // wave-uniform
    wave_sync();          // the previous round's readers of the slot table are done
    L.b[lane] = b;
    L.off[lane] = incl - n;
    if (lane == 63) L.off[64] = T;
    wave_sync();
    int sl = 0;
    uint32_t lo = 0, hi = L.off[1], sb = L.b[0];
#pragma unroll 1
    for (uint32_t base = 0; base < T; base += kCellCh) {
        constexpr int U = kCellCh / 64;
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // slot walk first (clamped to the last point), U loads in flight
            const uint32_t t = min(base + (uint32_t)(u * 64 + lane), T - 1);
            while (t >= hi) {
                ++sl;
                lo = hi;
                hi = L.off[sl + 1];
                sb = L.b[sl];
            }
            v[u] = g.pts[sb + (t - lo)];
        }
        const float Bw = wave_max_nonneg(take ? tk.worst() : 0.f);
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float gx = fmaxf(fmaxf(qb[0] - v[u].x, v[u].x - qb[1]), 0.f);
            const float gy = fmaxf(fmaxf(qb[2] - v[u].y, v[u].y - qb[3]), 0.f);
            const float gz = fmaxf(fmaxf(qb[4] - v[u].z, v[u].z - qb[5]), 0.f);
            const float gap2 = (gx * gx + gy * gy) + gz * gz;
            const bool in = base + (uint32_t)(u * 64 + lane) < T && !(gap2 * (1.f - 1e-5f) > Bw);
            const uint64_t m = __ballot(in);
            const uint32_t r = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (in) {
                L.x[r] = v[u].x;
                L.y[r] = v[u].y;
                L.z[r] = v[u].z;
                L.id[r] = __float_as_uint(v[u].w);
            }
            cnt += (uint32_t)__popcll(m);
        }
        const uint32_t cnt2 = (cnt + 1u) & ~1u;
        if (lane == 0 && cnt2 != cnt) {  // pad to a pair: +inf, kNone (never enters a list)
            L.x[cnt] = INFINITY;
            L.y[cnt] = INFINITY;
            L.z[cnt] = INFINITY;
            L.id[cnt] = (uint32_t)kNone;
        }
        wave_sync();
        const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
        for (uint32_t j = 0; j < cnt2; j += 2) {  // packed FP32 distances, ((dx*dx + dy*dy) + dz*dz) per element
            const float2 X = *reinterpret_cast<const float2*>(&L.x[j]);
            const float2 Y = *reinterpret_cast<const float2*>(&L.y[j]);
            const float2 Z = *reinterpret_cast<const float2*>(&L.z[j]);
            const uint2 I = *reinterpret_cast<const uint2*>(&L.id[j]);
            const f2v dx = qx2 - f2v{X.x, X.y}, dy = qy2 - f2v{Y.x, Y.y}, dz = qz2 - f2v{Z.x, Z.y};
            const f2v d = (dx * dx + dy * dy) + dz * dz;
            tk.push2(knn_key(d.x, (int)I.x), knn_key(d.y, (int)I.y));
        }
        wave_sync();  // chunk consumed before it is overwritten
    }
}

template <bool SEEDED>
__global__ void __launch_bounds__(kCellBlock) knn_cell_kernel(MatchArgs a) {
    __shared__ CellLds Ls[kCellBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    CellLds& L = Ls[wv];
    const GridDev& g = a.grid;
    const int slot = (xcd_block(blockIdx.x, gridDim.x) * (kCellBlock / 64) + wv) * 64 + lane;
    const bool act = slot < a.n;
    const int i = act ? a.perm[slot] : 0;
    float bx = 0.f, by = 0.f, bz = 0.f, wx = 0.f, wy = 0.f, wz = 0.f;
    if (act) {
        bx = a.body[3 * i];
        by = a.body[3 * i + 1];
        bz = a.body[3 * i + 2];
        body_to_world(a.pose, bx, by, bz, wx, wy, wz);
    }
    const int cx = cell_coord(wx, g.ox, g.inv_cell), cy = cell_coord(wy, g.oy, g.inv_cell),
              cz = cell_coord(wz, g.oz, g.inv_cell);
    const bool inside = act && (unsigned)cx < (unsigned)g.nx && (unsigned)cy < (unsigned)g.ny && (unsigned)cz < (unsigned)g.nz;
    float bound = a.range_sq;
    if constexpr (SEEDED) {
        if (act) {  // the triangle bound from this scan's previous kNN (group_knn_seeded)
            const float* M = a.knn_M;
            const float wox = ((M[0] * bx + M[1] * by) + M[2] * bz) + M[3];
            const float woy = ((M[4] * bx + M[5] * by) + M[6] * bz) + M[7];
            const float woz = ((M[8] * bx + M[9] * by) + M[10] * bz) + M[11];
            bound = seeded_bound(inside, a.nn_d5[i], wox, woy, woz, wx, wy, wz, a.range_sq, a.seed_scale);
        }
    }
    TopK<5> tk;
    tk.init(bound);
    // lanes that take no candidate (inactive, or the query outside the grid: the far pass searches its whole
    // box) test from a far-away point: d2 overflows to +inf and never enters the list
    const float qx = inside ? wx : 1e30f, qy = inside ? wy : 1e30f, qz = inside ? wz : 1e30f;
    const float qb[6] = {wave_ext_dpp<false>(inside ? wx : INFINITY), wave_ext_dpp<true>(inside ? wx : -INFINITY),
                         wave_ext_dpp<false>(inside ? wy : INFINITY), wave_ext_dpp<true>(inside ? wy : -INFINITY),
                         wave_ext_dpp<false>(inside ? wz : INFINITY), wave_ext_dpp<true>(inside ? wz : -INFINITY)};
    // the wave's distinct cells: a lane whose cell differs from its left neighbour's is a head (equal cells that
    // are not adjacent give a second head whose block is wholly inside the first's: skipped below)
    const uint32_t lin = inside ? ((uint32_t)cz * (uint32_t)g.ny + (uint32_t)cy) * (uint32_t)g.nx + (uint32_t)cx
                                : 0xffffffffu;
    const uint32_t prv = (uint32_t)__shfl_up((int)lin, 1, 64);
    const bool head = inside && (lane == 0 || lin != prv);
    const uint64_t hm = __ballot(head);
    const int D = __popcll(hm);
    if (head) {
        const int h = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
        L.hx[h] = cx;
        L.hy[h] = cy;
        L.hz[h] = cz;
    }
    wave_sync();
    const int ncand = 27 * D;  // (block offset o, head) pairs, offset-major: every head's own cell first
#pragma unroll 1
    for (int cb = 0; cb < ncand; cb += 64) {
        const int j = cb + lane;
        uint32_t b = 0, n = 0;
        if (j < ncand) {
            const int o = j / D, hh = j - o * D;
            const int k = o == 0 ? 13 : (o <= 13 ? o - 1 : o);  // 13 = the block's centre
            const int x = L.hx[hh] + k % 3 - 1, y = L.hy[hh] + (k / 3) % 3 - 1, z = L.hz[hh] + k / 9 - 1;
            bool keep = (unsigned)x < (unsigned)g.nx && (unsigned)y < (unsigned)g.ny && (unsigned)z < (unsigned)g.nz;
            for (int h2 = 0; keep && h2 < hh; ++h2)  // inside an earlier head's block: that head covers it
                keep = !(abs(x - L.hx[h2]) <= 1 && abs(y - L.hy[h2]) <= 1 && abs(z - L.hz[h2]) <= 1);
            if (keep) {
                const uint2 r = g.rng[((uint32_t)z * (uint32_t)g.ny + (uint32_t)y) * (uint32_t)g.nx + (uint32_t)x];
                b = r.x;
                n = r.y - r.x;
            }
        }
        cell_scan_round(g, L, b, n, inside, qx, qy, qz, qb, tk);
    }
    if (!act) return;
    // final / far decision: group_knn_near's (unseeded) and group_knn_seeded's
    bool done = false, whole = false;
    if (inside) {
        const float cs = g.cell, m = g.margin;
        const float lox = g.ox + (float)cx * cs, loy = g.oy + (float)cy * cs, loz = g.oz + (float)cz * cs;
        float own = fminf(fminf(wx - lox, lox + cs - wx), fminf(wy - loy, loy + cs - wy));
        own = fminf(own, fminf(wz - loz, loz + cs - wz)) - m;
        if constexpr (SEEDED) {
            if (tk.id(4) == kNone && bound < a.range_sq) {  // guard: not full under a finite bound
                tk.init(a.range_sq);
                whole = true;
            }
        }
        const float gr = own + cs;
        done = !whole && gr > 0.f && tk.worst() < gr * gr * 0.999999f;
    }
    if (!done && a.max_shell > 1) {
        const int fs = atomicAdd(a.far_count, 1);
        a.far_list[fs] = whole ? (int)((unsigned)i | 0x80000000u) : i;  // sign bit: search the block too
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            a.far_d[5 * (size_t)fs + j] = tk.d(j);
            a.far_id[5 * (size_t)fs + j] = tk.id(j);
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) a.nn_idx[5 * (size_t)i + j] = tk.id(j) == kNone ? -1 : tk.id(j);
    a.nn_d5[i] = tk.id(4) == kNone ? INFINITY : tk.d(4);
}

// Pass 2: the queued queries, one block each (block_knn_box_flat over the
// rest of the query's search box).  Fixed grid; every block strides the queue
// and exits once past its end.
template <int NT = kFarBlock, bool DEDUP = false>
__global__ void __launch_bounds__(NT) knn_far_kernel(MatchArgs a) {
    const PoseArg& ps = a.pose;
    __shared__ uint32_t s_b[NT], s_off[NT + 1], s_w[NT / 64];
    __shared__ uint64_t s_lists[(NT / 64) * 5];
    const int cnt = *a.far_count;
    for (int f = blockIdx.x; f < cnt; f += gridDim.x) {
        const int e = a.far_list[f];
        const int i = e & 0x7fffffff;
        float wx, wy, wz;
        body_to_world(ps, a.body[3 * i], a.body[3 * i + 1], a.body[3 * i + 2], wx, wy, wz);
        TopK<5> tk;
#pragma unroll
        for (int j = 0; j < 5; ++j) tk.k[j] = knn_key(a.far_d[5 * (size_t)f + j], a.far_id[5 * (size_t)f + j]);
        // DEDUP: a cell-grouped near list may already hold points outside this query's 3x3x3 block
        block_knn_box_flat<5, NT, DEDUP>(a.grid, wx, wy, wz, s_b, s_off, s_w, s_lists, tk, e < 0);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int j = 0; j < 5; ++j) a.nn_idx[5 * (size_t)i + j] = tk.id(j) == kNone ? -1 : tk.id(j);
            a.nn_d5[i] = tk.id(4) == kNone ? INFINITY : tk.d(4);
        }
    }
}

// Block partial -> global, and the LAST block to finish sums all partials
// (fixed order: deterministic) into the host-mapped result + sequence number,
// so no separate finalize launch.  Hand-off per MI355X_MICROARCH.md
// § visibility, row "one lane of each storing workgroup ... agent-scope atomic
// add / the workgroup whose add came last": the partial is stored
// write-through (sc1: agent-scope relaxed atomic store), the storing wave
// drains (vmcnt(0)), a barrier, ONE lane adds to the counter; the block
// whose add returns nblocks-1 reads every partial with sc1 loads
// (agent-scope relaxed atomic loads) after a barrier.  No release fence (an
// agent release per block writes back the XCD's L2: 8 -> 35 us measured).
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned int guint;
typedef __attribute__((address_space(1))) unsigned long long gull;

// Host hand-off in ONE round trip: wave lanes 0-31 store the 32 sums, lane 32
// the sequence number, lane 33 a checksum of (sums, seq), all write-through at
// system scope (sc0 sc1) and unordered.  The host (lio_capi.cpp wait_result)
// accepts a result once it reads the expected sequence number AND sums whose
// checksum matches: a word still in flight (or the previous evaluation's)
// fails the check and the host polls again; once the kernel has completed,
// every word has landed.  No system release (its write-back and the wait for
// the sums' completion before the flag cost 1.7-2 us per evaluation).
// Called by all 64 lanes of one wave; lane l < 32 passes sum l.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void publish_host(double t, double* out, unsigned long long* seq_out, unsigned long long seq) {
    const int lane = threadIdx.x & 63;
    unsigned long long h =
        lane < 32 ? mix64((unsigned long long)__double_as_longlong(t) ^ ((unsigned long long)lane * 0x9e3779b97f4a7c15ull))
                  : 0ull;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) h ^= __shfl_xor(h, off, 64);
    h = __shfl(h, 0, 64);
    if (lane < 32) __hip_atomic_store((gdouble*)(out + lane), t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (lane == 32) __hip_atomic_store((gull*)seq_out, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (lane == 33) __hip_atomic_store((gull*)(seq_out + 1), h ^ mix64(seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block partial -> global; returns true in the LAST block to finish, whose
// lanes < 32 then hold the 32 fixed-order sums in `t` (wave 0; block-uniform
// return value).
// slot: this block's partial index (-1: none); npart partials are summed; ncount
// blocks take part in the counter.  All threads of the block call it.
template <int BS = kBlock>
__device__ __forceinline__ bool block_partial_last(const MatchArgs& a, double (*red)[32], double& t, int slot, int npart,
                                                   int ncount) {
    __shared__ int s_last;
    const int nb = npart;
    t = 0.0;
    if (slot >= 0 && threadIdx.x < 32) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < BS / 64; ++w) s += red[w][threadIdx.x];
        __hip_atomic_store((gdouble*)(a.partials + (size_t)slot * 32 + threadIdx.x), s, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add((guint*)a.done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)(ncount - 1);
    }
    __syncthreads();
    if (!s_last) return false;  // block-uniform
    // fixed-order sum: 8 row groups x 32 columns, then the groups in order
    const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
    constexpr int NG = BS / 32;
    const int per = (nb + NG - 1) / NG;
    const int b0 = grp * per, b1 = min(nb, b0 + per);
    double acc = 0.0;
    int b = b0;
    // batches of 32 sc1 loads in flight per thread (cross-XCD: each batch is an L2 miss), the
    // last batch masked rather than finished one load at a time (a serial tail of 27 loads
    // doubled the kernel at C5's 469 blocks)
    for (; b < b1; b += 32) {
        double v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k)
            v[k] = b + k < b1 ? __hip_atomic_load((gdouble*)(a.partials + (size_t)(b + k) * 32 + col), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : 0.0;
#pragma unroll
        for (int k = 0; k < 32; ++k) acc += v[k];
    }
    __shared__ double sg[NG][33];
    sg[grp][col] = acc;
    __syncthreads();
    if (threadIdx.x < 32)
#pragma unroll
        for (int g = 0; g < NG; ++g) t += sg[g][threadIdx.x];
    if (threadIdx.x == 0)
        __hip_atomic_store((guint*)a.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    return true;
}

// the last block publishes the sums to the host (lio_match)
template <int BS = kBlock>
__device__ __forceinline__ void publish_and_finalize(const MatchArgs& a, double (*red)[32]) {
    double t;
    if (block_partial_last<BS>(a, red, t, blockIdx.x, gridDim.x, gridDim.x) && threadIdx.x < 64)
        publish_host(t, a.sums_out, a.seq_out, a.seq);
}

// One lane's H-row contribution [HTH(21), HTh(6), cnt, res, hh] added into v[32].
__device__ __forceinline__ void accum_row(double (&v)[32], const double J[6], double h, double res, double cnt) {
    int q = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) v[q++] += J[r] * J[c];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[21 + r] += J[r] * h;
    v[27] += cnt;
    v[28] += res;
    v[29] += h * h;
}

// Plane pass body, lane = PPL points (strided by the block size, coalesced): gate
// (found == 5 && d2[4] <= 5), esti_plane, pd2, s-gate, H row, summed into v.
template <int PPL, int BS = kBlock>
__device__ __forceinline__ void plane_points(const MatchArgs& a, const PoseArg& ps, int blk, double (&v)[32]) {
    const int i0 = blk * BS * PPL + threadIdx.x;
    // all points' ids first, then all neighbour gathers: PPL independent chains in flight
    int id[PPL][5];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
#pragma unroll
        for (int j = 0; j < 5; ++j) id[k][j] = i < a.n ? a.nn_idx[5 * (size_t)i + j] : -1;
    }
    float P[PPL][5][3];
#pragma unroll
    for (int k = 0; k < PPL; ++k)
        if (id[k][4] >= 0)
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float4 q = a.map_by_id[id[k][j]];
                P[k][j][0] = q.x;
                P[k][j][1] = q.y;
                P[k][j][2] = q.z;
            }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
        if (i < a.n) {
            // sorted list: the 5th exists => all exist, d2 <= range by construction
            bool sel = id[k][4] >= 0;
            if (sel) {
                const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
                float abcd[4];
                sel = esti_plane_dev(P[k], a.plane_thr, abcd);
                const float4 pl = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
                a.planes[i] = pl;
                if (sel) {
                    float wx, wy, wz;
                    body_to_world(ps, bx, by, bz, wx, wy, wz);
                    double J[6], h, res;
                    sel = residual_row(a, ps, bx, by, bz, wx, wy, wz, pl, J, h, res);
                    if (sel) accum_row(v, J, h, res, 1.0);
                }
            }
            a.sel[i] = sel ? 1 : 0;
        }
    }
}

// Reuse pass body (ekfom_data.converge == false: cached Nearest_Points / planes), PPL points per lane.
template <int PPL, int BS = kBlock>
__device__ __forceinline__ void reuse_points(const MatchArgs& a, const PoseArg& ps, int blk, double (&v)[32]) {
    const int i0 = blk * BS * PPL + threadIdx.x;
    // every point's three loads issued together (one round trip instead of sel -> body/plane)
    bool sel[PPL];
    float b[PPL][3];
    float4 pl[PPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
        sel[k] = false;
        if (i < a.n) {
            sel[k] = a.sel[i] != 0;
            b[k][0] = a.body[3 * i];
            b[k][1] = a.body[3 * i + 1];
            b[k][2] = a.body[3 * i + 2];
            pl[k] = a.planes[i];
        }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        if (sel[k]) {
            const int i = i0 + k * BS;
            float wx, wy, wz;
            body_to_world(ps, b[k][0], b[k][1], b[k][2], wx, wy, wz);
            double J[6], h, res;
            const bool s = residual_row(a, ps, b[k][0], b[k][1], b[k][2], wx, wy, wz, pl[k], J, h, res);
            if (s) accum_row(v, J, h, res, 1.0);
            a.sel[i] = s ? 1 : 0;
        }
    }
}

// Pass 3 (kNN evaluations): plane_points, wave sums, the block's wave partials
// combined in LDS -> block partial; the last block publishes.  Resets the far
// queue for the next kNN evaluation.
template <int PPL, int BS>
__global__ void __launch_bounds__(BS) plane_kernel(MatchArgs a) {
    const PoseArg& ps = a.pose;
    __shared__ double red[BS / 64][32];
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = 0.0;
    plane_points<PPL, BS>(a, ps, blockIdx.x, v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double tot = wave_sum32(v, lane);
    if (lane < 32) red[wid][wave_sum32_index(lane)] = tot;
    __syncthreads();
    publish_and_finalize<BS>(a, red);
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.far_count = 0;
}

// ekfom_data.converge == false: reuse_points, same reduction and publish.
template <int PPL, int BS>
__global__ void __launch_bounds__(BS) h_model_reuse_kernel(MatchArgs a) {
    const PoseArg& ps = a.pose;
    __shared__ double red[BS / 64][32];
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = 0.0;
    reuse_points<PPL, BS>(a, ps, blockIdx.x, v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double tot = wave_sum32(v, lane);
    if (lane < 32) red[wid][wave_sum32_index(lane)] = tot;
    __syncthreads();
    publish_and_finalize<BS>(a, red);
}

// ikd-Tree Nearest_Search(point, k, Nearest_Points, Point_Distance, max_dist)
// over a batch of query points: 8 lanes per query, exact (d2, id)-ordered
// 5-NN within d2 <= bound (bound = INFINITY: unbounded, any number of shells),
// the first k kept.  Missing neighbours: id -1, d2 = INFINITY.
__global__ void __launch_bounds__(256) map_knn_kernel(GridDev g, const float* __restrict__ q, int n, float bound,
                                                      int max_shell, int k, int32_t* __restrict__ idx,
                                                      float* __restrict__ d2) {
    constexpr int G = kGroup;
    const int sub = threadIdx.x % G;
    const int i = blockIdx.x * (256 / G) + threadIdx.x / G;
    if (i >= n) return;
    TopK<5> tk;
    tk.init(bound);
    group_knn_exact<5, G>(g, q[3 * (size_t)i], q[3 * (size_t)i + 1], q[3 * (size_t)i + 2], max_shell, sub, tk);
    if (sub < k) {
        int v = tk.id(0);
        float d = tk.d(0);
#pragma unroll
        for (int j = 1; j < 5; ++j)
            if (sub == j) {
                v = tk.id(j);
                d = tk.d(j);
            }
        const bool ok = v != kNone;
        idx[(size_t)i * k + sub] = ok ? v : -1;
        if (d2) d2[(size_t)i * k + sub] = ok ? d : INFINITY;
    }
}

// Debug: world points, d2 of the stored neighbours, pd2 of selected points.
__global__ void debug_kernel(MatchArgs a, float* __restrict__ world, float* __restrict__ d2,
                             float* __restrict__ abcd_pd2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    float wx, wy, wz;
    body_to_world(a.pose, a.body[3 * i], a.body[3 * i + 1], a.body[3 * i + 2], wx, wy, wz);
    if (world) {
        world[3 * i] = wx;
        world[3 * i + 1] = wy;
        world[3 * i + 2] = wz;
    }
    if (d2) {
        for (int j = 0; j < 5; ++j) {
            int id = a.nn_idx[5 * (size_t)i + j];
            float v = INFINITY;
            if (id >= 0) {
                float4 q = a.map_by_id[id];
                v = sqdist3(wx, wy, wz, q.x, q.y, q.z);
            }
            d2[5 * (size_t)i + j] = v;
        }
    }
    if (abcd_pd2) {
        float4 pl = make_float4(0, 0, 0, 0);
        float pd2 = 0.f;
        if (a.sel[i]) {
            pl = a.planes[i];
            pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
        }
        abcd_pd2[4 * (size_t)i] = pl.x;
        abcd_pd2[4 * (size_t)i + 1] = pl.y;
        abcd_pd2[4 * (size_t)i + 2] = pl.z;
        abcd_pd2[4 * (size_t)i + 3] = pd2;
    }
}

// Ordered compaction of the H rows of selected points (dof < 23 branch only):
// one block walks the points in index order.
__global__ void __launch_bounds__(1024) h_rows_kernel(MatchArgs a, double* __restrict__ rows, int64_t max_rows,
                                                      int64_t* __restrict__ n_rows) {
    __shared__ int wave_cnt[16];
    __shared__ int64_t base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int64_t off = 0; off < a.n; off += 1024) {
        const int64_t i = off + threadIdx.x;
        const bool s = i < a.n && a.sel[i];
        const unsigned long long m = __ballot(s);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wave_cnt[wid] = __popcll(m);
        __syncthreads();
        int wbase = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wid) wbase += wave_cnt[w];
            tot += wave_cnt[w];
        }
        if (s) {
            const int64_t r = base + wbase + before;
            if (r < max_rows) {
                const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
                float wx, wy, wz;
                body_to_world(a.pose, bx, by, bz, wx, wy, wz);
                const float4 pl = a.planes[i];
                const float pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
                double J[6];
                h_row(a.pose, bx, by, bz, pl.x, pl.y, pl.z, J);
                for (int k = 0; k < 6; ++k) rows[7 * r + k] = J[k];
                rows[7 * r + 6] = -(double)pd2;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_rows = base;
}

// ---------------------------------------------------------------- launchers
// The measured-best forms only (A/B history: DESIGN §4): near pass in 32-query blocks with 2 loads in
// flight in the seeded table scan and in the own-cell scan (no scratch spills); far pass one
// 128-thread block per queued query on a fixed 1024-block grid; plane pass 512 x 1 point per lane;
// reuse pass 512 x 2 points per lane.
int launch_h_model(const MatchArgs& a, bool redo, hipStream_t st, hipEvent_t* marks) {
    if (a.n == 0) return 0;
    // hipExtLaunchKernelGGL with null events is a plain launch; with events (timing) the command
    // processor stamps them at the kernel's own start / end
    hipEvent_t m[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (marks)
        for (int k = 0; k < 8; ++k) m[k] = marks[k];
    if (redo) {
        constexpr int qpb = kNearBlock / kGroup;
        const int nq = (a.n + qpb - 1) / qpb;
        if (a.dbg) {  // search statistics (lio_ctx_knn_stats): the per-query group walk
            hipExtLaunchKernelGGL((knn_near_kernel<true, false, 4, kNearBlock, 2>), dim3(nq), dim3(kNearBlock), 0, st,
                                  m[0], m[1], 0, a);
        } else if (a.perm) {  // cell-grouped near pass; the grouping once per scan (first kNN evaluation)
            const int nc = (a.n + kCellBlock - 1) / kCellBlock;
            if (!a.prior) {
                hipExtLaunchKernelGGL(knn_group_kernel, dim3((a.n + kGroupSort - 1) / kGroupSort), dim3(kGroupSort), 0,
                                      st, m[0], nullptr, 0, a);
                hipExtLaunchKernelGGL(knn_cell_kernel<false>, dim3(nc), dim3(kCellBlock), 0, st, nullptr, m[1], 0, a);
            } else {
                hipExtLaunchKernelGGL(knn_cell_kernel<true>, dim3(nc), dim3(kCellBlock), 0, st, m[0], m[1], 0, a);
            }
        } else if (a.prior) {
            hipExtLaunchKernelGGL((knn_near_kernel<false, true, 2, kNearBlock, 4>), dim3(nq), dim3(kNearBlock), 0, st,
                                  m[0], m[1], 0, a);
        } else {
            hipExtLaunchKernelGGL((knn_near_kernel<false, false, 4, kNearBlock, 2>), dim3(nq), dim3(kNearBlock), 0, st,
                                  m[0], m[1], 0, a);
        }
        if (a.max_shell > 1) {
            if (a.perm && !a.dbg)
                hipExtLaunchKernelGGL((knn_far_kernel<kFarBlock, true>), dim3(kFarBlocks), dim3(kFarBlock), 0, st, m[2],
                                      m[3], 0, a);
            else
                hipExtLaunchKernelGGL((knn_far_kernel<kFarBlock, false>), dim3(kFarBlocks), dim3(kFarBlock), 0, st,
                                      m[2], m[3], 0, a);
        }
        const int nbp = (a.n + kPlaneBlock - 1) / kPlaneBlock;
        hipExtLaunchKernelGGL((plane_kernel<1, kPlaneBlock>), dim3(nbp), dim3(kPlaneBlock), 0, st, m[4], m[5], 0, a);
        return nbp;
    }
    const int nbr = (a.n + kReusePpl * kReuseBlock - 1) / (kReusePpl * kReuseBlock);
    hipExtLaunchKernelGGL((h_model_reuse_kernel<kReusePpl, kReuseBlock>), dim3(nbr), dim3(kReuseBlock), 0, st, m[6],
                          m[7], 0, a);
    return nbr;
}

void launch_debug(const MatchArgs& a, float* world, float* d2, float* abcd_pd2, hipStream_t st) {
    if (a.n == 0) return;
    debug_kernel<<<(a.n + 255) / 256, 256, 0, st>>>(a, world, d2, abcd_pd2);
}

void launch_h_rows(const MatchArgs& a, double* rows, int64_t max_rows, int64_t* n_rows, hipStream_t st) {
    h_rows_kernel<<<1, 1024, 0, st>>>(a, rows, max_rows, n_rows);
}

void launch_map_knn(const GridDev& g, const float* q, int n, float bound, int max_shell, int k, int32_t* idx,
                    float* d2, hipStream_t st) {
    if (n <= 0) return;
    map_knn_kernel<<<(n + 256 / kGroup - 1) / (256 / kGroup), 256, 0, st>>>(g, q, n, bound, max_shell, k, idx, d2);
}

int match_blocks(int n) {  // partial slots (plane / reuse kernels): n / 256 bounds both grids
    return (n + kBlock - 1) / kBlock;
}

}  // namespace lio
