// lio_icp.hip — loop-closure ICP (PCL IterativeClosestPoint as configured at
// /root/reference/fast_lio_sam/src/loop_closure.cpp:3-14, aligned at :81) on gfx950.
//
// Per ICP iteration (this rank's shard of the source):
//   icp_tile_kernel  one wave per tile of <= 64 spatially compact source points (binned
//                    once per setInputSource): apply the previous T_inc to
//                    the incrementally transformed cloud (PCL transformCloud,
//                    float SSE order [U]), exact unbounded 1-NN in the target
//                    grid with the candidate points staged through LDS once
//                    per tile; tiles visited longest-first in the pass after
//                    the first (icp_order_share, from this pass's counts)
//   icp_stats_kernel one 1024-thread block per 4096-point record: Umeyama
//                    sufficient statistics of the accepted correspondences
//                    (d2 <= 52.5^2) in double about a fixed centre c0:
//                    count, sum p, sum q, sum q p^T, sum d2 (fixed order)
// The 4096-point records are what ranks all-gather (deterministic, identical
// for any number of ranks).  The fitness pass is the same pipeline on the
// ORIGINAL source transformed by the final T.
#include <hipcub/hipcub.hpp>

#include "lio_dev.hpp"
#include "lio_error.hpp"
#include "lio_kernels.hpp"

namespace lio {

struct IcpT {  // a float 4x4 (row-major) by value in kernel arguments
    float m[16];
};

// PCL 1.10 Transformer<float>::se3 (SSE): x' = m0*x + (m1*y + (m2*z + m3)) [U]
__device__ __forceinline__ void xform_pcl(const float* T, float x, float y, float z, float& ox, float& oy,
                                          float& oz) {
    ox = T[0] * x + (T[1] * y + (T[2] * z + T[3]));
    oy = T[4] * x + (T[5] * y + (T[6] * z + T[7]));
    oz = T[8] * x + (T[9] * y + (T[10] * z + T[11]));
}

// ----------------------------------------------------------------------------
// Exact 1-NN of a tile of source points (one wave, lane = query).
//
// The source is binned once per setInputSource into a grid of tile cells
// (icp_build_tiles): a tile is <= 64 source points of one cell, so its
// bounding box Q is compact.  The target grid is x-fastest, so a row of cells
// (fixed y, z) is ONE contiguous range of points: the wave works on rows,
// one lane per row (a batch of rows re-ordered nearest-first), and every range
// goes through the same staging step (scan_ranges: wave prefix sum -> chunks
// of 256 points, those farther from Q than every lane's current best dropped,
// the rest compacted into LDS -> every lane tests every staged point against
// its own query, LDS broadcast reads), so the candidate points are loaded once
// per tile instead of once per query.
//   1. bound: a lane starts from its previous correspondence when the pass
//      has one (an exact candidate: its distance bounds the answer), else
//      the rows of Q's own cells are scanned; while some lane has found
//      nothing, the box grows geometrically (empty surroundings).
//   2. final: B = the largest best over the lanes; every target point within
//      sqrt(B) of some query lies in a row whose (y, z) gap to Q is <= sqrt(B),
//      inside that row's x-range [Q.x0 - r, Q.x1 + r], r = sqrt(B - gap^2):
//      those rows (minus what step 1 scanned) are scanned once, and every
//      lane's best is then exact.
// Total order (d2, id), d2 = float ((dx*dx + dy*dy) + dz*dz): the result
// does not depend on the tiling.
// ----------------------------------------------------------------------------
// The measured-best search shape (A/B history in DESIGN §4; the build switches that selected the variants are
// gone): 256 candidates staged per LDS round (128 equal, 512 slower), a round's rows by z slice and then by y
// row centre-out from the tile, rows trimmed per 64-row batch by the lanes' current bests, the growing box
// doubled while r < 3 and then widened by one cell a round.
constexpr int kTileCh = 256;  // candidates staged per LDS round

// Tiles -> blocks (launch_icp_tiles: 8 x (kIcpSegs / 8) x ceil(n / kIcpSegs) blocks; block b runs on
// XCD b % 8).  The cell-ordered tiles form kIcpSegs contiguous segments; XCD x owns segments x, x + 8,
// ...: its blocks walk those in cell order (first pass) or in the order icp_order_share wrote for its
// share (later passes).  -1: a slot past the XCD's share.
constexpr int kIcpSegs = 64;
__device__ __forceinline__ int icp_seg_begin(int s, int n) { return (int)(((int64_t)s * n) / kIcpSegs); }
__device__ __forceinline__ int icp_tile_of(const uint32_t* order, int b, int n) {
    const int x = b & 7;
    int slot = b >> 3;
    if (order) {
        const int lo = (int)order[n + x], hi = (int)order[n + x + 1];
        return lo + slot < hi ? (int)order[lo + slot] : -1;
    }
    for (int s = x; s < kIcpSegs; s += 8) {
        const int b0 = icp_seg_begin(s, n), sz = icp_seg_begin(s + 1, n) - b0;
        if (slot < sz) return b0 + slot;
        slot -= sz;
    }
    return -1;
}

// staged candidates as structure of arrays: 4 consecutive x (y, z, id) are one
// 16-byte broadcast read, and two candidates' coordinates sit in one register
// pair for the packed FP32 distance (v_pk_add_f32 / v_pk_mul_f32)
struct alignas(16) TileLds {
    float x[kTileCh], y[kTileCh], z[kTileCh];
    uint32_t id[kTileCh];
    union {  // the row permutation is read into registers before the slot table is written
        struct {
            uint32_t b[2 * kIcpTileQ];
            uint32_t off[2 * kIcpTileQ + 1];
        };
        uint4 perm[kIcpTileQ];  // a batch of rows (b0, n0, b1, n1), re-ordered nearest-first
    };
};
// the transform history of up to 64 passes (64 x 16 floats) is staged in x, y, z, id before the first round
static_assert(4 * kTileCh >= 64 * 16, "TileLds: the staging area must hold the LDS transform history");

// squared gap between the closed intervals [lo, hi] and [a, b]
__device__ __forceinline__ float interval_gap(float lo, float hi, float a, float b) {
    const float gap = fmaxf(fmaxf(lo - b, a - hi), 0.f);
    return gap * gap;
}

// Every lane contributes two point ranges [b0, b0+n0), [b1, b1+n1); the concatenation is
// streamed through LDS in kTileCh chunks, wave w of the tile's NW
// taking chunks w, w + NW, ...; every active lane keeps the minimum
// (d2, id) key over the chunks its wave saw (merged across waves by the caller).
//
// Staging filter: a candidate whose squared distance to the tile's query box Q exceeds
// every active lane's current best cannot win for any lane (each query lies in Q), so
// it is dropped before the all-lanes test and the survivors are compacted into LDS.
// The bound is the wave's own maximum best, refreshed per chunk (each wave's lanes
// keep the best over the chunks that wave saw, which is all the filter needs); the
// margin (1 - 1e-5) covers the float rounding of both the box gap and d2.
template <int NW>  // waves per tile: the tile's candidate stream is split over them
__device__ __forceinline__ void scan_ranges(const GridDev& g, TileLds& L, uint32_t b0, uint32_t n0, uint32_t b1,
                                            uint32_t n1, bool act, float x, float y, float z, const float (&qb)[6],
                                            uint64_t& best, unsigned long long& cand, uint32_t& tested) {
    // the wave's index within its tile (several one-wave tiles per block: always 0)
    const int lane = threadIdx.x & 63, w = NW > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    const uint32_t n = n0 + n1;
    const uint32_t incl = wave_incl_scan_dpp(n);
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (T == 0) return;  // wave-uniform
    if (w == 0) cand += T;
    wave_sync();  // previous readers of the slot table are done
    L.b[2 * lane] = b0;
    L.b[2 * lane + 1] = b1;
    L.off[2 * lane] = incl - n;
    L.off[2 * lane + 1] = incl - n1;
    if (lane == 63) L.off[2 * kIcpTileQ] = T;
    wave_sync();
    int sl = 0;
    uint32_t lo = 0, hi = L.off[1], sb = L.b[0];
#pragma unroll 1
    for (uint32_t base = (uint32_t)w * kTileCh; base < T; base += NW * kTileCh) {
        constexpr int U = kTileCh / kIcpTileQ;
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // slot walk first (clamped to the last point), U loads in flight
            const uint32_t t = min(base + (uint32_t)(u * kIcpTileQ + lane), T - 1);
            while (t >= hi) {
                ++sl;
                lo = hi;
                hi = L.off[sl + 1];
                sb = L.b[sl];
            }
            v[u] = g.pts[sb + (t - lo)];
        }
        // the wave's bound: its active lanes' largest best (+inf while one has none)
        const float Bw = wave_max_nonneg(act ? __uint_as_float((uint32_t)(best >> 32)) : 0.f);
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {  // survivors compacted in stream order
            const float gx = fmaxf(fmaxf(qb[0] - v[u].x, v[u].x - qb[1]), 0.f);
            const float gy = fmaxf(fmaxf(qb[2] - v[u].y, v[u].y - qb[3]), 0.f);
            const float gz = fmaxf(fmaxf(qb[4] - v[u].z, v[u].z - qb[5]), 0.f);
            const float gap2 = (gx * gx + gy * gy) + gz * gz;
            const bool in = base + (uint32_t)(u * kIcpTileQ + lane) < T && !(gap2 * (1.f - 1e-5f) > Bw);
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
        const int cnt8 = ((int)cnt + 7) & ~7;
        tested += cnt;
        if ((uint32_t)lane < (uint32_t)cnt8 - cnt) {  // pad to 8: +inf points with id kNone (never win)
            L.x[cnt + lane] = INFINITY;
            L.y[cnt + lane] = INFINITY;
            L.z[cnt + lane] = INFINITY;
            L.id[cnt + lane] = (uint32_t)kNone;
        }
        wave_sync();
        // every lane (active or not: uniform control flow) tests 4 staged candidates per step,
        // distances two at a time in packed FP32 ((dx*dx + dy*dy) + dz*dz per element, no FMA)
        const f2v qx = {x, x}, qy = {y, y}, qz = {z, z};
        double bk = __longlong_as_double((long long)best);
        // four staged candidates -> the minimum of their (d2, id) keys
        auto step4 = [&](int j) {
            const float4 X = *reinterpret_cast<const float4*>(__builtin_assume_aligned(&L.x[j], 16));
            const float4 Y = *reinterpret_cast<const float4*>(__builtin_assume_aligned(&L.y[j], 16));
            const float4 Z = *reinterpret_cast<const float4*>(__builtin_assume_aligned(&L.z[j], 16));
            const uint4 I = *reinterpret_cast<const uint4*>(__builtin_assume_aligned(&L.id[j], 16));
            const f2v dx0 = qx - f2v{X.x, X.y}, dy0 = qy - f2v{Y.x, Y.y}, dz0 = qz - f2v{Z.x, Z.y};
            const f2v dx1 = qx - f2v{X.z, X.w}, dy1 = qy - f2v{Y.z, Y.w}, dz1 = qz - f2v{Z.z, Z.w};
            const f2v d0 = (dx0 * dx0 + dy0 * dy0) + dz0 * dz0;
            const f2v d1 = (dx1 * dx1 + dy1 * dy1) + dz1 * dz1;
            const double m0 = key_min_d(key_pk<0>(I.x, I.y, d0), key_pk<1>(I.x, I.y, d0));
            const double m1 = key_min_d(key_pk<0>(I.z, I.w, d1), key_pk<1>(I.z, I.w, d1));
            return key_min_d(m0, m1);
        };
#pragma unroll 1
        for (int j = 0; j < cnt8; j += 8) {  // two steps per trip: 8 LDS reads in flight
            const double ma = step4(j), mb = step4(j + 4);
            bk = key_min_d(bk, key_min_d(ma, mb));
        }
        best = (uint64_t)__double_as_longlong(bk);
        wave_sync();  // chunk consumed before it is overwritten
    }
}

struct CellBox {
    int x0, x1, y0, y1, z0, z1;  // empty when x0 > x1
};

// Scan the rows (y, z) of box N, minus the cells of box S (already scanned;
// S inside N or empty).  With a finite bound B, rows whose (y, z) gap to the
// tile box exceeds sqrt(B) are skipped and each row's x-range is trimmed to
// [qx0 - r, qx1 + r], r = sqrt(B - gap^2) (conservatively rounded).
// Row r of box N (y fastest) minus the cells of box S: its point ranges [b0, b0+n0), [b1, b1+n1) and the
// squared (y, z) gap g2 of the row to the tile box qb
// z slice j of [lo, hi] taken centre-out from c: c, c + 1, c - 1, c + 2, ... then the longer side's rest
__device__ __forceinline__ int center_out(int j, int lo, int hi, int c) {
    const int up = hi - c, dn = c - lo, m = min(up, dn);
    if (j <= 2 * m) return j == 0 ? c : ((j & 1) ? c + (j + 1) / 2 : c - j / 2);
    const int rest = j - 2 * m;
    return up > dn ? c + m + rest : c - m - rest;
}

__device__ __forceinline__ void row_pieces(const GridDev& g, const CellBox& N, const CellBox& S, float B,
                                           const float (&qb)[6], int r, int zc, int yc, uint32_t& b0, uint32_t& n0,
                                           uint32_t& b1, uint32_t& n1, float& g2) {
    const float cs = g.cell, m = g.margin;
    const int ny = N.y1 - N.y0 + 1;
    const bool sempty = S.x0 > S.x1;
    const uint32_t gnx = (uint32_t)g.nx, gnxy = (uint32_t)g.nx * (uint32_t)g.ny;
    // z slices nearest the tile first (its rows' batches come first, so the bests fall before the far slices)
    const int rz = center_out(r / ny, N.z0, N.z1, zc);
    const int ry = center_out(r % ny, N.y0, N.y1, yc);
    int x0 = N.x0, x1 = N.x1;
    bool keep = true;
    const float yl = g.oy + (float)ry * cs - m, zl = g.oz + (float)rz * cs - m;
    g2 = interval_gap(yl, yl + cs + 2.f * m, qb[2], qb[3]) + interval_gap(zl, zl + cs + 2.f * m, qb[4], qb[5]);
    if (B < INFINITY) {
        if (g2 * 0.999999f > B) {
            keep = false;
        } else {
            const float rx = sqrtf(fmaxf(B - g2 * 0.999999f, 0.f)) * 1.00001f + m;
            x0 = max(x0, cell_coord(qb[0] - rx, g.ox, g.inv_cell));
            x1 = min(x1, cell_coord(qb[1] + rx, g.ox, g.inv_cell));
        }
    }
    if (keep && x0 <= x1) {
        const uint32_t rowc = (uint32_t)rz * gnxy + (uint32_t)ry * gnx;
        const bool inS = !sempty && ry >= S.y0 && ry <= S.y1 && rz >= S.z0 && rz <= S.z1;
        // piece left of S (or the whole row), piece right of S
        const int lx1 = inS ? min(x1, S.x0 - 1) : x1;
        if (x0 <= lx1) {
            b0 = g.start[rowc + (uint32_t)x0];
            n0 = g.start[rowc + (uint32_t)lx1 + 1] - b0;
        }
        const int rx0 = max(x0, S.x1 + 1);
        if (inS && rx0 <= x1) {
            b1 = g.start[rowc + (uint32_t)rx0];
            n1 = g.start[rowc + (uint32_t)x1 + 1] - b1;
        }
    }
}

template <int NW>
__device__ void scan_rows(const GridDev& g, TileLds& L, const CellBox& N, const CellBox& S, float B, float qx0, float qx1,
                          float qy0, float qy1, float qz0, float qz1, bool act, float x, float y, float z,
                          uint64_t& best, unsigned long long& cand, uint32_t& tested) {
    const int lane = threadIdx.x & 63;
    const float cs = g.cell;
    const float qb[6] = {qx0, qx1, qy0, qy1, qz0, qz1};
    const int nrows = (N.y1 - N.y0 + 1) * (N.z1 - N.z0 + 1);
    const int zc = min(max((cell_coord(qz0, g.oz, g.inv_cell) + cell_coord(qz1, g.oz, g.inv_cell)) / 2, N.z0), N.z1);
    const int yc = min(max((cell_coord(qy0, g.oy, g.inv_cell) + cell_coord(qy1, g.oy, g.inv_cell)) / 2, N.y0), N.y1);
#pragma unroll 1
    for (int rb = 0; rb < nrows; rb += kIcpTileQ) {
        const int r = rb + lane;
        uint32_t b0 = 0, n0 = 0, b1 = 0, n1 = 0;
        float g2 = INFINITY;
        // the bound as it stands now: every active lane's best (+inf while one has none) only falls, so a row
        // farther than all of them cannot improve any lane, in this round or in the final sphere that follows
        const float Bb = fminf(B, wave_max_nonneg(act ? __uint_as_float((uint32_t)(best >> 32)) : 0.f));
        if (r < nrows) row_pieces(g, N, S, Bb, qb, r, zc, yc, b0, n0, b1, n1, g2);
        // nearest rows first (stable partition by the row's (y, z) gap to the tile box: 0, <= 1,
        // <= 2 cells, farther), so the staging filter's bound tightens early in the stream; any
        // order gives the same minima (total order on (d2, id))
        const float c2 = cs * cs;
        const int cls = g2 == 0.f ? 0 : (g2 <= c2 ? 1 : (g2 <= 4.f * c2 ? 2 : 3));
        uint32_t rank = 0, before = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint64_t mk = __ballot(cls == c);
            if (cls == c) rank = before + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
            before += (uint32_t)__popcll(mk);
        }
        wave_sync();  // previous batch's reads of perm are done
        L.perm[rank] = make_uint4(b0, n0, b1, n1);
        wave_sync();
        const uint4 pr = L.perm[lane];
        scan_ranges<NW>(g, L, pr.x, pr.y, pr.z, pr.w, act, x, y, z, qb, best, cand, tested);
    }
}

// min over the tile's waves of every lane's key (all waves end with the same best)
template <int NW>
__device__ __forceinline__ uint64_t tile_min(uint64_t best, uint64_t* s_best) {
    if constexpr (NW == 1) return best;  // one wave per tile: nothing to merge
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    s_best[w * kIcpTileQ + lane] = best;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NW; ++v) {
        const uint64_t o = s_best[v * kIcpTileQ + lane];
        best = o < best ? o : best;
    }
    return best;
}

// One tile's exact 1-NN (one wave per tile: NW = 1; NW > 1 splits the tile's candidate stream over NW
// waves with block-level merges — measured no faster, profiles/r02_icp_tile_experiments.txt).
template <int NW>
__device__ __forceinline__ void icp_tile_body(const IcpArgs& a, int tix, int ntiles, TileLds& L, uint64_t* s_best) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#ifdef LIO_DIAG
    const uint64_t t_start = wall_clock64();  // per-tile timeline (diagnostics build)
#endif
    // The pass's point from the binned source point (its coordinates are the source's, w its index) and the
    // transforms applied so far: PCL transforms its cloud in place once per iteration (float, SSE order), so
    // applying the history in order gives the stored cloud's bits without gathering it by index.  The history
    // goes through LDS (its loads beside the head's own: a CU's first scalar reads would miss, the previous
    // pass wrote it); x, y, z, id of the staging area are 1024 contiguous floats, free until the first round.
    const bool lds_hist = NW == 1 && !a.fitness && a.nT > 0 && a.nT <= 64;
    float hv[16];
    if (lds_hist) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int t = r * 64 + lane;
            hv[r] = t < a.nT * 16 ? a.thist[t] : 0.f;
        }
    }
    const uint2 tl = a.tiles[tix];
    const bool act = lane < (int)tl.y;
    const float4 q = act ? a.qpts[tl.x + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int i = act ? __float_as_int(q.w) : 0;
    const float* hist = a.thist;
    if (lds_hist) {
        float* sh = reinterpret_cast<float*>(&L);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int t = r * 64 + lane;
            if (t < a.nT * 16) sh[t] = hv[r];
        }
        wave_sync();
        hist = sh;
    }
    float x = 0.f, y = 0.f, z = 0.f;
    int prior = -1;
    if (act) {
        if (a.prior) prior = a.nn_id[i];
        if (a.fitness) {  // getFitnessScore: original source * final; kept in cur for `aligned_`
            xform_pcl(a.T, q.x, q.y, q.z, x, y, z);
        } else {
            x = q.x;
            y = q.y;
            z = q.z;
            for (int k = 0; k < a.nT; ++k) {
                float ox, oy, oz;
                xform_pcl(hist + 16 * k, x, y, z, ox, oy, oz);
                x = ox;
                y = oy;
                z = oz;
            }
            if (a.apply_T) {
                float ox, oy, oz;
                xform_pcl(a.T, x, y, z, ox, oy, oz);
                x = ox;
                y = oy;
                z = oz;
            }
        }
    }
    if (lds_hist) wave_sync();  // every lane has read the history before the staging rounds overwrite it
    // this pass's T joins the history of the later passes
    if (a.apply_T && !a.fitness && tix == 0 && lane < 16) a.thist[16 * a.nT + lane] = a.T[lane];
    const GridDev& g = a.grid;
    uint64_t best = knn_key(INFINITY, kNone);
    if (prior >= 0 && prior != kNone) {  // the previous correspondence: an exact candidate
        const float4 p = a.tgt_by_id[prior];
        best = knn_key(sqdist3(x, y, z, p.x, p.y, p.z), prior);
    }
    // tile bounding box (active lanes)
    const float qx0 = wave_ext_dpp<false>(act ? x : INFINITY), qx1 = wave_ext_dpp<true>(act ? x : -INFINITY);
    const float qy0 = wave_ext_dpp<false>(act ? y : INFINITY), qy1 = wave_ext_dpp<true>(act ? y : -INFINITY);
    const float qz0 = wave_ext_dpp<false>(act ? z : INFINITY), qz1 = wave_ext_dpp<true>(act ? z : -INFINITY);
    const CellBox Q{min(max(cell_coord(qx0, g.ox, g.inv_cell), 0), g.nx - 1),
                    min(max(cell_coord(qx1, g.ox, g.inv_cell), 0), g.nx - 1),
                    min(max(cell_coord(qy0, g.oy, g.inv_cell), 0), g.ny - 1),
                    min(max(cell_coord(qy1, g.oy, g.inv_cell), 0), g.ny - 1),
                    min(max(cell_coord(qz0, g.oz, g.inv_cell), 0), g.nz - 1),
                    min(max(cell_coord(qz1, g.oz, g.inv_cell), 0), g.nz - 1)};
    unsigned long long cand = 0;  // candidates streamed (wave 0 counts the tile's)
    uint32_t tested = 0;          // candidates past the staging filter (this wave's chunks)
    int rounds = 0;
    // 1. bound: grow a box around Q until every lane holds a candidate;
    // 2. final: everything within sqrt(B) of the tile box, minus what was scanned
    CellBox S{1, 0, 1, 0, 1, 0};  // scanned so far (empty)
    int r = a.r0;
#ifdef LIO_DIAG
    unsigned long long dg_cand = 0;  // candidates streamed before the final round, final rows
    int dg_rows = 0;
#endif
    for (;;) {
        const bool grow = __any(act && (uint32_t)best == (uint32_t)kNone);  // block-uniform (lists merged)
        CellBox N;
        float B = INFINITY;
        if (grow) {
            N = CellBox{max(Q.x0 - r, 0), min(Q.x1 + r, g.nx - 1), max(Q.y0 - r, 0), min(Q.y1 + r, g.ny - 1),
                        max(Q.z0 - r, 0), min(Q.z1 + r, g.nz - 1)};
        } else {
            B = wave_max_nonneg(act ? __uint_as_float((uint32_t)(best >> 32)) : 0.f);
            const float R = sqrtf(B) * 1.00001f + g.margin;
            N = CellBox{max(cell_coord(qx0 - R, g.ox, g.inv_cell), 0), min(cell_coord(qx1 + R, g.ox, g.inv_cell), g.nx - 1),
                        max(cell_coord(qy0 - R, g.oy, g.inv_cell), 0), min(cell_coord(qy1 + R, g.oy, g.inv_cell), g.ny - 1),
                        max(cell_coord(qz0 - R, g.oz, g.inv_cell), 0), min(cell_coord(qz1 + R, g.oz, g.inv_cell), g.nz - 1)};
        }
        // the scanned box may stick out of N (a grown box): clip it, the part outside N is not needed
        CellBox Sc{max(S.x0, N.x0), min(S.x1, N.x1), max(S.y0, N.y0), min(S.y1, N.y1), max(S.z0, N.z0), min(S.z1, N.z1)};
        if (Sc.y0 > Sc.y1 || Sc.z0 > Sc.z1) Sc.x0 = 1, Sc.x1 = 0;
#ifdef LIO_DIAG
        if (!grow) {
            dg_cand = cand;
            dg_rows = (N.y1 - N.y0 + 1) * (N.z1 - N.z0 + 1);
        }
#endif
        scan_rows<NW>(g, L, N, Sc, B, qx0, qx1, qy0, qy1, qz0, qz1, act, x, y, z, best, cand, tested);
        best = tile_min<NW>(best, s_best);
        ++rounds;
        const bool full = N.x0 == 0 && N.y0 == 0 && N.z0 == 0 && N.x1 == g.nx - 1 && N.y1 == g.ny - 1 && N.z1 == g.nz - 1;
        if (!grow || full) break;  // final pass done, or the whole grid scanned
        S = N;
        // empty surroundings: the box doubles while small, then grows by one cell a round (a doubled box
        // overshoots the nearest points by up to its own size, and every point it holds is streamed)
        r = r < 3 ? 2 * r + 1 : r + 1;
    }
    // the tile's cost for the next pass's longest-first order: candidates tested over its waves
    uint32_t tile_tested = tested;
    if constexpr (NW > 1) {
        __shared__ uint32_t s_tested[NW];
        if (lane == 0) s_tested[wv] = tested;
        __syncthreads();
        tile_tested = 0;
#pragma unroll
        for (int v = 0; v < NW; ++v) tile_tested += s_tested[v];
    }
    const bool lead = NW > 1 ? threadIdx.x == 0 : lane == 0;
    if (a.tile_cost && lead) a.tile_cost[tix] = tile_tested;
    if (a.dbg && lead) {
#ifdef LIO_DIAG
        a.dbg[8 + 2 * (size_t)tix] = t_start;
        a.dbg[8 + 2 * (size_t)tix + 1] = wall_clock64();
        unsigned long long* ex = a.dbg + 8 + 2 * (size_t)ntiles + 4 * (size_t)tix;
        ex[0] = dg_cand;
        ex[1] = cand - dg_cand;
        ex[2] = (unsigned long long)dg_rows;
        ex[3] = (unsigned long long)rounds;
#endif
#ifndef LIO_DIAG_TIMELINE  // the timeline build leaves out the same-address counters (they serialise)
        atomicAdd(a.dbg, cand);
        atomicAdd(a.dbg + 1, (unsigned long long)rounds);
        atomicAdd(a.dbg + 2, 1ull);
        atomicAdd(a.dbg + 3, (unsigned long long)tl.y);
        atomicAdd(a.dbg + 4, (unsigned long long)tile_tested);
#endif
    }
    if constexpr (NW > 1) __syncthreads();  // every wave has read cur[i] before it is overwritten
    if (act && (NW == 1 || wv == 0)) {
        if (a.fitness || a.apply_T) {
            a.cur[3 * i] = x;
            a.cur[3 * i + 1] = y;
            a.cur[3 * i + 2] = z;
        }
        a.nn_d2[i] = __uint_as_float((uint32_t)(best >> 32));
        a.nn_id[i] = (int)(uint32_t)best;
    }
}


// one wave per tile, tile = its XCD's next one (icp_tile_of)
__global__ void __launch_bounds__(kIcpTileQ) icp_tile_kernel(IcpArgs a, int ntiles) {
    __shared__ TileLds L;
    const int tix = icp_tile_of(a.order, (int)blockIdx.x, ntiles);
    if (tix < 0) return;  // block-uniform: a slot past its XCD's share
    icp_tile_body<1>(a, tix, ntiles, L, nullptr);
}

// One block = one 4096-point record -> super[record][kIcpStride]: each lane
// accumulates its 4 points (record-relative index lane + 1024 k, k ascending),
// each wave sums its lanes (wave_sum32, recursive halving), and the 16 wave
// sums are added in wave order.  A fixed order for a given record, so the
// records (what ranks all-gather) are bit-identical for any number of ranks.
constexpr int kIcpStatsThreads = 1024;
template <int NT>
__device__ void icp_order_share(const uint32_t* __restrict__ cost, int n, uint32_t* __restrict__ order, int x);

// Blocks [0, nsup) write the records; when `order` is given, blocks nsup .. nsup + 7 build the next
// pass's tile order for the eight XCD shares in the same launch (they only read this pass's tile costs),
// so the order runs beside the records instead of between them and the next pass.
// exclusive prefix over the 1024 threads of the block (16 waves), total -> tot
__device__ __forceinline__ uint32_t stats_block_excl(uint32_t v, uint32_t* s_w, uint32_t& tot) {
    constexpr int NW = kIcpStatsThreads / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t off = 0, t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t c = s_w[i];
        if (i < w) off += c;
        t += c;
    }
    __syncthreads();
    tot = t;
    return off + inc - v;
}

__global__ void __launch_bounds__(kIcpStatsThreads) icp_stats_kernel(IcpArgs a, double* __restrict__ super, int nsup,
                                                                     uint32_t* __restrict__ order, int ntiles,
                                                                     IcpCompact cp) {
    if ((int)blockIdx.x >= nsup) {  // block-uniform
        icp_order_share<kIcpStatsThreads>(a.tile_cost, ntiles, order, (int)blockIdx.x - nsup);
        return;
    }
    constexpr int NW = kIcpStatsThreads / 64, PER = kIcpSuper / kIcpStatsThreads;
    __shared__ double red[NW][kIcpStride];
    __shared__ uint32_t s_rec, s_off, s_w[NW];
    // the record: this block's, or with the compaction the arrival order's (a block only waits in the look-back
    // for records whose blocks are already running)
    int rec = blockIdx.x;
    if (cp.pairs) {
        if (threadIdx.x == 0) {
            s_rec = atomicAdd(cp.ticket, 1u);
            if (s_rec == (uint32_t)nsup - 1) *cp.ticket = 0u;  // every record block has its ticket
        }
        __syncthreads();
        rec = (int)s_rec;
    }
    double v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = 0.0;
    int ids[PER];
    float d2s[PER];
    const int base = rec * kIcpSuper + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER; ++k) {  // all correspondence loads first: one round trip
        const int i = base + k * kIcpStatsThreads;
        ids[k] = i < a.n ? a.nn_id[i] : -1;
        d2s[k] = i < a.n ? a.nn_d2[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = base + k * kIcpStatsThreads, id = ids[k];
        const float d2 = d2s[k];
        if (id < 0 || id == kNone) continue;
        if (a.fitness) {
            v[0] += 1.0;
            v[16] += (double)d2;
        } else if (!((double)d2 > a.max_d2)) {
            const float4 q = a.tgt_by_id[id];
            const double p0 = (double)a.cur[3 * i] - a.c0[0], p1 = (double)a.cur[3 * i + 1] - a.c0[1],
                         p2 = (double)a.cur[3 * i + 2] - a.c0[2];
            const double q0 = (double)q.x - a.c0[0], q1 = (double)q.y - a.c0[1], q2 = (double)q.z - a.c0[2];
            v[0] += 1.0;
            v[1] += p0; v[2] += p1; v[3] += p2;
            v[4] += q0; v[5] += q1; v[6] += q2;
            v[7] += q0 * p0; v[8] += q0 * p1; v[9] += q0 * p2;
            v[10] += q1 * p0; v[11] += q1 * p1; v[12] += q1 * p2;
            v[13] += q2 * p0; v[14] += q2 * p1; v[15] += q2 * p2;
            v[16] += (double)d2;
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double t = wave_sum32(v, lane);  // recursive halving (lio_dev.hpp)
    if (lane < 32) {
        const int k = wave_sum32_index(lane);
        if (k < 17) red[wid][k] = t;
    }
    __syncthreads();
    if (threadIdx.x < kIcpStride) {
        double s = 0.0;
        if (threadIdx.x < 17)
#pragma unroll
            for (int w = 0; w < NW; ++w) s += red[w][threadIdx.x];
        super[(size_t)rec * kIcpStride + threadIdx.x] = s;
    }
    if (!cp.pairs) return;  // block-uniform
    // The accepted pairs of the record in source order (pcl_compact_kernel's result, one launch fewer): slab k
    // = points rec * 4096 + 1024 k + t; the four slabs' flags packed two to a word (counts <= 1024) for the
    // block prefix, the record's count chained over the records by the look-back.
    bool ok[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) ok[k] = ids[k] >= 0 && ids[k] != kNone && !((double)d2s[k] > a.max_d2);
    static_assert(PER == 4, "the packed slab counts assume four 1024-point slabs per record");
    uint32_t t01, t23;
    const uint32_t e01 = stats_block_excl((ok[0] ? 1u : 0u) | (ok[1] ? 1u << 16 : 0u), s_w, t01);
    const uint32_t e23 = stats_block_excl((ok[2] ? 1u : 0u) | (ok[3] ? 1u << 16 : 0u), s_w, t23);
    const uint32_t T[PER] = {t01 & 0xffffu, t01 >> 16, t23 & 0xffffu, t23 >> 16};
    const uint32_t ex[PER] = {e01 & 0xffffu, e01 >> 16, e23 & 0xffffu, e23 >> 16};
    const uint32_t R = T[0] + T[1] + T[2] + T[3];
    if (threadIdx.x < 64) {  // wave 0: publish, look back, publish the prefix
        uint32_t acc = 0;
        if (rec > 0) {
            if (threadIdx.x == 0) lb_store(cp.st, rec, lb_word(cp.epoch, 1u, R));
            uint64_t unused;
            bool timeout;
            acc = lookback_excl<false>(cp.st, nullptr, nullptr, rec, cp.epoch, unused, timeout);
            if (timeout && threadIdx.x == 0) atomicOr(cp.ticket + 1, 1u);  // flagged in pcl_pack's output
        }
        if (threadIdx.x == 0) {
            lb_store(cp.st, rec, lb_word(cp.epoch, 2u, acc + R));
            s_off = acc;
            if (rec == nsup - 1) *cp.d_n = acc + R;
        }
    }
    __syncthreads();
    uint32_t before = s_off;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (ok[k]) {
            const int i = base + k * kIcpStatsThreads;
            const uint32_t slot = before + ex[k];
            const float4 q = a.tgt_by_id[ids[k]];
            const float vv[6] = {a.cur[3 * i], a.cur[3 * i + 1], a.cur[3 * i + 2], q.x, q.y, q.z};
#pragma unroll
            for (int d = 0; d < 6; ++d) cp.pairs[d * cp.cap + slot] = vv[d];
        }
        before += T[k];
    }
}

// one wave per tile (several waves per tile, or several one-wave tiles per block, measured no faster:
// profiles/r02_icp_tile_experiments.txt); grid = 8 XCD shares of the largest size (icp_tile_of)
void launch_icp_tiles(const IcpArgs& a, int ntiles, hipStream_t st) {
    if (a.n == 0 || ntiles == 0) return;
    const int seg = (ntiles + kIcpSegs - 1) / kIcpSegs;
    icp_tile_kernel<<<8 * (kIcpSegs / 8) * seg, kIcpTileQ, 0, st>>>(a, ntiles);
}

// Tile order for the next pass from this pass's candidate counts.  The cell-ordered tiles are cut
// into kIcpSegs contiguous segments (spatially compact: their target neighbourhoods stay in one
// XCD's L2), XCD x owns segments x, x + 8, ... (a misaligned region, which is spatially concentrated,
// is shared by every XCD; contiguous cost-balanced shares measured slower, profiles/r03_icp_contig_ab.txt),
// and inside each XCD's share the tiles run longest-first (log2 buckets of the count, descending) so the
// heavy ones do not form the tail.  Layout: order[0 .. n) the eight shares one after another,
// order[n + x] the first entry of share x (order[n + 8] = n).  One block per share (the share sizes
// follow from the segment bounds, so no block waits for another), run by icp_stats_kernel's last eight
// blocks beside the records.
__device__ __forceinline__ uint32_t cost_bucket(uint32_t c) { return c ? 32u - (uint32_t)__clz(c) : 0u; }
// entry f of share x in cell order (-1 past its end)
__device__ __forceinline__ int icp_share_tile(int x, int f, int n) {
#pragma unroll
    for (int j = 0; j < kIcpSegs / 8; ++j) {
        const int b0 = icp_seg_begin(x + 8 * j, n), sz = icp_seg_begin(x + 8 * j + 1, n) - b0;
        if (f < sz) return b0 + f;
        f -= sz;
    }
    return -1;
}
template <int NT>
__device__ void icp_order_share(const uint32_t* __restrict__ cost, int n, uint32_t* __restrict__ order, int x) {
    __shared__ uint32_t hist[33], base[33];
    if (threadIdx.x < 33) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int f = (int)threadIdx.x;; f += NT) {
        const int t = icp_share_tile(x, f, n);
        if (t < 0) break;
        atomicAdd(&hist[cost_bucket(cost[t])], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;  // this share's first entry: the sizes of shares 0 .. x-1
        for (int s = 0; s < kIcpSegs; ++s)
            if ((s & 7) < x) acc += (uint32_t)(icp_seg_begin(s + 1, n) - icp_seg_begin(s, n));
        order[n + x] = acc;
        if (x == 0) order[n + 8] = (uint32_t)n;
        for (int b = 32; b >= 0; --b) {  // longest first
            base[b] = acc;
            acc += hist[b];
        }
    }
    __syncthreads();
    for (int f = (int)threadIdx.x;; f += NT) {
        const int t = icp_share_tile(x, f, n);
        if (t < 0) break;
        order[atomicAdd(&base[cost_bucket(cost[t])], 1u)] = (uint32_t)t;
    }
}

// Tiles in Morton order of their cells (z, y, x bits interleaved): the kIcpSegs contiguous segments a pass
// deals to the XCDs are then compact 3-D blobs of the cloud instead of thin slabs of the x-fastest cell order
// (2 m tile cells: a slab one or two cells thick, whose target neighbourhood is mostly halo shared with the
// slabs on other XCDs — each XCD's L2 then fetched the same target rows).  Perf only: every 1-NN is exact in
// any tile order.  Grids wider than 1024 cells on an axis keep the cell order.
__device__ __forceinline__ uint32_t spread3_10(uint32_t v) {  // bits 0..9 -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
__global__ void tile_key_kernel(const uint32_t* __restrict__ start, GridGeom gm, int morton, uint32_t* __restrict__ key,
                                uint32_t* __restrict__ cell) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c >= gm.ncells) return;
    uint32_t k = 0xffffffffu;  // empty cells sort last (and carry no tiles)
    if (start[c + 1] > start[c]) {
        if (morton) {
            const uint32_t x = c % (uint32_t)gm.nx, yz = c / (uint32_t)gm.nx;
            const uint32_t y = yz % (uint32_t)gm.ny, z = yz / (uint32_t)gm.ny;
            k = (spread3_10(z) << 2) | (spread3_10(y) << 1) | spread3_10(x);
        } else {
            k = c;
        }
    }
    key[c] = k;
    cell[c] = c;
}
// per sorted cell: number of tiles (ceil(count / 64)); slot ncells = 0 for the scan's total
__global__ void tile_count_kernel(const uint32_t* __restrict__ start, uint32_t ncells, const uint32_t* __restrict__ cell,
                                  uint32_t* __restrict__ tcount) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i > ncells) return;
    uint32_t t = 0;
    if (i < ncells) {
        const uint32_t c = cell[i];
        t = (start[c + 1] - start[c] + kIcpTileQ - 1) / kIcpTileQ;
    }
    tcount[i] = t;
}
__global__ void tile_write_kernel(const uint32_t* __restrict__ start, uint32_t ncells, const uint32_t* __restrict__ cell,
                                  const uint32_t* __restrict__ toff, uint2* __restrict__ tiles) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= ncells) return;
    const uint32_t c = cell[i];
    const uint32_t b = start[c], n = start[c + 1] - b, nt = toff[i + 1] - toff[i];
    for (uint32_t t = 0; t < nt; ++t) {  // balanced split of the cell's points
        const uint32_t s0 = (uint32_t)((uint64_t)n * t / nt), s1 = (uint32_t)((uint64_t)n * (t + 1) / nt);
        tiles[toff[i] + t] = make_uint2(b + s0, s1 - s0);
    }
}

int icp_build_tiles(const GridBuf& q, uint2* tiles, uint32_t* scratch, void*& tmp, size_t& tmp_bytes, hipStream_t st) {
    const uint32_t nc = q.geom.ncells;
    uint32_t* tcount = scratch;             // nc + 1
    uint32_t* toff = tcount + nc + 1;       // nc + 1
    uint32_t* key = toff + nc + 1;          // nc
    uint32_t* key2 = key + nc;              // nc
    uint32_t* cell = key2 + nc;             // nc
    uint32_t* cell2 = cell + nc;            // nc
    const int nb = (int)((nc + 1 + 255) / 256);
    const int morton = q.geom.nx <= 1024 && q.geom.ny <= 1024 && q.geom.nz <= 1024 ? 1 : 0;
    tile_key_kernel<<<nb, 256, 0, st>>>(q.start, q.geom, morton, key, cell);
    size_t need_scan = 0, need_sort = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, need_scan, tcount, toff, (int)(nc + 1), st) != hipSuccess ||
        hipcub::DeviceRadixSort::SortPairs(nullptr, need_sort, key, key2, cell, cell2, (int)nc, 0, 32, st) != hipSuccess)
        return -1;
    const size_t need = std::max(need_scan, need_sort);
    if (need > tmp_bytes) {
        if (tmp) (void)hipFree(tmp);
        tmp = nullptr;
        tmp_bytes = 0;
        const size_t c = std::max(need + need / 2, 2 * tmp_bytes);  // geometric: the next source rarely needs more
        count_alloc();
        if (hipMalloc(&tmp, c) != hipSuccess) return -5;
        tmp_bytes = c;
    }
    size_t tb = tmp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, cell, cell2, (int)nc, 0, 32, st) != hipSuccess) return -1;
    tile_count_kernel<<<nb, 256, 0, st>>>(q.start, nc, cell2, tcount);
    tb = tmp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(tmp, tb, tcount, toff, (int)(nc + 1), st) != hipSuccess) return -1;
    tile_write_kernel<<<nb, 256, 0, st>>>(q.start, nc, cell2, toff, tiles);
    uint32_t total = 0;
    if (hipMemcpyAsync(&total, toff + nc, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess)
        return -1;
    return (int)total;
}

// ----------------------------------------------------------------------------
// PCL-order fidelity mode (lio_icp_params.umeyama_float): the float statistics of
// pcl::umeyama(cloud_src, cloud_tgt, false) as TransformationEstimationSVD<PointXYZI,
// PointXYZI, float> builds them [U] (common/impl/eigen.hpp, a copy of Eigen 3.3's
// Umeyama.h): the accepted correspondences in source order,
//   src_mean = src.rowwise().sum() * one_over_n   (a sequential float sum per row,
//              starting from the first element: Eigen's redux over a strided row)
//   sigma    = one_over_n * dst_demean * src_demean^T  (the depth sum sequential)
// A float sum's value depends on its order, so each of the 6 + 9 chains runs on ONE
// lane, in order; the block stages the correspondences through LDS around it.
// The serial fallback of the parallel seqsum path (lio_seqsum.hip); sharded, it runs on every rank over
// the gathered pairs of all ranks.  icp_pcl_means_kernel also writes the compacted pairs (src xyz,
// tgt xyz) for icp_pcl_sigma_kernel.
// ----------------------------------------------------------------------------
constexpr int kPclThreads = 1024;  // one block: a chunk of 1024 correspondences per round

// block-exclusive prefix count of `flag` (1024 threads): returns this thread's slot, *total = chunk count
__device__ __forceinline__ uint32_t block_compact_slot(bool flag, uint32_t* s_w, uint32_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t m = __ballot(flag);
    const uint32_t in_wave = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kPclThreads / 64; ++k) {
        const uint32_t c = s_w[k];
        before += k < w ? c : 0u;
        tot += c;
    }
    total = tot;
    return before + in_wave;
}

// one lane adds col[0 .. cnt) to acc in order (loads 8 ahead; the adds stay one dependent chain)
__device__ __forceinline__ void serial_add(const float* col, uint32_t cnt, float& acc, bool& first) {
    uint32_t k = 0;
    if (first && cnt > 0) {  // Eigen's redux starts from the first coefficient
        acc = col[0];
        first = false;
        k = 1;
    }
    for (; k + 8 <= cnt; k += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = col[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; k < cnt; ++k) acc += col[k];
}

// out[0..5] = float sums (src x y z, tgt x y z), out[6] = count (uint32 bits); pairs: n x 6 compacted
__global__ void __launch_bounds__(kPclThreads) icp_pcl_means_kernel(IcpArgs a, float* __restrict__ pairs, int64_t cap,
                                                                    float* __restrict__ out) {
    __shared__ float s[6][kPclThreads];
    __shared__ uint32_t s_w[kPclThreads / 64];
    float acc = 0.f;
    bool first = true;
    uint32_t done = 0;
    for (int base = 0; base < a.n; base += kPclThreads) {
        const int i = base + (int)threadIdx.x;
        bool ok = false;
        float v[6];
        if (i < a.n) {
            const int id = a.nn_id[i];
            const float d2 = a.nn_d2 ? a.nn_d2[i] : 0.f;  // no d2: the ids were gated already (-1 = rejected)
            ok = id >= 0 && id != kNone && !((double)d2 > a.max_d2);
            if (ok) {
                const float4 q = a.tgt_by_id[id];
                v[0] = a.cur[3 * i], v[1] = a.cur[3 * i + 1], v[2] = a.cur[3 * i + 2];
                v[3] = q.x, v[4] = q.y, v[5] = q.z;
            }
        }
        uint32_t cnt;
        const uint32_t slot = block_compact_slot(ok, s_w, cnt);
        if (ok) {
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                s[d][slot] = v[d];
                pairs[d * cap + (int64_t)(done + slot)] = v[d];  // column-major (PclBuf::pairs)
            }
        }
        __syncthreads();
        if (threadIdx.x < 6) serial_add(s[threadIdx.x], cnt, acc, first);
        done += cnt;
        __syncthreads();  // the chunk is consumed before the next overwrites it (and s_w is reused)
    }
    if (threadIdx.x < 6) out[threadIdx.x] = acc;
    if (threadIdx.x == 0) out[6] = __uint_as_float(done);
}

// sums / count from icp_pcl_means_kernel -> out[7 + 3 r + c] = sum_k (tgt_r - dm_r) (src_c - sm_c), in order
__global__ void __launch_bounds__(kPclThreads) icp_pcl_sigma_kernel(const float* __restrict__ pairs, int64_t cap,
                                                                    float* __restrict__ out) {
    __shared__ float s[6][kPclThreads];
    const uint32_t n = __float_as_uint(out[6]);
    const float one_over_n = 1.f / (float)n;
    // lane t < 9: row r (target), column c (source) of the row-major accumulator
    const int r = (int)threadIdx.x / 3, c = (int)threadIdx.x % 3;
    float dm = 0.f, sm = 0.f, acc = 0.f;
    if (threadIdx.x < 9) {
        dm = out[3 + r] * one_over_n;
        sm = out[c] * one_over_n;
    }
    for (uint32_t base = 0; base < n; base += kPclThreads) {
        const uint32_t cnt = min((uint32_t)kPclThreads, n - base);
#pragma unroll
        for (int d = 0; d < 6; ++d)  // coalesced: column-major in memory
            for (uint32_t k = threadIdx.x; k < cnt; k += kPclThreads) s[d][k] = pairs[d * cap + (int64_t)(base + k)];
        __syncthreads();
        if (threadIdx.x < 9) {
            const float* dst = s[3 + r];
            const float* src = s[c];
            uint32_t k = 0;
            for (; k + 8 <= cnt; k += 8) {
                float pr[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float dv = dst[k + u] - dm, sv = src[k + u] - sm;
                    pr[u] = dv * sv;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += pr[u];
            }
            for (; k < cnt; ++k) {
                const float dv = dst[k] - dm, sv = src[k] - sm;
                acc += dv * sv;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 9) out[7 + threadIdx.x] = acc;
}

void launch_icp_pcl_stats(const IcpArgs& a, float* pairs, int64_t cap, float* out16, hipStream_t st) {
    icp_pcl_means_kernel<<<1, kPclThreads, 0, st>>>(a, pairs, cap, out16);
    icp_pcl_sigma_kernel<<<1, kPclThreads, 0, st>>>(pairs, cap, out16);
}

void launch_icp_pcl_means_serial(const IcpArgs& a, float* pairs, int64_t cap, float* out16, hipStream_t st) {
    icp_pcl_means_kernel<<<1, kPclThreads, 0, st>>>(a, pairs, cap, out16);
}

// the serial means of pairs compacted already (the sharded fallback's gathered pairs): lanes 0 .. 5 each add
// their column in order (staged through LDS a chunk at a time), out[6] = the count
__global__ void __launch_bounds__(kPclThreads) icp_pcl_means_pairs_kernel(const float* __restrict__ pairs, int64_t cap,
                                                                          const uint32_t* __restrict__ d_n,
                                                                          float* __restrict__ out) {
    __shared__ float s[6][kPclThreads];
    const uint32_t n = *d_n;
    float acc = 0.f;
    bool first = true;
    for (uint32_t base = 0; base < n; base += kPclThreads) {
        const uint32_t cnt = min((uint32_t)kPclThreads, n - base);
#pragma unroll
        for (int d = 0; d < 6; ++d)
            if (threadIdx.x < cnt) s[d][threadIdx.x] = pairs[d * cap + (int64_t)(base + threadIdx.x)];
        __syncthreads();
        if (threadIdx.x < 6) serial_add(s[threadIdx.x], cnt, acc, first);
        __syncthreads();
    }
    if (threadIdx.x < 6) out[threadIdx.x] = acc;
    if (threadIdx.x == 0) out[6] = __uint_as_float(n);
}

void launch_icp_pcl_means_pairs(const float* pairs, int64_t cap, const uint32_t* d_n, float* out16, hipStream_t st) {
    icp_pcl_means_pairs_kernel<<<1, kPclThreads, 0, st>>>(pairs, cap, d_n, out16);
}

void launch_icp_pcl_sigma_serial(const float* pairs, int64_t cap, float* out16, hipStream_t st) {
    icp_pcl_sigma_kernel<<<1, kPclThreads, 0, st>>>(pairs, cap, out16);
}

// the records of every rank summed in global record order, one lane per statistic (lio_icp_combine's order):
// the records go through LDS in chunks, loaded by all lanes, so the 17 dependent chains read LDS, not HBM
constexpr int kCombChunk = 256;
__global__ void __launch_bounds__(256) icp_combine_kernel(const double* __restrict__ recv, int64_t nsup, int world,
                                                         int64_t rank_stride, double* __restrict__ out17) {
    __shared__ double s_rec[kCombChunk][17];
    const int k = threadIdx.x;
    double acc = 0.0;
    for (int64_t g0 = 0; g0 < nsup; g0 += kCombChunk) {
        const int m = (int)min((int64_t)kCombChunk, nsup - g0);
        for (int e = threadIdx.x; e < m * 17; e += 256) {
            const int64_t s = g0 + e / 17;
            // the rank holding record s (records split as nsup * r / world) and its slot in that rank's message
            int r = (int)(s * world / nsup);
            while (r + 1 < world && nsup * (r + 1) / world <= s) ++r;
            while (r > 0 && nsup * r / world > s) --r;
            const int64_t s0 = nsup * r / world;
            s_rec[e / 17][e % 17] = recv[(size_t)r * rank_stride + (size_t)(s - s0) * kIcpStride + e % 17];
        }
        __syncthreads();
        if (k < 17)
            for (int j = 0; j < m; ++j) acc += s_rec[j][k];
        __syncthreads();
    }
    if (k < 17) out17[k] = acc;
}

void launch_icp_combine(const double* recv, int64_t nsup, int world, int64_t rank_stride, double* out17, hipStream_t st) {
    icp_combine_kernel<<<1, 256, 0, st>>>(recv, nsup, world, rank_stride, out17);
}

void launch_icp_stats(const IcpArgs& a, double* super, hipStream_t st, uint32_t* order, int ntiles, const IcpCompact* cp) {
    if (a.n == 0) {
        if (cp && cp->d_n) (void)hipMemsetAsync(cp->d_n, 0, sizeof(uint32_t), st);  // no pairs
        return;
    }
    const int nsup = (a.n + kIcpSuper - 1) / kIcpSuper;
    const bool ord = order && ntiles > 0;
    icp_stats_kernel<<<nsup + (ord ? 8 : 0), kIcpStatsThreads, 0, st>>>(a, super, nsup, ord ? order : nullptr, ntiles,
                                                                         cp ? *cp : IcpCompact{});
}

}  // namespace lio
