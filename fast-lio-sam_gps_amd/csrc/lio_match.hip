// lio_match.hip — FAST-LIO h_share_model on gfx950.
//
// Two fused kernels per h-evaluation:
//
//   h_model_knn_kernel  (ekfom_data.converge == true), 512 threads = 64 points
//     phase 1 (8 lanes per point): body->world (double, stored float) -> exact
//       grid 5-NN, cell points scanned lane-strided (coalesced), private
//       top-5 lists merged by a shuffle butterfly
//     phase 2 (wave 0, lane = point): gate (found == 5 && d2[4] <= 5) ->
//       esti_plane (QR, registers) -> pd2, s-gate -> H row (double) ->
//       30-value wave reduction -> block partial
//     writes: nn_idx[5] (20 B), plane abcd (16 B), sel (1 B)
//   h_model_reuse_kernel (converge == false: reuse Nearest_Points), lane = point
//     body->world -> cached plane -> pd2, s-gate -> H row -> block partial
//   finalize_kernel: sums the block partials in a fixed order (deterministic)
//
// The per-point dense H (effct x 12 doubles) of the reference is never
// materialised: the IESKF only consumes H^T H and H^T h.
#include "lio_dev.hpp"
#include "lio_kernels.hpp"

#include <algorithm>

namespace lio {

constexpr int kBlock = 256;
constexpr int kNSum = 30;  // 21 HTH + 6 HTh + neff + res + hh (reduced in wave_reduce_store)
constexpr int kGroup = 8;   // lanes cooperating on one query's kNN
constexpr int kKnnBlock = 512;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Block reduction of one lane's contribution [HTH(21), HTh(6), cnt, res, hh]
// over the wave, lane 0 stores the wave's 30 partial sums to `dst`.
// Products are formed and reduced a few at a time so the 30 sums never need
// 60 live VGPRs (the kernel's occupancy is set by its peak register count).
__device__ __forceinline__ void wave_reduce_store(const double J[6], double h, double res, double cnt, double* dst) {
    const bool l0 = (threadIdx.x & 63) == 0;
    int q = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
        for (int c = r; c < 6; ++c) {
            const double v = wave_sum(J[r] * J[c]);
            if (l0) dst[q] = v;
            ++q;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const double v = wave_sum(J[r] * h);
        if (l0) dst[21 + r] = v;
    }
    __builtin_amdgcn_sched_barrier(0);
    const double s0 = wave_sum(cnt), s1 = wave_sum(res), s2 = wave_sum(h * h);
    if (l0) {
        dst[27] = s0;
        dst[28] = s1;
        dst[29] = s2;
        dst[30] = 0.0;
        dst[31] = 0.0;
    }
}

// pd2 / s-gate / H row of one selected point (h_share_model [U])
__device__ __forceinline__ bool residual_row(const MatchArgs& a, float bx, float by, float bz, float wx, float wy,
                                             float wz, const float4& pl, double J[6], double& h, double& res) {
    const float pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
    const double b0 = bx, b1 = by, b2 = bz;
    const double pn = sqrt((b0 * b0 + b1 * b1) + b2 * b2);
    const float s = (float)(1.0 - a.s_coef * (double)fabsf(pd2) / sqrt(pn));
    if (!((double)s > a.s_gate)) return false;
    h_row(a.pose, bx, by, bz, pl.x, pl.y, pl.z, J);
    h = -(double)pd2;
    res = (double)fabsf(pd2);
    return true;
}

// ekfom_data.converge == true: kNN + plane + H.  512 threads = 64 queries.
//   phase 1: 8 lanes per query run the exact grid 5-NN cooperatively
//   phase 2: wave 0, one lane per query: gate, esti_plane, s-gate, H row,
//            wave reduction -> block partial
template <bool DBG>
__global__ void __launch_bounds__(kKnnBlock) h_model_knn_kernel(MatchArgs a) {
    constexpr int QPB = kKnnBlock / kGroup;  // 64 queries per block
    __shared__ int s_id[QPB][5];
    __shared__ float s_w[QPB][3];
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int qloc = threadIdx.x / kGroup;
    const int sub = threadIdx.x % kGroup;
    const int i = blk * QPB + qloc;
    if (i < a.n) {
        const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
        float wx, wy, wz;
        body_to_world(a.pose, bx, by, bz, wx, wy, wz);
        TopK<5> tk;
        tk.init(a.range_sq);
        SearchStats st{0, 0, 0};
        group_knn_split<5, kGroup>(a.grid, wx, wy, wz, a.max_shell, sub, tk, DBG ? &st : nullptr);
        if constexpr (DBG) {
#pragma unroll
            for (int off = 1; off < kGroup; off <<= 1) {
                st.cells += __shfl_xor(st.cells, off, 64);
                st.points += __shfl_xor(st.points, off, 64);
            }
            if (sub == 0) {
                a.dbg[3 * (size_t)i] = st.cells;
                a.dbg[3 * (size_t)i + 1] = st.points;
                a.dbg[3 * (size_t)i + 2] = st.shell;
            }
        }
        if (sub < 5) {
            int v = tk.id[0];
#pragma unroll
            for (int j = 1; j < 5; ++j)
                if (sub == j) v = tk.id[j];
            s_id[qloc][sub] = v;
            a.nn_idx[5 * (size_t)i + sub] = v == kNone ? -1 : v;
        }
        if (sub == 0) {
            s_w[qloc][0] = wx;
            s_w[qloc][1] = wy;
            s_w[qloc][2] = wz;
        }
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;
    // ---- phase 2: lane = query
    const int lane = threadIdx.x;
    const int ip = blk * QPB + lane;
    double J[6] = {0, 0, 0, 0, 0, 0};
    double h = 0.0, res = 0.0, cnt = 0.0;
    if (ip < a.n) {
        // point_selected_surf = found == 5 && !(sqdist[4] > 5)   (d <= range by construction)
        bool sel = s_id[lane][4] != kNone;
        if (sel) {
            float P[5][3];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float4 q = a.map_by_id[s_id[lane][j]];
                P[j][0] = q.x;
                P[j][1] = q.y;
                P[j][2] = q.z;
            }
            float abcd[4];
            sel = esti_plane_dev(P, a.plane_thr, abcd);
            const float4 pl = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
            a.planes[ip] = pl;
            if (sel) {
                sel = residual_row(a, a.body[3 * ip], a.body[3 * ip + 1], a.body[3 * ip + 2], s_w[lane][0],
                                   s_w[lane][1], s_w[lane][2], pl, J, h, res);
                cnt = sel ? 1.0 : 0.0;
            }
        }
        a.sel[ip] = sel ? 1 : 0;
    }
    wave_reduce_store(J, h, res, cnt, a.partials + (size_t)blk * 32);
}

// ekfom_data.converge == true, one lane per point (kNN with deep memory-level
// parallelism, see lane_knn_exact), plane + H in the same lane, 4 wave
// partials combined in LDS.  256 threads = 256 points.
__global__ void __launch_bounds__(kBlock) h_model_knn_lane_kernel(MatchArgs a) {
    __shared__ double red[kBlock / 64][32];
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int i = blk * kBlock + threadIdx.x;
    double J[6] = {0, 0, 0, 0, 0, 0};
    double h = 0.0, res = 0.0, cnt = 0.0;
    if (i < a.n) {
        const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
        float wx, wy, wz;
        body_to_world(a.pose, bx, by, bz, wx, wy, wz);
        TopK<5> tk;
        tk.init(a.range_sq);
        lane_knn_exact<5>(a.grid, wx, wy, wz, a.max_shell, tk);
        int32_t* o = a.nn_idx + 5 * (size_t)i;
#pragma unroll
        for (int j = 0; j < 5; ++j) o[j] = tk.id[j] == kNone ? -1 : tk.id[j];
        bool sel = tk.id[4] != kNone;  // found == 5 && d2[4] <= range (by construction)
        if (sel) {
            float P[5][3];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float4 q = a.map_by_id[tk.id[j]];
                P[j][0] = q.x;
                P[j][1] = q.y;
                P[j][2] = q.z;
            }
            float abcd[4];
            sel = esti_plane_dev(P, a.plane_thr, abcd);
            const float4 pl = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
            a.planes[i] = pl;
            if (sel) {
                sel = residual_row(a, bx, by, bz, wx, wy, wz, pl, J, h, res);
                cnt = sel ? 1.0 : 0.0;
            }
        }
        a.sel[i] = sel ? 1 : 0;
    }
    const int wid = threadIdx.x >> 6;
    wave_reduce_store(J, h, res, cnt, red[wid]);
    __syncthreads();
    if (threadIdx.x < 32) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
        a.partials[(size_t)blk * 32 + threadIdx.x] = s;
    }
}

// ekfom_data.converge == false: reuse Nearest_Points / planes.  256 threads,
// one point per lane, 4 wave partials combined in LDS.
__global__ void __launch_bounds__(kBlock) h_model_reuse_kernel(MatchArgs a) {
    __shared__ double red[kBlock / 64][32];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double J[6] = {0, 0, 0, 0, 0, 0};
    double h = 0.0, res = 0.0, cnt = 0.0;
    if (i < a.n) {
        bool sel = a.sel[i] != 0;
        if (sel) {
            const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
            float wx, wy, wz;
            body_to_world(a.pose, bx, by, bz, wx, wy, wz);
            sel = residual_row(a, bx, by, bz, wx, wy, wz, a.planes[i], J, h, res);
            cnt = sel ? 1.0 : 0.0;
            a.sel[i] = sel ? 1 : 0;
        }
    }
    const int wid = threadIdx.x >> 6;
    wave_reduce_store(J, h, res, cnt, red[wid]);
    __syncthreads();
    if (threadIdx.x < 32) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
        a.partials[(size_t)blockIdx.x * 32 + threadIdx.x] = s;
    }
}

// Fixed-order sum of nblocks x 32 partials -> out[32] (one block of 1024).
// 32 row groups x 32 columns; each thread issues its rows' loads 8 at a time
// (independent, so the latency overlaps) and adds them in row order; the 32
// group sums are then added in group order: deterministic for a given nblocks.
__global__ void __launch_bounds__(1024) finalize_kernel(const double* __restrict__ partials, int nblocks,
                                                       double* __restrict__ out) {
    __shared__ double sg[32][33];
    const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
    const int per = (nblocks + 31) / 32;
    const int b0 = grp * per, b1 = min(nblocks, b0 + per);
    double s = 0.0;
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = partials[(size_t)(b + k) * 32 + col];
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; b < b1; ++b) s += partials[(size_t)b * 32 + col];
    sg[grp][col] = s;
    __syncthreads();
    if (threadIdx.x < 32) {
        double t = 0.0;
#pragma unroll
        for (int g = 0; g < 32; ++g) t += sg[g][threadIdx.x];
        out[threadIdx.x] = t;
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
int launch_h_model(const MatchArgs& a, bool redo, hipStream_t st) {
    if (a.n == 0) return 0;
    if (redo) {
        if (a.knn_mode == 0 && !a.dbg) {  // lane per point (default)
            const int nb = (a.n + kBlock - 1) / kBlock;
            h_model_knn_lane_kernel<<<nb, kBlock, 0, st>>>(a);
            return nb;
        }
        const int qpb = kKnnBlock / kGroup;  // 8 lanes per point (diagnostics / A-B)
        const int nb = (a.n + qpb - 1) / qpb;
        if (a.dbg)
            h_model_knn_kernel<true><<<nb, kKnnBlock, 0, st>>>(a);
        else
            h_model_knn_kernel<false><<<nb, kKnnBlock, 0, st>>>(a);
        return nb;
    }
    const int nb = (a.n + kBlock - 1) / kBlock;
    h_model_reuse_kernel<<<nb, kBlock, 0, st>>>(a);
    return nb;
}

void launch_finalize(const double* partials, int nblocks, double* out, hipStream_t st) {
    finalize_kernel<<<1, 1024, 0, st>>>(partials, nblocks, out);
}

void launch_debug(const MatchArgs& a, float* world, float* d2, float* abcd_pd2, hipStream_t st) {
    if (a.n == 0) return;
    debug_kernel<<<(a.n + 255) / 256, 256, 0, st>>>(a, world, d2, abcd_pd2);
}

void launch_h_rows(const MatchArgs& a, double* rows, int64_t max_rows, int64_t* n_rows, hipStream_t st) {
    h_rows_kernel<<<1, 1024, 0, st>>>(a, rows, max_rows, n_rows);
}

int match_blocks(int n) {  // partial slots needed by either kernel
    const int qpb = kKnnBlock / kGroup;
    return std::max((n + kBlock - 1) / kBlock, (n + qpb - 1) / qpb);
}

}  // namespace lio
