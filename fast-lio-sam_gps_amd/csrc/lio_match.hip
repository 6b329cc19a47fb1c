// lio_match.hip — FAST-LIO h_share_model on gfx950.
//
// One lane = one feats_down_body point.  Two fused kernels per h-evaluation:
//
//   h_model_kernel<REDO_KNN=true>  (ekfom_data.converge == true)
//     body->world (double, stored float) -> exact grid 5-NN -> gate
//     (found == 5 && d2[4] <= 5) -> esti_plane (QR, registers) -> pd2, s-gate
//     -> H row (double) -> 30-value block reduction -> block partial
//     writes: nn_idx[5] (20 B), plane abcd (16 B), sel (1 B)
//   h_model_kernel<REDO_KNN=false> (converge == false: reuse Nearest_Points)
//     body->world -> cached plane -> pd2, s-gate -> H row -> block partial
//   finalize_kernel: sums the block partials in a fixed order (deterministic)
//
// The per-point dense H (effct x 12 doubles) of the reference is never
// materialised: the IESKF only consumes H^T H and H^T h.
#include "lio_dev.hpp"
#include "lio_kernels.hpp"

namespace lio {

constexpr int kBlock = 256;
constexpr int kNSum = 30;  // 21 HTH + 6 HTh + neff + res + hh

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool REDO>
__global__ void __launch_bounds__(kBlock) h_model_kernel(MatchArgs a) {
    __shared__ double red[kBlock / 64][32];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    double J[6] = {0, 0, 0, 0, 0, 0};
    double h = 0.0, res = 0.0, cnt = 0.0;
    if (i < a.n) {
        const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
        float wx, wy, wz;
        body_to_world(a.pose, bx, by, bz, wx, wy, wz);
        bool sel;
        float4 pl;
        if constexpr (REDO) {
            TopK<5> tk;
            tk.init(a.range_sq);
            grid_knn_exact<5>(a.grid, wx, wy, wz, a.max_shell, tk);
            int32_t* o = a.nn_idx + 5 * (size_t)i;
#pragma unroll
            for (int j = 0; j < 5; ++j) o[j] = tk.id[j] == kNone ? -1 : tk.id[j];
            // point_selected_surf = found == 5 && !(sqdist[4] > 5)
            sel = tk.id[4] != kNone && !(tk.d[4] > a.range_sq);
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
                pl = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
                a.planes[i] = pl;
            }
        } else {
            sel = a.sel[i] != 0;
            if (sel) pl = a.planes[i];
        }
        if (sel) {
            const float pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
            const double b0 = bx, b1 = by, b2 = bz;
            const double pn = sqrt((b0 * b0 + b1 * b1) + b2 * b2);
            const float s = (float)(1.0 - a.s_coef * (double)fabsf(pd2) / sqrt(pn));
            sel = (double)s > a.s_gate;
            if (sel) {
                h_row(a.pose, bx, by, bz, pl.x, pl.y, pl.z, J);
                h = -(double)pd2;
                res = (double)fabsf(pd2);
                cnt = 1.0;
            }
        }
        a.sel[i] = sel ? 1 : 0;
    }
    // ---- block reduction of [HTH(21), HTh(6), cnt, res, hh]
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double v[kNSum];
    int q = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) v[q++] = J[r] * J[c];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[21 + r] = J[r] * h;
    v[27] = cnt;
    v[28] = res;
    v[29] = h * h;
#pragma unroll
    for (int k = 0; k < kNSum; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kNSum; ++k) red[wid][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < kNSum) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
        a.partials[(size_t)blockIdx.x * 32 + threadIdx.x] = s;
    }
}

// Fixed-order sum of nblocks x 32 partials -> out[32] (one block).
__global__ void __launch_bounds__(256) finalize_kernel(const double* __restrict__ partials, int nblocks,
                                                      double* __restrict__ out) {
    __shared__ double s8[8][32];
    const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
    double s = 0.0;
    for (int b = grp; b < nblocks; b += 8) s += partials[(size_t)b * 32 + col];
    s8[grp][col] = s;
    __syncthreads();
    if (threadIdx.x < 32) {
        double t = 0.0;
#pragma unroll
        for (int g = 0; g < 8; ++g) t += s8[g][threadIdx.x];
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
    const int nb = (a.n + kBlock - 1) / kBlock;
    if (nb == 0) return 0;
    if (redo)
        h_model_kernel<true><<<nb, kBlock, 0, st>>>(a);
    else
        h_model_kernel<false><<<nb, kBlock, 0, st>>>(a);
    return nb;
}

void launch_finalize(const double* partials, int nblocks, double* out, hipStream_t st) {
    finalize_kernel<<<1, 256, 0, st>>>(partials, nblocks, out);
}

void launch_debug(const MatchArgs& a, float* world, float* d2, float* abcd_pd2, hipStream_t st) {
    if (a.n == 0) return;
    debug_kernel<<<(a.n + 255) / 256, 256, 0, st>>>(a, world, d2, abcd_pd2);
}

void launch_h_rows(const MatchArgs& a, double* rows, int64_t max_rows, int64_t* n_rows, hipStream_t st) {
    h_rows_kernel<<<1, 1024, 0, st>>>(a, rows, max_rows, n_rows);
}

int match_blocks(int n) { return (n + kBlock - 1) / kBlock; }

}  // namespace lio
