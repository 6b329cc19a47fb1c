// lio_icp.hip — loop-closure ICP (PCL IterativeClosestPoint as configured at
// /root/reference/fast_lio_sam/src/loop_closure.cpp:3-14, aligned at :81) on gfx950.
//
// Per ICP iteration (one lane = one source point of this rank's shard):
//   icp_near_kernel  apply the previous T_inc to the incrementally transformed
//                    cloud (PCL transformCloud, float SSE order [U]), exact 1-NN
//                    in the target grid over shells 0..2; lanes whose answer is
//                    not yet certain go to a far list
//   icp_far_kernel   finishes those lanes with an unbounded shell walk
//   icp_stats_kernel per 256-point chunk: Umeyama sufficient statistics of the
//                    accepted correspondences (d2 <= 52.5^2) in double about a
//                    fixed centre c0: count, sum p, sum q, sum q p^T, sum d2
//   icp_reduce_kernel 16 chunks -> one 4096-point record, fixed order
// The 4096-point records are what ranks all-gather (deterministic, identical
// for any number of ranks).  The fitness pass is the same pipeline on the
// ORIGINAL source transformed by the final T, unbounded.
#include "lio_dev.hpp"
#include "lio_kernels.hpp"

namespace lio {

// PCL 1.10 Transformer<float>::se3 (SSE): x' = m0*x + (m1*y + (m2*z + m3)) [U]
__device__ __forceinline__ void xform_pcl(const float* T, float x, float y, float z, float& ox, float& oy,
                                          float& oz) {
    ox = T[0] * x + (T[1] * y + (T[2] * z + T[3]));
    oy = T[4] * x + (T[5] * y + (T[6] * z + T[7]));
    oz = T[8] * x + (T[9] * y + (T[10] * z + T[11]));
}

constexpr int kIcpGroup = 8;  // lanes cooperating on one query's 1-NN

// 256 threads = 32 source points, 8 lanes per point.
__global__ void __launch_bounds__(256) icp_near_kernel(IcpArgs a) {
    __shared__ uint32_t s_tab[256 / kIcpGroup][72];  // per-group shell-1 slot table
    const int i = xcd_block(blockIdx.x, gridDim.x) * (256 / kIcpGroup) + threadIdx.x / kIcpGroup;
    const int sub = threadIdx.x % kIcpGroup;
    if (i >= a.n) return;  // whole groups leave together
    float x, y, z;
    if (a.fitness) {  // getFitnessScore: original source * final; kept in cur for `aligned_`
        xform_pcl(a.T, a.src[3 * i], a.src[3 * i + 1], a.src[3 * i + 2], x, y, z);
    } else {
        x = a.cur[3 * i];
        y = a.cur[3 * i + 1];
        z = a.cur[3 * i + 2];
        if (a.apply_T) {
            float ox, oy, oz;
            xform_pcl(a.T, x, y, z, ox, oy, oz);
            x = ox;
            y = oy;
            z = oz;
        }
    }
    TopK<1> tk;
    tk.init(INFINITY);
    const bool done =
        group_knn_near<1, kIcpGroup>(a.grid, x, y, z, a.max_shell_near, sub, tk, nullptr, s_tab[threadIdx.x / kIcpGroup]);
    if (sub == 0) {
        if (a.fitness || a.apply_T) {
            a.cur[3 * i] = x;
            a.cur[3 * i + 1] = y;
            a.cur[3 * i + 2] = z;
        }
        a.far_d2[i] = tk.d(0);
        a.far_id[i] = tk.id(0);
        if (!done) {
            const int slot = atomicAdd(a.far_count, 1);
            a.far_list[slot] = i;
        }
    }
}

// Unresolved points: unbounded shell walk seeded with the near result.
__global__ void __launch_bounds__(256) icp_far_kernel(IcpArgs a) {
    const int cnt = *a.far_count;
    const int sub = threadIdx.x % kIcpGroup;
    const int gpb = 256 / kIcpGroup;
    for (int k = blockIdx.x * gpb + threadIdx.x / kIcpGroup; k < cnt; k += gridDim.x * gpb) {
        const int i = a.far_list[k];
        const float x = a.cur[3 * i], y = a.cur[3 * i + 1], z = a.cur[3 * i + 2];
        TopK<1> tk;
        tk.init(INFINITY);
        if (sub == 0) {  // the near pass's best is a valid starting bound (only lane 0 holds it)
            tk.k[0] = knn_key(a.far_d2[i], a.far_id[i]);
        }
        group_knn_exact<1, kIcpGroup>(a.grid, x, y, z, 0x3fffffff, sub, tk);
        if (sub == 0) {
            a.far_d2[i] = tk.d(0);
            a.far_id[i] = tk.id(0);
        }
    }
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// one block = one 256-point chunk -> partials[chunk][kIcpStride]
__global__ void __launch_bounds__(256) icp_stats_kernel(IcpArgs a) {
    __shared__ double red[4][kIcpStride];
    const int i = blockIdx.x * 256 + threadIdx.x;
    double v[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) v[k] = 0.0;
    if (i < a.n) {
        const int id = a.far_id[i];
        const float d2 = a.far_d2[i];
        if (a.fitness) {
            if (id >= 0 && id != kNone) {
                v[0] = 1.0;
                v[16] = (double)d2;
            }
        } else if (id >= 0 && id != kNone && !((double)d2 > a.max_d2)) {
            const float4 q = a.tgt_by_id[id];
            const double p0 = (double)a.cur[3 * i] - a.c0[0], p1 = (double)a.cur[3 * i + 1] - a.c0[1],
                         p2 = (double)a.cur[3 * i + 2] - a.c0[2];
            const double q0 = (double)q.x - a.c0[0], q1 = (double)q.y - a.c0[1], q2 = (double)q.z - a.c0[2];
            v[0] = 1.0;
            v[1] = p0; v[2] = p1; v[3] = p2;
            v[4] = q0; v[5] = q1; v[6] = q2;
            v[7] = q0 * p0; v[8] = q0 * p1; v[9] = q0 * p2;
            v[10] = q1 * p0; v[11] = q1 * p1; v[12] = q1 * p2;
            v[13] = q2 * p0; v[14] = q2 * p1; v[15] = q2 * p2;
            v[16] = (double)d2;
        }
    }
#pragma unroll
    for (int k = 0; k < 17; ++k) v[k] = wsum(v[k]);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 17; ++k) red[wid][k] = v[k];
    __syncthreads();
    if (threadIdx.x < kIcpStride) {
        double s = 0.0;
        if (threadIdx.x < 17)
            for (int w = 0; w < 4; ++w) s += red[w][threadIdx.x];
        a.partials[(size_t)blockIdx.x * kIcpStride + threadIdx.x] = s;
    }
}

// 16 consecutive chunk records -> one 4096-point record, ascending order
__global__ void icp_reduce_kernel(const double* __restrict__ partials, int nchunks, double* __restrict__ super) {
    const int sidx = blockIdx.x;
    const int k = threadIdx.x;
    if (k >= kIcpStride) return;
    constexpr int per = kIcpSuper / kIcpChunk;
    double s = 0.0;
    for (int c = sidx * per; c < min(nchunks, (sidx + 1) * per); ++c) s += partials[(size_t)c * kIcpStride + k];
    super[(size_t)sidx * kIcpStride + k] = s;
}

void launch_icp_near(const IcpArgs& a, hipStream_t st) {
    if (a.n == 0) return;
    const int ppb = 256 / kIcpGroup;
    icp_near_kernel<<<(a.n + ppb - 1) / ppb, 256, 0, st>>>(a);
}
void launch_icp_far(const IcpArgs& a, int max_far_blocks, hipStream_t st) {
    if (a.n == 0) return;
    icp_far_kernel<<<max_far_blocks, 256, 0, st>>>(a);
}
void launch_icp_stats(const IcpArgs& a, hipStream_t st) {
    if (a.n == 0) return;
    icp_stats_kernel<<<(a.n + 255) / 256, 256, 0, st>>>(a);
}
void launch_icp_reduce(const double* partials, int nchunks, double* super, hipStream_t st) {
    const int ns = (nchunks + (kIcpSuper / kIcpChunk) - 1) / (kIcpSuper / kIcpChunk);
    if (ns == 0) return;
    icp_reduce_kernel<<<ns, 64, 0, st>>>(partials, nchunks, super);
}

}  // namespace lio
