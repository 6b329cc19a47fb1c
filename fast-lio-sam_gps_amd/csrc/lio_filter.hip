// lio_filter.hip — point-cloud filters on either side of the hot path
// (SURVEY §8(f) rows 2 and 3), on gfx950:
//
//   voxel_grid      pcl::VoxelGrid<PointT>::filter (PCL 1.10 applyFilter) [U]:
//                   FAST-LIO's downSizeFilterSurf (filter_size_surf) and the
//                   loop closure's voxelizePcd (utilities.hpp:161-183)
//   transform_segs  pcl::transformPointCloud(cloud, out, Matrix4d) [U] per
//                   keyframe segment (transformPcd, utilities.hpp:132-143)
//   undistort       FAST-LIO ImuProcess::UndistortPcl backward propagation [U]
//   scan_select     FAST-LIO Preprocess point_filter_num / blind selection [U]
//
// VoxelGrid on the GPU: AABB -> (min_b, divb_mul) on the device -> one int
// voxel index per point -> stable radix sort (index, input position) -> run
// heads -> one lane per voxel sums its points' fields in input order and
// divides by the count (the PCL centroid; PCL sorts with std::sort, whose
// order inside a voxel is unspecified — the stable order makes the float sums
// reproducible).  Output in voxel-index order, as PCL.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "lio_dev.hpp"
#include "lio_error.hpp"
#include "lio_filter.hpp"

namespace lio {

namespace {

constexpr uint32_t kInvalid = 0xffffffffu;
constexpr int kPartBlocks = 4096;  // AABB partials b.part holds (a fused producer needs one per 256-row block)

// min / max over the NT lanes of the block (lo[3], hi[3] per lane) into s[0..2][0] / s[3..5][0]
template <int NT>
__device__ __forceinline__ void block_minmax(float (*s)[NT], const float* lo, const float* hi) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        s[d][threadIdx.x] = lo[d];
        s[3 + d][threadIdx.x] = hi[d];
    }
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                s[d][threadIdx.x] = fminf(s[d][threadIdx.x], s[d][threadIdx.x + w]);
                s[3 + d][threadIdx.x] = fmaxf(s[3 + d][threadIdx.x], s[3 + d][threadIdx.x + w]);
            }
        }
        __syncthreads();
    }
}

// PCL's voxel geometry from the cloud's AABB (getMinMax3D over finite points):
//   inverse_leaf = 1 / leaf;  min_b = floor(min_p * inv), max_b = floor(max_p * inv)
//   div_b = max_b - min_b + 1; divb_mul = (1, div_b.x, div_b.x * div_b.y)
//   overflow when div_b.x * div_b.y * div_b.z > INT_MAX (PCL then returns the input)
__device__ __forceinline__ VoxelGeom voxel_geom(const float* lo, const float* hi, float lx, float ly, float lz) {
    VoxelGeom g;
    const float inv[3] = {1.0f / lx, 1.0f / ly, 1.0f / lz};
    int64_t div[3];
    g.empty = !(lo[0] <= hi[0]);
    for (int d = 0; d < 3; ++d) {
        g.inv[d] = inv[d];
        g.min_b[d] = g.empty ? 0 : (int)floorf(lo[d] * inv[d]);
        const int max_b = g.empty ? 0 : (int)floorf(hi[d] * inv[d]);
        div[d] = (int64_t)max_b - g.min_b[d] + 1;
    }
    g.overflow = div[0] * div[1] * div[2] > (int64_t)0x7fffffff;
    g.mul[0] = 1;
    g.mul[1] = (int)div[0];
    g.mul[2] = (int)(div[0] * div[1]);
    const int64_t top = g.overflow ? 0 : div[0] * div[1] * div[2] - 1;
    g.key_bits = top > 0 ? 64 - __clzll((unsigned long long)top) : 1;
    return g;
}

// per block: min / max of the finite points it covers -> part[6 blockIdx.x ..] (lo xyz, hi xyz); no
// cross-block hand-off — the key kernel reduces the partials itself
__global__ void __launch_bounds__(256) minmax_partial_kernel(const float* __restrict__ p, int64_t n, int stride,
                                                             float* __restrict__ part) {
    __shared__ float s[6][256];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float* q = p + (size_t)i * stride;
        const float x = q[0], y = q[1], z = q[2];
        if (!(isfinite(x) && isfinite(y) && isfinite(z))) continue;
        lo[0] = fminf(lo[0], x);
        lo[1] = fminf(lo[1], y);
        lo[2] = fminf(lo[2], z);
        hi[0] = fmaxf(hi[0], x);
        hi[1] = fmaxf(hi[1], y);
        hi[2] = fmaxf(hi[2], z);
    }
    block_minmax<256>(s, lo, hi);
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

// minmax_partial_kernel over the first *cnt of n rows
__global__ void __launch_bounds__(256) minmax_partial_cnt_kernel(const float* __restrict__ p, int64_t n,
                                                                 const uint32_t* __restrict__ cnt, int stride,
                                                                 float* __restrict__ part) {
    __shared__ float s[6][256];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    n = min<int64_t>(n, *cnt);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float* q = p + (size_t)i * stride;
        const float x = q[0], y = q[1], z = q[2];
        if (!(isfinite(x) && isfinite(y) && isfinite(z))) continue;
        lo[0] = fminf(lo[0], x);
        lo[1] = fminf(lo[1], y);
        lo[2] = fminf(lo[2], z);
        hi[0] = fmaxf(hi[0], x);
        hi[1] = fmaxf(hi[1], y);
        hi[2] = fmaxf(hi[2], z);
    }
    block_minmax<256>(s, lo, hi);
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

// Every block first reduces the nbp AABB partials (a few KB from L2) and derives the voxel geometry itself
// — no single-block hand-off kernel between the AABB and the keys; block 0 also stores the geometry for
// the host (host-mapped gh).  Keys past `bits` bits (the width the sort will use) raise flags[0].
__global__ void __launch_bounds__(256) voxel_key_kernel(const float* __restrict__ p, int64_t n,
                                                        const uint32_t* __restrict__ cnt, int stride,
                                                        const float* __restrict__ part, int nbp, float lx, float ly,
                                                        float lz, VoxelGeom* __restrict__ gh, uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals, int bits,
                                                        uint32_t* __restrict__ flags) {
    __shared__ float s[6][256];
    __shared__ VoxelGeom s_g;
    {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int b = threadIdx.x; b < nbp; b += 256) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                lo[d] = fminf(lo[d], part[b * 6 + d]);
                hi[d] = fmaxf(hi[d], part[b * 6 + 3 + d]);
            }
        }
        block_minmax<256>(s, lo, hi);
        if (threadIdx.x == 0) {
            const float l3[3] = {s[0][0], s[1][0], s[2][0]}, h3[3] = {s[3][0], s[4][0], s[5][0]};
            s_g = voxel_geom(l3, h3, lx, ly, lz);
            if (blockIdx.x == 0) *gh = s_g;
        }
        __syncthreads();
    }
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const VoxelGeom g = s_g;
    const float* q = p + (size_t)i * stride;
    uint32_t k = kInvalid;
    if ((!cnt || i < (int64_t)*cnt) && isfinite(q[0]) && isfinite(q[1]) && isfinite(q[2]) && !g.overflow) {
        const int i0 = (int)(floorf(q[0] * g.inv[0]) - (float)g.min_b[0]);
        const int i1 = (int)(floorf(q[1] * g.inv[1]) - (float)g.min_b[1]);
        const int i2 = (int)(floorf(q[2] * g.inv[2]) - (float)g.min_b[2]);
        k = (uint32_t)(i0 * g.mul[0] + i1 * g.mul[1] + i2 * g.mul[2]);
        if (bits < 32 && k >= (1u << bits) - 1u) flags[0] = 1u;  // the all-ones pattern marks invalid keys
    }
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

__global__ void run_head_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ head) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j > n) return;
    head[j] = (j < n && keys[j] != kInvalid && (j == 0 || keys[j - 1] != keys[j])) ? 1u : 0u;
}

// Voxel runs of the sorted keys: run r = [starts[r], ends[r]).  The run index
// of element j is (inclusive head count) - 1 = vid[j] + head[j] - 1.
// lane 0 also publishes the voxel count and the key-width flag to host-mapped memory (hsm[0], hsm[kHostFlags])
// and clears the flag for the next call
__global__ void voxel_bounds_kernel(const uint32_t* __restrict__ keys, int64_t n, const uint32_t* __restrict__ head,
                                    const uint32_t* __restrict__ vid, uint32_t* __restrict__ starts,
                                    uint32_t* __restrict__ ends, uint32_t* __restrict__ flags, int* __restrict__ hsm) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j == 0) {
        hsm[0] = (int)vid[n];
        hsm[kHostFlags] = (int)flags[0];
        flags[0] = 0u;
    }
    if (j >= n) return;
    const uint32_t key = keys[j];
    if (key == kInvalid) return;
    const uint32_t h = head[j];
    const uint32_t r = vid[j] + h - 1;
    if (h) starts[r] = (uint32_t)j;
    if (j + 1 == n || keys[j + 1] != key) ends[r] = (uint32_t)(j + 1);
}

// Small inputs (n <= kRunsOneBlock): run heads, their exclusive count and the run bounds in ONE block —
// instead of run_head + the device scan (2 kernels) + voxel_bounds: 4 launches -> 1.  The block covers the
// sorted keys in kRunsTiles tiles of 4096 (16 B per lane per tile), all loads issued up front (one memory
// round trip, not one per tile); each lane counts the run heads of its 4 keys per tile, a wave prefix sum
// per tile from ballots (no shuffles) and the 16 wave totals per tile through LDS give every (tile, lane)
// its first run index.
// Publishes the count like voxel_bounds_kernel (hsm[0], the key-width flag) and stores it at *n_vox.
constexpr int kRunsTiles = 8;
constexpr int64_t kRunsOneBlock = 4096 * kRunsTiles;
__global__ void __launch_bounds__(1024) voxel_runs_block_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                                uint32_t* __restrict__ starts,
                                                                uint32_t* __restrict__ ends,
                                                                uint32_t* __restrict__ n_vox,
                                                                uint32_t* __restrict__ flags, int* __restrict__ hsm) {
    __shared__ uint32_t s_w[kRunsTiles][16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t k[kRunsTiles][4], prev[kRunsTiles], next[kRunsTiles];
#pragma unroll
    for (int t = 0; t < kRunsTiles; ++t) {
        const int64_t j0 = 4096 * (int64_t)t + 4 * (int64_t)tid;
        if (j0 + 3 < n) {
            const uint4 v = *reinterpret_cast<const uint4*>(keys + j0);
            k[t][0] = v.x, k[t][1] = v.y, k[t][2] = v.z, k[t][3] = v.w;
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) k[t][u] = j0 + u < n ? keys[j0 + u] : kInvalid;
        }
        prev[t] = (j0 > 0 && j0 - 1 < n) ? keys[j0 - 1] : kInvalid;
        next[t] = j0 + 4 < n ? keys[j0 + 4] : kInvalid;
    }
    uint32_t excl[kRunsTiles];
#pragma unroll
    for (int t = 0; t < kRunsTiles; ++t) {
        const int64_t j0 = 4096 * (int64_t)t + 4 * (int64_t)tid;
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t before = u == 0 ? prev[t] : k[t][u - 1];
            cnt += (k[t][u] != kInvalid && (j0 + u == 0 || before != k[t][u])) ? 1u : 0u;
        }
        // wave exclusive prefix of cnt (0..4) from its three bit planes: a ballot and a masked popcount each
        uint32_t ex = 0, wt = 0;
#pragma unroll
        for (int bit = 0; bit < 3; ++bit) {
            const uint64_t m = __ballot((cnt >> bit) & 1u);
            ex += (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << bit;
            wt += (uint32_t)__popcll(m) << bit;
        }
        if (lane == 0) s_w[t][w] = wt;
        excl[t] = ex;
    }
    __syncthreads();
    uint32_t run = 0;  // runs started before tile t
#pragma unroll
    for (int t = 0; t < kRunsTiles; ++t) {
        const int64_t j0 = 4096 * (int64_t)t + 4 * (int64_t)tid;
        uint32_t woff = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t x = s_w[t][i];
            woff += i < w ? x : 0u;
            tot += x;
        }
        uint32_t r = run + woff + excl[t];  // runs started before this lane's first key of the tile
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (k[t][u] == kInvalid) continue;
            const uint32_t j = (uint32_t)(j0 + u);
            const uint32_t before = u == 0 ? prev[t] : k[t][u - 1];
            if (j == 0 || before != k[t][u]) starts[r++] = j;
            const uint32_t after = u == 3 ? next[t] : k[t][u + 1];
            if (after != k[t][u]) ends[r - 1] = j + 1;  // past the end reads kInvalid != any valid key
        }
        run += tot;
    }
    if (tid == 0) {
        *n_vox = run;
        hsm[0] = (int)run;
        hsm[kHostFlags] = (int)flags[0];
        flags[0] = 0u;
    }
}

// the one-block run bounds up to kRunsOneBlock keys (the C5 sweep); larger inputs (map build, submaps) use
// run_head + the device scan + voxel_bounds
inline bool runs_one_block(int64_t n) { return n <= kRunsOneBlock; }

// Every voxel on its own wave (4 per block, the grid striding the voxels): the wave loads up to 64 of the
// run's points at once (index, then row: two dependent loads per chunk instead of one pair per point on
// one lane; the next chunk's loads in flight while this one is summed), stashes them in its LDS slice,
// and lane f adds field f over the chunk in input order — the same sums in the same order as
// round 4's lane-per-short-run + wave-per-long-run pair (20.6 vs 9.1 µs at C5), without its
// long-run list.
constexpr int kWaveCentroidBlocks = 1024;
__global__ void __launch_bounds__(256) voxel_centroid_wave_kernel(const float* __restrict__ p, int stride,
                                                                  const uint32_t* __restrict__ vals,
                                                                  const uint32_t* __restrict__ starts,
                                                                  const uint32_t* __restrict__ ends,
                                                                  const uint32_t* __restrict__ n_vox,
                                                                  float* __restrict__ out, float* __restrict__ xyz,
                                                                  uint8_t* __restrict__ sel) {
    __shared__ float s_q[4][64 * kMaxFields];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* sq = s_q[wv];
    const uint32_t nv = *n_vox;
    for (uint32_t v = blockIdx.x * 4 + wv; v < nv; v += gridDim.x * 4) {
        const uint32_t s = starts[v], e = ends[v];
        float acc = 0.f;
        float q[kMaxFields];
        auto load = [&](uint32_t k) {  // chunk k's rows into registers (lanes past the run: nothing)
            if (k + lane < e) {
                const float* r = p + (size_t)vals[k + lane] * stride;
#pragma unroll
                for (int f = 0; f < kMaxFields; ++f) q[f] = f < stride ? r[f] : 0.f;
            }
        };
        load(s);
        for (uint32_t k = s; k < e; k += 64) {
            const uint32_t m = min(64u, e - k);
            if ((uint32_t)lane < m) {
#pragma unroll
                for (int f = 0; f < kMaxFields; ++f)
                    if (f < stride) sq[lane * stride + f] = q[f];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (k + 64 < e) load(k + 64);  // the next chunk in flight while this one is summed
            if (lane < stride) {
                const float* col = sq + lane;
                uint32_t l = 0;
                for (; l + 4 <= m; l += 4) {
                    const float a0 = col[(l + 0) * stride], a1 = col[(l + 1) * stride];
                    const float a2 = col[(l + 2) * stride], a3 = col[(l + 3) * stride];
                    acc += a0;
                    acc += a1;
                    acc += a2;
                    acc += a3;
                }
                for (; l < m; ++l) acc += col[l * stride];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();  // the next chunk overwrites the slice
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const float c = (float)(e - s);
        if (lane < stride) out[(size_t)v * stride + lane] = acc / c;
        if (xyz && lane < 3) xyz[3 * (size_t)v + lane] = acc / c;
        if (xyz && lane == 0) sel[v] = 0;
    }
}

__global__ void copy_strided_kernel(const float* __restrict__ a, int64_t nf, float* __restrict__ b) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < nf) b[i] = a[i];
}

// transformPcd: double 4x4 per segment, ((m0 x + m1 y) + m2 z) + m3 in double, stored float;
// non-finite points copied unchanged (PCL's !is_dense branch); other fields copied
__global__ void transform_segs_kernel(const float* __restrict__ in, int64_t n, int stride,
                                      const int64_t* __restrict__ seg_off, int nseg, const double* __restrict__ T16,
                                      float* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    int lo = 0, hi = nseg;  // segment s: [seg_off[s], seg_off[s+1])
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (seg_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    const double* m = T16 + 16 * lo;
    const float* q = in + (size_t)i * stride;
    float* o = out + (size_t)i * stride;
    for (int f = 3; f < stride; ++f) o[f] = q[f];
    if (!(isfinite(q[0]) && isfinite(q[1]) && isfinite(q[2]))) {
        o[0] = q[0];
        o[1] = q[1];
        o[2] = q[2];
        return;
    }
    const double x = q[0], y = q[1], z = q[2];
    o[0] = (float)(((m[0] * x + m[1] * y) + m[2] * z) + m[3]);
    o[1] = (float)(((m[4] * x + m[5] * y) + m[6] * z) + m[7]);
    o[2] = (float)(((m[8] * x + m[9] * y) + m[10] * z) + m[11]);
}

// ---- scan preprocessing --------------------------------------------------------
// Preprocess (point_filter_num, blind) [U] and the time sort's key in one pass: input i is selected when
// i % every == 0 and x*x + y*y + z*z > blind^2 (float); its key is the float bits of the point time
// (curvature, ms) mapped to an unsigned order (negative times below every positive one), capped one below
// the largest key, which marks the rows not selected.  The stable sort then leaves the selected rows
// first, in time order and, inside a tie, in input order — compaction and sort in one.  every = 0: no
// selection (the host selected the rows), the time key only.
constexpr uint32_t kNotSelected = 0xffffffffu;
__device__ __forceinline__ uint32_t piece_row(const RowPieces& m, uint32_t i) {
    uint32_t base = m.src[0], s0 = m.start[0];
#pragma unroll
    for (int t = 1; t < kMaxPieces; ++t)
        if (t < m.n && i >= m.start[t]) base = m.src[t], s0 = m.start[t];
    return base + (i - s0);
}
__global__ void scan_key_kernel(const float* __restrict__ p, int64_t n, int stride, int every, float blind2,
                                int tfield, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, RowPieces rp) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k = kNotSelected;
    const float* q = p + (size_t)piece_row(rp, (uint32_t)i) * stride;
    if (every == 0 || (i % every == 0 && (q[0] * q[0] + q[1] * q[1] + q[2] * q[2]) > blind2)) {
        const uint32_t b = __float_as_uint(q[tfield]);
        k = min((b & 0x80000000u) ? ~b : (b | 0x80000000u), kNotSelected - 1);
    }
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

// sin / cos of the undistortion's SO3 Exp with ONE fixed-order routine on the device and in the
// CPU restatement (oracle/lio_oracle.cpp sincos_fixed), so the undistorted points agree bit for bit
// (the reference calls libm sin / cos, whose last bit is implementation-defined).  The published
// fdlibm algorithm: Cody-Waite reduction by pi/2 in three 33-bit parts (exact products for
// |n| < 2^20), then the __kernel_sin / __kernel_cos minimax polynomials on [-pi/4, pi/4]; < 1 ulp
// from the true value.  Arguments beyond 2^19 pi/2 do not occur (angular rate x dt of one sweep).
__device__ __forceinline__ double ksin_fixed(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if (fabs(x) < 7.450580596923828125e-09) return x;  // 2^-27
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
__device__ __forceinline__ double kcos_fixed(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double ax = fabs(x);
    if (ax < 7.450580596923828125e-09) return 1.0;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ax < 0.3) return 1.0 - (0.5 * z - z * r);
    double qx;
    if (ax > 0.78125) {
        qx = 0.28125;
    } else {  // |x| / 4 with the low word cleared
        const unsigned long long hi = (unsigned long long)__double_as_longlong(ax) >> 32;
        qx = __longlong_as_double((long long)((hi - 0x00200000ull) << 32));
    }
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    return a - (hz - z * r);
}
__device__ __forceinline__ void sincos_fixed(double x, double* s, double* c) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_2 = 6.07710050630396597660e-11, pio2_3 = 2.02226624871116645580e-21;
    int n = 0;
    double r = x;
    if (!(fabs(x) <= 7.85398163397448278999e-01)) {  // pi/4
        const double fn = rint(x * invpio2);
        n = (int)fn;
        r = ((x - fn * pio2_1) - fn * pio2_2) - fn * pio2_3;
    }
    const double ks = ksin_fixed(r), kc = kcos_fixed(r);
    switch (n & 3) {
        case 0: *s = ks, *c = kc; break;
        case 1: *s = kc, *c = -ks; break;
        case 2: *s = -ks, *c = -kc; break;
        default: *s = -kc, *c = ks; break;
    }
}

// FAST-LIO so3_math Exp(ang_vel, dt): I + sin(a) K + (1 - cos(a)) K K
__device__ __forceinline__ void so3_exp(const double w[3], double dt, double E[9]) {
    const double nrm = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    for (int k = 0; k < 9; ++k) E[k] = (k % 4 == 0) ? 1.0 : 0.0;
    if (!(nrm > 0.0000001)) return;
    const double r[3] = {w[0] / nrm, w[1] / nrm, w[2] / nrm};
    const double K[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
    double s, co;
    sincos_fixed(nrm * dt, &s, &co);
    const double c1 = 1.0 - co;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            // ((1 - cos) K) * K: Eigen's coefficient-based 3x3 product sums e0 + (e1 + e2)
            // (redux_novec_unroller halves the 3 terms 1 + 2)
            const double kk = (c1 * K[3 * i + 0]) * K[0 + j] + ((c1 * K[3 * i + 1]) * K[3 + j] + (c1 * K[3 * i + 2]) * K[6 + j]);
            E[3 * i + j] = (E[3 * i + j] + s * K[3 * i + j]) + kk;
        }
}

// M3D * V3D as Eigen evaluates it (coefficient-based product: e0 + (e1 + e2))
__device__ __forceinline__ void mv3(const double* M, const double* v, double* o) {
    for (int r = 0; r < 3; ++r) o[r] = M[3 * r] * v[0] + (M[3 * r + 1] * v[1] + M[3 * r + 2] * v[2]);
}

__device__ __forceinline__ void compensate(float* q, float tms, const ImuPose& hd, const ImuPose& tl,
                                           const UndistortEnd& end) {
    const double dt = (double)tms / double(1000) - hd.offset_time;
    double E[9], Ri[9];
    so3_exp(tl.gyr, dt, E);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            Ri[3 * r + c] = hd.rot[3 * r] * E[c] + (hd.rot[3 * r + 1] * E[3 + c] + hd.rot[3 * r + 2] * E[6 + c]);
    double Tei[3];
    for (int k = 0; k < 3; ++k) Tei[k] = ((hd.pos[k] + hd.vel[k] * dt) + ((0.5 * tl.acc[k]) * dt) * dt) - end.pos[k];
    // P_compensate = offset_R_L_I.conjugate() * (rot.conjugate() * (R_i * (offset_R_L_I * P_i +
    //                offset_T_L_I) + T_ei) - offset_T_L_I)  [U]; SO3 products as Eigen (quat_rotate)
    double a[3], b[3], c[3];
    quat_rotate(end.q_LI, false, (double)q[0], (double)q[1], (double)q[2], a[0], a[1], a[2]);
    for (int k = 0; k < 3; ++k) a[k] += end.t_LI[k];
    mv3(Ri, a, b);
    for (int k = 0; k < 3; ++k) b[k] += Tei[k];
    quat_rotate(end.q, true, b[0], b[1], b[2], c[0], c[1], c[2]);
    for (int k = 0; k < 3; ++k) c[k] -= end.t_LI[k];
    quat_rotate(end.q_LI, true, c[0], c[1], c[2], a[0], a[1], a[2]);
    q[0] = (float)a[0];
    q[1] = (float)a[1];
    q[2] = (float)a[2];
}

// UndistortPcl backward propagation, one lane per time-sorted row, gathered from the input through the
// sort's permutation: the lane at the end of the selected rows stores their count (cnt[0]).  head = the
// last IMU pose whose offset_time is < t (tail = head + 1 gives acc/gyr); points at or before the first
// pose are left unchanged, as the reference's loop never reaches them.  The reference's loop `break`s at
// the first point without stepping past it, so that point is compensated again by every older segment
// (head h-1, ..., 0) — reproduced for point 0.  np < 2: the rows are only gathered.
// skeys == nullptr: every row is selected (the host selected them; no count to find); order == nullptr:
// the rows are already in time order (identity).  hcnt: host-mapped copy of the count.
// row i (< n): false when it is past the selected rows (writes the count at the boundary)
__device__ __forceinline__ bool undistort_row(const float* __restrict__ in, int64_t i, int64_t n, int stride, int tfield,
                                              const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ order,
                                              const ImuPose* __restrict__ poses, int np, const UndistortEnd& end,
                                              float* __restrict__ out, uint32_t* __restrict__ cnt,
                                              int* __restrict__ hcnt, const RowPieces& rp) {
    if (skeys) {
        const uint32_t key = skeys[i];
        if (key == kNotSelected) {
            if (i == 0 || skeys[i - 1] != kNotSelected) cnt[0] = (uint32_t)i, *hcnt = (int)i;
            return false;
        }
        if (i + 1 == n) cnt[0] = (uint32_t)n, *hcnt = (int)n;
    }
    const float* r = in + (size_t)piece_row(rp, order ? order[i] : (uint32_t)i) * stride;
    float* o = out + (size_t)i * stride;
    for (int f = 3; f < stride; ++f) o[f] = r[f];
    float q[3] = {r[0], r[1], r[2]};
    const float tms = r[tfield];
    if (np >= 2) {
        const double t = (double)tms / double(1000);
        int h = -1;
        for (int k = np - 2; k >= 0; --k)
            if (t > poses[k].offset_time) {
                h = k;
                break;
            }
        if (h >= 0) {
            compensate(q, tms, poses[h], poses[h + 1], end);
            if (i == 0)  // the time field is not changed by the compensation
                for (int k = h - 1; k >= 0; --k)
                    if (t > poses[k].offset_time) compensate(q, tms, poses[k], poses[k + 1], end);
        }
    }
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    return true;
}

__global__ void undistort_gather_kernel(const float* __restrict__ in, int64_t n, int stride, int tfield,
                                        const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ order,
                                        const ImuPose* __restrict__ poses, int np, UndistortEnd end,
                                        float* __restrict__ out, uint32_t* __restrict__ cnt, int* __restrict__ hcnt,
                                        RowPieces rp) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    (void)undistort_row(in, i, n, stride, tfield, skeys, order, poses, np, end, out, cnt, hcnt, rp);
}

// the same, with the block's AABB partial of the rows it wrote (part[6 blockIdx.x ..]) for the voxel grid
// that follows: no separate pass over the undistorted rows
__global__ void __launch_bounds__(256) undistort_gather_aabb_kernel(const float* __restrict__ in, int64_t n, int stride,
                                                                    int tfield, const uint32_t* __restrict__ skeys,
                                                                    const uint32_t* __restrict__ order,
                                                                    const ImuPose* __restrict__ poses, int np,
                                                                    UndistortEnd end, float* __restrict__ out,
                                                                    uint32_t* __restrict__ cnt, int* __restrict__ hcnt,
                                                                    RowPieces rp, float* __restrict__ part) {
    __shared__ float s[6][256];
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (i < n && undistort_row(in, i, n, stride, tfield, skeys, order, poses, np, end, out, cnt, hcnt, rp)) {
        const float* o = out + (size_t)i * stride;
        const float x = o[0], y = o[1], z = o[2];
        if (isfinite(x) && isfinite(y) && isfinite(z)) {
            lo[0] = x, lo[1] = y, lo[2] = z;
            hi[0] = x, hi[1] = y, hi[2] = z;
        }
    }
    block_minmax<256>(s, lo, hi);
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

#define FCHK(x)                           \
    do {                                  \
        if ((x) != hipSuccess) return -2; \
    } while (0)

template <class T>
int fgrow(T** p, int64_t& cap, int64_t need) {
    if (need <= cap && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const int64_t c = std::max<int64_t>(need, cap + cap / 2);
    count_alloc();
    if (hipMalloc(p, (size_t)c * sizeof(T)) != hipSuccess) {
        cap = 0;
        return -5;
    }
    cap = c;
    return 0;
}

int ftmp(FilterBuf& b, size_t need) {  // grown geometrically (1 MiB floor): no per-call re-allocation
    if (need <= b.tmp_bytes && b.tmp) return 0;
    if (b.tmp) (void)hipFree(b.tmp);
    b.tmp = nullptr;
    const size_t c = std::max(std::max(need, b.tmp_bytes + b.tmp_bytes / 2), (size_t)1 << 20);
    count_alloc();
    if (hipMalloc(&b.tmp, c) != hipSuccess) {
        b.tmp_bytes = 0;
        return -5;
    }
    b.tmp_bytes = c;
    return 0;
}

int reserve(FilterBuf& b, int64_t n) {
    if (n <= b.cap && b.keys) return 0;
    const int64_t c = std::max<int64_t>(std::max<int64_t>(n, b.cap + b.cap / 2), b.min_cap);
    void* bufs[] = {b.keys, b.keys_alt, b.vals, b.vals_alt, b.head, b.vid};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    count_alloc(6);
    FCHK(hipMalloc(&b.keys, c * sizeof(uint32_t)));
    FCHK(hipMalloc(&b.keys_alt, c * sizeof(uint32_t)));
    FCHK(hipMalloc(&b.vals, c * sizeof(uint32_t)));
    FCHK(hipMalloc(&b.vals_alt, c * sizeof(uint32_t)));
    FCHK(hipMalloc(&b.head, (c + 1) * sizeof(uint32_t)));
    FCHK(hipMalloc(&b.vid, (c + 1) * sizeof(uint32_t)));
    b.cap = c;
    if (!b.part) FCHK(hipMalloc(&b.part, 6 * kPartBlocks * sizeof(float)));
    if (!b.geom) FCHK(hipMalloc(&b.geom, sizeof(VoxelGeom)));
    if (!b.h_small) {
        FCHK(hipHostMalloc(&b.h_small, 256, hipHostMallocMapped));
        FCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&b.d_small), b.h_small, 0));
    }
    if (!b.cnt) {  // [0] selected count, [2] key-width flag (zero between launches)
        FCHK(hipMalloc(&b.cnt, 64));
        FCHK(hipMemset(b.cnt, 0, 64));
    }
    // the sort / scan scratch for the whole capacity now, so a call up to it never re-allocates the scratch
    size_t sb = 0, xb = 0;
    FCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, b.keys, b.keys_alt, b.vals, b.vals_alt, (int)c, 0, 32));
    FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, xb, b.head, b.vid, (int)(c + 1)));
    return ftmp(b, std::max(sb, xb));
}

int exscan(FilterBuf& b, const uint32_t* in, uint32_t* out, int64_t n1, hipStream_t st) {
    size_t bytes = 0;
    FCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)n1, st));
    if (ftmp(b, bytes)) return -5;
    bytes = b.tmp_bytes;
    FCHK(hipcub::DeviceScan::ExclusiveSum(b.tmp, bytes, in, out, (int)n1, st));
    return 0;
}

// stable sort of (keys, vals) on key bits [0, bits) into (keys_alt, vals_alt)
int sort_pairs(FilterBuf& b, int64_t n, hipStream_t st, int bits = 32) {
    size_t bytes = 0;
    FCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, b.keys, b.keys_alt, b.vals, b.vals_alt, (int)n, 0, bits, st));
    if (ftmp(b, bytes)) return -5;
    bytes = b.tmp_bytes;
    FCHK(hipcub::DeviceRadixSort::SortPairs(b.tmp, bytes, b.keys, b.keys_alt, b.vals, b.vals_alt, (int)n, 0, bits, st));
    return 0;
}

inline int nblk(int64_t n) { return (int)std::max<int64_t>(1, (n + 255) / 256); }

__global__ void records_xyz_kernel(const float* __restrict__ rec, int64_t n, int stride, float* __restrict__ xyz) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    xyz[3 * i] = rec[(size_t)i * stride];
    xyz[3 * i + 1] = rec[(size_t)i * stride + 1];
    xyz[3 * i + 2] = rec[(size_t)i * stride + 2];
}

// sensor_msgs/PointField datatypes: INT8 1, UINT8 2, INT16 3, UINT16 4, INT32 5,
// UINT32 6, FLOAT32 7, FLOAT64 8 (unaligned reads byte by byte)
__device__ __forceinline__ float read_field(const uint8_t* p, int dt, bool be) {
    uint8_t b[8];
    const int sz = (dt <= 2) ? 1 : (dt <= 4) ? 2 : (dt <= 7) ? 4 : 8;
    for (int k = 0; k < sz; ++k) b[k] = be ? p[sz - 1 - k] : p[k];
    switch (dt) {
        case 1: return (float)(int8_t)b[0];
        case 2: return (float)b[0];
        case 3: return (float)(int16_t)(b[0] | (b[1] << 8));
        case 4: return (float)(uint16_t)(b[0] | (b[1] << 8));
        case 5: return (float)(int32_t)(b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24));
        case 6: return (float)(uint32_t)(b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24));
        case 7: return __uint_as_float(b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24));
        case 8: {
            uint64_t v = 0;
            for (int k = 7; k >= 0; --k) v = (v << 8) | b[k];
            return (float)__longlong_as_double((long long)v);
        }
        default: return 0.f;
    }
}

// one thread per point: record field f = value(offset_f, datatype_f) * scale_f (scale 1 => exact copy)
__global__ void cloud_decode_kernel(const uint8_t* __restrict__ data, int64_t n, int point_step, int be,
                                    CloudField fl0, CloudField fl1, CloudField fl2, CloudField fl3, CloudField fl4,
                                    CloudField fl5, CloudField fl6, CloudField fl7, int nf, float* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const CloudField fl[kMaxFields] = {fl0, fl1, fl2, fl3, fl4, fl5, fl6, fl7};
    const uint8_t* rec = data + (size_t)i * point_step;
#pragma unroll
    for (int f = 0; f < kMaxFields; ++f) {
        if (f >= nf) break;
        float v = fl[f].datatype ? read_field(rec + fl[f].offset, fl[f].datatype, be != 0) : 0.f;
        if (fl[f].scale != 1.f) v *= fl[f].scale;
        out[(size_t)i * nf + f] = v;
    }
}

// float records -> little-endian FLOAT32 fields at the given offsets (other bytes zero)
__global__ void cloud_encode_kernel(const float* __restrict__ rec, int64_t n, int stride, int point_step,
                                    CloudField fl0, CloudField fl1, CloudField fl2, CloudField fl3, CloudField fl4,
                                    CloudField fl5, CloudField fl6, CloudField fl7, int nf, uint8_t* __restrict__ data) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const CloudField fl[kMaxFields] = {fl0, fl1, fl2, fl3, fl4, fl5, fl6, fl7};
    uint8_t* o = data + (size_t)i * point_step;
    for (int k = 0; k < point_step; ++k) o[k] = 0;
    for (int f = 0; f < nf && f < stride; ++f) {
        if (fl[f].datatype != 7) continue;
        const uint32_t b = __float_as_uint(rec[(size_t)i * stride + f]);
        uint8_t* d = o + fl[f].offset;
        d[0] = (uint8_t)b;
        d[1] = (uint8_t)(b >> 8);
        d[2] = (uint8_t)(b >> 16);
        d[3] = (uint8_t)(b >> 24);
    }
}

}  // namespace

int cloud_decode(const uint8_t* d_data, int64_t n, int point_step, bool big_endian, const CloudField* fields, int nf,
                 float* d_out, hipStream_t st) {
    if (n <= 0) return 0;
    if (nf < 1 || nf > kMaxFields || point_step <= 0) return -1;
    CloudField f[kMaxFields] = {};
    for (int k = 0; k < nf; ++k) f[k] = fields[k];
    cloud_decode_kernel<<<nblk(n), 256, 0, st>>>(d_data, n, point_step, big_endian ? 1 : 0, f[0], f[1], f[2], f[3],
                                                 f[4], f[5], f[6], f[7], nf, d_out);
    FCHK(hipGetLastError());
    return 0;
}

int cloud_encode(const float* d_rec, int64_t n, int stride, int point_step, const CloudField* fields, int nf,
                 uint8_t* d_data, hipStream_t st) {
    if (n <= 0) return 0;
    if (nf < 1 || nf > kMaxFields || point_step <= 0) return -1;
    CloudField f[kMaxFields] = {};
    for (int k = 0; k < nf; ++k) f[k] = fields[k];
    cloud_encode_kernel<<<nblk(n), 256, 0, st>>>(d_rec, n, stride, point_step, f[0], f[1], f[2], f[3], f[4], f[5],
                                                 f[6], f[7], nf, d_data);
    FCHK(hipGetLastError());
    return 0;
}

__global__ void records_xyz_sel_kernel(const float* __restrict__ rec, int64_t n, int stride, float* __restrict__ xyz,
                                       uint8_t* __restrict__ sel) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    xyz[3 * i] = rec[(size_t)i * stride];
    xyz[3 * i + 1] = rec[(size_t)i * stride + 1];
    xyz[3 * i + 2] = rec[(size_t)i * stride + 2];
    sel[i] = 0;
}

int records_to_xyz_sel(const float* d_rec, int64_t n, int stride, float* d_xyz, uint8_t* sel, hipStream_t st) {
    if (n <= 0) return 0;
    records_xyz_sel_kernel<<<nblk(n), 256, 0, st>>>(d_rec, n, stride, d_xyz, sel);
    FCHK(hipGetLastError());
    return 0;
}

int records_to_xyz(const float* d_rec, int64_t n, int stride, float* d_xyz, hipStream_t st) {
    if (n <= 0) return 0;
    records_xyz_kernel<<<nblk(n), 256, 0, st>>>(d_rec, n, stride, d_xyz);
    FCHK(hipGetLastError());
    return 0;
}

void filter_free(FilterBuf& b) {
    void* bufs[] = {b.keys, b.keys_alt, b.vals, b.vals_alt, b.head, b.vid,
                    b.part, b.geom,     b.tmp,  b.a,    b.c,        b.aux,  b.cnt};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (b.h_small) (void)hipHostFree(b.h_small);
    if (b.h_stage) (void)hipHostFree(b.h_stage);
    b = FilterBuf{};
}

// Everything up to the centroids; the voxel count, the geometry and the key-width flag land in the
// host-mapped b.h_small ([0], [1..], [kHostFlags]) behind them: nothing waits for the device, nothing is
// copied.  cnt (optional, device): rows in use <= n.  The voxel sort uses b.vox_bits key bits (learnt from
// the previous call; a key past them raises the flag and the caller runs the call again at full width).
// nbp > 0: the producer of d_in already wrote nbp AABB partials into b.part (undistort_gather_aabb_kernel)
int voxel_grid_enqueue(FilterBuf& b, const float* d_in, int64_t n, const uint32_t* cnt, int stride, const float leaf[3],
                       float* d_out, hipStream_t st, float* xyz = nullptr, uint8_t* sel = nullptr, int nbp = 0) {
    if (stride < 3 || stride > kMaxFields || n >= (int64_t)0x7fffffff) return -1;
    if (reserve(b, n)) return -5;
    auto* hgeom = reinterpret_cast<VoxelGeom*>(b.d_small + 1);
    if (nbp <= 0) {  // no producer wrote the AABB partials: one pass over the input
        if (cnt) return -1;  // (the scan path's rows in use come with the undistortion's partials)
        nbp = (int)std::min<int64_t>(1024, (n + 255) / 256);
        minmax_partial_kernel<<<nbp, 256, 0, st>>>(d_in, n, stride, b.part);
    }
    const int bits = std::min(std::max(b.vox_bits, 1), 32);
    voxel_key_kernel<<<nblk(n), 256, 0, st>>>(d_in, n, cnt, stride, b.part, nbp, leaf[0], leaf[1], leaf[2], hgeom,
                                              b.keys, b.vals, bits, b.cnt + 2);
    int rc = sort_pairs(b, n, st, bits);
    if (rc) return rc;
    // runs -> [start, end) per voxel (b.keys / b.vals are free after the sort); the count at b.vid[n]
    if (runs_one_block(n)) {
        voxel_runs_block_kernel<<<1, 1024, 0, st>>>(b.keys_alt, n, b.keys, b.vals, b.vid + n, b.cnt + 2, b.d_small);
    } else {
        run_head_kernel<<<nblk(n + 1), 256, 0, st>>>(b.keys_alt, n, b.head);
        rc = exscan(b, b.head, b.vid, n + 1, st);
        if (rc) return rc;
        voxel_bounds_kernel<<<nblk(n), 256, 0, st>>>(b.keys_alt, n, b.head, b.vid, b.keys, b.vals, b.cnt + 2,
                                                     b.d_small);
    }
    const int nbw = (int)std::min<int64_t>(kWaveCentroidBlocks, (n + 3) / 4);
    voxel_centroid_wave_kernel<<<std::max(nbw, 1), 256, 0, st>>>(d_in, stride, b.vals_alt, b.keys, b.vals, b.vid + n,
                                                                 d_out, xyz, sel);
    FCHK(hipGetLastError());
    return 0;
}

// After the stream has drained: the voxel count; 2 when the key width was too narrow (b.vox_bits reset to
// 32: enqueue again), or 1 for PCL's "Leaf size is too small ... Integer indices would overflow": the m
// input rows copied to the output (the copy is enqueued, not waited on).  Learns the next call's key width.
static int voxel_grid_result(FilterBuf& b, const float* d_in, int64_t m, int stride, float* d_out, int64_t* n_out,
                             hipStream_t st) {
    VoxelGeom g;
    std::memcpy(&g, b.h_small + 1, sizeof(VoxelGeom));
    const bool narrow = b.h_small[kHostFlags] != 0;
    b.h_small[kHostFlags] = 0;
    if (narrow && !g.overflow) {
        b.vox_bits = 32;
        return 2;
    }
    // one spare bit: a sweep's extent may grow a little before the next call has to repeat itself
    b.vox_bits = g.overflow ? 32 : std::min(32, g.key_bits + 1);
    if (g.overflow) {
        if (m > 0) copy_strided_kernel<<<nblk(m * stride), 256, 0, st>>>(d_in, m * stride, d_out);
        FCHK(hipGetLastError());
        *n_out = m;
        return 1;
    }
    *n_out = (uint32_t)b.h_small[0];
    return 0;
}

int voxel_grid(FilterBuf& b, const float* d_in, int64_t n, int stride, const float leaf[3], float* d_out,
               int64_t* n_out, hipStream_t st) {
    *n_out = 0;
    if (n <= 0) return 0;
    int rc = 2;
    for (int attempt = 0; attempt < 2 && rc == 2; ++attempt) {
        rc = voxel_grid_enqueue(b, d_in, n, nullptr, stride, leaf, d_out, st);
        if (rc) return rc;
        FCHK(hipStreamSynchronize(st));
        rc = voxel_grid_result(b, d_in, n, stride, d_out, n_out, st);
    }
    if (rc < 0 || rc == 2) return rc < 0 ? rc : -2;
    if (rc == 1) FCHK(hipStreamSynchronize(st));
    return 0;
}

int transform_segments(const float* d_in, int64_t n, int stride, const int64_t* d_seg_off, int nseg,
                       const double* d_T16, float* d_out, hipStream_t st) {
    if (n <= 0) return 0;
    if (stride < 3) return -1;
    transform_segs_kernel<<<nblk(n), 256, 0, st>>>(d_in, n, stride, d_seg_off, nseg, d_T16, d_out);
    FCHK(hipGetLastError());
    return 0;
}

// fast_lio_sam's keyframe cloud, fused: FAST-LIO publishes /cloud_registered = feats_undistort through
// pointBodyToWorld (laserMapping [U]: double, stored float; dense_publish_en, kitti.yaml:31) and
// PosePcd takes it back with transformPcd(cloud, pose_eig_.inverse()) (pose_pcd.hpp:22-42,
// utilities.hpp:132-143: ((m0 x + m1 y) + m2 z) + m3 in double, stored float; other fields copied).
struct Mat16d {
    double m[16];
};
__global__ void keyframe_cloud_kernel(const float* __restrict__ rec, int64_t n, int stride, PoseArg ps, Mat16d T,
                                      float* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* q = rec + (size_t)i * stride;
    float wx, wy, wz;
    body_to_world(ps, q[0], q[1], q[2], wx, wy, wz);
    const double x = wx, y = wy, z = wz;
    const double* m = T.m;
    float* o = out + 4 * (size_t)i;
    o[0] = (float)(((m[0] * x + m[1] * y) + m[2] * z) + m[3]);
    o[1] = (float)(((m[4] * x + m[5] * y) + m[6] * z) + m[7]);
    o[2] = (float)(((m[8] * x + m[9] * y) + m[10] * z) + m[11]);
    o[3] = q[3];
}

int keyframe_cloud(const float* d_rec, int64_t n, int stride, const PoseArg& ps, const double* T16, float* d_out,
                   hipStream_t st) {
    if (n <= 0) return 0;
    if (stride < 4) return -1;
    Mat16d T;
    for (int k = 0; k < 16; ++k) T.m[k] = T16[k];
    keyframe_cloud_kernel<<<nblk(n), 256, 0, st>>>(d_rec, n, stride, ps, T, d_out);
    FCHK(hipGetLastError());
    return 0;
}

int scan_preprocess_enqueue(FilterBuf& b, const float* d_raw, int64_t n, int stride, const ScanPrepParams& p,
                            const ImuPose* d_poses, int np, const UndistortEnd& end, float* d_out, hipStream_t st,
                            int presel, float* xyz, uint8_t* sel, const RowPieces& rp) {
    b.prep_n = 0;
    b.prep_sel = -1;
    if (n <= 0) return 0;
    if (stride < 4 || stride > kMaxFields || p.time_field < 3 || p.time_field >= stride || n >= (int64_t)0x7fffffff)
        return -1;
    if (reserve(b, n)) return -5;
    int rc = fgrow(&b.c, b.c_cap, n * stride);
    if (rc) return rc;
    const uint32_t* cnt = nullptr;  // rows in use past this point: all n (host selection) or b.cnt[0]
    // the undistortion writes the AABB partials of its rows when the voxel grid follows (one pass fewer)
    const bool fuse = p.leaf > 0.f && nblk(n) <= kPartBlocks;
    auto undistort = [&](const uint32_t* skeys, const uint32_t* order, const RowPieces& pr) {
        if (fuse)
            undistort_gather_aabb_kernel<<<nblk(n), 256, 0, st>>>(d_raw, n, stride, p.time_field, skeys, order, d_poses,
                                                                  np, end, b.c, b.cnt, b.d_small + kHostSel, pr, b.part);
        else
            undistort_gather_kernel<<<nblk(n), 256, 0, st>>>(d_raw, n, stride, p.time_field, skeys, order, d_poses, np,
                                                             end, b.c, b.cnt, b.d_small + kHostSel, pr);
    };
    if (presel == 1) {  // selected and already in time order: the stable sort is the identity
        undistort(nullptr, nullptr, rp);
    } else if (presel == 0) {  // selected, times out of order: stable sort by time
        scan_key_kernel<<<nblk(n), 256, 0, st>>>(d_raw, n, stride, 0, 0.f, p.time_field, b.keys, b.vals, rp);
        rc = sort_pairs(b, n, st);
        if (rc) return rc;
        undistort(nullptr, b.vals_alt, rp);
    } else {
        // 1. Preprocess selection + 2. stable time sort in one sort over the n rows (the selected first),
        // 3. gather + undistort; the selected count stays on the device (b.cnt[0]) and in b.h_small
        const int every = p.point_filter_num > 0 ? p.point_filter_num : 1;
        scan_key_kernel<<<nblk(n), 256, 0, st>>>(d_raw, n, stride, every, p.blind * p.blind, p.time_field, b.keys,
                                                 b.vals, RowPieces{});
        rc = sort_pairs(b, n, st);
        if (rc) return rc;
        undistort(b.keys_alt, b.vals_alt, RowPieces{});
        cnt = b.cnt;
    }
    // 4. downSizeFilterSurf
    b.prep_leaf = p.leaf > 0.f;
    b.prep_n = n;
    b.prep_sel = presel >= 0 ? n : -1;
    if (b.prep_leaf) {
        const float leaf[3] = {p.leaf, p.leaf, p.leaf};
        if (!fuse && cnt) {  // more rows than partial slots on the device-selection path: a separate AABB pass
            minmax_partial_cnt_kernel<<<1024, 256, 0, st>>>(b.c, n, cnt, stride, b.part);
            return voxel_grid_enqueue(b, b.c, n, cnt, stride, leaf, d_out, st, xyz, sel, 1024);
        }
        return voxel_grid_enqueue(b, b.c, n, cnt, stride, leaf, d_out, st, xyz, sel, fuse ? nblk(n) : 0);
    }
    FCHK(hipMemcpyAsync(d_out, b.c, (size_t)n * stride * sizeof(float), hipMemcpyDeviceToDevice, st));
    return 0;
}

int scan_preprocess_finish(FilterBuf& b, int stride, float* d_out, int64_t* n_out, int64_t* n_undist, hipStream_t st) {
    *n_out = 0;
    if (n_undist) *n_undist = 0;
    FCHK(hipStreamSynchronize(st));
    if (b.prep_n <= 0) return 0;
    const int64_t m = b.prep_sel >= 0 ? b.prep_sel : (uint32_t)b.h_small[kHostSel];
    if (n_undist) *n_undist = m;
    if (!b.prep_leaf) {
        *n_out = m;
        return 0;
    }
    return voxel_grid_result(b, b.c, m, stride, d_out, n_out, st);
}

int scan_preprocess(FilterBuf& b, const float* d_raw, int64_t n, int stride, const ScanPrepParams& p,
                    const ImuPose* d_poses, int np, const UndistortEnd& end, float* d_out, int64_t* n_out,
                    hipStream_t st, int64_t* n_undist) {
    *n_out = 0;
    if (n_undist) *n_undist = 0;
    int rc = 2;
    for (int attempt = 0; attempt < 2 && rc == 2; ++attempt) {  // 2: the voxel key width was learnt too narrow
        rc = scan_preprocess_enqueue(b, d_raw, n, stride, p, d_poses, np, end, d_out, st);
        if (rc) return rc;
        rc = scan_preprocess_finish(b, stride, d_out, n_out, n_undist, st);
    }
    if (rc < 0 || rc == 2) return rc < 0 ? rc : -2;
    if (rc == 1) FCHK(hipStreamSynchronize(st));
    return 0;
}

}  // namespace lio
