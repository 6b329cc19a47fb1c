// lio_pcl.hip — the float statistics of pcl::umeyama for the ICP fidelity modes (lio_icp_params.umeyama_float).
//
// PCL 1.10 TransformationEstimationSVD<PointXYZI, PointXYZI, float> (use_umeyama_) hands the accepted
// correspondences, in source order, to pcl::umeyama(cloud_src, cloud_tgt, false) (common/impl/eigen.hpp,
// Eigen 3.3 Umeyama.h) [U]:
//   src_mean = src.rowwise().sum() * one_over_n      one sequential float chain per row (Eigen's redux of a
//   dst_mean = dst.rowwise().sum() * one_over_n      strided row starts from the first coefficient)
//   sigma    = one_over_n * dst_demean * src_demean^T  order 1: one sequential chain per entry, scaled at
//              the end; orders 2 / 3: Eigen 3.3's GEMM, the depth blocked by kc(L1 32 / 48 KiB) and
//              res += alpha * (block's sequential sum) per block (oracle/lio_oracle.cpp UmeyamaOrder)
// Here:
//   (icp_stats_kernel, IcpCompact)       the accepted pairs compacted in source order by the statistics launch
//                                        (one look-back over the 4096-point records)
//   seqsum (lio_seqsum.hip)              the six mean chains (and order 1's nine sigma chains), bit-exact
//                                        sequential float results computed in parallel
//   pcl_sigma_blocks                     orders 2 / 3: one wave per kc block, nine sequential lanes from LDS
//   pcl_pack                             res += alpha * C_b in block order; sums, count, sigma, status
// Sharded (lio_icp_host.cpp fid_sharded): each rank compacts its window of the source (the windows in rank
// order are the correspondence order); the chains are split over the windows (lio_seqsum.hpp seqsum_shard_*),
// the depth blocks are summed by the rank holding their first pair (pcl_sigma_shard) and gathered in block
// order (pcl_x3_merge) for pcl_pack.
#include "lio_error.hpp"
#include "lio_kernels.hpp"
#include "lio_pcl.hpp"

#include <algorithm>

namespace lio {

namespace {

constexpr int kMaxKc = kPclMaxKc;  // kc at a 48 KiB L1 (the largest modelled)
constexpr int kPackWin = 1024;     // GEMM depth blocks staged per window in pcl_pack (36 KiB of LDS)

// float means of the sequential sums (order 1's sigma chains read them)
__global__ void pcl_mean6_kernel(const float* __restrict__ sums6, const uint32_t* __restrict__ d_n,
                                 float* __restrict__ mean6) {
    const uint32_t n = *d_n;
    const float oon = 1.f / (float)n;
    if (threadIdx.x < 6) mean6[threadIdx.x] = sums6[threadIdx.x] * oon;
}

// orders 2 / 3: block q of the depth = pairs [q kc, (q + 1) kc): lane e < 9 (r = e / 3, c = e % 3) adds
// (tgt_r - dm_r) * (src_c - sm_c) in order from 0 (gebp's 1 x 1 remainder path: C0 += A0 * B0, no FMA).  256
// threads stage the block (4 loads per column each; 64 threads: 14.4 us per launch at C4 pair B, 256: 12.0), nine add.
constexpr int kSigThreads = 256;
__global__ void __launch_bounds__(kSigThreads) pcl_sigma_blocks_kernel(const float* __restrict__ pairs, int64_t cap,
                                                                       const uint32_t* __restrict__ d_n,
                                                                       const float* __restrict__ sums6, int l1,
                                                                       float* __restrict__ Cb) {
    __shared__ float s[6][kMaxKc];
    const uint32_t n = *d_n;
    if (n + 6 < 20) return;  // the lazy coefficient-based product: pcl_pack
    const int64_t kc = eigen_gemm_kc((int64_t)n, l1);
    const int64_t nkc = ((int64_t)n + kc - 1) / kc;
    const int lane = threadIdx.x;
    const float oon = 1.f / (float)n;
    const int r = lane / 3, c = lane % 3;
    const float dm = lane < 9 ? sums6[3 + r] * oon : 0.f;
    const float sm = lane < 9 ? sums6[c] * oon : 0.f;
    for (int64_t q = blockIdx.x; q < nkc; q += gridDim.x) {
        const int64_t k0 = q * kc;
        const int cnt = (int)((int64_t)n - k0 < kc ? (int64_t)n - k0 : kc);
        {  // coalesced per column; all six columns' loads in flight together (one round trip)
            constexpr int T = (kMaxKc + kSigThreads - 1) / kSigThreads;
            float v[6][T];
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int j = t * kSigThreads + lane;
                    v[d][t] = j < cnt ? pairs[d * cap + k0 + j] : 0.f;
                }
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int t = 0; t < T; ++t)
                    if (t * kSigThreads + lane < cnt) s[d][t * kSigThreads + lane] = v[d][t];
        }
        __syncthreads();
        if (lane < 9) {
            const float* dv = s[3 + r];
            const float* sv = s[c];
            float C0 = 0.f;
            int j = 0;
            for (; j + 8 <= cnt; j += 8) {
                float p[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) p[u] = (dv[j + u] - dm) * (sv[j + u] - sm);
#pragma unroll
                for (int u = 0; u < 8; ++u) C0 += p[u];
            }
            for (; j < cnt; ++j) C0 += (dv[j] - dm) * (sv[j] - sm);
            Cb[q * 9 + lane] = C0;
        }
        __syncthreads();
    }
}

// out[0..5] float sums (src xyz, tgt xyz), out[6] count bits, out[7 + 3r + c] sigma (orders 2 / 3: scaled by
// one_over_n as Eigen leaves it; order 1: the raw sequential accumulator, scaled on the host), out[16]
// verification failures (means bits 0-5, sigma chains 8-16), out[17] event-list overflows (same bits)
constexpr int kPackThreads = 1024;  // the staging loads spread wide; lanes 0 .. 8 then add in order
__global__ void __launch_bounds__(kPackThreads) pcl_pack_kernel(const float* __restrict__ pairs, int64_t cap,
                                                      const uint32_t* __restrict__ d_n,
                                                      const float* __restrict__ sums6, const float* __restrict__ sig9,
                                                      const float* __restrict__ Cb, int order, int l1,
                                                      const uint32_t* __restrict__ st_means,
                                                      const uint32_t* __restrict__ st_sig,
                                                      const int* __restrict__ nev6, const uint32_t* __restrict__ flags,
                                                      float* __restrict__ out, uint32_t seq) {
    __shared__ float s_c[9][kPackWin + 1];  // +1: the nine lanes' rows in different banks
    const uint32_t n = *d_n;
    const int lane = threadIdx.x;
    const float oon = 1.f / (float)n;
    if (lane < 6) out[lane] = sums6[lane];
    if (lane == 6) out[6] = __uint_as_float(n);
    const int r = lane / 3, c = lane % 3;
    float res = 0.f;
    if (order == 1 || n == 0) {
        if (lane < 9) res = order == 1 ? sig9[lane] : 0.f;
    } else if (n + 6 < 20) {
        // generic_product_impl::evalTo below EIGEN_GEMM_TO_COEFFBASED_THRESHOLD: the lazy product,
        // (alpha * dst_demean).row(r) . src_demean.row(c) summed from the first term
        if (lane < 9) {
            const float dm = sums6[3 + r] * oon, sm = sums6[c] * oon;
            const float* tr = pairs + (3 + r) * cap;
            const float* sc = pairs + c * cap;
            res = (oon * (tr[0] - dm)) * (sc[0] - sm);
            for (uint32_t k = 1; k < n; ++k) res += (oon * (tr[k] - dm)) * (sc[k] - sm);
        }
    } else {
        const int64_t kc = eigen_gemm_kc((int64_t)n, l1);
        const int64_t nkc = ((int64_t)n + kc - 1) / kc;
        for (int64_t q0 = 0; q0 < nkc; q0 += kPackWin) {  // dst.setZero(); res(r, c) += alpha * C0 per depth block
            const int m = (int)(nkc - q0 < kPackWin ? nkc - q0 : kPackWin);
            for (int e0 = 0; e0 < 9 * m; e0 += kPackThreads * 9) {  // the window in one round trip (9 loads per thread)
                float v[9];
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int e = e0 + t * kPackThreads + lane;
                    v[t] = e < 9 * m ? Cb[q0 * 9 + e] : 0.f;
                }
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int e = e0 + t * kPackThreads + lane;
                    if (e < 9 * m) s_c[e % 9][e / 9] = v[t];
                }
            }
            __syncthreads();
            if (lane < 9) {
                int q = 0;
                for (; q + 8 <= m; q += 8) {  // the LDS reads ahead of the dependent adds
                    float t[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) t[u] = oon * s_c[lane][q + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) res = res + t[u];
                }
                for (; q < m; ++q) res = res + oon * s_c[lane][q];
            }
            __syncthreads();
        }
    }
    if (lane < 9) out[7 + lane] = res;
    if (lane == 0) {
        const uint32_t f = (st_means[0] & 0x3fu) | (order == 1 ? (st_sig[0] & 0x1ffu) << 8 : 0u);
        const uint32_t o = (st_means[1] & 0x3fu) | (order == 1 ? (st_sig[1] & 0x1ffu) << 8 : 0u);
        out[16] = __uint_as_float(f);
        out[17] = __uint_as_float(o);
        int ev = 0;
        if (nev6)
            for (int k = 0; k < 6; ++k) ev = max(ev, nev6[k]);
        out[18] = __int_as_float(ev);
        out[19] = __uint_as_float(flags ? *flags : 0u);  // compaction look-back timed out (never expected)
    }
    if (seq) {
        // out host-mapped, the host polling out[23]: every word above stored and drained, then the sequence
        // number behind a system-scope release
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lane == 0) {
            __threadfence_system();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(reinterpret_cast<uint32_t*>(out + 23), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------- sharded statistics
// depth blocks [q0, q1) of the whole chain (q0 = the first block starting in this window), each summed as in
// pcl_sigma_blocks_kernel from the window's pairs and the ones appended after it; the results (9 floats per
// block) and the header (the ranks' statuses, q0, the block count) into the message
__global__ void __launch_bounds__(64) pcl_sigma_shard_kernel(const float* __restrict__ pairs, int64_t cap,
                                                             const uint32_t* __restrict__ d_n, const SeqShard* __restrict__ sh,
                                                             const float* __restrict__ sums6, int l1,
                                                             const uint32_t* __restrict__ st_means,
                                                             const uint32_t* __restrict__ lb_flag, double* __restrict__ msg,
                                                             int64_t nq_slot) {
    __shared__ float s[6][kMaxKc];
    const int64_t nl = *d_n, gb = sh->gbase, n = sh->n_global;
    const int lane = threadIdx.x;
    const bool blocked = n + 6 >= 20;  // below: the lazy product (pcl_pack)
    const int64_t kc = blocked ? eigen_gemm_kc(n, l1) : 1;
    const int64_t q0 = blocked ? (gb + kc - 1) / kc : 0, q1 = blocked ? (gb + nl + kc - 1) / kc : 0;
    if (blockIdx.x == 0 && lane == 0) {
        msg[0] = (double)(st_means[0] & 0x3fu);  // this rank's verification failures
        msg[1] = 0.0;
        msg[2] = (double)(lb_flag ? *lb_flag : 0u);
        msg[3] = (double)q0;
        msg[4] = (double)min(q1 - q0, nq_slot);
        msg[5] = (double)(q1 - q0 > nq_slot ? 1 : 0);  // more blocks than the slot (never with pcl_blocks_slot)
    }
    if (!blocked || nl == 0) return;
    float* Cb = reinterpret_cast<float*>(msg + kPclX3Hdr);
    const float oon = 1.f / (float)n;
    const int r = lane / 3, c = lane % 3;
    const float dm = lane < 9 ? sums6[3 + r] * oon : 0.f;
    const float sm = lane < 9 ? sums6[c] * oon : 0.f;
    for (int64_t q = q0 + blockIdx.x; q < min(q1, q0 + nq_slot); q += gridDim.x) {
        const int64_t k0 = q * kc - gb;  // in the window's pairs (the tail of the last block: the appended ones)
        const int cnt = (int)(n - q * kc < kc ? n - q * kc : kc);
        {
            constexpr int T = (kMaxKc + 63) / 64;
            float v[6][T];
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int j = t * 64 + lane;
                    v[d][t] = j < cnt ? pairs[d * cap + k0 + j] : 0.f;
                }
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int t = 0; t < T; ++t)
                    if (t * 64 + lane < cnt) s[d][t * 64 + lane] = v[d][t];
        }
        __syncthreads();
        if (lane < 9) {
            const float* dv = s[3 + r];
            const float* sv = s[c];
            float C0 = 0.f;
            int j = 0;
            for (; j + 8 <= cnt; j += 8) {
                float pp[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) pp[u] = (dv[j + u] - dm) * (sv[j + u] - sm);
#pragma unroll
                for (int u = 0; u < 8; ++u) C0 += pp[u];
            }
            for (; j < cnt; ++j) C0 += (dv[j] - dm) * (sv[j] - sm);
            Cb[(q - q0) * 9 + lane] = C0;
        }
        __syncthreads();
    }
}

// order 1: the header only (no depth blocks), the sigma chains' statuses beside the means'
__global__ void pcl_x3_header_kernel(const uint32_t* __restrict__ st_means, const uint32_t* __restrict__ st_sig,
                                     const uint32_t* __restrict__ lb_flag, double* __restrict__ msg) {
    msg[0] = (double)(st_means[0] & 0x3fu);
    msg[1] = (double)(st_sig ? st_sig[0] & 0x1ffu : 0u);
    msg[2] = (double)(lb_flag ? *lb_flag : 0u);
    msg[3] = 0.0;
    msg[4] = 0.0;
    msg[5] = 0.0;
}

// every rank's depth blocks into Cbg (global order; block r copies rank r's), the statuses OR-ed (block 0):
// merged = {means bad, means overflow, sigma bad, sigma overflow, look-back}; the overflow words are the seqsum
// merges' (already global); out[20..22]
__global__ void __launch_bounds__(256) pcl_x3_merge_kernel(const double* __restrict__ recv, int64_t stride, int world,
                                                           float* __restrict__ Cbg, int64_t Cbg_cap,
                                                           const uint32_t* __restrict__ over_means,
                                                           const uint32_t* __restrict__ over_sig,
                                                           const SeqShard* __restrict__ shm, const SeqShard* __restrict__ shs,
                                                           uint32_t* __restrict__ merged, float* __restrict__ out) {
    {
        const double* m = recv + (size_t)blockIdx.x * (size_t)stride;
        const int64_t q0 = (int64_t)m[3], nq = (int64_t)m[4];
        const float* cb = reinterpret_cast<const float*>(m + kPclX3Hdr);
        for (int64_t e = threadIdx.x; e < 9 * nq; e += 256)
            if (q0 * 9 + e < 9 * Cbg_cap) Cbg[q0 * 9 + e] = cb[e];
    }
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint32_t o0 = 0u, o1 = 0u, o2 = 0u, o3 = 0u;
    for (int r = 0; r < world; ++r) {
        const double* m = recv + (size_t)r * (size_t)stride;
        o0 |= (uint32_t)m[0];
        o1 |= (uint32_t)m[1];
        o2 |= (uint32_t)m[2];
        o3 |= (uint32_t)m[5];
    }
    merged[0] = o0;
    merged[1] = over_means[1] | (o3 ? 0x3fu : 0u);
    merged[2] = o1;
    merged[3] = over_sig ? over_sig[1] : 0u;
    merged[4] = o2;
    const uint32_t xf = (shm ? shm->xflags : 0u) | (shs ? shs->xflags << 8 : 0u) | (o3 ? 4u : 0u);
    out[20] = __uint_as_float(xf);
    out[21] = __int_as_float(shm ? shm->max_nev : 0);
    out[22] = __int_as_float(shs ? shs->max_nev : 0);
}

__global__ void __launch_bounds__(256) pcl_gather_pack_kernel(const float* __restrict__ pairs, int64_t cap,
                                                              const uint32_t* __restrict__ d_n, int64_t round, int64_t chunk,
                                                              double* __restrict__ msg) {
    const int64_t n = *d_n;
    if (blockIdx.x == 0 && threadIdx.x == 0) msg[0] = (double)n;
    float* out = reinterpret_cast<float*>(msg + 2);
    const int64_t b = round * chunk;
    for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < 6 * chunk; e += (int64_t)gridDim.x * 256) {
        const int d = (int)(e / chunk);
        const int64_t j = e % chunk;
        out[e] = b + j < n ? pairs[d * cap + b + j] : 0.f;
    }
}

__global__ void __launch_bounds__(256) pcl_gather_unpack_kernel(const double* __restrict__ recv, int64_t stride, int world,
                                                                int64_t round, int64_t chunk, float* __restrict__ pairs,
                                                                int64_t cap, uint32_t* __restrict__ n_all) {
    int64_t base = 0;
    for (int r = 0; r < world; ++r) {  // block-uniform
        const double* m = recv + (size_t)r * (size_t)stride;
        const int64_t nr = (int64_t)m[0];
        const int64_t b = round * chunk, take = max((int64_t)0, min(chunk, nr - b));
        const float* in = reinterpret_cast<const float*>(m + 2);
        for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < 6 * take; e += (int64_t)gridDim.x * 256) {
            const int d = (int)(e / take);
            const int64_t j = e % take;
            if (base + b + j < cap) pairs[d * cap + base + b + j] = in[d * chunk + j];
        }
        base += nr;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_all = (uint32_t)base;
}

}  // namespace

int pcl_reserve_plain(PclBuf& p, int64_t n, hipStream_t st) {
    n = n < 1 ? 1 : n;
    if (n > p.cap) {
        n = std::max<int64_t>(n + n / 2, 2 * p.cap);
        count_alloc(2);
        for (void* q : {(void*)p.pairs, (void*)p.Cb})
            if (q) (void)hipFree(q);
        p.pairs = nullptr;
        p.Cb = nullptr;
        p.cap = 0;
        if (hipMalloc(&p.pairs, (size_t)n * 6 * sizeof(float)) != hipSuccess ||
            hipMalloc(&p.Cb, (size_t)(n / 340 + 2) * 9 * sizeof(float)) != hipSuccess)
            return -5;
        p.cap = n;
    }
    if (!p.small) {
        count_alloc();
        if (hipMalloc(&p.small, 64 * sizeof(float)) != hipSuccess) return -5;
        (void)hipMemsetAsync(p.small, 0, 64 * sizeof(float), st);
    }
    return 0;
}

int pcl_shard_reserve(PclBuf& p, int64_t n_blocks_global, hipStream_t st) {
    if (!p.ghead || !p.merged) {
        count_alloc(2);
        if (hipMalloc(&p.ghead, 6 * kPclTinyN * sizeof(float)) != hipSuccess ||
            hipMalloc(&p.merged, kPclMerged * sizeof(uint32_t)) != hipSuccess)
            return -5;
        (void)hipMemsetAsync(p.merged, 0, kPclMerged * sizeof(uint32_t), st);
    }
    if (n_blocks_global > p.Cbg_cap) {
        const int64_t c = std::max<int64_t>(n_blocks_global + n_blocks_global / 2, 2 * p.Cbg_cap);
        if (p.Cbg) (void)hipFree(p.Cbg);
        p.Cbg = nullptr;
        p.Cbg_cap = 0;
        count_alloc();
        if (hipMalloc(&p.Cbg, (size_t)c * 9 * sizeof(float)) != hipSuccess) return -5;
        p.Cbg_cap = c;
    }
    return 0;
}

void launch_pcl_sigma_shard(PclBuf& p, int order, double* msg3, int64_t nq_slot, hipStream_t st) {
    const uint32_t* lb = p.small + kPclTicket + 1;
    if (order == 1) {
        pcl_x3_header_kernel<<<1, 1, 0, st>>>(p.means.status, p.sig.status, lb, msg3);
        return;
    }
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(nq_slot, 4096));
    pcl_sigma_shard_kernel<<<(int)grid, 64, 0, st>>>(p.pairs, p.cap, p.small + kPclN, p.means.sh, p.means.result,
                                                     pcl_l1(order), p.means.status, lb, msg3, nq_slot);
}

void launch_pcl_x3_merge(PclBuf& p, int order, const double* recv, int64_t stride, int world, int64_t nq_slot,
                         float* out, hipStream_t st) {
    (void)nq_slot;
    pcl_x3_merge_kernel<<<world, 256, 0, st>>>(recv, stride, world, p.Cbg, p.Cbg_cap, p.means.status,
                                           order == 1 ? p.sig.status : nullptr, p.means.sh,
                                           order == 1 ? p.sig.sh : nullptr, p.merged, out);
}

void launch_pcl_pack_shard(PclBuf& p, int order, float* out, hipStream_t st) {
    pcl_pack_kernel<<<1, kPackThreads, 0, st>>>(p.ghead, kPclTinyN, p.n_all, p.means.result,
                                                order == 1 ? p.sig.result : p.means.result, p.Cbg, order, pcl_l1(order),
                                                p.merged, p.merged + 2, p.means.floor_e + p.means.nch, p.merged + 4, out, 0u);
}

void launch_pcl_mean6(PclBuf& p, const float* sums6, hipStream_t st) {
    pcl_mean6_kernel<<<1, 64, 0, st>>>(sums6, p.n_all ? p.n_all : p.small + kPclN,
                                       reinterpret_cast<float*>(p.small + kPclMean6));
}

void launch_pcl_gather_pack(const PclBuf& p, const uint32_t* d_n, int64_t round, int64_t chunk, double* msg, hipStream_t st) {
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((6 * chunk + 255) / 256, 1024));
    pcl_gather_pack_kernel<<<(int)nb, 256, 0, st>>>(p.pairs, p.cap, d_n, round, chunk, msg);
}

void launch_pcl_gather_unpack(PclBuf& g, const double* recv, int64_t stride, int world, int64_t round, int64_t chunk,
                              hipStream_t st) {
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((6 * chunk + 255) / 256, 1024));
    pcl_gather_unpack_kernel<<<(int)nb, 256, 0, st>>>(recv, stride, world, round, chunk, g.pairs, g.cap, g.small + kPclN);
}

int pcl_reserve(PclBuf& p, int64_t n, int order, hipStream_t st) {
    n = n < 1 ? 1 : n;
    if (n > p.cap) {
        n = std::max<int64_t>(n + n / 2, 2 * p.cap);  // geometric: a growing submap sequence re-allocates rarely
        count_alloc(3);
        void* ptrs[] = {p.pairs, p.bst, p.Cb};
        for (void* q : ptrs)
            if (q) (void)hipFree(q);
        p.pairs = nullptr;
        p.bst = nullptr;
        p.Cb = nullptr;
        p.cap = 0;
        const int64_t nb = (n + kIcpSuper - 1) / kIcpSuper + 1;  // one look-back word per 4096-point record
        const int64_t nkc = n / 340 + 2;  // kc >= max_kc / 2 >= 340 once the depth is blocked
        if (hipMalloc(&p.pairs, (size_t)n * 6 * sizeof(float)) != hipSuccess ||
            hipMalloc(&p.bst, (size_t)nb * sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc(&p.Cb, (size_t)nkc * 9 * sizeof(float)) != hipSuccess)
            return -5;
        (void)hipMemsetAsync(p.bst, 0, (size_t)nb * sizeof(unsigned long long), st);  // epoch 0: never current
        p.cap = n;
    }
    if (!p.small) {
        if (hipMalloc(&p.small, 64 * sizeof(float)) != hipSuccess) return -5;
        (void)hipMemsetAsync(p.small, 0, 64 * sizeof(float), st);
    }
    if (seqsum_reserve(p.means, 6, p.cap, st)) return -5;
    if (order == 1 && seqsum_reserve(p.sig, 9, p.cap, st)) return -5;
    return 0;
}

void pcl_free(PclBuf& p) {
    void* ptrs[] = {p.pairs, p.bst, p.Cb, p.small, p.ghead, p.Cbg, p.merged};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    seqsum_free(p.means);
    seqsum_free(p.sig);
    p = PclBuf{};
}

IcpCompact pcl_compact_args(PclBuf& p) {
    p.epoch = p.epoch + 1u >= (1u << 30) ? 1u : p.epoch + 1u;  // 30 bits, 0 reserved for "never written"
    IcpCompact c;
    c.pairs = p.pairs;
    c.cap = p.cap;
    c.st = p.bst;
    c.ticket = p.small + kPclTicket;
    c.epoch = p.epoch;
    c.d_n = p.small + kPclN;
    return c;
}

void launch_pcl_means(PclBuf& p, int pass, hipStream_t st) {
    seqsum_launch(SeqPairs{p.pairs, p.cap}, 6, p.small + kPclN, p.means, pass, st);
}

void launch_pcl_sigma(PclBuf& p, int order, int pass, hipStream_t st, const float* sums6) {
    const uint32_t* d_n = p.small + kPclN;
    if (!sums6) sums6 = p.means.result;
    if (order == 1) {
        float* mean6 = reinterpret_cast<float*>(p.small + kPclMean6);
        pcl_mean6_kernel<<<1, 64, 0, st>>>(sums6, d_n, mean6);
        seqsum_launch(SeqSigma{p.pairs, mean6, p.cap}, 9, d_n, p.sig, pass, st);
    } else {
        // one workgroup per depth block of the largest n possible (n_hint: the source points, else the capacity)
        const int64_t nmax = p.n_hint > 0 ? std::min(p.n_hint, p.cap) : p.cap;
        const int64_t grid = std::min<int64_t>(nmax / 340 + 2, 4096);
        pcl_sigma_blocks_kernel<<<(int)grid, kSigThreads, 0, st>>>(p.pairs, p.cap, d_n, sums6, pcl_l1(order), p.Cb);
    }
}

void launch_pcl_pack(PclBuf& p, int order, float* out, hipStream_t st, const float* sums6, uint32_t seq) {
    const uint32_t* d_n = p.small + kPclN;
    const uint32_t* zero = p.small + kPclZero;  // the serial fallback's sums need no verification
    const bool serial = sums6 != nullptr;
    if (!sums6) sums6 = p.means.result;
    pcl_pack_kernel<<<1, kPackThreads, 0, st>>>(p.pairs, p.cap, d_n, sums6, order == 1 ? p.sig.result : sums6, p.Cb, order,
                                      pcl_l1(order), serial ? zero : p.means.status,
                                      order == 1 && !serial ? p.sig.status : zero,
                                      serial ? nullptr : p.means.floor_e + p.means.nch, p.small + kPclTicket + 1, out, seq);
}

}  // namespace lio
