// lio_pcl.hpp — pcl::umeyama's float statistics for the ICP fidelity modes (lio_pcl.hip).
#pragma once
#include "lio_kernels.hpp"
#include "lio_seqsum.hpp"

namespace lio {

// summation orders on the GPU (lio_icp_params.umeyama_float; oracle UmeyamaOrder 1-3)
constexpr int kPclSeq = 1;     // sequential means, sequential sigma depth (scaled at the end)
constexpr int kPclGemm32 = 2;  // sequential means, Eigen 3.3 GEMM sigma, kc from a 32 KiB L1 (the default fidelity mode)
constexpr int kPclGemm48 = 3;  // as 2 with a 48 KiB L1
inline int pcl_l1(int order) { return order == kPclGemm48 ? 48 * 1024 : 32 * 1024; }

// small device words (PclBuf::small, uint32 slots)
constexpr int kPclN = 0;       // accepted correspondences of the pass
constexpr int kPclMean6 = 8;   // float means (order 1's sigma chains)
constexpr int kPclZero = 16;   // two zero words (status of sums that need no verification)
constexpr int kPclTicket = 20; // compaction block ticket (reset by the last block); [21] look-back time-out flag
constexpr int kPclOutWords = 20;  // pcl_pack output: 16 statistics, 2 status words, events (max over the means),
                                  // the compaction's time-out flag

struct PclBuf {
    float* pairs = nullptr;   // accepted (src xyz, tgt xyz) in source order, column-major: pairs[d * cap + k]
                              // (the chains' per-thread loads are then contiguous, not 24 bytes apart)
    unsigned long long* bst = nullptr;  // per compaction block: look-back status word (epoch, flag, value)
    uint32_t epoch = 0;                 // compaction launches so far (mod 2^30, 0 skipped)
    float* Cb = nullptr;      // orders 2 / 3: per depth block, 9 sequential block sums
    uint32_t* small = nullptr;
    int64_t cap = 0;
    SeqSumBuf means;          // 6 chains
    SeqSumBuf sig;            // 9 chains (order 1)
};

int pcl_reserve(PclBuf& p, int64_t n, int order, hipStream_t st);
void pcl_free(PclBuf& p);
// the accepted correspondences of the pass (a.nn_id / a.nn_d2 / a.cur after the correspondence kernel)
void launch_pcl_compact(const IcpArgs& a, PclBuf& p, hipStream_t st);
void launch_pcl_means(PclBuf& p, int pass, hipStream_t st);
// sums6: the six float sums the sigma / pack use (nullptr: the seqsum result of launch_pcl_means; the serial
// fallback passes its own, which need no verification)
void launch_pcl_sigma(PclBuf& p, int order, int pass, hipStream_t st, const float* sums6 = nullptr);
// kPclOutWords floats -> out (device)
void launch_pcl_pack(PclBuf& p, int order, float* out, hipStream_t st, const float* sums6 = nullptr);

}  // namespace lio
