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
constexpr int kPclOutWords = 24;  // pcl_pack output: 16 statistics, 2 status words, events (max over the means),
                                  // the compaction's time-out flag; sharded: [20] exchange flags (means | sigma << 8),
                                  // [21] / [22] the largest per-rank event list of the means / sigma chains; [23] the
                                  // sequence number a polling host waits for (one rank, lio_icp_host.cpp pcl_wait)

constexpr int kPclMaxKc = 1016;   // the largest GEMM depth block modelled (kc at a 48 KiB L1)
constexpr int kPclTinyN = 16;     // n + 6 < 20: Eigen's lazy coefficient-based product (pcl_pack)
constexpr int kPclX3Hdr = 8;      // sharded depth-block message: header doubles (statuses, q0, nq)
constexpr int kPclMerged = 8;     // PclBuf::merged words

struct PclBuf {
    float* pairs = nullptr;   // accepted (src xyz, tgt xyz) in source order, column-major: pairs[d * cap + k]
                              // (the chains' per-thread loads are then contiguous, not 24 bytes apart);
                              // sharded: this rank's window, then the next kPclMaxKc pairs of the ranks after it
    unsigned long long* bst = nullptr;  // per 4096-point record of the statistics launch: look-back status word (epoch, flag, value)
    uint32_t epoch = 0;                 // compaction launches so far (mod 2^30, 0 skipped)
    float* Cb = nullptr;      // orders 2 / 3: per depth block, 9 sequential block sums
    uint32_t* small = nullptr;
    int64_t cap = 0;
    int64_t n_hint = 0;       // > 0: no more accepted pairs than this in the next passes (the source's points)
    SeqSumBuf means;          // 6 chains
    SeqSumBuf sig;            // 9 chains (order 1)
    // sharded (world > 1, lio_icp_host.cpp): the whole chain's count (means.sh->n32), the first kPclTinyN pairs
    // of the whole source order (the lazy product), every rank's depth blocks in global order, and the ranks'
    // statuses combined: {means bad, means overflow, sigma bad, sigma overflow, look-back time-out}
    const uint32_t* n_all = nullptr;
    float* ghead = nullptr;
    float* Cbg = nullptr;
    int64_t Cbg_cap = 0;
    uint32_t* merged = nullptr;
    float* mean6 = nullptr;   // (device view of small + kPclMean6)
};

// a plain pair buffer (the sharded serial fallback's gathered pairs): pairs, Cb, small only
int pcl_reserve_plain(PclBuf& p, int64_t n, hipStream_t st);
int pcl_shard_reserve(PclBuf& p, int64_t n_blocks_global, hipStream_t st);

// ---- sharded statistics (lio_icp_host.cpp fid_sharded): the means' seqsum event message carries this rank's
// first kPclMaxKc pairs (SeqHeads: a depth block starting in one window may end in the next; seq_shard_merge
// appends the next ranks' after the window and puts the first kPclTinyN of the whole order in ghead)
inline int64_t pcl_heads_words() { return 3 * (int64_t)kPclMaxKc; }
// depth blocks of the whole chain whose first element is in this window (orders 2 / 3), with the statuses, into
// the message (kPclX3Hdr + nq_slot * 9 floats); nq_slot from pcl_blocks_slot
inline int64_t pcl_blocks_slot(int64_t n_window_max) { return n_window_max / 340 + 3; }
inline int64_t pcl_x3_words(int64_t nq_slot) { return kPclX3Hdr + (nq_slot * 9 + 1) / 2; }
void launch_pcl_sigma_shard(PclBuf& p, int order, double* msg3, int64_t nq_slot, hipStream_t st);
// every rank's depth blocks -> Cbg, statuses combined -> merged; out[20..22]: exchange flags and the largest
// event lists (the caller's slot for the next pass)
void launch_pcl_x3_merge(PclBuf& p, int order, const double* recv, int64_t stride, int world, int64_t nq_slot,
                         float* out, hipStream_t st);
void launch_pcl_pack_shard(PclBuf& p, int order, float* out, hipStream_t st);
void launch_pcl_mean6(PclBuf& p, const float* sums6, hipStream_t st);
// serial fallback: this window's pairs in rounds of `chunk` (message: n, then 6 columns of chunk floats), and
// every rank's into g (the whole source order; g.small[kPclN] = the total)
inline int64_t pcl_gather_words(int64_t chunk) { return 2 + 3 * chunk; }
void launch_pcl_gather_pack(const PclBuf& p, const uint32_t* d_n, int64_t round, int64_t chunk, double* msg, hipStream_t st);
void launch_pcl_gather_unpack(PclBuf& g, const double* recv, int64_t stride, int world, int64_t round, int64_t chunk,
                              hipStream_t st);

int pcl_reserve(PclBuf& p, int64_t n, int order, hipStream_t st);
void pcl_free(PclBuf& p);
// the accepted correspondences of the pass (a.nn_id / a.nn_d2 / a.cur after the correspondence kernel)
// the compaction's arguments for the statistics launch (launch_icp_stats' IcpCompact; a new look-back epoch)
IcpCompact pcl_compact_args(PclBuf& p);
void launch_pcl_means(PclBuf& p, int pass, hipStream_t st);
// sums6: the six float sums the sigma / pack use (nullptr: the seqsum result of launch_pcl_means; the serial
// fallback passes its own, which need no verification)
void launch_pcl_sigma(PclBuf& p, int order, int pass, hipStream_t st, const float* sums6 = nullptr);
// kPclOutWords floats -> out (device)
// seq != 0: out is host-mapped and out[23] = seq is stored last (system scope) for a host that polls it
void launch_pcl_pack(PclBuf& p, int order, float* out, hipStream_t st, const float* sums6 = nullptr, uint32_t seq = 0);

}  // namespace lio
