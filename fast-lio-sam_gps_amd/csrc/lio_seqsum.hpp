// lio_seqsum.hpp — sequential float summation chains, evaluated in parallel and bit-exact.
//
// pcl::umeyama's float sums (PCL 1.10 TransformationEstimationSVD -> Eigen 3.3 redux) are one
// dependent chain per row: s_0 = x_0, s_k = fl(s_{k-1} + x_k).  At C4 (500 k correspondences) a chain
// is 500 k dependent adds — ~1 ms on one GPU lane.  seqsum computes the same float result in parallel:
//
//   * inside one binade of the running sum (grid u = 2^(E-23)) every add rounds on the same grid, so
//     fl(s + x) = s + rn_u(x) whenever s is already a multiple of u and no tie occurs: the increments
//     rn_u(x_k) are independent of s and add associatively (fixed point, per chain unit 2^(floor-23));
//   * each element's binade is PREDICTED (pass 1: from a double prefix sum; later passes: from the
//     previous pass's reconstruction).  An element whose predicted binade is above its predecessor's
//     (grid coarsens: the rounding depends on the running sum's low bits), a tie, a tiny or non-finite
//     value is an EVENT: a walker (one wave per chain) replays only the events, each as a real float add
//     between exact run sums (double, exact by the chain's floor: runs span <= 28 binades);
//   * a parallel VERIFY pass rebuilds every s_k from the events and the run sums and checks
//     s_k == fl(s_{k-1} + x_k) for every k.  All pass => the result IS the sequential chain (induction
//     from s_0 = x_0), whatever the predictions were.  A failure marks its elements as events and
//     re-predicts from the reconstruction (pass 2, 3); the caller falls back to the serial kernel after.
//
// Chains are supplied by a source functor: value(c, k) of chain c at element k (k < n, n on the device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lio {

constexpr int kSeqThreads = 256;                 // threads per block
constexpr int kSeqPer = 4;                       // consecutive elements per thread (8: slower)
constexpr int kSeqBlock = kSeqThreads * kSeqPer;  // elements per block
constexpr int kSeqMaxChains = 9;

struct SeqSumBuf {
    int nch = 0;
    int64_t nmax = 0;       // element capacity
    int64_t evcap = 0;      // events per chain in use (<= evcap_alloc; tests lower it to force the fallback)
    int64_t evcap_alloc = 0;
    int dbg_noinc = 0;      // tests: pass 1 ignores the grid-coarsening event rule (forces verification failures)
    int nblk = 0;           // blocks for nmax
    double* bsum = nullptr;     // [nch][nblk] double block sums (prediction)
    double* babs = nullptr;     // [nch][nblk] sum |x| (bound on |s|)
    double* boff = nullptr;     // [nch][nblk] exclusive prefix of bsum
    double* bdelta = nullptr;   // [nch][nblk] drift allowance of the pass-1 prediction through the block's end
    uint64_t* btot = nullptr;   // [nch][nblk] block increment totals (fixed point, wrapping)
    int* bev = nullptr;         // [nch][nblk] block event counts
    uint64_t* bPoff = nullptr;  // [nch][nblk] exclusive prefix of btot
    int* bEoff = nullptr;       // [nch][nblk] exclusive prefix of bev
    int* floor_e = nullptr;     // [nch] binade floor (run exactness) ; [nch..2nch) nev ; [2nch..3nch) ok
    uint64_t* ptot = nullptr;   // [nch] total increments
    int* ev_pos = nullptr;      // [nch][evcap]
    uint64_t* ev_P = nullptr;   // [nch][evcap] exclusive increment prefix at the event
    float* ev_x = nullptr;      // [nch][evcap]
    float* ev_s = nullptr;      // [nch][evcap] the event's result (walker)
    float* recon = nullptr;     // [nch][nmax] reconstructed chain (verify; predictions of the next pass)
    uint32_t* forced = nullptr; // [nch][nmax / 32 + 1] elements forced to be events (failed verification)
    bool forced_dirty = true;   // host: forced bits may be set (a re-pass ran since the last clear): the next
                                // pass 1 clears them (verification sets bits only where it fails, and every
                                // failure the caller acts on goes through a pass > 1)
    uint32_t* status = nullptr; // [0] chains failing verification (bits), [1] event overflow (bits)
    float* result = nullptr;    // [nch] final sums
};

int seqsum_reserve(SeqSumBuf& b, int nch, int64_t nmax, hipStream_t st);
void seqsum_free(SeqSumBuf& b);

// chain sources
struct SeqPairs {  // means of pcl::umeyama: chain c < 6 = column c of the compacted pairs (src xyz, tgt xyz)
    const float* pairs;
    int64_t cstride = 0;  // 0: pair-major (pairs[6 k + c]); else column-major (pairs[c cstride + k]: a wave's
                          // loads of one chain are contiguous instead of 24 bytes apart)
    __device__ __forceinline__ float operator()(int c, int64_t k) const {
        return cstride ? pairs[c * cstride + k] : pairs[6 * k + c];
    }
};
struct SeqSigma {  // sigma of the sequential order: chain c < 9 = (tgt_r - dm_r) * (src_col - sm_col), r = c / 3
    const float* pairs;  // column-major (pairs[d * cstride + k])
    const float* mean6;  // device: src mean xyz, tgt mean xyz (float)
    int64_t cstride;
    __device__ __forceinline__ float operator()(int c, int64_t k) const {
        const int r = c / 3, cc = c % 3;
        return (pairs[(3 + r) * cstride + k] - mean6[3 + r]) * (pairs[cc * cstride + k] - mean6[cc]);
    }
};

// Eigen 3.3 evaluateProductBlockingSizesHeuristic (GeneralBlockPanelKernel.h), one thread: the depth block
// kc of a 3 x k by k x 3 float GEMM on an SSE2 build (no FMA: gebp_traits<float, float> mr = 8, nr = 4,
// KcFactor 1) with an L1 data cache of l1 bytes; problems below 48 are not blocked (oracle: the same).
__host__ __device__ inline int64_t eigen_gemm_kc(int64_t k, int64_t l1) {
    const int64_t mr = 8, nr = 4, k_peeling = 8;
    const int64_t k_div = mr * 4 + nr * 4, k_sub = mr * nr * 4;
    if ((k > 3 ? k : 3) < 48) return k;
    int64_t max_kc = ((l1 - k_sub) / k_div) & ~(k_peeling - 1);
    if (max_kc < 1) max_kc = 1;
    if (k > max_kc)
        k = (k % max_kc) == 0 ? max_kc
                              : max_kc - k_peeling * ((max_kc - 1 - (k % max_kc)) / (k_peeling * (k / max_kc + 1)));
    return k;
}

// One pass over nch chains of *d_n elements (d_n: device count, <= b.nmax).  pass 1 predicts from a double
// prefix sum, pass > 1 from the previous pass's reconstruction and its failed elements.  Enqueued only;
// the results are b.result[0 .. nch) and b.status (0 = verified) once the stream reaches them.
template <class Src>
void seqsum_launch(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, hipStream_t st);

}  // namespace lio
