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
//
// Sharded (SeqSumBuf::sh != nullptr): the chain's elements are split over ranks in order, this rank holding
// the window [gbase, gbase + n) (lio_icp_host.cpp, the loop ICP over several GPUs).  Every rank predicts,
// counts and lists the events of its own window — from the double prefix of the elements before it and a
// binade floor common to all ranks (seq_bsum's block sums -> all-gather -> seq_shard_offsets) — the event lists
// are all-gathered (seq_shard_pack -> all-gather -> seq_shard_merge: global positions and increment prefixes),
// every rank walks ALL events (the serial floor, redundantly), and verifies its own window.  The result is the
// sequential chain on every rank, whatever the window split, because the verification covers every element.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lio {

constexpr int kSeqThreads = 256;                 // threads per block
constexpr int kSeqPer = 4;                       // consecutive elements per thread (8: slower)
constexpr int kSeqBlock = kSeqThreads * kSeqPer;  // elements per block
constexpr int kSeqMaxChains = 9;

// one rank's window of sharded chains (device memory; seq_shard_offsets / seq_shard_merge write it)
struct SeqShard {
    double off0[kSeqMaxChains];   // double prefix of the elements before the window (pass-1 prediction)
    double var0[kSeqMaxChains];   // drift-allowance variance accumulated before it
    int floor_e[kSeqMaxChains];   // the chain's binade floor: the same on every rank
    float x0[kSeqMaxChains];      // the chain's first element (global element 0)
    float prev_s[kSeqMaxChains];  // s at global element gbase - 1 (the last verification's; pass > 1 predictions)
    int64_t gbase;                // global index of local element 0
    int64_t n_global;             // elements over all ranks
    uint32_t n32;                 // the same as a 32-bit count (the PCL kernels' d_n of the whole chain)
    uint32_t xflags;              // exchange: bit 0 an event list longer than the slot, bit 1 global capacity
    int max_nev;                  // largest per-rank per-chain event count of the last merge
    // the window's own lists (seq_scan2; the merge overwrites the SeqSumBuf copies with the chain's global ones, and
    // a re-exchange packs the same lists again) and what the last merge added to its block offsets (a re-exchange
    // merges again: the offsets move by the difference only)
    int nev_loc[kSeqMaxChains];
    uint64_t ptot_loc[kSeqMaxChains];
    int e_added[kSeqMaxChains];
    uint64_t p_added[kSeqMaxChains];
};

// exchange message layout (doubles): block sums (seq_bsum's tot_out: [0] the window's element count, then per chain
// `nb_slot` pairs (block double sum, block sum |x|) of its kSeqBlock-element blocks), event lists (seq_shard_pack)
constexpr int kSeqTotHdr = 8;
constexpr int kSeqHdrWords = 32;                     // event message header: n, flags, ptot[9], nev[9], x0[9]
__host__ __device__ inline int64_t seq_tot_words(int nch, int64_t nb_slot) { return kSeqTotHdr + (int64_t)nch * 2 * nb_slot; }

__host__ __device__ inline int64_t seq_bits(double v) {
    int64_t b;
    __builtin_memcpy(&b, &v, sizeof(b));
    return b;
}
__host__ __device__ inline double seq_from_bits(int64_t b) {
    double v;
    __builtin_memcpy(&v, &b, sizeof(v));
    return v;
}
// half an ulp of a float of magnitude v >= 0 (2^(ilogb(v) - 24); 0 for 0), from the exponent bits
__host__ __device__ inline double seq_half_ulp_f32(double v) {
    if (!(v > 0.0)) return 0.0;
    const int64_t e = ((seq_bits(v) >> 52) & 0x7ff) - 1023;
    if (e < -990) return 0.0;
    return seq_from_bits((int64_t)((uint64_t)(e - 24 + 1023) << 52));
}

// Chain c of the gathered block sums (rank r's message at recv + r * stride, nb_slot blocks per chain) -> this
// window's starting prefix and drift variance, the chain's common floor, the window's first global index and the
// chain's length: the formulas of seq_scan1 run over every window's blocks in chain order (offset, bound
// |offset| + block sum |x|, variance + kSeqBlock (ulp / 2)^2 per block), so a window's predictions are as good as
// one rank's.  This is the host mirror (lio_seq_shard_offsets); the device's seq_shard_offsets computes the same
// quantities with the prefix re-associated (seq_scan1's block prefix over windows of 2048 blocks, one workgroup per
// chain), so its off0 / var0 may differ from these in the last bits: every rank runs that kernel over the same
// gathered bytes, so the floors and prefixes agree across ranks bit for bit, which is all the predictions need
// (they are checked by the verification either way).
__host__ __device__ inline void seq_shard_offsets_chain(const double* recv, int64_t stride, int64_t nb_slot, int rank,
                                                        int world, int c, double& off0, double& var0, int& floor_e,
                                                        int64_t& gbase, int64_t& n_global) {
    double off = 0.0, var = 0.0, mb = 0.0;
    int64_t pos = 0;
    off0 = var0 = 0.0;
    gbase = 0;
    for (int r = 0; r < world; ++r) {
        const double* m = recv + (int64_t)r * stride;
        const int64_t nr = (int64_t)m[0];
        if (r == rank) {
            off0 = off;
            var0 = var;
            gbase = pos;
        }
        const int64_t nb = (nr + kSeqBlock - 1) / kSeqBlock;
        const double* bl = m + kSeqTotHdr + (int64_t)c * 2 * nb_slot;
        for (int64_t j = 0; j < nb && j < nb_slot; ++j) {
            const double bound = (off < 0.0 ? -off : off) + bl[2 * j + 1];
            mb = mb > bound ? mb : bound;
            const double hu = seq_half_ulp_f32(bound);
            var = var + (double)kSeqBlock * hu * hu;
            off = off + bl[2 * j];
        }
        pos += nr;
    }
    floor_e = mb > 0.0 ? ilogb(mb) - 27 : -200;
    n_global = pos;
}

// Chain c of the gathered event messages (rank r's at recv + r * stride): every rank's place in the chain's
// global event lists (eoff, world + 1 entries), in its increments (poff) and in its elements (pos), the chain's
// first element x0 and the longest list; returns the problems: 1 a rank's own list overflowed, 2 a list is
// longer than the slot, 4 more events than evs (the device's seq_shard_merge and the host mirror share it).
__host__ __device__ inline int seq_shard_merge_chain(const double* recv, int64_t stride, int world, int slot, int c,
                                                     int64_t evs, int* eoff, uint64_t* poff, int64_t* pos, float& x0,
                                                     int& max_nev) {
    int e = 0, mx = 0, bad = 0;
    uint64_t P = 0;
    int64_t p = 0;
    bool have_x0 = false;
    x0 = 0.f;
    for (int r = 0; r < world; ++r) {
        const double* m = recv + (int64_t)r * stride;
        const int64_t nr = seq_bits(m[0]);
        const uint32_t of = (uint32_t)seq_bits(m[1]);
        const int ner = (int)seq_bits(m[2 + kSeqMaxChains + c]);
        eoff[r] = e;
        poff[r] = P;
        pos[r] = p;
        if (!have_x0 && nr > 0) {
            x0 = (float)m[2 + 2 * kSeqMaxChains + c];
            have_x0 = true;
        }
        if ((of >> c) & 1u) bad |= 1;
        if (ner > slot) bad |= 2;
        mx = mx > ner ? mx : ner;
        e += ner;
        P += (uint64_t)seq_bits(m[2 + c]);
        p += nr;
    }
    eoff[world] = e;
    poff[world] = P;
    pos[world] = p;
    if (e > evs) bad |= 4;
    max_nev = mx;
    return bad;
}

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
    // the fused tail (seq_tail, single rank): event blocks' flag words, the walkers' progress words, the look-back's
    // status words and 64-bit sums, the launch's epoch (host; tags the words, its low 30 bits never 0)
    unsigned long long* evflag = nullptr; // [nch][nblk] epoch << 32 | inclusive event count
    uint64_t* wprog = nullptr;            // [nch] epoch << 32 | events walked and stored
    unsigned long long* lbst = nullptr;   // [nch][nblk] lio_dev.hpp lb_word
    unsigned long long* lbagg = nullptr;  // [nch][nblk] the block's increment sum
    unsigned long long* lbinc = nullptr;  // [nch][nblk] its inclusive prefix
    uint32_t tail_epoch = 0;
    // sharded: sh (device) set, evs the per-chain stride of the walk's (global) event lists ev_*, the local
    // lists in lev_* (stride evcap); single rank: sh == nullptr, evs == evcap, events straight into ev_*
    SeqShard* sh = nullptr;
    int64_t evs = 0;
    int64_t evs_alloc = 0;
    int* lev_pos = nullptr;
    uint64_t* lev_P = nullptr;
    float* lev_x = nullptr;
};

int seqsum_reserve(SeqSumBuf& b, int nch, int64_t nmax, hipStream_t st);
// sharded mode on / off (nmax already reserved): the SeqShard block and the global event lists (evs_global
// events per chain; kept O(window): 2 x the local capacity)
int seqsum_shard(SeqSumBuf& b, bool on, hipStream_t st);
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

// Sharded pass, in three enqueued pieces around the caller's two all-gathers:
//   seqsum_shard_head  pass 1: block sums (also -> tot_out, seq_tot_words(nch, nb_slot) doubles)
//   seqsum_shard_mid   pass 1: seq_shard_offsets over the gathered block sums (rank `rank` of `world`, ranks'
//                      messages tot_stride doubles apart); every pass: count, block offsets, local events,
//                      the event message -> msg_out (kSeqHdrWords + nch * 2 * slot doubles)
//   seqsum_shard_tail  seq_shard_merge over the gathered messages, the walk over all events, the verification
//                      of the window
// heads (nhead > 0): the event message also carries the first nhead elements of each chain (floats, after the
// events); the merge appends the next ranks' heads after the window at ext[c * ext_stride + n ..] and the chain's
// first nghead elements at ghead[c * nghead ..] (the PCL depth blocks that cross a window boundary)
struct SeqHeads {
    int nhead = 0;
    float* ext = nullptr;
    int64_t ext_stride = 0;
    float* ghead = nullptr;
    int nghead = 0;
};
// An extra job for seqsum_shard_mid's offsets launch (one more workgroup): nrec records of `width` doubles, rank r
// holding records [nrec r / world, nrec (r + 1) / world) at recv + r * stride, their first nval values summed in
// record order into out (the ICP's per-pass statistics: lio_icp_combine's order, bit for bit)
struct SeqRecordSum {
    const double* recv = nullptr;
    int64_t nrec = 0;
    int world = 1;
    int64_t stride = 0;
    int width = 0;
    int nval = 0;
    double* out = nullptr;
};
template <class Src>
void seqsum_shard_head(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, double* tot_out, int64_t nb_slot,
                       hipStream_t st);
template <class Src>
void seqsum_shard_mid(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, const double* tot_recv,
                      int64_t tot_stride, int64_t nb_slot, int rank, int world, double* msg_out, int slot, int nhead,
                      hipStream_t st, const SeqRecordSum* rs = nullptr);
template <class Src>
void seqsum_shard_tail(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, const double* msg_recv,
                       int64_t msg_stride, int rank, int world, int slot, const SeqHeads& hd, hipStream_t st);
// the event message again with another slot (the local lists are unchanged; the caller clears status[1])
template <class Src>
void seqsum_shard_repack(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, double* msg_out, int slot,
                         int nhead, hipStream_t st);
inline int64_t seqsum_msg_words(int nch, int slot, int nhead = 0) {
    return kSeqHdrWords + (int64_t)nch * 2 * slot + ((int64_t)nch * nhead + 1) / 2;
}

}  // namespace lio
