// lio_seqsum.hip — sequential float summation chains evaluated in parallel, bit-exact (lio_seqsum.hpp).
//
// Per pass, for every chain:
//   seq_bsum     block double prefix (prediction) totals, sum |x| (bound on |s|)
//   seq_scan1    per chain, sequential over blocks: double block offsets, the binade floor
//   count        per element: predicted binade, event flag, fixed-point increment -> block totals
//   offsets      exclusive block offsets of increments and events
//   events       the events in element order: position, increment prefix, x
//   walk         one workgroup per chain replays the events (run sums exact in double) -> event results, sum
//   verify       every s_k rebuilt from the events; s_k == fl(s_{k-1} + x_k) checked for every k
// One rank: count .. verify are ONE launch, seq_tail (the offsets by a look-back, the walk following the event
// blocks as they publish, the verification following the walk).  Sharded: seq_count, seq_scan2 and seq_events on
// the window, the event exchange, seq_shard_merge, then walk and verify as one launch (seq_shard_walkverify).
#include "lio_seqsum.hpp"

#include <cmath>

#include "lio_dev.hpp"
#include "lio_error.hpp"

namespace lio {

namespace {

constexpr int kSpecial = -1000;  // zero, subnormal or non-finite: no binade
// prediction slack near binade edges (mantissa bits): pass 1 predicts from a double prefix sum that drifts
// from the float chain by its accumulated rounding (measured: a few units on C4 chains of |s| ~ 1e4-1e5,
// ~2^-12 relative), later passes from a reconstruction within a few ulps of it
// 10 bits: 2^-13 relative (round 6, with the 3-sigma drift band below; 13 before): C4 pair B's longest event list
// 4 634 -> 4 100, 2.24 -> 2.20 ms per alignment, still no re-pass; 7 bits: re-passes return
// (profiles/r06_drift_sigmas_ab.txt)
#ifndef LIO_PRED_SLACK1
#define LIO_PRED_SLACK1 10
#endif
constexpr int kPredSlack1 = LIO_PRED_SLACK1;
constexpr int kPredSlack2 = 4;   // 16 ulps

__device__ __forceinline__ int binade_f(float f) {
    const uint32_t b = __float_as_uint(f);
    const int e = (int)((b >> 23) & 0xffu);
    return (e == 0 || e == 255) ? kSpecial : e - 127;
}

// a prediction within 2^-(23 - lg) of a binade edge (lg mantissa bits of slack) is ambiguous: kSpecial
// makes the element (and its successor) an event, replayed exactly by the walker
__device__ __forceinline__ int binade_pred(float f, int lg) {
    const uint32_t m = __float_as_uint(f) & 0x7fffffu;
    const uint32_t tol = 1u << lg;
    if (m < tol || m > 0x7fffffu - tol) return kSpecial;
    return binade_f(f);
}

// pass 1 also needs the prediction's absolute distance from the binade edges: the double prefix drifts from
// the float chain by the chain's accumulated rounding, which near a zero crossing is large against |s| (C4
// means chains: predictions of -0.98 with ~2.3 of drift).  delta bounds that drift (seq_scan1); an element whose
// prediction lies within delta of an edge (or of zero) is ambiguous, i.e. an event.
__device__ __forceinline__ int binade_pred_abs(float f, int lg, double delta) {
    const int e = binade_pred(f, lg);
    if (e == kSpecial) return e;
    const double a = fabs((double)f), lo = ldexp(1.0, e);
    return (a - lo < delta || 2.0 * lo - a < delta) ? kSpecial : e;
}

template <typename T>
__device__ __forceinline__ T wave_incl(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T u = __shfl_up(v, d, 64);
        if (lane >= d) v = v + u;
    }
    return v;
}

// exclusive block prefix of v (integer types: any order is exact); total -> *tot (all threads)
template <typename T>
__device__ __forceinline__ T block_excl(T v, T* s_w, T& tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const T inc = wave_incl(v);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    T off = 0, t = 0;
#pragma unroll
    for (int i = 0; i < kSeqThreads / 64; ++i) {
        const T c = s_w[i];
        if (i < w) off = off + c;
        t = t + c;
    }
    __syncthreads();
    tot = t;
    return off + inc - v;
}

// The block's double prefix D_local[i] of its elements (thread t holds elements 4t .. 4t + 3) and the block
// total, in ONE fixed order: seq_bsum stores the total, seq_count rebuilds every D_k from the same code, so
// the prediction of the block's last element (boff[b] + total) equals the next block's boff bit for bit.
__device__ __forceinline__ double block_dprefix(const float (&x)[kSeqPer], double (&D)[kSeqPer], double* s_w, double& tot) {
    double run = (double)x[0];
    double loc[kSeqPer];
    loc[0] = run;
#pragma unroll
    for (int i = 1; i < kSeqPer; ++i) {
        run = run + (double)x[i];
        loc[i] = run;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double inc = wave_incl(run);
    double ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = 0.0;
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    double off = 0.0;
    for (int i = 0; i < w; ++i) off = off + s_w[i];
    const double base = off + ex;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) D[i] = base + loc[i];
    __syncthreads();
    // the total IS the last element's D (not a separately ordered sum of the wave totals)
    if (threadIdx.x == kSeqThreads - 1) s_w[0] = D[kSeqPer - 1];
    __syncthreads();
    tot = s_w[0];
    __syncthreads();
    return base;
}

struct ElemInfo {
    float x[kSeqPer];
    int e[kSeqPer];   // predicted binade of s_k
    int ep;           // predicted binade of the element before this thread's first
};

// event / increment of element k >= 1 from its value, predicted binade e, the predecessor's ep, the floor
__device__ __forceinline__ bool seq_event(float x, int e, int ep, int floor_e, bool forced, bool noinc, uint64_t& inc) {
    inc = 0;
    if (forced || e == kSpecial || ep == kSpecial || (e != ep && !noinc) || e < floor_e || e - floor_e > 60) return true;
    if (!(fabsf(x) <= 3.402823466e38f)) return true;  // non-finite
    const double t = ldexp((double)x, 23 - e);
    if (!(fabs(t) < 0x1p52)) return true;
    const double r = rint(t);
    if (fabs(t - r) == 0.5) return true;  // a tie: the parity of the running sum decides
    const int64_t m = (int64_t)r;
    inc = (uint64_t)m << (e - floor_e);
    return false;
}

template <class Src>
__device__ __forceinline__ void load_x(const Src& src, int c, int64_t k0, int64_t n, float (&x)[kSeqPer]) {
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        const int64_t k = k0 + i;
        x[i] = k < n ? src(c, k) : 0.f;
    }
}

__device__ __forceinline__ bool forced_bit(const uint32_t* f, int64_t k) { return f && ((f[k >> 5] >> (k & 31)) & 1u); }

// predictions for this thread's elements (pass 1: double prefix; later: the previous reconstruction)
template <class Src>
__device__ __forceinline__ void predict(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                        ElemInfo& in, double* s_wd) {
    const int64_t k0 = (int64_t)blk * kSeqBlock + (int64_t)threadIdx.x * kSeqPer;
    load_x(src, c, k0, n, in.x);
    if (pass <= 1) {
        double D[kSeqPer], tot;
        block_dprefix(in.x, D, s_wd, tot);
        const double bo = b.boff[(size_t)c * b.nblk + blk];
        const double dl = b.bdelta[(size_t)c * b.nblk + blk];
#pragma unroll
        for (int i = 0; i < kSeqPer; ++i) in.e[i] = binade_pred_abs((float)(bo + D[i]), kPredSlack1, dl);
        // predecessor of the thread's first element: the previous thread's last (block's first: boff)
        int prev = __shfl_up(in.e[kSeqPer - 1], 1, 64);
        __shared__ int s_last[kSeqThreads / 64];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        if (lane == 63) s_last[w] = in.e[kSeqPer - 1];
        __syncthreads();
        if (lane == 0) {
            if (w > 0) {
                prev = s_last[w - 1];
            } else if (blk > 0) {  // the previous block's last prediction, as that block computed it
                const size_t pb = (size_t)c * b.nblk + blk - 1;
                prev = binade_pred_abs((float)(b.boff[pb] + b.bsum[pb]), kPredSlack1, b.bdelta[pb]);
            } else {
                prev = binade_pred_abs((float)bo, kPredSlack1, dl);
            }
        }
        __syncthreads();
        in.ep = prev;
    } else {
        const float* rc = b.recon + (size_t)c * b.nmax;
#pragma unroll
        for (int i = 0; i < kSeqPer; ++i) in.e[i] = k0 + i < n ? binade_pred(rc[k0 + i], kPredSlack2) : kSpecial;
        // a window's first element: its predecessor lives on the previous rank (the last verification's s)
        in.ep = k0 > 0 ? binade_pred(rc[k0 - 1], kPredSlack2)
                       : (b.sh && b.sh->gbase > 0 ? binade_pred(b.sh->prev_s[c], kPredSlack2) : kSpecial);
    }
    if (k0 == 0 && (!b.sh || b.sh->gbase == 0)) in.e[0] = binade_f(in.x[0]);  // s_0 = x_0 exactly
}

// per element: event flag and increment (element 0: the start, neither)
template <class Src>
__device__ __forceinline__ void classify(const SeqSumBuf& b, int c, int blk, int64_t n, const ElemInfo& in, int floor_e,
                                         int pass, bool (&ev)[kSeqPer], uint64_t (&inc)[kSeqPer]) {
    const bool noinc = b.dbg_noinc && pass <= 1;
    const int64_t k0 = (int64_t)blk * kSeqBlock + (int64_t)threadIdx.x * kSeqPer;
    const uint32_t* fb = b.forced ? b.forced + (size_t)c * (b.nmax / 32 + 1) : nullptr;
    const int64_t gb = b.sh ? b.sh->gbase : 0;  // global index of local element 0 (sharded windows)
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        const int64_t k = k0 + i;
        ev[i] = false;
        inc[i] = 0;
        if (gb + k == 0 || k >= n) continue;  // the chain's start: neither event nor increment
        const int ep = i == 0 ? in.ep : in.e[i - 1];
        ev[i] = seq_event(in.x[i], in.e[i], ep, floor_e, forced_bit(fb, k), noinc, inc[i]);
    }
}

template <class Src>
__global__ void __launch_bounds__(kSeqThreads) seq_bsum(Src src, SeqSumBuf b, const uint32_t* d_n,
                                                          double* __restrict__ tot_out = nullptr, int64_t nb_slot = 0) {
    __shared__ double s_wd[kSeqThreads / 64];
    __shared__ double s_abs[kSeqThreads / 64];
    const int c = blockIdx.y;
    const int64_t n = *d_n;
    // sharded: the block sums go straight into this window's message too (seq_shard_offsets on every rank)
    if (tot_out && c == 0 && blockIdx.x == 0 && threadIdx.x == 0) tot_out[0] = (double)n;
    if ((int64_t)blockIdx.x * kSeqBlock >= n) return;  // block-uniform
    float x[kSeqPer];
    load_x(src, c, (int64_t)blockIdx.x * kSeqBlock + (int64_t)threadIdx.x * kSeqPer, n, x);
    double D[kSeqPer], tot;
    block_dprefix(x, D, s_wd, tot);
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) a += fabs((double)x[i]);
    double atot;
    block_excl(a, s_abs, atot);
    if (threadIdx.x == 0) {
        b.bsum[(size_t)c * b.nblk + blockIdx.x] = tot;
        b.babs[(size_t)c * b.nblk + blockIdx.x] = atot;
        if (tot_out && blockIdx.x < nb_slot) {
            tot_out[kSeqTotHdr + (size_t)c * 2 * nb_slot + 2 * blockIdx.x] = tot;
            tot_out[kSeqTotHdr + (size_t)c * 2 * nb_slot + 2 * blockIdx.x + 1] = atot;
        }
    }
}

// per chain: boff[j] = boff[j-1] + bsum[j-1] (sequential: the bits every block's prediction relies on),
// the bound on |s| and the floor binade that keeps every run sum exact in double
// the block values go through LDS in windows (coalesced loads by all lanes), the dependent chain runs on lane 0
constexpr int kScanWin = 2048;

// The drift allowance: the float chain's rounding errors (at most half an ulp of |s| each) modelled as a random
// walk, bounded per block by the block's largest |s| (|offset| + sum |x|): V += kSeqBlock (ulp / 2)^2,
// delta = kDriftSigmas sqrt(V) through the block's end (non-decreasing, so conservative for every element of
// the block).  Only a performance model: a drift past it fails verification and the chain takes a second pass.
// 3 sigmas (round 6; 2 before): C4 pair B's re-passes 11 -> 0 in 110 passes for ~1 % more events, 2.35 -> 2.25 ms per
// alignment, pair A +7 us; 4 sigmas: more events, no fewer re-passes (profiles/r06_drift_sigmas_ab.txt)
#ifndef LIO_DRIFT_SIGMAS
#define LIO_DRIFT_SIGMAS 3.0
#endif
constexpr double kDriftSigmas = LIO_DRIFT_SIGMAS;

// half an ulp of a float of magnitude v >= 0 (2^(ilogb(v) - 24); 0 for 0), from the exponent bits
__device__ __forceinline__ double half_ulp_f32(double v) {
    if (!(v > 0.0)) return 0.0;
    const int64_t e = (int64_t)((__double_as_longlong(v) >> 52) & 0x7ff) - 1023;
    if (e < -990) return 0.0;
    return __longlong_as_double((long long)((uint64_t)(e - 24 + 1023) << 52));
}

__global__ void __launch_bounds__(256) seq_scan1(SeqSumBuf b, const uint32_t* d_n, int pass) {
    __shared__ double s_sum[kScanWin], s_abs[kScanWin], s_off[kScanWin], s_dl[kScanWin];
    __shared__ double s_vw[256 / 64];
    const int c = blockIdx.x;
    const int64_t n = *d_n;
    const int nb = (int)((n + kSeqBlock - 1) / kSeqBlock);
    // the offsets carried over windows (every thread's copy); this thread's max; every thread's copy of the
    // allowance's running variance — a sharded window starts from the ranks before it (seq_shard_offsets)
    double off = b.sh ? b.sh->off0[c] : 0.0, mb = 0.0;
    double var = b.sh ? b.sh->var0[c] : 0.0;
    constexpr int kPerT = kScanWin / 256;
    for (int w0 = 0; w0 < nb; w0 += kScanWin) {
        const int m = min(kScanWin, nb - w0);
        for (int j = threadIdx.x; j < m; j += blockDim.x) {
            s_sum[j] = b.bsum[(size_t)c * b.nblk + w0 + j];
            s_abs[j] = b.babs[(size_t)c * b.nblk + w0 + j];
        }
        __syncthreads();
        // block offsets by a block prefix (thread t: blocks t kPerT .. +kPerT-1 in order, then the threads' runs
        // in a fixed order): deterministic, and every kernel reads these stored offsets, so the predictions agree
        // between the count, events and verification roles (predict() takes a block's first predecessor from
        // boff[b-1] + bsum[b-1], the previous block's own last prediction)
        {
            double loc[kPerT], run = 0.0;
#pragma unroll
            for (int i = 0; i < kPerT; ++i) {
                const int j = (int)threadIdx.x * kPerT + i;
                loc[i] = run;  // exclusive within the thread
                run = run + (j < m ? s_sum[j] : 0.0);
            }
            double tot;
            const double ex = block_excl(run, s_vw, tot);
#pragma unroll
            for (int i = 0; i < kPerT; ++i) {
                const int j = (int)threadIdx.x * kPerT + i;
                if (j < m) {
                    const double o = off + (ex + loc[i]);
                    s_off[j] = o;
                    mb = fmax(mb, fabs(o) + s_abs[j]);
                }
            }
            off = off + tot;
        }
        __syncthreads();
        // the allowance off lane 0's chain: every thread its kScanWin / 256 consecutive blocks, one block prefix
        {
            double loc[kPerT], run = 0.0;
#pragma unroll
            for (int i = 0; i < kPerT; ++i) {
                const int j = (int)threadIdx.x * kPerT + i;
                const double big = j < m ? fabs(s_off[j]) + s_abs[j] : 0.0;
                const double hu = half_ulp_f32(big);
                run = run + (double)kSeqBlock * hu * hu;
                loc[i] = run;
            }
            double tot;
            const double ex = block_excl(run, s_vw, tot);  // fixed order: every thread sees the same total
#pragma unroll
            for (int i = 0; i < kPerT; ++i) {
                const int j = (int)threadIdx.x * kPerT + i;
                if (j < m) s_dl[j] = kDriftSigmas * sqrt(var + ex + loc[i]);
            }
            var = var + tot;
        }
        __syncthreads();
        for (int j = threadIdx.x; j < m; j += blockDim.x) {
            b.boff[(size_t)c * b.nblk + w0 + j] = s_off[j];
            b.bdelta[(size_t)c * b.nblk + w0 + j] = s_dl[j];
        }
        __syncthreads();
    }
    // the bound's max over the threads (max: any order is exact)
    {
        __shared__ double s_mb[256 / 64];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) mb = fmax(mb, __shfl_xor(mb, d, 64));
        if ((threadIdx.x & 63) == 0) s_mb[threadIdx.x >> 6] = mb;
        __syncthreads();
        mb = fmax(fmax(s_mb[0], s_mb[1]), fmax(s_mb[2], s_mb[3]));
    }
    if (threadIdx.x == 0) {
        // |s_k| < 2^(ilogb(mb) + 2) with a binade of margin for the float chain's own drift; a run's sum
        // then has <= 53 significant bits when its binades stay >= floor
        // (sharded: the floor every rank computed from all ranks' totals, so the fixed-point unit is common)
        b.floor_e[c] = b.sh ? b.sh->floor_e[c] : (mb > 0.0 ? ilogb(mb) - 27 : -200);
        if (c == 0 && pass <= 1) {
            b.status[0] = 0u;
            b.status[1] = 0u;
        }
    }
}

template <class Src>
__global__ void __launch_bounds__(kSeqThreads) seq_count(Src src, SeqSumBuf b, const uint32_t* d_n, int pass) {
    __shared__ double s_wd[kSeqThreads / 64];
    __shared__ uint64_t s_u[kSeqThreads / 64];
    __shared__ int s_i[kSeqThreads / 64];
    const int c = blockIdx.y;
    const int64_t n = *d_n;
    if ((int64_t)blockIdx.x * kSeqBlock >= n) return;
    ElemInfo in;
    predict(src, b, c, (int)blockIdx.x, n, pass, in, s_wd);
    bool ev[kSeqPer];
    uint64_t inc[kSeqPer];
    classify<Src>(b, c, (int)blockIdx.x, n, in, b.floor_e[c], pass, ev, inc);
    uint64_t su = 0;
    int se = 0;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        su += inc[i];
        se += ev[i] ? 1 : 0;
    }
    uint64_t tu;
    int te;
    block_excl(su, s_u, tu);
    block_excl(se, s_i, te);
    if (threadIdx.x == 0) {
        b.btot[(size_t)c * b.nblk + blockIdx.x] = tu;
        b.bev[(size_t)c * b.nblk + blockIdx.x] = te;
    }
}

// exclusive block offsets of the increments (wrapping) and event counts: integers, any order is exact
__global__ void __launch_bounds__(kSeqThreads) seq_scan2(SeqSumBuf b, const uint32_t* d_n) {
    __shared__ uint64_t s_u[kSeqThreads / 64];
    __shared__ int s_i[kSeqThreads / 64];
    const int c = blockIdx.x;
    const int64_t n = *d_n;
    const int nb = (int)((n + kSeqBlock - 1) / kSeqBlock);
    uint64_t P = 0;
    int E = 0;
    for (int j0 = 0; j0 < nb; j0 += kSeqThreads) {  // block-uniform trip count
        const int j = j0 + (int)threadIdx.x;
        const uint64_t u = j < nb ? b.btot[(size_t)c * b.nblk + j] : 0;
        const int e = j < nb ? b.bev[(size_t)c * b.nblk + j] : 0;
        uint64_t tu;
        int te;
        const uint64_t pu = block_excl(u, s_u, tu);
        const int pe = block_excl(e, s_i, te);
        if (j < nb) {
            b.bPoff[(size_t)c * b.nblk + j] = P + pu;
            b.bEoff[(size_t)c * b.nblk + j] = E + pe;
        }
        P += tu;
        E += te;
    }
    if (threadIdx.x == 0) {
        b.ptot[c] = P;
        b.floor_e[b.nch + c] = E;  // events of the chain
        if (E > b.evcap) atomicOr(&b.status[1], 1u << c);
        if (b.sh) {
            b.sh->nev_loc[c] = E;
            b.sh->ptot_loc[c] = P;
            b.sh->e_added[c] = 0;
            b.sh->p_added[c] = 0;
        }
    }
}

// the block's elements with their exclusive increment prefix and inclusive event count within the block, and the
// block's totals
template <class Src>
__device__ __forceinline__ void block_scan_local(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                                 ElemInfo& in, bool (&ev)[kSeqPer], uint64_t (&Pex)[kSeqPer],
                                                 int (&Ein)[kSeqPer], uint64_t& tu, int& te) {
    __shared__ double s_wd[kSeqThreads / 64];
    __shared__ uint64_t s_u[kSeqThreads / 64];
    __shared__ int s_i[kSeqThreads / 64];
    predict(src, b, c, blk, n, pass, in, s_wd);
    uint64_t inc[kSeqPer];
    classify<Src>(b, c, blk, n, in, b.floor_e[c], pass, ev, inc);
    uint64_t su = 0;
    int se = 0;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        su += inc[i];
        se += ev[i] ? 1 : 0;
    }
    uint64_t pu = block_excl(su, s_u, tu);
    int pe = block_excl(se, s_i, te);
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        Pex[i] = pu;
        pu += inc[i];
        pe += ev[i] ? 1 : 0;
        Ein[i] = pe;
    }
}

// ... and with the block's offsets in the chain (seq_scan2's)
template <class Src>
__device__ __forceinline__ void block_scan_elems(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                                 ElemInfo& in, bool (&ev)[kSeqPer], uint64_t (&Pex)[kSeqPer],
                                                 int (&Ein)[kSeqPer]) {
    uint64_t tu;
    int te;
    block_scan_local(src, b, c, blk, n, pass, in, ev, Pex, Ein, tu, te);
    const uint64_t P0 = b.bPoff[(size_t)c * b.nblk + blk];
    const int E0 = b.bEoff[(size_t)c * b.nblk + blk];
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        Pex[i] += P0;
        Ein[i] += E0;
    }
}

// The fused tail's in-launch hand-offs (seq_tail) use agent-scope (sc1) accesses on both sides, MI355X_MICROARCH.md's
// hand-off table row 1: every storing wave stores its payload sc1 and waits (s_waitcnt vmcnt(0)), a workgroup barrier,
// then one lane stores the flag sc1; the consumer polls the flag sc1 and loads the payload sc1.  F = false: the
// separate launches (kernel boundaries order everything), plain accesses.
typedef __attribute__((address_space(1))) uint32_t sq_gu32;
typedef __attribute__((address_space(1))) unsigned long long sq_gu64;
template <bool F>
__device__ __forceinline__ uint32_t ld32(const void* p) {
    if constexpr (F) return __hip_atomic_load((const sq_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *(const uint32_t*)p;
}
template <bool F>
__device__ __forceinline__ uint64_t ld64(const void* p) {
    if constexpr (F) return __hip_atomic_load((const sq_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *(const unsigned long long*)p;
}
template <bool F>
__device__ __forceinline__ void st32(void* p, uint32_t v) {
    if constexpr (F) __hip_atomic_store((sq_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(uint32_t*)p = v;
}
template <bool F>
__device__ __forceinline__ void st64(void* p, uint64_t v) {
    if constexpr (F) __hip_atomic_store((sq_gu64*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *(unsigned long long*)p = v;
}
// a spin's safety valve (wall_clock64 counts at 100 MHz): 20 ms, far beyond any pass; a time-out is a verification
// failure (re-pass) or an event overflow (the serial kernel), never a wrong result
constexpr uint64_t kSpinTicks = 2000000;

// the events of block blk in element order (position, increment prefix, x) from its prefixes Pex / Ein
template <bool F>
__device__ __forceinline__ void store_events(const SeqSumBuf& b, int c, int blk, const ElemInfo& in,
                                             const bool (&ev)[kSeqPer], const uint64_t (&Pex)[kSeqPer],
                                             const int (&Ein)[kSeqPer]) {
    const int64_t k0 = (int64_t)blk * kSeqBlock + (int64_t)threadIdx.x * kSeqPer;
    // single rank: the walk's lists; sharded: this window's lists (local positions and prefixes, seq_shard_pack)
    int* EPOS = b.sh ? b.lev_pos : b.ev_pos;
    uint64_t* EPP = b.sh ? b.lev_P : b.ev_P;
    float* EXX = b.sh ? b.lev_x : b.ev_x;
    const int64_t es = b.sh ? b.evcap : b.evs;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i)
        if (ev[i]) {
            const int idx = Ein[i] - 1;
            if (idx < b.evcap) {
                st32<F>(EPOS + (size_t)c * es + idx, (uint32_t)(k0 + i));
                st64<F>(EPP + (size_t)c * es + idx, Pex[i]);
                st32<F>(EXX + (size_t)c * es + idx, __float_as_uint(in.x[i]));
            }
        }
}

template <class Src>
__global__ void __launch_bounds__(kSeqThreads) seq_events(Src src, SeqSumBuf b, const uint32_t* d_n, int pass) {
    const int c = blockIdx.y, blk = blockIdx.x;
    const int64_t n = *d_n;
    if ((int64_t)blk * kSeqBlock >= n) return;
    ElemInfo in;
    bool ev[kSeqPer];
    uint64_t Pex[kSeqPer];
    int Ein[kSeqPer];
    block_scan_elems(src, b, c, blk, n, pass, in, ev, Pex, Ein);
    store_events<false>(b, c, blk, in, ev, Pex, Ein);
}

// The walk: s_{event-1} = s_{previous event} + run sum R (exact), s_event = fl(s_{event-1} + x_event), one chain
// per block.  The chain of dependent operations is the serial floor; everything else is kept off it:
//   * the event records stream through LDS in chunks of C events, double-buffered: while wave 0 walks chunk k,
//     waves 1-3 prepare chunk k+1 (run sums from the increment prefixes, the fast-path test) and store chunk
//     k-1's results, so the walk never waits on a global load;
//   * fast groups: when every run sum R of a 64-event group is a float exactly (tested while preparing), the
//     chain stays in float, two dependent adds per event: s_{event-1} = fl32(s + R) and s_event = fl32(that + x).
//     That is the general form's value bit for bit: fl32(fl64(s + R)) = fl32(s + R) for the two binary32
//     operands (53 >= 2 * 24 + 2: double rounding is innocuous for a sum), and when the increments are right
//     s + R is the float s_{event-1} itself;
//   * other groups (a run spanning more than 24 bits of the chain's fixed-point unit) take the general form,
//     fl32(fl32(fl64(s + R)) + x).  The verification checks every element either way.
constexpr int kWalkThreads = 256;
// events per LDS chunk (x 2 buffers x 20 bytes: 20 KB, so the other roles of the launch keep their occupancy); C4 pair
// B per alignment: 256 2.20-2.22 ms, 512 2.18-2.21, 1024 2.29-2.31 (profiles/r06_seq_tail_ab.txt)
#ifndef LIO_TAIL_CHUNK
#define LIO_TAIL_CHUNK 512
#endif
constexpr int kTailChunk = LIO_TAIL_CHUNK;
constexpr int kWalkU = 8;
template <int C>
struct alignas(16) WalkChunk {
    double R[C];  // run sums (exact)
    float Rf[C];  // the same as floats (fast groups)
    float x[C];
    float f[C];   // the walk's results
    int fast[C / 64];
    int m;        // events in the chunk (the fused tail: known once its events are published)
};

// chunk k's m records into B by the threads [t0, t0 + nt) (nt a multiple of 64, t0 wave-aligned, nt >= 192): every
// load of the thread's share is issued before the first is used (the preparation runs beside the walk and must
// stay shorter than it: one round trip to memory per chunk, not one per step)
template <int C, bool F>
__device__ __forceinline__ void walk_prepare(WalkChunk<C>& B, int k, int m, double unit, const uint64_t* EP,
                                             const float* EX, int t, int nt) {
    constexpr int kPrepMax = (C + 191) / 192;
    const int e0 = k * C;
    uint64_t P[kPrepMax], Pp[kPrepMax];
    float X[kPrepMax];
#pragma unroll
    for (int q = 0; q < kPrepMax; ++q) {
        const int j = t + q * nt, i = e0 + j;
        const bool in = j < m;
        P[q] = in ? ld64<F>(EP + i) : 0;
        Pp[q] = in && i > 0 ? ld64<F>(EP + i - 1) : 0;
        X[q] = in ? __uint_as_float(ld32<F>(EX + i)) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kPrepMax; ++q) {
        const int j = t + q * nt;
        if (j >= C) break;  // wave-uniform: one 64-event group per wave and step
        const double R = j < m ? (double)(int64_t)(P[q] - Pp[q]) * unit : 0.0;  // a run sum: exact (<= 53 bits)
        const float Rf = (float)R;
        B.R[j] = R;
        B.Rf[j] = Rf;
        B.x[j] = X[q];
        // a float exactly, and normal or zero (no denormal operand on the fast path)
        const uint64_t all = __ballot((double)Rf == R && (Rf == 0.f || fabsf(Rf) >= 1.17549435e-38f));
        if ((threadIdx.x & 63) == 0) B.fast[j >> 6] = all == ~0ull;
    }
}

// the float form over one 64-event group (all fast), in four steps of 16: a step's operands are read from LDS while
// the step before it adds (the LDS latency off the chain), results stored 4 at a time
__device__ __forceinline__ float walk_fast(const float* Rf, const float* Xs, float* Fo, float s) {
    constexpr int nsteps = 4;
    const float4* R4 = reinterpret_cast<const float4*>(Rf);
    const float4* X4 = reinterpret_cast<const float4*>(Xs);
    float4* F4 = reinterpret_cast<float4*>(Fo);
    float4 r0[4], x0[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r0[q] = R4[q];
        x0[q] = X4[q];
    }
#pragma unroll
    for (int st = 0; st < nsteps; ++st) {
        float4 r1[4], x1[4];
        if (st + 1 < nsteps) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                r1[q] = R4[4 * (st + 1) + q];
                x1[q] = X4[4 * (st + 1) + q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 o;
            s = (s + r0[q].x) + x0[q].x;
            o.x = s;
            s = (s + r0[q].y) + x0[q].y;
            o.y = s;
            s = (s + r0[q].z) + x0[q].z;
            o.z = s;
            s = (s + r0[q].w) + x0[q].w;
            o.w = s;
            F4[4 * st + q] = o;
        }
        if (st + 1 < nsteps) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                r0[q] = r1[q];
                x0[q] = x1[q];
            }
        }
    }
    return s;
}

// wave 0, lane 0: chunk B's m events from s
template <int C>
__device__ __forceinline__ float walk_chunk(WalkChunk<C>& B, int m, float s) {
    for (int g = 0; g < m; g += 64) {
        const int cnt = min(64, m - g);
        if (cnt == 64 && B.fast[g >> 6]) {
            s = walk_fast(B.Rf + g, B.x + g, B.f + g, s);
        } else if (cnt == 64) {
            for (int l = g; l < g + 64; l += kWalkU) {
                double r[kWalkU];
                float x[kWalkU];
#pragma unroll
                for (int u = 0; u < kWalkU; ++u) {
                    r[u] = B.R[l + u];
                    x[u] = B.x[l + u];
                }
#pragma unroll
                for (int u = 0; u < kWalkU; ++u) {
                    s = (float)((double)s + r[u]) + x[u];
                    B.f[l + u] = s;
                }
            }
        } else {
            for (int l = g; l < g + cnt; ++l) {
                s = (float)((double)s + B.R[l]) + B.x[l];
                B.f[l] = s;
            }
        }
    }
    return s;
}

// F: the walk's progress word of chain c, epoch << 32 | events whose results are stored (sc1)
__device__ __forceinline__ void walk_publish(const SeqSumBuf& b, int c, uint32_t epoch, uint32_t done) {
    st64<true>(b.wprog + c, ((uint64_t)epoch << 32) | done);
}

// the walker of chain c when every event is listed before it starts (sharded, after seq_shard_merge).  F: the
// results stored sc1 and published chunk by chunk for the verification blocks of the same launch
// (seq_shard_walkverify)
template <class Src, int C, bool F>
__device__ __forceinline__ void walk_known(const Src& src, const SeqSumBuf& b, int c, int64_t n, uint32_t epoch,
                                           WalkChunk<C>* wb) {
    const int t = threadIdx.x, w = t >> 6;
    if (n <= 0) {
        if (t == 0) b.result[c] = 0.f;
        return;
    }
    if ((b.status[1] >> c) & 1u) return;  // event overflow: the caller falls back (verification blocks skip too)
    const int nev = b.floor_e[b.nch + c];
    const double unit = ldexp(1.0, b.floor_e[c] - 23);
    const uint64_t* EP = b.ev_P + (size_t)c * b.evs;
    const float* EX = b.ev_x + (size_t)c * b.evs;
    float* ES = b.ev_s + (size_t)c * b.evs;
    const int nchunk = (nev + C - 1) / C;
    float s = b.sh ? b.sh->x0[c] : src(c, 0);  // the chain (lane 0 of wave 0)
    if (nchunk > 0) walk_prepare<C, false>(wb[0], 0, min(C, nev), unit, EP, EX, t, kWalkThreads);
    __syncthreads();
    for (int k = 0; k < nchunk; ++k) {
        if (w == 0) {
            if (t == 0) s = walk_chunk(wb[k & 1], min(C, nev - k * C), s);
        } else {
            if (F && t == 64 && k > 1) walk_publish(b, c, epoch, (uint32_t)((k - 1) * C));  // chunks < k-1: stored
            if (k + 1 < nchunk)
                walk_prepare<C, false>(wb[(k + 1) & 1], k + 1, min(C, nev - (k + 1) * C), unit, EP, EX, t - 64,
                                       kWalkThreads - 64);
            if (k > 0) {  // chunk k-1's results (its buffer's f: the preparation above writes only R, Rf, x)
                const WalkChunk<C>& B = wb[(k - 1) & 1];
                const int e0 = (k - 1) * C;
                for (int j = t - 64; j < C; j += kWalkThreads - 64) st32<F>(ES + e0 + j, __float_as_uint(B.f[j]));
                if (F) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
    }
    if (nchunk > 0) {
        const WalkChunk<C>& B = wb[(nchunk - 1) & 1];
        const int e0 = (nchunk - 1) * C;
        for (int j = t; j < nev - e0; j += kWalkThreads) st32<F>(ES + e0 + j, __float_as_uint(B.f[j]));
    }
    if constexpr (F) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) walk_publish(b, c, epoch, (uint32_t)nev);
    }
    if (t == 0) {
        const uint64_t Plast = nev > 0 ? EP[nev - 1] : 0;
        b.result[c] = (float)((double)s + (double)(int64_t)(b.ptot[c] - Plast) * unit);
    }
}

// s_k for every element of block blk (its offsets E0 / P0 in the chain, its prefixes already including them) rebuilt
// from the events; checks s_k == fl(s_{k-1} + x_k); stores the reconstruction.  F: the event lists and results
// were written in this launch (sc1 loads)
template <class Src, bool F>
__device__ __forceinline__ void verify_check(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                             const ElemInfo& in, const bool (&ev)[kSeqPer],
                                             const uint64_t (&Pex)[kSeqPer], const int (&Ein)[kSeqPer], int E0,
                                             uint64_t P0) {
    __shared__ float s_lastv[kSeqThreads / 64];
    __shared__ uint32_t s_bad;
    if (threadIdx.x == 0) s_bad = 0;
    const double unit = ldexp(1.0, b.floor_e[c] - 23);
    const uint64_t* EP = b.ev_P + (size_t)c * b.evs;
    const float* ES = b.ev_s + (size_t)c * b.evs;
    const float x0 = b.sh ? b.sh->x0[c] : src(c, 0);
    const int64_t gb = b.sh ? b.sh->gbase : 0;  // sharded: event positions are global, k0 local
    const int64_t k0 = (int64_t)blk * kSeqBlock + (int64_t)threadIdx.x * kSeqPer;
    // s of element k from (inclusive event count E, inclusive increment prefix P, is-event)
    auto rebuild = [&](bool is_ev, int E, uint64_t Pin) -> float {
        const int idx = E - 1;
        if (is_ev) return __uint_as_float(ld32<F>(ES + idx));
        const float bs = idx >= 0 ? __uint_as_float(ld32<F>(ES + idx)) : x0;
        const uint64_t bp = idx >= 0 ? ld64<F>(EP + idx) : 0;
        return (float)((double)bs + (double)(int64_t)(Pin - bp) * unit);
    };
    // inclusive increment prefix = exclusive + the element's own increment (classify is deterministic)
    float s[kSeqPer];
    {
        bool ev2[kSeqPer];
        uint64_t inc2[kSeqPer];
        classify<Src>(b, c, blk, n, in, b.floor_e[c], pass, ev2, inc2);
#pragma unroll
        for (int i = 0; i < kSeqPer; ++i) {
            const int64_t k = k0 + i;
            s[i] = gb + k == 0 ? x0 : (k < n ? rebuild(ev[i], Ein[i], Pex[i] + inc2[i]) : 0.f);
        }
    }
    // predecessor of the thread's first element
    float prev = __shfl_up(s[kSeqPer - 1], 1, 64);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 63) s_lastv[w] = s[kSeqPer - 1];
    __syncthreads();
    if (lane == 0) {
        if (w > 0) {
            prev = s_lastv[w - 1];
        } else if (gb + k0 > 0) {
            // the previous block's last element (a window's first block: the previous rank's last): the block's
            // offsets are its inclusive values (global once seq_shard_merge has added the ranks before); whether
            // it is an event is read back from the event list (global position)
            const bool is_ev = E0 > 0 && (int)ld32<F>(b.ev_pos + (size_t)c * b.evs + (E0 - 1)) == (int)(gb + k0 - 1);
            prev = rebuild(is_ev, E0, P0);
            if (k0 == 0) b.sh->prev_s[c] = prev;  // (k0 == 0 here only when sharded) the next pass's prediction
        }
    }
    bool bad = false;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        const int64_t k = k0 + i;
        if (k >= n) break;
        const float sp = i == 0 ? prev : s[i - 1];
        if (gb + k > 0) {
            const float want = sp + in.x[i];
            if (__float_as_uint(want) != __float_as_uint(s[i]) && !(want != want && s[i] != s[i])) {
                bad = true;
                uint32_t* fb = b.forced + (size_t)c * (b.nmax / 32 + 1);
                atomicOr(&fb[k >> 5], 1u << (k & 31));
            }
        }
        b.recon[(size_t)c * b.nmax + k] = s[i];
    }
    if (bad) s_bad = 1;
    __syncthreads();
    if (threadIdx.x == 0 && s_bad) atomicOr(&b.status[0], 1u << c);
}

// ---------------------------------------------------------------- the fused tail (single rank)
// seq_count + seq_scan2 + seq_events + seq_walk + seq_verify as ONE launch, seq_tail.  Roles by workgroup index:
// [0, nch) the walkers, then the event blocks, then the verification blocks, both element-major.
//   * an event block classifies its elements (seq_count's work), takes its place in the chain by a decoupled
//     look-back over its predecessors (event counts in the status words, increment sums beside them; lio_dev.hpp
//     lookback_excl), lists its events and publishes its flag word, epoch << 32 | inclusive event count;
//   * a walker follows the flag words in block order and walks each chunk once all its events are listed; every
//     stored chunk of results is published by its progress word, epoch << 32 | events walked;
//   * a verification block does its own classification first, then waits for its event block's offsets and for
//     the walk to pass its last event, then checks.
// Event blocks wait only on lower event blocks, walkers on event blocks, verification blocks on both.  Workgroups
// are dispatched in index order (observed, not promised): every walker and event block is then resident before a
// verification block.  Were it not, the waits' time-outs (kSpinTicks) end them as a failed verification (a
// re-pass) or an event overflow (the serial kernel) — slower, never wrong, never hung.

// the event block (c, blk)
template <class Src>
__device__ __forceinline__ void tail_events(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                            uint32_t epoch, int nb) {
    __shared__ uint64_t s_P;
    __shared__ int s_E;
    ElemInfo in;
    bool ev[kSeqPer];
    uint64_t Pex[kSeqPer];
    int Ein[kSeqPer];
    uint64_t tu;
    int te;
    block_scan_local(src, b, c, blk, n, pass, in, ev, Pex, Ein, tu, te);
    const size_t bi = (size_t)c * b.nblk + blk;
    const uint32_t ep30 = epoch & 0x3fffffffu;  // the status words' epoch field (never 0: seqsum_launch_impl)
    if (threadIdx.x < 64) {  // wave 0: publish the aggregate, look back, publish the inclusive prefix
        unsigned long long* lst = b.lbst + (size_t)c * b.nblk;
        unsigned long long* lag = b.lbagg + (size_t)c * b.nblk;
        unsigned long long* lin = b.lbinc + (size_t)c * b.nblk;
        uint32_t E = 0;
        uint64_t P = 0;
        if (blk > 0) {
            if (threadIdx.x == 0) {
                st64<true>(lag + blk, tu);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                lb_store(lst, blk, lb_word(ep30, 1u, (uint32_t)te));
            }
            bool timeout;
            E = lookback_excl<true>(lst, lag, lin, blk, ep30, P, timeout);
            if (timeout && threadIdx.x == 0) atomicOr(&b.status[1], 1u << c);  // never expected: the serial kernel
        }
        if (threadIdx.x == 0) {
            st64<true>(lin + blk, P + tu);
            // the block's offsets for its verification block, the chain's totals from the last block (sc1: read in
            // this launch)
            st32<true>(b.bEoff + bi, E);
            st64<true>(b.bPoff + bi, P);
            if (blk == nb - 1) {
                st32<true>(b.floor_e + b.nch + c, E + (uint32_t)te);
                st64<true>(b.ptot + c, P + tu);
            }
            if ((int64_t)E + te > b.evcap) atomicOr(&b.status[1], 1u << c);  // the lists overflow: the serial kernel
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lb_store(lst, blk, lb_word(ep30, 2u, E + (uint32_t)te));
            s_E = (int)E;
            s_P = P;
        }
    }
    __syncthreads();
    const int E0 = s_E;
    const uint64_t P0 = s_P;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        Pex[i] += P0;
        Ein[i] += E0;
    }
    store_events<true>(b, c, blk, in, ev, Pex, Ein);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st64<true>(b.evflag + (size_t)c * b.nblk + blk, ((uint64_t)epoch << 32) | (uint32_t)(E0 + te));
}

// the walker's view of the event blocks (one per wave, wave-uniform): blocks [0, jdone) seen published, their
// events [0, eknown) listed.  Advances until eknown >= e_end or every block is seen (then eknown = the total).
// false: time-out
__device__ __forceinline__ bool tail_wait(const SeqSumBuf& b, int c, int nb, int e_end, int& jdone, int& eknown,
                                          uint32_t epoch) {
    const int lane = threadIdx.x & 63;
    const unsigned long long* FL = b.evflag + (size_t)c * b.nblk;
    const uint64_t t0 = wall_clock64();
    while (eknown < e_end && jdone < nb) {
        const int j = jdone + lane;
        const uint64_t wv = j < nb ? ld64<true>(FL + j) : 0ull;
        const bool valid = j < nb && (uint32_t)(wv >> 32) == epoch;
        const uint64_t inval = __ballot(j < nb && !valid);
        const int lim = min(64, nb - jdone);
        const int f = inval ? (int)__builtin_ctzll(inval) : lim;  // published prefix of the window
        if (f > 0) {
            eknown = __shfl((int)(uint32_t)wv, f - 1, 64);
            jdone += f;
        }
        if (f < lim && eknown < e_end) {
            if (wall_clock64() - t0 > kSpinTicks) return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return true;
}

// the walker of chain c
template <class Src>
__device__ __forceinline__ void tail_walk(const Src& src, const SeqSumBuf& b, int c, int64_t n, uint32_t epoch, int nb) {
    constexpr int C = kTailChunk;
    __shared__ WalkChunk<C> wb[2];
    __shared__ int s_abort;
    const int t = threadIdx.x, w = t >> 6;
    if (n <= 0) {
        if (t == 0) b.result[c] = 0.f;
        return;
    }
    const double unit = ldexp(1.0, b.floor_e[c] - 23);
    const uint64_t* EP = b.ev_P + (size_t)c * b.evs;
    const float* EX = b.ev_x + (size_t)c * b.evs;
    float* ES = b.ev_s + (size_t)c * b.evs;
    int jdone = 0, eknown = 0;  // this wave's view of the event blocks
    float s = src(c, 0);        // the chain (lane 0 of wave 0)
    // the events of chunk k (every wave of the caller agrees): m = 0 past the last chunk; false: give up
    auto chunk_events = [&](int k, int& m) -> bool {
        if (!tail_wait(b, c, nb, (k + 1) * C, jdone, eknown, epoch)) return false;
        if (eknown > b.evcap) return false;  // the lists overflowed (the event block flagged it)
        m = max(0, min(C, eknown - k * C));
        return true;
    };
    if (t == 0) s_abort = 0;
    __syncthreads();
    {
        int m0 = 0;
        if (!chunk_events(0, m0)) s_abort = 1;
        walk_prepare<C, true>(wb[0], 0, m0, unit, EP, EX, t, kWalkThreads);
        if (t == 0) wb[0].m = m0;
    }
    __syncthreads();
    int k = 0;
    for (; !s_abort && wb[k & 1].m > 0; ++k) {
        if (w == 0) {
            if (t == 0) s = walk_chunk(wb[k & 1], wb[k & 1].m, s);
        } else {
            if (t == 64 && k > 1) walk_publish(b, c, epoch, (uint32_t)((k - 1) * C));  // chunks < k-1: stored
            int m1 = 0;
            if (wb[k & 1].m == C && !chunk_events(k + 1, m1)) s_abort = 1;
            walk_prepare<C, true>(wb[(k + 1) & 1], k + 1, m1, unit, EP, EX, t - 64, kWalkThreads - 64);
            if (t == 64) wb[(k + 1) & 1].m = m1;
            if (k > 0) {  // chunk k-1's results (its buffer's f: the preparation above writes only R, Rf, x, m)
                const WalkChunk<C>& B = wb[(k - 1) & 1];
                const int e0 = (k - 1) * C;
                for (int j = t - 64; j < C; j += kWalkThreads - 64) st32<true>(ES + e0 + j, __float_as_uint(B.f[j]));
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
    }
    if (s_abort) {  // a time-out or an overflow: the chain goes to the serial kernel
        if (t == 0) {
            atomicOr(&b.status[1], 1u << c);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            walk_publish(b, c, epoch, 0xffffffffu);
        }
        return;
    }
    // k = the chunks walked, every one full but the last; its results are in wb[(k - 1) & 1]
    const int nev = k > 0 ? (k - 1) * C + wb[(k - 1) & 1].m : 0;
    if (k > 0) {
        const WalkChunk<C>& B = wb[(k - 1) & 1];
        const int e0 = (k - 1) * C;
        for (int j = t; j < nev - e0; j += kWalkThreads) st32<true>(ES + e0 + j, __float_as_uint(B.f[j]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        walk_publish(b, c, epoch, (uint32_t)nev);
        const uint64_t Plast = nev > 0 ? ld64<true>(EP + nev - 1) : 0;
        b.result[c] = (float)((double)s + (double)(int64_t)(ld64<true>(b.ptot + c) - Plast) * unit);
    }
}

// the verification block (c, blk)
template <class Src>
__device__ __forceinline__ void tail_verify(const Src& src, const SeqSumBuf& b, int c, int blk, int64_t n, int pass,
                                            uint32_t epoch) {
    __shared__ uint32_t s_skip;
    __shared__ int s_E;
    __shared__ uint64_t s_P;
    ElemInfo in;
    bool ev[kSeqPer];
    uint64_t Pex[kSeqPer];
    int Ein[kSeqPer];
    uint64_t tu;
    int te;
    block_scan_local(src, b, c, blk, n, pass, in, ev, Pex, Ein, tu, te);  // needs no other block
    if (threadIdx.x == 0) {
        const size_t bi = (size_t)c * b.nblk + blk;
        const uint64_t t0 = wall_clock64();
        uint32_t skip = 0, need = 0;
        for (;;) {  // the event block: its offsets
            const uint64_t wv = ld64<true>(b.evflag + bi);
            if ((uint32_t)(wv >> 32) == epoch) {
                need = (uint32_t)wv;
                break;
            }
            if (wall_clock64() - t0 > kSpinTicks) {
                skip = 2;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!skip) {
            s_E = (int)ld32<true>(b.bEoff + bi);
            s_P = ld64<true>(b.bPoff + bi);
        }
        while (!skip) {  // the walk past this block's last event
            const uint64_t wv = ld64<true>(b.wprog + c);
            if ((uint32_t)(wv >> 32) == epoch && (uint32_t)wv >= need) break;
            if (wall_clock64() - t0 > kSpinTicks) {
                skip = 2;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!skip && ((ld32<true>(b.status + 1) >> c) & 1u)) skip = 1;  // the serial kernel takes the chain
        s_skip = skip;
    }
    __syncthreads();
    if (s_skip) {
        if (threadIdx.x == 0 && s_skip == 2) atomicOr(&b.status[0], 1u << c);  // time-out: a re-pass
        return;
    }
    const int E0 = s_E;
    const uint64_t P0 = s_P;
#pragma unroll
    for (int i = 0; i < kSeqPer; ++i) {
        Pex[i] += P0;
        Ein[i] += E0;
    }
    verify_check<Src, true>(src, b, c, blk, n, pass, in, ev, Pex, Ein, E0, P0);
}

template <class Src>
__global__ void __launch_bounds__(kSeqThreads) seq_tail(Src src, SeqSumBuf b, const uint32_t* d_n, int pass, int nch,
                                                        uint32_t epoch) {
    static_assert(kSeqThreads == kWalkThreads, "one block size for every role");
    const uint32_t r = blockIdx.x;
    const int64_t n = *d_n;
    const int nb = (int)((n + kSeqBlock - 1) / kSeqBlock);
    if (r < (uint32_t)nch) {
        tail_walk<Src>(src, b, (int)r, n, epoch, nb);
        return;
    }
    uint32_t i = r - (uint32_t)nch;
    const uint32_t nrole = (uint32_t)b.nblk * (uint32_t)nch;
    const bool verify = i >= nrole;
    if (verify) i -= nrole;
    const int c = (int)(i % (uint32_t)nch), blk = (int)(i / (uint32_t)nch);
    if (blk >= nb) return;
    if (verify)
        tail_verify<Src>(src, b, c, blk, n, pass, epoch);
    else
        tail_events<Src>(src, b, c, blk, n, pass, epoch, nb);
}

// sharded, after seq_shard_merge: the walk over every rank's events and this window's verification in ONE launch.
// Workgroups [0, nch) walk (every event already listed), the rest verify the window's blocks, element-major, each
// after its own classification waiting for the walk to pass its last event (the walkers' progress words; the same
// hand-off as seq_tail's, and its time-out: a failed verification, so a re-pass)
template <class Src>
__global__ void __launch_bounds__(kSeqThreads) seq_shard_walkverify(Src src, SeqSumBuf b, const uint32_t* d_n, int pass,
                                                                    int nch, uint32_t epoch) {
    static_assert(kSeqThreads == kWalkThreads, "one block size for every role");
    __shared__ WalkChunk<kTailChunk> wb[2];
    __shared__ uint32_t s_skip;
    const uint32_t r = blockIdx.x;
    if (r < (uint32_t)nch) {
        walk_known<Src, kTailChunk, true>(src, b, (int)r, b.sh->n_global, epoch, wb);
        return;
    }
    const uint32_t i = r - (uint32_t)nch;
    const int c = (int)(i % (uint32_t)nch), blk = (int)(i / (uint32_t)nch);
    const int64_t n = *d_n;
    if ((int64_t)blk * kSeqBlock >= n) return;
    if ((b.status[1] >> c) & 1u) return;
    ElemInfo in;
    bool ev[kSeqPer];
    uint64_t Pex[kSeqPer];
    int Ein[kSeqPer];
    block_scan_elems(src, b, c, blk, n, pass, in, ev, Pex, Ein);
    const size_t bi = (size_t)c * b.nblk + blk;
    if (threadIdx.x == 0) {
        const uint32_t need = (uint32_t)(b.bEoff[bi] + b.bev[bi]);  // global (merged) offsets: the block's last event
        const uint64_t t0 = wall_clock64();
        uint32_t skip = 0;
        for (;;) {
            const uint64_t wv = ld64<true>(b.wprog + c);
            if ((uint32_t)(wv >> 32) == epoch && (uint32_t)wv >= need) break;
            if (wall_clock64() - t0 > kSpinTicks) {
                skip = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        s_skip = skip;
    }
    __syncthreads();
    if (s_skip) {
        if (threadIdx.x == 0) atomicOr(&b.status[0], 1u << c);  // time-out: a re-pass
        return;
    }
    verify_check<Src, true>(src, b, c, blk, n, pass, in, ev, Pex, Ein, b.bEoff[bi], b.bPoff[bi]);
}

// ---------------------------------------------------------------- sharded chains (lio_seqsum.hpp)
// Every window's place in the chains from the gathered block sums, for this rank's window: seq_scan1's
// formulas run over all ranks' blocks in chain order — a block prefix in windows of kScanWin blocks (the same
// structure as seq_scan1; every rank runs it over the same data with the same launch, so the floors agree bit
// for bit).  One block per chain; lio_seqsum.hpp's seq_shard_offsets_chain states the same arithmetic
// sequentially (the host mirror).  The blocks of rank r are blocks rb[r] .. rb[r + 1) of the chain.
// SeqRecordSum's job (the offsets launch's last workgroup): the records through LDS in chunks, loaded by all lanes,
// then summed by nval lanes in record order
__device__ void seq_record_sum(const SeqRecordSum& rs, double* s_buf, int cap_rec) {
    const int k = threadIdx.x;
    double acc = 0.0;
    for (int64_t g0 = 0; g0 < rs.nrec; g0 += cap_rec) {
        const int m = (int)min((int64_t)cap_rec, rs.nrec - g0);
        for (int e = threadIdx.x; e < m * rs.nval; e += blockDim.x) {
            const int64_t sidx = g0 + e / rs.nval;
            int r = (int)(sidx * rs.world / rs.nrec);  // the rank holding record sidx
            while (r + 1 < rs.world && rs.nrec * (r + 1) / rs.world <= sidx) ++r;
            while (r > 0 && rs.nrec * r / rs.world > sidx) --r;
            const int64_t s0 = rs.nrec * r / rs.world;
            s_buf[e] = rs.recv[(size_t)r * rs.stride + (size_t)(sidx - s0) * rs.width + e % rs.nval];
        }
        __syncthreads();
        if (k < rs.nval)
            for (int j = 0; j < m; ++j) acc += s_buf[j * rs.nval + k];
        __syncthreads();
    }
    if (k < rs.nval) rs.out[k] = acc;
}

__global__ void __launch_bounds__(256) seq_shard_offsets(SeqSumBuf b, const double* __restrict__ recv, int64_t stride,
                                                         int64_t nb_slot, int rank, int world, SeqRecordSum rs) {
    __shared__ double s_sum[kScanWin], s_abs[kScanWin];
    if (rs.out && (int)blockIdx.x == b.nch) {  // block-uniform: the extra job
        seq_record_sum(rs, s_sum, kScanWin / max(rs.nval, 1));
        return;
    }
    __shared__ double s_vw[256 / 64];
    __shared__ int64_t s_rb[65];
    __shared__ double s_off0, s_var0;
    __shared__ int64_t s_n[64];
    const int c = blockIdx.x;
    SeqShard* sh = b.sh;
    if (threadIdx.x < world) s_n[threadIdx.x] = (int64_t)recv[(size_t)threadIdx.x * (size_t)stride];
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t g = 0, pos = 0;
        for (int r = 0; r < world; ++r) {
            const int64_t nr = s_n[r];
            s_rb[r] = g;
            if (r == rank && c == 0) sh->gbase = pos;
            g += min((nr + kSeqBlock - 1) / kSeqBlock, nb_slot);
            pos += nr;
        }
        s_rb[world] = g;
        if (c == 0) {
            sh->n_global = pos;
            sh->n32 = (uint32_t)pos;
        }
        s_off0 = 0.0;
        s_var0 = 0.0;
    }
    __syncthreads();
    const int64_t G = s_rb[world], gmine = s_rb[rank];
    double off = 0.0, mb = 0.0, var = 0.0;
    constexpr int kPerT = kScanWin / 256;
    for (int64_t w0 = 0; w0 < G; w0 += kScanWin) {
        const int m = (int)min((int64_t)kScanWin, G - w0);
        for (int j = threadIdx.x; j < m; j += blockDim.x) {
            const int64_t g = w0 + j;
            int r = 0;
            while (s_rb[r + 1] <= g) ++r;
            const double* bl = recv + (size_t)r * (size_t)stride + kSeqTotHdr + (size_t)c * 2 * nb_slot;
            s_sum[j] = bl[2 * (g - s_rb[r])];
            s_abs[j] = bl[2 * (g - s_rb[r]) + 1];
        }
        __syncthreads();
        double o[kPerT], loc[kPerT], run = 0.0;
#pragma unroll
        for (int i = 0; i < kPerT; ++i) {
            const int j = (int)threadIdx.x * kPerT + i;
            loc[i] = run;
            run = run + (j < m ? s_sum[j] : 0.0);
        }
        double tot;
        const double ex = block_excl(run, s_vw, tot);
        double vrun = 0.0, vloc[kPerT];
#pragma unroll
        for (int i = 0; i < kPerT; ++i) {
            const int j = (int)threadIdx.x * kPerT + i;
            o[i] = off + (ex + loc[i]);
            const double big = j < m ? fabs(o[i]) + s_abs[j] : 0.0;
            if (j < m) mb = fmax(mb, big);
            const double hu = half_ulp_f32(big);
            vloc[i] = vrun;
            vrun = vrun + (j < m ? (double)kSeqBlock * hu * hu : 0.0);
        }
        double vtot;
        const double vex = block_excl(vrun, s_vw, vtot);
#pragma unroll
        for (int i = 0; i < kPerT; ++i) {
            const int64_t g = w0 + (int64_t)threadIdx.x * kPerT + i;
            if (g == gmine && g < w0 + m) {  // this window's first block: its prefix and variance
                s_off0 = o[i];
                s_var0 = var + (vex + vloc[i]);
            }
        }
        off = off + tot;
        var = var + vtot;
        __syncthreads();
    }
    {
        __shared__ double s_mb[256 / 64];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) mb = fmax(mb, __shfl_xor(mb, d, 64));
        if ((threadIdx.x & 63) == 0) s_mb[threadIdx.x >> 6] = mb;
        __syncthreads();
        mb = fmax(fmax(s_mb[0], s_mb[1]), fmax(s_mb[2], s_mb[3]));
    }
    if (threadIdx.x == 0) {
        sh->off0[c] = gmine >= G ? off : s_off0;  // a window without blocks: everything before it
        sh->var0[c] = gmine >= G ? var : s_var0;
        sh->floor_e[c] = mb > 0.0 ? ilogb(mb) - 27 : -200;
    }
}

// The window's event lists for the other ranks (kSeqHdrWords + nch * 2 * slot doubles): n, the overflow bits of
// its own lists, per chain the increment total, the event count and the first element, then per chain `slot`
// events (the increment prefix; the position and the value packed in one word).  A list longer than the slot
// travels cut: every rank sees its count and seq_shard_merge flags it.  One block per chain.
template <class Src>
__global__ void __launch_bounds__(256) seq_shard_pack(Src src, SeqSumBuf b, const uint32_t* d_n, double* __restrict__ msg,
                                                      int slot, int nhead) {
    const int c = blockIdx.x;
    const int64_t n = *d_n;
    // heads (nhead > 0): the first nhead elements of every chain after the events, float, chain-major (a depth block
    // that starts in one window may end in the next: seq_shard_merge appends them after that window)
    if (nhead > 0) {
        float* h = reinterpret_cast<float*>(msg + kSeqHdrWords + (size_t)b.nch * 2 * slot) + (size_t)c * nhead;
        for (int j = threadIdx.x; j < nhead; j += 256) h[j] = j < n ? src(c, j) : 0.f;
    }
    const int nev = b.sh->nev_loc[c];  // this window's events (seq_scan2)
    if (threadIdx.x == 0) {
        if (c == 0) {
            msg[0] = __longlong_as_double((long long)n);
            msg[1] = __longlong_as_double((long long)b.status[1]);
            b.sh->max_nev = 0;  // seq_shard_merge's outputs for this exchange
            b.sh->xflags = 0u;
        }
        msg[2 + c] = __longlong_as_double((long long)b.sh->ptot_loc[c]);
        msg[2 + kSeqMaxChains + c] = __longlong_as_double((long long)nev);
        msg[2 + 2 * kSeqMaxChains + c] = n > 0 ? (double)src(c, 0) : 0.0;
    }
    const int m = min(min(nev, slot), (int)b.evcap);
    double* ev = msg + kSeqHdrWords + (size_t)c * 2 * slot;
    for (int j = threadIdx.x; j < m; j += 256) {
        const size_t i = (size_t)c * b.evcap + j;
        ev[2 * j] = __longlong_as_double((long long)b.lev_P[i]);
        const uint64_t w = (uint64_t)(uint32_t)b.lev_pos[i] | ((uint64_t)__float_as_uint(b.lev_x[i]) << 32);
        ev[2 * j + 1] = __longlong_as_double((long long)w);
    }
}

// Every rank's event lists (rank r's message at recv + r * stride) -> the chain's global lists in element order:
// rank r's events move by the elements and the increments of the ranks before it; this window's block offsets
// become global the same way, the chain's total increment and event count and its first element are set.  A
// rank's list longer than the slot, an overflow of its own list or more events than the global lists hold sets
// the chain's overflow bit (the walk and the verification skip it; the caller re-exchanges or falls back).
// One block per chain.
__global__ void __launch_bounds__(256) seq_shard_merge(SeqSumBuf b, const uint32_t* d_n, const double* __restrict__ recv,
                                                       int64_t stride, int rank, int world, int slot, int nhead,
                                                       float* __restrict__ ext, int64_t ext_stride, float* __restrict__ ghead,
                                                       int nghead) {
    __shared__ int s_eoff[65];
    __shared__ uint64_t s_poff[65];
    __shared__ int64_t s_pos[65];
    __shared__ int s_bad;
    __shared__ double s_hdr[64 * kSeqHdrWords];  // every rank's header, loaded by all lanes at once
    const int c = blockIdx.x;
    SeqShard* sh = b.sh;
    for (int e = threadIdx.x; e < world * kSeqHdrWords; e += 256)
        s_hdr[e] = recv[(size_t)(e / kSeqHdrWords) * (size_t)stride + e % kSeqHdrWords];
    __syncthreads();
    if (threadIdx.x == 0) {
        float x0;
        int mx;
        const int bad = seq_shard_merge_chain(s_hdr, kSeqHdrWords, world, slot, c, b.evs, s_eoff, s_poff, s_pos, x0, mx);
        s_bad = bad;
        b.floor_e[b.nch + c] = s_eoff[world];
        b.ptot[c] = s_poff[world];
        sh->x0[c] = x0;
        atomicMax(&sh->max_nev, mx);
        if (bad) {
            atomicOr(&b.status[1], 1u << c);
            atomicOr(&sh->xflags, (bad & 2 ? 1u : 0u) | (bad & 5 ? 2u : 0u));
        }
    }
    __syncthreads();
    if (nhead > 0 && ext) {
        // the elements after this window: the next ranks' heads in order, up to nhead, appended at ext[c][n ..];
        // the chain's first nghead elements -> ghead[c][..]
        const int64_t nw = *d_n;
        int64_t got = 0;
        for (int r = rank + 1; r < world && got < nhead; ++r) {  // block-uniform
            const double* m = recv + (size_t)r * (size_t)stride;
            const int64_t nr = seq_bits(s_hdr[r * kSeqHdrWords]);
            const int64_t take = min(min(nr, (int64_t)nhead), (int64_t)nhead - got);
            const float* h = reinterpret_cast<const float*>(m + kSeqHdrWords + (size_t)b.nch * 2 * slot) + (size_t)c * nhead;
            for (int64_t j = threadIdx.x; j < take; j += 256) ext[(size_t)c * ext_stride + nw + got + j] = h[j];
            got += take;
        }
        int64_t g = 0;
        for (int r = 0; r < world && g < nghead; ++r) {
            const double* m = recv + (size_t)r * (size_t)stride;
            const int64_t nr = seq_bits(s_hdr[r * kSeqHdrWords]);
            const int64_t take = min(min(nr, (int64_t)nhead), (int64_t)nghead - g);
            const float* h = reinterpret_cast<const float*>(m + kSeqHdrWords + (size_t)b.nch * 2 * slot) + (size_t)c * nhead;
            for (int64_t j = threadIdx.x; j < take; j += 256) ghead[(size_t)c * nghead + g + j] = h[j];
            g += take;
        }
    }
    if (s_bad) return;
    for (int r = 0; r < world; ++r) {
        const double* ev = recv + (size_t)r * (size_t)stride + kSeqHdrWords + (size_t)c * 2 * slot;
        const int ner = s_eoff[r + 1] - s_eoff[r];
        for (int j = threadIdx.x; j < ner; j += 256) {
            const size_t d = (size_t)c * b.evs + s_eoff[r] + j;
            const uint64_t w = (uint64_t)__double_as_longlong(ev[2 * j + 1]);
            b.ev_P[d] = s_poff[r] + (uint64_t)__double_as_longlong(ev[2 * j]);
            b.ev_pos[d] = (int)(s_pos[r] + (int64_t)(uint32_t)w);
            b.ev_x[d] = __uint_as_float((uint32_t)(w >> 32));
        }
    }
    // this window's block offsets: global (its rank's place in the lists; after a re-exchange only the change)
    const int64_t n = *d_n;
    const int nb = (int)((n + kSeqBlock - 1) / kSeqBlock);
    const int de = s_eoff[rank] - sh->e_added[c];
    const uint64_t dp = s_poff[rank] - sh->p_added[c];
    for (int j = threadIdx.x; j < nb; j += 256) {
        b.bEoff[(size_t)c * b.nblk + j] += de;
        b.bPoff[(size_t)c * b.nblk + j] += dp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sh->e_added[c] = s_eoff[rank];
        sh->p_added[c] = s_poff[rank];
    }
}

template <class Src>
void seqsum_launch_impl(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, hipStream_t st) {
    b.evs = b.evcap;  // single rank: the walk reads the lists seq_events writes
    const dim3 g(b.nblk, nch);
    if (pass <= 1) {
        // the forced-event bits of a previous alignment's failures are stale (none were set unless a re-pass ran)
        if (b.forced_dirty) {
            (void)hipMemsetAsync(b.forced, 0, (size_t)nch * (b.nmax / 32 + 1) * sizeof(uint32_t), st);
            b.forced_dirty = false;
        }
        seq_bsum<Src><<<g, kSeqThreads, 0, st>>>(src, b, d_n);
        seq_scan1<<<nch, 256, 0, st>>>(b, d_n, pass);
    } else {
        b.forced_dirty = true;  // the failures that led here set forced bits
        (void)hipMemsetAsync(b.status, 0, 2 * sizeof(uint32_t), st);
    }
    // count, offsets, events, walk and verification: one launch (seq_tail); its grid is sized for the capacity, the
    // blocks past n leave at once
    const uint32_t total = (uint32_t)nch * (1u + 2u * (uint32_t)b.nblk);
    // flags and progress words of earlier launches never match (the look-back's status words keep 30 bits of it)
    do {
        ++b.tail_epoch;
    } while ((b.tail_epoch & 0x3fffffffu) == 0);
    seq_tail<Src><<<total, kSeqThreads, 0, st>>>(src, b, d_n, pass, nch, b.tail_epoch);
}

}  // namespace

template <class Src>
void seqsum_launch(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, hipStream_t st) {
    seqsum_launch_impl(src, nch, d_n, b, pass, st);
}
template void seqsum_launch<SeqPairs>(const SeqPairs&, int, const uint32_t*, SeqSumBuf&, int, hipStream_t);
template void seqsum_launch<SeqSigma>(const SeqSigma&, int, const uint32_t*, SeqSumBuf&, int, hipStream_t);

// sharded pass 1, before the totals exchange: the stale forced bits cleared, the window's block sums, its totals
template <class Src>
void seqsum_shard_head(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, double* tot_out, int64_t nb_slot,
                       hipStream_t st) {
    const dim3 g(b.nblk, nch);
    if (b.forced_dirty) {
        (void)hipMemsetAsync(b.forced, 0, (size_t)nch * (b.nmax / 32 + 1) * sizeof(uint32_t), st);
        b.forced_dirty = false;
    }
    seq_bsum<Src><<<g, kSeqThreads, 0, st>>>(src, b, d_n, tot_out, nb_slot);
}

// after the totals exchange (pass 1) or straight away (pass > 1): offsets, counts, local events, the message
template <class Src>
void seqsum_shard_mid(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, const double* tot_recv,
                      int64_t tot_stride, int64_t nb_slot, int rank, int world, double* msg_out, int slot, int nhead,
                      hipStream_t st, const SeqRecordSum* rs) {
    const dim3 g(b.nblk, nch);
    if (pass <= 1) {
        const SeqRecordSum job = rs && rs->out ? *rs : SeqRecordSum{};
        seq_shard_offsets<<<nch + (job.out ? 1 : 0), 256, 0, st>>>(b, tot_recv, tot_stride, nb_slot, rank, world, job);
        seq_scan1<<<nch, 256, 0, st>>>(b, d_n, pass);
    } else {
        b.forced_dirty = true;  // the failures that led here set forced bits
        (void)hipMemsetAsync(b.status, 0, 2 * sizeof(uint32_t), st);
    }
    seq_count<Src><<<g, kSeqThreads, 0, st>>>(src, b, d_n, pass);
    seq_scan2<<<nch, kSeqThreads, 0, st>>>(b, d_n);
    seq_events<Src><<<g, kSeqThreads, 0, st>>>(src, b, d_n, pass);
    seq_shard_pack<Src><<<nch, 256, 0, st>>>(src, b, d_n, msg_out, slot, nhead);
}

// after the event exchange: the global lists, the walk over all of them, the window's verification
template <class Src>
void seqsum_shard_tail(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, int pass, const double* msg_recv,
                       int64_t msg_stride, int rank, int world, int slot, const SeqHeads& hd, hipStream_t st) {
    const dim3 g(b.nblk, nch);
    seq_shard_merge<<<nch, 256, 0, st>>>(b, d_n, msg_recv, msg_stride, rank, world, slot, hd.nhead, hd.ext,
                                         hd.ext_stride, hd.ghead, hd.nghead);
    (void)g;
    do {
        ++b.tail_epoch;
    } while ((b.tail_epoch & 0x3fffffffu) == 0);
    seq_shard_walkverify<Src><<<(uint32_t)nch * (1u + (uint32_t)b.nblk), kSeqThreads, 0, st>>>(src, b, d_n, pass, nch,
                                                                                                 b.tail_epoch);
}

template <class Src>
void seqsum_shard_repack(const Src& src, int nch, const uint32_t* d_n, SeqSumBuf& b, double* msg_out, int slot,
                         int nhead, hipStream_t st) {
    seq_shard_pack<Src><<<nch, 256, 0, st>>>(src, b, d_n, msg_out, slot, nhead);
}

#define LIO_SEQ_SHARD_INST(S)                                                                                      \
    template void seqsum_shard_head<S>(const S&, int, const uint32_t*, SeqSumBuf&, double*, int64_t, hipStream_t); \
    template void seqsum_shard_mid<S>(const S&, int, const uint32_t*, SeqSumBuf&, int, const double*, int64_t,     \
                                      int64_t, int, int, double*, int, int, hipStream_t, const SeqRecordSum*);     \
    template void seqsum_shard_tail<S>(const S&, int, const uint32_t*, SeqSumBuf&, int, const double*, int64_t, int, \
                                       int, int, const SeqHeads&, hipStream_t);                                    \
    template void seqsum_shard_repack<S>(const S&, int, const uint32_t*, SeqSumBuf&, double*, int, int, hipStream_t);
LIO_SEQ_SHARD_INST(SeqPairs)
LIO_SEQ_SHARD_INST(SeqSigma)
#undef LIO_SEQ_SHARD_INST

int seqsum_shard(SeqSumBuf& b, bool on, hipStream_t st) {
    if (!on) {
        b.sh = nullptr;
        return 0;
    }
    if (b.nch < 1) return -1;
    if (!b.lev_pos) {
        count_alloc(4);
        bool ok = hipMalloc(&b.sh, sizeof(SeqShard)) == hipSuccess &&
                  hipMalloc(&b.lev_pos, (size_t)b.nch * b.evcap_alloc * sizeof(int)) == hipSuccess &&
                  hipMalloc(&b.lev_P, (size_t)b.nch * b.evcap_alloc * sizeof(uint64_t)) == hipSuccess &&
                  hipMalloc(&b.lev_x, (size_t)b.nch * b.evcap_alloc * sizeof(float)) == hipSuccess;
        if (!ok) return -5;
        (void)hipMemsetAsync(b.sh, 0, sizeof(SeqShard), st);
    }
    b.evs = b.evs_alloc;
    return 0;
}

int seqsum_reserve(SeqSumBuf& b, int nch, int64_t nmax, hipStream_t st) {
    if (nch > kSeqMaxChains || nch < 1) return -1;
    nmax = nmax < 1 ? 1 : nmax;
    if (b.nch >= nch && b.nmax >= nmax) return 0;
    const int dbg = b.dbg_noinc;
    seqsum_free(b);
    b.dbg_noinc = dbg;
    b.nch = nch;
    b.nmax = nmax;
    b.nblk = (int)((nmax + kSeqBlock - 1) / kSeqBlock);
    count_alloc(23);
    b.evcap = b.evcap_alloc = nmax / 4 + 1024;  // events are ~0.3 % of a C4 chain; past a quarter the serial kernel is as fast
    b.evs = b.evcap;
    b.evs_alloc = 2 * b.evcap_alloc;  // the walk's lists: sharded, every rank's events (O(window): 2 x its own)
    const size_t nb = (size_t)nch * b.nblk;
    bool ok = hipMalloc(&b.bsum, nb * sizeof(double)) == hipSuccess && hipMalloc(&b.babs, nb * sizeof(double)) == hipSuccess &&
              hipMalloc(&b.boff, nb * sizeof(double)) == hipSuccess && hipMalloc(&b.bdelta, nb * sizeof(double)) == hipSuccess &&
              hipMalloc(&b.btot, nb * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.bev, nb * sizeof(int)) == hipSuccess && hipMalloc(&b.bPoff, nb * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.bEoff, nb * sizeof(int)) == hipSuccess && hipMalloc(&b.floor_e, 3 * nch * sizeof(int)) == hipSuccess &&
              hipMalloc(&b.ptot, nch * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.ev_pos, (size_t)nch * b.evs_alloc * sizeof(int)) == hipSuccess &&
              hipMalloc(&b.ev_P, (size_t)nch * b.evs_alloc * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.ev_x, (size_t)nch * b.evs_alloc * sizeof(float)) == hipSuccess &&
              hipMalloc(&b.ev_s, (size_t)nch * b.evs_alloc * sizeof(float)) == hipSuccess &&
              hipMalloc(&b.recon, (size_t)nch * nmax * sizeof(float)) == hipSuccess &&
              hipMalloc(&b.forced, (size_t)nch * (nmax / 32 + 1) * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&b.status, 4 * sizeof(uint32_t)) == hipSuccess && hipMalloc(&b.result, nch * sizeof(float)) == hipSuccess &&
              hipMalloc(&b.evflag, nb * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.lbst, nb * sizeof(uint64_t)) == hipSuccess && hipMalloc(&b.lbagg, nb * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.lbinc, nb * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&b.wprog, nch * sizeof(uint64_t)) == hipSuccess;
    if (!ok) {
        seqsum_free(b);
        return -5;
    }
    (void)hipMemsetAsync(b.status, 0, 4 * sizeof(uint32_t), st);
    (void)hipMemsetAsync(b.evflag, 0, nb * sizeof(uint64_t), st);
    (void)hipMemsetAsync(b.lbst, 0, nb * sizeof(uint64_t), st);
    (void)hipMemsetAsync(b.wprog, 0, nch * sizeof(uint64_t), st);
    b.tail_epoch = 0;
    return 0;
}

void seqsum_free(SeqSumBuf& b) {
    void* ptrs[] = {b.bsum, b.babs, b.boff,   b.bdelta, b.btot,   b.bev,   b.bPoff, b.bEoff, b.floor_e,
                    b.ptot, b.ev_pos, b.ev_P, b.ev_x, b.ev_s, b.recon, b.forced, b.status, b.result,
                    b.evflag, b.wprog, b.lbst, b.lbagg, b.lbinc,
                    b.sh,   b.lev_pos, b.lev_P, b.lev_x};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    b = SeqSumBuf{};
}

}  // namespace lio
