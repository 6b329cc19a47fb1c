// lio_match.hip — FAST-LIO h_share_model on gfx950.
//
// Per h-evaluation:
//
//   ekfom_data.converge == true (redo the kNN):
//     knn_near_kernel  512 threads = 64 points, 8 lanes per point:
//       body->world (double, stored float) -> exact grid 5-NN over shells 0-1,
//       cell points scanned lane-strided (coalesced), private top-5 lists
//       merged by a shuffle butterfly; unresolved points -> far queue
//     knn_far_kernel   one block per queued point, the rest of its search box
//     plane_kernel     lane = point: gate (found == 5 && d2[4] <= 5) ->
//       esti_plane (QR, registers) -> pd2, s-gate -> H row (double) ->
//       30-value DPP wave reduction -> block partial
//     writes: nn_idx[5] (20 B), plane abcd (16 B), sel (1 B)
//   ekfom_data.converge == false: h_model_reuse_kernel, lane = point
//     body->world -> cached plane -> pd2, s-gate -> H row -> block partial
//   the last block of plane/reuse to finish (agent-scope counter) sums the
//     block partials in a fixed order (deterministic) into host-mapped memory
//     + a sequence number (zero-copy result, no finalize launch)
//
// The per-point dense H (effct x 12 doubles) of the reference is never
// materialised: the IESKF only consumes H^T H and H^T h.
#include <hip/hip_ext.h>

#include "ieskf_dev.hpp"
#include "lio_dev.hpp"
#include "lio_kernels.hpp"

#include <algorithm>
#include <cstdlib>

namespace lio {

constexpr int kBlock = 256;  // plane / reuse: 1 point per lane (1024-thread blocks measured slower)

constexpr int kGroup = 8;   // lanes cooperating on one query's kNN
constexpr int kKnnBlock = 512;
constexpr int kFarBlock = 128;  // threads per far query (64 / 256 / 512: LIO_FAR_THREADS, measured slower)
constexpr int kFarBlocks = 1024;  // blocks striding the far queue (one query per block)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// pd2 / s-gate / H row of one selected point (h_share_model [U])
__device__ __forceinline__ bool residual_row(const MatchArgs& a, const PoseArg& ps, float bx, float by, float bz, float wx, float wy,
                                             float wz, const float4& pl, double J[6], double& h, double& res) {
    const float pd2 = ((pl.x * wx + pl.y * wy) + pl.z * wz) + pl.w;
    const double b0 = bx, b1 = by, b2 = bz;
    const double pn = sqrt((b0 * b0 + b1 * b1) + b2 * b2);
    const float s = (float)(1.0 - a.s_coef * (double)fabsf(pd2) / sqrt(pn));
    if (!((double)s > a.s_gate)) return false;
    h_row(ps, bx, by, bz, pl.x, pl.y, pl.z, J);
    h = -(double)pd2;
    res = (double)fabsf(pd2);
    return true;
}

// ekfom_data.converge == true, pass 1: 512 threads = 64 queries, 8 lanes per
// query run the exact 5-NN over shells 0-1 cooperatively (group_knn_near).
// Queries whose 5th neighbour is not yet provably final (sparse
// neighbourhoods, ~0.4% of a dense scan) are queued, with their list, for
// the wave-per-query far pass instead of holding their wave: a kernel runs as
// long as its slowest wave.  Written for 8 waves/SIMD (<= 64 VGPRs).
template <bool DBG, bool SEEDED, int U = 4, bool DEV = false, int NB = kKnnBlock, int UO = 4>
__global__ void __launch_bounds__(NB) __attribute__((amdgpu_waves_per_eu(8, 8))) knn_near_kernel(MatchArgs a) {
    if constexpr (DEV)  // device-resident update: this slot runs only while the loop asks for a kNN
        if (a.ctl->done || !a.ctl->converge) return;
    const PoseArg& ps = DEV ? a.ctl->pose : a.pose;
    constexpr int G = kGroup;
    constexpr int QPB = NB / G;  // 64 queries per block
    __shared__ uint32_t s_tab[QPB][72];      // per-group shell-1 slot table
    __shared__ float s_q[4][QPB];            // per query: world point (and the seeded pass's bound)
    __shared__ int s_c[3][QPB];              //            its cell
    const int blk = xcd_block(blockIdx.x, gridDim.x);
    const int sub = threadIdx.x % G;
    const int q = threadIdx.x / G;
    const int i = blk * QPB + q;
    const unsigned long long t_beg = a.tdbg ? wall_clock64() : 0ull;
    // the per-query transforms once per query, not once per lane of its group: wave 0, lane = query
    if (threadIdx.x < QPB) {
        const int iq = blk * QPB + (int)threadIdx.x;
        if (iq < a.n) {
            const float bx = a.body[3 * iq], by = a.body[3 * iq + 1], bz = a.body[3 * iq + 2];
            float wx, wy, wz;
            body_to_world(ps, bx, by, bz, wx, wy, wz);
            s_q[0][threadIdx.x] = wx;
            s_q[1][threadIdx.x] = wy;
            s_q[2][threadIdx.x] = wz;
            const int cx = cell_coord(wx, a.grid.ox, a.grid.inv_cell);
            const int cy = cell_coord(wy, a.grid.oy, a.grid.inv_cell);
            const int cz = cell_coord(wz, a.grid.oz, a.grid.inv_cell);
            s_c[0][threadIdx.x] = cx;
            s_c[1][threadIdx.x] = cy;
            s_c[2][threadIdx.x] = cz;
            if constexpr (SEEDED) {
                float wox, woy, woz;
                if constexpr (DEV) {
                    body_to_world(a.ctl->pose_knn, bx, by, bz, wox, woy, woz);
                } else {  // float affine map of the previous kNN pose: w_old within ~1e-5 m, covered by the bound's margin
                    const float* M = a.knn_M;
                    wox = ((M[0] * bx + M[1] * by) + M[2] * bz) + M[3];
                    woy = ((M[4] * bx + M[5] * by) + M[6] * bz) + M[7];
                    woz = ((M[8] * bx + M[9] * by) + M[10] * bz) + M[11];
                }
                const bool inside = (unsigned)cx < (unsigned)a.grid.nx && (unsigned)cy < (unsigned)a.grid.ny &&
                                    (unsigned)cz < (unsigned)a.grid.nz;
                s_q[3][threadIdx.x] = seeded_bound(inside, a.nn_d5[iq], wox, woy, woz, wx, wy, wz, a.range_sq, a.seed_scale);
            }
        }
    }
    __syncthreads();
    if (i >= a.n) return;
    const float wx = s_q[0][q], wy = s_q[1][q], wz = s_q[2][q];
    TopK<5> tk;
    tk.init(a.range_sq);
    SearchStats st{0, 0, 0};
    bool done, whole = false;
    if constexpr (SEEDED) {  // this scan's previous kNN against the same map: the triangle bound (no re-gathers)
        const int r = group_knn_seeded<5, G, U>(a.grid, s_q[3][q], s_c[0][q], s_c[1][q], s_c[2][q], wx, wy, wz, a.range_sq, sub,
                                                tk, s_tab[threadIdx.x / G]);
        done = r > 0;
        whole = r < 0;
    } else {
        done = group_knn_near<5, G, false, U, UO>(a.grid, wx, wy, wz, s_c[0][q], s_c[1][q], s_c[2][q], 1, sub, tk,
                                              DBG ? &st : nullptr, s_tab[threadIdx.x / G]);
    }
    const bool far = !done && a.max_shell > 1;
    if constexpr (DBG) {
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            st.cells += __shfl_xor(st.cells, off, 64);
            st.points += __shfl_xor(st.points, off, 64);
        }
        if (sub == 0) {
            a.dbg[3 * (size_t)i] = st.cells;
            a.dbg[3 * (size_t)i + 1] = st.points;
            a.dbg[3 * (size_t)i + 2] = far ? 2 : st.shell;
        }
    }
    if (far) {
        if (sub == 0) {
            const int slot = atomicAdd(a.far_count, 1);
            a.far_list[slot] = whole ? (int)((unsigned)i | 0x80000000u) : i;  // sign bit: search the block too
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                a.far_d[5 * (size_t)slot + j] = tk.d(j);
                a.far_id[5 * (size_t)slot + j] = tk.id(j);
            }
        }
        if (a.tdbg && (threadIdx.x & 63) == 0) {
            const size_t wv = (size_t)blockIdx.x * (NB / 64) + (threadIdx.x >> 6);
            a.tdbg[2 * wv] = t_beg;
            a.tdbg[2 * wv + 1] = wall_clock64();
        }
        return;
    }
#pragma unroll
    for (int js = 0; js < 5; js += G) {
        const int jj = js + sub;
        if (jj < 5) {
            int v = tk.id(0);
#pragma unroll
            for (int j = 1; j < 5; ++j)
                if (jj == j) v = tk.id(j);
            a.nn_idx[5 * (size_t)i + jj] = v == kNone ? -1 : v;
        }
    }
    if (sub == 5) a.nn_d5[i] = tk.id(4) == kNone ? INFINITY : tk.d(4);
    if (a.tdbg && (threadIdx.x & 63) == 0) {
        const size_t wv = (size_t)blockIdx.x * (NB / 64) + (threadIdx.x >> 6);
        a.tdbg[2 * wv] = t_beg;
        a.tdbg[2 * wv + 1] = wall_clock64();
    }
}

// Pass 2: the queued queries, one block each (block_knn_box_flat over the
// rest of the query's search box).  Fixed grid; every block strides the queue
// and exits once past its end.
template <bool DEV = false, int NT = kFarBlock>
__global__ void __launch_bounds__(NT) knn_far_kernel(MatchArgs a) {
    if constexpr (DEV)
        if (a.ctl->done || !a.ctl->converge) return;
    const PoseArg& ps = DEV ? a.ctl->pose : a.pose;
    __shared__ uint32_t s_b[NT], s_off[NT + 1], s_w[NT / 64];
    __shared__ uint64_t s_lists[(NT / 64) * 5];
    const int cnt = *a.far_count;
    for (int f = blockIdx.x; f < cnt; f += gridDim.x) {
        const int e = a.far_list[f];
        const int i = e & 0x7fffffff;
        float wx, wy, wz;
        body_to_world(ps, a.body[3 * i], a.body[3 * i + 1], a.body[3 * i + 2], wx, wy, wz);
        TopK<5> tk;
#pragma unroll
        for (int j = 0; j < 5; ++j) tk.k[j] = knn_key(a.far_d[5 * (size_t)f + j], a.far_id[5 * (size_t)f + j]);
        block_knn_box_flat<5, NT>(a.grid, wx, wy, wz, s_b, s_off, s_w, s_lists, tk, e < 0);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int j = 0; j < 5; ++j) a.nn_idx[5 * (size_t)i + j] = tk.id(j) == kNone ? -1 : tk.id(j);
            a.nn_d5[i] = tk.id(4) == kNone ? INFINITY : tk.d(4);
        }
    }
}

// Block partial -> global, and the LAST block to finish sums all partials
// (fixed order: deterministic) into the host-mapped result + sequence number,
// so no separate finalize launch.  Hand-off per MI355X_MICROARCH.md
// § visibility, row "one lane of each storing workgroup ... agent-scope atomic
// add / the workgroup whose add came last": the partial is stored
// write-through (sc1: agent-scope relaxed atomic store), the storing wave
// drains (vmcnt(0)), a barrier, ONE lane adds to the counter; the block
// whose add returns nblocks-1 reads every partial with sc1 loads
// (agent-scope relaxed atomic loads) after a barrier.  No release fence (an
// agent release per block writes back the XCD's L2: 8 -> 35 us measured).
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned int guint;
typedef __attribute__((address_space(1))) unsigned long long gull;

// Host hand-off in ONE round trip: wave lanes 0-31 store the 32 sums, lane 32
// the sequence number, lane 33 a checksum of (sums, seq), all write-through at
// system scope (sc0 sc1) and unordered.  The host (lio_capi.cpp wait_result)
// accepts a result once it reads the expected sequence number AND sums whose
// checksum matches: a word still in flight (or the previous evaluation's)
// fails the check and the host polls again; once the kernel has completed,
// every word has landed.  No system release (its write-back and the wait for
// the sums' completion before the flag cost 1.7-2 us per evaluation).
// Called by all 64 lanes of one wave; lane l < 32 passes sum l.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void publish_host(double t, double* out, unsigned long long* seq_out, unsigned long long seq) {
    const int lane = threadIdx.x & 63;
    unsigned long long h =
        lane < 32 ? mix64((unsigned long long)__double_as_longlong(t) ^ ((unsigned long long)lane * 0x9e3779b97f4a7c15ull))
                  : 0ull;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) h ^= __shfl_xor(h, off, 64);
    h = __shfl(h, 0, 64);
    if (lane < 32) __hip_atomic_store((gdouble*)(out + lane), t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (lane == 32) __hip_atomic_store((gull*)seq_out, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (lane == 33) __hip_atomic_store((gull*)(seq_out + 1), h ^ mix64(seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block partial -> global; returns true in the LAST block to finish, whose
// lanes < 32 then hold the 32 fixed-order sums in `t` (wave 0; block-uniform
// return value).  fused_final == 0: partial only, the finalize launch sums.
// slot: this block's partial index (-1: none); npart partials are summed; ncount
// blocks take part in the counter.  All threads of the block call it.
template <int BS = kBlock>
__device__ __forceinline__ bool block_partial_last(const MatchArgs& a, double (*red)[32], double& t, int slot, int npart,
                                                   int ncount) {
    __shared__ int s_last;
    const int nb = npart;
    t = 0.0;
    if (!a.fused_final) {  // separate finalize_kernel launch (A/B switch LIO_FUSED_FINAL=0)
        if (threadIdx.x < 32) {
            double s = 0.0;
#pragma unroll
            for (int w = 0; w < BS / 64; ++w) s += red[w][threadIdx.x];
            a.partials[(size_t)blockIdx.x * 32 + threadIdx.x] = s;
        }
        return false;
    }
    if (slot >= 0 && threadIdx.x < 32) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < BS / 64; ++w) s += red[w][threadIdx.x];
        __hip_atomic_store((gdouble*)(a.partials + (size_t)slot * 32 + threadIdx.x), s, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add((guint*)a.done_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)(ncount - 1);
    }
    __syncthreads();
    if (!s_last) return false;  // block-uniform
    // fixed-order sum: 8 row groups x 32 columns, then the groups in order
    const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
    constexpr int NG = BS / 32;
    const int per = (nb + NG - 1) / NG;
    const int b0 = grp * per, b1 = min(nb, b0 + per);
    double acc = 0.0;
    int b = b0;
    // batches of 32 sc1 loads in flight per thread (cross-XCD: each batch is an L2 miss), the
    // last batch masked rather than finished one load at a time (a serial tail of 27 loads
    // doubled the kernel at C5's 469 blocks)
    for (; b < b1; b += 32) {
        double v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k)
            v[k] = b + k < b1 ? __hip_atomic_load((gdouble*)(a.partials + (size_t)(b + k) * 32 + col), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : 0.0;
#pragma unroll
        for (int k = 0; k < 32; ++k) acc += v[k];
    }
    __shared__ double sg[NG][33];
    sg[grp][col] = acc;
    __syncthreads();
    if (threadIdx.x < 32)
#pragma unroll
        for (int g = 0; g < NG; ++g) t += sg[g][threadIdx.x];
    if (threadIdx.x == 0)
        __hip_atomic_store((guint*)a.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    return true;
}

// the last block publishes the sums to the host (lio_match)
template <int BS = kBlock>
__device__ __forceinline__ void publish_and_finalize(const MatchArgs& a, double (*red)[32]) {
    double t;
    if (block_partial_last<BS>(a, red, t, blockIdx.x, gridDim.x, gridDim.x) && threadIdx.x < 64)
        publish_host(t, a.sums_out, a.seq_out, a.seq);
}

// One lane's H-row contribution [HTH(21), HTh(6), cnt, res, hh] added into v[32].
__device__ __forceinline__ void accum_row(double (&v)[32], const double J[6], double h, double res, double cnt) {
    int q = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) v[q++] += J[r] * J[c];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[21 + r] += J[r] * h;
    v[27] += cnt;
    v[28] += res;
    v[29] += h * h;
}

// Points per lane of the plane / reuse kernels (LIO_PPL, default kPplDefault): PPL > 1 gives each
// lane several points' loads in flight and fewer block partials for the last block to gather.
constexpr int kPplDefault = 2;
static int ppl_setting() {
    static const int v = [] {
        const char* e = std::getenv("LIO_PPL");
        const int p = e ? std::atoi(e) : kPplDefault;
        return (p == 1 || p == 2 || p == 4) ? p : kPplDefault;
    }();
    return v;
}

// Host-loop path: the plane kernel in 512-thread blocks, 1 point per lane (2 waves per SIMD at 88
// VGPRs instead of 1 at 120 with 256 x 2; same partial count): 14.5 -> 13.5 us at C3; the reuse kernel
// in 512-thread blocks, 2 points per lane (half the partials for the last block): 9.1 -> 8.8 us.  An
// explicit LIO_PPL selects the 256-thread kernels with that PPL (diagnostics).
constexpr int kPlaneBlock = 512;
static bool plane_wide() {
    static const bool v = std::getenv("LIO_PPL") == nullptr;
    return v;
}

// Plane pass body, lane = PPL points (strided by the block size, coalesced): gate
// (found == 5 && d2[4] <= 5), esti_plane, pd2, s-gate, H row, summed into v.
template <int PPL, int BS = kBlock>
__device__ __forceinline__ void plane_points(const MatchArgs& a, const PoseArg& ps, int blk, double (&v)[32]) {
    const int i0 = blk * BS * PPL + threadIdx.x;
    // all points' ids first, then all neighbour gathers: PPL independent chains in flight
    int id[PPL][5];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
#pragma unroll
        for (int j = 0; j < 5; ++j) id[k][j] = i < a.n ? a.nn_idx[5 * (size_t)i + j] : -1;
    }
    float P[PPL][5][3];
#pragma unroll
    for (int k = 0; k < PPL; ++k)
        if (id[k][4] >= 0)
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const float4 q = a.map_by_id[id[k][j]];
                P[k][j][0] = q.x;
                P[k][j][1] = q.y;
                P[k][j][2] = q.z;
            }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
        if (i < a.n) {
            // sorted list: the 5th exists => all exist, d2 <= range by construction
            bool sel = id[k][4] >= 0;
            if (sel) {
                const float bx = a.body[3 * i], by = a.body[3 * i + 1], bz = a.body[3 * i + 2];
                float abcd[4];
                sel = esti_plane_dev(P[k], a.plane_thr, abcd);
                const float4 pl = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
                a.planes[i] = pl;
                if (sel) {
                    float wx, wy, wz;
                    body_to_world(ps, bx, by, bz, wx, wy, wz);
                    double J[6], h, res;
                    sel = residual_row(a, ps, bx, by, bz, wx, wy, wz, pl, J, h, res);
                    if (sel) accum_row(v, J, h, res, 1.0);
                }
            }
            a.sel[i] = sel ? 1 : 0;
        }
    }
}

// Reuse pass body (ekfom_data.converge == false: cached Nearest_Points / planes), PPL points per lane.
template <int PPL, int BS = kBlock>
__device__ __forceinline__ void reuse_points(const MatchArgs& a, const PoseArg& ps, int blk, double (&v)[32]) {
    const int i0 = blk * BS * PPL + threadIdx.x;
    // every point's three loads issued together (one round trip instead of sel -> body/plane)
    bool sel[PPL];
    float b[PPL][3];
    float4 pl[PPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = i0 + k * BS;
        sel[k] = false;
        if (i < a.n) {
            sel[k] = a.sel[i] != 0;
            b[k][0] = a.body[3 * i];
            b[k][1] = a.body[3 * i + 1];
            b[k][2] = a.body[3 * i + 2];
            pl[k] = a.planes[i];
        }
    }
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        if (sel[k]) {
            const int i = i0 + k * BS;
            float wx, wy, wz;
            body_to_world(ps, b[k][0], b[k][1], b[k][2], wx, wy, wz);
            double J[6], h, res;
            const bool s = residual_row(a, ps, b[k][0], b[k][1], b[k][2], wx, wy, wz, pl[k], J, h, res);
            if (s) accum_row(v, J, h, res, 1.0);
            a.sel[i] = s ? 1 : 0;
        }
    }
}

// Pass 3 (kNN evaluations): plane_points, wave sums, 4 wave partials combined in
// LDS -> block partial; the last block publishes.  Resets the far queue for the
// next kNN evaluation.
// GATED: queued ahead of the host's decision (launch_h_model_gated): the pose comes from the control
// block the gate kernel fills, and a cancelled evaluation (ctl->done) does nothing.
template <int PPL, bool GATED = false, int BS = kBlock>
__global__ void __launch_bounds__(BS) plane_kernel(MatchArgs a) {
    if constexpr (GATED)
        if (a.ctl->done) return;
    const PoseArg& ps = GATED ? a.ctl->pose : a.pose;
    __shared__ double red[BS / 64][32];
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = 0.0;
    plane_points<PPL, BS>(a, ps, blockIdx.x, v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double tot = wave_sum32(v, lane);
    if (lane < 32) red[wid][wave_sum32_index(lane)] = tot;
    __syncthreads();
    publish_and_finalize<BS>(a, red);
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.far_count = 0;
}

// ekfom_data.converge == false: reuse_points, same reduction and publish.
template <int PPL, bool GATED = false, int BS = kBlock>
__global__ void __launch_bounds__(BS) h_model_reuse_kernel(MatchArgs a) {
    if constexpr (GATED)
        if (a.ctl->done) return;
    const PoseArg& ps = GATED ? a.ctl->pose : a.pose;
    __shared__ double red[BS / 64][32];
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = 0.0;
    reuse_points<PPL, BS>(a, ps, blockIdx.x, v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double tot = wave_sum32(v, lane);
    if (lane < 32) red[wid][wave_sum32_index(lane)] = tot;
    __syncthreads();
    publish_and_finalize<BS>(a, red);
}

// Device-resident update (lio_ieskf_update): one h-evaluation slot of
// the enqueued sequence.  Gate and path come from the control block: nothing
// once the loop has finished, the plane pass when this iteration redoes the
// kNN (ekfom_data.converge), the reuse pass otherwise.  Grid = 1 + point
// blocks: block 0 runs the IESKF pre-step (state-only part, ieskf_dev.hpp)
// while blocks 1.. do the points; the last block to finish (any of them) sums
// the partials and runs the post-step, which publishes the finished update.
template <int PPL>
__global__ void __launch_bounds__(kBlock) h_eval_dev_kernel(MatchArgs a) {
    IeskfCtl* g = a.ctl;
    if (g->done) return;
    const bool knn = g->converge != 0;
    __shared__ double red[kBlock / 64][32];
    __shared__ IeskfShared S;
    const int np = (int)gridDim.x - 1;  // point blocks
    double t;
    bool last;
    if (blockIdx.x == 0) {
        if (threadIdx.x < 64) ieskf_prestep(g, S);
        last = block_partial_last(a, red, t, -1, np, np + 1);
    } else {
        double v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) v[q] = 0.0;
        if (knn)
            plane_points<PPL>(a, g->pose, blockIdx.x - 1, v);
        else
            reuse_points<PPL>(a, g->pose, blockIdx.x - 1, v);
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        const double tot = wave_sum32(v, lane);
        if (lane < 32) red[wid][wave_sum32_index(lane)] = tot;
        __syncthreads();
        if (knn && blockIdx.x == 1 && threadIdx.x == 0) *a.far_count = 0;
        last = block_partial_last(a, red, t, blockIdx.x - 1, np, np + 1);
    }
    if (!last || threadIdx.x >= 64) return;
    if (threadIdx.x < 32) S.sums[threadIdx.x] = t;
    wsync();
    ieskf_poststep(g, S, a.ieskf_out);
}

// Gate of an evaluation queued before the host's decision (launch_h_model_gated): one lane
// waits for the host to publish gate word `seq` (host-mapped, written after the pose) and copies
// the command and the poses into the control block, which the evaluation's kernels behind it read
// (DEV near / far, GATED plane / reuse).  Command: 1 run, 2 cancel.  The wait is bounded (20 ms,
// then cancel), so a host that never answers cannot hold the queue.
__global__ void __launch_bounds__(64) eval_gate_kernel(IeskfCtl* g, const GateIn* in, unsigned long long seq, int knn) {
    typedef __attribute__((address_space(1))) const unsigned long long cgull;
    typedef __attribute__((address_space(1))) const double cgdouble;
    const int lane = threadIdx.x;
    int ok = 0;
    if (lane == 0) {  // one lane polls (relaxed, uncached system-scope loads: an acquire would
                      // invalidate the L2 on every poll); the others wait at the reconvergence point
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            if (__hip_atomic_load((cgull*)&in->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= seq) {
                ok = 1;
                break;
            }
            if (wall_clock64() - t0 > 2000000ull) break;  // 100 MHz constant clock: 20 ms
            __builtin_amdgcn_s_sleep(8);  // ~0.2 us between PCIe polls
        }
    }
    ok = __shfl(ok, 0, 64);
    unsigned long long cmd = 2;
    if (ok && lane == 0) cmd = __hip_atomic_load((cgull*)&in->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    cmd = __shfl(cmd, 0, 64);
    if (cmd == 1) {
        // the two poses (2 x 32 words) in ONE round trip: a word per lane, issued after seq was seen
        // (the host wrote them before seq)
        constexpr int W = (int)(sizeof(PoseArg) / sizeof(double));
        static_assert(2 * W <= 64, "eval_gate_kernel: a pose word per lane");
        if (lane < 2 * W && (knn || lane < W)) {
            const double* src = lane < W ? reinterpret_cast<const double*>(&in->pose) + lane
                                         : reinterpret_cast<const double*>(&in->pose_knn) + (lane - W);
            double* dst = lane < W ? reinterpret_cast<double*>(&g->pose) + lane
                                   : reinterpret_cast<double*>(&g->pose_knn) + (lane - W);
            *dst = __hip_atomic_load((cgdouble*)src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (lane == 0) {
        g->converge = knn;
        g->done = cmd == 1 ? 0 : 1;
    }
}

// Device-resident update: the control block from the host-mapped input (one block).
__global__ void __launch_bounds__(256) ieskf_init_kernel(IeskfCtl* g, const double* in, unsigned long long seq) {
    ieskf_init(g, in, seq);
}

// Fixed-order sum of nblocks x 32 partials -> 32 sums (one block of 1024):
// 32 row groups x 32 columns, each thread issues its rows' loads 8 at a time
// and adds them in row order, then the 32 group sums in group order
// (deterministic for a given nblocks).  The sums go straight to the ctx's
// host-mapped result (zero-copy), followed by the sequence number the host
// waits on (no copy launch, no stream-sync round trip).
__global__ void __launch_bounds__(1024) finalize_kernel(const double* __restrict__ partials, int nblocks,
                                                       double* __restrict__ out, unsigned long long* seq_out,
                                                       unsigned long long seq) {
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
    if (threadIdx.x < 64) {
        double t = 0.0;
        if (threadIdx.x < 32)
#pragma unroll
            for (int g = 0; g < 32; ++g) t += sg[g][threadIdx.x];
        publish_host(t, out, seq_out, seq);
    }
}

// ikd-Tree Nearest_Search(point, k, Nearest_Points, Point_Distance, max_dist)
// over a batch of query points: 8 lanes per query, exact (d2, id)-ordered
// 5-NN within d2 <= bound (bound = INFINITY: unbounded, any number of shells),
// the first k kept.  Missing neighbours: id -1, d2 = INFINITY.
__global__ void __launch_bounds__(256) map_knn_kernel(GridDev g, const float* __restrict__ q, int n, float bound,
                                                      int max_shell, int k, int32_t* __restrict__ idx,
                                                      float* __restrict__ d2) {
    constexpr int G = kGroup;
    const int sub = threadIdx.x % G;
    const int i = blockIdx.x * (256 / G) + threadIdx.x / G;
    if (i >= n) return;
    TopK<5> tk;
    tk.init(bound);
    group_knn_exact<5, G>(g, q[3 * (size_t)i], q[3 * (size_t)i + 1], q[3 * (size_t)i + 2], max_shell, sub, tk);
    if (sub < k) {
        int v = tk.id(0);
        float d = tk.d(0);
#pragma unroll
        for (int j = 1; j < 5; ++j)
            if (sub == j) {
                v = tk.id(j);
                d = tk.d(j);
            }
        const bool ok = v != kNone;
        idx[(size_t)i * k + sub] = ok ? v : -1;
        if (d2) d2[(size_t)i * k + sub] = ok ? d : INFINITY;
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
// Near pass on the host-loop path (A/B: profiles/r02_near_ab.txt):
//  * 2 loads in flight in the seeded table scan and in the own-cell scan (56 / 58 VGPRs, no scratch):
//    the 4-load forms sit at the 64-VGPR cap with 8-12 B/lane of spills (kNN h-evaluation traffic
//    23.2 vs 18.6 MB at C3) for ~0.5 us less per pass; LIO_NEAR_NOSPILL=0 restores them;
//  * 256-thread blocks (32 queries; finer grain for the second round of blocks at C3): near pass
//    -0.5 to -0.8 us; LIO_NEAR_BLOCK=512 restores 64 queries per block.
static bool near_nospill() {
    static const bool v = [] {
        const char* e = std::getenv("LIO_NEAR_NOSPILL");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}

static int near_block() {
    static const int v = [] {
        const char* e = std::getenv("LIO_NEAR_BLOCK");
        const int b = e ? std::atoi(e) : 256;
        return (b == 512 || b == 128) ? b : 256;
    }();
    return v;
}

template <int NB>
static void launch_near_nb(const MatchArgs& a, int nq, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    if (a.prior) {
        if (near_nospill())
            hipExtLaunchKernelGGL((knn_near_kernel<false, true, 2, false, NB, 4>), dim3(nq), dim3(NB), 0, st, e0, e1, 0, a);
        else
            hipExtLaunchKernelGGL((knn_near_kernel<false, true, 4, false, NB, 4>), dim3(nq), dim3(NB), 0, st, e0, e1, 0, a);
    } else {
        if (near_nospill())
            hipExtLaunchKernelGGL((knn_near_kernel<false, false, 4, false, NB, 2>), dim3(nq), dim3(NB), 0, st, e0, e1, 0, a);
        else
            hipExtLaunchKernelGGL((knn_near_kernel<false, false, 4, false, NB, 4>), dim3(nq), dim3(NB), 0, st, e0, e1, 0, a);
    }
}

static void launch_near(const MatchArgs& a, int nq, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    if (near_block() == 256)
        launch_near_nb<256>(a, nq, st, e0, e1);
    else if (near_block() == 128)
        launch_near_nb<128>(a, nq, st, e0, e1);
    else
        launch_near_nb<512>(a, nq, st, e0, e1);
}

int launch_h_model(const MatchArgs& a, bool redo, hipStream_t st, hipEvent_t* marks) {
    if (a.n == 0) return 0;
    const int ppl = ppl_setting();
    const int nb = (a.n + kBlock * ppl - 1) / (kBlock * ppl);
    // hipExtLaunchKernelGGL with null events is a plain launch; with events (timing) the command
    // processor stamps them at the kernel's own start / end
    hipEvent_t m[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (marks)
        for (int k = 0; k < 8; ++k) m[k] = marks[k];
    if (redo) {
        const int qpb = (a.dbg ? kKnnBlock : near_block()) / kGroup;
        const int nq = (a.n + qpb - 1) / qpb;
        if (a.dbg)
            hipExtLaunchKernelGGL(knn_near_kernel<true, false>, dim3(nq), dim3(kKnnBlock), 0, st, m[0], m[1], 0, a);
        else
            launch_near(a, nq, st, m[0], m[1]);
        static const int far_blocks = [] {  // LIO_FAR_BLOCKS: diagnostics override of the far-pass grid
            const char* e = std::getenv("LIO_FAR_BLOCKS");
            const int v = e ? std::atoi(e) : 0;
            return v > 0 ? std::min(v, 4096) : kFarBlocks;
        }();
        static const int far_nt = [] {  // LIO_FAR_THREADS: threads per far query (diagnostics: 64 / 256 / 512)
            const char* e = std::getenv("LIO_FAR_THREADS");
            return e ? std::atoi(e) : kFarBlock;
        }();
        if (a.max_shell > 1) {
            if (far_nt == 64)
                hipExtLaunchKernelGGL((knn_far_kernel<false, 64>), dim3(far_blocks), dim3(64), 0, st, m[2], m[3], 0, a);
            else if (far_nt == 256)
                hipExtLaunchKernelGGL((knn_far_kernel<false, 256>), dim3(far_blocks), dim3(256), 0, st, m[2], m[3], 0, a);
            else if (far_nt == 512)
                hipExtLaunchKernelGGL((knn_far_kernel<false, 512>), dim3(far_blocks), dim3(512), 0, st, m[2], m[3], 0, a);
            else
                hipExtLaunchKernelGGL(knn_far_kernel<false>, dim3(far_blocks), dim3(kFarBlock), 0, st, m[2], m[3], 0, a);
        }
        if (plane_wide()) {
            const int nbp = (a.n + kPlaneBlock - 1) / kPlaneBlock;
            hipExtLaunchKernelGGL((plane_kernel<1, false, kPlaneBlock>), dim3(nbp), dim3(kPlaneBlock), 0, st, m[4], m[5], 0, a);
            return nbp;
        }
        if (ppl == 4)
            hipExtLaunchKernelGGL(plane_kernel<4>, dim3(nb), dim3(kBlock), 0, st, m[4], m[5], 0, a);
        else if (ppl == 2)
            hipExtLaunchKernelGGL(plane_kernel<2>, dim3(nb), dim3(kBlock), 0, st, m[4], m[5], 0, a);
        else
            hipExtLaunchKernelGGL(plane_kernel<1>, dim3(nb), dim3(kBlock), 0, st, m[4], m[5], 0, a);
        return nb;
    }
    if (plane_wide()) {
        const int nbr = (a.n + 2 * kPlaneBlock - 1) / (2 * kPlaneBlock);
        hipExtLaunchKernelGGL((h_model_reuse_kernel<2, false, kPlaneBlock>), dim3(nbr), dim3(kPlaneBlock), 0, st, m[6], m[7], 0, a);
        return nbr;
    }
    if (ppl == 4)
        hipExtLaunchKernelGGL(h_model_reuse_kernel<4>, dim3(nb), dim3(kBlock), 0, st, m[6], m[7], 0, a);
    else if (ppl == 2)
        hipExtLaunchKernelGGL(h_model_reuse_kernel<2>, dim3(nb), dim3(kBlock), 0, st, m[6], m[7], 0, a);
    else
        hipExtLaunchKernelGGL(h_model_reuse_kernel<1>, dim3(nb), dim3(kBlock), 0, st, m[6], m[7], 0, a);
    return nb;
}

void launch_h_model_gated(const MatchArgs& a, bool redo, const GateIn* in, unsigned long long gate_seq, hipStream_t st) {
    if (a.n == 0) return;
    const int ppl = ppl_setting();
    const int nb = (a.n + kBlock * ppl - 1) / (kBlock * ppl);
    eval_gate_kernel<<<1, 64, 0, st>>>(a.ctl, in, gate_seq, redo ? 1 : 0);
    if (redo) {  // only the near pass: far + plane are launched at release (launch_knn_tail), hidden behind it
        const int nq = (a.n + kKnnBlock / kGroup - 1) / (kKnnBlock / kGroup);
        if (a.prior)
            knn_near_kernel<false, true, 4, true><<<nq, kKnnBlock, 0, st>>>(a);
        else
            knn_near_kernel<false, false, 4, true><<<nq, kKnnBlock, 0, st>>>(a);
        return;
    }
    if (ppl == 4)
        h_model_reuse_kernel<4, true><<<nb, kBlock, 0, st>>>(a);
    else if (ppl == 2)
        h_model_reuse_kernel<2, true><<<nb, kBlock, 0, st>>>(a);
    else
        h_model_reuse_kernel<1, true><<<nb, kBlock, 0, st>>>(a);
}

int launch_knn_tail(const MatchArgs& a, hipStream_t st) {
    if (a.n == 0) return 0;
    const int ppl = ppl_setting();
    const int nb = (a.n + kBlock * ppl - 1) / (kBlock * ppl);
    if (a.max_shell > 1) knn_far_kernel<false><<<kFarBlocks, kFarBlock, 0, st>>>(a);
    if (ppl == 4)
        plane_kernel<4, false><<<nb, kBlock, 0, st>>>(a);
    else if (ppl == 2)
        plane_kernel<2, false><<<nb, kBlock, 0, st>>>(a);
    else
        plane_kernel<1, false><<<nb, kBlock, 0, st>>>(a);
    return nb;
}

void launch_ieskf_dev(const MatchArgs& a, const double* in, unsigned long long seq, int max_iter, hipStream_t st,
                      hipEvent_t* marks) {
    const int ppl = ppl_setting();
    const int nb = (a.n + kBlock * ppl - 1) / (kBlock * ppl);
    const int nq = (a.n + kKnnBlock / kGroup - 1) / (kKnnBlock / kGroup);
    static const int far_blocks = [] {
        const char* e = std::getenv("LIO_FAR_BLOCKS");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? std::min(v, 4096) : kFarBlocks;
    }();
    ieskf_init_kernel<<<1, 256, 0, st>>>(a.ctl, in, seq);
    for (int e = 0; e <= max_iter; ++e) {
        hipEvent_t* m = marks ? marks + 6 * e : nullptr;
        hipEvent_t m0 = m ? m[0] : nullptr, m1 = m ? m[1] : nullptr, m2 = m ? m[2] : nullptr, m3 = m ? m[3] : nullptr,
                   m4 = m ? m[4] : nullptr, m5 = m ? m[5] : nullptr;
        // slot 0 always redoes the kNN (converge starts true); later kNN slots are seeded by the
        // scan's previous lists against the unchanged map
        if (e == 0)
            hipExtLaunchKernelGGL((knn_near_kernel<false, false, 4, true>), dim3(nq), dim3(kKnnBlock), 0, st, m0, m1, 0, a);
        else
            hipExtLaunchKernelGGL((knn_near_kernel<false, true, 4, true>), dim3(nq), dim3(kKnnBlock), 0, st, m0, m1, 0, a);
        if (a.max_shell > 1)
            hipExtLaunchKernelGGL(knn_far_kernel<true>, dim3(far_blocks), dim3(kFarBlock), 0, st, m2, m3, 0, a);
        if (ppl == 4)
            hipExtLaunchKernelGGL(h_eval_dev_kernel<4>, dim3(nb + 1), dim3(kBlock), 0, st, m4, m5, 0, a);
        else if (ppl == 2)
            hipExtLaunchKernelGGL(h_eval_dev_kernel<2>, dim3(nb + 1), dim3(kBlock), 0, st, m4, m5, 0, a);
        else
            hipExtLaunchKernelGGL(h_eval_dev_kernel<1>, dim3(nb + 1), dim3(kBlock), 0, st, m4, m5, 0, a);
    }
}

size_t ieskf_ctl_bytes() { return sizeof(IeskfCtl); }

void launch_debug(const MatchArgs& a, float* world, float* d2, float* abcd_pd2, hipStream_t st) {
    if (a.n == 0) return;
    debug_kernel<<<(a.n + 255) / 256, 256, 0, st>>>(a, world, d2, abcd_pd2);
}

void launch_h_rows(const MatchArgs& a, double* rows, int64_t max_rows, int64_t* n_rows, hipStream_t st) {
    h_rows_kernel<<<1, 1024, 0, st>>>(a, rows, max_rows, n_rows);
}


void launch_finalize(const MatchArgs& a, int nblocks, hipStream_t st) {
    if (!a.fused_final) finalize_kernel<<<1, 1024, 0, st>>>(a.partials, nblocks, a.sums_out, a.seq_out, a.seq);
}

void launch_map_knn(const GridDev& g, const float* q, int n, float bound, int max_shell, int k, int32_t* idx,
                    float* d2, hipStream_t st) {
    if (n <= 0) return;
    map_knn_kernel<<<(n + 256 / kGroup - 1) / (256 / kGroup), 256, 0, st>>>(g, q, n, bound, max_shell, k, idx, d2);
}

int match_blocks(int n) {  // partial slots (plane / reuse kernels)
    return (n + kBlock - 1) / kBlock;  // the PPL = 1 count bounds every PPL
}

}  // namespace lio
