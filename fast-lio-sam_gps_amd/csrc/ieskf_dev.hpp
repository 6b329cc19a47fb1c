// ieskf_dev.hpp — the iterated ESKF step on the device (one workgroup, double).
//
// Same algebra, same operation order as the host restatement csrc/ieskf.cpp
// (esekfom::update_iterated_dyn_share_modified [U: IKFoM esekfom.hpp, MTK
// SO3.hpp / S2.hpp]): boxminus -> SO3 / S2 Jacobian transport of dx and P ->
// Woodbury 6x6 gain -> boxplus -> convergence test -> (last iteration)
// covariance update, split in two so only the part that needs the sums sits
// on the critical path:
//   pre-step  (block 0 of the evaluation's slot kernel, one wave, concurrent
//             with the point blocks): boxminus, Jacobian transport of dx and
//             of P_prop — they depend on the state only;
//   post-step (the slot kernel's LAST block, one wave, straight after it has
//             summed H^T H / H^T h): Woodbury gain, dx, boxplus, convergence,
//             the final covariance, the next evaluation's pose.
// A whole scan's update is then one enqueued launch sequence with no host
// round trip between the evaluations: the state, the next pose and the loop
// flags live in an IeskfCtl block in HBM, and the kernels of later
// evaluations read their gate (done / converge) and pose from it.  Row /
// column work is spread over the wave's lanes, the manifold maps (SO3 / S2)
// run on lanes 0 / 1 / 2 at once, the 6x6 LU is register-resident.
// Transcendentals come from the device libm (ocml), so results agree with the
// host path to a few ulps, not bit for bit.
//
// The dof < 23 branch (dense rows, a dof x dof inverse) is not run here: the
// step marks the update kIeskfNeedHost and the host re-runs it (lio_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "lio_dev.hpp"

namespace lio {

constexpr int kN = 23;  // state dimension

struct DQuat {
    double w, x, y, z;
};

// same layout as lio::host::State and lio_state (26 doubles)
struct DState {
    double pos[3];
    DQuat rot;
    DQuat offR;
    double offT[3];
    double vel[3], bg[3], ba[3];
    double grav[3];
};
constexpr int kStateWords = 26;
static_assert(sizeof(DState) == kStateWords * sizeof(double), "DState layout");

enum : int { kIeskfRunning = 0, kIeskfOk = 1, kIeskfNeedHost = 2, kIeskfSingular = 3 };

// Published result (host-mapped), in doubles:
//   [0, 26) x, [26, 555) P, [555, 581) x at the last kNN evaluation,
//   [581, 607) x at the last evaluation, [607] res_mean,
//   [608..613] h_evals, knn_calls, converged, n_eff, status, knn_mask (as doubles),
//   [kIeskfOutWords] sequence number, [kIeskfOutWords + 1] checksum
constexpr int kIeskfOutX = 0, kIeskfOutP = 26, kIeskfOutXKnn = 555, kIeskfOutXLast = 581, kIeskfOutRes = 607,
              kIeskfOutInts = 608;
constexpr int kIeskfOutWords = 614;
// Input (host-mapped, written by the host before the launch): x (26), P (529), R, epsi, max_iter
constexpr int kIeskfInWords = 26 + 529 + 3;

struct IeskfCtl {          // HBM, one per ctx
    PoseArg pose;          // pose of the next evaluation
    PoseArg pose_knn;      // pose of the last kNN evaluation (seeded near pass)
    DState x, xp;          // state, propagated state
    double P[kN * kN];     // working covariance (published)
    double Pp[kN * kN];    // propagated covariance
    double Pt[kN * kN];    // this iteration's P_prop transported by the pre-step
    double dxn[kN];        // this iteration's dx_new (pre-step)
    double R, epsi;
    double res_mean;
    int max_iter, i, t, converge, done, status, h_evals, knn_calls, converged, n_eff, knn_mask, pad;
    DState x_knn, x_last;
    unsigned long long seq;
};

// Host-mapped gate of a queued evaluation (launch_h_model_gated): the host writes the poses and
// the command, then the sequence number the gate kernel waits for.
struct GateIn {
    unsigned long long seq;  // alone on its cache line: the only word the gate polls
    unsigned long long pad0[15];
    unsigned long long cmd;  // 1 run, 2 cancel
    unsigned long long pad1[15];
    PoseArg pose;            // the evaluation's pose
    PoseArg pose_knn;        // the last kNN evaluation's pose (seeded near pass)
};

struct IeskfShared {  // the step's LDS
    double P[kN * kN];
    double L[kN * kN];
    double Kx[kN * 12];
    double Mm[36], Minv[36];
    double At[2][9];
    double T2[4];
    double dx[kN], dxn[kN], dxu[kN], Kh[kN];
    double sums[32];
    DState x, xp;
};

namespace dv {

constexpr double kTol = 1e-11;                  // MTK::tolerance<double>()
constexpr double kGravLen = 98090.0 / 10000.0;  // S2<double, 98090, 10000, 1>

__device__ inline DQuat qmul(const DQuat& a, const DQuat& b) {
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}

__device__ inline DQuat qexp(const double* v, double h) {
    const double nrm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (nrm < kTol) return {1.0, h * v[0], h * v[1], h * v[2]};
    const double a = h * nrm, s = sin(a) / nrm;
    return {cos(a), s * v[0], s * v[1], s * v[2]};
}

__device__ inline void qlog(const DQuat& q, double* out) {
    double nv = sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
    if (nv < kTol) nv = kTol;
    const double s = 2.0 / nv * atan(nv / q.w);
    out[0] = s * q.x;
    out[1] = s * q.y;
    out[2] = s * q.z;
}

__device__ inline void skew(const double* v, double* m) {
    m[0] = 0;
    m[1] = -v[2];
    m[2] = v[1];
    m[3] = v[2];
    m[4] = 0;
    m[5] = -v[0];
    m[6] = -v[1];
    m[7] = v[0];
    m[8] = 0;
}
__device__ inline void mul3(const double* A, const double* B, double* C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
__device__ inline void transpose3(const double* A, double* T) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[3 * r + c] = A[3 * c + r];
}

__device__ inline void quat_to_mat(const DQuat& q, double R[9]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz);
    R[1] = txy - twz;
    R[2] = txz + twy;
    R[3] = txy + twz;
    R[4] = 1 - (txx + tzz);
    R[5] = tyz - twx;
    R[6] = txz - twy;
    R[7] = tyz + twx;
    R[8] = 1 - (txx + tyy);
}

// MTK::A_matrix(v)
__device__ inline void a_matrix(const double* v, double* A) {
    const double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double nrm = sqrt(sq);
    for (int k = 0; k < 9; ++k) A[k] = (k % 4 == 0) ? 1.0 : 0.0;
    if (nrm < kTol) return;
    double H[9], H2[9];
    skew(v, H);
    mul3(H, H, H2);
    const double c1 = (1 - cos(nrm)) / sq, c2 = (1 - sin(nrm) / nrm) / sq;
    for (int k = 0; k < 9; ++k) A[k] += c1 * H[k] + c2 * H2[k];
}

__device__ inline void s2_basis(const double* v, double B[6]) {
    const double L = kGravLen;
    if (v[0] + L > kTol) {
        const double d = L + v[0];
        const double b[6] = {-v[1], -v[2], L - v[1] * v[1] / d, -v[2] * v[1] / d, -v[2] * v[1] / d, L - v[2] * v[2] / d};
        for (int k = 0; k < 6; ++k) B[k] = b[k] / L;
    } else {
        const double b[6] = {0, 0, 0, -1, 1, 0};
        for (int k = 0; k < 6; ++k) B[k] = b[k];
    }
}

__device__ inline void s2_jac(const double* gx, const double* gprop, const double* delta, double T[4]) {
    double B[6];
    s2_basis(gx, B);
    double Hx[9];
    skew(gx, Hx);
    double Nm[6];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            Nm[3 * i + j] = (B[i] * Hx[j] + B[2 + i] * Hx[3 + j] + B[4 + i] * Hx[6 + j]) / kGravLen / kGravLen;
    double Bp[6];
    s2_basis(gprop, Bp);
    double Hp[9];
    skew(gprop, Hp);
    double Mx[6];
    const double dn = sqrt(delta[0] * delta[0] + delta[1] * delta[1]);
    if (dn < kTol) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 2; ++c)
                Mx[2 * r + c] = -(Hp[3 * r] * Bp[c] + Hp[3 * r + 1] * Bp[2 + c] + Hp[3 * r + 2] * Bp[4 + c]);
    } else {
        double Bu[3];
        for (int r = 0; r < 3; ++r) Bu[r] = Bp[2 * r] * delta[0] + Bp[2 * r + 1] * delta[1];
        double Re[9];
        quat_to_mat(qexp(Bu, 0.0), Re);  // MTK S2_Mx scalar(1/2) == 0 quirk, as the host
        double Am[9], At[9], RH[9], K[9];
        a_matrix(Bu, Am);
        transpose3(Am, At);
        mul3(Re, Hp, RH);
        mul3(RH, At, K);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 2; ++c)
                Mx[2 * r + c] = -(K[3 * r] * Bp[c] + K[3 * r + 1] * Bp[2 + c] + K[3 * r + 2] * Bp[4 + c]);
    }
    for (int r = 0; r < 2; ++r)
        for (int c = 0; c < 2; ++c)
            T[2 * r + c] = Nm[3 * r] * Mx[c] + Nm[3 * r + 1] * Mx[2 + c] + Nm[3 * r + 2] * Mx[4 + c];
}

__device__ inline void s2_plus(double* g, const double* delta) {
    double B[6];
    s2_basis(g, B);
    double Bu[3];
    for (int r = 0; r < 3; ++r) Bu[r] = B[2 * r] * delta[0] + B[2 * r + 1] * delta[1];
    double Re[9];
    quat_to_mat(qexp(Bu, 0.5), Re);
    const double o0 = Re[0] * g[0] + Re[1] * g[1] + Re[2] * g[2], o1 = Re[3] * g[0] + Re[4] * g[1] + Re[5] * g[2],
                 o2 = Re[6] * g[0] + Re[7] * g[1] + Re[8] * g[2];
    g[0] = o0;
    g[1] = o1;
    g[2] = o2;
}

__device__ inline void s2_minus(const double* v, const double* o, double* res) {
    double Hv[9];
    skew(v, Hv);
    double c[3];
    for (int r = 0; r < 3; ++r) c[r] = Hv[3 * r] * o[0] + Hv[3 * r + 1] * o[1] + Hv[3 * r + 2] * o[2];
    const double vs = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double vc = v[0] * o[0] + v[1] * o[1] + v[2] * o[2];
    const double th = atan2(vs, vc);
    if (vs < kTol) {
        res[0] = fabs(th) > kTol ? 3.1415926 : 0.0;
        res[1] = 0.0;
        return;
    }
    double B[6];
    s2_basis(o, B);
    double Ho[9];
    skew(o, Ho);
    double hv[3];
    for (int r = 0; r < 3; ++r) hv[r] = Ho[3 * r] * v[0] + Ho[3 * r + 1] * v[1] + Ho[3 * r + 2] * v[2];
    for (int i = 0; i < 2; ++i) res[i] = th / vs * (B[i] * hv[0] + B[2 + i] * hv[1] + B[4 + i] * hv[2]);
}

__device__ inline void boxminus(const DState& x, const DState& y, double* d) {
    for (int i = 0; i < 3; ++i) d[i] = x.pos[i] - y.pos[i];
    const DQuat yc{y.rot.w, -y.rot.x, -y.rot.y, -y.rot.z};
    qlog(qmul(yc, x.rot), d + 3);
    const DQuat oc{y.offR.w, -y.offR.x, -y.offR.y, -y.offR.z};
    qlog(qmul(oc, x.offR), d + 6);
    for (int i = 0; i < 3; ++i) {
        d[9 + i] = x.offT[i] - y.offT[i];
        d[12 + i] = x.vel[i] - y.vel[i];
        d[15 + i] = x.bg[i] - y.bg[i];
        d[18 + i] = x.ba[i] - y.ba[i];
    }
    s2_minus(x.grav, y.grav, d + 21);
}

__device__ inline void boxplus(DState& x, const double* d) {
    for (int i = 0; i < 3; ++i) x.pos[i] += d[i];
    x.rot = qmul(x.rot, qexp(d + 3, 0.5));
    x.offR = qmul(x.offR, qexp(d + 6, 0.5));
    for (int i = 0; i < 3; ++i) {
        x.offT[i] += d[9 + i];
        x.vel[i] += d[12 + i];
        x.bg[i] += d[15 + i];
        x.ba[i] += d[18 + i];
    }
    s2_plus(x.grav, d + 21);
}

// 6x6 inverse by LU with partial pivoting, the host's lu_inverse operation order.
// One lane; A and the LU / column scratch live in LDS (no dynamically indexed
// register arrays, which would go to scratch memory).
__device__ inline bool lu_inverse6(double* A, double* LU, double* col, int* piv) {
    for (int k = 0; k < 36; ++k) LU[k] = A[k];
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double best = fabs(LU[k * 6 + k]);
        for (int r = k + 1; r < 6; ++r) {
            const double v = fabs(LU[r * 6 + k]);
            if (v > best) {
                best = v;
                p = r;
            }
        }
        piv[k] = p;
        if (best == 0.0) return false;
        if (p != k)
            for (int c = 0; c < 6; ++c) {
                const double t = LU[k * 6 + c];
                LU[k * 6 + c] = LU[p * 6 + c];
                LU[p * 6 + c] = t;
            }
        const double inv = 1.0 / LU[k * 6 + k];
        for (int r = k + 1; r < 6; ++r) {
            const double f = (LU[r * 6 + k] *= inv);
            if (f != 0.0)
                for (int c = k + 1; c < 6; ++c) LU[r * 6 + c] -= f * LU[k * 6 + c];
        }
    }
    for (int j = 0; j < 6; ++j) {
        for (int i = 0; i < 6; ++i) col[i] = (i == j) ? 1.0 : 0.0;
        for (int k = 0; k < 6; ++k)
            if (piv[k] != k) {
                const double t = col[k];
                col[k] = col[piv[k]];
                col[piv[k]] = t;
            }
        for (int i = 0; i < 6; ++i) {
            double s = col[i];
            for (int k = 0; k < i; ++k) s -= LU[i * 6 + k] * col[k];
            col[i] = s;
        }
        for (int i = 5; i >= 0; --i) {
            double s = col[i];
            for (int k = i + 1; k < 6; ++k) s -= LU[i * 6 + k] * col[k];
            col[i] = s / LU[i * 6 + i];
        }
        for (int i = 0; i < 6; ++i) A[i * 6 + j] = col[i];
    }
    return true;
}

// Dst rows [idx, idx+D), column c := T * Src rows (one column per lane; in place when Dst == Src)
template <int D>
__device__ inline void rows_col(double* Dst, const double* Src, int stride, int idx, const double* T, int c) {
    double tmp[D];
#pragma unroll
    for (int r = 0; r < D; ++r) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) s += T[r * D + k] * Src[(idx + k) * stride + c];
        tmp[r] = s;
    }
#pragma unroll
    for (int r = 0; r < D; ++r) Dst[(idx + r) * stride + c] = tmp[r];
}
// row r, columns [idx, idx+D) := row * T^T (one row per lane)
template <int D>
__device__ inline void cols_row(double* M, int stride, int idx, const double* T, int r) {
    double tmp[D];
    double* row = M + r * stride + idx;
#pragma unroll
    for (int c = 0; c < D; ++c) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < D; ++k) s += row[k] * T[c * D + k];
        tmp[c] = s;
    }
#pragma unroll
    for (int c = 0; c < D; ++c) row[c] = tmp[c];
}

__device__ inline void state_pose(const DState& x, PoseArg& p) {
    quat_to_mat(x.rot, p.R);
    quat_to_mat(x.offR, p.RLI);
    p.q[0] = x.rot.w;
    p.q[1] = x.rot.x;
    p.q[2] = x.rot.y;
    p.q[3] = x.rot.z;
    p.qLI[0] = x.offR.w;
    p.qLI[1] = x.offR.x;
    p.qLI[2] = x.offR.y;
    p.qLI[3] = x.offR.z;
    for (int k = 0; k < 3; ++k) {
        p.t[k] = x.pos[k];
        p.tLI[k] = x.offT[k];
    }
}

__device__ inline unsigned long long mix64(unsigned long long z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

}  // namespace dv

typedef __attribute__((address_space(1))) double gdouble_t;
typedef __attribute__((address_space(1))) unsigned long long gull_t;
typedef __attribute__((address_space(1))) int gint_t;

// Control-block words written by another workgroup of the same kernel (the
// pre-step block) or by other lanes: vector agent-scope loads / stores (sc1),
// never the scalar cache, which is not coherent with vector stores.
__device__ inline double ctl_ld(const double* p) {
    return __hip_atomic_load((gdouble_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline int ctl_ldi(const int* p) {
    return __hip_atomic_load((gint_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void ctl_st(double* p, double v) {
    __hip_atomic_store((gdouble_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void ctl_sti(int* p, int v) {
    __hip_atomic_store((gint_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS hand-off between the lanes of one wave
__device__ inline void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave publishes the finished update to host-mapped memory in one round
// trip: every word stored write-through at system scope, then the sequence
// number and a checksum over (words, seq); the host accepts a result only when
// both match (the same protocol as the per-evaluation sums).
__device__ inline void ieskf_publish(const IeskfCtl* g, double* out, unsigned long long seq) {
    const int lane = threadIdx.x & 63;
    const double* xw = reinterpret_cast<const double*>(&g->x);
    const double* xk = reinterpret_cast<const double*>(&g->x_knn);
    const double* xl = reinterpret_cast<const double*>(&g->x_last);
    unsigned long long h = 0;
    for (int w = lane; w < kIeskfOutWords; w += 64) {
        double v;
        if (w < kIeskfOutP) v = ctl_ld(xw + w);
        else if (w < kIeskfOutXKnn) v = ctl_ld(g->P + (w - kIeskfOutP));
        else if (w < kIeskfOutXLast) v = ctl_ld(xk + (w - kIeskfOutXKnn));
        else if (w < kIeskfOutRes) v = ctl_ld(xl + (w - kIeskfOutXLast));
        else if (w == kIeskfOutRes) v = ctl_ld(&g->res_mean);
        else {
            const int k = w - kIeskfOutInts;
            const int* ip = k == 0 ? &g->h_evals : k == 1 ? &g->knn_calls : k == 2 ? &g->converged
                          : k == 3 ? &g->n_eff : k == 4 ? &g->status : &g->knn_mask;
            v = (double)ctl_ldi(ip);
        }
        h ^= dv::mix64((unsigned long long)__double_as_longlong(v) ^ ((unsigned long long)w * 0x9e3779b97f4a7c15ull));
        __hip_atomic_store((gdouble_t*)(out + w), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) h ^= __shfl_xor(h, off, 64);
    if (lane == 0) {
        __hip_atomic_store((gull_t*)(out + kIeskfOutWords), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store((gull_t*)(out + kIeskfOutWords + 1), h ^ dv::mix64(seq), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// Pre-step (one wave of the slot kernel's block 0, concurrent with the point
// blocks): everything of the iteration that depends on the state alone —
//   dx = x [-] x_prop; dx_new = J^T dx (SO3 A_matrix for rot / offset_R_L_I,
//   S2 Jacobian for grav); P = J^T P_prop J (rows then columns, rot, offR, grav)
// written to g->Pt / g->dxn with agent-scope stores, drained before return.
// The three manifold pieces run on lanes 0 / 1 / 2 at once.
// ---------------------------------------------------------------------------
__device__ inline void ieskf_prestep(IeskfCtl* g, IeskfShared& S) {
    const int lane = threadIdx.x & 63;
    if (lane < kStateWords) {
        reinterpret_cast<double*>(&S.x)[lane] = ctl_ld(reinterpret_cast<const double*>(&g->x) + lane);
        reinterpret_cast<double*>(&S.xp)[lane] = ctl_ld(reinterpret_cast<const double*>(&g->xp) + lane);
    }
#pragma unroll
    for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
        const int e = lane + 64 * k;
        if (e < kN * kN) S.P[e] = g->Pp[e];  // Pp: written by the init kernel only
    }
    wsync();
    if (lane == 0 || lane == 1) {  // SO3 blocks
        const int idx = 3 + 3 * lane;
        const DQuat& a = lane == 0 ? S.x.rot : S.x.offR;
        const DQuat& b = lane == 0 ? S.xp.rot : S.xp.offR;
        const DQuat bc{b.w, -b.x, -b.y, -b.z};
        double d[3];
        dv::qlog(dv::qmul(bc, a), d);
        double Am[9];
        dv::a_matrix(d, Am);
        double* At = S.At[lane];
        dv::transpose3(Am, At);
        for (int r = 0; r < 3; ++r) S.dx[idx + r] = d[r];
        for (int r = 0; r < 3; ++r) S.dxn[idx + r] = At[3 * r] * d[0] + At[3 * r + 1] * d[1] + At[3 * r + 2] * d[2];
    } else if (lane == 2) {  // S2 block
        double d[2];
        dv::s2_minus(S.x.grav, S.xp.grav, d);
        dv::s2_jac(S.x.grav, S.xp.grav, d, S.T2);
        S.dx[21] = d[0];
        S.dx[22] = d[1];
        S.dxn[21] = S.T2[0] * d[0] + S.T2[1] * d[1];
        S.dxn[22] = S.T2[2] * d[0] + S.T2[3] * d[1];
    } else if (lane == 3) {  // linear parts
        for (int i = 0; i < 3; ++i) {
            S.dxn[i] = S.dx[i] = S.x.pos[i] - S.xp.pos[i];
            S.dxn[9 + i] = S.dx[9 + i] = S.x.offT[i] - S.xp.offT[i];
            S.dxn[12 + i] = S.dx[12 + i] = S.x.vel[i] - S.xp.vel[i];
            S.dxn[15 + i] = S.dx[15 + i] = S.x.bg[i] - S.xp.bg[i];
            S.dxn[18 + i] = S.dx[18 + i] = S.x.ba[i] - S.xp.ba[i];
        }
    }
    wsync();
    for (int j = 0; j < 2; ++j) {  // rot, offset_R_L_I: rows, then columns (host order)
        if (lane < kN) dv::rows_col<3>(S.P, S.P, kN, 3 + 3 * j, S.At[j], lane);
        wsync();
        if (lane < kN) dv::cols_row<3>(S.P, kN, 3 + 3 * j, S.At[j], lane);
        wsync();
    }
    if (lane < kN) dv::rows_col<2>(S.P, S.P, kN, 21, S.T2, lane);  // grav
    wsync();
    if (lane < kN) dv::cols_row<2>(S.P, kN, 21, S.T2, lane);
    wsync();
#pragma unroll
    for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
        const int e = lane + 64 * k;
        if (e < kN * kN) ctl_st(g->Pt + e, S.P[e]);
    }
    if (lane < kN) ctl_st(g->dxn + lane, S.dxn[lane]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the block's counter add
}

// 6x6 inverse, the host's lu_inverse (partial-pivot LU, then column solves) in
// registers: every lane factors redundantly (statically indexed, row swaps as
// selects), lane j < 6 solves column j into Minv (LDS).  Returns false if singular.
__device__ inline bool lu_inverse6_wave(const double* Mm, double* Minv) {
    const int lane = threadIdx.x & 63;
    double LU[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) LU[k] = Mm[k];
    int piv[6];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int p = k;
        double best = fabs(LU[k * 6 + k]);
#pragma unroll
        for (int r = k + 1; r < 6; ++r) {
            const double v = fabs(LU[r * 6 + k]);
            if (v > best) {
                best = v;
                p = r;
            }
        }
        piv[k] = p;
        if (best == 0.0) ok = false;
#pragma unroll
        for (int r = k + 1; r < 6; ++r) {
            const bool sw = p == r;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const double u = LU[k * 6 + c], v = LU[r * 6 + c];
                LU[k * 6 + c] = sw ? v : u;
                LU[r * 6 + c] = sw ? u : v;
            }
        }
        const double inv = 1.0 / LU[k * 6 + k];
#pragma unroll
        for (int r = k + 1; r < 6; ++r) {
            const double f = (LU[r * 6 + k] *= inv);
#pragma unroll
            for (int c = k + 1; c < 6; ++c) {
                const double nv = LU[r * 6 + c] - f * LU[k * 6 + c];
                LU[r * 6 + c] = f != 0.0 ? nv : LU[r * 6 + c];
            }
        }
    }
    if (!ok) return false;
    if (lane < 6) {
        const int j = lane;
        double col[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k)
#pragma unroll
            for (int r = k + 1; r < 6; ++r) {
                const bool sw = piv[k] == r;
                const double u = col[k], v = col[r];
                col[k] = sw ? v : u;
                col[r] = sw ? u : v;
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double s = col[i];
#pragma unroll
            for (int k = 0; k < i; ++k) s -= LU[i * 6 + k] * col[k];
            col[i] = s;
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
            double s = col[i];
#pragma unroll
            for (int k = i + 1; k < 6; ++k) s -= LU[i * 6 + k] * col[k];
            col[i] = s / LU[i * 6 + i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) Minv[i * 6 + j] = col[i];
    }
    return true;
}

// ---------------------------------------------------------------------------
// Post-step (one wave of the slot kernel's last block, sums in S.sums; the
// pre-step's g->Pt / g->dxn are complete): bookkeeping, Woodbury gain, dx,
// boxplus, convergence, the final covariance on the last iteration, the next
// evaluation's pose; publishes the update when it has finished.
// ---------------------------------------------------------------------------
__device__ inline void ieskf_poststep(IeskfCtl* g, IeskfShared& S, double* out) {
    const int lane = threadIdx.x & 63;
    const int dof = (int)S.sums[27];
    const int it = ctl_ldi(&g->i), max_iter = ctl_ldi(&g->max_iter);
    const bool conv_in = ctl_ldi(&g->converge) != 0;
    const double R = ctl_ld(&g->R);
    // this evaluation's bookkeeping (host: ++h_evals, knn_calls, n_eff, res_mean, last / kNN pose)
    if (lane < kStateWords) {
        const double v = ctl_ld(reinterpret_cast<const double*>(&g->x) + lane);
        reinterpret_cast<double*>(&S.x)[lane] = v;
        reinterpret_cast<double*>(&S.xp)[lane] = ctl_ld(reinterpret_cast<const double*>(&g->xp) + lane);
        ctl_st(reinterpret_cast<double*>(&g->x_last) + lane, v);
        if (conv_in) ctl_st(reinterpret_cast<double*>(&g->x_knn) + lane, v);
    }
    if (conv_in) {  // this evaluation's pose seeds the next kNN (read before it is overwritten below)
        constexpr int kPoseWords = (int)(sizeof(PoseArg) / sizeof(double));
        if (lane < kPoseWords)
            ctl_st(reinterpret_cast<double*>(&g->pose_knn) + lane, ctl_ld(reinterpret_cast<const double*>(&g->pose) + lane));
    }
    if (lane == 0) {
        ctl_sti(&g->h_evals, ctl_ldi(&g->h_evals) + 1);
        if (conv_in) {
            ctl_sti(&g->knn_calls, ctl_ldi(&g->knn_calls) + 1);
            ctl_sti(&g->knn_mask, ctl_ldi(&g->knn_mask) | (1 << (it + 1)));
        }
        ctl_sti(&g->n_eff, dof);
        ctl_st(&g->res_mean, dof > 0 ? S.sums[28] / dof : 0.0);
    }
    if (dof < 1) {  // ekfom_data.valid = false: the iteration is skipped ("No Effective Points!")
        const bool fin = it + 1 >= max_iter;
        if (lane == 0) {
            ctl_sti(&g->i, it + 1);
            if (fin) {
                ctl_sti(&g->done, 1);
                ctl_sti(&g->status, kIeskfOk);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (fin) ieskf_publish(g, out, g->seq);
        return;
    }
    if (dof < kN) {  // dense-rows branch: the host re-runs this update
        if (lane == 0) {
            ctl_sti(&g->done, 1);
            ctl_sti(&g->status, kIeskfNeedHost);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ieskf_publish(g, out, g->seq);
        return;
    }
#pragma unroll
    for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
        const int e = lane + 64 * k;
        if (e < kN * kN) S.P[e] = ctl_ld(g->Pt + e);
    }
    if (lane < kN) S.dxn[lane] = ctl_ld(g->dxn + lane);
    wsync();
    // ---- gain (Woodbury): Mm = I + HTH (P/R)[:6,:6]
    auto hth = [&](int a, int b) {  // unpacked upper triangle of the sums
        const int r = a < b ? a : b, c = a < b ? b : a;
        return S.sums[r * 6 - r * (r - 1) / 2 + (c - r)];
    };
    if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        double s = 0;
        for (int m = 0; m < 6; ++m) s += hth(a, m) * (S.P[m * kN + b] / R);
        S.Mm[a * 6 + b] = s + (a == b ? 1.0 : 0.0);
    }
    wsync();
    if (!lu_inverse6_wave(S.Mm, S.Minv)) {
        if (lane == 0) {
            ctl_sti(&g->done, 1);
            ctl_sti(&g->status, kIeskfSingular);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ieskf_publish(g, out, g->seq);
        return;
    }
    wsync();
    if (lane < kN) {
        const int r = lane;
        double q[6];
        for (int c = 0; c < 6; ++c) {
            double s = 0;
            for (int m = 0; m < 6; ++m) s += (S.P[r * kN + m] / R) * S.Minv[m * 6 + c];
            q[c] = s;
        }
        double kh = 0;
        for (int c = 0; c < 6; ++c) kh += q[c] * S.sums[21 + c];
        S.Kh[r] = kh;
        for (int c = 0; c < 6; ++c) {
            double s = 0;
            for (int m = 0; m < 6; ++m) s += q[m] * hth(m, c);
            S.Kx[r * 12 + c] = s;
        }
        for (int c = 6; c < 12; ++c) S.Kx[r * 12 + c] = 0.0;
        // dx update: K_h + (K_x - I) dx_new over all 23 columns (K_x zero beyond column 6)
        double s = 0;
        for (int c = 0; c < kN; ++c) s += ((c < 6 ? S.Kx[r * 12 + c] : 0.0) - (r == c ? 1.0 : 0.0)) * S.dxn[c];
        S.dxu[r] = kh + s;
    }
    wsync();
    // ---- boxplus: rot / offR / grav on lanes 0 / 1 / 2, the linear parts on lane 3
    if (lane == 0) S.x.rot = dv::qmul(S.x.rot, dv::qexp(S.dxu + 3, 0.5));
    else if (lane == 1) S.x.offR = dv::qmul(S.x.offR, dv::qexp(S.dxu + 6, 0.5));
    else if (lane == 2) dv::s2_plus(S.x.grav, S.dxu + 21);
    else if (lane == 3)
        for (int i = 0; i < 3; ++i) {
            S.x.pos[i] += S.dxu[i];
            S.x.offT[i] += S.dxu[9 + i];
            S.x.vel[i] += S.dxu[12 + i];
            S.x.bg[i] += S.dxu[15 + i];
            S.x.ba[i] += S.dxu[18 + i];
        }
    const double epsi = ctl_ld(&g->epsi);
    const bool big = lane < kN && fabs(S.dxu[lane]) > epsi;
    bool conv = __ballot(big) == 0ull;
    int t = ctl_ldi(&g->t);
    if (conv) ++t;
    if (!t && it == max_iter - 2) conv = true;
    const bool fin = t > 1 || it == max_iter - 1;
    wsync();
    if (fin) {  // covariance transport by the final dx (host: a_matrix(dxu) / s2_jac(x, x_prop, dxu))
        if (lane == 0 || lane == 1) {
            double Am[9];
            dv::a_matrix(S.dxu + 3 + 3 * lane, Am);
            dv::transpose3(Am, S.At[lane]);
        } else if (lane == 2) {
            dv::s2_jac(S.x.grav, S.xp.grav, S.dxu + 21, S.T2);
        }
#pragma unroll
        for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
            const int e = lane + 64 * k;
            if (e < kN * kN) S.L[e] = S.P[e];
        }
        wsync();
        for (int j = 0; j < 2; ++j) {
            const int idx = 3 + 3 * j;
            if (lane < kN) dv::rows_col<3>(S.L, S.P, kN, idx, S.At[j], lane);                  // L rows from P
            else if (lane < kN + 12) dv::rows_col<3>(S.Kx, S.Kx, 12, idx, S.At[j], lane - kN);  // K_x rows
            wsync();
            if (lane < kN) dv::cols_row<3>(S.L, kN, idx, S.At[j], lane);
            else if (lane < 2 * kN) dv::cols_row<3>(S.P, kN, idx, S.At[j], lane - kN);
            wsync();
        }
        if (lane < kN) dv::rows_col<2>(S.L, S.P, kN, 21, S.T2, lane);
        else if (lane < kN + 12) dv::rows_col<2>(S.Kx, S.Kx, 12, 21, S.T2, lane - kN);
        wsync();
        if (lane < kN) dv::cols_row<2>(S.L, kN, 21, S.T2, lane);
        else if (lane < 2 * kN) dv::cols_row<2>(S.P, kN, 21, S.T2, lane - kN);
        wsync();
#pragma unroll
        for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
            const int e = lane + 64 * k;
            if (e < kN * kN) {
                const int r = e / kN, c = e % kN;
                double s = 0;
                for (int m = 0; m < 12; ++m) s += S.Kx[r * 12 + m] * S.P[m * kN + c];
                ctl_st(g->P + e, S.L[e] - s);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < (kN * kN + 63) / 64; ++k) {
            const int e = lane + 64 * k;
            if (e < kN * kN) ctl_st(g->P + e, S.P[e]);
        }
    }
    // next evaluation's pose and the new state
    if (lane == 0) {
        double Rm[9];
        dv::quat_to_mat(S.x.rot, Rm);
        for (int k = 0; k < 9; ++k) ctl_st(g->pose.R + k, Rm[k]);
        ctl_st(g->pose.q, S.x.rot.w);
        ctl_st(g->pose.q + 1, S.x.rot.x);
        ctl_st(g->pose.q + 2, S.x.rot.y);
        ctl_st(g->pose.q + 3, S.x.rot.z);
        for (int k = 0; k < 3; ++k) ctl_st(g->pose.t + k, S.x.pos[k]);
    } else if (lane == 1) {
        double Rm[9];
        dv::quat_to_mat(S.x.offR, Rm);
        for (int k = 0; k < 9; ++k) ctl_st(g->pose.RLI + k, Rm[k]);
        ctl_st(g->pose.qLI, S.x.offR.w);
        ctl_st(g->pose.qLI + 1, S.x.offR.x);
        ctl_st(g->pose.qLI + 2, S.x.offR.y);
        ctl_st(g->pose.qLI + 3, S.x.offR.z);
        for (int k = 0; k < 3; ++k) ctl_st(g->pose.tLI + k, S.x.offT[k]);
    }
    if (lane < kStateWords) ctl_st(reinterpret_cast<double*>(&g->x) + lane, reinterpret_cast<const double*>(&S.x)[lane]);
    if (lane == 0) {
        ctl_sti(&g->converge, conv ? 1 : 0);
        ctl_sti(&g->t, t);
        ctl_sti(&g->i, it + 1);
        if (fin) {
            ctl_sti(&g->done, 1);
            ctl_sti(&g->status, kIeskfOk);
            ctl_sti(&g->converged, t > 1 ? 1 : 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (fin) ieskf_publish(g, out, g->seq);
}

// Loads the update's input from host-mapped memory into the control block
// (one workgroup, before the first evaluation of the sequence).
__device__ inline void ieskf_init(IeskfCtl* g, const double* in, unsigned long long seq) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int k = tid; k < kStateWords; k += nt) {
        const double v = in[k];
        reinterpret_cast<double*>(&g->x)[k] = v;
        reinterpret_cast<double*>(&g->xp)[k] = v;
        reinterpret_cast<double*>(&g->x_knn)[k] = v;
        reinterpret_cast<double*>(&g->x_last)[k] = v;
    }
    for (int k = tid; k < kN * kN; k += nt) {
        const double v = in[kStateWords + k];
        g->P[k] = v;
        g->Pp[k] = v;
    }
    if (tid == 0) {
        g->R = in[kStateWords + kN * kN];
        g->epsi = in[kStateWords + kN * kN + 1];
        g->max_iter = (int)in[kStateWords + kN * kN + 2];
        g->res_mean = 0.0;
        g->i = -1;
        g->t = 0;
        g->converge = 1;
        g->done = 0;
        g->status = kIeskfRunning;
        g->h_evals = g->knn_calls = g->converged = g->n_eff = g->knn_mask = 0;
        g->seq = seq;
        DState x;
        double* xw = reinterpret_cast<double*>(&x);
        for (int k = 0; k < kStateWords; ++k) xw[k] = in[k];
        dv::state_pose(x, g->pose);
        g->pose_knn = g->pose;
    }
}

}  // namespace lio
