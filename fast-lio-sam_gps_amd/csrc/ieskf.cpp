// ieskf.cpp — iterated error-state Kalman update on the IKFoM manifold.
//
// Restates esekfom::esekf<state_ikfom, 12, input_ikfom>::
// update_iterated_dyn_share_modified(R, solve_time) [U: IKFoM esekfom.hpp,
// MTK SO3.hpp / S2.hpp, FAST-LIO use-ikfom.hpp] for the state order
//   pos(0) rot(3) offset_R_L_I(6) offset_T_L_I(9) vel(12) bg(15) ba(18) grav(21, S2)
// The measurement model is the GPU h_share_model (lio_match): it returns
// H^T H / H^T h over the effective points, so the dense effct x 12 Jacobian is
// only materialised in the rare dof < 23 branch.
#include "ieskf.hpp"

#include <chrono>
#include <cmath>
#include <cstring>

namespace lio {
namespace host {

namespace {

constexpr double kTol = 1e-11;                  // MTK::tolerance<double>()
constexpr double kGravLen = 98090.0 / 10000.0;  // S2<double, 98090, 10000, 1>
constexpr int kSO3[2] = {3, 6};
constexpr int kS2 = 21;

Quat qmul(const Quat& a, const Quat& b) {
    return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}

// MTK::exp: quaternion of rotation vector v with half-angle factor h
Quat qexp(const double* v, double h) {
    const double nrm = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (nrm < kTol) return {1.0, h * v[0], h * v[1], h * v[2]};
    const double a = h * nrm, s = std::sin(a) / nrm;
    return {std::cos(a), s * v[0], s * v[1], s * v[2]};
}

// SO3::log (MTK::log, scale 2, plus/minus periodicity)
void qlog(const Quat& q, double* out) {
    double nv = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
    if (nv < kTol) nv = kTol;
    const double s = 2.0 / nv * std::atan(nv / q.w);
    out[0] = s * q.x;
    out[1] = s * q.y;
    out[2] = s * q.z;
}

struct M3 {
    double a[9];
    double& operator()(int r, int c) { return a[3 * r + c]; }
    double operator()(int r, int c) const { return a[3 * r + c]; }
};

M3 skew(const double* v) {
    M3 m{{0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0}};
    return m;
}
M3 mul(const M3& A, const M3& B) {
    M3 C;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C(r, c) = A(r, 0) * B(0, c) + A(r, 1) * B(1, c) + A(r, 2) * B(2, c);
    return C;
}
M3 transpose(const M3& A) {
    M3 T;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T(r, c) = A(c, r);
    return T;
}

// MTK::A_matrix(v)
M3 a_matrix(const double* v) {
    const double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double nrm = std::sqrt(sq);
    M3 A{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    if (nrm < kTol) return A;
    const M3 H = skew(v), H2 = mul(H, H);
    const double c1 = (1 - std::cos(nrm)) / sq, c2 = (1 - std::sin(nrm) / nrm) / sq;
    for (int i = 0; i < 9; ++i) A.a[i] += c1 * H.a[i] + c2 * H2.a[i];
    return A;
}

// S2 (typ 1) tangent basis, 3x2 row-major
void s2_basis(const double* v, double B[6]) {
    const double L = kGravLen;
    if (v[0] + L > kTol) {
        const double d = L + v[0];
        const double b[6] = {-v[1], -v[2], L - v[1] * v[1] / d, -v[2] * v[1] / d, -v[2] * v[1] / d, L - v[2] * v[2] / d};
        for (int i = 0; i < 6; ++i) B[i] = b[i] / L;
    } else {
        const double b[6] = {0, 0, 0, -1, 1, 0};
        std::memcpy(B, b, sizeof(b));
    }
}

// res_temp_S2 = Nx(x) * Mx(x_prop, delta), 2x2 row-major
void s2_jac(const double* gx, const double* gprop, const double* delta, double T[4]) {
    double B[6];
    s2_basis(gx, B);
    const M3 Hx = skew(gx);
    double N[6];  // 2x3 = B^T Hx / L^2
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            N[3 * i + j] = (B[i] * Hx(0, j) + B[2 + i] * Hx(1, j) + B[4 + i] * Hx(2, j)) / kGravLen / kGravLen;
    double Bp[6];
    s2_basis(gprop, Bp);
    const M3 Hp = skew(gprop);
    double Mx[6];  // 3x2
    const double dn = std::sqrt(delta[0] * delta[0] + delta[1] * delta[1]);
    if (dn < kTol) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 2; ++c)
                Mx[2 * r + c] = -(Hp(r, 0) * Bp[c] + Hp(r, 1) * Bp[2 + c] + Hp(r, 2) * Bp[4 + c]);
    } else {
        double Bu[3];
        for (int r = 0; r < 3; ++r) Bu[r] = Bp[2 * r] * delta[0] + Bp[2 * r + 1] * delta[1];
        // MTK S2_Mx passes scalar(1/2) == 0 to MTK::exp => identity rotation [U quirk]
        M3 Re;
        quat_to_mat(qexp(Bu, 0.0), Re.a);
        const M3 At = transpose(a_matrix(Bu));
        const M3 K = mul(mul(Re, Hp), At);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 2; ++c) Mx[2 * r + c] = -(K(r, 0) * Bp[c] + K(r, 1) * Bp[2 + c] + K(r, 2) * Bp[4 + c]);
    }
    for (int r = 0; r < 2; ++r)
        for (int c = 0; c < 2; ++c) T[2 * r + c] = N[3 * r] * Mx[c] + N[3 * r + 1] * Mx[2 + c] + N[3 * r + 2] * Mx[4 + c];
}

void s2_plus(double* g, const double* delta) {
    double B[6];
    s2_basis(g, B);
    double Bu[3];
    for (int r = 0; r < 3; ++r) Bu[r] = B[2 * r] * delta[0] + B[2 * r + 1] * delta[1];
    double Re[9];
    quat_to_mat(qexp(Bu, 0.5), Re);
    const double o[3] = {Re[0] * g[0] + Re[1] * g[1] + Re[2] * g[2], Re[3] * g[0] + Re[4] * g[1] + Re[5] * g[2],
                         Re[6] * g[0] + Re[7] * g[1] + Re[8] * g[2]};
    std::memcpy(g, o, sizeof(o));
}

void s2_minus(const double* v, const double* o, double* res) {
    const M3 Hv = skew(v);
    double c[3];
    for (int r = 0; r < 3; ++r) c[r] = Hv(r, 0) * o[0] + Hv(r, 1) * o[1] + Hv(r, 2) * o[2];
    const double vs = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double vc = v[0] * o[0] + v[1] * o[1] + v[2] * o[2];
    const double th = std::atan2(vs, vc);
    if (vs < kTol) {
        res[0] = std::fabs(th) > kTol ? 3.1415926 : 0.0;
        res[1] = 0.0;
        return;
    }
    double B[6];
    s2_basis(o, B);
    const M3 Ho = skew(o);
    double hv[3];
    for (int r = 0; r < 3; ++r) hv[r] = Ho(r, 0) * v[0] + Ho(r, 1) * v[1] + Ho(r, 2) * v[2];
    for (int i = 0; i < 2; ++i) res[i] = th / vs * (B[i] * hv[0] + B[2 + i] * hv[1] + B[4 + i] * hv[2]);
}

void boxminus(const State& x, const State& y, double* d) {
    for (int i = 0; i < 3; ++i) d[i] = x.pos[i] - y.pos[i];
    const Quat yc{y.rot.w, -y.rot.x, -y.rot.y, -y.rot.z};
    qlog(qmul(yc, x.rot), d + 3);
    const Quat oc{y.offR.w, -y.offR.x, -y.offR.y, -y.offR.z};
    qlog(qmul(oc, x.offR), d + 6);
    for (int i = 0; i < 3; ++i) {
        d[9 + i] = x.offT[i] - y.offT[i];
        d[12 + i] = x.vel[i] - y.vel[i];
        d[15 + i] = x.bg[i] - y.bg[i];
        d[18 + i] = x.ba[i] - y.ba[i];
    }
    s2_minus(x.grav, y.grav, d + 21);
}

void boxplus(State& x, const double* d) {
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

// In-place inverse by LU with partial pivoting (PartialPivLU::inverse()).
bool lu_inverse(Mat& A, int n) {
    std::vector<int> piv(n);
    Mat LU = A;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = std::fabs(LU[(size_t)k * n + k]);
        for (int r = k + 1; r < n; ++r) {
            const double v = std::fabs(LU[(size_t)r * n + k]);
            if (v > best) {
                best = v;
                p = r;
            }
        }
        piv[k] = p;
        if (best == 0.0) return false;
        if (p != k)
            for (int c = 0; c < n; ++c) std::swap(LU[(size_t)k * n + c], LU[(size_t)p * n + c]);
        const double inv = 1.0 / LU[(size_t)k * n + k];
        for (int r = k + 1; r < n; ++r) {
            const double f = (LU[(size_t)r * n + k] *= inv);
            if (f != 0.0)
                for (int c = k + 1; c < n; ++c) LU[(size_t)r * n + c] -= f * LU[(size_t)k * n + c];
        }
    }
    // solve LU X = P I column by column
    Mat X((size_t)n * n, 0.0);
    std::vector<double> col(n);
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < n; ++i) col[i] = (i == j) ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k)
            if (piv[k] != k) std::swap(col[k], col[piv[k]]);
        for (int i = 0; i < n; ++i) {
            double s = col[i];
            for (int k = 0; k < i; ++k) s -= LU[(size_t)i * n + k] * col[k];
            col[i] = s;
        }
        for (int i = n - 1; i >= 0; --i) {
            double s = col[i];
            for (int k = i + 1; k < n; ++k) s -= LU[(size_t)i * n + k] * col[k];
            col[i] = s / LU[(size_t)i * n + i];
        }
        for (int i = 0; i < n; ++i) X[(size_t)i * n + j] = col[i];
    }
    A.swap(X);
    return true;
}

// rows [idx, idx+d) of Dst := T * rows of Src (columns [0, ncols))
void rows_apply(Mat& Dst, const Mat& Src, int stride, int idx, const double* T, int d, int ncols) {
    double tmp[3];
    for (int c = 0; c < ncols; ++c) {
        for (int r = 0; r < d; ++r) {
            double s = 0;
            for (int k = 0; k < d; ++k) s += T[r * d + k] * Src[(size_t)(idx + k) * stride + c];
            tmp[r] = s;
        }
        for (int r = 0; r < d; ++r) Dst[(size_t)(idx + r) * stride + c] = tmp[r];
    }
}
// columns [idx, idx+d) := columns * T^T
void cols_apply(Mat& M, int nrows, int stride, int idx, const double* T, int d) {
    double tmp[3];
    for (int r = 0; r < nrows; ++r) {
        double* row = &M[(size_t)r * stride + idx];
        for (int c = 0; c < d; ++c) {
            double s = 0;
            for (int k = 0; k < d; ++k) s += row[k] * T[c * d + k];
            tmp[c] = s;
        }
        for (int c = 0; c < d; ++c) row[c] = tmp[c];
    }
}

void unpack_hth(const double* sums, double HTH[36]) {
    int q = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b) {
            HTH[6 * a + b] = sums[q];
            HTH[6 * b + a] = sums[q];
            ++q;
        }
}

}  // namespace

void quat_to_mat(const Quat& q, double R[9]) {
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

int update_iterated(State& x, Mat& P, double R, int max_iter, double epsi, const HModelFn& hfn, IeskfResult& out) {
    using clk = std::chrono::steady_clock;
    const State x_prop = x;
    const Mat P_prop = P;
    Mat K_x((size_t)N * N, 0.0), Mm(36);
    double K_h[N], dx_new[N], dxu[N];
    bool converge = true;
    int t = 0;
    HModel hm;
    out = IeskfResult{};
    double solve_s = 0.0;
    for (int i = -1; i < max_iter; ++i) {
        const bool want_rows_hint = false;
        ++out.h_evals;
        if (converge) ++out.knn_calls;
        int rc = hfn(x, converge, want_rows_hint, hm);
        if (rc != 0) return rc;
        const int dof = (int)hm.sums[27];
        out.n_eff = dof;
        out.res_mean = dof > 0 ? hm.sums[28] / dof : 0.0;
        if (dof < 1) continue;  // ekfom_data.valid = false: "No Effective Points!"
        if (dof < N && hm.rows.size() != (size_t)7 * dof) {
            rc = hfn(x, false, true, hm);  // fetch the H rows of this same evaluation
            if (rc != 0) return rc;
        }
        const auto t0 = clk::now();
        double dx[N];
        boxminus(x, x_prop, dx);
        std::memcpy(dx_new, dx, sizeof(dx));
        P = P_prop;
        for (int idx : kSO3) {
            const M3 At = transpose(a_matrix(dx + idx));  // res_temp_SO3
            double v[3];
            for (int r = 0; r < 3; ++r) v[r] = At(r, 0) * dx_new[idx] + At(r, 1) * dx_new[idx + 1] + At(r, 2) * dx_new[idx + 2];
            std::memcpy(dx_new + idx, v, sizeof(v));
            rows_apply(P, P, N, idx, At.a, 3, N);
            cols_apply(P, N, N, idx, At.a, 3);
        }
        {
            double T2[4];
            s2_jac(x.grav, x_prop.grav, dx + kS2, T2);
            const double v0 = T2[0] * dx_new[kS2] + T2[1] * dx_new[kS2 + 1];
            const double v1 = T2[2] * dx_new[kS2] + T2[3] * dx_new[kS2 + 1];
            dx_new[kS2] = v0;
            dx_new[kS2 + 1] = v1;
            rows_apply(P, P, N, kS2, T2, 2, N);
            cols_apply(P, N, N, kS2, T2, 2);
        }
        std::fill(K_x.begin(), K_x.end(), 0.0);
        if (N > dof) {
            // K = P H^T (H P H^T / R + I)^-1 / R ; H = rows (dof x 6, zero elsewhere)
            const double* H = hm.rows.data();
            Mat PHt((size_t)N * dof);
            for (int r = 0; r < N; ++r)
                for (int m = 0; m < dof; ++m) {
                    double s = 0;
                    for (int c = 0; c < 6; ++c) s += P[(size_t)r * N + c] * H[7 * m + c];
                    PHt[(size_t)r * dof + m] = s;
                }
            Mat S((size_t)dof * dof);
            for (int a = 0; a < dof; ++a)
                for (int b = 0; b < dof; ++b) {
                    double s = 0;
                    for (int c = 0; c < 6; ++c) s += H[7 * a + c] * PHt[(size_t)c * dof + b];
                    S[(size_t)a * dof + b] = s / R + (a == b ? 1.0 : 0.0);
                }
            if (!lu_inverse(S, dof)) return -4;
            for (int r = 0; r < N; ++r) {
                double kh = 0;
                double kx[6] = {0, 0, 0, 0, 0, 0};
                for (int b = 0; b < dof; ++b) {
                    double s = 0;
                    for (int a = 0; a < dof; ++a) s += PHt[(size_t)r * dof + a] * S[(size_t)a * dof + b];
                    const double k = s / R;
                    kh += k * H[7 * b + 6];
                    for (int c = 0; c < 6; ++c) kx[c] += k * H[7 * b + c];
                }
                K_h[r] = kh;
                for (int c = 0; c < 6; ++c) K_x[(size_t)r * N + c] = kx[c];
            }
        } else {
            // Reference: P_temp = (P/R)^-1; P_temp[:6,:6] += HTH; P_inv = P_temp^-1;
            // K_h = P_inv[:, :6] HTh; K_x[:, :6] = P_inv[:, :6] HTH.  Only P_inv's
            // first 6 columns are used, and with A = P/R, E = [I6; 0]:
            //   (A^-1 + E HTH E^T)^-1 E = A E (I6 + HTH A11)^-1   (Woodbury + push-through)
            // so one 6x6 inverse replaces the two 23x23 inverses (equal in exact
            // arithmetic; the IESKF parity bar is a tolerance).
            double HTH[36];
            unpack_hth(hm.sums, HTH);
            // A = P / R on the first 6 columns, each element divided once (the same values the
            // products below used when they divided inline)
            double PR[N * 6];
            for (int r = 0; r < N; ++r)
                for (int m = 0; m < 6; ++m) PR[r * 6 + m] = P[(size_t)r * N + m] / R;
            Mm.assign(36, 0.0);
            for (int a = 0; a < 6; ++a)
                for (int b = 0; b < 6; ++b) {
                    double s = 0;
                    for (int m = 0; m < 6; ++m) s += HTH[6 * a + m] * PR[m * 6 + b];
                    Mm[(size_t)a * 6 + b] = s + (a == b ? 1.0 : 0.0);
                }
            if (!lu_inverse(Mm, 6)) return -4;
            for (int r = 0; r < N; ++r) {
                double q[6];
                for (int c = 0; c < 6; ++c) {
                    double s = 0;
                    for (int m = 0; m < 6; ++m) s += PR[r * 6 + m] * Mm[(size_t)m * 6 + c];
                    q[c] = s;
                }
                double kh = 0;
                for (int c = 0; c < 6; ++c) kh += q[c] * hm.sums[21 + c];
                K_h[r] = kh;
                for (int c = 0; c < 6; ++c) {
                    double s = 0;
                    for (int m = 0; m < 6; ++m) s += q[m] * HTH[6 * m + c];
                    K_x[(size_t)r * N + c] = s;
                }
            }
        }
        // (K_x - I) dx_new: K_x is zero outside its first 6 columns, so the rest of row r contributes
        // exact zeros and -dx_new[r] (same sum, the zero terms skipped)
        for (int r = 0; r < N; ++r) {
            double s = 0;
            for (int c = 0; c < 6; ++c) s += (K_x[(size_t)r * N + c] - (r == c ? 1.0 : 0.0)) * dx_new[c];
            if (r >= 6) s += -dx_new[r];
            dxu[r] = K_h[r] + s;
        }
        boxplus(x, dxu);
        converge = true;
        for (int r = 0; r < N; ++r)
            if (std::fabs(dxu[r]) > epsi) {
                converge = false;
                break;
            }
        if (converge) ++t;
        if (!t && i == max_iter - 2) converge = true;
        if (t > 1 || i == max_iter - 1) {
            Mat L = P;
            for (int idx : kSO3) {
                const M3 At = transpose(a_matrix(dxu + idx));
                rows_apply(L, P, N, idx, At.a, 3, N);
                rows_apply(K_x, K_x, N, idx, At.a, 3, 12);
                cols_apply(L, N, N, idx, At.a, 3);
                cols_apply(P, N, N, idx, At.a, 3);
            }
            {
                double T2[4];
                s2_jac(x.grav, x_prop.grav, dxu + kS2, T2);
                rows_apply(L, P, N, kS2, T2, 2, N);
                rows_apply(K_x, K_x, N, kS2, T2, 2, 12);
                cols_apply(L, N, N, kS2, T2, 2);
                cols_apply(P, N, N, kS2, T2, 2);
            }
            Mat Pn((size_t)N * N);
            // K_x columns 6..11 stay zero (the block transforms above mix rows only): their terms are
            // exact zeros, skipped
            for (int r = 0; r < N; ++r)
                for (int c = 0; c < N; ++c) {
                    double s = 0;
                    for (int m = 0; m < 6; ++m) s += K_x[(size_t)r * N + m] * P[(size_t)m * N + c];
                    Pn[(size_t)r * N + c] = L[(size_t)r * N + c] - s;
                }
            P.swap(Pn);
            out.converged = t > 1 ? 1 : 0;
            solve_s += std::chrono::duration<double>(clk::now() - t0).count();
            break;
        }
        solve_s += std::chrono::duration<double>(clk::now() - t0).count();
    }
    out.solve_ms = solve_s * 1e3;
    return 0;
}

}  // namespace host
}  // namespace lio
