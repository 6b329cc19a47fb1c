// =============================================================================
// lio_oracle.cpp — CPU restatement of the reference scan-matching hot path.
//
// THIS IS TEST INFRASTRUCTURE, NOT PRODUCT CODE.  Only tests/, the smoke check
// in __graft_entry__.py and bench.py's cpu_baseline leg may load it, and only
// as the checker / the timed CPU baseline.  The product (liblio_gpu.so) never
// links, loads or calls anything in this directory.
//
// PARITY STATUS: **parity unpinned** against the real reference binary.
//   * The FAST-LIO front end (ikd-Tree, esti_plane, h_share_model, IKFoM
//     esekfom) is an EMPTY git submodule in the reference
//     (/root/reference/.gitmodules:1-3, third_party/FAST_LIO/ is empty), so
//     its semantics are restated from the public upstream hku-mars sources
//     (tagged [U] below) and cannot be compiled or run here.
//   * The loop-closure ICP (/root/reference/fast_lio_sam/src/loop_closure.cpp
//     :69-92) needs PCL/Eigen/ROS/GTSAM, none of which exist in this image,
//     so PCL's IterativeClosestPoint is restated from PCL-1.10 semantics [U].
//   * The reference ships no tests, fixtures or golden vectors.
//   The restatement is cross-checked against independent implementations
//   (scipy cKDTree, numpy brute force, numpy SVD) in tests/test_oracle.py and
//   the committed fixtures in tests/golden/ are generated from it.
//
// Floating-point contract (compile with -ffp-contract=off, no -ffast-math):
//   * kNN squared distance: float ((dx*dx + dy*dy) + dz*dz)  [ikd-Tree calc_dist, U]
//   * ties in the kNN ordering are broken by the lower map point id (the
//     ikd-Tree breaks them by traversal order, which is not reproducible).
//   * world point: double s.rot * (s.offset_R_L_I * p + t_LI) + pos, the two SO3 products as
//     Eigen's QuaternionBase::_transformVector evaluates them (quat_rotate), stored as float [U]
// =============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <unordered_map>
#include <unordered_set>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// ---------------------------------------------------------------------------
// float helpers
// ---------------------------------------------------------------------------
static inline float sqdist(const float* a, const float* b) {
    float dx = a[0] - b[0];
    float dy = a[1] - b[1];
    float dz = a[2] - b[2];
    return (dx * dx + dy * dy) + dz * dz;
}
static inline bool lex_less(float da, int32_t ia, float db, int32_t ib) {
    return da < db || (da == db && ia < ib);
}

// ---------------------------------------------------------------------------
// Static kd-tree (oracle + CPU baseline).  Exact k-NN with an inclusive range
// bound; results ascending by (d2, id).   Follows the result semantics of
// ikd-Tree KD_TREE::Nearest_Search (k nearest, ascending sq-distances) [U]
// and pcl::KdTreeFLANN::nearestKSearch(k=1) [U, PCL 1.10].
// ---------------------------------------------------------------------------
struct KdTree {
    struct Node {
        float split;
        int dim;  // -1 => leaf
        int left, right, begin, end;
    };
    std::vector<float> xyz;     // original order, n*3
    std::vector<int32_t> perm;  // tree order -> original id
    std::vector<float> pxyz;    // tree-order copy
    std::vector<Node> nodes;
    static const int LEAF = 12;

    // Median split on the widest axis, ties by id.  The top levels build their two subtrees as
    // OpenMP tasks into separate node vectors that are then appended (indices shifted): the node
    // numbering differs from a serial build, the tree (and every search result) does not.
    int build_rec(std::vector<Node>& out, int b, int e, int depth) {
        Node nd;
        nd.begin = b;
        nd.end = e;
        nd.left = nd.right = -1;
        nd.split = 0.f;
        nd.dim = -1;
        if (e - b > LEAF) {
            float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            for (int i = b; i < e; ++i)
                for (int d = 0; d < 3; ++d) {
                    float v = xyz[3 * (size_t)perm[i] + d];
                    lo[d] = std::min(lo[d], v);
                    hi[d] = std::max(hi[d], v);
                }
            int dim = 0;
            float ext = hi[0] - lo[0];
            for (int d = 1; d < 3; ++d)
                if (hi[d] - lo[d] > ext) { ext = hi[d] - lo[d]; dim = d; }
            if (ext > 0.f) {
                int m = (b + e) / 2;
                const float* X = xyz.data();
                std::nth_element(perm.begin() + b, perm.begin() + m, perm.begin() + e,
                                 [X, dim](int32_t a, int32_t c) {
                                     float va = X[3 * (size_t)a + dim], vc = X[3 * (size_t)c + dim];
                                     return va < vc || (va == vc && a < c);
                                 });
                nd.dim = dim;
                nd.split = xyz[3 * (size_t)perm[m] + dim];
                const int self = (int)out.size();
                out.push_back(nd);
                if (depth < 4 && e - b > (1 << 16)) {
                    std::vector<Node> L, R;
#pragma omp task shared(L)
                    build_rec(L, b, m, depth + 1);
#pragma omp task shared(R)
                    build_rec(R, m, e, depth + 1);
#pragma omp taskwait
                    out[self].left = append(out, L);
                    out[self].right = append(out, R);
                } else {
                    const int l = build_rec(out, b, m, depth + 1);
                    const int r = build_rec(out, m, e, depth + 1);
                    out[self].left = l;
                    out[self].right = r;
                }
                return self;
            }
        }
        out.push_back(nd);
        return (int)out.size() - 1;
    }
    static int append(std::vector<Node>& out, const std::vector<Node>& sub) {
        const int off = (int)out.size();
        for (Node nd : sub) {
            if (nd.left >= 0) nd.left += off;
            if (nd.right >= 0) nd.right += off;
            out.push_back(nd);
        }
        return off;  // the subtree's root is its first node
    }

    void build(const float* p, int64_t n) {
        std::vector<int32_t> ids(n);
        std::iota(ids.begin(), ids.end(), 0);
        build_ids(p, n, ids);
    }
    // tree over the subset `ids` of the n_all points p (ids are reported)
    void build_ids(const float* p, int64_t n_all, const std::vector<int32_t>& ids) {
        xyz.assign(p, p + 3 * n_all);
        perm = ids;
        const int64_t n = (int64_t)perm.size();
        nodes.clear();
        nodes.reserve(2 * (n / LEAF + 1) + 8);
        if (n > 0) {
#pragma omp parallel num_threads(8)
#pragma omp single
            build_rec(nodes, 0, (int)n, 0);
        }
        pxyz.resize(3 * n);
        for (int64_t i = 0; i < n; ++i)
            for (int d = 0; d < 3; ++d) pxyz[3 * i + d] = xyz[3 * (size_t)perm[i] + d];
    }

    struct TopK {
        int k, cnt;
        float range;
        float d[8];
        int32_t id[8];
        float worst() const { return cnt < k ? range : d[k - 1]; }
        void consider(float d2, int32_t i) {
            if (d2 > range) return;
            if (cnt == k && !lex_less(d2, i, d[k - 1], id[k - 1])) return;
            int pos = cnt < k ? cnt++ : k - 1;
            while (pos > 0 && lex_less(d2, i, d[pos - 1], id[pos - 1])) {
                d[pos] = d[pos - 1];
                id[pos] = id[pos - 1];
                --pos;
            }
            d[pos] = d2;
            id[pos] = i;
        }
    };

    void search(int ni, const float* q, TopK& tk) const {
        const Node& nd = nodes[ni];
        if (nd.dim < 0) {
            for (int i = nd.begin; i < nd.end; ++i) tk.consider(sqdist(q, &pxyz[3 * (size_t)i]), perm[i]);
            return;
        }
        double diff = (double)q[nd.dim] - (double)nd.split;
        int nearc = diff < 0 ? nd.left : nd.right;
        int farc = diff < 0 ? nd.right : nd.left;
        search(nearc, q, tk);
        // conservative prune: the far side's exact distance lower bound is |diff|;
        // a float-rounded d2 can undercut the exact value by < 1e-6 relative.
        if (diff * diff <= (double)tk.worst() * (1.0 + 1e-6)) search(farc, q, tk);
    }

    int knn(const float* q, int k, float range_sq, int32_t* id_out, float* d_out) const {
        TopK tk;
        tk.k = k;
        tk.cnt = 0;
        tk.range = range_sq;
        if (!nodes.empty()) search(0, q, tk);
        for (int j = 0; j < k; ++j) {
            id_out[j] = j < tk.cnt ? tk.id[j] : -1;
            d_out[j] = j < tk.cnt ? tk.d[j] : INFINITY;
        }
        return tk.cnt;
    }
};

// ---------------------------------------------------------------------------
// esti_plane<float>(pca_result, points_near, threshold)   [U: FAST-LIO
// include/common_lib.h].  Least squares A(5x3) n = -1 through Eigen's
// ColPivHouseholderQR (restated from Eigen 3.3 computeInPlace/_solve_impl:
// stable norm downdate, first-max pivot, makeHouseholder, column-oriented
// upper-triangular back substitution), then n/|n|, d = 1.0/|n| (double
// division stored as float) and the |a x + b y + c z + d| > thr flatness gate.
// ---------------------------------------------------------------------------
bool esti_plane(float out[4], const float P[5][3], float thr) {
    const int rows = 5;
    float A[3][5];  // column-major: A[col][row]
    for (int j = 0; j < 5; ++j) {
        A[0][j] = P[j][0];
        A[1][j] = P[j][1];
        A[2][j] = P[j][2];
    }
    float cnU[3], cnD[3];
    for (int k = 0; k < 3; ++k) {
        float s = 0.f;
        for (int i = 0; i < 5; ++i) s += A[k][i] * A[k][i];
        cnD[k] = std::sqrt(s);
        cnU[k] = cnD[k];
    }
    float mx = cnU[0];
    for (int k = 1; k < 3; ++k)
        if (cnU[k] > mx) mx = cnU[k];
    const float eps = FLT_EPSILON;
    const float th_help = ((mx * eps) * (mx * eps)) / (float)rows;
    const float ndt = std::sqrt(eps);
    int nzp = 3;
    int tr[3];
    float hc[3];
    for (int k = 0; k < 3; ++k) {
        int bi = k;
        float bn = cnU[k];
        for (int j = k + 1; j < 3; ++j)
            if (cnU[j] > bn) { bn = cnU[j]; bi = j; }
        float bsq = bn * bn;
        if (nzp == 3 && bsq < th_help * (float)(rows - k)) nzp = k;
        tr[k] = bi;
        if (bi != k) {
            for (int i = 0; i < 5; ++i) std::swap(A[k][i], A[bi][i]);
            std::swap(cnU[k], cnU[bi]);
            std::swap(cnD[k], cnD[bi]);
        }
        // makeHouseholderInPlace on A[k][k..4]
        float c0 = A[k][k];
        float tsq = 0.f;
        for (int i = k + 1; i < 5; ++i) tsq += A[k][i] * A[k][i];
        float beta, tau;
        if (tsq <= FLT_MIN) {
            tau = 0.f;
            beta = c0;
            for (int i = k + 1; i < 5; ++i) A[k][i] = 0.f;
        } else {
            beta = std::sqrt(c0 * c0 + tsq);
            if (c0 >= 0.f) beta = -beta;
            float den = c0 - beta;
            for (int i = k + 1; i < 5; ++i) A[k][i] = A[k][i] / den;
            tau = (beta - c0) / beta;
        }
        A[k][k] = beta;
        hc[k] = tau;
        // applyHouseholderOnTheLeft on the bottom-right corner
        if (tau != 0.f) {
            for (int j = k + 1; j < 3; ++j) {
                float tmp = 0.f;
                for (int i = k + 1; i < 5; ++i) tmp += A[k][i] * A[j][i];
                tmp += A[j][k];
                A[j][k] -= tau * tmp;
                for (int i = k + 1; i < 5; ++i) A[j][i] -= (tau * A[k][i]) * tmp;
            }
        }
        // column norm downdate (LAPACK xGEQPF)
        for (int j = k + 1; j < 3; ++j) {
            if (cnU[j] != 0.f) {
                float temp = std::fabs(A[j][k]) / cnU[j];
                temp = (1.f + temp) * (1.f - temp);
                temp = temp < 0.f ? 0.f : temp;
                float r = cnU[j] / cnD[j];
                float temp2 = temp * (r * r);
                if (temp2 <= ndt) {
                    float s = 0.f;
                    for (int i = k + 1; i < 5; ++i) s += A[j][i] * A[j][i];
                    cnD[j] = std::sqrt(s);
                    cnU[j] = cnD[j];
                } else {
                    cnU[j] *= std::sqrt(temp);
                }
            }
        }
    }
    float x[3] = {0.f, 0.f, 0.f};
    if (nzp > 0) {
        float c[5] = {-1.f, -1.f, -1.f, -1.f, -1.f};
        for (int k = 0; k < nzp; ++k) {
            if (hc[k] != 0.f) {
                float tmp = 0.f;
                for (int i = k + 1; i < 5; ++i) tmp += A[k][i] * c[i];
                tmp += c[k];
                c[k] -= hc[k] * tmp;
                for (int i = k + 1; i < 5; ++i) c[i] -= (hc[k] * A[k][i]) * tmp;
            }
        }
        for (int i = nzp - 1; i >= 0; --i) {
            if (c[i] != 0.f) {
                c[i] /= A[i][i];
                for (int j = 0; j < i; ++j) c[j] -= c[i] * A[i][j];
            }
        }
        int perm[3] = {0, 1, 2};
        for (int k = 0; k < 3; ++k) std::swap(perm[k], perm[tr[k]]);
        for (int i = 0; i < 3; ++i) x[perm[i]] = i < nzp ? c[i] : 0.f;
    }
    float n = std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
    out[0] = x[0] / n;
    out[1] = x[1] / n;
    out[2] = x[2] / n;
    out[3] = (float)(1.0 / (double)n);
    for (int j = 0; j < 5; ++j) {
        float r = ((out[0] * P[j][0] + out[1] * P[j][1]) + out[2] * P[j][2]) + out[3];
        if (std::fabs(r) > thr) return false;
    }
    return true;
}

// ---------------------------------------------------------------------------
// Match parameters and pose (mirrors lio_match_params / lio_pose in the C-ABI)
// ---------------------------------------------------------------------------
struct MatchParams {
    float knn_range_sq;  // 5.0  : kNN gate `sqdist[4] > 5` rejects [U]; also the search bound
    float plane_thr;     // 0.1f : esti_plane threshold [U]
    double s_coef;       // 0.9  : s = 1 - s_coef*|pd2|/sqrt(|p_body|) [U]
    double s_gate;       // 0.9  : keep if s > s_gate [U]
};
// The parts of state_ikfom the measurement model reads.  rot / offset_R_L_I are MTK::SO3<double>,
// i.e. Eigen::Quaternion<double> [U: IKFoM use-ikfom.hpp, MTK SO3.hpp]: q, qLI = (w, x, y, z) of the
// state; every `SO3 * v` below is evaluated as Eigen does it (quat_rotate).  R / RLI are the row-major
// matrices of the same rotations (kept in the C-ABI for callers that hold matrices; when q is all zero
// it is derived from R by Eigen's Matrix3 -> Quaternion conversion, pose_fill_quat).
struct Pose {
    double R[9], t[3], RLI[9], tLI[3];
    double q[4], qLI[4];
};

// Eigen 3.3 QuaternionBase<Derived>::_transformVector (Geometry/Quaternion.h) — how
// `Eigen::Quaternion<double> * Vector3d` (RotationBase::operator* -> _transformVector) is computed:
//   Vector3 uv = this->vec().cross(v); uv += uv; return v + this->w() * uv + this->vec().cross(uv);
// with MatrixBase::cross = (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0) (Geometry/OrthoMethods.h).
// conj: rotate by q.conjugate() (vec negated, w kept), as `s.rot.conjugate() * n`.
static inline void quat_rotate(const double* q, bool conj, const double v[3], double o[3]) {
    const double w = q[0];
    const double x = conj ? -q[1] : q[1], y = conj ? -q[2] : q[2], z = conj ? -q[3] : q[3];
    double u0 = y * v[2] - z * v[1];
    double u1 = z * v[0] - x * v[2];
    double u2 = x * v[1] - y * v[0];
    u0 += u0;
    u1 += u1;
    u2 += u2;
    const double c0 = y * u2 - z * u1;
    const double c1 = z * u0 - x * u2;
    const double c2 = x * u1 - y * u0;
    o[0] = (v[0] + w * u0) + c0;
    o[1] = (v[1] + w * u1) + c1;
    o[2] = (v[2] + w * u2) + c2;
}

// Eigen 3.3 quaternionbase_assign_impl<Other,3,3>::run (Geometry/Quaternion.h): rotation matrix ->
// quaternion; trace() = m00 + (m11 + m22) (the unrolled redux splits the 3 terms 1 + 2).  Only
// for callers that pass matrices without the state quaternion.
static void mat_to_quat(const double* m, double* q) {
    auto M = [&](int r, int c) { return m[3 * r + c]; };
    double t = M(0, 0) + (M(1, 1) + M(2, 2));
    double c[4];  // x, y, z, w (Eigen coeffs order)
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        c[3] = 0.5 * t;
        t = 0.5 / t;
        c[0] = (M(2, 1) - M(1, 2)) * t;
        c[1] = (M(0, 2) - M(2, 0)) * t;
        c[2] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        c[3] = (M(k, j) - M(j, k)) * t;
        c[j] = (M(j, i) + M(i, j)) * t;
        c[k] = (M(k, i) + M(i, k)) * t;
    }
    q[0] = c[3];
    q[1] = c[0];
    q[2] = c[1];
    q[3] = c[2];
}

static void pose_fill_quat(Pose& ps) {
    if (ps.q[0] == 0.0 && ps.q[1] == 0.0 && ps.q[2] == 0.0 && ps.q[3] == 0.0) mat_to_quat(ps.R, ps.q);
    if (ps.qLI[0] == 0.0 && ps.qLI[1] == 0.0 && ps.qLI[2] == 0.0 && ps.qLI[3] == 0.0) mat_to_quat(ps.RLI, ps.qLI);
}

// pointBodyToWorld / h_share_model [U]:
//   V3D p_global(s.rot * (s.offset_R_L_I * p_body + s.offset_T_L_I) + s.pos);  stored as float
static inline void body_to_world(const Pose& ps, const float* pb, float* pw) {
    const double b[3] = {pb[0], pb[1], pb[2]};
    double a[3], pi[3], w[3];
    quat_rotate(ps.qLI, false, b, a);
    for (int r = 0; r < 3; ++r) pi[r] = a[r] + ps.tLI[r];
    quat_rotate(ps.q, false, pi, w);
    for (int r = 0; r < 3; ++r) w[r] = w[r] + ps.t[r];
    pw[0] = (float)w[0];
    pw[1] = (float)w[1];
    pw[2] = (float)w[2];
}

// H row (extrinsic_est_en = false): [n, (R_LI p + t_LI) x (R^T n), 0 ...] [U]
//   point_this = s.offset_R_L_I * point_this_be + s.offset_T_L_I;  C = s.rot.conjugate() * norm_vec;
//   A = point_crossmat * C  (SKEW_SYM_MATRX rows: 0*C0 + (-p2)*C1 + p1*C2 = p1*C2 - p2*C1 exactly, ...)
static inline void h_row(const Pose& ps, const float* pb, const float* nrm, double J[6]) {
    const double b[3] = {pb[0], pb[1], pb[2]};
    double a[3], pi[3];
    quat_rotate(ps.qLI, false, b, a);
    for (int r = 0; r < 3; ++r) pi[r] = a[r] + ps.tLI[r];
    const double n[3] = {nrm[0], nrm[1], nrm[2]};
    double C[3];
    quat_rotate(ps.q, true, n, C);
    J[0] = n[0];
    J[1] = n[1];
    J[2] = n[2];
    J[3] = pi[1] * C[2] - pi[2] * C[1];
    J[4] = pi[2] * C[0] - pi[0] * C[2];
    J[5] = pi[0] * C[1] - pi[1] * C[0];
}

// Output layout of one h-evaluation (shared with the GPU C-ABI, see
// include/lio_gpu.h LIO_SUMS_*): HTH upper triangle (21, row-major i<=j),
// HTh (6), n_eff, total_residual, sum h^2.
enum { S_HTH = 0, S_HTh = 21, S_NEFF = 27, S_RES = 28, S_HH = 29, S_LEN = 32 };

struct HModelWork {
    std::vector<float> world;
    std::vector<float> res_last;
};

// h_share_model(state, ekfom_data)  [U: FAST-LIO src/laserMapping.cpp]
// nn_idx: n*5 (in/out), sel: n (in/out), planes: n*4 (out: a,b,c,pd2 of selected)
int h_share_model(const KdTree& map, const float* body, int64_t n, const Pose& ps, int redo_knn,
                  int32_t* nn_idx, uint8_t* sel, float* planes, const MatchParams& mp, double* sums,
                  int threads, std::vector<double>* rows_out) {
    std::vector<float> res_last(n, 0.f);
#pragma omp parallel for schedule(dynamic, 512) num_threads(threads)
    for (int64_t i = 0; i < n; ++i) {
        float pw[3];
        body_to_world(ps, body + 3 * i, pw);
        int32_t* idx = nn_idx + 5 * i;
        if (redo_knn) {
            float d2[5];
            int cnt = map.knn(pw, 5, mp.knn_range_sq, idx, d2);
            sel[i] = (cnt < 5) ? 0 : (d2[4] > mp.knn_range_sq ? 0 : 1);
        }
        if (!sel[i]) continue;
        float nb[5][3];
        for (int j = 0; j < 5; ++j)
            for (int d = 0; d < 3; ++d) nb[j][d] = map.xyz[3 * (size_t)idx[j] + d];
        float pabcd[4];
        sel[i] = 0;
        if (esti_plane(pabcd, nb, mp.plane_thr)) {
            float pd2 = ((pabcd[0] * pw[0] + pabcd[1] * pw[1]) + pabcd[2] * pw[2]) + pabcd[3];
            double bx = body[3 * i], by = body[3 * i + 1], bz = body[3 * i + 2];
            double pnorm = std::sqrt((bx * bx + by * by) + bz * bz);
            float s = (float)(1.0 - mp.s_coef * (double)std::fabs(pd2) / std::sqrt(pnorm));
            if ((double)s > mp.s_gate) {
                sel[i] = 1;
                planes[4 * i + 0] = pabcd[0];
                planes[4 * i + 1] = pabcd[1];
                planes[4 * i + 2] = pabcd[2];
                planes[4 * i + 3] = pd2;
                res_last[i] = std::fabs(pd2);
            }
        }
    }
    // serial compaction + H^T H / H^T h in point order
    for (int j = 0; j < S_LEN; ++j) sums[j] = 0.0;
    int64_t neff = 0;
    double total_residual = 0.0;
    if (rows_out) rows_out->clear();
    for (int64_t i = 0; i < n; ++i) {
        if (!sel[i]) continue;
        ++neff;
        total_residual += res_last[i];
        double J[6];
        h_row(ps, body + 3 * i, planes + 4 * i, J);
        double h = -(double)planes[4 * i + 3];
        int q = 0;
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 6; ++b) sums[S_HTH + q++] += J[a] * J[b];
        for (int a = 0; a < 6; ++a) sums[S_HTh + a] += J[a] * h;
        sums[S_HH] += h * h;
        if (rows_out) {
            for (int a = 0; a < 6; ++a) rows_out->push_back(J[a]);
            rows_out->push_back(h);
        }
    }
    sums[S_NEFF] = (double)neff;
    sums[S_RES] = total_residual;
    return 0;
}

// ---------------------------------------------------------------------------
// IKFoM manifold + iterated ESKF update [U: IKFoM esekfom.hpp
// update_iterated_dyn_share_modified, MTK SO3/S2, FAST-LIO use-ikfom.hpp].
// State order: pos(0) rot(3) offset_R_L_I(6) offset_T_L_I(9) vel(12) bg(15)
// ba(18) grav S2(21)  => n = 23.
// ---------------------------------------------------------------------------
static const int NX = 23;
static const double MTK_TOL = 1e-11;
static const double GRAV_LEN = 98090.0 / 10000.0;  // S2<double, 98090, 10000, 1>

struct Quat { double w, x, y, z; };
struct State {
    double pos[3];
    Quat rot;
    Quat offR;
    double offT[3];
    double vel[3], bg[3], ba[3];
    double grav[3];
};

static Quat qmul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
static Quat qconj(const Quat& a) { return {a.w, -a.x, -a.y, -a.z}; }
static void qtomat(const Quat& q, double R[9]) {
    double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
// MTK::exp(result, vec, scale) -> quaternion for rotation vector with half-angle scale
static Quat so3_exp(const double v[3], double scale_half) {
    double n2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    double nrm = std::sqrt(n2);
    double alpha = scale_half * nrm;
    Quat q;
    if (nrm < MTK_TOL) {
        q.w = 1.0;
        q.x = scale_half * v[0];
        q.y = scale_half * v[1];
        q.z = scale_half * v[2];
        return q;
    }
    double s = std::sin(alpha) / nrm;
    q.w = std::cos(alpha);
    q.x = s * v[0];
    q.y = s * v[1];
    q.z = s * v[2];
    return q;
}
// SO3::log (MTK::log with scale 2, plus_minus_periodicity = true)
static void so3_log(const Quat& q, double out[3]) {
    double nv = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
    if (nv < MTK_TOL) nv = MTK_TOL;
    double s = 2.0 / nv * std::atan(nv / q.w);
    out[0] = s * q.x;
    out[1] = s * q.y;
    out[2] = s * q.z;
}
static void hat(const double v[3], double M[9]) {
    M[0] = 0;     M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0;     M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0;
}
static void mm3(const double* A, const double* B, double* C, int m, int k, int n) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0;
            for (int t = 0; t < k; ++t) s += A[i * k + t] * B[t * n + j];
            C[i * n + j] = s;
        }
}
// MTK::A_matrix(v)
static void A_matrix(const double v[3], double A[9]) {
    double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    double nrm = std::sqrt(sq);
    for (int i = 0; i < 9; ++i) A[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (nrm < MTK_TOL) return;
    double H[9], H2[9];
    hat(v, H);
    mm3(H, H, H2, 3, 3, 3);
    double c1 = (1 - std::cos(nrm)) / sq;
    double c2 = (1 - std::sin(nrm) / nrm) / sq;
    for (int i = 0; i < 9; ++i) A[i] += c1 * H[i] + c2 * H2[i];
}
// S2 (typ 1) basis B(x)
static void s2_Bx(const double v[3], double B[6]) {
    const double L = GRAV_LEN;
    if (v[0] + L > MTK_TOL) {
        double d = L + v[0];
        B[0] = -v[1];              B[1] = -v[2];
        B[2] = L - v[1] * v[1] / d; B[3] = -v[2] * v[1] / d;
        B[4] = -v[2] * v[1] / d;    B[5] = L - v[2] * v[2] / d;
        for (int i = 0; i < 6; ++i) B[i] /= L;
    } else {
        for (int i = 0; i < 6; ++i) B[i] = 0;
        B[3] = -1;
        B[4] = 1;
    }
}
static void s2_Nx_yy(const double v[3], double N[6]) {  // 2x3 = 1/L^2 Bx^T hat(v)
    double B[6], H[9];
    s2_Bx(v, B);
    hat(v, H);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int t = 0; t < 3; ++t) s += B[t * 2 + i] * H[t * 3 + j];
            N[i * 3 + j] = s / GRAV_LEN / GRAV_LEN;
        }
}
static void s2_Mx(const double v[3], const double dl[2], double M[6]) {  // 3x2
    double B[6], H[9];
    s2_Bx(v, B);
    hat(v, H);
    double dn = std::sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
    if (dn < MTK_TOL) {
        double HB[6];
        mm3(H, B, HB, 3, 3, 2);
        for (int i = 0; i < 6; ++i) M[i] = -HB[i];
        return;
    }
    double Bu[3];
    for (int r = 0; r < 3; ++r) Bu[r] = B[2 * r] * dl[0] + B[2 * r + 1] * dl[1];
    // MTK uses scalar(1/2) here, which is integer 0 => identity rotation [U quirk]
    Quat e = so3_exp(Bu, 0.0);
    double Re[9], A[9], At[9], T1[9], T2[9], T3[6];
    qtomat(e, Re);
    A_matrix(Bu, A);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) At[i * 3 + j] = A[j * 3 + i];
    mm3(Re, H, T1, 3, 3, 3);
    mm3(T1, At, T2, 3, 3, 3);
    mm3(T2, B, T3, 3, 3, 2);
    for (int i = 0; i < 6; ++i) M[i] = -T3[i];
}
static void s2_boxplus(double v[3], const double dl[2]) {
    double B[6];
    s2_Bx(v, B);
    double Bu[3];
    for (int r = 0; r < 3; ++r) Bu[r] = B[2 * r] * dl[0] + B[2 * r + 1] * dl[1];
    Quat e = so3_exp(Bu, 0.5);
    double Re[9];
    qtomat(e, Re);
    double o[3];
    for (int r = 0; r < 3; ++r) o[r] = Re[3 * r] * v[0] + Re[3 * r + 1] * v[1] + Re[3 * r + 2] * v[2];
    v[0] = o[0];
    v[1] = o[1];
    v[2] = o[2];
}
static void s2_boxminus(const double v[3], const double o[3], double res[2]) {
    double H[9];
    hat(v, H);
    double c[3];
    for (int r = 0; r < 3; ++r) c[r] = H[3 * r] * o[0] + H[3 * r + 1] * o[1] + H[3 * r + 2] * o[2];
    double vs = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    double vc = v[0] * o[0] + v[1] * o[1] + v[2] * o[2];
    double th = std::atan2(vs, vc);
    if (vs < MTK_TOL) {
        res[0] = std::fabs(th) > MTK_TOL ? 3.1415926 : 0.0;
        res[1] = 0.0;
        return;
    }
    double B[6], Ho[9];
    s2_Bx(o, B);
    hat(o, Ho);
    double hv[3];
    for (int r = 0; r < 3; ++r) hv[r] = Ho[3 * r] * v[0] + Ho[3 * r + 1] * v[1] + Ho[3 * r + 2] * v[2];
    for (int i = 0; i < 2; ++i) res[i] = th / vs * (B[i] * hv[0] + B[2 + i] * hv[1] + B[4 + i] * hv[2]);
}

static void state_boxminus(const State& x, const State& y, double dx[NX]) {
    for (int i = 0; i < 3; ++i) dx[i] = x.pos[i] - y.pos[i];
    so3_log(qmul(qconj(y.rot), x.rot), dx + 3);
    so3_log(qmul(qconj(y.offR), x.offR), dx + 6);
    for (int i = 0; i < 3; ++i) dx[9 + i] = x.offT[i] - y.offT[i];
    for (int i = 0; i < 3; ++i) dx[12 + i] = x.vel[i] - y.vel[i];
    for (int i = 0; i < 3; ++i) dx[15 + i] = x.bg[i] - y.bg[i];
    for (int i = 0; i < 3; ++i) dx[18 + i] = x.ba[i] - y.ba[i];
    s2_boxminus(x.grav, y.grav, dx + 21);
}
static void state_boxplus(State& x, const double dx[NX]) {
    for (int i = 0; i < 3; ++i) x.pos[i] += dx[i];
    x.rot = qmul(x.rot, so3_exp(dx + 3, 0.5));
    x.offR = qmul(x.offR, so3_exp(dx + 6, 0.5));
    for (int i = 0; i < 3; ++i) x.offT[i] += dx[9 + i];
    for (int i = 0; i < 3; ++i) x.vel[i] += dx[12 + i];
    for (int i = 0; i < 3; ++i) x.bg[i] += dx[15 + i];
    for (int i = 0; i < 3; ++i) x.ba[i] += dx[18 + i];
    s2_boxplus(x.grav, dx + 21);
}

// dense helpers (row-major n x n)
static bool invert(const std::vector<double>& A, std::vector<double>& Ainv, int n) {
    // PartialPivLU-style Gauss-Jordan with partial pivoting
    std::vector<double> M(A);
    Ainv.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) Ainv[(size_t)i * n + i] = 1.0;
    for (int c = 0; c < n; ++c) {
        int p = c;
        double best = std::fabs(M[(size_t)c * n + c]);
        for (int r = c + 1; r < n; ++r)
            if (std::fabs(M[(size_t)r * n + c]) > best) { best = std::fabs(M[(size_t)r * n + c]); p = r; }
        if (best == 0.0) return false;
        if (p != c)
            for (int j = 0; j < n; ++j) {
                std::swap(M[(size_t)p * n + j], M[(size_t)c * n + j]);
                std::swap(Ainv[(size_t)p * n + j], Ainv[(size_t)c * n + j]);
            }
        double inv = 1.0 / M[(size_t)c * n + c];
        for (int j = 0; j < n; ++j) {
            M[(size_t)c * n + j] *= inv;
            Ainv[(size_t)c * n + j] *= inv;
        }
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            double f = M[(size_t)r * n + c];
            if (f == 0.0) continue;
            for (int j = 0; j < n; ++j) {
                M[(size_t)r * n + j] -= f * M[(size_t)c * n + j];
                Ainv[(size_t)r * n + j] -= f * Ainv[(size_t)c * n + j];
            }
        }
    }
    return true;
}

struct IeskfStats {
    int iterations;   // h-evaluations performed
    int knn_calls;    // h-evaluations that redid the kNN
    int converged;    // t > 1 exit (1) vs max-iteration exit (0)
    int last_neff;
    double last_res_sum;
};

static void pose_from_state(const State& x, Pose& ps) {
    qtomat(x.rot, ps.R);
    qtomat(x.offR, ps.RLI);
    ps.q[0] = x.rot.w, ps.q[1] = x.rot.x, ps.q[2] = x.rot.y, ps.q[3] = x.rot.z;
    ps.qLI[0] = x.offR.w, ps.qLI[1] = x.offR.x, ps.qLI[2] = x.offR.y, ps.qLI[3] = x.offR.z;
    for (int i = 0; i < 3; ++i) {
        ps.t[i] = x.pos[i];
        ps.tLI[i] = x.offT[i];
    }
}

// Apply a 3x3 (or 2x2) block transform to rows idx..idx+d-1 (M := T * M) of an
// n x ncols matrix.
static void rows_xform(std::vector<double>& M, int ncols, int idx, const double* T, int d,
                       const std::vector<double>* src = nullptr, int col_lim = -1) {
    const std::vector<double>& S = src ? *src : M;
    int cl = col_lim < 0 ? ncols : col_lim;
    std::vector<double> tmp((size_t)d * cl);
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < cl; ++c) {
            double s = 0;
            for (int t = 0; t < d; ++t) s += T[r * d + t] * S[(size_t)(idx + t) * ncols + c];
            tmp[(size_t)r * cl + c] = s;
        }
    for (int r = 0; r < d; ++r)
        for (int c = 0; c < cl; ++c) M[(size_t)(idx + r) * ncols + c] = tmp[(size_t)r * cl + c];
}
// M := M * T^T on columns idx..idx+d-1 of an nrows x n matrix
static void cols_xform(std::vector<double>& M, int nrows, int ncols, int idx, const double* T, int d) {
    for (int r = 0; r < nrows; ++r) {
        double tmp[3];
        for (int c = 0; c < d; ++c) {
            double s = 0;
            for (int t = 0; t < d; ++t) s += M[(size_t)r * ncols + idx + t] * T[c * d + t];
            tmp[c] = s;
        }
        for (int c = 0; c < d; ++c) M[(size_t)r * ncols + idx + c] = tmp[c];
    }
}

int ieskf_update(const KdTree& map, const float* body, int64_t n, State& x, std::vector<double>& P,
                 const MatchParams& mp, double R, int max_iter, double limit, int threads,
                 IeskfStats* st, double* trace /* optional: per h-eval 8 doubles */, State* knn_state = nullptr) {
    std::vector<int32_t> nn_idx(5 * n, -1);
    std::vector<uint8_t> sel(n, 0);
    std::vector<float> planes(4 * n, 0.f);
    State x_prop = x;
    std::vector<double> P_prop = P;
    std::vector<double> K_x((size_t)NX * NX, 0.0);
    double K_h[NX];
    double dx_new[NX];
    bool converge = true;
    int t = 0;
    int evals = 0, knns = 0;
    st->converged = 0;
    std::vector<double> rows;
    for (int i = -1; i < max_iter; ++i) {
        Pose ps;
        pose_from_state(x, ps);
        double sums[S_LEN];
        ++evals;
        if (converge) ++knns;
        if (converge && knn_state) *knn_state = x;  // the state Nearest_Points belong to (map_incremental)
        h_share_model(map, body, n, ps, converge ? 1 : 0, nn_idx.data(), sel.data(), planes.data(), mp,
                      sums, threads, &rows);
        int dof = (int)sums[S_NEFF];
        st->last_neff = dof;
        st->last_res_sum = sums[S_RES];
        if (trace) {
            double* tr = trace + 8 * (evals - 1);
            tr[0] = i; tr[1] = converge ? 1 : 0; tr[2] = dof; tr[3] = sums[S_RES];
            tr[4] = x.pos[0]; tr[5] = x.pos[1]; tr[6] = x.pos[2]; tr[7] = 0;
        }
        if (dof < 1) continue;  // ekfom_data.valid = false ("No Effective Points")

        double dx[NX];
        state_boxminus(x, x_prop, dx);
        std::memcpy(dx_new, dx, sizeof(dx));
        P = P_prop;
        for (int idx : {3, 6}) {
            double A[9], At[9];
            A_matrix(dx + idx, A);
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) At[a * 3 + b] = A[b * 3 + a];  // res_temp_SO3 = A^T
            double v[3];
            for (int r = 0; r < 3; ++r) v[r] = At[3 * r] * dx_new[idx] + At[3 * r + 1] * dx_new[idx + 1] + At[3 * r + 2] * dx_new[idx + 2];
            for (int r = 0; r < 3; ++r) dx_new[idx + r] = v[r];
            rows_xform(P, NX, idx, At, 3);
            cols_xform(P, NX, NX, idx, At, 3);
        }
        {
            double Nx[6], Mx[6], T2[4];
            s2_Nx_yy(x.grav, Nx);
            s2_Mx(x_prop.grav, dx + 21, Mx);
            mm3(Nx, Mx, T2, 2, 3, 2);
            double v0 = T2[0] * dx_new[21] + T2[1] * dx_new[22];
            double v1 = T2[2] * dx_new[21] + T2[3] * dx_new[22];
            dx_new[21] = v0;
            dx_new[22] = v1;
            rows_xform(P, NX, 21, T2, 2);
            cols_xform(P, NX, NX, 21, T2, 2);
        }
        std::fill(K_x.begin(), K_x.end(), 0.0);
        if (NX > dof) {
            // K = P H^T (H P H^T / R + I)^-1 / R with H = dof x 23 (zero beyond col 6)
            std::vector<double> PHt((size_t)NX * dof, 0.0);
            for (int r = 0; r < NX; ++r)
                for (int m = 0; m < dof; ++m) {
                    double s = 0;
                    for (int c = 0; c < 6; ++c) s += P[(size_t)r * NX + c] * rows[7 * m + c];
                    PHt[(size_t)r * dof + m] = s;
                }
            std::vector<double> S((size_t)dof * dof), Sinv;
            for (int a = 0; a < dof; ++a)
                for (int b = 0; b < dof; ++b) {
                    double s = 0;
                    for (int c = 0; c < 6; ++c) s += rows[7 * a + c] * PHt[(size_t)c * dof + b];
                    S[(size_t)a * dof + b] = s / R + (a == b ? 1.0 : 0.0);
                }
            invert(S, Sinv, dof);
            std::vector<double> K((size_t)NX * dof, 0.0);
            for (int r = 0; r < NX; ++r)
                for (int b = 0; b < dof; ++b) {
                    double s = 0;
                    for (int a = 0; a < dof; ++a) s += PHt[(size_t)r * dof + a] * Sinv[(size_t)a * dof + b];
                    K[(size_t)r * dof + b] = s / R;
                }
            for (int r = 0; r < NX; ++r) {
                double s = 0;
                for (int b = 0; b < dof; ++b) s += K[(size_t)r * dof + b] * rows[7 * b + 6];
                K_h[r] = s;
                for (int c = 0; c < 6; ++c) {
                    double s2 = 0;
                    for (int b = 0; b < dof; ++b) s2 += K[(size_t)r * dof + b] * rows[7 * b + c];
                    K_x[(size_t)r * NX + c] = s2;
                }
            }
        } else {
            std::vector<double> Pr((size_t)NX * NX), Ptemp, Pinv;
            for (size_t q = 0; q < Pr.size(); ++q) Pr[q] = P[q] / R;
            invert(Pr, Ptemp, NX);
            double HTH[36];
            int q = 0;
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) {
                    HTH[a * 6 + b] = sums[S_HTH + q];
                    HTH[b * 6 + a] = sums[S_HTH + q];
                    ++q;
                }
            for (int a = 0; a < 6; ++a)
                for (int b = 0; b < 6; ++b) Ptemp[(size_t)a * NX + b] += HTH[a * 6 + b];
            invert(Ptemp, Pinv, NX);
            for (int r = 0; r < NX; ++r) {
                double s = 0;
                for (int c = 0; c < 6; ++c) s += Pinv[(size_t)r * NX + c] * sums[S_HTh + c];
                K_h[r] = s;
                for (int c = 0; c < 6; ++c) {
                    double s2 = 0;
                    for (int m = 0; m < 6; ++m) s2 += Pinv[(size_t)r * NX + m] * HTH[m * 6 + c];
                    K_x[(size_t)r * NX + c] = s2;
                }
            }
        }
        double dxu[NX];
        for (int r = 0; r < NX; ++r) {
            double s = 0;
            for (int c = 0; c < NX; ++c) s += (K_x[(size_t)r * NX + c] - (r == c ? 1.0 : 0.0)) * dx_new[c];
            dxu[r] = K_h[r] + s;
        }
        state_boxplus(x, dxu);
        converge = true;
        for (int r = 0; r < NX; ++r)
            if (std::fabs(dxu[r]) > limit) { converge = false; break; }
        if (converge) ++t;
        if (!t && i == max_iter - 2) converge = true;
        if (t > 1 || i == max_iter - 1) {
            std::vector<double> L = P;
            for (int idx : {3, 6}) {
                double A[9], At[9];
                A_matrix(dxu + idx, A);
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) At[a * 3 + b] = A[b * 3 + a];
                rows_xform(L, NX, idx, At, 3, &P);
                rows_xform(K_x, NX, idx, At, 3, nullptr, 12);
                cols_xform(L, NX, NX, idx, At, 3);
                cols_xform(P, NX, NX, idx, At, 3);
            }
            {
                double Nx[6], Mx[6], T2[4];
                s2_Nx_yy(x.grav, Nx);
                s2_Mx(x_prop.grav, dxu + 21, Mx);
                mm3(Nx, Mx, T2, 2, 3, 2);
                rows_xform(L, NX, 21, T2, 2, &P);
                rows_xform(K_x, NX, 21, T2, 2, nullptr, 12);
                cols_xform(L, NX, NX, 21, T2, 2);
                cols_xform(P, NX, NX, 21, T2, 2);
            }
            std::vector<double> Pn((size_t)NX * NX);
            for (int r = 0; r < NX; ++r)
                for (int c = 0; c < NX; ++c) {
                    double s = 0;
                    for (int m = 0; m < 12; ++m) s += K_x[(size_t)r * NX + m] * P[(size_t)m * NX + c];
                    Pn[(size_t)r * NX + c] = L[(size_t)r * NX + c] - s;
                }
            P = Pn;
            st->converged = t > 1 ? 1 : 0;
            break;
        }
    }
    st->iterations = evals;
    st->knn_calls = knns;
    return 0;
}

// ---------------------------------------------------------------------------
// PCL-1.10 IterativeClosestPoint<PointXYZI,PointXYZI> as configured at
// /root/reference/fast_lio_sam/src/loop_closure.cpp:3-14 and aligned at
// :69-92 [R call sites; PCL internals U]:
//   * correspondences: KdTreeFLANN 1-NN of every (incrementally transformed)
//     source point, rejected if d2 > max_corr_dist^2 (52.5^2, fast_lio_sam.cpp:73)
//   * TransformationEstimationSVD (Umeyama, no scale).  PCL computes it in
//     float through Eigen's vectorised reductions (implementation-defined
//     order); this restatement accumulates the sufficient statistics in double
//     about a fixed centre c0, which is within PCL's own float noise.
//   * transformPointCloud float SSE order x' = m0 x + (m1 y + (m2 z + m3)) [U]
//   * final = T_inc * final (float 4x4, sequential k)
//   * DefaultConvergenceCriteria: max_iter, transform (cos >= 1 - eps_t and
//     |t|^2 <= eps_t), |dMSE| < 1e-12 abs, |dMSE|/MSE_prev < eps_fit rel.
//   * getFitnessScore(): mean unbounded 1-NN d2 of input transformed by final.
// ---------------------------------------------------------------------------
struct IcpParams {
    double max_corr_dist;   // 52.5
    double trans_eps;       // 0.01
    double fitness_eps;     // 0.01
    int max_iter;           // 50
    double rot_eps;         // 0 => 1 - trans_eps
    double score_threshold; // 1.5 (config.yaml:16)
    int umeyama_float = 2;  // internal: 0 = double statistics (the opt-in mode); > 0 = pcl::umeyama in float +
                            //    Eigen JacobiSVD (umeyama_pcl_float) in that summation order (UmeyamaOrder
                            //    below; PCL's own order depends on its Eigen build).  The C entry point takes
                            //    the GPU's values: -1 double (LIO_ICP_UMEYAMA_DOUBLE), 0 default = order 2
};

// Float summation orders of pcl::umeyama (IcpParams::umeyama_float > 0).  Eigen-plausible variants of the
// same arithmetic; their spread at C4 bounds how far "PCL's float result" is defined at all.
//   1 kSeqSeq       means: sequential row sums; sigma: one sequential depth sum, scaled once at the end
//   2 kSeqGemm32    means: sequential; sigma: Eigen 3.3 GEMM, depth blocked by kc from a 32 KiB L1
//                   (res += alpha * block sum per kc block; SSE2 float gebp, mr = 8, nr = 4 => kc = 680)
//   3 kSeqGemm48    as 2 with a 48 KiB L1 (kc = 1016)
//   4 kPacketSeq    means: Eigen's vectorised redux (two 4-float packet accumulators, predux, scalar tail),
//                   which Eigen applies only to contiguous rows — NOT to the strided rows of a col-major
//                   3 x N matrix; kept as a deliberately different order; sigma sequential
//   5 kPacketGemm32 means as 4, sigma as 2
enum UmeyamaOrder { kSeqSeq = 1, kSeqGemm32 = 2, kSeqGemm48 = 3, kPacketSeq = 4, kPacketGemm32 = 5 };

static inline void xform_pt(const float T[16], const float* p, float* o) {
    // T row-major 4x4
    for (int r = 0; r < 3; ++r) {
        float a = T[4 * r] * p[0];
        float b = T[4 * r + 1] * p[1];
        float c = T[4 * r + 2] * p[2];
        o[r] = a + (b + (c + T[4 * r + 3]));
    }
}

// symmetric 3x3 Jacobi eigen-decomposition, used for the SVD of sigma
static void jacobi_eig3(double A[9], double V[9], double w[3]) {
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        if (off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double apq = A[3 * p + q];
                if (std::fabs(apq) < 1e-300) continue;
                double app = A[3 * p + p], aqq = A[3 * q + q];
                double tau = (aqq - app) / (2 * apq);
                double tt = (tau >= 0 ? 1.0 : -1.0) / (std::fabs(tau) + std::sqrt(1 + tau * tau));
                double c = 1 / std::sqrt(1 + tt * tt), s = tt * c;
                for (int k = 0; k < 3; ++k) {  // A := J^T A J
                    double akp = A[3 * k + p], akq = A[3 * k + q];
                    A[3 * k + p] = c * akp - s * akq;
                    A[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = A[3 * p + k], aqk = A[3 * q + k];
                    A[3 * p + k] = c * apk - s * aqk;
                    A[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < 3; ++i) w[i] = A[4 * i];
}
static double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// Umeyama (no scaling) from double sufficient statistics about centre c0.
// stats: [0]=n [1..3]=sum p [4..6]=sum q [7..15]=sum q p^T (row-major) [16]=sum d2
static void umeyama(const double* st, const double c0[3], double Rout[9], double tout[3]) {
    double inv_n = 1.0 / st[0];
    double pm[3], qm[3], S[9];
    for (int i = 0; i < 3; ++i) { pm[i] = st[1 + i] * inv_n; qm[i] = st[4 + i] * inv_n; }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) S[3 * r + c] = st[7 + 3 * r + c] * inv_n - qm[r] * pm[c];
    // SVD via eigen-decomposition of S^T S (V) and U = S V / sigma, sorted descending
    double StS[9], V[9], w[3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) StS[3 * r + c] = S[r] * S[c] + S[3 + r] * S[3 + c] + S[6 + r] * S[6 + c];
    jacobi_eig3(StS, V, w);
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int a, int b) { return w[a] > w[b]; });
    double Vs[9], U[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Vs[3 * r + c] = V[3 * r + ord[c]];
    // U columns: u_i = S v_i / |S v_i|, Gram-Schmidt, third = u0 x u1 (then sign fixed by det)
    double u[3][3];
    for (int i = 0; i < 2; ++i) {
        for (int r = 0; r < 3; ++r) u[i][r] = S[3 * r] * Vs[i] + S[3 * r + 1] * Vs[3 + i] + S[3 * r + 2] * Vs[6 + i];
        if (i == 1) {
            double d = u[1][0] * u[0][0] + u[1][1] * u[0][1] + u[1][2] * u[0][2];
            for (int r = 0; r < 3; ++r) u[1][r] -= d * u[0][r];
        }
        double nn = std::sqrt(u[i][0] * u[i][0] + u[i][1] * u[i][1] + u[i][2] * u[i][2]);
        for (int r = 0; r < 3; ++r) u[i][r] /= nn;
    }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    // sign of the third left vector consistent with S v_2 (sigma_2 may be ~0)
    double sv2[3];
    for (int r = 0; r < 3; ++r) sv2[r] = S[3 * r] * Vs[2] + S[3 * r + 1] * Vs[5] + S[3 * r + 2] * Vs[8];
    if (sv2[0] * u[2][0] + sv2[1] * u[2][1] + sv2[2] * u[2][2] < 0)
        for (int r = 0; r < 3; ++r) u[2][r] = -u[2][r];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) U[3 * r + c] = u[c][r];
    double D = (det3(U) * det3(Vs) < 0) ? -1.0 : 1.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            Rout[3 * r + c] = U[3 * r] * Vs[3 * c] + U[3 * r + 1] * Vs[3 * c + 1] + D * U[3 * r + 2] * Vs[3 * c + 2];
    for (int r = 0; r < 3; ++r) {
        double rp = Rout[3 * r] * (pm[0] + c0[0]) + Rout[3 * r + 1] * (pm[1] + c0[1]) + Rout[3 * r + 2] * (pm[2] + c0[2]);
        tout[r] = (qm[r] + c0[r]) - rp;
    }
}

// ---------------------------------------------------------------------------
// Float mode (IcpParams::umeyama_float): PCL 1.10 TransformationEstimationSVD<PointXYZI, PointXYZI, float>
// with use_umeyama_ = true calls pcl::umeyama(cloud_src, cloud_tgt, false) on 3 x N float matrices
// (common/impl/eigen.hpp, a copy of Eigen 3.3 Geometry/Umeyama.h) [U]:
//   one_over_n = 1 / n; src_mean = src.rowwise().sum() * one_over_n (likewise dst);
//   demean; sigma = one_over_n * dst_demean * src_demean^T; JacobiSVD(sigma, FullU | FullV);
//   S = I, S(2) = -1 if det(U) det(V) < 0; R = U S V^T; t = dst_mean - R src_mean.
// Restated in float.  The summation order is a build property of PCL's Eigen, so it is a parameter
// (UmeyamaOrder): the row sums are sequential in Eigen 3.3 (its partial redux over a strided row is not
// vectorised; order 4/5 models the vectorised redux of a contiguous row as a deliberately different
// order); sigma's depth sum is one sequential chain (order 1) or, as Eigen 3.3's GEMM evaluates a
// 3 x N by N x 3 product past 13 columns, blocked by an L1-size-dependent kc with res += alpha * (block
// sum) per block (orders 2/3/5, eigen_gemm_kc).  JacobiSVD (Eigen 3.3 JacobiSVD::compute,
// real_2x2_jacobi_svd, JacobiRotation::makeJacobi, apply_rotation_in_the_plane) is restated exactly.
// Small fixed products (R = U S V^T, R * src_mean) sum their 3 terms as e0 + (e1 + e2).
// ---------------------------------------------------------------------------
struct JRot { float c, s; };

static bool make_jacobi(float x, float y, float z, JRot& j) {  // JacobiRotation::makeJacobi (real)
    const float deno = 2.f * std::fabs(y);
    if (deno < FLT_MIN) {
        j.c = 1.f;
        j.s = 0.f;
        return false;
    }
    const float tau = (x - z) / deno;
    const float w = std::sqrt(tau * tau + 1.f);
    const float t = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
    const float sign_t = t > 0.f ? 1.f : -1.f;
    const float n = 1.f / std::sqrt(t * t + 1.f);
    j.s = ((-sign_t) * (y / std::fabs(y))) * std::fabs(t) * n;
    j.c = n;
    return true;
}

// apply_rotation_in_the_plane(x, y, j) over 3 strided elements
static void rot_plane(float* x, float* y, int inc, JRot j) {
    if (j.c == 1.f && j.s == 0.f) return;
    for (int i = 0; i < 3; ++i) {
        const float xi = x[i * inc], yi = y[i * inc];
        x[i * inc] = j.c * xi + j.s * yi;
        y[i * inc] = -j.s * xi + j.c * yi;
    }
}
// M is column-major 3x3 (M[3*col + row]), as Eigen stores Matrix3f
static void apply_left(float* M, int p, int q, JRot j) { rot_plane(M + p, M + q, 3, j); }          // rows
static void apply_right(float* M, int p, int q, JRot j) { rot_plane(M + 3 * p, M + 3 * q, 1, {j.c, -j.s}); }  // cols, j^T

static void jacobi_svd3f(const float* A, float U[9], float V[9], float sv[3]) {
    float scale = 0.f;
    for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(A[i]));  // cwiseAbs().maxCoeff()
    if (scale == 0.f) scale = 1.f;
    float W[9];
    for (int i = 0; i < 9; ++i) W[i] = A[i] / scale;
    for (int i = 0; i < 9; ++i) U[i] = V[i] = (i % 4 == 0) ? 1.f : 0.f;
    const float precision = 2.f * FLT_EPSILON, consider_zero = FLT_MIN;
    auto w = [&](int r, int c) -> float& { return W[3 * c + r]; };
    float max_diag = std::max(std::max(std::fabs(w(0, 0)), std::fabs(w(1, 1))), std::fabs(w(2, 2)));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 1000; ++sweep) {
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const float threshold = std::max(consider_zero, precision * max_diag);
                if (std::fabs(w(p, q)) > threshold || std::fabs(w(q, p)) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd(W, p, q, &j_left, &j_right)
                    float m00 = w(p, p), m01 = w(p, q), m10 = w(q, p), m11 = w(q, q);
                    JRot rot1;
                    const float t = m00 + m11, d = m10 - m01;
                    if (std::fabs(d) < FLT_MIN) {
                        rot1 = {1.f, 0.f};
                    } else {
                        const float u = t / d;
                        const float tmp = std::sqrt(1.f + u * u);
                        rot1.s = 1.f / tmp;
                        rot1.c = u / tmp;
                    }
                    {  // m.applyOnTheLeft(0, 1, rot1)
                        float x0 = m00, y0 = m10, x1 = m01, y1 = m11;
                        if (!(rot1.c == 1.f && rot1.s == 0.f)) {
                            m00 = rot1.c * x0 + rot1.s * y0;
                            m10 = -rot1.s * x0 + rot1.c * y0;
                            m01 = rot1.c * x1 + rot1.s * y1;
                            m11 = -rot1.s * x1 + rot1.c * y1;
                        }
                    }
                    JRot jr;
                    make_jacobi(m00, m01, m11, jr);
                    const JRot jrt{jr.c, -jr.s};                 // j_right.transpose()
                    const JRot jl{rot1.c * jrt.c - rot1.s * jrt.s,  // rot1 * j_right^T
                                  rot1.c * jrt.s + rot1.s * jrt.c};
                    apply_left(W, p, q, jl);
                    apply_right(U, p, q, {jl.c, -jl.s});  // U.applyOnTheRight(p, q, j_left.transpose())
                    apply_right(W, p, q, jr);
                    apply_right(V, p, q, jr);
                    max_diag = std::max(max_diag, std::max(std::fabs(w(p, p)), std::fabs(w(q, q))));
                }
            }
    }
    for (int i = 0; i < 3; ++i) {
        const float a = w(i, i);
        sv[i] = std::fabs(a);
        if (a < 0.f)
            for (int r = 0; r < 3; ++r) U[3 * i + r] = -U[3 * i + r];
    }
    for (int i = 0; i < 3; ++i) sv[i] *= scale;
    for (int i = 0; i < 3; ++i) {  // sort descending (maxCoeff: first maximum)
        int pos = i;
        for (int k = i + 1; k < 3; ++k)
            if (sv[k] > sv[pos]) pos = k;
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int r = 0; r < 3; ++r) {
                std::swap(U[3 * i + r], U[3 * pos + r]);
                std::swap(V[3 * i + r], V[3 * pos + r]);
            }
        }
    }
}

static float det3f_colmajor(const float* M) {  // Eigen determinant_impl<3>: bruteforce_det3_helper
    auto m = [&](int r, int c) { return M[3 * c + r]; };
    auto h = [&](int a, int b, int c) { return m(a, 0) * (m(b, 1) * m(c, 2) - m(b, 2) * m(c, 1)); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// Eigen 3.3 evaluateProductBlockingSizesHeuristic (GeneralBlockPanelKernel.h), one thread: the depth
// block kc of a 3 x k by k x 3 float GEMM on an SSE2 build (no FMA: gebp_traits<float, float> mr = 8,
// nr = 4; KcFactor 1) whose L1 data cache holds l1 bytes.  Problems below 48 are not blocked.
int64_t eigen_gemm_kc(int64_t k, int64_t l1) {
    const int64_t mr = 8, nr = 4, k_peeling = 8;
    const int64_t k_div = mr * 4 + nr * 4, k_sub = mr * nr * 4;
    if (std::max<int64_t>(k, 3) < 48) return k;
    const int64_t max_kc = std::max<int64_t>(((l1 - k_sub) / k_div) & ~(k_peeling - 1), 1);
    if (k > max_kc)
        k = (k % max_kc) == 0 ? max_kc
                              : max_kc - k_peeling * ((max_kc - 1 - (k % max_kc)) / (k_peeling * (k / max_kc + 1)));
    return k;
}

// A row sum of pcl::umeyama: sequential from the first coefficient (Eigen redux, DefaultTraversal) or,
// packet4, Eigen's LinearVectorizedTraversal (packets p0 / p1 alternating over 8-float strides, p0 += p1,
// one more packet if it fits, predux = (p0[0] + p0[2]) + (p0[1] + p0[3]), then the scalar tail).
static float row_sum(const std::vector<float>& v, int d, int64_t n, bool packet4) {
    auto x = [&](int64_t i) { return v[3 * i + d]; };
    if (!packet4 || n < 4) {
        float a = x(0);
        for (int64_t i = 1; i < n; ++i) a += x(i);
        return a;
    }
    const int64_t end2 = (n / 8) * 8, end1 = (n / 4) * 4;
    float p0[4], p1[4];
    for (int l = 0; l < 4; ++l) p0[l] = x(l);
    if (end1 > 4) {
        for (int l = 0; l < 4; ++l) p1[l] = x(4 + l);
        for (int64_t i = 8; i < end2; i += 8)
            for (int l = 0; l < 4; ++l) {
                p0[l] += x(i + l);
                p1[l] += x(i + 4 + l);
            }
        for (int l = 0; l < 4; ++l) p0[l] += p1[l];
        if (end1 > end2)
            for (int l = 0; l < 4; ++l) p0[l] += x(end2 + l);
    }
    float a = (p0[0] + p0[2]) + (p0[1] + p0[3]);
    for (int64_t i = end1; i < n; ++i) a += x(i);
    return a;
}

// src / tgt: the correspondence pairs in correspondence (source index) order, xyz interleaved;
// order: UmeyamaOrder (summation order of the means and of sigma's depth)
void umeyama_pcl_float(const std::vector<float>& src, const std::vector<float>& tgt, float Ti[16], int order,
                       float* stats15 = nullptr) {
    const int64_t n = (int64_t)(src.size() / 3);
    const float one_over_n = 1.f / (float)n;
    const bool packet = order == kPacketSeq || order == kPacketGemm32;
    float sm[3], dm[3];
    for (int d = 0; d < 3; ++d) {
        sm[d] = row_sum(src, d, n, packet) * one_over_n;
        dm[d] = row_sum(tgt, d, n, packet) * one_over_n;
    }
    float sigma[9];  // column-major
    auto prod = [&](int64_t i, int r, int c) {  // dst_demean(r, i) * src_demean(c, i), both demeaned in float
        return (tgt[3 * i + r] - dm[r]) * (src[3 * i + c] - sm[c]);
    };
    const int64_t l1 = (order == kSeqGemm48) ? 48 * 1024 : 32 * 1024;
    if (order == kSeqGemm32 || order == kSeqGemm48 || order == kPacketGemm32) {
        if (n + 3 + 3 < 20) {
            // generic_product_impl::evalTo: rhs.rows() + dst.rows() + dst.cols() < 20 => the lazy
            // coefficient-based product, (alpha * dst_demean).row(r) . src_demean.row(c), sequential
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    float a = (one_over_n * (tgt[r] - dm[r])) * (src[c] - sm[c]);
                    for (int64_t i = 1; i < n; ++i) a += (one_over_n * (tgt[3 * i + r] - dm[r])) * (src[3 * i + c] - sm[c]);
                    sigma[3 * c + r] = a;
                }
        } else {
            // dst.setZero(); gemm: for each depth block, gebp's 1 x 1 remainder path (3 rows < LhsProgress 4,
            // 3 cols < nr 4): C0 = sequential sum of the block's products; res(r, c) += alpha * C0
            const int64_t kc = eigen_gemm_kc(n, l1);
            for (int i = 0; i < 9; ++i) sigma[i] = 0.f;
            for (int64_t k2 = 0; k2 < n; k2 += kc) {
                const int64_t k3 = std::min(n, k2 + kc);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) {
                        float C0 = 0.f;
                        for (int64_t i = k2; i < k3; ++i) C0 += prod(i, r, c);
                        sigma[3 * c + r] += one_over_n * C0;
                    }
            }
        }
    } else {
        float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // sum_k dst_demean(r, k) src_demean(c, k), row-major r, c
        for (int64_t i = 0; i < n; ++i)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) acc[3 * r + c] += prod(i, r, c);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) sigma[3 * c + r] = one_over_n * acc[3 * r + c];
    }
    if (stats15) {  // src mean, tgt mean, sigma row-major
        for (int d = 0; d < 3; ++d) stats15[d] = sm[d], stats15[3 + d] = dm[d];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) stats15[6 + 3 * r + c] = sigma[3 * c + r];
    }
    float U[9], V[9], svals[3];
    jacobi_svd3f(sigma, U, V, svals);
    float S[3] = {1.f, 1.f, 1.f};
    if (det3f_colmajor(U) * det3f_colmajor(V) < 0.f) S[2] = -1.f;
    float R[9];  // row-major
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            const float e0 = (U[r] * S[0]) * V[c], e1 = (U[3 + r] * S[1]) * V[3 + c], e2 = (U[6 + r] * S[2]) * V[6 + c];
            R[3 * r + c] = e0 + (e1 + e2);
        }
    for (int i = 0; i < 16; ++i) Ti[i] = 0.f;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) Ti[4 * r + c] = R[3 * r + c];
        Ti[4 * r + 3] = dm[r] - (R[3 * r] * sm[0] + (R[3 * r + 1] * sm[1] + R[3 * r + 2] * sm[2]));
    }
    Ti[15] = 1.f;
}

struct IcpResult {
    float T[16];
    double fitness;
    int converged;
    int iterations;
    int state;  // 0 not conv, 1 iterations, 2 transform, 3 abs mse, 4 rel mse, 5 no correspondences
};

int icp_align(const float* src, int64_t ns, const float* dst, int64_t nd, const IcpParams& ip,
              const float* guess, IcpResult* res, float* aligned, double* trace, int max_trace, int threads) {
    KdTree tree;
    tree.build(dst, nd);
    // fixed accumulation centre: target bounding-box centre (float)
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = 0; i < nd; ++i)
        for (int d = 0; d < 3; ++d) {
            lo[d] = std::min(lo[d], dst[3 * i + d]);
            hi[d] = std::max(hi[d], dst[3 * i + d]);
        }
    double c0[3];
    for (int d = 0; d < 3; ++d) c0[d] = (double)(0.5f * (lo[d] + hi[d]));
    if (nd == 0) for (int d = 0; d < 3; ++d) c0[d] = 0.0;

    std::vector<float> cur(src, src + 3 * ns);
    float fin[16];
    bool ident = true;
    for (int i = 0; i < 16; ++i) {
        fin[i] = guess[i];
        if (guess[i] != ((i % 5 == 0) ? 1.f : 0.f)) ident = false;
    }
    if (!ident)
        for (int64_t i = 0; i < ns; ++i) xform_pt(guess, src + 3 * i, &cur[3 * i]);
    const double max_d2 = ip.max_corr_dist * ip.max_corr_dist;
    const double rot_thr = ip.rot_eps > 0 ? ip.rot_eps : 1.0 - ip.trans_eps;
    double prev_mse = std::numeric_limits<double>::max();
    int iters = 0, similar = 0;
    res->converged = 0;
    res->state = 0;
    std::vector<int32_t> nn(ns);
    std::vector<float> nd2(ns);
    for (;;) {
#pragma omp parallel for schedule(dynamic, 1024) num_threads(threads)
        for (int64_t i = 0; i < ns; ++i) {
            float d2;
            tree.knn(&cur[3 * i], 1, INFINITY, &nn[i], &d2);
            nd2[i] = d2;
        }
        double st[17] = {0};
        for (int64_t i = 0; i < ns; ++i) {
            if (nn[i] < 0 || (double)nd2[i] > max_d2) continue;
            const float* p = &cur[3 * i];
            const float* q = dst + 3 * (size_t)nn[i];
            double pd[3] = {p[0] - c0[0], p[1] - c0[1], p[2] - c0[2]};
            double qd[3] = {q[0] - c0[0], q[1] - c0[1], q[2] - c0[2]};
            st[0] += 1.0;
            for (int d = 0; d < 3; ++d) { st[1 + d] += pd[d]; st[4 + d] += qd[d]; }
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) st[7 + 3 * r + c] += qd[r] * pd[c];
            st[16] += (double)nd2[i];
        }
        if (st[0] < 3) {
            res->converged = 0;
            res->state = 5;
            break;
        }
        float Ti[16] = {0};
        if (ip.umeyama_float) {
            std::vector<float> ps, qs;
            ps.reserve(3 * (size_t)st[0]);
            qs.reserve(3 * (size_t)st[0]);
            for (int64_t i = 0; i < ns; ++i) {
                if (nn[i] < 0 || (double)nd2[i] > max_d2) continue;
                ps.insert(ps.end(), &cur[3 * i], &cur[3 * i] + 3);
                qs.insert(qs.end(), dst + 3 * (size_t)nn[i], dst + 3 * (size_t)nn[i] + 3);
            }
            umeyama_pcl_float(ps, qs, Ti, ip.umeyama_float);
        } else {
            double Rd[9], td[3];
            umeyama(st, c0, Rd, td);
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) Ti[4 * r + c] = (float)Rd[3 * r + c];
                Ti[4 * r + 3] = (float)td[r];
            }
            Ti[15] = 1.f;
        }
        for (int64_t i = 0; i < ns; ++i) {
            float o[3];
            xform_pt(Ti, &cur[3 * i], o);
            cur[3 * i] = o[0]; cur[3 * i + 1] = o[1]; cur[3 * i + 2] = o[2];
        }
        float nf[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                float s = Ti[4 * r] * fin[c];
                s += Ti[4 * r + 1] * fin[4 + c];
                s += Ti[4 * r + 2] * fin[8 + c];
                s += Ti[4 * r + 3] * fin[12 + c];
                nf[4 * r + c] = s;
            }
        std::memcpy(fin, nf, sizeof(fin));
        ++iters;
        double mse = st[16] / st[0];
        if (trace && iters <= max_trace) {
            double* tr = trace + 20 * (iters - 1);
            tr[0] = st[0];
            tr[1] = mse;
            for (int k = 0; k < 16; ++k) tr[2 + k] = Ti[k];
            tr[18] = tr[19] = 0;
        }
        // DefaultConvergenceCriteria::hasConverged
        bool done = false, is_similar = false;
        if (iters >= ip.max_iter) {
            res->state = 1;
            done = true;
        } else {
            // PCL 1.10 DefaultConvergenceCriteria<float>: the coefficients of the Matrix4f are summed and
            // squared in float, then widened (0.5 * float -> double; float -> double translation_sqr)
            const float tr_f = Ti[0] + Ti[5] + Ti[10] - 1.f;
            const float tsq_f = Ti[3] * Ti[3] + Ti[7] * Ti[7] + Ti[11] * Ti[11];
            double cosang = 0.5 * (double)tr_f;
            double tsq = (double)tsq_f;
            if (cosang >= rot_thr && tsq <= ip.trans_eps) {
                if (similar >= 0) { res->state = 2; done = true; }
                is_similar = true;
            }
            if (!done && std::fabs(mse - prev_mse) < 1e-12) {
                if (similar >= 0) { res->state = 3; done = true; }
                is_similar = true;
            }
            if (!done && std::fabs(mse - prev_mse) / prev_mse < ip.fitness_eps) {
                if (similar >= 0) { res->state = 4; done = true; }
                is_similar = true;
            }
            if (!done) {
                similar = is_similar ? similar + 1 : 0;
                prev_mse = mse;
            }
        }
        if (done) {
            res->converged = 1;
            break;
        }
    }
    std::memcpy(res->T, fin, sizeof(fin));
    res->iterations = iters;
    // getFitnessScore(): original source transformed by the final transform
    std::vector<float> al(3 * ns);
    for (int64_t i = 0; i < ns; ++i) xform_pt(fin, src + 3 * i, &al[3 * i]);
#pragma omp parallel for schedule(dynamic, 1024) num_threads(threads)
    for (int64_t i = 0; i < ns; ++i) {
        float d2;
        tree.knn(&al[3 * i], 1, INFINITY, &nn[i], &d2);
        nd2[i] = d2;
    }
    double fs = 0.0;
    int64_t nr = 0;
    for (int64_t i = 0; i < ns; ++i)
        if (nn[i] >= 0) { fs += nd2[i]; ++nr; }
    res->fitness = nr > 0 ? fs / nr : std::numeric_limits<double>::max();
    if (aligned) std::memcpy(aligned, al.data(), sizeof(float) * 3 * ns);
    return 0;
}


// ---------------------------------------------------------------------------
// Incremental map maintenance.
//
// DynMap: every point ever inserted keeps its id (insertion order); deleted
// points stay as tombstones.  The kNN tree is rebuilt over the alive ids.
//
// add_points   = ikd-Tree KD_TREE::Add_Points(PointToAdd, downsample_on) [U]:
//   for each point p (in order), with downsample:
//     box  = [floor(p/ds)*ds, +ds) per axis (float), half-open like
//            Search_by_range's `min <= x < max` [U]
//     mid  = box_min + (box_max - box_min)/2.0 (double, stored float)
//     S    = alive points in the box; winner = p, then any s in S with
//            calc_dist(s, mid) < calc_dist(winner, mid) (strict, first wins)
//     if |S| > 1 || same_point(p, winner): delete the box, add the winner
//   without downsample: plain add.
//   Ids: the survivor of a box keeps its id when it was already in the map;
//   new survivors get ids appended in input order when the call ends (a new
//   point superseded later in the same call never receives an id).  The
//   ikd-Tree re-inserts a surviving point as a new node; ids are internal to
//   this restatement and the GPU path, so the point set is what matches.
// delete_boxes = KD_TREE::Delete_Point_Boxes [U]: alive points with
//   min <= x < max on all axes are deleted.
// map_incremental = FAST-LIO laserMapping.cpp map_incremental() [U]: see
//   classify() below.
// ---------------------------------------------------------------------------
static inline float calc_dist3(const float* a, const float* b) { return sqdist(a, b); }
static inline bool same_point3(const float* a, const float* b) {
    return std::fabs(a[0] - b[0]) < 1e-6f && std::fabs(a[1] - b[1]) < 1e-6f && std::fabs(a[2] - b[2]) < 1e-6f;
}

struct DynMap {
    std::vector<float> xyz;      // all ids
    std::vector<uint8_t> alive;  // per id
    KdTree tree;
    bool dirty = true;

    int64_t n_ids() const { return (int64_t)alive.size(); }
    void refresh() {
        if (!dirty) return;
        std::vector<int32_t> ids;
        for (int64_t i = 0; i < n_ids(); ++i)
            if (alive[i]) ids.push_back((int32_t)i);
        tree.build_ids(xyz.data(), n_ids(), ids);
        dirty = false;
    }
    int64_t alive_count() const {
        int64_t c = 0;
        for (uint8_t a : alive) c += a;
        return c;
    }

    int64_t add_points(const float* p, int64_t n, bool downsample, float ds) {
        if (!downsample) {
            for (int64_t i = 0; i < 3 * n; ++i) xyz.push_back(p[i]);
            alive.insert(alive.end(), (size_t)n, 1);
            dirty = true;
            return n;
        }
        // pending new points (index into p), alive until superseded.  Candidate
        // lookup through integer voxel buckets (the exact float box test below
        // decides; the 27 neighbouring buckets cover any rounding at the faces).
        std::vector<uint8_t> pend(n, 0);
        int64_t counter = 0;
        auto bkey = [ds](const float* a) {
            const int64_t kx = (int64_t)std::floor(a[0] / ds), ky = (int64_t)std::floor(a[1] / ds),
                          kz = (int64_t)std::floor(a[2] / ds);
            return ((kx + (1 << 20)) << 42) | ((ky + (1 << 20)) << 21) | (kz + (1 << 20));
        };
        std::unordered_map<int64_t, std::vector<int64_t>> bmap, bnew;
        {   // only the buckets a lookup below can reach (the 27 around each input point's bucket)
            std::unordered_set<int64_t> need;
            for (int64_t i = 0; i < n; ++i) {
                const int64_t k0 = bkey(p + 3 * i);
                for (int dx = -1; dx <= 1; ++dx)
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dz = -1; dz <= 1; ++dz)
                            need.insert(k0 + (int64_t)dx * (int64_t(1) << 42) + (int64_t)dy * (int64_t(1) << 21) + dz);
            }
            for (int64_t id = 0; id < n_ids(); ++id)
                if (alive[id]) {
                    const int64_t k = bkey(&xyz[3 * id]);
                    if (need.count(k)) bmap[k].push_back(id);
                }
        }
        auto gather = [&](std::unordered_map<int64_t, std::vector<int64_t>>& bm, int64_t k0, std::vector<int64_t>& out) {
            for (int dx = -1; dx <= 1; ++dx)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dz = -1; dz <= 1; ++dz) {
                        auto it = bm.find(k0 + (int64_t)dx * (int64_t(1) << 42) + (int64_t)dy * (int64_t(1) << 21) + dz);
                        if (it != bm.end()) out.insert(out.end(), it->second.begin(), it->second.end());
                    }
            std::sort(out.begin(), out.end());
        };
        for (int64_t i = 0; i < n; ++i) {
            const float* q = p + 3 * i;
            float vmin[3], vmax[3], mid[3];
            for (int d = 0; d < 3; ++d) {
                vmin[d] = std::floor(q[d] / ds) * ds;
                vmax[d] = vmin[d] + ds;
                mid[d] = (float)((double)vmin[d] + (double)(vmax[d] - vmin[d]) / 2.0);
            }
            auto inbox = [&](const float* a) {
                return vmin[0] <= a[0] && vmax[0] > a[0] && vmin[1] <= a[1] && vmax[1] > a[1] && vmin[2] <= a[2] &&
                       vmax[2] > a[2];
            };
            // storage: alive map points in id order, then pending new points in input order
            std::vector<int64_t> cand_map, cand_new, st_map, st_new;
            const int64_t k0 = bkey(q);
            gather(bmap, k0, cand_map);
            gather(bnew, k0, cand_new);
            for (int64_t id : cand_map)
                if (alive[id] && inbox(&xyz[3 * id])) st_map.push_back(id);
            for (int64_t j : cand_new)
                if (pend[j] && inbox(p + 3 * j)) st_new.push_back(j);
        const size_t ns = st_map.size() + st_new.size();
            float md = calc_dist3(q, mid);
            const float* win = q;
            int64_t win_map = -1, win_new = i;
            for (int64_t id : st_map) {
                const float t = calc_dist3(&xyz[3 * id], mid);
                if (t < md) { md = t; win = &xyz[3 * id]; win_map = id; win_new = -1; }
            }
            for (int64_t j : st_new) {
                const float t = calc_dist3(p + 3 * j, mid);
                if (t < md) { md = t; win = p + 3 * j; win_map = -1; win_new = j; }
            }
            if (ns > 1 || same_point3(q, win)) {
                for (int64_t id : st_map)
                    if (id != win_map) alive[id] = 0;
                for (int64_t j : st_new)
                    if (j != win_new) pend[j] = 0;
                if (win_new == i) {
                    pend[i] = 1;
                    bnew[k0].push_back(i);
                }
                ++counter;
            }
        }
        for (int64_t i = 0; i < n; ++i)
            if (pend[i]) {
                xyz.insert(xyz.end(), p + 3 * i, p + 3 * i + 3);
                alive.push_back(1);
            }
        dirty = true;
        return counter;
    }

    int64_t delete_boxes(const float* boxes, int nb) {
        int64_t cnt = 0;
        for (int64_t id = 0; id < n_ids(); ++id) {
            if (!alive[id]) continue;
            const float* a = &xyz[3 * id];
            for (int b = 0; b < nb; ++b) {
                const float* bx = boxes + 6 * b;
                if (bx[0] <= a[0] && bx[3] > a[0] && bx[1] <= a[1] && bx[4] > a[1] && bx[2] <= a[2] && bx[5] > a[2]) {
                    alive[id] = 0;
                    ++cnt;
                    break;
                }
            }
        }
        dirty = true;
        return cnt;
    }
};

// map_incremental() [U]: Nearest_Points come from the last kNN evaluation
// (unbounded 5-NN at pose_knn: ikd-Tree Nearest_Search with max_dist = INF);
// the world points use the final state.  Per point:
//   mid  = floor(w/fs)*fs + 0.5*fs (double, stored float); dist = calc_dist(w, mid)
//   |near0 - mid| > 0.5*fs on all three axes          -> PointNoNeedDownsample
//   else need_add unless some near_j (j < 5, only when 5 exist) has
//        calc_dist(near_j, mid) < dist                 -> PointToAdd / skip
//   then Add_Points(PointToAdd, true); Add_Points(PointNoNeedDownsample, false).
// stats: [to_add, no_need, skipped, added_by_downsample_call]
static void map_incremental(DynMap& dm, const float* body, int64_t n, const Pose& pk, const Pose& pf, double fs,
                            float ds, int64_t* stats) {
    dm.refresh();
    std::vector<float> to_add, no_need;
    int64_t skipped = 0;
    // the unbounded 5-NN of every point against the map as it is before this call's adds
    // (independent queries: parallel; the classification below stays sequential)
    std::vector<int32_t> nn_all(5 * (size_t)n);
    std::vector<int> found_all(n);
#pragma omp parallel for schedule(dynamic, 512) num_threads(8)
    for (int64_t i = 0; i < n; ++i) {
        float wk[3], d2[5];
        body_to_world(pk, body + 3 * i, wk);
        found_all[i] = dm.tree.knn(wk, 5, INFINITY, &nn_all[5 * (size_t)i], d2);
    }
    for (int64_t i = 0; i < n; ++i) {
        float w[3];
        body_to_world(pf, body + 3 * i, w);
        const int32_t* nn = &nn_all[5 * (size_t)i];
        const int found = found_all[i];
        if (found == 0) {
            to_add.insert(to_add.end(), w, w + 3);
            continue;
        }
        float mid[3];
        for (int d = 0; d < 3; ++d) mid[d] = (float)(std::floor((double)w[d] / fs) * fs + 0.5 * fs);
        const float dist = calc_dist3(w, mid);
        const float* n0 = &dm.xyz[3 * (size_t)nn[0]];
        if (std::fabs(n0[0] - mid[0]) > 0.5 * fs && std::fabs(n0[1] - mid[1]) > 0.5 * fs &&
            std::fabs(n0[2] - mid[2]) > 0.5 * fs) {
            no_need.insert(no_need.end(), w, w + 3);
            continue;
        }
        bool need_add = true;
        for (int j = 0; j < 5; ++j) {
            if (found < 5) break;
            if (calc_dist3(&dm.xyz[3 * (size_t)nn[j]], mid) < dist) {
                need_add = false;
                break;
            }
        }
        if (need_add)
            to_add.insert(to_add.end(), w, w + 3);
        else
            ++skipped;
    }
    const int64_t na = (int64_t)to_add.size() / 3, nn_ = (int64_t)no_need.size() / 3;
    const int64_t c = dm.add_points(to_add.data(), na, true, ds);
    dm.add_points(no_need.data(), nn_, false, ds);
    stats[0] = na;
    stats[1] = nn_;
    stats[2] = skipped;
    stats[3] = c;
}


// ---------------------------------------------------------------------------
// Point-cloud filters.
//
// voxel_grid = pcl::VoxelGrid<PointT>::applyFilter, PCL 1.10 [U], with
//   downsample_all_data_ = true and min_points_per_voxel_ = 0:
//   getMinMax3D over finite points; inverse_leaf = 1/leaf (float);
//   min_b = (int)floor(min_p * inv), max_b = (int)floor(max_p * inv);
//   div_b = max_b - min_b + 1, divb_mul = (1, div_b.x, div_b.x*div_b.y);
//   overflow (div_b product > INT_MAX) -> output = input;
//   idx = (int)(floor(p*inv) - (float)min_b) . divb_mul; sort by idx (PCL's
//   std::sort leaves the order inside a voxel unspecified: here input order);
//   centroid = fields summed in that order, / (float)count; output by idx.
// transform_segments = pcl::transformPointCloud(in, out, Matrix4d) [U]:
//   Transformer<double>::se3, ((m0 x + m1 y) + m2 z) + m3 in double -> float;
//   non-finite points kept unchanged (the !is_dense branch).
// preprocess = FAST-LIO Preprocess selection (i % point_filter_num == 0 and
//   x*x+y*y+z*z > blind^2) + ImuProcess::UndistortPcl (sort by time — stable
//   here, std::sort in the reference — and backward propagation, rotations as
//   matrices) + downSizeFilterSurf (voxel_grid) [U].
// ---------------------------------------------------------------------------
static int64_t voxel_grid(const float* p, int64_t n, int stride, const float leaf[3], float* out) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i) {
        const float* q = p + (size_t)i * stride;
        if (!(std::isfinite(q[0]) && std::isfinite(q[1]) && std::isfinite(q[2]))) continue;
        for (int d = 0; d < 3; ++d) {
            lo[d] = std::min(lo[d], q[d]);
            hi[d] = std::max(hi[d], q[d]);
        }
    }
    if (!(lo[0] <= hi[0])) return 0;
    float inv[3];
    int min_b[3];
    int64_t div[3];
    for (int d = 0; d < 3; ++d) {
        inv[d] = 1.0f / leaf[d];
        min_b[d] = (int)std::floor(lo[d] * inv[d]);
        const int max_b = (int)std::floor(hi[d] * inv[d]);
        div[d] = (int64_t)max_b - min_b[d] + 1;
    }
    if (div[0] * div[1] * div[2] > (int64_t)std::numeric_limits<int32_t>::max()) {
        std::memcpy(out, p, (size_t)n * stride * sizeof(float));
        return n;
    }
    const int mul[3] = {1, (int)div[0], (int)(div[0] * div[1])};
    std::vector<std::pair<int, int64_t>> idx;
    idx.reserve(n);
    for (int64_t i = 0; i < n; ++i) {
        const float* q = p + (size_t)i * stride;
        if (!(std::isfinite(q[0]) && std::isfinite(q[1]) && std::isfinite(q[2]))) continue;
        int k = 0;
        for (int d = 0; d < 3; ++d) k += (int)(std::floor(q[d] * inv[d]) - (float)min_b[d]) * mul[d];
        idx.emplace_back(k, i);
    }
    std::stable_sort(idx.begin(), idx.end(), [](const std::pair<int, int64_t>& a, const std::pair<int, int64_t>& b) {
        return a.first < b.first;
    });
    int64_t m = 0;
    for (size_t j = 0; j < idx.size();) {
        size_t e = j;
        float acc[16] = {0};
        while (e < idx.size() && idx[e].first == idx[j].first) {
            const float* q = p + (size_t)idx[e].second * stride;
            for (int f = 0; f < stride; ++f) acc[f] += q[f];
            ++e;
        }
        for (int f = 0; f < stride; ++f) out[(size_t)m * stride + f] = acc[f] / (float)(e - j);
        ++m;
        j = e;
    }
    return m;
}

static void transform_segments(const float* in, int64_t n, int stride, const int64_t* seg, int nseg,
                               const double* T16, float* out) {
    for (int s = 0; s < nseg; ++s) {
        const double* m = T16 + 16 * s;
        for (int64_t i = seg[s]; i < seg[s + 1] && i < n; ++i) {
            const float* q = in + (size_t)i * stride;
            float* o = out + (size_t)i * stride;
            std::memcpy(o, q, stride * sizeof(float));
            if (!(std::isfinite(q[0]) && std::isfinite(q[1]) && std::isfinite(q[2]))) continue;
            const double x = q[0], y = q[1], z = q[2];
            o[0] = (float)(((m[0] * x + m[1] * y) + m[2] * z) + m[3]);
            o[1] = (float)(((m[4] * x + m[5] * y) + m[6] * z) + m[7]);
            o[2] = (float)(((m[8] * x + m[9] * y) + m[10] * z) + m[11]);
        }
    }
}

struct ImuPoseO {
    double offset_time;
    double acc[3], gyr[3], vel[3], pos[3], rot[9];
};

static inline unsigned long long dbits(double v) {
    unsigned long long u;
    std::memcpy(&u, &v, sizeof(u));
    return u;
}
static inline double bitsd(unsigned long long u) {
    double v;
    std::memcpy(&v, &u, sizeof(v));
    return v;
}
// sin / cos for UndistortPcl's SO3 Exp.  The reference calls libm sin / cos, whose last bit is
// implementation-defined (glibc, the device's ocml and PCL's build may differ by an ulp); the
// restatement pins ONE fixed-order routine, and the GPU path (lio_filter.hip) evaluates the same
// published algorithm, so undistorted points agree bit for bit.  tests/test_oracle.py checks it
// against numpy sin / cos (<= 1 ulp).  The published
// fdlibm algorithm: Cody-Waite reduction by pi/2 in three 33-bit parts (exact products for
// |n| < 2^20), then the __kernel_sin / __kernel_cos minimax polynomials on [-pi/4, pi/4]; < 1 ulp
// from the true value.  Arguments beyond 2^19 pi/2 do not occur (angular rate x dt of one sweep).
static inline double ksin_fixed(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if (std::fabs(x) < 7.450580596923828125e-09) return x;  // 2^-27
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
static inline double kcos_fixed(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double ax = std::fabs(x);
    if (ax < 7.450580596923828125e-09) return 1.0;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ax < 0.3) return 1.0 - (0.5 * z - z * r);
    double qx;
    if (ax > 0.78125) {
        qx = 0.28125;
    } else {  // |x| / 4 with the low word cleared
        const unsigned long long hi = (unsigned long long)dbits(ax) >> 32;
        qx = bitsd((hi - 0x00200000ull) << 32);
    }
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    return a - (hz - z * r);
}
// Measurement switch (orc_set_sincos_libm): UndistortPcl's Exp through the host libm std::sin / std::cos,
// as the reference's build calls them, instead of the pinned routine — to count how many undistorted
// points the choice changes.  Off by default; the GPU path evaluates sincos_fixed.
static bool g_sincos_libm = false;

void sincos_fixed(double x, double* s, double* c) {
    if (g_sincos_libm) {
        *s = std::sin(x);
        *c = std::cos(x);
        return;
    }
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_2 = 6.07710050630396597660e-11, pio2_3 = 2.02226624871116645580e-21;
    int n = 0;
    double r = x;
    if (!(std::fabs(x) <= 7.85398163397448278999e-01)) {  // pi/4
        const double fn = std::nearbyint(x * invpio2);
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

// FAST-LIO so3_math.h Exp(ang_vel, dt) [U] (sin / cos: sincos_fixed above)
static void so3_exp(const double w[3], double dt, double E[9]) {
    const double nrm = std::sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    for (int k = 0; k < 9; ++k) E[k] = (k % 4 == 0) ? 1.0 : 0.0;
    if (!(nrm > 0.0000001)) return;
    const double r[3] = {w[0] / nrm, w[1] / nrm, w[2] / nrm};
    const double K[9] = {0.0, -r[2], r[1], r[2], 0.0, -r[0], -r[1], r[0], 0.0};
    double sn, co;
    sincos_fixed(nrm * dt, &sn, &co);
    const double c1 = 1.0 - co;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            // ((1 - cos) K) * K: Eigen's coefficient-based 3x3 product sums e0 + (e1 + e2)
            // (redux_novec_unroller halves the 3 terms 1 + 2)
            const double kk = (c1 * K[3 * i + 0]) * K[0 + j] + ((c1 * K[3 * i + 1]) * K[3 + j] + (c1 * K[3 * i + 2]) * K[6 + j]);
            E[3 * i + j] = (E[3 * i + j] + sn * K[3 * i + j]) + kk;
        }
}

// UndistortPcl's backward loop over a time-sorted cloud [U], literally: the
// point iterator walks back through the IMU segments; at the first point the
// inner loop `break`s without stepping, so every later (earlier-in-time)
// segment whose head is older than that point compensates it again — a quirk
// of the reference kept here (it only bites when the earliest point lies past
// the first IMU sample).
static void compensate(float* q, int tf, const ImuPoseO& hd, const ImuPoseO& tl, const Pose& end) {
    const double dt = (double)q[tf] / double(1000) - hd.offset_time;
    double E[9], Ri[9];
    so3_exp(tl.gyr, dt, E);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            Ri[3 * r + c] = hd.rot[3 * r] * E[c] + (hd.rot[3 * r + 1] * E[3 + c] + hd.rot[3 * r + 2] * E[6 + c]);  // M3D*M3D
    double Tei[3];
    for (int k = 0; k < 3; ++k) Tei[k] = ((hd.pos[k] + hd.vel[k] * dt) + ((0.5 * tl.acc[k]) * dt) * dt) - end.t[k];
    // P_compensate = offset_R_L_I.conjugate() * (rot.conjugate() * (R_i * (offset_R_L_I * P_i +
    //                offset_T_L_I) + T_ei) - offset_T_L_I)   (quaternion products as Eigen evaluates them)
    const double Pi[3] = {q[0], q[1], q[2]};
    double a[3], b[3], c[3];
    quat_rotate(end.qLI, false, Pi, a);
    for (int r = 0; r < 3; ++r) a[r] = a[r] + end.tLI[r];
    // R_i * (...) + T_ei: M3D * V3D, Eigen's coefficient-based product e0 + (e1 + e2)
    for (int r = 0; r < 3; ++r) b[r] = (Ri[3 * r] * a[0] + (Ri[3 * r + 1] * a[1] + Ri[3 * r + 2] * a[2])) + Tei[r];
    quat_rotate(end.q, true, b, c);
    for (int r = 0; r < 3; ++r) c[r] = c[r] - end.tLI[r];
    quat_rotate(end.qLI, true, c, a);
    q[0] = (float)a[0];
    q[1] = (float)a[1];
    q[2] = (float)a[2];
}

static void undistort(float* p, int64_t n, int stride, int tf, const ImuPoseO* poses, int np, const Pose& end) {
    if (np < 2 || n == 0) return;
    int64_t it = n - 1;
    for (int kp = np - 1; kp >= 1; --kp) {
        const ImuPoseO& hd = poses[kp - 1];
        const ImuPoseO& tl = poses[kp];
        for (; (double)p[(size_t)it * stride + tf] / double(1000) > hd.offset_time; --it) {
            compensate(p + (size_t)it * stride, tf, hd, tl, end);
            if (it == 0) break;
        }
    }
}

static int64_t preprocess(const float* raw, int64_t n, int stride, int every, float blind, float leaf, int tf,
                          const ImuPoseO* poses, int np, const Pose& end, float* out) {
    std::vector<float> sel;
    sel.reserve((size_t)n * stride);
    if (every < 1) every = 1;
    for (int64_t i = 0; i < n; ++i) {
        const float* q = raw + (size_t)i * stride;
        if (i % every == 0 && (q[0] * q[0] + q[1] * q[1] + q[2] * q[2]) > blind * blind) sel.insert(sel.end(), q, q + stride);
    }
    const int64_t m = (int64_t)sel.size() / stride;
    std::vector<int64_t> order(m);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return sel[(size_t)a * stride + tf] < sel[(size_t)b * stride + tf];
    });
    std::vector<float> srt((size_t)m * stride);
    for (int64_t i = 0; i < m; ++i)
        std::memcpy(&srt[(size_t)i * stride], &sel[(size_t)order[i] * stride], stride * sizeof(float));
    undistort(srt.data(), m, stride, tf, poses, np, end);
    if (leaf > 0.f) {
        const float lf[3] = {leaf, leaf, leaf};
        return voxel_grid(srt.data(), m, stride, lf, out);
    }
    std::memcpy(out, srt.data(), srt.size() * sizeof(float));
    return m;
}

}  // namespace orc

// =============================================================================
// C ABI for ctypes (tests / bench cpu_baseline only)
// =============================================================================
extern "C" {

// sincos_fixed over an array (tests/test_oracle.py pins it against numpy within 1 ulp)
void orc_sincos(const double* a, int64_t n, double* s, double* c) {
    for (int64_t i = 0; i < n; ++i) orc::sincos_fixed(a[i], s + i, c + i);
}

struct orc_match_params { float knn_range_sq; float plane_thr; double s_coef; double s_gate; };
struct orc_state {
    double pos[3]; double rot[4]; double offset_R_L_I[4]; double offset_T_L_I[3];
    double vel[3]; double bg[3]; double ba[3]; double grav[3];
};
struct orc_icp_params {
    double max_corr_dist, trans_eps, fitness_eps;
    int max_iter;
    double rot_eps, score_threshold;
    int umeyama_float;  // as lio_icp_params: -1 double statistics, 0 the default (order 2), 1..5 UmeyamaOrder
};

int orc_version(void) { return 4; }

// UndistortPcl through libm sin / cos (1) or the pinned sincos_fixed (0, default); returns the old value
int orc_set_sincos_libm(int on) {
    const int old = orc::g_sincos_libm ? 1 : 0;
    orc::g_sincos_libm = on != 0;
    return old;
}

// pcl::umeyama in float over n correspondence pairs (xyz interleaved) in summation order `order`
// (UmeyamaOrder 1..5) -> the row-major 4x4 incremental transform
int orc_umeyama_float(const float* src, const float* tgt, int64_t n, int order, float* T16, float* stats15) {
    if (n < 1 || order < 1 || order > 5) return -1;
    std::vector<float> s(src, src + 3 * n), t(tgt, tgt + 3 * n);
    orc::umeyama_pcl_float(s, t, T16, order, stats15);
    return 0;
}

int64_t orc_eigen_gemm_kc(int64_t k, int64_t l1) { return orc::eigen_gemm_kc(k, l1); }

// ---- filters ----
int64_t orc_voxel_grid(const float* p, int64_t n, int stride, const float* leaf3, float* out) {
    if (stride < 3 || stride > 16) return -1;
    return orc::voxel_grid(p, n, stride, leaf3, out);
}
int64_t orc_submap_voxelize(const float* p, const int64_t* seg, int nseg, int stride, const double* T16,
                            float voxel_res, float* out) {
    if (stride < 3 || stride > 16) return -1;
    const int64_t n = nseg > 0 ? seg[nseg] : 0;
    std::vector<float> tf((size_t)n * stride);
    orc::transform_segments(p, n, stride, seg, nseg, T16, tf.data());
    const float leaf[3] = {voxel_res, voxel_res, voxel_res};
    return orc::voxel_grid(tf.data(), n, stride, leaf, out);
}
int64_t orc_preprocess(const float* raw, int64_t n, int stride, int every, float blind, float leaf, int tf,
                       const double* poses, int np, const double* end24, float* out) {
    orc::Pose e;
    std::memcpy(&e, end24, sizeof(e)); orc::pose_fill_quat(e);
    return orc::preprocess(raw, n, stride, every, blind, leaf, tf, (const orc::ImuPoseO*)poses, np, e, out);
}


// ---- incremental map (DynMap) ----
void* orc_dmap_create(const float* xyz, int64_t n) {
    auto* d = new orc::DynMap();
    d->xyz.assign(xyz, xyz + 3 * n);
    d->alive.assign((size_t)n, 1);
    return d;
}
void orc_dmap_free(void* m) { delete (orc::DynMap*)m; }
int64_t orc_dmap_num_ids(void* m) { return ((orc::DynMap*)m)->n_ids(); }
int64_t orc_dmap_alive_count(void* m) { return ((orc::DynMap*)m)->alive_count(); }
int orc_dmap_get(void* m, float* xyz, uint8_t* alive) {
    auto* d = (orc::DynMap*)m;
    if (xyz) std::memcpy(xyz, d->xyz.data(), d->xyz.size() * sizeof(float));
    if (alive) std::memcpy(alive, d->alive.data(), d->alive.size());
    return 0;
}
int64_t orc_dmap_add(void* m, const float* xyz, int64_t n, int downsample, float ds) {
    return ((orc::DynMap*)m)->add_points(xyz, n, downsample != 0, ds);
}
int64_t orc_dmap_delete_boxes(void* m, const float* boxes, int nb) {
    return ((orc::DynMap*)m)->delete_boxes(boxes, nb);
}
// the DynMap's kd-tree over its alive ids (refreshed): usable wherever an orc_map_build handle is
// (orc_h_share_model, orc_ieskf_update), with the map's own ids.  Owned by the DynMap.
void* orc_dmap_tree(void* m) {
    auto* d = (orc::DynMap*)m;
    d->refresh();
    return &d->tree;
}
int orc_dmap_knn(void* m, const float* q, int64_t nq, int k, float range_sq, int32_t* idx, float* d2) {
    if (k < 1 || k > 8) return -1;
    auto* d = (orc::DynMap*)m;
    d->refresh();
    for (int64_t i = 0; i < nq; ++i) d->tree.knn(q + 3 * i, k, range_sq, idx + (size_t)k * i, d2 + (size_t)k * i);
    return 0;
}
int orc_map_incremental(void* m, const float* body, int64_t n, const double* pose_knn24, const double* pose24,
                        double fs, float ds, int64_t* stats4) {
    orc::Pose pk, pf;
    std::memcpy(&pk, pose_knn24, sizeof(pk)); orc::pose_fill_quat(pk);
    std::memcpy(&pf, pose24, sizeof(pf)); orc::pose_fill_quat(pf);
    orc::map_incremental(*(orc::DynMap*)m, body, n, pk, pf, fs, ds, stats4);
    return 0;
}


void* orc_map_build(const float* xyz, int64_t n) {
    auto* t = new orc::KdTree();
    t->build(xyz, n);
    return t;
}
void orc_map_free(void* m) { delete (orc::KdTree*)m; }

int orc_map_knn(void* m, const float* q, int64_t nq, int k, float range_sq, int32_t* idx, float* d2, int threads) {
    if (k < 1 || k > 8) return -1;
    auto* t = (orc::KdTree*)m;
#pragma omp parallel for schedule(dynamic, 512) num_threads(threads)
    for (int64_t i = 0; i < nq; ++i) t->knn(q + 3 * i, k, range_sq, idx + (size_t)k * i, d2 + (size_t)k * i);
    return 0;
}

int orc_esti_plane(const float* pts15, float thr, float* out4) {
    float P[5][3];
    for (int j = 0; j < 5; ++j)
        for (int d = 0; d < 3; ++d) P[j][d] = pts15[3 * j + d];
    return orc::esti_plane(out4, P, thr) ? 1 : 0;
}

int orc_body_to_world(const double* pose24, const float* body, int64_t n, float* world) {
    orc::Pose ps;
    std::memcpy(&ps, pose24, sizeof(ps));
    orc::pose_fill_quat(ps);
    for (int64_t i = 0; i < n; ++i) orc::body_to_world(ps, body + 3 * i, world + 3 * i);
    return 0;
}

int orc_h_share_model(void* m, const float* body, int64_t n, const double* pose24, int redo_knn,
                      int32_t* nn_idx, uint8_t* sel, float* planes, const orc_match_params* mp,
                      double* sums32, int threads) {
    orc::Pose ps;
    std::memcpy(&ps, pose24, sizeof(ps));
    orc::pose_fill_quat(ps);
    orc::MatchParams p{mp->knn_range_sq, mp->plane_thr, mp->s_coef, mp->s_gate};
    return orc::h_share_model(*(orc::KdTree*)m, body, n, ps, redo_knn, nn_idx, sel, planes, p, sums32, threads, nullptr);
}

static void to_state(const orc_state* s, orc::State& x) {
    std::memcpy(x.pos, s->pos, sizeof(x.pos));
    x.rot = {s->rot[0], s->rot[1], s->rot[2], s->rot[3]};
    x.offR = {s->offset_R_L_I[0], s->offset_R_L_I[1], s->offset_R_L_I[2], s->offset_R_L_I[3]};
    std::memcpy(x.offT, s->offset_T_L_I, sizeof(x.offT));
    std::memcpy(x.vel, s->vel, sizeof(x.vel));
    std::memcpy(x.bg, s->bg, sizeof(x.bg));
    std::memcpy(x.ba, s->ba, sizeof(x.ba));
    std::memcpy(x.grav, s->grav, sizeof(x.grav));
}
static void from_state(const orc::State& x, orc_state* s) {
    std::memcpy(s->pos, x.pos, sizeof(x.pos));
    s->rot[0] = x.rot.w; s->rot[1] = x.rot.x; s->rot[2] = x.rot.y; s->rot[3] = x.rot.z;
    s->offset_R_L_I[0] = x.offR.w; s->offset_R_L_I[1] = x.offR.x; s->offset_R_L_I[2] = x.offR.y; s->offset_R_L_I[3] = x.offR.z;
    std::memcpy(s->offset_T_L_I, x.offT, sizeof(x.offT));
    std::memcpy(s->vel, x.vel, sizeof(x.vel));
    std::memcpy(s->bg, x.bg, sizeof(x.bg));
    std::memcpy(s->ba, x.ba, sizeof(x.ba));
    std::memcpy(s->grav, x.grav, sizeof(x.grav));
}

// stats_out: [iterations, knn_calls, converged, last_neff, last_res_sum]
int orc_ieskf_update(void* m, const float* body, int64_t n, orc_state* state, double* P529,
                     const orc_match_params* mp, double R, int max_iter, double limit, int threads,
                     double* stats_out, double* trace, orc_state* knn_state_out) {
    orc::State x;
    to_state(state, x);
    std::vector<double> P(P529, P529 + 529);
    orc::MatchParams p{mp->knn_range_sq, mp->plane_thr, mp->s_coef, mp->s_gate};
    orc::IeskfStats st{};
    orc::State xk = x;
    int rc = orc::ieskf_update(*(orc::KdTree*)m, body, n, x, P, p, R, max_iter, limit, threads, &st, trace, &xk);
    from_state(x, state);
    if (knn_state_out) from_state(xk, knn_state_out);
    std::memcpy(P529, P.data(), sizeof(double) * 529);
    if (stats_out) {
        stats_out[0] = st.iterations;
        stats_out[1] = st.knn_calls;
        stats_out[2] = st.converged;
        stats_out[3] = st.last_neff;
        stats_out[4] = st.last_res_sum;
    }
    return rc;
}

// out8: [fitness, converged, iterations, state, ...]; trace: 20 doubles / iteration
int orc_icp_align(const float* src, int64_t ns, const float* dst, int64_t nd, const orc_icp_params* ipp,
                  const float* guess16, float* T16, double* out8, float* aligned, double* trace,
                  int max_trace, int threads) {
    // the GPU's sentinels (include/lio_gpu.h): -1 = double statistics, 0 = the default float order 2
    const int mode = ipp->umeyama_float < 0 ? 0 : (ipp->umeyama_float == 0 ? 2 : ipp->umeyama_float);
    orc::IcpParams ip{ipp->max_corr_dist, ipp->trans_eps, ipp->fitness_eps, ipp->max_iter, ipp->rot_eps,
                      ipp->score_threshold, mode};
    orc::IcpResult r{};
    static const float kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    int rc = orc::icp_align(src, ns, dst, nd, ip, guess16 ? guess16 : kIdentity, &r, aligned, trace, max_trace,
                            threads);  // no guess = identity, as pcl::Registration::align(output)
    std::memcpy(T16, r.T, sizeof(r.T));
    out8[0] = r.fitness;
    out8[1] = r.converged;
    out8[2] = r.iterations;
    out8[3] = r.state;
    out8[4] = (r.converged && r.fitness < ip.score_threshold) ? 1.0 : 0.0;  // is_valid_
    return rc;
}

}  // extern "C"
