// ieskf.hpp — host-side iterated ESKF (IKFoM esekfom::update_iterated_dyn_share_modified
// [U]) driving the GPU measurement model.  Host C++, double precision, 23-dim.
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <vector>

namespace lio {
namespace host {

constexpr int N = 23;

struct Quat {
    double w, x, y, z;
};

struct State {
    double pos[3];
    Quat rot;
    Quat offR;
    double offT[3];
    double vel[3], bg[3], ba[3];
    double grav[3];
};

using Mat = std::vector<double>;  // row-major, sized by caller

// Result of one measurement evaluation (one lio_match call).
struct HModel {
    double sums[32];          // LIO_SUMS_* layout
    std::vector<double> rows; // 7 doubles per effective point, only when n_eff < N
};

// h_share_model callback: (state, redo_knn, want_rows, out) -> status
using HModelFn = std::function<int(const State&, bool, bool, HModel&)>;

struct IeskfResult {
    int h_evals = 0, knn_calls = 0, converged = 0, n_eff = 0;
    double res_mean = 0.0, solve_ms = 0.0;
};

int update_iterated(State& x, Mat& P, double R, int max_iter, double epsi, const HModelFn& h, IeskfResult& out);

void quat_to_mat(const Quat& q, double R[9]);

}  // namespace host
}  // namespace lio
