// Host-only pieces of the C++ C5 stream (include/lio_gpu.hpp), no GPU call: odom_matrix (pose_pcd.hpp's tf
// formula), inverse4 (pose_eig_.inverse()), fetch_closest_keyframe_idx (loop_closure.cpp:18-40).  Prints
// the values for tests/test_cpp_stream.py to compare with the Python glue (lio_gpu.pipeline).
#include <cstdio>
#include <vector>

#include "lio_gpu.hpp"

int main() {
    lio_state x{};
    const double q[4] = {0.9238795325112867, 0.0123, -0.0456, 0.3826834323650898};  // (w, x, y, z), not unit
    for (int k = 0; k < 4; ++k) x.rot[k] = q[k];
    x.pos[0] = 12.5, x.pos[1] = -3.25, x.pos[2] = 0.75;
    double T[16], I[16];
    lio_gpu::odom_matrix(x, T);
    lio_gpu::inverse4(T, I);
    for (int k = 0; k < 16; ++k) std::printf("T %d %.17g\n", k, T[k]);
    for (int k = 0; k < 16; ++k) std::printf("I %d %.17g\n", k, I[k]);
    // keyframes along a loop: out along +x, back 40 s later
    lio_gpu::LoopClosureConfig cfg;
    std::vector<lio_gpu::PosePcd> kfs(8);
    for (int k = 0; k < 8; ++k) {
        const double px = k < 4 ? 3.7 * k : 3.7 * (7 - k) + 1.5;
        kfs[k].pose_corrected_eig_[3] = px;
        kfs[k].pose_corrected_eig_[7] = k < 4 ? 0.0 : -0.3;
        kfs[k].timestamp_ = k < 4 ? 0.1 * k : 40.0 + 0.1 * (k - 4);
        kfs[k].idx_ = k;
    }
    std::printf("closest %d\n", lio_gpu::fetch_closest_keyframe_idx(cfg, kfs.back(), kfs));
    std::vector<lio_gpu::PosePcd> early(kfs.begin(), kfs.begin() + 4);  // no keyframe 30 s older
    std::printf("closest_early %d\n", lio_gpu::fetch_closest_keyframe_idx(cfg, early.back(), early));
    return 0;
}
