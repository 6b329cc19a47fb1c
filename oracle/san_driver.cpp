// san_driver.cpp — runs every oracle entry point once on small seeded inputs under
// AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle san`).  Test
// infrastructure only (see lio_oracle.cpp's header): it checks the checker for
// out-of-bounds reads, leaks and UB on the edge cases the parity tests feed it
// (empty and single-point maps, k = 1..8, empty ICP overlap, boxes deleting the
// whole map).  Built from the same translation unit, so no second copy of the
// algorithm exists.
#include "lio_oracle.cpp"

#include <cstdio>
#include <random>

namespace {

std::vector<float> cloud(std::mt19937& g, int n, float span) {
    std::uniform_real_distribution<float> u(-span, span);
    std::vector<float> p((size_t)3 * n);
    for (auto& v : p) v = u(g);
    for (int i = 0; i < n / 2; ++i) p[3 * i + 2] = 0.01f * u(g);  // half the points on a plane: planes pass
    return p;
}

// pose vector: R(9) t(3) R_LI(9) t_LI(3) q(4) q_LI(4); q = (w, x, y, z).  Odd calls leave the
// quaternions zero, so the oracle derives them from R (pose_fill_quat) under the sanitizers too.
void identity_pose(double* p32) {
    static int k = 0;
    std::memset(p32, 0, 32 * sizeof(double));
    p32[0] = p32[4] = p32[8] = 1.0;
    p32[12] = p32[16] = p32[20] = 1.0;
    if (k++ % 2 == 0) p32[24] = p32[28] = 1.0;
}

int fail(const char* what) {
    std::fprintf(stderr, "san_driver: %s failed\n", what);
    return 1;
}

}  // namespace

int main() {
    std::mt19937 g(7);
    const orc_match_params mp{5.0f, 0.1f, 0.9, 0.9};

    // static kd-tree: empty, single point, regular
    for (int n : {0, 1, 2000}) {
        auto m = cloud(g, n, 8.f);
        void* t = orc_map_build(m.data(), n);
        auto q = cloud(g, 300, 10.f);
        for (int k = 1; k <= 8; ++k) {
            std::vector<int32_t> idx((size_t)300 * k);
            std::vector<float> d2((size_t)300 * k);
            for (float r2 : {0.f, 1.f, INFINITY})
                if (orc_map_knn(t, q.data(), 300, k, r2, idx.data(), d2.data(), 2) != 0) return fail("knn");
        }
        // h-evaluation (kNN + plane) and one IESKF update
        double pose[32];
        identity_pose(pose);
        std::vector<int32_t> nn((size_t)300 * 5);
        std::vector<uint8_t> sel(300);
        std::vector<float> planes((size_t)300 * 4);
        double sums[32];
        for (int redo : {1, 0})
            if (orc_h_share_model(t, q.data(), 300, pose, redo, nn.data(), sel.data(), planes.data(), &mp, sums, 2) != 0)
                return fail("h_share_model");
        orc_state s{};
        s.rot[0] = s.offset_R_L_I[0] = 1.0;
        s.grav[2] = -9.809;
        std::vector<double> P(529, 0.0);
        for (int i = 0; i < 23; ++i) P[24 * i] = 1e-3;
        double stats[8], trace[64];
        orc_ieskf_update(t, q.data(), 300, &s, P.data(), &mp, 0.001, 3, 0.001, 2, stats, trace, nullptr);
        orc_map_free(t);
    }

    float pts15[15];
    for (int j = 0; j < 15; ++j) pts15[j] = (j % 3 == 2) ? 0.f : (float)(j % 5);
    float abcd[4];
    orc_esti_plane(pts15, 0.1f, abcd);

    // ICP: regular, disjoint (no correspondences), single target point
    {
        auto src = cloud(g, 1500, 5.f), dst = src;
        for (size_t i = 0; i < dst.size(); i += 3) dst[i] += 0.2f;
        orc_icp_params ip{52.5, 0.01, 0.01, 50, 0.0, 1.5, -1};  // the double statistics first
        float T[16];
        double out8[8], tr[20 * 64];
        std::vector<float> al(src.size());
        orc_icp_align(src.data(), 1500, dst.data(), 1500, &ip, nullptr, T, out8, al.data(), tr, 64, 2);
        auto far = dst;
        for (size_t i = 0; i < far.size(); i += 3) far[i] += 1000.f;
        orc_icp_align(src.data(), 1500, far.data(), 1500, &ip, nullptr, T, out8, nullptr, tr, 64, 2);
        orc_icp_align(src.data(), 1500, dst.data(), 1, &ip, nullptr, T, out8, nullptr, tr, 64, 2);
        ip.umeyama_float = 1;  // float pcl::umeyama + JacobiSVD restatement
        orc_icp_align(src.data(), 1500, dst.data(), 1500, &ip, nullptr, T, out8, al.data(), tr, 64, 2);
        orc_icp_align(src.data(), 1500, dst.data(), 1, &ip, nullptr, T, out8, nullptr, tr, 64, 2);
    }

    // filters: VoxelGrid at stride 4, submap voxelize over two segments
    {
        std::uniform_real_distribution<float> u(-20.f, 20.f);
        std::vector<float> p4((size_t)4 * 5000);
        for (auto& v : p4) v = u(g);
        std::vector<float> out(p4.size());
        const float leaf[3] = {0.5f, 0.5f, 0.5f};
        if (orc_voxel_grid(p4.data(), 5000, 4, leaf, out.data()) < 0) return fail("voxel_grid");
        const int64_t seg[3] = {0, 2000, 5000};
        double T2[32] = {};
        for (int k = 0; k < 2; ++k) T2[16 * k] = T2[16 * k + 5] = T2[16 * k + 10] = T2[16 * k + 15] = 1.0;
        if (orc_submap_voxelize(p4.data(), seg, 2, 4, T2, 0.3f, out.data()) < 0) return fail("submap_voxelize");
        // Preprocess + UndistortPcl + downSizeFilterSurf: stride 5 (x y z intensity time[ms]), 2 IMU poses
        std::vector<float> raw((size_t)5 * 3000);
        std::uniform_real_distribution<float> t01(0.f, 100.f);
        for (int i = 0; i < 3000; ++i) {
            for (int d = 0; d < 4; ++d) raw[5 * i + d] = u(g);
            raw[5 * i + 4] = t01(g);
        }
        double imu[2][22] = {};
        for (int k = 0; k < 2; ++k) {
            imu[k][0] = 0.05 * k;
            imu[k][13] = imu[k][17] = imu[k][21] = 1.0;  // rot = I
            imu[k][7] = 1.0;                             // vel x
        }
        double end24[32];
        identity_pose(end24);
        std::vector<float> pout(raw.size());
        if (orc_preprocess(raw.data(), 3000, 5, 4, 2.f, 0.5f, 4, &imu[0][0], 2, end24, pout.data()) < 0)
            return fail("preprocess");
    }

    // incremental map: add (downsampled and not), delete boxes (all), knn, map_incremental
    {
        auto m = cloud(g, 3000, 10.f);
        void* d = orc_dmap_create(m.data(), 3000);
        auto add = cloud(g, 1000, 12.f);
        orc_dmap_add(d, add.data(), 1000, 1, 0.5f);
        orc_dmap_add(d, add.data(), 1000, 0, 0.5f);
        auto q = cloud(g, 200, 12.f);
        std::vector<int32_t> idx(200 * 5);
        std::vector<float> d2(200 * 5);
        orc_dmap_knn(d, q.data(), 200, 5, 5.f, idx.data(), d2.data());
        const float box[6] = {-1.f, -1.f, -1.f, 1.f, 1.f, 1.f};
        orc_dmap_delete_boxes(d, box, 1);
        const float all[6] = {-100.f, -100.f, -100.f, 100.f, 100.f, 100.f};
        orc_dmap_delete_boxes(d, all, 1);
        orc_dmap_knn(d, q.data(), 200, 5, INFINITY, idx.data(), d2.data());
        double pose[32];
        identity_pose(pose);
        int64_t st4[4];
        orc_map_incremental(d, q.data(), 200, pose, pose, 0.5, 0.5f, st4);
        std::vector<float> xyz((size_t)3 * orc_dmap_num_ids(d));
        std::vector<uint8_t> alive((size_t)orc_dmap_num_ids(d));
        orc_dmap_get(d, xyz.data(), alive.data());
        orc_dmap_free(d);
    }
    std::printf("san_driver: ok\n");
    return 0;
}
