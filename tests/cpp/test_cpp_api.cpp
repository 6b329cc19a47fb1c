// C++ drop-in surface (include/lio_gpu.hpp) exercised the way laserMapping.cpp
// and LoopClosure use the reference classes.  Checks, on one GPU:
//   * KdTreeGPU::Nearest_Search (batch and single point) against a brute-force
//     (sq-distance, id) scan — bit-exact ids and distances — before and after
//     Add_Points / Delete_Point_Boxes;
//   * ScanMatcherGPU::update_iterated_dyn_share_modified recovers a known pose
//     offset of a scan of a planar scene; map_incremental grows the map;
//   * LoopClosureICP::icpAlignment converges on a displaced copy.
// Built by tests/test_cpp_api.py with g++ -ffp-contract=off (same float
// operation order as the device distances).  Prints "ALL OK" on success.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "lio_gpu.hpp"

struct PointXYZI {  // pcl::PointXYZI's fields
    float x, y, z, intensity;
};
using PointVector = std::vector<PointXYZI>;

static int g_fail = 0;
#define EXPECT(cond, ...)                          \
    do {                                           \
        if (!(cond)) {                             \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);              \
            std::printf("\n");                     \
            ++g_fail;                              \
        }                                          \
    } while (0)

static float sqdist(const PointXYZI& a, const float* b) {
    const float dx = a.x - b[0], dy = a.y - b[1], dz = a.z - b[2];
    return (dx * dx + dy * dy) + dz * dz;
}

// k nearest alive points in (d2, id) order within d2 <= bound
static void brute_knn(const std::vector<float>& xyz, const std::vector<uint8_t>& alive, const PointXYZI& q, int k,
                      float bound, std::vector<int32_t>& ids, std::vector<float>& d2) {
    std::vector<std::pair<float, int32_t>> c;
    for (size_t i = 0; i < alive.size(); ++i) {
        if (!alive[i]) continue;
        const float d = sqdist(q, &xyz[3 * i]);
        if (d <= bound) c.emplace_back(d, (int32_t)i);
    }
    const size_t m = std::min<size_t>((size_t)k, c.size());
    std::partial_sort(c.begin(), c.begin() + m, c.end());
    ids.assign((size_t)k, -1);
    d2.assign((size_t)k, INFINITY);
    for (size_t j = 0; j < m; ++j) {
        ids[j] = c[j].second;
        d2[j] = c[j].first;
    }
}

// walls of a street canyon + ground + a few boxes: enough planes to constrain 6 DoF
static PointVector make_scene(int n, std::mt19937& rng) {
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    PointVector pts;
    pts.reserve(n);
    for (int i = 0; i < n; ++i) {
        PointXYZI p{0, 0, 0, 1};
        const int s = i % 6;
        const float a = 20.f * u(rng), b = 4.f * u(rng) + 4.f;
        if (s == 0) p = {a, 6.f, b, 1};                                   // left wall
        else if (s == 1) p = {a, -6.f, b, 1};                             // right wall
        else if (s == 2) p = {a, 6.f * u(rng), 0.f, 1};                   // ground
        else if (s == 3) p = {8.f, 2.f * u(rng) + 3.f, 1.5f * u(rng) + 1.5f, 1};  // box face x
        else if (s == 4) p = {2.f * u(rng) - 5.f, -3.f, 1.5f * u(rng) + 1.5f, 1}; // box face y
        else p = {2.f * u(rng) - 5.f, 1.f * u(rng) - 2.f, 3.f, 1};       // box top
        pts.push_back(p);
    }
    return pts;
}

static void check_knn(lio_gpu::KdTreeGPU<PointXYZI>& tree, const PointVector& q, int k, double max_dist) {
    std::vector<int32_t> ids;
    std::vector<float> d2;
    tree.Nearest_Search_Batch(q, k, ids, d2, max_dist);
    std::vector<float> xyz;
    std::vector<uint8_t> alive;
    tree.by_id(xyz, alive);
    const float bound = std::isinf(max_dist) ? INFINITY : (float)(max_dist * max_dist);
    int bad = 0;
    for (size_t i = 0; i < q.size(); ++i) {
        std::vector<int32_t> bi;
        std::vector<float> bd;
        brute_knn(xyz, alive, q[i], k, bound, bi, bd);
        for (int j = 0; j < k; ++j)
            if (bi[j] != ids[i * k + j] || !(bd[j] == d2[i * k + j] || (std::isinf(bd[j]) && std::isinf(d2[i * k + j]))))
                ++bad;
    }
    EXPECT(bad == 0, "Nearest_Search k=%d max_dist=%g: %d mismatches", k, max_dist, bad);
}

// pcl::VoxelGrid (PCL 1.10 applyFilter) restated on the host: voxel index from floor(p / leaf)
// relative to the min voxel, stable order inside a voxel, fields summed in input order (float)
static PointVector brute_voxel(const PointVector& in, float leaf) {
    const float inv = 1.0f / leaf;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const auto& p : in) {
        const float v[3] = {p.x, p.y, p.z};
        for (int d = 0; d < 3; ++d) lo[d] = std::min(lo[d], v[d]), hi[d] = std::max(hi[d], v[d]);
    }
    long long mn[3], dv[3];
    for (int d = 0; d < 3; ++d) {
        mn[d] = (long long)std::floor(lo[d] * inv);
        dv[d] = (long long)std::floor(hi[d] * inv) - mn[d] + 1;
    }
    std::vector<std::pair<long long, size_t>> key;
    for (size_t i = 0; i < in.size(); ++i) {
        const float v[3] = {in[i].x, in[i].y, in[i].z};
        long long ijk[3];
        for (int d = 0; d < 3; ++d) ijk[d] = (long long)(std::floor(v[d] * inv) - (float)mn[d]);
        key.emplace_back(ijk[0] + ijk[1] * dv[0] + ijk[2] * dv[0] * dv[1], i);
    }
    std::stable_sort(key.begin(), key.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    PointVector out;
    for (size_t j = 0; j < key.size();) {
        size_t e = j;
        PointXYZI acc{0, 0, 0, 0};
        while (e < key.size() && key[e].first == key[j].first) {
            const PointXYZI& q = in[key[e].second];
            acc.x += q.x, acc.y += q.y, acc.z += q.z, acc.intensity += q.intensity;
            ++e;
        }
        const float c = (float)(e - j);
        out.push_back({acc.x / c, acc.y / c, acc.z / c, acc.intensity / c});
        j = e;
    }
    return out;
}

static bool same_cloud(const PointVector& a, const PointVector& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i].x != b[i].x || a[i].y != b[i].y || a[i].z != b[i].z || a[i].intensity != b[i].intensity) return false;
    return true;
}

int main() {
    if (lio_device_count() < 1) {
        std::printf("no GPU\n");
        return 2;
    }
    std::mt19937 rng(7);
    const PointVector map_pts = make_scene(60000, rng);

    // ---------------------------------------------------------------- ikd-Tree surface
    lio_gpu::KdTreeGPU<PointXYZI> tree(1.0f, 0.5f);
    tree.set_downsample_param(0.5f);
    tree.Build(map_pts);
    EXPECT(tree.size() == (int)map_pts.size() && tree.validnum() == (int)map_pts.size(), "Build size");
    std::uniform_real_distribution<float> uq(-25.f, 25.f);
    PointVector q(800);
    for (auto& p : q) p = {uq(rng), 0.3f * uq(rng), 0.2f * uq(rng) + 3.f, 0};
    for (int k : {1, 5}) {
        check_knn(tree, q, k, INFINITY);
        check_knn(tree, q, k, std::sqrt(5.0));
    }
    // single point, as h_share_model calls it
    {
        PointVector near;
        std::vector<float> dist;
        tree.Nearest_Search(q[0], 5, near, dist);
        std::vector<float> xyz;
        std::vector<uint8_t> alive;
        tree.by_id(xyz, alive);
        std::vector<int32_t> bi;
        std::vector<float> bd;
        brute_knn(xyz, alive, q[0], 5, INFINITY, bi, bd);
        bool same = near.size() == 5 && dist.size() == 5;
        for (size_t j = 0; same && j < 5; ++j)
            same = near[j].x == xyz[3 * bi[j]] && near[j].y == xyz[3 * bi[j] + 1] && near[j].z == xyz[3 * bi[j] + 2] &&
                   dist[j] == bd[j];
        EXPECT(same, "single-point Nearest_Search");
    }
    // Add_Points (no downsample) + Delete_Point_Boxes, then kNN again
    {
        PointVector extra = make_scene(5000, rng);
        for (auto& p : extra) p.x += 0.05f;
        EXPECT(tree.Add_Points(extra, false) == (int)extra.size(), "Add_Points count");
        std::vector<lio_gpu::BoxPointType> boxes(1);
        boxes[0] = {{-30.f, -10.f, -1.f}, {0.f, 0.f, 10.f}};
        const int del = tree.Delete_Point_Boxes(boxes);
        EXPECT(del > 0 && tree.validnum() == tree.size() - del, "Delete_Point_Boxes");
        check_knn(tree, q, 5, INFINITY);
        PointVector flat;
        tree.flatten(flat);
        EXPECT((int)flat.size() == tree.validnum(), "flatten");
    }

    // ------------------------------------------------ matcher built before set_downsample_param
    // (laserMapping may configure the tree after the objects that use it exist): the parameters
    // change in place, the matcher keeps a valid map, and the tree refuses to die under it
    {
        lio_gpu::KdTreeGPU<PointXYZI> early(1.0f, 0.5f);
        lio_gpu::ScanMatcherGPU m0(early);
        early.set_downsample_param(0.3f);
        early.Build(map_pts);
        m0.set_scan(PointVector(q.begin(), q.begin() + 200));
        lio_state x{};
        x.rot[0] = 1.0;
        x.offset_R_L_I[0] = 1.0;
        std::vector<double> P(23 * 23, 0.0);
        for (int i = 0; i < 23; ++i) P[i * 23 + i] = 1e-4;
        const lio_ieskf_stats st = m0.update_iterated_dyn_share_modified(x, P.data(), 0.001, 3, 0.001);
        EXPECT(st.h_evals >= 1, "matcher built before set_downsample_param still runs");
        bool refused = false;
        try {
            early.set_downsample_param(0.5f);  // map now holds points
        } catch (const lio_gpu::Error&) {
            refused = true;
        }
        EXPECT(refused, "set_downsample_param after Build refused");
        lio_map_params pp{0.f, 0.5f, 0, 0};
        EXPECT(lio_map_destroy(early.handle()) == LIO_ERR_STATE, "map destroy refused while a matcher exists");
        (void)pp;
    }

    // ------------------------------------------------------------- scan matching
    {
        lio_gpu::KdTreeGPU<PointXYZI> map(1.0f, 0.5f);
        map.Build(map_pts);
        lio_gpu::ScanMatcherGPU matcher(map);
        // body-frame scan: a subset of the scene seen from the true pose (yaw 2 deg, t = (0.3, -0.2, 0.05))
        const double yaw = 2.0 * M_PI / 180.0, c = std::cos(yaw), s = std::sin(yaw);
        const double t[3] = {0.3, -0.2, 0.05};
        std::mt19937 r2(11);
        PointVector world = make_scene(8000, r2), body;
        for (const auto& w : world) {
            const double dx = w.x - t[0], dy = w.y - t[1], dz = w.z - t[2];  // R^T (w - t)
            body.push_back({(float)(c * dx + s * dy), (float)(-s * dx + c * dy), (float)dz, w.intensity});
        }
        matcher.set_scan(body);
        lio_state x{};
        x.rot[0] = 1.0;
        x.offset_R_L_I[0] = 1.0;
        x.grav[2] = -9.809;
        std::vector<double> P(23 * 23, 0.0);
        for (int i = 0; i < 23; ++i) P[i * 23 + i] = i < 6 ? 1e-2 : 1e-4;
        double err = 1e9;
        for (int it = 0; it < 4 && err > 0.01; ++it) {  // successive scans from the same place
            const lio_ieskf_stats st = matcher.update_iterated_dyn_share_modified(x, P.data(), 0.001, 3, 0.001);
            EXPECT(st.n_eff > 1000, "n_eff %d", st.n_eff);
            err = std::sqrt((x.pos[0] - t[0]) * (x.pos[0] - t[0]) + (x.pos[1] - t[1]) * (x.pos[1] - t[1]) +
                            (x.pos[2] - t[2]) * (x.pos[2] - t[2]));
        }
        const double yaw_est = 2.0 * std::atan2(x.rot[3], x.rot[0]);
        EXPECT(err < 0.01 && std::fabs(yaw_est - yaw) < 1e-3, "IESKF pose error %.4f m, yaw %.5f vs %.5f", err, yaw_est,
               yaw);
        const int before = map.size();
        const lio_incremental_stats inc = matcher.map_incremental(x, 0.5);
        EXPECT(map.size() > before, "map_incremental grew the map: %d -> %d", before, map.size());
        EXPECT(inc.n_to_add + inc.n_no_downsample + inc.n_skipped == (int64_t)body.size(), "map_incremental classes");
        lio_gpu::LocalMap lm;
        const double pos_lid[3] = {x.pos[0], x.pos[1], x.pos[2]};
        const auto boxes = lm.segment(pos_lid, 1000.0, 300.f, 1.5f);
        EXPECT(boxes.empty() && lm.state().initialized, "lasermap_fov_segment first call");
    }

    // ---------------------------------------------------------------- filters / formats
    {
        lio_gpu::FilterGPU filt;
        std::mt19937 r4(3);
        PointVector cloud = make_scene(30000, r4);
        std::uniform_real_distribution<float> ui(0.f, 255.f);
        for (auto& p : cloud) p.intensity = ui(r4);
        lio_gpu::VoxelGrid<PointXYZI> vg(filt);
        vg.setLeafSize(0.5f, 0.5f, 0.5f);
        vg.setInputCloud(&cloud);
        PointVector down;
        vg.filter(down);
        EXPECT(same_cloud(down, brute_voxel(cloud, 0.5f)), "VoxelGrid bit-exact (%zu points)", down.size());
        // setSrcAndDstCloud side: two keyframes through transformPcd (double 4x4) + voxelizePcd
        const double T0[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        const double c = std::cos(0.3), s = std::sin(0.3);
        const double T1[16] = {c, -s, 0, 2.5, s, c, 0, -1.0, 0, 0, 1, 0.2, 0, 0, 0, 1};
        PointVector half(cloud.begin(), cloud.begin() + 15000), rest(cloud.begin() + 15000, cloud.end());
        const PointVector sub = lio_gpu::submap_voxelize<PointXYZI>(filt, {&half, &rest}, {T0, T1}, 0.3f);
        PointVector tf = half;
        for (const auto& p : rest) {
            const double x = p.x, y = p.y, z = p.z;
            tf.push_back({(float)(((T1[0] * x + T1[1] * y) + T1[2] * z) + T1[3]),
                          (float)(((T1[4] * x + T1[5] * y) + T1[6] * z) + T1[7]),
                          (float)(((T1[8] * x + T1[9] * y) + T1[10] * z) + T1[11]), p.intensity});
        }
        EXPECT(same_cloud(sub, brute_voxel(tf, 0.3f)), "submap_voxelize bit-exact");
        // PCD round trip
        const std::string path = "/tmp/lio_cpp_api_test.pcd";
        lio_gpu::savePCDFileBinary(path, down, {"x", "y", "z", "intensity"});
        const PointVector back = lio_gpu::loadPCDFile<PointXYZI>(filt, path, {"x", "y", "z", "intensity"});
        EXPECT(same_cloud(back, down), "PCD binary round trip");
        std::remove(path.c_str());
    }

    // ---------------------------------------------------------------- loop ICP
    {
        std::mt19937 r3(5);
        const PointVector src = make_scene(40000, r3);
        PointVector dst;
        const double a = 1.0 * M_PI / 180.0, c = std::cos(a), s = std::sin(a);
        for (const auto& p : src)
            dst.push_back({(float)(c * p.x - s * p.y + 0.05), (float)(s * p.x + c * p.y - 0.03), p.z + 0.02f, p.intensity});
        lio_gpu::LoopClosureICP icp(lio_gpu::LoopClosureConfig{}, 0);
        const lio_gpu::RegistrationOutput r = icp.icpAlignment(src, dst);
        EXPECT(r.is_converged_ && r.is_valid_ && r.score_ < 0.05, "icpAlignment converged=%d score=%g", (int)r.is_converged_,
               r.score_);
        EXPECT(std::fabs(r.pose_between_eig_[3]) < 0.2 && std::fabs(r.pose_between_eig_[7]) < 0.2, "icp translation");
        // the same alignment served by a group of 3 ranks (all on device 0 here: host exchange; distinct
        // devices use RCCL) and by the one-shot icp_align: bit-identical transforms
        lio_gpu::LoopClosureICPGroup grp(lio_gpu::LoopClosureConfig{}, 3, {0, 0, 0});
        const lio_gpu::RegistrationOutput rg = grp.icpAlignment(src, dst);
        bool same = rg.is_valid_ == r.is_valid_ && grp.last().iterations == icp.last().iterations &&
                    grp.last().score == icp.last().score;
        for (int k = 0; k < 16; ++k) same = same && grp.last().T[k] == icp.last().T[k];
        EXPECT(same && !grp.uses_rccl(), "3-rank group bit-identical to one handle");
        std::vector<float> s3, d3;
        for (const auto& p : src) s3.insert(s3.end(), {p.x, p.y, p.z});
        for (const auto& p : dst) d3.insert(d3.end(), {p.x, p.y, p.z});
        lio_icp_params ip{52.5, 0.01, 0.01, 50, 0.0, 1.5, 1.0f, 0, 0};
        float T1[16];
        double fit = 0.0;
        int conv = 0, its = 0;
        EXPECT(icp_align(s3.data(), (int64_t)src.size(), d3.data(), (int64_t)dst.size(), &ip, 1, T1, &fit, &conv, &its,
                         nullptr) == LIO_OK,
               "icp_align n_gpus=1");
        bool same1 = its == icp.last().iterations && fit == icp.last().score;
        for (int k = 0; k < 16; ++k) same1 = same1 && T1[k] == icp.last().T[k];
        EXPECT(same1, "icp_align(n_gpus=1) bit-identical to lio_icp_align");
    }

    if (g_fail) {
        std::printf("%d FAILURES\n", g_fail);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
