// The C5 stream driven from C++ through include/lio_gpu.hpp: raw sweeps ->
// FastLioSamStream (preprocess -> IESKF update -> map_incremental -> keyframe) -> the loop leg on the newest
// keyframe (fetchClosestKeyframeIdx -> setSrcAndDstCloud -> icpAlignment), fast_lio_sam.cpp:367-573,682-730.
//
//   c5_stream <input.bin> <output.bin>
//
// The input (written by tests/test_cpp_stream.py / bench.py from lio_gpu.synth) holds the map, the raw sweeps
// with their IMU poses, scan-end poses, initial states and timestamps, P0 and the submap range; the output
// every sweep's state, IESKF counts, sizes, stage times, keyframe cloud and pose, then the loop result and the
// two submaps — the test checks them against the oracle.  One JSON line on stdout: the stage-time medians.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "lio_gpu.hpp"

namespace {

struct Reader {
    FILE* f;
    template <typename T>
    T get() {
        T v;
        if (std::fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("input truncated");
        return v;
    }
    template <typename T>
    void get(T* p, size_t n) {
        if (n && std::fread(p, sizeof(T), n, f) != n) throw std::runtime_error("input truncated");
    }
};

struct Writer {
    FILE* f;
    template <typename T>
    void put(const T& v) {
        std::fwrite(&v, sizeof(T), 1, f);
    }
    template <typename T>
    void put(const T* p, size_t n) {
        if (n) std::fwrite(p, sizeof(T), n, f);
    }
};

struct Sweep {
    std::vector<float> raw;
    int64_t n = 0;
    int stride = 0;
    std::vector<lio_imu_pose> imu;
    lio_pose end{};
    lio_state init{};
    double t = 0;
};

struct Pxyz {
    float x, y, z;
};

double median(std::vector<double> v) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    const size_t h = v.size() / 2;
    return v.size() % 2 ? v[h] : 0.5 * (v[h - 1] + v[h]);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <input.bin> <output.bin>\n", argv[0]);
        return 2;
    }
    try {
        FILE* fi = std::fopen(argv[1], "rb");
        if (!fi) throw std::runtime_error("cannot open the input");
        Reader in{fi};
        char magic[8];
        in.get(magic, 8);
        if (std::memcmp(magic, "LIOC5IN1", 8) != 0) throw std::runtime_error("bad input magic");
        const int64_t n_map = in.get<int64_t>();
        std::vector<Pxyz> map((size_t)n_map);
        in.get(reinterpret_cast<float*>(map.data()), (size_t)n_map * 3);
        const int n_sweeps = in.get<int32_t>();
        std::vector<Sweep> sweeps((size_t)n_sweeps);
        for (Sweep& s : sweeps) {
            s.n = in.get<int64_t>();
            s.stride = in.get<int32_t>();
            s.raw.resize((size_t)s.n * s.stride);
            in.get(s.raw.data(), s.raw.size());
            s.imu.resize((size_t)in.get<int32_t>());
            in.get(s.imu.data(), s.imu.size());
            in.get(&s.end, 1);
            in.get(&s.init, 1);
            s.t = in.get<double>();
        }
        std::vector<double> P0(23 * 23);
        in.get(P0.data(), P0.size());
        const int submap_range = in.get<int32_t>();
        std::fclose(fi);

        lio_gpu::KdTreeGPU<Pxyz> tree(1.0f, 0.5f, 0);
        tree.Build(map);
        lio_gpu::FastLioSamStream stream(tree, lio_gpu::LoopClosureConfig{});
        std::vector<lio_gpu::SweepResult> res;
        for (const Sweep& s : sweeps)
            res.push_back(stream.process(s.raw.data(), s.n, s.stride, s.imu, s.end, s.init, P0.data(), s.t));
        using clk = std::chrono::steady_clock;
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        lio_gpu::RegistrationOutput reg;
        const auto tl0 = clk::now();
        const int idx = stream.loop(&reg, submap_range);
        const double loop_ms = ms(tl0, clk::now());
        lio_gpu::LoopClosure& lc = stream.loop_closure();
        const lio_icp_result last = lc.last_result();
        // the loop leg's two stages timed separately (median of 5), as bench.py times the Python stream
        std::vector<double> t_sub, t_icp;
        if (idx >= 0)
            for (int r = 0; r < 5; ++r) {
                const auto a = clk::now();
                auto sd = lc.setSrcAndDstCloud(stream.keyframes(), stream.keyframes().back().idx_, idx, submap_range,
                                               lc.config().voxel_res_);
                const auto b = clk::now();
                (void)lc.icpAlignment(sd.first, sd.second);
                const auto c = clk::now();
                t_sub.push_back(ms(a, b));
                t_icp.push_back(ms(b, c));
            }

        FILE* fo = std::fopen(argv[2], "wb");
        if (!fo) throw std::runtime_error("cannot open the output");
        Writer out{fo};
        out.put("LIOC5OU1", 8);
        out.put<int32_t>(n_sweeps);
        for (int k = 0; k < n_sweeps; ++k) {
            const lio_gpu::SweepResult& r = res[(size_t)k];
            const lio_gpu::PosePcd& kf = stream.keyframes()[(size_t)k];
            out.put(r.x);
            const int32_t cnt[4] = {r.stats.h_evals, r.stats.knn_calls, r.stats.converged, r.stats.n_eff};
            out.put(cnt, 4);
            out.put<int64_t>(r.n_down);
            out.put<int64_t>(r.n_undistorted);
            const double t4[4] = {r.ms_preprocess, r.ms_update, r.ms_map_incremental, r.ms_keyframe};
            out.put(t4, 4);
            out.put(kf.pose_eig_, 16);
            out.put<int64_t>((int64_t)kf.pcd_.size());
            out.put(reinterpret_cast<const float*>(kf.pcd_.data()), kf.pcd_.size() * 4);
        }
        out.put<int32_t>(idx);
        out.put<int32_t>(reg.is_valid_ ? 1 : 0);
        out.put(reg.score_);
        out.put(last.T, 16);
        out.put<int32_t>(last.iterations);
        out.put<int32_t>(last.state);
        for (const auto* c : {&lc.getSourceCloud(), &lc.getTargetCloud()}) {
            out.put<int64_t>((int64_t)c->size());
            out.put(reinterpret_cast<const float*>(c->data()), c->size() * 4);
        }
        std::fclose(fo);

        // stage medians over the sweeps after the first (the first allocates the stream's buffers)
        std::vector<double> pre, upd, mapi, kfm, tot;
        for (size_t k = res.size() > 1 ? 1 : 0; k < res.size(); ++k) {
            const auto& r = res[k];
            pre.push_back(r.ms_preprocess);
            upd.push_back(r.ms_update);
            mapi.push_back(r.ms_map_incremental);
            kfm.push_back(r.ms_keyframe);
            tot.push_back(r.ms_preprocess + r.ms_update + r.ms_map_incremental + r.ms_keyframe);
        }
        std::printf("{\"sweeps\": %d, \"ms_per_sweep_median\": %.4f, \"stage_ms_median\": {\"preprocess\": %.4f, "
                    "\"update\": %.4f, \"map_incremental\": %.4f, \"keyframe\": %.4f}, \"loop\": {\"closest_idx\": %d, "
                    "\"is_valid\": %s, \"iterations\": %d, \"ms\": %.4f, \"submaps_ms\": %.4f, \"icp_ms\": %.4f}}\n",
                    n_sweeps, median(tot), median(pre), median(upd), median(mapi), median(kfm), idx,
                    reg.is_valid_ ? "true" : "false", last.iterations, loop_ms, median(t_sub), median(t_icp));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "c5_stream: %s\n", e.what());
        return 1;
    }
    return 0;
}
