// The loop leg as the fast_lio_sam node runs it: one lio_gpu::LoopClosure handle, a
// growing keyframe database, and per call loopTimerFunc's timed region (fast_lio_sam.cpp:682-728: t1 before
// fetchClosestKeyframeIdx, t2 after performLoopClosure), so submaps of a different size on every call.
//
//   loop_sequence <input.bin>
//
// Input (written by lio_gpu.pipeline.write_loop_sequence): "LIOLS001", int32 keyframes, per keyframe int64 n,
// n x (x, y, z, intensity) float, the pose_corrected_eig_ (16 doubles, row-major), the timestamp (double);
// then int32 calls, per call the index k of the newest keyframe (keyframes_ = keyframes[0 .. k]).
// Output: one line per call ("call k ms closest n_src n_dst iterations valid score T0..T15 allocs") and a
// JSON summary line; allocs = lio_alloc_count() growth across the call (device / pinned allocations).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    const size_t i = std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5));
    return v[i];
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: loop_sequence <input.bin>\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", argv[1]);
        return 2;
    }
    try {
        Reader r{f};
        char magic[8];
        r.get(magic, 8);
        if (std::string(magic, 8) != "LIOLS001") throw std::runtime_error("bad magic");
        const int nkf = r.get<int32_t>();
        std::vector<lio_gpu::PosePcd> all((size_t)nkf);
        for (int k = 0; k < nkf; ++k) {
            const int64_t n = r.get<int64_t>();
            all[(size_t)k].pcd_.resize((size_t)n);
            r.get(reinterpret_cast<float*>(all[(size_t)k].pcd_.data()), (size_t)n * 4);
            r.get(all[(size_t)k].pose_corrected_eig_, 16);
            std::copy(all[(size_t)k].pose_corrected_eig_, all[(size_t)k].pose_corrected_eig_ + 16, all[(size_t)k].pose_eig_);
            all[(size_t)k].timestamp_ = r.get<double>();
            all[(size_t)k].idx_ = k;
        }
        const int ncalls = r.get<int32_t>();
        std::vector<int> calls((size_t)ncalls);
        r.get(calls.data(), (size_t)ncalls);
        std::fclose(f);
        f = nullptr;

        using clk = std::chrono::steady_clock;
        lio_gpu::LoopClosure lc(lio_gpu::LoopClosureConfig{});  // the node's one loop_closure_ (PCL float order 2)
        // node start-up: LOOP_SEQ_PREWARM=0 leaves the first call to pay the set-up (buffers, code objects)
        double prewarm_ms = 0.0;
        const char* pw = std::getenv("LOOP_SEQ_PREWARM");
        if (!pw || std::string(pw) != "0") {
            const auto p0 = std::chrono::steady_clock::now();
            lc.prewarm();
            prewarm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
        }
        std::vector<double> ms;
        std::vector<long long> allocs;
        for (int c = 0; c < ncalls; ++c) {
            const int k = calls[(size_t)c];
            // keyframes_ as the node holds it when keyframe k is the newest
            const std::vector<lio_gpu::PosePcd> keyframes(all.begin(), all.begin() + k + 1);
            const auto& latest = keyframes.back();
            const int64_t a0 = lio_alloc_count();
            // loopTimerFunc's timed region; performLoopClosure's body (loop_closure.cpp:95-126) spelled out so
            // its two stages are timed too: setSrcAndDstCloud (GPU submaps) and icpAlignment
            const auto t1 = clk::now();
            const int closest = lc.fetchClosestKeyframeIdx(latest, keyframes);
            lio_gpu::RegistrationOutput reg;
            size_t ns = 0, nd = 0;
            auto ta = t1, tb = t1;
            if (closest >= 0) {
                ta = clk::now();
                const auto sd = lc.setSrcAndDstCloud(keyframes, latest.idx_, closest, lc.config().num_submap_keyframes_,
                                                     lc.config().voxel_res_);
                tb = clk::now();
                reg = lc.icpAlignment(sd.first, sd.second);
                ns = sd.first.size();
                nd = sd.second.size();
            }
            const auto t2 = clk::now();
            const int64_t a1 = lio_alloc_count();
            auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            const double t = msd(t1, t2);
            ms.push_back(t);
            allocs.push_back((long long)(a1 - a0));
            const lio_icp_result& last = lc.last_result();
            std::printf("call %d %.4f %d %zu %zu %d %d %.9g", k, t, closest, ns, nd, closest >= 0 ? last.iterations : 0,
                        reg.is_valid_ ? 1 : 0, closest >= 0 ? last.score : -1.0);
            for (int j = 0; j < 16; ++j) std::printf(" %.9g", closest >= 0 ? (double)last.T[j] : 0.0);
            std::printf(" %lld %.4f %.4f\n", (long long)(a1 - a0), msd(ta, tb), msd(tb, t2));
        }
        std::vector<double> warm(ms.begin() + (ms.size() > 1 ? 1 : 0), ms.end());
        long long warm_allocs = 0;
        for (size_t c = 1; c < allocs.size(); ++c) warm_allocs += allocs[c];
        std::printf("{\"calls\": %d, \"prewarm_ms\": %.4f, \"first_ms\": %.4f, \"warm_p50_ms\": %.4f, \"warm_p99_ms\": %.4f, "
                    "\"warm_max_ms\": %.4f, \"first_call_allocs\": %lld, \"warm_allocs\": %lld}\n",
                    ncalls, prewarm_ms, ms.empty() ? 0.0 : ms[0], warm.empty() ? 0.0 : pct(warm, 0.5),
                    warm.empty() ? 0.0 : pct(warm, 0.99), warm.empty() ? 0.0 : *std::max_element(warm.begin(), warm.end()),
                    allocs.empty() ? 0LL : allocs[0], warm_allocs);
    } catch (const std::exception& e) {
        if (f) std::fclose(f);
        std::fprintf(stderr, "loop_sequence: %s\n", e.what());
        return 1;
    }
    return 0;
}
