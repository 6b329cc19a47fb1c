// HostPool (fast-lio-sam_gps_amd/csrc/lio_pool.hpp): every index of every job runs exactly once, with one
// caller and with three callers at once; built by tests/test_host_pool.py (also under ThreadSanitizer).
#include "lio_pool.hpp"
#include <cstdio>
#include <vector>
#include <atomic>
#include <chrono>
int main() {
    auto& P = lio::HostPool::get();
    int bad = 0;
    for (int it = 0; it < 20000; ++it) {
        const int n = 1 + it % 9;
        std::vector<std::atomic<int>> hit(n);
        for (auto& h : hit) h = 0;
        P.parallel_for(n, [&](int i) { hit[i]++; });
        for (int i = 0; i < n; ++i) if (hit[i] != 1) ++bad;
    }
    // concurrent callers
    std::vector<std::thread> th;
    std::atomic<int> bad2{0};
    for (int t = 0; t < 3; ++t) th.emplace_back([&] {
        for (int it = 0; it < 3000; ++it) { std::vector<std::atomic<int>> hit(4); for (auto& h : hit) h = 0;
            P.parallel_for(4, [&](int i) { hit[i]++; }); for (auto& h : hit) if (h != 1) bad2++; } });
    for (auto& t : th) t.join();
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < 1000; ++it) P.parallel_for(4, [&](int) {});
    auto t1 = std::chrono::steady_clock::now();
    printf("bad %d bad2 %d  empty job %.1f us\n", bad, (int)bad2, std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    return (bad || bad2) ? 1 : 0;
}
