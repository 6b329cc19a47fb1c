// lio_error.hpp — thread-local last-error text shared by every C-ABI entry point.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

namespace lio {
inline std::string& last_error() {
    thread_local std::string s;
    return s;
}
// device / pinned allocations made by the library's growth paths (the loop leg's: ICP, grids, filters, scan
// buffers) since the process started — lio_alloc_count(), which shows that a warm loop-closure sequence
// allocates nothing
inline std::atomic<int64_t>& alloc_counter() {
    static std::atomic<int64_t> n{0};
    return n;
}
inline void count_alloc(int k = 1) { alloc_counter().fetch_add(k, std::memory_order_relaxed); }
}  // namespace lio
