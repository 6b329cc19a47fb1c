// lio_error.hpp — thread-local last-error text shared by every C-ABI entry point.
#pragma once
#include <string>

namespace lio {
inline std::string& last_error() {
    thread_local std::string s;
    return s;
}
}  // namespace lio
