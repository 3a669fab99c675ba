// fls_common.hpp -- error reporting shared by the C-ABI entry points.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace fls {

// thread-local last error (fls_last_error)
std::string &last_error();

inline int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    last_error() = buf;
    return code;
}

inline bool debug_enabled() {
    // reference prints DEBUG traces when the DEBUG env var is set
    // (src/fastlanes_facade.cpp:28,36,43,50-54,62,75-78)
    static const bool on = std::getenv("DEBUG") != nullptr;
    return on;
}

}  // namespace fls
