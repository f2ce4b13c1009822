// trace.hpp — opt-in host-side trace of the multi-device group's frame and teardown steps (RRAY_TRACE_FILE=<path>):
// one line per step, appended and flushed at once, so a process that hangs or is killed mid-call still leaves the
// last step it reached on disk (pytest's output capture would lose stderr).  Off unless the variable is set.
#pragma once
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace rr {
inline void trace(const char* fmt, ...) {
    static std::mutex mu;
    static FILE* f = nullptr;
    static bool tried = false;
    std::lock_guard<std::mutex> lock(mu);
    if (!tried) {
        tried = true;
        if (const char* p = std::getenv("RRAY_TRACE_FILE")) f = std::fopen(p, "a");
    }
    if (!f) return;
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(f, "%.6f ", t);
    va_list ap;
    va_start(ap, fmt);
    std::vfprintf(f, fmt, ap);
    va_end(ap);
    std::fputc('\n', f);
    std::fflush(f);
}
}  // namespace rr
