// device_guard.hpp — the caller's current HIP device is restored when an ABI entry point returns.
// Entry points select their context's device(s) with hipSetDevice; without the guard a caller that
// shares the process (torch, another library) would silently continue on whichever device the
// library touched last.
#pragma once
#include <hip/hip_runtime.h>

namespace rr {

struct DeviceGuard {
    int prev = -1;
    DeviceGuard() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace rr
