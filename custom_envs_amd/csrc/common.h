// Shared host-side plumbing for the C ABI: thread-local error text and the
// HIP-call check used by every entry point (nothing throws across the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/custom_envs_amd.h"

namespace ce {

inline std::string &last_error() {
    static thread_local std::string msg;
    return msg;
}

inline int fail(int code, const std::string &msg) {
    last_error() = msg;
    return code;
}

inline size_t align16(size_t v) { return (v + 15) & ~static_cast<size_t>(15); }

}  // namespace ce

#define CE_HIP(call)                                                              \
    do {                                                                          \
        hipError_t err_ = (call);                                                 \
        if (err_ != hipSuccess)                                                   \
            return ce::fail(CE_EHIP, std::string(#call " failed: ") +             \
                                         hipGetErrorString(err_));                \
    } while (0)
