// gstex_error.h — status / last-error plumbing of the C-ABI (thread-local message, no globals
// shared across threads).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/gstex_hip.h"

namespace gstex {

void set_error(const char* fmt, ...);
int launch_status(const char* what);  // hipGetLastError() -> status + message

#define GSTEX_REQUIRE(cond, ...)                                \
    do {                                                        \
        if (!(cond)) {                                          \
            ::gstex::set_error(__VA_ARGS__);                    \
            return GSTEX_ERR_INVALID_ARG;                       \
        }                                                       \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace gstex
