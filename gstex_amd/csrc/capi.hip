// capi.hip — error reporting and version entry points of the C-ABI.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "gstex_error.h"

namespace gstex {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}

}  // namespace gstex

extern "C" const char* gstex_last_error(void) { return gstex::g_last_error.c_str(); }

extern "C" int gstex_abi_version(void) { return GSTEX_ABI_VERSION; }
