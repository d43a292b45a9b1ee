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

// Device-writable host words (ABI 13): the pair-capacity guard writes each render's pair total into one of them
// (gstex_scan_offsets_guarded), the host reads it after the stream has passed the scan -- no copy, no sync.
extern "C" int gstex_host_words_alloc(int32_t n, int32_t** host, int32_t** device) {
    if (n <= 0 || !host || !device) {
        gstex::set_error("gstex_host_words_alloc: invalid arguments");
        return GSTEX_ERR_INVALID_ARG;
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, (size_t)n * sizeof(int32_t), hipHostMallocMapped) != hipSuccess || !p) {
        gstex::set_error("gstex_host_words_alloc: hipHostMalloc failed");
        return GSTEX_ERR_LAUNCH;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
        (void)hipHostFree(p);
        gstex::set_error("gstex_host_words_alloc: hipHostGetDevicePointer failed");
        return GSTEX_ERR_LAUNCH;
    }
    for (int32_t i = 0; i < n; ++i) static_cast<int32_t*>(p)[i] = 0;
    *host = static_cast<int32_t*>(p);
    *device = static_cast<int32_t*>(d);
    return GSTEX_OK;
}

extern "C" int gstex_host_words_free(int32_t* host) {
    if (host && hipHostFree(host) != hipSuccess) {
        gstex::set_error("gstex_host_words_free: hipHostFree failed");
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}

// Lightweight events (ABI 14, see gstex_hip.h)
extern "C" int gstex_event_create(int32_t kind, void** event) {
    if (!event || (kind != GSTEX_EVENT_TIMING && kind != GSTEX_EVENT_ORDER)) {
        gstex::set_error("gstex_event_create: invalid arguments (kind %d)", kind);
        return GSTEX_ERR_INVALID_ARG;
    }
    const unsigned flags = kind == GSTEX_EVENT_TIMING ? hipEventDisableSystemFence
                                                      : (hipEventDisableTiming | hipEventReleaseToDevice);
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess) {
        gstex::set_error("gstex_event_create: hipEventCreateWithFlags failed");
        return GSTEX_ERR_LAUNCH;
    }
    *event = (void*)e;
    return GSTEX_OK;
}

extern "C" int gstex_event_record(void* event, void* stream) {
    if (!event || hipEventRecord((hipEvent_t)event, gstex::as_stream(stream)) != hipSuccess) {
        gstex::set_error("gstex_event_record: hipEventRecord failed");
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}

extern "C" int gstex_event_elapsed(void* start, void* end, float* ms) {
    if (!start || !end || !ms || hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end) != hipSuccess) {
        gstex::set_error("gstex_event_elapsed: hipEventElapsedTime failed (timing events, recorded and complete?)");
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}

extern "C" int gstex_stream_wait_event(void* stream, void* event) {
    if (!event || hipStreamWaitEvent(gstex::as_stream(stream), (hipEvent_t)event, 0) != hipSuccess) {
        gstex::set_error("gstex_stream_wait_event: hipStreamWaitEvent failed");
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}

extern "C" int gstex_event_destroy(void* event) {
    if (event && hipEventDestroy((hipEvent_t)event) != hipSuccess) {
        gstex::set_error("gstex_event_destroy: hipEventDestroy failed");
        return GSTEX_ERR_LAUNCH;
    }
    return GSTEX_OK;
}
