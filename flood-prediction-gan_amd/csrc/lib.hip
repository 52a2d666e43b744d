// Library plumbing: error reporting, version, device check.
#include <string.h>
#include <string>

#include "fg_common.hpp"

namespace {
thread_local char g_err[1024] = "";
thread_local const char* g_last = "";
}

namespace fg {

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code == 0 ? FG_ERR_INVALID : code;
}

int launched(const char* what) {
    g_last = what;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail((int)e, "%s: launch failed: %s", what, hipGetErrorString(e));
    return 0;
}

int num_cus() {
    // compute units of the current device (cached per device; 256 on MI355X)
    static thread_local int cached_dev = -1, cached_cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return cached_cus;
    if (dev != cached_dev) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            cached_cus = cus;
        cached_dev = dev;
    }
    return cached_cus;
}

thread_local hipEvent_t g_arm_start = nullptr, g_arm_stop = nullptr;

}  // namespace fg

FG_API const char* fg_last_error(void) { return g_err; }

FG_API const char* fg_last_launch(void) { return g_last; }

FG_API int fg_version(void) { return 1; }

FG_API int fg_device_ok(void) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fg::fail((int)e, "hipGetDevice: %s", hipGetErrorString(e));
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return fg::fail((int)e, "hipGetDeviceProperties: %s", hipGetErrorString(e));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fg::fail(FG_ERR_INVALID, "device %d is %s, this build targets gfx950 only", dev, prop.gcnArchName);
    return 0;
}

// Timing events for the bench's live per-kernel measurement (KernelTimer).  mode 0: hipEventDefault, the
// system-scope release torch.cuda.Event records with; 1: hipEventReleaseToDevice; 2: hipEventDisableSystemFence.
// Modes 1 and 2 skip the L2 writeback + invalidate the default record performs, which at a kernel boundary of the
// step costs ~6 us each (profiles/round6/r6k_*).
FG_API int fg_timing_event_create(int mode, void** ev) {
    if (!ev || mode < 0 || mode > 2) return fg::fail(FG_ERR_INVALID, "fg_timing_event_create: mode %d", mode);
    const unsigned flags = mode == 1 ? hipEventReleaseToDevice : mode == 2 ? hipEventDisableSystemFence : hipEventDefault;
    hipEvent_t e = nullptr;
    const hipError_t rc = hipEventCreateWithFlags(&e, flags);
    if (rc != hipSuccess) return fg::fail((int)rc, "hipEventCreateWithFlags(%#x): %s", flags, hipGetErrorString(rc));
    *ev = (void*)e;
    return 0;
}

FG_API int fg_timing_event_record(void* ev, hipStream_t stream) {
    const hipError_t rc = hipEventRecord((hipEvent_t)ev, stream);
    return rc == hipSuccess ? 0 : fg::fail((int)rc, "hipEventRecord: %s", hipGetErrorString(rc));
}

// Waits for `end`, then *ms = the time between the two records.
FG_API int fg_timing_event_elapsed(void* start, void* end, float* ms) {
    hipError_t rc = hipEventSynchronize((hipEvent_t)end);
    if (rc == hipSuccess) rc = hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end);
    return rc == hipSuccess ? 0 : fg::fail((int)rc, "hipEventElapsedTime: %s", hipGetErrorString(rc));
}

// Arms the calling thread's next convolution kernel launch (FG_LAUNCH) with `start` / `stop`; they then carry that
// kernel's dispatch timestamps.
FG_API int fg_timing_arm(void* start, void* stop) {
    if (!start || !stop) return fg::fail(FG_ERR_INVALID, "fg_timing_arm: null event");
    fg::g_arm_start = (hipEvent_t)start;
    fg::g_arm_stop = (hipEvent_t)stop;
    return 0;
}

// Clears the arm; returns 1 if it was still pending (no FG_LAUNCH consumed it), else 0.
FG_API int fg_timing_disarm(void) {
    const int pending = fg::g_arm_start != nullptr;
    fg::g_arm_start = fg::g_arm_stop = nullptr;
    return pending;
}

FG_API int fg_timing_event_destroy(void* ev) {
    const hipError_t rc = hipEventDestroy((hipEvent_t)ev);
    return rc == hipSuccess ? 0 : fg::fail((int)rc, "hipEventDestroy: %s", hipGetErrorString(rc));
}
