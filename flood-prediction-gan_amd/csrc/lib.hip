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
