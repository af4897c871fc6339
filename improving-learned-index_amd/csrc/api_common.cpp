// api_common.cpp -- process-wide C-ABI entry points (errors, version, devices).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "di_common.h"

namespace di {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

const char *last_error() { return g_err.c_str(); }

// compute units of the current device (persistent-kernel grid sizes)
int n_cu() {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    return v > 0 ? v : 256;
}

}  // namespace di

extern "C" {

const char *di_last_error(void) { return di::last_error(); }

int di_version(void) { return (0 << 16) | 1; }

int di_device_count(int *n) {
    return di::guard([&] {
        DI_REQUIRE(n, DI_EINVAL, "null argument");
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        *n = (e == hipSuccess) ? c : 0;
    });
}

}  // extern "C"
