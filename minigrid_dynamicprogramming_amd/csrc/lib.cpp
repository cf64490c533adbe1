// lib.cpp -- library-level entry points of libmgdp (error state, version, device query).
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace mgdp {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace mgdp

extern "C" {

const char *mgdp_last_error(void) { return mgdp::g_err; }

static_assert(sizeof(mgdp_vi_desc) == 88, "mgdp_vi_desc layout is part of the ABI");
int mgdp_abi_version(void) { return MGDP_ABI_VERSION; }

int mgdp_device_count(int32_t *n) {
    MGDP_CHECK(n, MGDP_E_INVALID, "null argument");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return 0;
}

}  // extern "C"
