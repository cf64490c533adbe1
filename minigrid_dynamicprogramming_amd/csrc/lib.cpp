// lib.cpp -- library-level entry points of libmgdp (error state, version, device query, host
// thread placement).
#include <sched.h>

#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

// The calling thread onto the CPUs of the device's own NUMA node (sysfs local_cpulist of its PCI
// function), within the thread's current affinity.  A lone-grid solve is a request word written
// and a result word polled in host memory: measured on the MI355X box (2 sockets), the same solve
// takes 9.1 us from a CPU of the GPU's node and 10.8 us from the other node (tools/probe_numa.cpp).
int mgdp_pin_host_thread(int32_t device, int32_t *ncpus_out) {
    MGDP_CHECK(ncpus_out, MGDP_E_INVALID, "null argument");
    *ncpus_out = 0;
    char bus[64] = {0};
    MGDP_CHECK(hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) == hipSuccess, MGDP_E_INVALID,
               "no HIP device %d", (int)device);
    for (char *c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/local_cpulist", bus);
    FILE *f = std::fopen(path, "r");
    if (!f) return 0;  // no sysfs view of the device: leave the thread where it is
    char list[4096] = {0};
    const size_t len = std::fread(list, 1, sizeof list - 1, f);
    std::fclose(f);
    list[len] = 0;
    cpu_set_t allowed, want;
    CPU_ZERO(&want);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return 0;
    for (char *tok = std::strtok(list, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {  // "0-63,128-191"
        char *dash = std::strchr(tok, '-');
        const int lo = std::atoi(tok), hi = dash ? std::atoi(dash + 1) : lo;
        for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
    }
    const int n = CPU_COUNT(&want);
    if (n == 0 || sched_setaffinity(0, sizeof want, &want) != 0) return 0;
    *ncpus_out = n;
    return 0;
}

}  // extern "C"
