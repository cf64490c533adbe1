// common.h -- shared definitions of libmgdp (HIP, gfx950).  See include/mgdp.h for the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/mgdp.h"

namespace mgdp {

// OBJECT_TO_IDX, minigrid/core/constants.py:25-37
enum : int {
    T_UNSEEN = 0, T_EMPTY = 1, T_WALL = 2, T_FLOOR = 3, T_DOOR = 4, T_KEY = 5, T_BALL = 6,
    T_BOX = 7, T_GOAL = 8, T_LAVA = 9, T_AGENT = 10
};
enum : int { C_GREY = 5 };                               // COLOR_TO_IDX, constants.py:20
enum : int { D_OPEN = 0, D_CLOSED = 1, D_LOCKED = 2 };   // STATE_TO_IDX, constants.py:42-46

void set_error(const char *fmt, ...);

inline int hip_fail(hipError_t e, const char *what, const char *file, int line) {
    set_error("%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    return MGDP_E_HIP;
}

#define MGDP_HIP(call)                                                       \
    do {                                                                     \
        hipError_t _e = (call);                                              \
        if (_e != hipSuccess) return ::mgdp::hip_fail(_e, #call, __FILE__, __LINE__); \
    } while (0)

#define MGDP_CHECK(cond, code, ...)                                          \
    do {                                                                     \
        if (!(cond)) { ::mgdp::set_error(__VA_ARGS__); return (code); }      \
    } while (0)

// Sets the device for the calling thread and restores the previous one on scope exit.  A guard
// nested inside another guard of the same device on the same thread makes no runtime call at all
// (`active`): a batched solve crosses five guarded entry points (solve, reset, run_local, run_to,
// finish), and each hipGetDevice is a runtime call on the host's critical path of the solve loop.
struct DeviceGuard {
    static inline thread_local int active = -1;  // the device an enclosing guard holds current
    int prev = -1;
    int outer = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        outer = active;
        if (outer == dev) { ok = true; return; }
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == dev) {
            prev = -1;
            ok = true;
        } else {
            ok = hipSetDevice(dev) == hipSuccess;
        }
        if (ok) active = dev;
    }
    ~DeviceGuard() {
        if (outer == active) return;  // nested: nothing was changed
        if (prev >= 0) (void)hipSetDevice(prev);
        active = outer;
    }
};

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace mgdp
