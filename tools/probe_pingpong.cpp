// Host <-> GPU signalling latency, the lone-grid server's hand-off: a resident one-wave kernel polls
// a request word and answers in host-mapped memory; the host posts N requests back to back and
// reports the round trip.  Variant A: request word in host-mapped memory (the server's design);
// variant B: request word in fine-grained device memory written by the host through its mapping
// (only with an argument: on the MI355X box the reported host pointer segfaulted when written).
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/probe_pingpong tools/probe_pingpong.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void pong(const unsigned long long *req, unsigned long long *ans, int n, unsigned long long limit) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= n; ++i) {
        while (__hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (unsigned long long)i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > limit) return;  // bounded: never outlives 1 s
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(ans, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static void run(const char *tag, unsigned long long *h_req, unsigned long long *d_req) {
    unsigned long long *h_ans, *d_ans;
    if (hipHostMalloc((void **)&h_ans, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return;
    if (hipHostGetDevicePointer((void **)&d_ans, h_ans, 0) != hipSuccess) return;
    std::fprintf(stderr, "%s: ans %p/%p req %p/%p\n", tag, (void *)h_ans, (void *)d_ans, (void *)h_req, (void *)d_req);
    *h_ans = 0;
    std::fprintf(stderr, "ans written\n");
    *(volatile unsigned long long *)h_req = 0;
    std::fprintf(stderr, "req written\n");
    const int n = 20000;
    hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, d_req, d_ans, n, 100000000ull);
    std::fprintf(stderr, "launched: %s\n", hipGetErrorString(hipGetLastError()));
    std::vector<double> t(n);
    for (int i = 1; i <= n; ++i) {
        auto a = std::chrono::steady_clock::now();
        __atomic_store_n(h_req, (unsigned long long)i, __ATOMIC_RELEASE);
        while (__atomic_load_n(h_ans, __ATOMIC_ACQUIRE) != (unsigned long long)i) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count() > 0.5) {
                std::printf("{\"tag\": \"%s\", \"error\": \"timeout at %d\"}\n", tag, i);
                (void)hipDeviceSynchronize();
                return;
            }
        }
        t[i - 1] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    (void)hipDeviceSynchronize();
    std::sort(t.begin(), t.end());
    std::printf("{\"tag\": \"%s\", \"n\": %d, \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f}\n", tag, n, t[n / 2],
                t[n / 10], t[n * 9 / 10]);
    (void)hipHostFree(h_ans);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    unsigned long long *h_req, *d_req;
    if (hipHostMalloc((void **)&h_req, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
        hipHostGetDevicePointer((void **)&d_req, h_req, 0) == hipSuccess)
        run("host_mapped_request", h_req, d_req);
    if (argc < 2) return 0;  // device-memory variants: host writes through hostPointer segfaulted on the box
    unsigned long long *f = nullptr;
    if (hipExtMallocWithFlags((void **)&f, 64, hipDeviceMallocFinegrained) == hipSuccess) {
        hipPointerAttribute_t at{};
        const hipError_t e = hipPointerGetAttributes(&at, f);
        std::printf("{\"finegrained_device\": {\"attr_rc\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}}\n", (int)e,
                    at.hostPointer, at.devicePointer);
        if (e == hipSuccess && at.hostPointer) run("device_finegrained_request", (unsigned long long *)at.hostPointer, f);
    }
    unsigned long long *u = nullptr;
    if (hipExtMallocWithFlags((void **)&u, 64, hipDeviceMallocUncached) == hipSuccess) {
        hipPointerAttribute_t at{};
        const hipError_t e = hipPointerGetAttributes(&at, u);
        std::printf("{\"uncached_device\": {\"attr_rc\": %d, \"hostPointer\": \"%p\"}}\n", (int)e, at.hostPointer);
        if (e == hipSuccess && at.hostPointer) run("device_uncached_request", (unsigned long long *)at.hostPointer, u);
    }
    return 0;
}
