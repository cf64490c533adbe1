// What a resident batch server would save over a launch per solve: B
// one-wave workgroups (the one-wave batch kernel's shape), each doing `work` dependent VALU steps,
// then the in-launch reduction's two-level counter tree (256 shard counters, a top counter; the last
// arrival publishes a tagged word to host-mapped memory), timed host-side per request:
//   launch  -- one kernel launch per request (what mgdp_vi_solve does for a resident batch today);
//   server  -- one persistent launch: lane 0 of workgroup 0 polls the host's request word and
//              forwards it to a device word that every workgroup polls (s_sleep between polls).
// Every wait is bounded (s_memrealtime idle limits), so the grid always drains.
// Build: hipcc -O2 --offload-arch=gfx950 -o tools/probe_batch_server tools/probe_batch_server.cpp
// Run:   tools/probe_batch_server [B] [work] [requests] [sleep: 2 / 10 / 40, 0 = lane 0 polls without
//        s_sleep, -1 = every lane polls without s_sleep]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;
constexpr int kShards = 256;
constexpr int kLine = 16;  // u64 words per 128-B line
constexpr u64 kQuit = ~0ull;
// tree layout (u64 words): [kShards counter lines][top line][kShards shard values][B grid values]
__host__ __device__ inline int top_off() { return kShards * kLine; }
__host__ __device__ inline int shard_val_off() { return top_off() + kLine; }
__host__ __device__ inline int grid_val_off() { return shard_val_off() + kShards; }

__device__ __forceinline__ u64 wave_max_u64(u64 v) {
    for (int o = 32; o > 0; o >>= 1) {
        const u64 w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// the in-launch reduction of vi_loops.h's gk_exit, one value (max) per grid
__device__ void tree_exit(u64 *tree, int e, int B, u64 val, u64 *res, u64 epoch) {
    const int lane = threadIdx.x & 63;
    const int nsh = B < kShards ? B : kShards;
    const int s = e % nsh;
    const int size = B / nsh + (s < B % nsh ? 1 : 0);
    u64 t = 0;
    if (lane == 0) {
        __hip_atomic_store(tree + grid_val_off() + e, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t = __hip_atomic_fetch_add(tree + s * kLine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    t = __shfl(t, 0);
    if (t != (u64)(size - 1)) return;
    u64 m = 0;
    for (int i = lane; i < size; i += 64) {
        const u64 x = __hip_atomic_load(tree + grid_val_off() + s + i * nsh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = x > m ? x : m;
    }
    m = wave_max_u64(m);
    u64 t2 = 0;
    if (lane == 0) {
        __hip_atomic_exchange(tree + s * kLine, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(tree + shard_val_off() + s, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t2 = __hip_atomic_fetch_add(tree + top_off(), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    t2 = __shfl(t2, 0);
    if (t2 != (u64)(nsh - 1)) return;
    m = 0;
    for (int i = lane; i < nsh; i += 64) {
        const u64 x = __hip_atomic_load(tree + shard_val_off() + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = x > m ? x : m;
    }
    m = wave_max_u64(m);
    if (lane == 0) {
        __hip_atomic_exchange(tree + top_off(), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(res, (epoch << 32) | (m & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__device__ __forceinline__ u64 do_work(int e, int work) {
    float x = (float)(e & 1023);
    for (int i = 0; i < work; ++i) x = x * 1.0000001f + 1e-7f;
    return (u64)(e % 997) + (x > 1e30f ? 1ull : 0ull);
}

__global__ void __launch_bounds__(64) once(int B, int work, u64 *tree, u64 *res, u64 epoch) {
    tree_exit(tree, blockIdx.x, B, do_work(blockIdx.x, work), res, epoch);
}

__global__ void __launch_bounds__(64) server(int B, int work, u64 *tree, const u64 *req, u64 *res, u64 *dflag,
                                             int sleep, u64 idle) {
    const int e = blockIdx.x, lane = threadIdx.x;
    u64 t_last = __builtin_amdgcn_s_memrealtime();
    u64 epoch = 0;
    while (true) {
        const u64 want = epoch + 1;
        if (e == 0 && lane == 0) {  // the poller: host word -> device word
            while (true) {
                const u64 r = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (r >= want) {
                    __hip_atomic_store(dflag, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t_last > idle) {
                    __hip_atomic_store(dflag, kQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        u64 f = 0;
        if (sleep < 0) {  // variant: every lane polls (no divergent loop), no s_sleep
            while (true) {
                f = __hip_atomic_load(dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                f = __builtin_amdgcn_readfirstlane((unsigned)(f >> 32)) == (unsigned)(f >> 32) ? f : f;
                if (f >= want) break;
                if (__builtin_amdgcn_s_memrealtime() - t_last > 2 * idle) {
                    f = kQuit;
                    break;
                }
            }
        } else if (lane == 0) {
            while (true) {
                f = __hip_atomic_load(dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (f >= want) break;
                if (__builtin_amdgcn_s_memrealtime() - t_last > 2 * idle) {
                    f = kQuit;
                    break;
                }
                if (sleep >= 40) __builtin_amdgcn_s_sleep(40);
                else if (sleep >= 10) __builtin_amdgcn_s_sleep(10);
                else if (sleep >= 1) __builtin_amdgcn_s_sleep(2);
            }
        }
        f = __shfl(f, 0);
        if (f == kQuit) return;
        epoch = f;
        tree_exit(tree, e, B, do_work(e, work), res, epoch);
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

static bool wait_res(volatile u64 *res, u64 epoch, double *us, std::chrono::steady_clock::time_point a) {
    while ((*res >> 32) != epoch) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count() > 1.0) return false;
    }
    *us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    return true;
}

static void report(const char *tag, int B, int work, int sleep, std::vector<double> &t) {
    std::sort(t.begin(), t.end());
    const size_t n = t.size();
    std::printf("{\"tag\": \"%s\", \"B\": %d, \"work\": %d, \"sleep\": %d, \"n\": %zu, \"median_us\": %.3f, "
                "\"p10_us\": %.3f, \"p90_us\": %.3f}\n",
                tag, B, work, sleep, n, t[n / 2], t[n / 10], t[n * 9 / 10]);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    int B = argc > 1 ? std::atoi(argv[1]) : 8192;
    const int work = argc > 2 ? std::atoi(argv[2]) : 0;
    const int n = argc > 3 ? std::atoi(argv[3]) : 500;
    const int sleep = argc > 4 ? std::atoi(argv[4]) : 10;
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, server, 64, 0);
    if (B > per_cu * cus) {
        std::printf("{\"error\": \"B %d above the resident capacity %d\"}\n", B, per_cu * cus);
        return 1;
    }
    u64 *h, *d_h, *tree, *dflag;
    if (hipHostMalloc((void **)&h, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 2;
    if (hipHostGetDevicePointer((void **)&d_h, h, 0) != hipSuccess) return 2;
    const size_t words = (size_t)grid_val_off() + B;
    if (hipMalloc((void **)&tree, words * 8) != hipSuccess || hipMalloc((void **)&dflag, 64) != hipSuccess) return 2;
    (void)hipMemset(tree, 0, words * 8);
    (void)hipMemset(dflag, 0, 64);
    (void)hipDeviceSynchronize();
    volatile u64 *req = h, *res = h + 8;
    *req = 0;
    *res = 0;
    std::vector<double> t;
    // launch per request
    for (int i = 1; i <= n + 20; ++i) {
        auto a = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(once, dim3(B), dim3(64), 0, 0, B, work, tree, d_h + 8, (u64)i);
        double us;
        if (!wait_res(res, (u64)i, &us, a)) {
            std::printf("{\"tag\": \"launch\", \"error\": \"timeout at %d\"}\n", i);
            (void)hipDeviceSynchronize();
            return 3;
        }
        if (i > 20) t.push_back(us);
    }
    (void)hipDeviceSynchronize();
    report("launch", B, work, sleep, t);
    // persistent server (its own epochs from 1)
    (void)hipMemset(dflag, 0, 64);
    (void)hipDeviceSynchronize();
    *req = 0;
    *res = 0;
    t.clear();
    hipLaunchKernelGGL(server, dim3(B), dim3(64), 0, 0, B, work, tree, d_h, d_h + 8, dflag, sleep, 20000000ull);
    bool ok = true;
    for (int i = 1; i <= n + 20 && ok; ++i) {
        auto a = std::chrono::steady_clock::now();
        __atomic_store_n((u64 *)req, (u64)i, __ATOMIC_RELEASE);
        double us;
        if (!wait_res(res, (u64)i, &us, a)) {
            std::printf("{\"tag\": \"server\", \"error\": \"timeout at %d\"}\n", i);
            ok = false;
        } else if (i > 20) {
            t.push_back(us);
        }
    }
    __atomic_store_n((u64 *)req, kQuit, __ATOMIC_RELEASE);  // the poller forwards it; every wave leaves
    (void)hipDeviceSynchronize();
    if (ok) report("server", B, work, sleep, t);
    (void)hipFree(tree);
    (void)hipFree(dflag);
    (void)hipHostFree(h);
    return ok ? 0 : 4;
}
