// Read+write stream ceiling on this box, for the sweep kernel's HBM fraction:
// a 268 MB float4 array copied into another: the V bytes a sweep of Empty-16 x 65536 reads and writes.
// Variants: plain / nontemporal accesses, grid-stride with U float4 per thread in flight, grid size.
// Prints one JSON line per variant: median µs per copy over 20 launches and TB/s (read + write).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const float4 *__restrict__ src, float4 *__restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float *s = reinterpret_cast<const float *>(src + i + u * stride);
            if (NT) {
                v[u].x = __builtin_nontemporal_load(s);
                v[u].y = __builtin_nontemporal_load(s + 1);
                v[u].z = __builtin_nontemporal_load(s + 2);
                v[u].w = __builtin_nontemporal_load(s + 3);
            } else {
                v[u] = src[i + u * stride];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float *d = reinterpret_cast<float *>(dst + i + u * stride);
            if (NT) {
                __builtin_nontemporal_store(v[u].x, d);
                __builtin_nontemporal_store(v[u].y, d + 1);
                __builtin_nontemporal_store(v[u].z, d + 2);
                __builtin_nontemporal_store(v[u].w, d + 3);
            } else {
                dst[i + u * stride] = v[u];
            }
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// Buffers rotate so no launch finds its source in the 256 MB Infinity Cache by repetition: "pp" copies
// 0 -> 1 -> 0 (the sweep's ping-pong: the source was written by the previous launch), "rot" copies
// 2r -> 2r+1 mod 5 (the source was last touched three launches earlier).  A single src -> dst pair
// repeated measured 8.1 TB/s, above the HBM peak: part of the source stayed in the cache.
float4 *g_buf[5];
int g_mode = 0;  // 0 pp, 1 rot
template <int U, bool NT>
int run(const char *name, const float4 *, float4 *, long long n, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < 23; ++r) {
        const float4 *src = g_mode ? g_buf[(2 * r) % 5] : g_buf[r & 1];
        float4 *dst = g_mode ? g_buf[(2 * r + 1) % 5] : g_buf[(r + 1) & 1];
        CK(hipEventRecord(a, 0));
        copy_kernel<U, NT><<<blocks, 256>>>(src, dst, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3;
    printf("{\"mode\": \"%s\", \"variant\": \"%s\", \"U\": %d, \"nt\": %d, \"blocks\": %d, \"us\": %.2f, \"tbs\": %.3f, "
           "\"min_us\": %.2f}\n",
           g_mode ? "rot" : "pp", name, U, (int)NT, blocks, us, 2.0 * n * 16 / us / 1e6, ts[0] * 1e3);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    const long long bytes = 65536LL * 1024 * 4;  // one V array of Empty-16 x 65536 (268 MB; a sweep reads one, writes one)
    const long long n = bytes / 16;
    for (auto &b : g_buf) {
        CK(hipMalloc(&b, n * 16));
        CK(hipMemset(b, 0x3c, n * 16));
    }
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grids[] = {cus * 2, cus * 4, cus * 8, cus * 16, (int)std::min<long long>(n / 256, 1 << 30)};
    for (g_mode = 0; g_mode < 2; ++g_mode) {
        for (int g : grids) {
            if (run<1, false>("plain", nullptr, nullptr, n, g)) return 1;
            if (run<1, true>("nt", nullptr, nullptr, n, g)) return 1;
            if (g <= cus * 16 && run<2, true>("nt", nullptr, nullptr, n, g)) return 1;
        }
    }
    for (auto &b : g_buf) CK(hipFree(b));
    return 0;
}
