// Host cost of one batched step launch through the C ABI (no Python): DoorKey-16x16 x 65536 envs
// from mgdp_gen_grids_host, then N asynchronous mgdp_envs_step_device launches; reports the host
// time per launch call, the wall time per step (host loop + final sync) and the step kernel's
// event time, with and without launch timing.
// Build: hipcc -O2 -o tools/probe_step tools/probe_step.cpp -Iinclude -Lminigrid_dynamicprogramming_amd -lmgdp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mgdp.h"

#define CK(x) do { if (x) { std::printf("%s\n", mgdp_last_error()); std::exit(1); } } while (0)

int main() {
    const int B = 65536, W = 16, H = 16, N = 2000;
    mgdp_gen_desc g{};
    g.family = MGDP_GEN_DOORKEY; g.W = W; g.H = H;
    std::vector<uint8_t> enc((size_t)B * W * H * 3);
    std::vector<int32_t> ag((size_t)B * 3), ms(B, 10 * W * H);
    std::vector<uint8_t> see(B, 0);
    CK(mgdp_gen_grids_host(&g, 0, 0, B, enc.data(), nullptr, ag.data()));
    mgdp_envs *E = nullptr;
    CK(mgdp_envs_create(0, B, W, H, 7, &E));
    CK(mgdp_envs_load(E, enc.data(), ag.data(), ms.data(), see.data(), nullptr));
    int32_t *act, *dir, *stat;
    uint8_t *obs, *term, *trunc;
    double *rew;
    hipMalloc(&act, 4 * (size_t)B * N / 100); hipMalloc(&dir, 4 * B); hipMalloc(&stat, 4 * B);
    hipMalloc(&obs, (size_t)B * 147); hipMalloc(&term, B); hipMalloc(&trunc, B); hipMalloc(&rew, 8 * B);
    std::vector<int32_t> ha((size_t)B * N / 100);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = (int32_t)((i * 2654435761u) >> 7) % 7;
    hipMemcpy(act, ha.data(), 4 * ha.size(), hipMemcpyHostToDevice);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    CK(mgdp_envs_set_stream(E, s));
    for (int timing = 0; timing < 2; ++timing) {
        for (int i = 0; i < 50; ++i) CK(mgdp_envs_step_device(E, act + (size_t)(i % 20) * B, obs, dir, rew, term, trunc, stat));
        hipStreamSynchronize(s);
        CK(mgdp_envs_enable_timing(E, timing));
        double host = 0;
        auto T0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) {
            auto a = std::chrono::steady_clock::now();
            CK(mgdp_envs_step_device(E, act + (size_t)(i % 20) * B, obs, dir, rew, term, trunc, stat));
            host += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        }
        hipStreamSynchronize(s);
        const double wall = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - T0).count();
        double kms = 0;
        int64_t nl = 0;
        CK(mgdp_envs_kernel_time(E, &kms, &nl));
        std::printf("{\"timing\": %d, \"launches\": %d, \"host_us_per_call\": %.3f, \"wall_us_per_step\": %.3f, "
                    "\"kernel_us\": %.3f, \"env_steps_per_s\": %.4g}\n",
                    timing, N, host / N, wall / N, nl ? kms * 1000.0 / nl : 0.0, (double)B * N / (wall * 1e-6));
    }
    CK(mgdp_envs_destroy(E));
    return 0;
}
