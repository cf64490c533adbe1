// Lone-grid solve latency through the C ABI only (no Python): per-solve wall time distribution of
// mgdp_vi_solve on Empty-16x16 (29 sweeps) and with max_sweeps = 1 (the fixed cost).
// Build: hipcc -O2 -o tools/probe_serve tools/probe_serve.cpp -Iinclude -Lminigrid_dynamicprogramming_amd -lmgdp
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mgdp.h"

static double g_gap_us = 0.0;  // busy-wait between solves (not timed): the request then comes later

static void run(int max_sweeps, int n, const char *tag) {
    const int W = 16, H = 16;
    std::vector<uint8_t> cells(W * H, 1);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            if (x == 0 || y == 0 || x == W - 1 || y == H - 1) cells[y * W + x] = 2;
    cells[(H - 2) * W + (W - 2)] = 8;
    mgdp_vi_desc d{};
    d.model = MGDP_MODEL_XYD; d.dtype = MGDP_F32; d.method = MGDP_METHOD_FUSED; d.mapping = MGDP_MAP_CELL;
    d.B = 1; d.W = W; d.H = H; d.max_sweeps = max_sweeps; d.device = 0;
    d.gamma = 0.99; d.tol = 1e-6; d.slip_p = -1.0; d.death_cost = -1.0;
    mgdp_vi *vi = nullptr;
    if (mgdp_vi_create(&d, &vi) || mgdp_vi_load_cells(vi, cells.data())) { std::printf("%s\n", mgdp_last_error()); std::exit(1); }
    int32_t k = 0, conv = 0;
    double dv = 0;
    for (int i = 0; i < 100; ++i) mgdp_vi_solve(vi, &k, &dv, &conv);
    std::vector<double> t(n);
    auto T0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        if (g_gap_us > 0) {
            const auto g0 = std::chrono::steady_clock::now();
            while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g0).count() < g_gap_us) {
            }
        }
        auto a = std::chrono::steady_clock::now();
        if (mgdp_vi_solve(vi, &k, &dv, &conv)) { std::printf("%s\n", mgdp_last_error()); std::exit(1); }
        auto b = std::chrono::steady_clock::now();
        t[i] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    double tot = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - T0).count();
    std::sort(t.begin(), t.end());
    std::printf("{\"tag\": \"%s\", \"gap_us\": %.2f, \"max_sweeps\": %d, \"sweeps\": %d, \"n\": %d, \"mean_us\": %.3f, \"min_us\": %.3f, "
                "\"p10_us\": %.3f, \"median_us\": %.3f, \"p90_us\": %.3f, \"p99_us\": %.3f}\n",
                tag, g_gap_us, max_sweeps, k, n, tot / n, t[0], t[n / 10], t[n / 2], t[n * 9 / 10], t[n * 99 / 100]);
    mgdp_vi_destroy(vi);
}

int main(int argc, char **argv) {
    const char *tag = argc > 1 ? argv[1] : "default";
    int32_t pinned = 0;  // the polling thread on the GPU's NUMA node (MGDP_PROBE_PIN=0: unpinned)
    if (!getenv("MGDP_PROBE_PIN") || atoi(getenv("MGDP_PROBE_PIN")) != 0) mgdp_pin_host_thread(0, &pinned);
    std::fprintf(stderr, "pinned to %d CPUs\n", (int)pinned);
    if (getenv("MGDP_PROBE_GAP_US")) g_gap_us = atof(getenv("MGDP_PROBE_GAP_US"));
    run(1, 5000, tag);
    run(2, 5000, tag);
    run(10000, 5000, tag);
    return 0;
}
