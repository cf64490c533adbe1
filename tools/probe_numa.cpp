// Lone-solve latency (mgdp_vi_solve on Empty-16x16, 29 sweeps) with the calling thread pinned to
// one CPU at a time: a CPU on the GPU's own NUMA node vs CPUs on other nodes.  The handle (and its
// host-mapped request / result words) is created after pinning, so the pages are the pinned
// CPU's node's.  Prints one JSON line per CPU tried.
// Build: hipcc -O2 -o tools/probe_numa tools/probe_numa.cpp -Iinclude -Lminigrid_dynamicprogramming_amd -lmgdp
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "mgdp.h"

static std::string read_file(const std::string &p) {
    std::ifstream f(p);
    std::stringstream s;
    s << f.rdbuf();
    std::string r = s.str();
    while (!r.empty() && (r.back() == '\n' || r.back() == ' ')) r.pop_back();
    return r;
}

static std::vector<int> parse_list(const std::string &s) {  // "0-3,8-11"
    std::vector<int> v;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
        if (tok.empty()) continue;
        const size_t d = tok.find('-');
        if (d == std::string::npos) {
            v.push_back(std::atoi(tok.c_str()));
        } else {
            for (int i = std::atoi(tok.substr(0, d).c_str()); i <= std::atoi(tok.substr(d + 1).c_str()); ++i) v.push_back(i);
        }
    }
    return v;
}

static void measure(int cpu, const char *where) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    if (sched_setaffinity(0, sizeof set, &set) != 0) {
        std::printf("{\"cpu\": %d, \"where\": \"%s\", \"error\": \"sched_setaffinity refused\"}\n", cpu, where);
        return;
    }
    const int W = 16, H = 16;
    std::vector<uint8_t> cells(W * H, 1);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            if (x == 0 || y == 0 || x == W - 1 || y == H - 1) cells[y * W + x] = 2;
    cells[(H - 2) * W + (W - 2)] = 8;
    mgdp_vi_desc d{};
    d.model = MGDP_MODEL_XYD; d.dtype = MGDP_F32; d.method = MGDP_METHOD_FUSED; d.mapping = MGDP_MAP_CELL;
    d.B = 1; d.W = W; d.H = H; d.max_sweeps = 10000; d.device = 0;
    d.gamma = 0.99; d.tol = 1e-6; d.slip_p = -1.0; d.death_cost = -1.0;
    mgdp_vi *vi = nullptr;
    if (mgdp_vi_create(&d, &vi) || mgdp_vi_load_cells(vi, cells.data())) { std::printf("%s\n", mgdp_last_error()); std::exit(1); }
    int32_t k = 0, conv = 0;
    double dv = 0;
    for (int i = 0; i < 200; ++i) mgdp_vi_solve(vi, &k, &dv, &conv);
    const int n = 4000;
    std::vector<double> t(n);
    for (int i = 0; i < n; ++i) {
        auto a = std::chrono::steady_clock::now();
        if (mgdp_vi_solve(vi, &k, &dv, &conv)) { std::printf("%s\n", mgdp_last_error()); std::exit(1); }
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"cpu\": %d, \"where\": \"%s\", \"sweeps\": %d, \"p10_us\": %.3f, \"median_us\": %.3f, \"p90_us\": %.3f}\n", cpu,
                where, k, t[n / 10], t[n / 2], t[n * 9 / 10]);
    std::fflush(stdout);
    mgdp_vi_destroy(vi);
}

int main() {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) { std::printf("no bus id\n"); return 1; }
    std::string id(bus);
    std::transform(id.begin(), id.end(), id.begin(), ::tolower);
    const std::string dev = "/sys/bus/pci/devices/" + id;
    const std::string node = read_file(dev + "/numa_node");
    const std::string local = read_file(dev + "/local_cpulist");
    cpu_set_t allowed;
    sched_getaffinity(0, sizeof allowed, &allowed);
    std::printf("{\"pci\": \"%s\", \"numa_node\": \"%s\", \"local_cpulist\": \"%s\", \"allowed_cpus\": %d}\n", id.c_str(),
                node.c_str(), local.c_str(), CPU_COUNT(&allowed));
    std::vector<int> loc = parse_list(local);
    std::vector<int> tried;
    for (size_t i = 0; i < loc.size() && tried.size() < 2; i += std::max<size_t>(1, loc.size() / 2))
        if (CPU_ISSET(loc[i], &allowed)) { measure(loc[i], "local"); tried.push_back(loc[i]); }
    for (int nd = 0; nd < 16; ++nd) {
        const std::string l = read_file("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
        if (l.empty()) continue;
        std::vector<int> c = parse_list(l);
        if (c.empty() || std::find(loc.begin(), loc.end(), c[0]) != loc.end()) continue;
        if (CPU_ISSET(c[0], &allowed)) measure(c[0], ("node" + std::to_string(nd)).c_str());
    }
    return 0;
}
