// vi.hip -- Jacobi value iteration over batches of Minigrid grids on MI355X (gfx950).
//
// DP semantics (DESIGN.md "A9"): the transition is MiniGridEnv.step, minigrid/minigrid_env.py:520-583
// (front_pos :392-419, DIR_TO_VEC minigrid/core/constants.py:49-58, cell predicates
// minigrid/core/world_object.py:46-64,114,129,142,165,178-195,244); the value-iteration rule is
// build-defined because the reference has none.  The CPU oracle
// (oracle/mgdp_oracle.c) states the same arithmetic in the same order; both are compiled with
// -ffp-contract=off so fp32 and fp64 results agree bit for bit.
//
// Data layout in HBM (one handle = B grids of W x H on one device):
//   cells  uint8  [B][HWp]      OBJECT_TO_IDX per cell, row-major y*W+x, padded to 16 B per grid
//   V      T      [2][B][S]     value double-buffer (fused method uses buffer 0 in place)
//   pi     int8   [B][S]        greedy action of the last sweep (-1 = absorbing state)
//   kenv   int32  [B], dvenv f64 [B]   sweeps done / last max|dV| per grid (fused method)
//   red    u64    [64][4] + u32 ticket fused-launch reduction (kmax, dV bits, kmin) -> host-mapped
//   shards u64    [max_sweeps][8]      per-sweep global max|dV| as f64 bits (sweep method),
//                                      8 atomic shards (blockIdx & 7) to spread contention
//
// Kernels (vi_kernels.h)
//   vi_fused_kernel   one workgroup per grid: cells + both V tiles + pi live in LDS for the
//                     whole solve; many sweeps per launch, one __syncthreads per sweep.
//   vi_serve_kernel   the same solve in a persistent workgroup serving lone-grid requests.
//   vi_fused_opts_kernel  the fused solve with NoDeath lava / finite horizon.
//   vi_sweep_kernel   one Jacobi sweep of every grid: per grid, V'[grid] is staged HBM->LDS (the
//                     LDS tile of the neighbourhood), updated from LDS, written back.
// Device code is split into vi_model.h (model), vi_loops.h (workgroup loops), vi_kernels.h
// (kernels); this file holds the host side and the C ABI.
// Thread mappings (template MAP): MGDP_MAP_CELL = one thread per cell updating its 4 (XYD) or
// 16 (DoorKey) states from 16-B LDS vectors; MGDP_MAP_SA = one thread per (state, action),
// 8 lanes per state, wave shuffle max-reduce with the lowest action index winning ties.
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <climits>
#include <limits>
#include <type_traits>
#include <cstring>
#include <vector>

#include "common.h"
#include "comm.h"

#include "vi_model.h"
#include "vi_loops.h"
#include "vi_kernels.h"


// ================================================================================================
// Host side
// ================================================================================================
using namespace mgdp;

struct mgdp_vi {
    mgdp_vi_desc d;
    int S = 0, HW = 0, HWp = 0, A = 0, tsize = 0;
    int HWs = 0, Ss = 0;  // see Geo
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint8_t *d_cells = nullptr;
    void *d_V[2] = {nullptr, nullptr};
    int8_t *d_pi = nullptr;
    int32_t *d_kenv = nullptr;
    int32_t *d_kexec = nullptr;  // per grid: the sweep it last computed (fixed-point grids keep theirs)
    // learned dispatch (Geo::order / kprio): set up from d_kexec at the first solve of cells that were
    // already solved once (MGDP_LEARN_ORDER=0 turns the order off, MGDP_LEARN_PRIO=1 the priority on)
    int32_t *d_order = nullptr;
    bool order_valid = false;
    int solves_since_load = 0;
    int kprio[3] = {0, 0, 0};
    // measured (profiles/r05_ab2/): the order alone +3-6 % (LavaS11N5 x 8192 / x 65536, FourRooms x
    // 4096, DoorKey-16 x 65536); the priority on top of it nothing or worse -- off by default
    bool learn_order = true, learn_prio = false;
    int order_src = 1;  // dispatch order key: 1 the cells' depth proxy (at load), 2 the last solve's sweeps, 0 none (MGDP_ORDER)
    double *d_dvenv = nullptr;
    unsigned long long *d_shards = nullptr;
    unsigned long long *d_red = nullptr;    // fused reduction shards [64][4]
    unsigned long long *d_pub1 = nullptr;   // device copy of a run_local launch's {kmax, dV, kmin, 0} (chained solve)
    bool chain = true;                      // batched fused solve: run_local -> run_to(K from device memory), one host wait (MGDP_CHAIN=0: two)
    int inkernel_max = kInKernelReduceMaxB; // batches up to this fold {k, dV} in the fused launch itself (MGDP_INKERNEL_MAX)
    unsigned int *d_ticket = nullptr;       // arrival ticket of the fused reduction
    bool reduce_multi = true;               // B > inkernel_max: vi_reduce_multi_kernel (MGDP_REDUCE_MULTI)
    // host-mapped words (kHoutWords): [0..3] {kmax, dV hi, dV lo, kmin} of a launch (each tagged with
    // its epoch), [5..7] the server's tagged result, [8..9] trace stamps, [11] server exit word,
    // [12..13] the run_to mirror (tagged),
    // [16] request word and [17] its source word (their own 128-B line: the server polls the pair)
    unsigned long long *h_out = nullptr;
    unsigned long long *d_hout = nullptr;   // device alias of h_out
    int cur = 0;        // V buffer holding the current V (sweep method)
    int k_min = 0;      // min / max sweeps over grids after the last reduce (fused method)
    int k_max = 0;
    bool k_done_valid = false;  // k_min / dv_red describe the current device state
    double dv_red = 0.0;
    int k_done = 0;     // sweeps completed by every grid (uniform after run_to / sweep)
    int32_t sweeps = 0, converged = 0;
    bool cells_loaded = false;
    // timing of the dominant kernel
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev, ev_pool;
    std::vector<int> ev_sweep;  // sweep index of each timed sweep launch (-1 = fused launch)
    double total_ms = 0.0;
    int64_t launches = 0;
    int fused_block = 256;
    int sweep_grid = 2048;
    int fresh = 1;          // next fused launch starts from V_0 = 0
    unsigned int epoch = 0; // tag of the last fused launch; its result lands in h_out[0..3]
    int nbuf = 2;                 // fused LDS V buffers (3 = two-sweep XYD step)
    int quad = 0;                 // fused XYD: 4 threads per cell
    int pair = 0;                 // fused XYD: two-sweep step
    int wave_p = 0;               // lone XYD grid on one wave: cells per lane (fused_wave_xyd)
    int cpt = 1;                  // batched XYD fused path: cells per thread (MGDP_CPT; 2 = fused_fast_xyd_soa_x2)
    int serve_ew = 0;             // served lone deterministic XYD grid on fused_serve_xyd (MGDP_SERVE_EW=0: off)
    int serve_pair = 0;           // ... two sweeps per barrier, fused_serve_pair (MGDP_SERVE_PAIR=0: off)
    int dk1t = 0;                 // batched fp32 DoorKey on one LDS tile (MGDP_DK_1T; fused_fast_dk_1t)
    int dkhalf = 0;               // batched DoorKey, states split by has_key over two threads (MGDP_DK_HALF; fused_dk_half)
    int dkrow = 0;                // batched DoorKey of width 16 on whole-row thread maps (MGDP_DK_ROWS; fused_dk_rows)
    int pair2 = 1;                // batched plain XYD with cpt 2: adjacent-cell pairs (MGDP_PAIR2=0: fused_fast_xyd_soa_xn)
    int wave2 = 0;                // batched plain XYD on one wave per grid: cells per lane P (fused_wave2_xyd; 0 = off)
    int wave2n = 0;               // ... on two waves per grid instead: blocks per wave PW (fused_wave2n_xyd; 0 = off)
    // ... mixed: two waves for the learned order's long grids, one for the rest (kWpMix; MGDP_MIX=1,
    // fp32, P = wave2 in 2..6); nmix = the long grids (kexec >= mix_frac x the longest), set with the order
    bool mix = false;
    int nmix = 0;
    double mix_frac = 0.75;
    int band = 0;                 // ... on column bands of this many rows instead (fused_band_xyd; MGDP_BAND)
    int sweep_block = 256;
    int sweep_m = 1;              // grids staged per workgroup iteration (measured: m>1 no faster)
    int sweep_pipe = 2;           // register-pipelined sweep kernel: grids fetched ahead (0 = staged kernel)
    int pipe_grid = 0;            // its grid: resident workgroups (set at the first launch)
    // SURVEY 8(f) item-3 options (NoDeath lava, finite horizon): vi_fused_opts_kernel
    bool opts = false;
    void *d_rgoal = nullptr;      // T[H]: the exact _reward() of step_count t+1, per t
    int8_t *d_pi_t = nullptr;     // int8[H][B][S] with MGDP_KEEP_POLICY_T
    // persistent solver (lone grid, fused one-thread-per-cell path): see vi_serve_kernel
    bool persistent = true;       // MGDP_PERSISTENT=0 disables it
    bool serving = false;         // a vi_serve_kernel launch may be resident on `stream`
    // The server leaves after serve_idle_ticks without a request, which also bounds how long a
    // device-wide synchronisation by another component can wait on it.
    unsigned long long serve_idle_ticks = 10000;     // 100 us at 100 MHz
    unsigned long long serve_life_ticks = 200000000; // 2 s
    int serve_pollers = 1;  // waves polling the request word (MGDP_SERVE_POLLERS; 1 measured 0.2-0.4 us faster than 4)
    int serve_poll_dma = 1; // the server's polls land in an LDS mailbox, several in flight (MGDP_SERVE_POLL_DMA=0: one at a time)
    std::chrono::steady_clock::time_point serve_last{};  // host time of the last served result
    // A new lone grid for a resident server: the bytes wait at pending_src (host-mapped staging
    // h_stage, or the caller's device memory) and the next request carries kServeNewCells; a server
    // stop before that copies them into d_cells instead.
    uint8_t *h_stage = nullptr;   // pinned, mapped: W*H bytes (B == 1 handles)
    uint8_t *d_stage = nullptr;   // its device alias
    unsigned long long pending_src = 0;
    bool last_req = false;        // the request being posted is the server's last (mgdp_vi_solve_last)
    bool exiting = false;         // a server told to leave after its last request is the stream's last work
    unsigned long long serve_tag = 0;  // tag of the latest server launch: its exit word (h_out[11]) carries it
    // clock of the departed servers since enable_timing (mgdp_vi_serve_clock): shader-clock cycles and
    // 100 MHz ticks of their lives, summed as each one's exit word is seen (kHoutClk)
    unsigned long long clk_tag = 0;  // the last server launch whose clock words were added
    double clk_cycles = 0.0, clk_ticks = 0.0, clk_busy = 0.0, clk_solves = 0.0;
    long long clk_launches = 0;
    // the in-launch reduction (GkCtx, the wave2 family): one launch per batched deterministic solve
    // (MGDP_GK=0 turns it off)
    bool gk = false;
    int gk_capacity = 0;          // resident workgroups of the wave2 kernel on this device (MGDP_GK=2)
    unsigned long long *d_gk = nullptr;
    // the resident batch server (vi_bserve_kernel): one-wave batches within its resident capacity,
    // solves with launch timing off (MGDP_BSERVE=0: off)
    bool bserve = true;
    bool bserve_any = false;             // also batches past its resident capacity, several grids per workgroup (MGDP_BSERVE=2)
    int bserve_cap = 0;                  // resident workgroups of vi_bserve_kernel on this device
    int bserve_copies = kBreqCopies;     // request lines the workgroups poll (MGDP_BSERVE_COPIES)
    int bserve_nap = 1;                  // s_sleep(10)s between polls (MGDP_BSERVE_NAP)
    int bserve_wait_pub = 1;             // the forwarder polls the host only after the publication (MGDP_BSERVE_WAIT_PUB)
    bool solving = false;                // inside mgdp_vi_solve: its run_local may use the batch server
    double bserve_prio_frac = 0.0;       // this fraction of the dispatch order's longest grids sweeps at a higher issue priority (MGDP_BSERVE_PRIO_FRAC)
    unsigned long long *d_breq = nullptr;  // its device words (kBreqWords): forwarded request, exit counter
};

namespace {

Geo make_geo(const mgdp_vi *vi) {
    Geo g;
    g.B = vi->d.B;
    g.W = vi->d.W;
    g.H = vi->d.H;
    g.HW = vi->HW;
    g.HWp = vi->HWp;
    g.HWs = vi->HWs;
    g.Ss = vi->Ss;
    g.S = vi->S;
    g.off[0] = 1;
    g.off[1] = vi->d.W;
    g.off[2] = -1;
    g.off[3] = -vi->d.W;
    g.max_sweeps = vi->d.max_sweeps;
    g.nbuf = vi->nbuf;
    g.quad = vi->quad;
    g.pair = vi->pair;
    g.tol = vi->d.tol;
    g.kexec = vi->d_kexec;
    g.order = vi->order_valid && vi->learn_order ? vi->d_order : nullptr;
    for (int i = 0; i < 3; ++i) g.kprio[i] = vi->order_valid && vi->learn_prio ? vi->kprio[i] : 0;
    g.nmix = g.order && vi->mix ? vi->nmix : 0;
    g.wt = vi->gk_capacity > 0 && vi->d.B <= vi->gk_capacity;
    return g;
}

template <typename T>
Coef<T> make_coef(const mgdp_vi *vi) {
    Coef<T> c;
    c.g = (T)vi->d.gamma;
    const double p = vi->d.slip_p;
    c.p = (T)p;
    c.c = (T)((1.0 - p) / 6.0);
    T t = (T)vi->d.tol;
    if ((double)t < vi->d.tol) t = std::nextafter(t, std::numeric_limits<T>::infinity());
    c.tol = t;
    c.dc = (T)vi->d.death_cost;
    return c;
}

// Timed launches go through hipExtLaunchKernelGGL with a start/stop event pair, so the events carry
// the dispatch's own begin/end timestamps (what rocprofv3's kernel trace reports) rather than the
// times of separate marker packets.  Event pairs are pooled: no hipEventCreate in the timed loop.
struct TimedPair { hipEvent_t a = nullptr, b = nullptr; };
int timed_begin(mgdp_vi *vi, int sweep_idx, TimedPair *tp) {
    tp->a = tp->b = nullptr;
    if (!vi->timing) return 0;
    std::pair<hipEvent_t, hipEvent_t> e;
    if (!vi->ev_pool.empty()) {
        e = vi->ev_pool.back();
        vi->ev_pool.pop_back();
    } else {
        MGDP_HIP(hipEventCreate(&e.first));
        MGDP_HIP(hipEventCreate(&e.second));
    }
    vi->ev.push_back(e);
    vi->ev_sweep.push_back(sweep_idx);
    tp->a = e.first;
    tp->b = e.second;
    return 0;
}
// Fold completed events into total_ms (called after a stream sync).  Sweep launches past the
// stopping sweep no-op and were marked uncounted (ev_sweep = INT_MAX) by sweep_run.
int timed_collect(mgdp_vi *vi) {
    for (size_t i = 0; i < vi->ev.size(); ++i) {
        if (vi->ev_sweep[i] != INT32_MAX) {
            float ms = 0.f;
            MGDP_HIP(hipEventElapsedTime(&ms, vi->ev[i].first, vi->ev[i].second));
            vi->total_ms += ms;
            vi->launches += 1;
        }
        vi->ev_pool.push_back(vi->ev[i]);
    }
    vi->ev.clear();
    vi->ev_sweep.clear();
    return 0;
}

// {kmax, dV, kmin} of a launch too large to reduce in itself: kRedShards workgroups on the
// fused reduction's idle shards (MGDP_REDUCE_MULTI=0: the one-workgroup kernel)
// The epoch of a launch whose result goes to the host-mapped words (never 0: publish() writes a
// device buffer's raw words for epoch 0)
inline unsigned int next_host_epoch(mgdp_vi *vi) {
    if (++vi->epoch == 0u) ++vi->epoch;
    return vi->epoch;
}

inline void launch_reduce(mgdp_vi *vi, unsigned long long *pub) {
    if (vi->reduce_multi)
        hipLaunchKernelGGL(vi_reduce_multi_kernel, dim3(kRedShards), dim3(256), 0, vi->stream, vi->d_kenv, vi->d_dvenv,
                           vi->d.B, vi->d_red, vi->d_ticket, pub, pub == vi->d_hout ? vi->epoch : 0u);
    else
        hipLaunchKernelGGL(vi_reduce_kernel, dim3(1), dim3(1024), 0, vi->stream, vi->d_kenv, vi->d_dvenv, vi->d.B,
                           pub, pub == vi->d_hout ? vi->epoch : 0u);
}

template <typename T, int MODEL, bool SLIP, bool ND, int HMODE>
int launch_opts_t(mgdp_vi *vi, int k_target) {
    const Geo g = make_geo(vi);
    const Smem L = smem_layout(vi->Ss, vi->HWp, sizeof(T), vi->nbuf);
    auto kern = vi_fused_opts_kernel<T, MODEL, SLIP, ND, HMODE>;
    if (L.total() > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, L.total()));
    TimedPair tp;
    if (int rc = timed_begin(vi, -1, &tp)) return rc;
    hipExtLaunchKernelGGL(kern, dim3(vi->d.B), dim3(vi->fused_block), L.total(), vi->stream, tp.a, tp.b, 0, g,
                          make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv, vi->d_dvenv,
                          vi->d_red, vi->d_ticket, vi->d_hout, k_target, vi->fresh,
                          vi->d.B <= vi->inkernel_max ? 1 : 0, next_host_epoch(vi), (const T *)vi->d_rgoal, vi->d_pi_t);
    MGDP_HIP(hipGetLastError());
    vi->fresh = 0;
    if (vi->d.B > vi->inkernel_max) {
        launch_reduce(vi, vi->d_hout);
        MGDP_HIP(hipGetLastError());
    }
    return 0;
}

// runtime options -> template instantiation of the options kernel
template <typename T, int MODEL, bool SLIP, bool ND>
int launch_opts_h(mgdp_vi *vi, int k_target) {
    const int hm = vi->d.horizon > 0 ? ((vi->d.flags & MGDP_KEEP_POLICY_T) ? 2 : 1) : 0;
    if (hm == 2) return launch_opts_t<T, MODEL, SLIP, ND, 2>(vi, k_target);
    if (hm == 1) return launch_opts_t<T, MODEL, SLIP, ND, 1>(vi, k_target);
    return launch_opts_t<T, MODEL, SLIP, ND, 0>(vi, k_target);
}
template <typename T>
int launch_opts(mgdp_vi *vi, int k_target) {
    if (vi->d.model == MGDP_MODEL_DOORKEY) return launch_opts_h<T, MGDP_MODEL_DOORKEY, false, false>(vi, k_target);
    const bool slip = vi->d.slip_p >= 0.0, nd = vi->d.lava_mode == MGDP_LAVA_NODEATH;
    if (slip) return nd ? launch_opts_h<T, MGDP_MODEL_XYD, true, true>(vi, k_target)
                        : launch_opts_h<T, MGDP_MODEL_XYD, true, false>(vi, k_target);
    return nd ? launch_opts_h<T, MGDP_MODEL_XYD, false, true>(vi, k_target)
              : launch_opts_h<T, MGDP_MODEL_XYD, false, false>(vi, k_target);
}

// Kernel variant: the one-wave lone-grid instantiation when vi->wave_p is set (XYD, cell mapping).
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP>
auto pick_wave(const mgdp_vi *vi) -> decltype(K<T, MODEL, SLIP, MAP, 0>::fn) {
    if constexpr (MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL) {
        switch (vi->wave_p) {
        case 1: return K<T, MODEL, SLIP, MAP, 1>::fn;
        case 2: return K<T, MODEL, SLIP, MAP, 2>::fn;
        case 4: return K<T, MODEL, SLIP, MAP, 4>::fn;
        case 8: return K<T, MODEL, SLIP, MAP, 8>::fn;
        default: break;
        }
    }
    return K<T, MODEL, SLIP, MAP, 0>::fn;
}
template <typename T, int MODEL, bool SLIP, int MAP, int WP>
struct FusedK { static constexpr auto fn = vi_fused_kernel<T, MODEL, SLIP, MAP, WP>; };
// The one-wave-per-grid instantiation for P cells per lane (1..8); `dflt` if P is out of range.
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP, typename F>
F pick_wave2(int P, F dflt) {
    constexpr int PMAX = 8;
    switch (P) {
    case 1: return K<T, MODEL, SLIP, MAP, kWpWave2 - 1>::fn;
    case 2: return K<T, MODEL, SLIP, MAP, kWpWave2 - 2>::fn;
    case 3: return K<T, MODEL, SLIP, MAP, kWpWave2 - 3>::fn;
    case 4: return K<T, MODEL, SLIP, MAP, kWpWave2 - 4>::fn;
    default: break;
    }
    if constexpr (PMAX > 4) {
        switch (P) {
        case 5: return K<T, MODEL, SLIP, MAP, kWpWave2 - 5>::fn;
        case 6: return K<T, MODEL, SLIP, MAP, kWpWave2 - 6>::fn;
        case 7: return K<T, MODEL, SLIP, MAP, kWpWave2 - 7>::fn;
        case 8: return K<T, MODEL, SLIP, MAP, kWpWave2 - 8>::fn;
        default: break;
        }
    }
    return dflt;
}
// The column-band instantiation for HB rows per band (1..8); `dflt` if out of range.
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP, typename F>
F pick_band(int HB, F dflt) {
    switch (HB) {
    case 1: return K<T, MODEL, SLIP, MAP, kWpBand - 1>::fn;
    case 2: return K<T, MODEL, SLIP, MAP, kWpBand - 2>::fn;
    case 3: return K<T, MODEL, SLIP, MAP, kWpBand - 3>::fn;
    case 4: return K<T, MODEL, SLIP, MAP, kWpBand - 4>::fn;
    case 5: return K<T, MODEL, SLIP, MAP, kWpBand - 5>::fn;
    case 6: return K<T, MODEL, SLIP, MAP, kWpBand - 6>::fn;
    case 7: return K<T, MODEL, SLIP, MAP, kWpBand - 7>::fn;
    case 8: return K<T, MODEL, SLIP, MAP, kWpBand - 8>::fn;
    default: return dflt;
    }
}
// The mixed-wave-count instantiation for P blocks of 64 cells (2..6, fp32); `dflt` otherwise.
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP, typename F>
F pick_mix(int P, F dflt) {
    if constexpr (std::is_same<T, float>::value) {
        switch (P) {
        case 2: return K<T, MODEL, SLIP, MAP, kWpMix - 2>::fn;
        case 3: return K<T, MODEL, SLIP, MAP, kWpMix - 3>::fn;
        case 4: return K<T, MODEL, SLIP, MAP, kWpMix - 4>::fn;
        case 5: return K<T, MODEL, SLIP, MAP, kWpMix - 5>::fn;
        case 6: return K<T, MODEL, SLIP, MAP, kWpMix - 6>::fn;
        default: break;
        }
    }
    return dflt;
}
// The two-waves-per-grid instantiation for PW blocks per wave (2..4); `dflt` if out of range.
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP, typename F>
F pick_wave2n(int PW, F dflt) {
    switch (PW) {
    case 2: return K<T, MODEL, SLIP, MAP, kWpWave2n - 2>::fn;
    case 3: return K<T, MODEL, SLIP, MAP, kWpWave2n - 3>::fn;
    case 4: return K<T, MODEL, SLIP, MAP, kWpWave2n - 4>::fn;
    default: return dflt;
    }
}
template <typename T, int MODEL, bool SLIP, int MAP, int WP>
struct ServeK { static constexpr auto fn = vi_serve_kernel<T, MODEL, SLIP, MAP, WP>; };
// fused_dk_half variants by plane stride HWs = 64 * n (the host allows n <= 8)
template <template <typename, int, bool, int, int> class K, typename T, int MODEL, bool SLIP, int MAP, typename F>
F pick_dkhalf(int n, F dflt) {
    switch (n) {
    case 1: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 1>::fn;
    case 2: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 2>::fn;
    case 3: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 3>::fn;
    case 4: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 4>::fn;
    case 5: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 5>::fn;
    case 6: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 6>::fn;
    case 7: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 7>::fn;
    case 8: return K<T, MODEL, SLIP, MAP, kWpDkHalf - 8>::fn;
    default: return dflt;
    }
}

// pub: where the launch's {kmax, dV bits, kmin} go (default: the host-mapped words the host polls,
// epoch-tagged; the multi-GPU device protocol passes a device buffer it all-reduces, raw); k_dev: the target
// sweep read from device memory instead of k_target (mgdp_vi_run_to_dev).
template <typename T, int MODEL, bool SLIP, int MAP>
int launch_fused_t(mgdp_vi *vi, int k_target, unsigned long long *pub = nullptr, const long long *k_dev = nullptr,
                   unsigned long long *mirror = nullptr) {
    if (vi->opts) return launch_opts<T>(vi, k_target);
    if (!pub) pub = vi->d_hout;
    const Geo g = make_geo(vi);
    const Smem L = smem_layout(vi->Ss, vi->HWp, sizeof(T), vi->nbuf);
    auto kern = pick_wave<FusedK, T, MODEL, SLIP, MAP>(vi);
    if constexpr (MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL) {
        if (vi->cpt == 2) kern = FusedK<T, MODEL, SLIP, MAP, -2>::fn;
        else if (vi->cpt == 4) kern = FusedK<T, MODEL, SLIP, MAP, -4>::fn;
        if constexpr (!SLIP) {  // two adjacent cells per thread, compile-time plane stride
            if (vi->cpt == 2 && vi->pair2 && vi->HWs == 2 * vi->fused_block && vi->HWs % 128 == 0 && vi->HWs <= 1024) {
                switch (vi->HWs / 128) {
                case 1: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 1>::fn; break;
                case 2: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 2>::fn; break;
                case 3: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 3>::fn; break;
                case 4: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 4>::fn; break;
                case 5: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 5>::fn; break;
                case 6: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 6>::fn; break;
                case 7: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 7>::fn; break;
                case 8: kern = FusedK<T, MODEL, SLIP, MAP, kWpPair - 8>::fn; break;
                default: break;
                }
            }
        }
    }
    if constexpr (MODEL == MGDP_MODEL_DOORKEY && MAP == MGDP_MAP_CELL && !SLIP) {
        if (vi->dk1t) kern = FusedK<T, MODEL, SLIP, MAP, kWpDk1t>::fn;
        else if (vi->dkhalf) kern = pick_dkhalf<FusedK, T, MODEL, SLIP, MAP>(vi->HWs / 64, kern);
        else if (vi->dkrow)  // fp32 16x16 own-rule launches: the compile-time 256-thread variant
            kern = (sizeof(T) == 4 && vi->HWs == 256 && vi->fused_block == 256 && k_target < 0 && !k_dev)
                       ? FusedK<T, MODEL, SLIP, MAP, kWpDkRow16>::fn
                       : FusedK<T, MODEL, SLIP, MAP, kWpDkRow>::fn;
    }
    if constexpr (MAP == MGDP_MAP_CELL) {  // one cell per thread, direction-major: the stripped variant
        if (kern == FusedK<T, MODEL, SLIP, MAP, 0>::fn && !vi->pair && !vi->quad && vi->HW <= vi->fused_block)
            kern = FusedK<T, MODEL, SLIP, MAP, kWpSoa>::fn;
    }
    int smem = L.total();
    if constexpr (MODEL == MGDP_MODEL_DOORKEY && MAP == MGDP_MAP_CELL && !SLIP) {
        if (vi->dkrow && !vi->dk1t && !vi->dkhalf) smem = dkrow_smem_bytes(vi->HWp, vi->HWs, (int)sizeof(T));
    }
    if constexpr (MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL && !SLIP) {
        if (vi->mix) {
            kern = pick_mix<FusedK, T, MODEL, SLIP, MAP>(vi->wave2, kern);
            smem = mix_smem_bytes(vi->HWp, vi->d.W, vi->wave2, (int)sizeof(T));
        } else if (vi->wave2n) {
            kern = pick_wave2n<FusedK, T, MODEL, SLIP, MAP>(vi->wave2n, kern);
            smem = wave2n_smem_bytes(vi->HWp, vi->d.W, 2 * vi->wave2n, (int)sizeof(T));
        } else if (vi->band) {
            kern = pick_band<FusedK, T, MODEL, SLIP, MAP>(vi->band, kern);
            smem = 256 + (vi->HWp + 15) / 16 * 16;
        } else if (vi->wave2) {
            kern = pick_wave2<FusedK, T, MODEL, SLIP, MAP>(vi->wave2, kern);
            smem = wave2_smem_bytes(vi->HWp, vi->d.W, vi->wave2, (int)sizeof(T));
        }
    }
    if (smem > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    static const bool debug_occ = std::getenv("MGDP_DEBUG_OCC") != nullptr;  // read once, not per launch
    if (debug_occ) {  // diagnostics: resident workgroups per CU of this launch
        int per_cu = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kern, vi->fused_block, smem);
        std::fprintf(stderr, "mgdp occupancy: %d workgroups/CU (block %d, LDS %d B)\n", per_cu, vi->fused_block, smem);
    }
    TimedPair tp;
    if (int rc = timed_begin(vi, -1, &tp)) return rc;
    // the in-launch reduction (GkCtx): a fresh own-rule launch of a resident one-wave batch folds
    // each grid's {k_e, dV at k_e} through the counter tree and publishes {kmax, dV, kmin} itself (no
    // reduce kernel); grids at an exact fixed point are complete for any K (fixed-point completion),
    // so run_to has nothing to launch unless some grid stopped with dV > 0
    unsigned long long *gk = (vi->gk && k_target < 0 && vi->fresh && !k_dev) ? vi->d_gk : nullptr;
    hipExtLaunchKernelGGL(kern, dim3(vi->d.B), dim3(vi->fused_block), smem, vi->stream, tp.a, tp.b, 0, g,
                       make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv,
                       vi->d_dvenv, vi->d_red, vi->d_ticket, pub, k_target, vi->fresh,
                       vi->d.B <= vi->inkernel_max ? 1 : 0, pub == vi->d_hout ? next_host_epoch(vi) : 0u, k_dev, mirror, gk);
    MGDP_HIP(hipGetLastError());
    vi->fresh = 0;
    if (vi->d.B > vi->inkernel_max && !gk) {  // a launch-wide-rule launch publishes its own reduction
        launch_reduce(vi, pub);
        MGDP_HIP(hipGetLastError());
    }
    return 0;
}

void account_server_clock(mgdp_vi *vi);

// The batch server's instantiation for P cells per lane (the wave2 kernel's P); nullptr if out of range.
template <typename T>
const void *pick_bserve(int P) {  // the resident instantiation (the capacity of both is the same by bserve_min_waves)
    switch (P) {
    case 1: return (const void *)vi_bserve_kernel<T, 1>;
    case 2: return (const void *)vi_bserve_kernel<T, 2>;
    case 3: return (const void *)vi_bserve_kernel<T, 3>;
    case 4: return (const void *)vi_bserve_kernel<T, 4>;
    case 5: return (const void *)vi_bserve_kernel<T, 5>;
    case 6: return (const void *)vi_bserve_kernel<T, 6>;
    case 7: return (const void *)vi_bserve_kernel<T, 7>;
    case 8: return (const void *)vi_bserve_kernel<T, 8>;
    default: return nullptr;
    }
}
template <typename T, int P>
int launch_bserve_p(mgdp_vi *vi, unsigned int served, TimedPair tp) {
    const int smem = wave2_smem_bytes(vi->HWp, vi->d.W, P, (int)sizeof(T));
    static const bool force_multi = std::getenv("MGDP_BSERVE_FORCE_MULTI") != nullptr;  // diagnostics
    auto kern = (vi->d.B > vi->bserve_cap || force_multi) ? vi_bserve_kernel<T, P, true> : vi_bserve_kernel<T, P, false>;
    hipExtLaunchKernelGGL(kern, dim3(std::min(vi->d.B, vi->bserve_cap)), dim3(64), smem, vi->stream, tp.a, tp.b, 0, make_geo(vi),
                          make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv, vi->d_dvenv, vi->d_hout,
                          vi->d_hout + kHoutReq, vi->d_breq, vi->d_gk, (unsigned long long)served, vi->serve_idle_ticks,
                          vi->serve_life_ticks, vi->serve_tag, vi->bserve_copies, vi->bserve_nap, vi->bserve_wait_pub,
                          vi->order_valid && vi->learn_order ? (int)(vi->bserve_prio_frac * vi->d.B) : 0);
    MGDP_HIP(hipGetLastError());
    return 0;
}

template <typename T, int MODEL, bool SLIP, int MAP>
int launch_serve_t(mgdp_vi *vi, unsigned int served) {
    if (vi->d.B > 1) {  // the resident batch server (bserve_eligible: deterministic XYD, one wave per grid)
        if constexpr (MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL) {
            TimedPair tp;
            if (int rc = timed_begin(vi, -1, &tp)) return rc;
            account_server_clock(vi);
            ++vi->serve_tag;
            switch (vi->wave2) {
            case 1: return launch_bserve_p<T, 1>(vi, served, tp);
            case 2: return launch_bserve_p<T, 2>(vi, served, tp);
            case 3: return launch_bserve_p<T, 3>(vi, served, tp);
            case 4: return launch_bserve_p<T, 4>(vi, served, tp);
            case 5: return launch_bserve_p<T, 5>(vi, served, tp);
            case 6: return launch_bserve_p<T, 6>(vi, served, tp);
            case 7: return launch_bserve_p<T, 7>(vi, served, tp);
            case 8: return launch_bserve_p<T, 8>(vi, served, tp);
            default: break;
            }
        }
        MGDP_CHECK(false, MGDP_E_INVALID, "batch server: not a one-wave deterministic XYD batch");
    }
    const Geo g = make_geo(vi);
    const Smem L = smem_layout(vi->Ss, vi->HWp, sizeof(T), vi->nbuf);
    auto kern = pick_wave<ServeK, T, MODEL, SLIP, MAP>(vi);
    int smem = L.total();
    if constexpr (MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL) {
        if (vi->cpt == 2) kern = ServeK<T, MODEL, SLIP, MAP, -2>::fn;
        if constexpr (!SLIP) {
            if (vi->serve_ew) kern = vi->serve_pair ? ServeK<T, MODEL, SLIP, MAP, kWpServePair>::fn
                                                    : ServeK<T, MODEL, SLIP, MAP, kWpServeEw>::fn;
            if (vi->band) kern = pick_band<ServeK, T, MODEL, SLIP, MAP>(vi->band, kern);
        }
    }
    if constexpr (MODEL == MGDP_MODEL_DOORKEY && MAP == MGDP_MAP_CELL && !SLIP) {
        if (vi->dkhalf) kern = pick_dkhalf<ServeK, T, MODEL, SLIP, MAP>(vi->HWs / 64, kern);
    }
    if (smem > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    TimedPair tp;
    if (int rc = timed_begin(vi, -1, &tp)) return rc;
    account_server_clock(vi);  // a server that left on its own (idle / life limit) before this relaunch
    ++vi->serve_tag;
    hipExtLaunchKernelGGL(kern, dim3(1), dim3(vi->fused_block), smem, vi->stream, tp.a, tp.b, 0, g,
                          make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv, vi->d_dvenv,
                          vi->d_hout, vi->d_hout + kHoutReq, (unsigned long long)served, vi->serve_idle_ticks,
                          vi->serve_life_ticks, vi->serve_pollers, vi->serve_tag, vi->serve_poll_dma);
    MGDP_HIP(hipGetLastError());
    return 0;
}

template <typename T, int MODEL, bool SLIP, int MAP, bool POLICY>
int launch_sweep_kernel(mgdp_vi *vi, const T *Vin, T *Vout, int k, int check_prev, TimedPair tp = {}) {
    const int m = vi->sweep_m;
    const int smem = sweep_smem_bytes(vi->S, vi->HWp, sizeof(T), m);
    auto kern = vi_sweep_kernel<T, MODEL, SLIP, MAP, POLICY>;
    if (smem > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    const int groups = (vi->d.B + m - 1) / m;
    const int grid = std::min(groups, vi->sweep_grid);
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(vi->sweep_block), smem, vi->stream, tp.a, tp.b, 0, make_geo(vi), make_coef<T>(vi),
                       vi->d_cells, Vin, Vout, vi->d_pi, POLICY ? nullptr : vi->d_shards, k, check_prev, m);
    MGDP_HIP(hipGetLastError());
    return 0;
}

template <typename T, int MODEL, bool SLIP, int DEPTH>
int launch_sweep_pipe(mgdp_vi *vi, const T *Vin, T *Vout, int k, int check_prev, TimedPair tp) {
    const int smem = sweep_pipe_smem_bytes(vi->S, vi->HW, vi->HWs, vi->HWp, sizeof(T));
    auto kern = vi_sweep_pipe_kernel<T, MODEL, SLIP, DEPTH>;
    if (smem > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    if (vi->pipe_grid == 0) {  // resident workgroups, at most 4 per CU
        // Empty-16 x 65536 (profiles/r06_sweep2/): 8 per CU (every resident slot, 2048 workgroups)
        // 98.5 us per sweep, 6 per CU 100.1, 5 94.4, 4 90.3-90.8 (6.10-6.13 TB/s compulsory), 3 92.5,
        // 2 109.3: four 256-thread workgroups, each with two grids' loads in flight, keep enough bytes
        // moving, and fewer co-resident workgroups contend less for the channels.
        int per_cu = 0, cus = 0;
        MGDP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kern, vi->HWs, smem));
        MGDP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, vi->d.device));
        vi->pipe_grid = std::min(4, std::max(1, per_cu)) * std::max(1, cus);
        if (const char *ev = std::getenv("MGDP_SWEEP_GRID")) vi->pipe_grid = std::max(1, std::atoi(ev));
    }
    const int grid = std::min(vi->d.B, vi->pipe_grid);
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(vi->HWs), smem, vi->stream, tp.a, tp.b, 0, make_geo(vi), make_coef<T>(vi),
                          vi->d_cells, Vin, Vout, vi->d_shards, k, check_prev);
    MGDP_HIP(hipGetLastError());
    return 0;
}

template <typename T, int MODEL, bool SLIP, int MAP>
int launch_sweep_t(mgdp_vi *vi, int k, int check_prev, bool policy) {
    const T *Vin = (const T *)vi->d_V[(k - 1) & 1];
    T *Vout = (T *)vi->d_V[k & 1];
    if (policy) return launch_sweep_kernel<T, MODEL, SLIP, MAP, true>(vi, Vin, Vout, k, 0);
    TimedPair tp;
    if (int rc = timed_begin(vi, k, &tp)) return rc;
    if constexpr (MAP == MGDP_MAP_CELL) {
        if (vi->sweep_pipe == 1) return launch_sweep_pipe<T, MODEL, SLIP, 1>(vi, Vin, Vout, k, check_prev, tp);
        if (vi->sweep_pipe == 2) return launch_sweep_pipe<T, MODEL, SLIP, 2>(vi, Vin, Vout, k, check_prev, tp);
        if (vi->sweep_pipe == 3) return launch_sweep_pipe<T, MODEL, SLIP, 3>(vi, Vin, Vout, k, check_prev, tp);
        if (vi->sweep_pipe == 4) return launch_sweep_pipe<T, MODEL, SLIP, 4>(vi, Vin, Vout, k, check_prev, tp);
    }
    return launch_sweep_kernel<T, MODEL, SLIP, MAP, false>(vi, Vin, Vout, k, check_prev, tp);
}

// Dispatch on (dtype, model, slip, mapping).
template <template <typename, int, bool, int> class F, typename... Args>
int dispatch(mgdp_vi *vi, Args... args) {
    const bool slip = vi->d.slip_p >= 0.0;
    const bool sa = vi->d.mapping == MGDP_MAP_SA;
    if (vi->d.dtype == MGDP_F32) {
        if (vi->d.model == MGDP_MODEL_XYD) {
            if (slip) return sa ? F<float, 0, true, 1>::run(vi, args...) : F<float, 0, true, 0>::run(vi, args...);
            return sa ? F<float, 0, false, 1>::run(vi, args...) : F<float, 0, false, 0>::run(vi, args...);
        }
        return sa ? F<float, 1, false, 1>::run(vi, args...) : F<float, 1, false, 0>::run(vi, args...);
    }
    if (vi->d.model == MGDP_MODEL_XYD) {
        if (slip) return sa ? F<double, 0, true, 1>::run(vi, args...) : F<double, 0, true, 0>::run(vi, args...);
        return sa ? F<double, 0, false, 1>::run(vi, args...) : F<double, 0, false, 0>::run(vi, args...);
    }
    return sa ? F<double, 1, false, 1>::run(vi, args...) : F<double, 1, false, 0>::run(vi, args...);
}

template <typename T, int MODEL, bool SLIP, int MAP>
struct FusedF {
    static int run(mgdp_vi *vi, int k_target, unsigned long long *pub = nullptr, const long long *k_dev = nullptr,
                   unsigned long long *mirror = nullptr) {
        return launch_fused_t<T, MODEL, SLIP, MAP>(vi, k_target, pub, k_dev, mirror);
    }
};
template <typename T, int MODEL, bool SLIP, int MAP>
struct ServeF {
    static int run(mgdp_vi *vi, unsigned int served) { return launch_serve_t<T, MODEL, SLIP, MAP>(vi, served); }
};
template <typename T, int MODEL, bool SLIP, int MAP>
struct SweepF {
    static int run(mgdp_vi *vi, int k, int check_prev, bool policy) {
        return launch_sweep_t<T, MODEL, SLIP, MAP>(vi, k, check_prev, policy);
    }
};

// Read the reduction the last fused launch published to host-mapped memory: max k, max dV, min k.
int reduce_env(mgdp_vi *vi, int32_t *kmax, double *dvmax) {
    // The last workgroup (or the reduce kernel) publishes {kmax, dV hi, dV lo, kmin} to host-mapped
    // memory as four epoch-tagged words; the persistent server publishes three (words 5..7).  Poll them rather
    // than synchronise the stream (lower completion latency); everything else stays stream-ordered.
    // Poll the stream now and then to surface faults -- and, in serving mode, to relaunch a server
    // that left before it saw the request.
    const volatile unsigned long long *h = vi->h_out;
    const unsigned long long ep = (unsigned long long)vi->epoch;
    const bool served = vi->serving;                 // a resident server answers (a relaunch may be needed)
    const bool tagged = served && vi->d.B == 1;      // ... in the lone server's words [5..7]
    auto ready = [&]() -> bool {
        if (!tagged) return (h[0] >> 32) == ep && (h[1] >> 32) == ep && (h[2] >> 32) == ep && (h[3] >> 32) == ep;
        return (h[5] >> 32) == ep && (h[6] >> 32) == ep && (h[7] >> 32) == ep;
    };
    int relaunches = 0;
    // probe knobs (MGDP_QUERY_SPINS, MGDP_QUERY_AFTER_US, MGDP_SPIN_PAUSE): how often the wait
    // queries the stream, after how long, and whether each spin pauses
    static const int q_mask = [] { const char *e = std::getenv("MGDP_QUERY_SPINS"); return e ? std::atoi(e) - 1 : 1023; }();
    static const double q_after = [] { const char *e = std::getenv("MGDP_QUERY_AFTER_US"); return e ? std::atof(e) : 0.0; }();
    static const bool s_pause = [] { const char *e = std::getenv("MGDP_SPIN_PAUSE"); return e && std::atoi(e) != 0; }();
    bool query = q_after <= 0.0;
    const auto t_wait = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; !ready(); ++spin) {
        if (s_pause) __builtin_ia32_pause();
        if ((spin & (uint64_t)q_mask) == (uint64_t)q_mask) {
            if (!query) {
                query = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_wait).count() > q_after;
                if (!query) continue;
            }
            const hipError_t q = hipStreamQuery(vi->stream);
            if (q == hipSuccess) {
                if (ready()) break;
                if (served && relaunches < 4) {
                    ++relaunches;
                    DeviceGuard guard(vi->d.device);  // the served fast path of mgdp_vi_solve holds none
                    if (int rc = dispatch<ServeF>(vi, vi->epoch - 1u)) return rc;
                    continue;
                }
                MGDP_CHECK(false, MGDP_E_HIP, "fused launch finished without publishing its result (epoch %u)", vi->epoch);
            }
            if (q != hipErrorNotReady) return hip_fail(q, "fused value-iteration launch", __FILE__, __LINE__);
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
#ifdef MGDP_SERVE_TRACE
    // trace build (tools/probe_serve_trace.sh): server-side s_memrealtime stamps, 10 ns ticks --
    // [8] request seen by the workgroup, [9] result about to be published
    if (tagged) {  // each block of 1000 solves: mean GPU-side time, the shader clock over it, and when
        static double n = 0, solve = 0, cyc = 0;
        static const auto t_first = std::chrono::steady_clock::now();
        n += 1;
        solve += (double)(h[9] - h[8]) * 0.01;
        cyc += (double)(h[15] - h[14]);
        if ((long long)n % 1000 == 0) {
            const double t_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_first).count();
            std::fprintf(stderr, "serve trace: solves %.0f-%.0f, t %.1f ms, request seen -> publish %.3f us, sclk %.0f MHz (sweeps %llu)\n",
                         n - 999, n, t_ms, solve / 1000.0, cyc / solve, (unsigned long long)(h[5] & 0xffffffffull));
            solve = 0;
            cyc = 0;
        }
    }
#endif
    unsigned long long km, dvb, kmin;
    if (tagged) {
        km = kmin = h[5] & 0xffffffffull;
        dvb = ((h[6] & 0xffffffffull) << 32) | (h[7] & 0xffffffffull);
    } else {
        km = h[0] & 0xffffffffull;
        dvb = ((h[1] & 0xffffffffull) << 32) | (h[2] & 0xffffffffull);
        kmin = h[3] & 0xffffffffull;
    }
    std::memcpy(&vi->dv_red, (const void *)&dvb, sizeof(double));  // non-negative doubles order like their bits
    vi->k_min = (int)kmin;
    vi->k_max = (int)km;
    vi->k_done_valid = true;
    if (kmax) *kmax = (int32_t)km;
    if (dvmax) *dvmax = vi->dv_red;
    return 0;
}

// Persistent solver hand-off (lone grid on the one-thread-per-cell fused path).
bool serve_eligible(const mgdp_vi *vi) {
    return vi->persistent && !vi->opts && vi->d.method == MGDP_METHOD_FUSED && vi->d.B == 1 && vi->d.mapping == MGDP_MAP_CELL &&
           (vi->HW <= vi->cpt * vi->fused_block || vi->wave_p || vi->band) && !vi->pair && !vi->quad;
}
// The resident batch server (vi_bserve_kernel): a deterministic XYD batch on one wave per grid
// (the wave2 kernel with its in-launch reduction) that fits the server's resident capacity, solved
// with launch timing off (a timed solve is a launch, so kernel_time() keeps timing one solve per
// launch), from V_0 = 0 under the own rule with at least one sweep.
bool bserve_eligible(const mgdp_vi *vi) {
    return vi->persistent && vi->bserve && vi->d_breq && vi->d_gk && !vi->timing && vi->d.B > 1 &&
           (vi->d.B <= vi->bserve_cap || vi->bserve_any) &&
           !vi->opts && vi->d.method == MGDP_METHOD_FUSED && vi->d.horizon == 0 && vi->d.max_sweeps >= 1;
}
bool served_eligible(const mgdp_vi *vi) { return serve_eligible(vi) || bserve_eligible(vi); }
// Ask a resident server to leave and drain the stream.  Every entry point that enqueues other
// work on the stream, or reads results, calls this first.  A grid handed over for the next request
// but not yet served goes to d_cells here, so every other launch sees it.
// drain = false (mgdp_vi_synchronize): wait for the server's exit word -- its V / pi stores are
// then complete and visible, and nothing else is queued behind it -- instead of the stream's
// completion signal, which a later device synchronize still observes.
// Wait for the exit word of the latest server launch (its own tag: a late store of an earlier
// server cannot satisfy it); a server that never started or faulted is reported by the stream.
// Add a departed server's clock words (written before its exit word, which is a release) once.
void account_server_clock(mgdp_vi *vi) {
    const volatile unsigned long long *h = vi->h_out;
    if (vi->serve_tag == 0 || vi->clk_tag == vi->serve_tag || h[11] != vi->serve_tag) return;
    std::atomic_thread_fence(std::memory_order_acquire);
    vi->clk_cycles += (double)h[kHoutClk];
    vi->clk_ticks += (double)h[kHoutClk + 1];
    vi->clk_busy += (double)h[kHoutClk + 2];
    vi->clk_solves += (double)h[kHoutClk + 3];
    ++vi->clk_launches;
    vi->clk_tag = vi->serve_tag;
}
int wait_server_exit(mgdp_vi *vi) {
    const volatile unsigned long long *h = vi->h_out;
    for (uint64_t spin = 0; h[11] != vi->serve_tag; ++spin) {
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(vi->stream);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return hip_fail(q, "persistent server", __FILE__, __LINE__);
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    account_server_clock(vi);
    return 0;
}
int server_stop(mgdp_vi *vi, bool drain = true) {
    if (vi->serving) {
        __atomic_store_n(vi->h_out + kHoutReq, kServeQuit, __ATOMIC_RELEASE);
        vi->serving = false;
        if (drain) {
            MGDP_HIP(hipStreamSynchronize(vi->stream));
            account_server_clock(vi);
        } else if (int rc = wait_server_exit(vi)) {
            return rc;
        }
    }
    // Whatever the caller enqueues next follows the departed server on the stream, so its exit
    // word no longer says the stream is idle (mgdp_vi_synchronize's shortcut).
    vi->exiting = false;
    if (vi->pending_src) {
        MGDP_HIP(hipMemcpyAsync(vi->d_cells, reinterpret_cast<const void *>(vi->pending_src), vi->HW, hipMemcpyDefault,
                                vi->stream));
        MGDP_HIP(hipStreamSynchronize(vi->stream));
        vi->pending_src = 0;
    }
    return 0;
}
// Post the next request word: epoch, plus kServeNewCells and the tagged source word when a new
// grid is pending (source first, then the request, both release stores: x86 keeps them in order).
void post_request(mgdp_vi *vi) {
    if (++vi->epoch == 0u) ++vi->epoch;  // never 0: a batch server publishes tagged with it (publish())
    unsigned long long w = (unsigned long long)vi->epoch;
    if (vi->last_req) w |= kServeLast;
    if (vi->pending_src) {
        __atomic_store_n(vi->h_out + kHoutReq + 1, vi->pending_src | ((w & 0xffffull) << 48), __ATOMIC_RELEASE);
        w |= kServeNewCells;
        vi->pending_src = 0;
    }
    __atomic_store_n(vi->h_out + kHoutReq, w, __ATOMIC_RELEASE);
}
// Hand a new lone grid to a resident server (no drain): true if it was taken.
bool serve_handoff(mgdp_vi *vi, const void *src) {
    const unsigned long long a = (unsigned long long)(uintptr_t)src;
    if (!vi->serving || !serve_eligible(vi) || (a >> 48) != 0) return false;
    vi->pending_src = a;
    return true;
}
// Post request `epoch` (the server serves any request word != the last epoch it served) and make
// sure a server is resident; reduce_env then waits for the published result.
int serve_request(mgdp_vi *vi) {
    // A server idle for more than half its limit may be leaving: restart it deterministically
    // (quit + drain, then a fresh launch) instead of discovering its exit while polling.
    if (vi->serving) {
        const double idle_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - vi->serve_last).count();
        if (idle_us * 100.0 > 0.5 * (double)vi->serve_idle_ticks)
            if (int rc = server_stop(vi)) return rc;
    }
    post_request(vi);
    if (!vi->serving) {
        vi->exiting = false;  // a departing earlier server is no longer the stream's last work
        if (int rc = dispatch<ServeF>(vi, vi->epoch - 1u)) return rc;
        vi->serving = true;
    }
    vi->fresh = 0;
    return 0;
}

double shard_max(const unsigned long long *sh) {
    double m = 0.0;
    for (int i = 0; i < 8; ++i) {
        double v;
        std::memcpy(&v, &sh[i], sizeof(double));
        m = v > m ? v : m;
    }
    return m;
}

// Sweep method: run sweeps k_done+1.. with the device-global rule; force = run exactly to k_stop.
int sweep_run(mgdp_vi *vi, int k_stop, bool force, double *dv_out) {
    const int chunk = 8;
    std::vector<unsigned long long> host(8 * chunk);
    double dv = 0.0;
    while (vi->k_done < k_stop) {
        const size_t ev0 = vi->ev_sweep.size();
        const int n = std::min(chunk, k_stop - vi->k_done);
        for (int i = 1; i <= n; ++i)
            if (int rc = dispatch<SweepF>(vi, vi->k_done + i, force ? 0 : 1, false)) return rc;
        MGDP_HIP(hipMemcpyAsync(host.data(), vi->d_shards + (long long)vi->k_done * 8, 8 * n * sizeof(unsigned long long), hipMemcpyDeviceToHost, vi->stream));
        MGDP_HIP(hipStreamSynchronize(vi->stream));
        int last = vi->k_done + n;
        bool stop = false;
        for (int i = 0; i < n; ++i) {
            dv = shard_max(&host[8 * i]);
            if (!force && dv < vi->d.tol) {
                last = vi->k_done + i + 1;
                stop = true;
                break;
            }
        }
        for (size_t i = ev0; i < vi->ev_sweep.size(); ++i)
            if (vi->ev_sweep[i] > last) vi->ev_sweep[i] = INT32_MAX;
        vi->k_done = last;
        vi->cur = last & 1;
        if (stop) break;
    }
    if (dv_out) *dv_out = dv;
    return 0;
}

int validate_cells(const mgdp_vi_desc &d, const uint8_t *cells) {
    const int HW = d.W * d.H;
    for (int b = 0; b < d.B; ++b) {
        const uint8_t *c = cells + (int64_t)b * HW;
        int doors = 0, keys = 0;
        for (int y = 0; y < d.H; ++y)
            for (int x = 0; x < d.W; ++x) {
                const int t = c[y * d.W + x];
                const bool border = x == 0 || y == 0 || x == d.W - 1 || y == d.H - 1;
                bool ok = t == T_EMPTY || t == T_WALL || t == T_FLOOR || t == T_GOAL || t == T_LAVA;
                if (d.model == MGDP_MODEL_DOORKEY) {
                    if (t == T_DOOR) { ++doors; ok = !border; }
                    if (t == T_KEY) { ++keys; ok = !border; }
                }
                MGDP_CHECK(ok, MGDP_E_UNSUPPORTED, "grid %d cell (%d,%d): type %d is outside the %s model", b, x, y, t,
                           d.model == MGDP_MODEL_XYD ? "XYD" : "DoorKey");
                MGDP_CHECK(!(border && (t == T_EMPTY || t == T_FLOOR || (d.lava_mode == MGDP_LAVA_NODEATH && t == T_LAVA))),
                           MGDP_E_UNSUPPORTED,
                           "grid %d border cell (%d,%d) is walkable; the model needs a closed border", b, x, y);
            }
        if (d.model == MGDP_MODEL_DOORKEY)
            MGDP_CHECK(doors == 1 && keys == 1, MGDP_E_UNSUPPORTED,
                       "grid %d: DoorKey model needs exactly one door and one key (found %d, %d)", b, doors, keys);
    }
    return 0;
}

}  // namespace

extern "C" {

int mgdp_vi_num_states(const mgdp_vi_desc *d, int64_t *S) {
    MGDP_CHECK(d && S, MGDP_E_INVALID, "null argument");
    *S = (int64_t)d->W * d->H * (d->model == MGDP_MODEL_XYD ? 4 : 16);
    return 0;
}

int mgdp_vi_create(const mgdp_vi_desc *desc, mgdp_vi **out) {
    MGDP_CHECK(desc && out, MGDP_E_INVALID, "null argument");
    const mgdp_vi_desc &d = *desc;
    MGDP_CHECK(d.model == MGDP_MODEL_XYD || d.model == MGDP_MODEL_DOORKEY, MGDP_E_INVALID, "unknown model %d", d.model);
    MGDP_CHECK(d.dtype == MGDP_F32 || d.dtype == MGDP_F64, MGDP_E_INVALID, "unknown dtype %d", d.dtype);
    MGDP_CHECK(d.method == MGDP_METHOD_FUSED || d.method == MGDP_METHOD_SWEEP, MGDP_E_INVALID, "unknown method %d", d.method);
    MGDP_CHECK(d.mapping == MGDP_MAP_CELL || d.mapping == MGDP_MAP_SA, MGDP_E_INVALID, "unknown mapping %d", d.mapping);
    MGDP_CHECK(d.B > 0 && d.W >= 3 && d.H >= 3, MGDP_E_INVALID, "bad shape B=%d W=%d H=%d", d.B, d.W, d.H);
    MGDP_CHECK(d.max_sweeps > 0, MGDP_E_INVALID, "max_sweeps must be > 0");
    MGDP_CHECK(d.gamma >= 0.0 && (d.gamma < 1.0 || (d.horizon > 0 && d.gamma <= 1.0)), MGDP_E_INVALID,
               "gamma must be in [0, 1) (or [0, 1] with a finite horizon)");
    MGDP_CHECK(d.tol > 0.0, MGDP_E_INVALID, "tol must be > 0");
    MGDP_CHECK(!(d.slip_p >= 0.0 && d.model != MGDP_MODEL_XYD), MGDP_E_UNSUPPORTED,
               "slip transitions are defined for the XYD model only");
    MGDP_CHECK(d.slip_p <= 1.0, MGDP_E_INVALID, "slip_p must be <= 1");
    MGDP_CHECK(d.horizon >= 0, MGDP_E_INVALID, "horizon must be >= 0");
    MGDP_CHECK(d.lava_mode == MGDP_LAVA_TERMINAL || d.lava_mode == MGDP_LAVA_NODEATH, MGDP_E_INVALID,
               "unknown lava_mode %d", d.lava_mode);
    MGDP_CHECK(!(d.lava_mode == MGDP_LAVA_NODEATH && d.model != MGDP_MODEL_XYD), MGDP_E_UNSUPPORTED,
               "NoDeath lava is defined for the XYD model (DoorKey grids hold no lava)");
    MGDP_CHECK(!((d.flags & MGDP_KEEP_POLICY_T) && d.horizon == 0), MGDP_E_INVALID,
               "MGDP_KEEP_POLICY_T needs a finite horizon");
    MGDP_CHECK(!((d.horizon > 0 || d.lava_mode) && (d.method != MGDP_METHOD_FUSED || d.mapping != MGDP_MAP_CELL)),
               MGDP_E_UNSUPPORTED, "horizon / lava_mode options run on the fused MGDP_MAP_CELL path only");
    MGDP_CHECK(!(d.horizon > 0 && (long long)d.W * d.H > 1024), MGDP_E_UNSUPPORTED, "horizon needs W*H <= 1024");
    int ndev = 0;
    MGDP_HIP(hipGetDeviceCount(&ndev));
    MGDP_CHECK(d.device >= 0 && d.device < ndev, MGDP_E_HIP, "device %d not available (%d visible)", d.device, ndev);
    DeviceGuard guard(d.device);
    MGDP_CHECK(guard.ok, MGDP_E_HIP, "hipSetDevice(%d) failed", d.device);

    mgdp_vi *vi = new mgdp_vi();
    vi->d = d;
    vi->HW = d.W * d.H;
    vi->HWp = (int)round_up(vi->HW, 16);
    vi->S = vi->HW * (d.model == MGDP_MODEL_XYD ? 4 : 16);
    vi->HWs = vi->HW <= 1024 ? (int)round_up(vi->HW, 64) : vi->HW;
    vi->Ss = vi->S / vi->HW * vi->HWs;
    vi->A = d.model == MGDP_MODEL_XYD ? 7 : 5;
    vi->tsize = d.dtype == MGDP_F32 ? 4 : 8;
    // Two-sweep XYD step (3 LDS buffers): halves the barriers of the fused loop at 1.5x the VALU
    // work.  Off by default (MGDP_PAIR=1 enables it; tests cover both steps).
    {
        const bool eligible = d.model == MGDP_MODEL_XYD && d.mapping == MGDP_MAP_CELL && vi->HW <= 1024;
        int pair = 0;  // measured slower than the one-sweep step on MI355X (VALU chain, not barriers, bound it)
        if (const char *ev = std::getenv("MGDP_PAIR")) pair = std::atoi(ev);
        vi->pair = eligible && pair ? 1 : 0;
        // Four threads per cell (one per direction, DPP quad exchange): MGDP_QUAD=1 enables it
        // for grids with <= 256 cells (tests cover it).
        int quad = 0;  // measured slower than one thread per cell (LDS/barrier latency bound it)
        if (const char *ev = std::getenv("MGDP_QUAD")) quad = std::atoi(ev);
        vi->quad = eligible && !vi->pair && quad && 4 * vi->HW <= 1024 ? 1 : 0;
        vi->opts = d.horizon > 0 || d.lava_mode != MGDP_LAVA_TERMINAL;
        if (vi->opts) vi->pair = vi->quad = 0;  // the options kernel runs the direction-major path only
        vi->nbuf = vi->pair ? 3 : 2;
    }
    const Smem L = smem_layout(vi->Ss, vi->HWp, vi->tsize, vi->nbuf);
    if (L.total() > 160 * 1024) {
        delete vi;
        set_error("grid too large for the LDS-resident kernels (%d B > 160 KiB)", L.total());
        return MGDP_E_UNSUPPORTED;
    }
    // fused: one workgroup per grid.  MAP_CELL: one thread per cell (register topology) when the
    // grid has <= 1024 cells; MAP_SA: 8 lanes per state, a lone grid gets the widest workgroup.
    if (d.mapping == MGDP_MAP_CELL) {
        vi->fused_block = (int)std::min<int64_t>(1024, round_up(vi->HW * (vi->quad ? 4 : 1), 64));
        // A lone XYD grid of <= 64*MGDP_WAVE cells runs on ONE wave, P = 1, 2, 4 or 8 cells per
        // lane: no workgroup barrier per sweep, the stopping rule is a wave ballot.  Measured per
        // sweep against the multi-wave loop: P = 1 faster (0.10 vs 0.12 us), P = 2 even, P = 4 and 8
        // slower (0.27 vs 0.17, 0.55 vs 0.18 us: one SIMD issues every cell's VALU work), so the
        // default is P = 1 (grids of <= 64 cells); MGDP_WAVE=8 enables the rest (tests cover them).
        int wave_max = 1;
        if (const char *ev = std::getenv("MGDP_WAVE")) wave_max = std::atoi(ev);
        if (d.B == 1 && d.model == MGDP_MODEL_XYD && d.method == MGDP_METHOD_FUSED && !vi->pair && !vi->quad &&
            !vi->opts && vi->HW <= 64 * std::min(wave_max, 8)) {
            int P = 1;
            while (64 * P < vi->HW) P *= 2;
            vi->wave_p = P;
            vi->HWs = 64 * P;
            vi->Ss = vi->S / vi->HW * vi->HWs;
            vi->fused_block = 64;
        }
        // Batched XYD grids: N cells per thread divides the waves per grid by N (MGDP_CPT=1|2|4;
        // measured on MI355X, profiles/r01_cpt/: 2 beats 1 by 7-25 %).
        int cpt = 2;
        if (const char *ev = std::getenv("MGDP_CPT")) cpt = std::atoi(ev);
        int lone_cpt = 1;  // a lone grid (latency) keeps one cell per thread unless MGDP_LONE_CPT=2
        if (const char *ev = std::getenv("MGDP_LONE_CPT")) lone_cpt = std::atoi(ev) == 2 ? 2 : 1;
        if (vi->wave_p) cpt = 1;
        else if (d.B == 1) cpt = lone_cpt;
        if ((cpt == 2 || cpt == 4) && d.model == MGDP_MODEL_XYD && d.method == MGDP_METHOD_FUSED &&
            !vi->pair && !vi->quad && !vi->opts && vi->HW <= 1024) {
            vi->cpt = cpt;
            vi->fused_block = (int)round_up((vi->HW + cpt - 1) / cpt, 64);
            vi->HWs = cpt * vi->fused_block;
            vi->Ss = vi->S / vi->HW * vi->HWs;
        }
        if (const char *ev = std::getenv("MGDP_PAIR2")) vi->pair2 = std::atoi(ev) != 0;
        // Batched deterministic XYD grids: one wave per grid, no workgroup barrier (fused_wave2_xyd)
        // up to MGDP_WAVE2 cells per lane (0 disables it).
        int wave2_max = 8;
        if (const char *ev = std::getenv("MGDP_WAVE2")) wave2_max = std::atoi(ev);
        const int P2 = (vi->HW + 63) / 64;
        if (d.B > 1 && d.model == MGDP_MODEL_XYD && d.method == MGDP_METHOD_FUSED && d.slip_p < 0.0 && !vi->pair &&
            !vi->quad && !vi->opts && !vi->wave_p && P2 <= std::min(wave2_max, 8)) {
            vi->wave2 = P2;
            vi->cpt = 1;
            vi->fused_block = 64;
            vi->HWs = (int)round_up(vi->HW, 64);
            vi->Ss = vi->S / vi->HW * vi->HWs;
        }
        if (vi->wave2) {
            int cus = 0;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d.device);
            // Two waves per grid (MGDP_WAVE2N=1, grids of >= 3 blocks of 64 cells): measured slower
            // than one wave per grid even where one wave per grid leaves the SIMDs short of waves --
            // FourRooms x 4096: 64-65 us per solve (74 VGPRs, 6 waves / SIMD) or 57 us compiled for
            // 8 waves / SIMD, vs 55-56 us on one wave (profiles/r04_w2nab/) -- so it is off by default.
            int w2n = 0;
            if (const char *ev = std::getenv("MGDP_WAVE2N")) w2n = std::atoi(ev) != 0 && vi->wave2 >= 3;
            if (w2n) {
                vi->wave2n = (vi->wave2 + 1) / 2;
                vi->fused_block = 128;
            }
            if (const char *ev = std::getenv("MGDP_MIX"))
                vi->mix = std::atoi(ev) != 0 && !vi->wave2n && d.dtype == MGDP_F32 && vi->wave2 >= 2 && vi->wave2 <= 6;
            if (const char *ev = std::getenv("MGDP_MIX_FRAC")) vi->mix_frac = std::atof(ev);
            if (vi->mix) vi->fused_block = 128;
            // Column bands instead of row-major blocks (fused_band_xyd: north / south fronts in
            // registers, no LDS tile): MGDP_BAND=1 (A/B; off by default until measured per size)
            int band_on = 0;
            if (const char *ev = std::getenv("MGDP_BAND")) band_on = std::atoi(ev);
            const int hb = band_rows(d.W, d.H);
            if (band_on && !vi->wave2n && !vi->mix && hb >= 1 && hb <= 8) vi->band = hb;
            // The in-launch reduction (GkCtx) while the batch is resident at once (MGDP_GK=2, the
            // default).  Since fixed-point completion no grid waits for another, so the counter tree
            // would work for any B (MGDP_GK=1), but past the resident capacity every grid's exit
            // waits for its counter's atomic while the next grid could start: LavaS11N5 x 65536
            // 153 vs 144-145 us per launch, Empty-16 x 65536 314-319 vs 309-312
            // (profiles/r05_mix/) -- the reduce kernel is cheaper there.  MGDP_GK=0: never.
            int gk_on = 2;
            if (const char *ev = std::getenv("MGDP_GK")) gk_on = std::atoi(ev);
            const bool f32 = d.dtype == MGDP_F32;
            const void *k2 = nullptr;
            int smem2 = 0;
            if (vi->band) {
                smem2 = 256 + (vi->HWp + 15) / 16 * 16;
                k2 = f32 ? (const void *)pick_band<FusedK, float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->band, FusedK<float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn)
                         : (const void *)pick_band<FusedK, double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->band, FusedK<double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn);
            } else if (vi->mix) {
                smem2 = mix_smem_bytes(vi->HWp, d.W, vi->wave2, vi->tsize);
                k2 = (const void *)pick_mix<FusedK, float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                    vi->wave2, FusedK<float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn);
            } else if (vi->wave2n) {
                smem2 = wave2n_smem_bytes(vi->HWp, d.W, 2 * vi->wave2n, vi->tsize);
                k2 = f32 ? (const void *)pick_wave2n<FusedK, float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->wave2n, FusedK<float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn)
                         : (const void *)pick_wave2n<FusedK, double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->wave2n, FusedK<double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn);
            } else {
                smem2 = wave2_smem_bytes(vi->HWp, d.W, vi->wave2, vi->tsize);
                k2 = f32 ? (const void *)pick_wave2<FusedK, float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->wave2, FusedK<float, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn)
                         : (const void *)pick_wave2<FusedK, double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL>(
                               vi->wave2, FusedK<double, MGDP_MODEL_XYD, false, MGDP_MAP_CELL, 0>::fn);
            }
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k2, vi->fused_block, smem2) == hipSuccess)
                vi->gk_capacity = per_cu * cus;
            vi->gk = gk_on == 1 || (gk_on == 2 && d.B <= vi->gk_capacity);
            // the resident batch server runs the same loop (wave2 layout, in-launch reduction)
            if (const char *ev = std::getenv("MGDP_BSERVE")) {
                vi->bserve = std::atoi(ev) != 0;
                vi->bserve_any = std::atoi(ev) == 2;
            }
            if (const char *ev = std::getenv("MGDP_BSERVE_COPIES")) vi->bserve_copies = std::min(kBreqCopies, std::max(1, std::atoi(ev)));
            if (const char *ev = std::getenv("MGDP_BSERVE_NAP")) vi->bserve_nap = std::min(64, std::max(0, std::atoi(ev)));
            if (const char *ev = std::getenv("MGDP_BSERVE_WAIT_PUB")) vi->bserve_wait_pub = std::atoi(ev) != 0;
            if (const char *ev = std::getenv("MGDP_BSERVE_PRIO_FRAC")) vi->bserve_prio_frac = std::min(1.0, std::max(0.0, std::atof(ev)));
            if (vi->bserve && (vi->gk || vi->bserve_any) && !vi->band && !vi->mix && !vi->wave2n && d.slip_p < 0.0 && d.B > 1) {
                const void *kb = f32 ? pick_bserve<float>(vi->wave2) : pick_bserve<double>(vi->wave2);
                int per_cu = 0;
                if (kb && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kb, 64, smem2) == hipSuccess)
                    vi->bserve_cap = per_cu * cus;
            }
        }
        // The served lone deterministic XYD grid: east / west fronts by DPP, <= 4 waves (one dword
        // of stop flags); the two-plane padded tiles must fit the usual V buffers.
        int serve_ew = 1;
        if (const char *ev = std::getenv("MGDP_SERVE_EW")) serve_ew = std::atoi(ev);
        const int padw = serve_ew_padw(d.W);
        vi->serve_ew = serve_ew && d.B == 1 && d.model == MGDP_MODEL_XYD && d.method == MGDP_METHOD_FUSED &&
                       d.slip_p < 0.0 && !vi->pair && !vi->quad && !vi->opts && !vi->wave_p && vi->cpt == 1 &&
                       vi->fused_block <= 256 && vi->HWs >= vi->fused_block && 2 * vi->HWs >= 3 * padw;
        // ... with two sweeps per workgroup barrier (fused_serve_pair): its two four-plane tiles take the
        // first V buffers (nbuf raised to hold them; MGDP_SERVE_PAIR=0: off)
        int serve_pair = 1;
        if (const char *ev = std::getenv("MGDP_SERVE_PAIR")) serve_pair = std::atoi(ev);
        if (vi->serve_ew && serve_pair) {
            const int need = 2 * serve_pair_tile_elems(vi->HWs, d.W);
            const int nbuf = std::max(2, (need + vi->Ss - 1) / vi->Ss);
            if (smem_layout(vi->Ss, vi->HWp, vi->tsize, nbuf).total() <= 64 * 1024) {
                vi->serve_pair = 1;
                vi->nbuf = nbuf;
            }
        }
        // The served lone deterministic XYD grid on ONE wave in column bands (fused_band_xyd: no
        // barrier, no LDS tile; MGDP_SERVE_BAND=1, A/B)
        int serve_band = 0;
        if (const char *ev = std::getenv("MGDP_SERVE_BAND")) serve_band = std::atoi(ev);
        const int hb1 = band_rows(d.W, d.H);
        if (serve_band && d.B == 1 && d.model == MGDP_MODEL_XYD && d.method == MGDP_METHOD_FUSED && d.slip_p < 0.0 &&
            !vi->pair && !vi->quad && !vi->opts && hb1 >= 1 && hb1 <= 8) {
            vi->band = hb1;
            vi->serve_ew = 0;
            if (vi->serve_pair) vi->nbuf = 2;
            vi->serve_pair = 0;
            vi->wave_p = 0;
            vi->cpt = 1;
            vi->fused_block = 64;
        }
        int dk1t = 0;
        if (const char *ev = std::getenv("MGDP_DK_1T")) dk1t = std::atoi(ev) != 0;
        if (dk1t && d.B > 1 && d.model == MGDP_MODEL_DOORKEY && d.dtype == MGDP_F32 && d.method == MGDP_METHOD_FUSED &&
            !vi->opts && vi->HW <= vi->fused_block) {
            vi->dk1t = 1;
            vi->nbuf = 1;  // one V tile in LDS
        }
        // Batched DoorKey grids of <= 512 cells: each cell's 16 states over two threads split by
        // has_key (fused_dk_half).  Default for fp64 and for lone grids: measured on DoorKey-16
        // (profiles/r02_dk_half/), x 65536 fp64 9.9e12 vs 2.8e12 updates/s (the one-thread-per-cell
        // fp64 loop spills: 138 VGPRs of scratch) but fp32 1.90e13 vs 2.22e13 (the same 4 grids per
        // CU, LDS-bound, with twice the LDS instructions); a lone grid, served: fp32 26.1 vs
        // 28.4 us, fp64 34.8 vs 85.0 us per solve.  MGDP_DK_HALF=0|1 forces it off / on.
        int dkhalf = (d.dtype == MGDP_F64 || d.B == 1) ? 1 : 0;
        if (const char *ev = std::getenv("MGDP_DK_HALF")) dkhalf = std::atoi(ev) != 0;
        if (dkhalf && !vi->dk1t && d.model == MGDP_MODEL_DOORKEY && d.method == MGDP_METHOD_FUSED &&
            !vi->opts && vi->HW <= 512) {
            vi->dkhalf = 1;
            vi->HWs = (int)round_up(vi->HW, 64);
            vi->Ss = vi->S / vi->HW * vi->HWs;
            vi->fused_block = 2 * vi->HWs;
        }
        // Batched DoorKey grids of width 16 (DoorKey-16x16): whole grid rows per 16 lanes, east / west
        // fronts by DPP, two conflict-free LDS planes (fused_dk_rows).  The special-first cell map of
        // fused_fast_dk_soa spent half its LDS-array cycles on bank conflicts (round-4 counters).
        // MGDP_DK_ROWS=0 keeps fused_fast_dk_soa.
        int dkrow = 1;
        if (const char *ev = std::getenv("MGDP_DK_ROWS")) dkrow = std::atoi(ev) != 0;
        if (dkrow && !vi->dk1t && !vi->dkhalf && d.B > 1 && d.model == MGDP_MODEL_DOORKEY &&
            d.method == MGDP_METHOD_FUSED && d.slip_p < 0.0 && !vi->opts && !vi->pair && !vi->quad && d.W == 16 &&
            vi->HW <= 1024) {
            vi->dkrow = 1;
            vi->HWs = (int)round_up(vi->HW, 64);
            vi->Ss = vi->S / vi->HW * vi->HWs;
            vi->fused_block = vi->HWs;
        }
    } else {
        int blk = d.B == 1 ? 1024 : 256;
        while (blk > 64 && blk / 2 >= vi->S * 8) blk /= 2;
        vi->fused_block = blk;
    }

    const size_t BS = (size_t)d.B * vi->S;
    hipError_t e = hipSuccess;
    auto al = [&](void **p, size_t n) { if (e == hipSuccess) e = hipMalloc(p, n); };
    al((void **)&vi->d_cells, (size_t)d.B * vi->HWp);
    al(&vi->d_V[0], BS * vi->tsize);
    if (d.method == MGDP_METHOD_SWEEP) al(&vi->d_V[1], BS * vi->tsize);
    al((void **)&vi->d_pi, BS);
    al((void **)&vi->d_kenv, sizeof(int32_t) * d.B);
    al((void **)&vi->d_kexec, sizeof(int32_t) * d.B);
    if (e == hipSuccess) e = hipMemset(vi->d_kexec, 0, sizeof(int32_t) * d.B);
    al((void **)&vi->d_dvenv, sizeof(double) * d.B);
    al((void **)&vi->d_shards, sizeof(unsigned long long) * 8 * (size_t)(d.max_sweeps + 1));
    al((void **)&vi->d_red, sizeof(unsigned long long) * (kRedShards * 4 + 2));
    al((void **)&vi->d_pub1, sizeof(unsigned long long) * 4);
    if (vi->gk || (vi->bserve && vi->bserve_cap > 0 && vi->bserve_any)) {
        al((void **)&vi->d_gk, sizeof(unsigned long long) * gk_words(d.B));
        if (e == hipSuccess) e = hipMemset(vi->d_gk, 0, sizeof(unsigned long long) * gk_words(d.B));
    }
    if (vi->bserve && vi->bserve_cap > 0 && (d.B <= vi->bserve_cap || vi->bserve_any)) {
        al((void **)&vi->d_breq, sizeof(unsigned long long) * kBreqWords);
        if (e == hipSuccess) e = hipMemset(vi->d_breq, 0, sizeof(unsigned long long) * kBreqWords);
    }
    if (d.horizon > 0) {
        al(&vi->d_rgoal, (size_t)d.horizon * vi->tsize);
        if (d.flags & MGDP_KEEP_POLICY_T) al((void **)&vi->d_pi_t, (size_t)d.horizon * BS);
        if (e == hipSuccess) {  // goal reward of step_count t+1: _reward(), minigrid_env.py:235-240
            std::vector<unsigned char> rg((size_t)d.horizon * vi->tsize);
            for (int t = 0; t < d.horizon; ++t) {
                const double r = 1.0 - 0.9 * ((double)(t + 1) / (double)d.horizon);
                if (vi->tsize == 4) reinterpret_cast<float *>(rg.data())[t] = (float)r;
                else reinterpret_cast<double *>(rg.data())[t] = r;
            }
            e = hipMemcpy(vi->d_rgoal, rg.data(), rg.size(), hipMemcpyHostToDevice);
        }
    }
    if (e == hipSuccess) e = hipHostMalloc((void **)&vi->h_out, kHoutWords * sizeof(unsigned long long),
                                           hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&vi->d_hout, vi->h_out, 0);
    if (e == hipSuccess && d.B == 1) {
        e = hipHostMalloc((void **)&vi->h_stage, (size_t)vi->HWp, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&vi->d_stage, vi->h_stage, 0);
    }
    if (e == hipSuccess) {
        e = hipStreamCreateWithFlags(&vi->stream, hipStreamNonBlocking);
        vi->own_stream = e == hipSuccess;
    }
    if (e == hipSuccess) e = hipMemset(vi->d_cells, 0, (size_t)d.B * vi->HWp);
    if (const char *ev = std::getenv("MGDP_SWEEP_M")) vi->sweep_m = std::max(1, std::atoi(ev));
    // keep the staged group within the LDS budget (two groups per CU at least)
    while (vi->sweep_m > 1 && sweep_smem_bytes(vi->S, vi->HWp, vi->tsize, vi->sweep_m) > 80 * 1024) --vi->sweep_m;
    if (const char *ev = std::getenv("MGDP_SWEEP_GRID")) vi->sweep_grid = std::max(1, std::atoi(ev));
    if (const char *ev = std::getenv("MGDP_SWEEP_BLOCK")) vi->sweep_block = std::min(256, std::max(64, std::atoi(ev) / 64 * 64));
    if (const char *ev = std::getenv("MGDP_PERSISTENT")) vi->persistent = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_CHAIN")) vi->chain = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_LEARN_ORDER")) vi->learn_order = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_LEARN_PRIO")) vi->learn_prio = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_ORDER")) vi->order_src = std::strcmp(ev, "learned") == 0 ? 2 : (std::strcmp(ev, "off") == 0 ? 0 : 1);
    if (const char *ev = std::getenv("MGDP_REDUCE_MULTI")) vi->reduce_multi = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_INKERNEL_MAX")) vi->inkernel_max = std::max(0, std::atoi(ev));
    // DoorKey (64-128 B of V per thread) measured slower on the register pipeline (5.38 -> 3.3 TB/s
    // compulsory: the prefetch registers collide with the 16-state backup's), so it keeps the
    // staged kernel unless MGDP_SWEEP_PIPE asks otherwise.
    if (d.model == MGDP_MODEL_DOORKEY) vi->sweep_pipe = 0;
    if (const char *ev = std::getenv("MGDP_SWEEP_PIPE")) vi->sweep_pipe = std::min(4, std::max(0, std::atoi(ev)));
    if (vi->HW > 1024 || d.mapping != MGDP_MAP_CELL ||
        sweep_pipe_smem_bytes(vi->S, vi->HW, vi->HWs, vi->HWp, vi->tsize) > 160 * 1024)
        vi->sweep_pipe = 0;  // one thread per cell: grids of <= 1024 cells
    if (const char *ev = std::getenv("MGDP_SERVE_IDLE_US"))  // s_memrealtime ticks at 100 MHz
        vi->serve_idle_ticks = (unsigned long long)std::max(1LL, std::atoll(ev)) * 100ull;
    if (const char *ev = std::getenv("MGDP_SERVE_POLLERS")) vi->serve_pollers = std::max(1, std::atoi(ev));
    if (const char *ev = std::getenv("MGDP_SERVE_POLL_DMA")) vi->serve_poll_dma = std::atoi(ev) != 0;
    if (const char *ev = std::getenv("MGDP_SERVE_LIFE_US"))
        vi->serve_life_ticks = (unsigned long long)std::max(1LL, std::atoll(ev)) * 100ull;
    if (vi->h_out) std::memset(vi->h_out, 0, kHoutWords * sizeof(unsigned long long));
    if (e == hipSuccess) {  // arm the fused reduction (every launch re-arms it for the next)
        std::vector<unsigned long long> init((size_t)kRedShards * 4 + 2, 0ull);
        for (size_t i = 2; i < (size_t)kRedShards * 4; i += 4) init[i] = 0x7fffffffull;
        e = hipMemcpy(vi->d_red, init.data(), init.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
        vi->d_ticket = reinterpret_cast<unsigned int *>(vi->d_red + kRedShards * 4);
    }
    if (e != hipSuccess) {
        mgdp_vi_destroy(vi);
        return hip_fail(e, "mgdp_vi_create allocation", __FILE__, __LINE__);
    }
    *out = vi;
    return mgdp_vi_reset(vi);
}

int mgdp_vi_destroy(mgdp_vi *vi) {
    if (!vi) return 0;
    DeviceGuard guard(vi->d.device);
    (void)server_stop(vi);
    if (vi->stream) (void)hipStreamSynchronize(vi->stream);
    for (auto &p : vi->ev) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    for (auto &p : vi->ev_pool) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    (void)hipFree(vi->d_cells);
    (void)hipFree(vi->d_V[0]);
    (void)hipFree(vi->d_V[1]);
    (void)hipFree(vi->d_pi);
    (void)hipFree(vi->d_kenv);
    (void)hipFree(vi->d_kexec);
    (void)hipFree(vi->d_order);
    (void)hipFree(vi->d_dvenv);
    (void)hipFree(vi->d_shards);
    (void)hipFree(vi->d_red);
    (void)hipFree(vi->d_pub1);
    (void)hipFree(vi->d_gk);
    (void)hipFree(vi->d_breq);
    (void)hipFree(vi->d_rgoal);
    (void)hipFree(vi->d_pi_t);
    if (vi->h_out) (void)hipHostFree(vi->h_out);
    if (vi->h_stage) (void)hipHostFree(vi->h_stage);
    if (vi->own_stream) (void)hipStreamDestroy(vi->stream);
    delete vi;
    return 0;
}

int mgdp_vi_set_stream(mgdp_vi *vi, void *s) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    if (vi->own_stream) { (void)hipStreamDestroy(vi->stream); vi->own_stream = false; vi->stream = nullptr; }
    if (s) {
        vi->stream = (hipStream_t)s;
    } else {
        MGDP_HIP(hipStreamCreateWithFlags(&vi->stream, hipStreamNonBlocking));
        vi->own_stream = true;
    }
    return 0;
}

namespace {
int cells_dispatch(mgdp_vi *vi);  // the dispatch order from the cells just loaded (below)
}  // namespace

int mgdp_vi_load_cells(mgdp_vi *vi, const uint8_t *cells) {
    MGDP_CHECK(vi && cells, MGDP_E_INVALID, "null argument");
    if (int rc = validate_cells(vi->d, cells)) return rc;
    // a resident lone-grid server takes the grid with its next request: staged in host memory
    // (a solve is synchronous, so the server is not reading the staging buffer now)
    if (vi->h_stage && vi->serving && serve_eligible(vi)) {
        std::memcpy(vi->h_stage, cells, vi->HW);
        if (serve_handoff(vi, vi->d_stage)) {
            vi->cells_loaded = true;
            vi->k_done_valid = false;
            return 0;
        }
    }
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    std::vector<uint8_t> pad((size_t)vi->d.B * vi->HWp, 0);
    for (int b = 0; b < vi->d.B; ++b) std::memcpy(&pad[(size_t)b * vi->HWp], cells + (size_t)b * vi->HW, vi->HW);
    MGDP_HIP(hipMemcpyAsync(vi->d_cells, pad.data(), pad.size(), hipMemcpyHostToDevice, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    vi->cells_loaded = true;
    vi->k_done_valid = false;
    vi->order_valid = false;
    vi->solves_since_load = 0;
    return cells_dispatch(vi);
}

int mgdp_vi_load_cells_device(mgdp_vi *vi, const uint8_t *d_cells) {
    MGDP_CHECK(vi && d_cells, MGDP_E_INVALID, "null argument");
    // The resident server reads the bytes itself with its next request, unordered with respect to
    // any stream: only on the handle's own stream, where no caller kernel can still be producing
    // them.  On a caller-bound stream (mgdp_vi_set_stream) the copy below is ordered after whatever
    // the caller enqueued there before this call.
    if (vi->own_stream && serve_handoff(vi, d_cells)) {
        vi->cells_loaded = true;
        vi->k_done_valid = false;
        return 0;
    }
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipMemcpy2DAsync(vi->d_cells, vi->HWp, d_cells, vi->HW, vi->HW, vi->d.B, hipMemcpyDeviceToDevice, vi->stream));
    vi->cells_loaded = true;
    vi->k_done_valid = false;
    vi->order_valid = false;
    vi->solves_since_load = 0;
    return cells_dispatch(vi);
}

namespace {
// Dispatch order (Geo::order / kprio): the grids ranked longest first in dispatch order (an LPT
// schedule: the launch's tail holds short grids, and at full residency every CU gets a stratified
// mix), and optionally (learn_prio) the top 1 / 10 / 50 % raise their waves' issue priority.  The
// key per grid is (order_src) 1 = its cells' depth proxy (vi_depth_kernel, computed at each cells
// load: the order holds from the first solve of fresh grids), 2 = the sweeps it executed in the
// previous solve (d_kexec; round 5's learned order, from the second solve on).  V, pi and the sweep
// counts never depend on it.
constexpr int kLearnMinB = 1024;
int set_order(mgdp_vi *vi, const std::vector<int32_t> &kx) {
    const int B = vi->d.B;
    std::vector<int32_t> idx(B);
    for (int i = 0; i < B; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return kx[a] > kx[b]; });
    if (!vi->d_order) MGDP_HIP(hipMalloc((void **)&vi->d_order, sizeof(int32_t) * (size_t)B));
    MGDP_HIP(hipMemcpyAsync(vi->d_order, idx.data(), sizeof(int32_t) * (size_t)B, hipMemcpyHostToDevice, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    const int t1 = kx[idx[B / 100]], t10 = kx[idx[B / 10]], t50 = kx[idx[B / 2]];
    if (t50 > 0 && t1 > t50) {
        vi->kprio[0] = t1;
        vi->kprio[1] = std::max(t10, t50 + 1);
        vi->kprio[2] = t50 + 1;
    } else {
        vi->kprio[0] = vi->kprio[1] = vi->kprio[2] = 0;  // no spread to exploit
    }
    // mixed wave counts: the grids with keys >= mix_frac x the largest on two waves (they are the
    // first workgroups of the order just set)
    vi->nmix = 0;
    if (vi->mix && kx[idx[0]] > 0) {
        const int thr = std::max(1, (int)std::ceil(vi->mix_frac * kx[idx[0]]));
        while (vi->nmix < B && kx[idx[vi->nmix]] >= thr) ++vi->nmix;
    }
    vi->order_valid = true;
    return 0;
}
bool order_eligible(const mgdp_vi *vi) {
    return vi->order_src != 0 && (vi->learn_order || vi->learn_prio) && vi->d.B >= kLearnMinB &&
           vi->d.method == MGDP_METHOD_FUSED && !vi->opts && !serve_eligible(vi);
}
// order_src 2: from the executed sweeps of the previous solve
int learn_dispatch(mgdp_vi *vi) {
    std::vector<int32_t> kx(vi->d.B);
    MGDP_HIP(hipMemcpyAsync(kx.data(), vi->d_kexec, sizeof(int32_t) * (size_t)vi->d.B, hipMemcpyDeviceToHost, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return set_order(vi, kx);
}
// order_src 1: from the cells just loaded (one small launch, a D2H copy of B words and a sort)
int cells_dispatch(mgdp_vi *vi) {
    if (!order_eligible(vi) || vi->order_src != 1 || vi->HW > kDepthMaxHW) return 0;
    int32_t *d_depth = nullptr;
    MGDP_HIP(hipMallocAsync((void **)&d_depth, sizeof(int32_t) * (size_t)vi->d.B, vi->stream));
    hipLaunchKernelGGL(vi_depth_kernel, dim3(vi->d.B), dim3(64), 0, vi->stream, make_geo(vi),
                       (const uint8_t *)vi->d_cells, (int)vi->d.model, d_depth);
    hipError_t e = hipGetLastError();
    std::vector<int32_t> kx(vi->d.B);
    if (e == hipSuccess) e = hipMemcpyAsync(kx.data(), d_depth, sizeof(int32_t) * (size_t)vi->d.B, hipMemcpyDeviceToHost, vi->stream);
    if (e == hipSuccess) e = hipFreeAsync(d_depth, vi->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(vi->stream);
    if (e != hipSuccess) return hip_fail(e, "dispatch order from the cells", __FILE__, __LINE__);
    return set_order(vi, kx);
}
}  // namespace

int mgdp_vi_reset(mgdp_vi *vi) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (!vi->order_valid && vi->order_src == 2 && vi->solves_since_load > 0 && order_eligible(vi)) {
        if (int rc = server_stop(vi)) return rc;
        if (int rc = learn_dispatch(vi)) return rc;
    }
    if (vi->d.method == MGDP_METHOD_SWEEP) {  // V_0 = 0 and an empty dV trace
        const size_t BS = (size_t)vi->d.B * vi->S;
        MGDP_HIP(hipMemsetAsync(vi->d_V[0], 0, BS * vi->tsize, vi->stream));
        MGDP_HIP(hipMemsetAsync(vi->d_shards, 0, sizeof(unsigned long long) * 8 * (size_t)(vi->d.max_sweeps + 1), vi->stream));
    }
    vi->fresh = 1;  // the next fused launch ignores kenv/dvenv and starts from V_0 = 0
    vi->cur = 0;
    vi->k_done = 0;
    vi->k_min = 0;
    vi->k_done_valid = false;
    vi->sweeps = 0;
    vi->converged = 0;
    return 0;
}

int mgdp_vi_run_local(mgdp_vi *vi, int32_t *k_local_max) {
    MGDP_CHECK(vi && k_local_max, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->cells_loaded, MGDP_E_INVALID, "no cells loaded");
    DeviceGuard guard(vi->d.device);
    if (vi->d.method == MGDP_METHOD_FUSED) {
        // the batch server only for mgdp_vi_solve's own run_local: a caller driving run_local / run_to
        // itself (a collective protocol) may enqueue device work between them that needs the CU slots a
        // resident batch server holds
        const bool serve = (serve_eligible(vi) || (vi->solving && bserve_eligible(vi))) && vi->fresh;
        if (serve) {
            if (int rc = serve_request(vi)) return rc;
        } else {
            if (int rc = server_stop(vi)) return rc;
            // a finite horizon is exactly H backward sweeps from V_H = 0
            if (vi->d.horizon > 0) MGDP_CHECK(vi->fresh, MGDP_E_INVALID, "finite horizon: call mgdp_vi_reset first");
            if (int rc = dispatch<FusedF>(vi, vi->d.horizon > 0 ? vi->d.horizon : -1)) return rc;
        }
        int32_t km;
        if (int rc = reduce_env(vi, &km, nullptr)) return rc;
        if (serve) vi->serve_last = std::chrono::steady_clock::now();
        *k_local_max = km;
        return 0;
    }
    double dv = 0.0;
    if (int rc = sweep_run(vi, vi->d.max_sweeps, false, &dv)) return rc;
    vi->k_min = vi->k_max = vi->k_done;  // the sweep method stops the whole batch at once
    vi->dv_red = dv;
    vi->k_done_valid = true;
    *k_local_max = vi->k_done;
    return 0;
}

int mgdp_vi_run_to(mgdp_vi *vi, int32_t k_target, double *dv_out) {
    MGDP_CHECK(vi && dv_out, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(k_target >= 0 && k_target <= vi->d.max_sweeps, MGDP_E_INVALID, "k_target %d out of range", k_target);
    DeviceGuard guard(vi->d.device);
    if (vi->d.method == MGDP_METHOD_FUSED) {
        // every grid is already there: at k_target, or every grid at an exact fixed point (the
        // largest |dV| of the last launch is 0) at or below it -- fixed-point completion (fused_grid):
        // its V and pi are those of every later sweep, so no launch is needed
        const bool all_fixed = vi->dv_red == 0.0 && vi->k_min > 0 && vi->k_max <= k_target && vi->d.horizon == 0;
        if (vi->k_done_valid && (vi->k_min == k_target || all_fixed)) {
            vi->k_done = vi->k_min = vi->k_max = k_target;
            *dv_out = vi->dv_red;
            return 0;
        }
        MGDP_CHECK(vi->d.horizon == 0, MGDP_E_INVALID,
                   "finite horizon: the DP is exactly H sweeps (mgdp_vi_run_local / mgdp_vi_solve)");
        if (int rc = server_stop(vi)) return rc;
        if (int rc = dispatch<FusedF>(vi, k_target)) return rc;
        int32_t km;
        if (int rc = reduce_env(vi, &km, dv_out)) return rc;
        MGDP_CHECK(km == k_target, MGDP_E_INVALID, "run_to(%d): a grid is already at sweep %d", k_target, km);
        vi->k_done = k_target;
        return 0;
    }
    MGDP_CHECK(k_target >= vi->k_done, MGDP_E_INVALID, "run_to(%d) behind sweep %d", k_target, vi->k_done);
    if (k_target == vi->k_done) {
        std::vector<unsigned long long> sh(8);
        if (k_target == 0) { *dv_out = 0.0; return 0; }
        MGDP_HIP(hipMemcpy(sh.data(), vi->d_shards + (long long)(k_target - 1) * 8, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        *dv_out = shard_max(sh.data());
        return 0;
    }
    return sweep_run(vi, k_target, true, dv_out);
}

// Multi-GPU device protocol (distributed.py): the two launches of a sharded solve are enqueued on
// the handle's stream with their results in a caller-owned device buffer, so the all-reduces
// between them (RCCL, ordered on the same stream) need no host round trip; the host reads K and dV
// once at the end and hands them back with mgdp_vi_set_result.
int mgdp_vi_run_local_dev(mgdp_vi *vi, int64_t *d_pub) {
    MGDP_CHECK(vi && d_pub, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->cells_loaded, MGDP_E_INVALID, "no cells loaded");
    MGDP_CHECK(vi->d.method == MGDP_METHOD_FUSED && !vi->opts, MGDP_E_UNSUPPORTED,
               "the device protocol runs the fused method without horizon / lava options");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    vi->k_done_valid = false;
    return dispatch<FusedF>(vi, -1, reinterpret_cast<unsigned long long *>(d_pub), (const long long *)nullptr);
}

int mgdp_vi_run_to_dev(mgdp_vi *vi, const int64_t *d_k, int64_t *d_pub) {
    MGDP_CHECK(vi && d_k && d_pub, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->d.method == MGDP_METHOD_FUSED && !vi->opts, MGDP_E_UNSUPPORTED,
               "the device protocol runs the fused method without horizon / lava options");
    MGDP_CHECK(!vi->fresh, MGDP_E_INVALID, "mgdp_vi_run_to_dev before mgdp_vi_run_local_dev");
    DeviceGuard guard(vi->d.device);
    vi->k_done_valid = false;
    return dispatch<FusedF>(vi, 0, reinterpret_cast<unsigned long long *>(d_pub), reinterpret_cast<const long long *>(d_k));
}

int mgdp_vi_run_to_dev_sync(mgdp_vi *vi, const int64_t *d_kdv, int32_t *k_out, double *dv_out, double *dv_rule_out) {
    MGDP_CHECK(vi && d_kdv, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->d.method == MGDP_METHOD_FUSED && !vi->opts, MGDP_E_UNSUPPORTED,
               "the device protocol runs the fused method without horizon / lava options");
    MGDP_CHECK(!vi->fresh, MGDP_E_INVALID, "mgdp_vi_run_to_dev_sync before mgdp_vi_run_local_dev");
    DeviceGuard guard(vi->d.device);
    vi->k_done_valid = false;
    int32_t km = 0;
    double dv = 0.0;
    // The gate (one wave): with E = d_kdv[1] == 0 every grid of every rank stopped its own rule at an
    // exact fixed point, so every grid is at K already (fixed-point completion) and the gate
    // publishes the result {K, dV 0}; else it publishes "more" and run_to(K) follows.  Either way
    // E goes to h_out[12..13] and the host waits on host-mapped words only.
    hipLaunchKernelGGL(vi_gate_kernel, dim3(1), dim3(64), 0, vi->stream, reinterpret_cast<const long long *>(d_kdv),
                       vi->d_hout, next_host_epoch(vi));
    MGDP_HIP(hipGetLastError());
    if (int rc = reduce_env(vi, &km, &dv)) return rc;
    if (vi->k_min != km) {
        // result -> host-mapped words (reduce_env polls them), d_kdv[1] -> h_out[12..13] by the launch
        if (int rc = dispatch<FusedF>(vi, 0, (unsigned long long *)nullptr, reinterpret_cast<const long long *>(d_kdv),
                                      vi->d_hout + 12))
            return rc;
        if (int rc = reduce_env(vi, &km, &dv)) return rc;
    }
    MGDP_CHECK(vi->k_min == km, MGDP_E_INVALID, "run_to_dev_sync: grids ended at sweeps %d..%d, not at one common K",
               vi->k_min, km);
    vi->k_done = km;
    // the mirror's two tagged words were stored with the result's (no order between them)
    const volatile unsigned long long *h = vi->h_out;
    const unsigned long long ep = (unsigned long long)vi->epoch;
    for (uint64_t spin = 1; (h[12] >> 32) != ep || (h[13] >> 32) != ep; ++spin) {
        if ((spin & 1023u) == 0u) {
            const hipError_t q = hipStreamQuery(vi->stream);
            if (q == hipSuccess && ((h[12] >> 32) != ep || (h[13] >> 32) != ep))
                MGDP_CHECK(false, MGDP_E_HIP, "run_to_dev_sync: the launch finished without its E words (epoch %u)", vi->epoch);
            if (q != hipSuccess && q != hipErrorNotReady) return hip_fail(q, "run_to_dev_sync", __FILE__, __LINE__);
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const unsigned long long rb = ((h[12] & 0xffffffffull) << 32) | (h[13] & 0xffffffffull);
    double rule;
    std::memcpy(&rule, &rb, sizeof(double));
    if (k_out) *k_out = km;
    if (dv_out) *dv_out = dv;
    if (dv_rule_out) *dv_rule_out = rule;
    return 0;
}

int mgdp_vi_local_result(const mgdp_vi *vi, int32_t *k_max, double *dv, int32_t *k_min) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    MGDP_CHECK(vi->k_done_valid, MGDP_E_INVALID, "no launch result to report (run mgdp_vi_run_local first)");
    if (k_max) *k_max = vi->k_max;
    if (dv) *dv = vi->dv_red;
    if (k_min) *k_min = vi->k_min;
    return 0;
}

int mgdp_vi_set_result(mgdp_vi *vi, int32_t k, double dv) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    MGDP_CHECK(k >= 0 && k <= vi->d.max_sweeps, MGDP_E_INVALID, "sweep %d out of range", k);
    vi->k_min = vi->k_max = vi->k_done = k;
    vi->dv_red = dv;
    vi->k_done_valid = true;
    return 0;
}

int mgdp_vi_sweep(mgdp_vi *vi, double *dv_out) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    if (vi->d.method == MGDP_METHOD_FUSED) {
        MGDP_CHECK(vi->k_done_valid && vi->k_min == vi->k_max, MGDP_E_INVALID,
                   "mgdp_vi_sweep: grids are not at a common sweep index (call mgdp_vi_run_to first)");
        return mgdp_vi_run_to(vi, vi->k_max + 1, dv_out);
    }
    return mgdp_vi_run_to(vi, vi->k_done + 1, dv_out);
}

int mgdp_vi_finish(mgdp_vi *vi, int32_t sweeps) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    vi->sweeps = sweeps;
    if (vi->d.method == MGDP_METHOD_SWEEP && sweeps > 0) {
        MGDP_CHECK(sweeps == vi->k_done, MGDP_E_INVALID, "finish(%d) but %d sweeps were run", sweeps, vi->k_done);
        // pi of sweep k = argmax evaluated on V_{k-1} (bit-identical to what sweep k computed)
        if (int rc = dispatch<SweepF>(vi, sweeps, 0, true)) return rc;
        vi->cur = sweeps & 1;
        MGDP_HIP(hipStreamSynchronize(vi->stream));
    }
    // fused: V and pi were written by the launch whose result was already observed; later reads
    // (mgdp_vi_get_*) are ordered on the stream
    return 0;
}

int mgdp_vi_solve(mgdp_vi *vi, int32_t *sweeps_out, double *dv_out, int32_t *converged_out) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    // Resident lone-grid server: a solve is a request word and a wait on host memory, so the
    // steady state makes no HIP call at all (no device guard either); anything else -- a server
    // that may be leaving, a rounding-level fallback sweep -- takes the general path below.
    // (a batch whose learned dispatch order is due takes the general path: mgdp_vi_reset learns it)
    const bool learn_due = vi->d.B > 1 && !vi->order_valid && vi->order_src == 2 && vi->solves_since_load > 0;
    if (vi->serving && served_eligible(vi) && vi->d.horizon == 0 && !learn_due) {
        const double idle_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - vi->serve_last).count();
        if (idle_us * 100.0 <= 0.5 * (double)vi->serve_idle_ticks) {
            vi->cur = 0;
            vi->k_done = 0;
            vi->k_done_valid = false;
            post_request(vi);
            vi->fresh = 0;
            int32_t k = 0;
            if (int rc = reduce_env(vi, &k, nullptr)) return rc;
            vi->serve_last = std::chrono::steady_clock::now();
            const double dv = vi->dv_red;
            // a batch is complete at K when every grid ended there or at an exact fixed point (mgdp_vi_run_to)
            const bool at_k = vi->d.B == 1 || vi->k_min == k || (vi->dv_red == 0.0 && vi->k_min > 0);
            if (vi->d.B > 1) ++vi->solves_since_load;
            if (at_k && (dv < vi->d.tol || k >= vi->d.max_sweeps)) {
                vi->k_done = k;
                vi->sweeps = k;
                vi->converged = dv < vi->d.tol;
                if (sweeps_out) *sweeps_out = k;
                if (dv_out) *dv_out = dv;
                if (converged_out) *converged_out = vi->converged;
                return 0;
            }
            // rounding broke the contraction: continue under the global rule on the general path
            double dv2 = dv;
            if (int rc = mgdp_vi_run_to(vi, k, &dv2)) return rc;
            while (!(dv2 < vi->d.tol) && k < vi->d.max_sweeps) {
                if (int rc = mgdp_vi_sweep(vi, &dv2)) return rc;
                ++k;
            }
            if (int rc = mgdp_vi_finish(vi, k)) return rc;
            vi->converged = dv2 < vi->d.tol;
            if (sweeps_out) *sweeps_out = k;
            if (dv_out) *dv_out = dv2;
            if (converged_out) *converged_out = vi->converged;
            return 0;
        }
    }
    DeviceGuard guard(vi->d.device);  // the entry points below nest inside it (no runtime call each)
    if (int rc = mgdp_vi_reset(vi)) return rc;
    int32_t k = 0;
    double dv = 0.0;
    // Deterministic batches take the plain path: their grids end their own rule at exact fixed
    // points, so run_local's result completes the solve (run_to launches nothing, see
    // mgdp_vi_run_to) -- one launch and one wait.  Slip batches keep the chained pair.
    if (vi->chain && !vi->gk && vi->d.slip_p >= 0.0 && vi->d.method == MGDP_METHOD_FUSED && vi->d.horizon == 0 &&
        !vi->opts && !serve_eligible(vi)) {
        // The single-GPU form of the multi-GPU device protocol: run_local publishes {K, ...} to
        // device memory and run_to(K) reads K there, enqueued back to back -- no host round trip
        // and no launch gap between the two; the host waits once, for run_to's result.
        DeviceGuard guard(vi->d.device);
        if (int rc = server_stop(vi)) return rc;
        if (int rc = dispatch<FusedF>(vi, -1, vi->d_pub1, (const long long *)nullptr)) return rc;
        if (int rc = dispatch<FusedF>(vi, 0, (unsigned long long *)nullptr, (const long long *)vi->d_pub1)) return rc;
        if (int rc = reduce_env(vi, &k, &dv)) return rc;
        // run_to read K on the device: every grid must have ended exactly there (the host path's
        // km == k_target check)
        MGDP_CHECK(vi->k_min == k && vi->k_max == k, MGDP_E_INVALID,
                   "chained solve: grids ended at sweeps %d..%d, not at one common K", vi->k_min, vi->k_max);
        vi->k_done = k;
    } else {
        vi->solving = true;
        const int rc = mgdp_vi_run_local(vi, &k);
        vi->solving = false;
        if (rc) return rc;
        if (int rc2 = mgdp_vi_run_to(vi, k, &dv)) return rc2;
    }
    while (vi->d.horizon == 0 && !(dv < vi->d.tol) && k < vi->d.max_sweeps) {  // contraction broken by rounding: global rule
        if (int rc = mgdp_vi_sweep(vi, &dv)) return rc;
        ++k;
    }
    if (int rc = mgdp_vi_finish(vi, k)) return rc;
    ++vi->solves_since_load;
    vi->converged = vi->d.horizon > 0 ? 1 : dv < vi->d.tol;  // a finite horizon is exact after H sweeps
    if (sweeps_out) *sweeps_out = k;
    if (dv_out) *dv_out = dv;
    if (converged_out) *converged_out = vi->converged;
    return 0;
}

// The sharded solve with the library's own collectives (include/mgdp.h, ABI 11): the device
// protocol of distributed.py with RCCL called from here on the handle's stream instead of through
// torch.distributed -- run_local_dev publishes {K_r, E_r bits, kmin, 0} into the communicator's
// device words, ncclAllReduce(MAX) of the first two is enqueued right behind it, the gate (or
// run_to(K)) reads them on the device, and the host waits once on host-mapped words.  Only when
// some grid anywhere stopped its own rule with dV > 0 (E != 0: slip, rounding, a cap) is dV(K)
// all-reduced too, and only a rounding-level breach of the contraction runs fallback sweeps.
namespace {
int comm_max_double(mgdp_comm *c, hipStream_t s, double *x) {
    // one word through the communicator's device buffer: non-negative doubles order like their bits
    int64_t *h = comm_host_word(c), *d = comm_proto(c) + 5;
    std::memcpy(h, x, sizeof(double));
    MGDP_HIP(hipMemcpyAsync(d, h, sizeof(int64_t), hipMemcpyHostToDevice, s));
    if (int rc = comm_allreduce_max_dev(c, d, 1, s)) return rc;
    MGDP_HIP(hipMemcpyAsync(h, d, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    MGDP_HIP(hipStreamSynchronize(s));
    comm_note_host_wait(c);
    std::memcpy(x, h, sizeof(double));
    return 0;
}
}  // namespace

int mgdp_vi_solve_sharded(mgdp_vi *vi, mgdp_comm *comm, int32_t *sweeps_out, double *dv_out, int32_t *converged_out) {
    MGDP_CHECK(vi && comm, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->d.method == MGDP_METHOD_FUSED && !vi->opts, MGDP_E_UNSUPPORTED,
               "the sharded solve runs the fused method without horizon / lava options");
    MGDP_CHECK(comm_device(comm) == vi->d.device, MGDP_E_INVALID, "communicator on device %d, handle on device %d",
               comm_device(comm), vi->d.device);
    DeviceGuard guard(vi->d.device);
    if (int rc = mgdp_vi_reset(vi)) return rc;
    int64_t *p = comm_proto(comm);
    if (int rc = mgdp_vi_run_local_dev(vi, p)) return rc;                  // {K_r, E_r bits, kmin, 0}
    if (int rc = comm_allreduce_max_dev(comm, p, 2, vi->stream)) return rc;  // {K, E} over every rank
    int32_t k = 0;
    double dv = 0.0, rule = 0.0;
    if (int rc = mgdp_vi_run_to_dev_sync(vi, p, &k, &dv, &rule)) return rc;  // the solve's one host wait
    comm_note_host_wait(comm);
    if (rule == 0.0) {
        // every grid of every rank stopped at an exact fixed point: dV at K is 0 everywhere
        MGDP_CHECK(dv == 0.0, MGDP_E_INVALID, "fixed-point invariant violated: dV at sweep %d is %g", k, dv);
    } else if (int rc = comm_max_double(comm, vi->stream, &dv)) {
        return rc;
    }
    if (int rc = mgdp_vi_set_result(vi, k, dv)) return rc;
    while (!(dv < vi->d.tol) && k < vi->d.max_sweeps) {  // contraction broken by rounding: global rule
        if (int rc = mgdp_vi_sweep(vi, &dv)) return rc;
        if (int rc = comm_max_double(comm, vi->stream, &dv)) return rc;
        ++k;
        vi->dv_red = dv;
    }
    if (int rc = mgdp_vi_finish(vi, k)) return rc;
    ++vi->solves_since_load;
    vi->converged = dv < vi->d.tol;
    if (sweeps_out) *sweeps_out = k;
    if (dv_out) *dv_out = dv;
    if (converged_out) *converged_out = vi->converged;
    return 0;
}

// Checkpoint / resume (aux "checkpoint / resume"): Jacobi is memoryless given V_k,
// so a solve stopped at sweep k (a max_sweeps cap) continues from {V_k, k, dV_k} -- on this handle
// or on a new one in another process -- to the same global stopping sweep, V and pi, bit for bit,
// as the uninterrupted solve.  Every grid restarts its own rule at k (kenv / dvenv), then the
// batch is taken to the global K as in mgdp_vi_solve.  A converged checkpoint (dV < tol) has
// nothing left to do, and its pi (argmax on V_{k-1}) cannot be rebuilt from V_k: refused.
int mgdp_vi_resume(mgdp_vi *vi, const void *V, int32_t k, double dv, int32_t *sweeps_out, double *dv_out,
                   int32_t *converged_out) {
    MGDP_CHECK(vi && V, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->cells_loaded, MGDP_E_INVALID, "no cells loaded");
    MGDP_CHECK(vi->d.method == MGDP_METHOD_FUSED && vi->d.horizon == 0, MGDP_E_INVALID,
               "resume: the fused method with an infinite horizon");
    MGDP_CHECK(k >= 1 && k < vi->d.max_sweeps, MGDP_E_INVALID, "resume: sweep %d outside [1, max_sweeps)", k);
    MGDP_CHECK(!(dv < vi->d.tol), MGDP_E_INVALID,
               "resume: the checkpoint has converged (dV %g < tol %g); its V and pi are final", dv, vi->d.tol);
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    // the copies below go through the null stream: drain the handle's own (or a caller-bound,
    // possibly non-blocking) stream first, so no earlier launch still reads V / kenv / dvenv
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    const size_t BS = (size_t)vi->d.B * vi->S;
    MGDP_HIP(hipMemcpy(vi->d_V[0], V, BS * vi->tsize, hipMemcpyHostToDevice));
    std::vector<int32_t> kk((size_t)vi->d.B, k);
    std::vector<double> dd((size_t)vi->d.B, dv);
    MGDP_HIP(hipMemcpy(vi->d_kenv, kk.data(), kk.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    MGDP_HIP(hipMemcpy(vi->d_kexec, kk.data(), kk.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    MGDP_HIP(hipMemcpy(vi->d_dvenv, dd.data(), dd.size() * sizeof(double), hipMemcpyHostToDevice));
    vi->fresh = 0;  // the next fused launch continues each grid from kenv / dvenv and V in HBM
    vi->cur = 0;
    vi->k_done = k;
    vi->k_min = k;
    vi->k_done_valid = false;
    vi->sweeps = k;
    vi->converged = 0;
    int32_t K = k;
    double dv2 = dv;
    if (int rc = mgdp_vi_run_local(vi, &K)) return rc;
    if (int rc = mgdp_vi_run_to(vi, K, &dv2)) return rc;
    while (!(dv2 < vi->d.tol) && K < vi->d.max_sweeps) {  // contraction broken by rounding: global rule
        if (int rc = mgdp_vi_sweep(vi, &dv2)) return rc;
        ++K;
    }
    if (int rc = mgdp_vi_finish(vi, K)) return rc;
    vi->converged = dv2 < vi->d.tol;
    if (sweeps_out) *sweeps_out = K;
    if (dv_out) *dv_out = dv2;
    if (converged_out) *converged_out = vi->converged;
    return 0;
}

int mgdp_vi_solve_last(mgdp_vi *vi, int32_t *sweeps_out, double *dv_out, int32_t *converged_out) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    vi->last_req = true;
    const int rc = mgdp_vi_solve(vi, sweeps_out, dv_out, converged_out);
    vi->last_req = false;
    if (vi->serving) {  // the request carried kServeLast: the server is leaving (or already gone)
        vi->serving = false;
        vi->exiting = true;
    }
    return rc;
}

int mgdp_vi_persistent(const mgdp_vi *vi, int32_t *on) {
    MGDP_CHECK(vi && on, MGDP_E_INVALID, "null argument");
    *on = serve_eligible(vi) ? 1 : 0;
    return 0;
}

const char *mgdp_vi_kernel_name(const mgdp_vi *vi) {
    if (!vi) { set_error("null handle"); return nullptr; }
    if (vi->d.method == MGDP_METHOD_FUSED) {
        if (vi->opts) return "vi_fused_opts_kernel";
        return serve_eligible(vi) ? "vi_serve_kernel" : "vi_fused_kernel";
    }
    return vi->d.mapping == MGDP_MAP_CELL && vi->sweep_pipe ? "vi_sweep_pipe_kernel" : "vi_sweep_kernel";
}

const char *mgdp_vi_variant(const mgdp_vi *vi) {
    if (!vi) { set_error("null handle"); return nullptr; }
    if (vi->d.method != MGDP_METHOD_FUSED) return vi->d.mapping == MGDP_MAP_CELL && vi->sweep_pipe ? "sweep_pipe" : "sweep";
    if (vi->opts) return "opts";
    if (vi->d.mapping == MGDP_MAP_SA) return "sa";
    if (serve_eligible(vi)) {
        if (vi->dkhalf) return "serve_dk_half";
        if (vi->band) return "serve_band";
        if (vi->serve_ew) return vi->serve_pair ? "serve_pair" : "serve_ew";
        return vi->wave_p ? "serve_wave" : "serve";
    }
    if (vi->dkrow) return "dk_rows";
    if (vi->dkhalf) return "dk_half";
    if (vi->dk1t) return "dk_1t";
    if (vi->band) return "band";
    if (vi->mix) return "mix";
    if (vi->wave2n) return "wave2n";
    if (vi->wave2) return "wave2";
    if (vi->wave_p) return "wave";
    if (vi->pair) return "pair";
    if (vi->quad) return "quad";
    if (vi->cpt == 2) return vi->pair2 && vi->d.slip_p < 0.0 ? "xyd_pair2" : "xyd_x2";
    if (vi->cpt == 4) return "xyd_x4";
    return vi->d.model == MGDP_MODEL_DOORKEY ? "dk_soa" : "xyd_soa";
}

int mgdp_vi_get_values(mgdp_vi *vi, void *V) {
    MGDP_CHECK(vi && V, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    const void *src = vi->d.method == MGDP_METHOD_SWEEP ? vi->d_V[vi->cur] : vi->d_V[0];
    MGDP_HIP(hipMemcpyAsync(V, src, (size_t)vi->d.B * vi->S * vi->tsize, hipMemcpyDeviceToHost, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
}

int mgdp_vi_get_policy_t(mgdp_vi *vi, int8_t *pi_t) {
    MGDP_CHECK(vi && pi_t, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(vi->d_pi_t, MGDP_E_INVALID, "no per-step policy: create with horizon > 0 and MGDP_KEEP_POLICY_T");
    DeviceGuard guard(vi->d.device);
    MGDP_HIP(hipMemcpyAsync(pi_t, vi->d_pi_t, (size_t)vi->d.horizon * vi->d.B * vi->S, hipMemcpyDeviceToHost, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
}

int mgdp_vi_get_policy(mgdp_vi *vi, int8_t *pi) {
    MGDP_CHECK(vi && pi, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipMemcpyAsync(pi, vi->d_pi, (size_t)vi->d.B * vi->S, hipMemcpyDeviceToHost, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
}

int mgdp_vi_get_grid_sweeps(mgdp_vi *vi, int32_t *k) {
    MGDP_CHECK(vi && k, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    if (vi->d.method == MGDP_METHOD_SWEEP) {
        std::fill(k, k + vi->d.B, (int32_t)vi->k_done);
        return 0;
    }
    MGDP_HIP(hipMemcpyAsync(k, vi->d_kexec, sizeof(int32_t) * (size_t)vi->d.B, hipMemcpyDeviceToHost, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
}

int mgdp_vi_get_dv_trace(mgdp_vi *vi, double *trace, int32_t n) {
    MGDP_CHECK(vi && trace && n >= 0 && n <= vi->d.max_sweeps, MGDP_E_INVALID, "bad argument");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    std::vector<unsigned long long> sh((size_t)8 * n);
    if (n) MGDP_HIP(hipMemcpy(sh.data(), vi->d_shards, sh.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) trace[i] = shard_max(&sh[8 * (size_t)i]);
    return 0;
}

int mgdp_vi_device_buffers(mgdp_vi *vi, void **d_V, void **d_pi) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    if (d_V) *d_V = vi->d.method == MGDP_METHOD_SWEEP ? vi->d_V[vi->cur] : vi->d_V[0];
    if (d_pi) *d_pi = vi->d_pi;
    return 0;
}

int mgdp_vi_synchronize(mgdp_vi *vi) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    // A resident server, or one leaving after its last request (mgdp_vi_solve_last), is the stream's
    // last work while nothing else was enqueued since (every other enqueue goes through server_stop
    // or a relaunch, which clear `exiting`): its tagged exit word then means the stream is done.
    if (vi->serving && !vi->pending_src) return server_stop(vi, false);
    if (vi->exiting && !vi->pending_src) {
        if (int rc = wait_server_exit(vi)) return rc;
        vi->exiting = false;
        return 0;
    }
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
}

int mgdp_vi_enable_timing(mgdp_vi *vi, int32_t on) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    if (int rc = timed_collect(vi)) return rc;  // drop launches timed before this call
    vi->timing = on != 0;
    vi->total_ms = 0.0;
    vi->launches = 0;
    vi->clk_cycles = vi->clk_ticks = vi->clk_busy = vi->clk_solves = 0.0;
    vi->clk_launches = 0;
    return 0;
}

int mgdp_vi_serve_clock(mgdp_vi *vi, double *sclk_mhz, double *server_us, int64_t *launches, double *solve_us,
                        int64_t *solves) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    account_server_clock(vi);
    if (sclk_mhz) *sclk_mhz = vi->clk_ticks > 0 ? vi->clk_cycles / (vi->clk_ticks * 0.01) : 0.0;
    if (server_us) *server_us = vi->clk_ticks * 0.01;
    if (launches) *launches = vi->clk_launches;
    if (solve_us) *solve_us = vi->clk_solves > 0 ? vi->clk_busy * 0.01 / vi->clk_solves : 0.0;
    if (solves) *solves = (int64_t)vi->clk_solves;
    return 0;
}

int mgdp_vi_kernel_time(mgdp_vi *vi, double *total_ms, int64_t *launches) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    if (int rc = timed_collect(vi)) return rc;
    if (total_ms) *total_ms = vi->total_ms;
    if (launches) *launches = vi->launches;
    return 0;
}

}  // extern "C"
