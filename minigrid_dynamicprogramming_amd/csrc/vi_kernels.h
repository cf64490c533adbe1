// vi_kernels.h -- the value-iteration kernels: fused solve, persistent lone-grid server,
// options kernel, reduce kernel, per-sweep HBM kernel.
// Part of the single translation unit vi.hip (included in order: vi_model.h, vi_loops.h,
// vi_kernels.h); see vi.hip for the DP semantics and the data layout.
#pragma once

namespace mgdp {
constexpr int kWpDk1t = -100;  // vi_fused_kernel variant tag: batched DoorKey on one LDS tile
// vi_fused_kernel variant tag: batched DoorKey grids of width 16 on whole-row thread maps, DPP
// east / west fronts and two conflict-free LDS planes (fused_dk_rows; its own LDS layout, dkrow_*)
constexpr int kWpDkRow = -800;
// ... the same for exactly 16x16 cells (DoorKey-16x16: 256 threads, plane stride known at compile time,
// so one LDS base register serves every tile access) and own-rule launches only (one copy of the sweep
// loops: the run_to copy kept values live across both).  Both are what let the fp32 loop fit 80 VGPRs
// -- 6 waves per SIMD -- with no scratch (round 5's 6-wave build spilled 76 B per thread).
constexpr int kWpDkRow16 = -801;
__host__ __device__ constexpr bool wp_is_dkrow(int wp) { return wp == kWpDkRow || wp == kWpDkRow16; }
// vi_fused_kernel variant tag: the direction-major one-thread-per-cell path alone.  The generic
// variant (WP = 0) also holds the cell-major, pair and quad loops, and a kernel's VGPR budget is
// that of its hungriest path: stripping them is what sets the batched kernels' occupancy.
constexpr int kWpSoa = -200;
// Tags -301 .. -308: batched deterministic XYD, two adjacent cells per thread, plane stride
// HWS = 128 * (-tag - 300) known at compile time (fused_pair_xyd).
constexpr int kWpPair = -300;
__host__ __device__ constexpr bool wp_is_pair(int wp) { return wp <= kWpPair - 1 && wp >= kWpPair - 8; }
// Tags -401 .. -408: batched deterministic XYD, one wave per grid, P = -tag - 400 cells per lane
// (fused_wave2_xyd, its own compact LDS layout; vi_fused_kernel only).
constexpr int kWpWave2 = -400;
__host__ __device__ constexpr bool wp_is_wave2(int wp) { return wp <= kWpWave2 - 1 && wp >= kWpWave2 - 8; }
// Tags -901 .. -908: batched deterministic XYD, one wave per grid in column bands of HB = -tag - 900
// rows (fused_band_xyd; no LDS tile, vi_fused_kernel only).
constexpr int kWpBand = -900;
__host__ __device__ constexpr bool wp_is_band(int wp) { return wp <= kWpBand - 1 && wp >= kWpBand - 8; }
// Tags -702 .. -704: batched deterministic XYD, TWO waves per grid, PW = -tag - 700 blocks of 64
// cells per wave (fused_wave2n_xyd; 128-thread workgroups, vi_fused_kernel only).
constexpr int kWpWave2n = -700;
__host__ __device__ constexpr bool wp_is_wave2n(int wp) { return wp <= kWpWave2n - 2 && wp >= kWpWave2n - 4; }
// Tags -1002 .. -1006 (fp32): batched deterministic XYD, P = -tag - 1000 blocks of 64 cells, 128-thread
// workgroups with MIXED wave counts: the first Geo::nmix workgroups of the learned dispatch order
// (the grids whose previous solve ran longest) sweep on two waves (fused_wave2n_xyd, PW = ceil(P / 2)
// blocks each), every other grid on one (fused_wave2_xyd; its second wave leaves at once).  For
// batches whose launch is set by a long tail of slow grids (an 8-way LavaS11N5 shard: median 24
// sweeps, max 47): splitting a long grid's sweep chain over two waves shortens the tail.
constexpr int kWpMix = -1000;
__host__ __device__ constexpr bool wp_is_mix(int wp) { return wp <= kWpMix - 2 && wp >= kWpMix - 6; }
// Minimum waves per SIMD the one-wave kernels are compiled for.  Left alone, the fp32 P <= 2
// variants (LavaS11N5: 121 cells) take 57 VGPRs but 106 SGPRs, and the SGPRs cap them at 7 waves
// per SIMD (28 workgroups / CU, 7168 grids resident): 8 makes the compiler fit 8 waves' SGPRs too
// (78 SGPRs, 32 / CU, 8192 resident -- an 8-way shard of LavaS11N5 x 65536 then fits the
// launch-wide rule in one launch: 89 -> 60 us per solve; the whole 65536 batch +4.5 %).  Same for
// fp64 P = 1 (57 VGPRs); the other variants are VGPR-bound at <= 6 waves.  Batches at the SGPR-bound
// residency also hit a dispatcher limit the occupancy API does not see: LavaS11N5 x 7168 at 28 / CU
// took 199 us (waiting grids ran to the cap) against 57 us at 32 / CU (profiles/r03_w8/).
// MGDP_WAVE2_W8=0 (A/B builds) keeps the compiler's default.
#ifndef MGDP_WAVE2_W8
#define MGDP_WAVE2_W8 1
#endif
#ifndef MGDP_WAVE2_P4_W6  // A/B builds: fp32 P = 4 (Empty-16) at 6 waves instead of its 91-VGPR 5
#define MGDP_WAVE2_P4_W6 0
#endif
#ifndef MGDP_WAVE2N_MINW  // A/B builds: minimum waves per SIMD of the two-waves-per-grid kernels
#define MGDP_WAVE2N_MINW 1
#endif
// Minimum waves per SIMD of fp32 fused_dk_rows: round 5's 6 (80 VGPRs and 76-80 B of scratch, 6 grids per
// CU) measured 1950-1960 vs 1992-1996 us per DoorKey-16 x 65536 solve at 5, neutral at 8192 grids
// (profiles/r05_dkw6/), but its spill stores doubled the launch's HBM writes.  Now: the 16x16 own-rule
// variant (kWpDkRow16) at 6 waves, 80 VGPRs, no scratch; the general one at 5 (96 VGPRs, no scratch).
// A/B builds: MGDP_DKROW16_MINW / MGDP_DKROW_MINW (1 = the compiler's choice).
#ifndef MGDP_DKROW_MINW
#define MGDP_DKROW_MINW 5
#endif
#ifndef MGDP_DKROW16_MINW
#define MGDP_DKROW16_MINW 6
#endif
template <typename T>
__host__ __device__ constexpr int wave2_min_waves(int wp) {
    return wp == kWpDkRow     ? (sizeof(T) == 4 ? MGDP_DKROW_MINW : 1)  // fp64 at 6 waves spills 492 B
           : wp == kWpDkRow16 ? (sizeof(T) == 4 ? MGDP_DKROW16_MINW : 1)
           : wp_is_wave2n(wp) ? MGDP_WAVE2N_MINW
           : (MGDP_WAVE2_W8 && wp_is_mix(wp) && kWpMix - wp <= 2) ? 8
           : (MGDP_WAVE2_W8 && wp_is_wave2(wp) && kWpWave2 - wp <= (sizeof(T) == 4 ? 2 : 1)) ? 8
           : (MGDP_WAVE2_P4_W6 && wp_is_wave2(wp) && sizeof(T) == 4 && kWpWave2 - wp == 4) ? 6
                                                                                            : 1;
}
// vi_fused_kernel variant tag: batched DoorKey, a cell's states split over two threads by has_key
// (fused_dk_half; workgroup = 2 * HWs threads)
// Tags -501 .. -508: plane stride HWs = 64 * (-tag - 500) known at compile time.
constexpr int kWpDkHalf = -500;
// vi_serve_kernel variant tag: the served lone deterministic XYD grid on fused_serve_xyd (east / west
// fronts by DPP; <= 4 waves), fused_fast_xyd_soa for a grid whose wave edges do not allow it
constexpr int kWpServeEw = -600;
// ... the same grids with two sweeps per workgroup barrier (fused_serve_pair, round 6)
constexpr int kWpServePair = -601;
__host__ __device__ constexpr bool wp_is_serve_ew(int wp) { return wp == kWpServeEw || wp == kWpServePair; }
// MGDP_DK_PERM=0 (A/B builds): batched DoorKey grids keep thread t on cell t (no dk_class_perm)
#ifndef MGDP_DK_PERM
#define MGDP_DK_PERM 1
#endif
__host__ __device__ constexpr bool wp_is_dkhalf(int wp) { return wp <= kWpDkHalf - 1 && wp >= kWpDkHalf - 8; }
template <typename T, int MODEL> struct TopoOf { using type = XydTopo<T>; };
template <typename T> struct TopoOf<T, MGDP_MODEL_DOORKEY> { using type = DkTopo; };

// pre: the cell topology a persistent server resolved once per residency (SERVED only)
template <typename T, int MODEL, bool SLIP, int MAP, bool SERVED = false, int WP = 0>
__device__ __forceinline__ bool fused_grid(const Geo &geo, const Coef<T> &cf, const uint8_t *__restrict__ cells,
                                           T *__restrict__ V, int8_t *__restrict__ pi, int32_t *__restrict__ kenv,
                                           double *__restrict__ dvenv, unsigned long long *__restrict__ host_out,
                                           int k_target, int fresh, bool lone, unsigned int epoch, int e,
                                           int &k, double &dvl, const typename TopoOf<T, MODEL>::type *pre = nullptr,
                                           unsigned long long *gk = nullptr, int ew = 0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    T *V0 = reinterpret_cast<T *>(smem);
    T *V1 = reinterpret_cast<T *>(smem + L.v_bytes);
    int8_t *pis = reinterpret_cast<int8_t *>(smem + L.pi_off());
    uint8_t *cl = reinterpret_cast<uint8_t *>(smem + L.cells_off());
    T *slots = reinterpret_cast<T *>(smem + L.slots_off());
    uint8_t *flags = reinterpret_cast<uint8_t *>(smem + L.flags_off());

    // workgroup-uniform: in SGPRs (as VGPRs they stayed live across the sweep loops -- a register
    // pair the batched DoorKey loop at 80 VGPRs had to spill to scratch)
    k = __builtin_amdgcn_readfirstlane(fresh ? 0 : kenv[e]);
    {
        const long long b = fresh ? 0ll : __double_as_longlong(dvenv[e]);
        const unsigned int lo = __builtin_amdgcn_readfirstlane((unsigned int)b);
        const unsigned int hi = __builtin_amdgcn_readfirstlane((unsigned int)(b >> 32));
        dvl = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    }
    if (geo.kprio[2] > 0 && k_target < 0) {
        // learned priority: the grids that ran longest last time get the SIMDs' issue slots first, so
        // the launch's critical path (its longest grids) is not stretched by the short ones
        const int kp = geo.kexec[e];
        if (kp >= geo.kprio[0]) __builtin_amdgcn_s_setprio(3);
        else if (kp >= geo.kprio[1]) __builtin_amdgcn_s_setprio(2);
        else if (kp >= geo.kprio[2]) __builtin_amdgcn_s_setprio(1);
    }
    // Fixed-point completion: a grid whose last sweep changed nothing (|dV| = 0 exactly, so
    // V_k == V_{k-1} bit for bit) reproduces V_k at every later sweep (a Jacobi sweep is a function
    // of V alone), and pi_{k'} = argmax on V_{k'-1} = pi_k: it is at sweep k_target already, with
    // dV 0.  Only its sweep count moves (the reduce kernel reads it).
    if (k_target > k && k > 0 && dvl == 0.0) {
        if (threadIdx.x == 0) kenv[e] = k_target;
        k = k_target;
        return false;
    }
    const bool work = k_target < 0 ? (!(k > 0 && dvl < geo.tol) && k < geo.max_sweeps) : (k < k_target);
    if (!work) return false;
    const long long vb = (long long)e * geo.S;
    if constexpr (wp_is_mix(WP)) {  // two waves for the first nmix workgroups, one for the rest
        static_assert(MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL && !SERVED, "mix: batched plain XYD");
        constexpr int P = kWpMix - WP, PW = (P + 1) / 2;
        uint8_t *cl2 = smem + 256;
        copy16(cl2, cells + (long long)e * geo.HWp, geo.HWp);
        T *tile = reinterpret_cast<T *>(smem + wave2_tile_off(geo.HWp));
        auto done2 = [&](int kk, double dv) {
            if (lone && threadIdx.x == 0)
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
        };
        if ((int)blockIdx.x < geo.nmix) {  // workgroup-uniform: both waves are here
            __syncthreads();
            if (k_target < 0)
                fused_wave2n_xyd<T, true, PW>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2,
                                              GkCtx{gk, epoch, e, geo.B, host_out});
            else
                fused_wave2n_xyd<T, false, PW>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        } else {  // wave 0 alone (vi_fused_kernel let wave 1 go)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (k_target < 0)
                fused_wave2_xyd<T, true, P>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2,
                                            GkCtx{gk, epoch, e, geo.B, host_out});
            else
                fused_wave2_xyd<T, false, P>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        }
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    if constexpr (wp_is_wave2n(WP)) {  // two waves per grid: cells, then two N/S tiles (wave2n_*)
        static_assert(MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL && !SERVED, "wave2n: batched plain XYD");
        constexpr int PW = kWpWave2n - WP;
        uint8_t *cl2 = smem + 256;
        copy16(cl2, cells + (long long)e * geo.HWp, geo.HWp);
        __syncthreads();
        T *tile = reinterpret_cast<T *>(smem + wave2_tile_off(geo.HWp));
        auto done2 = [&](int kk, double dv) {
            if (lone && threadIdx.x == 0)
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
        };
        if (k_target < 0)
            fused_wave2n_xyd<T, true, PW>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2,
                                          GkCtx{gk, epoch, e, geo.B, host_out});
        else
            fused_wave2n_xyd<T, false, PW>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    if constexpr (wp_is_band(WP)) {  // LDS: slots, then the cells (no tile); served: the server's staged cells
        static_assert(MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL, "band: plain XYD");
        constexpr int HB = kWpBand - WP;
        uint8_t *cl2 = SERVED ? reinterpret_cast<uint8_t *>(smem + L.cells_off()) : smem + 256;
        if (!SERVED) {
            copy16(cl2, cells + (long long)e * geo.HWp, geo.HWp);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS writes are ordered
        }
        auto done2 = [&](int kk, double dv) {
            if (SERVED) {
                if (threadIdx.x == 0) publish_tagged(host_out, kk, dv, epoch);
            } else if (lone && threadIdx.x == 0) {
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
            }
        };
        if (k_target < 0)
            fused_band_xyd<T, true, HB>(geo, cf, cl2, V + vb, V + vb, pi + vb, k, k_target, dvl, done2,
                                        GkCtx{gk, epoch, e, geo.B, host_out});
        else
            fused_band_xyd<T, false, HB>(geo, cf, cl2, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    if constexpr (wp_is_wave2(WP)) {  // its own LDS layout (wave2_*): cells, then the N/S tile
        static_assert(MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL && !SERVED, "wave2: batched plain XYD");
        constexpr int P = kWpWave2 - WP;
        uint8_t *cl2 = smem + 256;
        copy16(cl2, cells + (long long)e * geo.HWp, geo.HWp);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS writes are ordered
        T *tile = reinterpret_cast<T *>(smem + wave2_tile_off(geo.HWp));
        auto done2 = [&](int kk, double dv) {
            if (lone && threadIdx.x == 0)
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
        };
        if (k_target < 0 && (gk != nullptr || geo.wt)) {  // resident: write-through exit stores (and the
                                                          // in-launch reduction unless a protocol launch)
            fused_wave2_xyd<T, true, P, true>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2,
                                              GkCtx{gk, epoch, e, geo.B, host_out});
        } else if (k_target < 0) {
            fused_wave2_xyd<T, true, P>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        } else {
            fused_wave2_xyd<T, false, P>(geo, cf, cl2, tile, V + vb, V + vb, pi + vb, k, k_target, dvl, done2);
        }
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    if constexpr (wp_is_dkrow(WP)) {  // its own LDS layout (dkrow_*): slots, flags, row map, cells, tiles
        static_assert(MODEL == MGDP_MODEL_DOORKEY && !SLIP && MAP == MGDP_MAP_CELL && !SERVED, "dkrow: batched DoorKey");
        uint8_t *cl2 = smem + dkrow_cells_off();
        copy16(cl2, cells + (long long)e * geo.HWp, geo.HWp);
        __syncthreads();
        T *tiles = reinterpret_cast<T *>(smem + dkrow_tile_off(geo.HWp));
        T *slots2 = reinterpret_cast<T *>(smem);
        // after the loop the thread index is late_tid's (fused_dk_rows): nothing below reads threadIdx.x
        int tl = 0;
        auto done2 = [&](int kk, double dv) {
            if (lone && tl == 0)
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
        };
        if constexpr (WP == kWpDkRow16) {  // own-rule launches only (the host picks kWpDkRow for run_to)
            fused_dk_rows<T, true, 256>(geo, cf, cl2, tiles, slots2, smem + 256, smem + 320, V + vb, V + vb, pi + vb, k,
                                        k_target, dvl, done2, tl);
        } else if (k_target < 0) {
            fused_dk_rows<T, true>(geo, cf, cl2, tiles, slots2, smem + 256, smem + 320, V + vb, V + vb, pi + vb, k,
                                   k_target, dvl, done2, tl);
        } else {
            fused_dk_rows<T, false>(geo, cf, cl2, tiles, slots2, smem + 256, smem + 320, V + vb, V + vb, pi + vb, k,
                                    k_target, dvl, done2, tl);
        }
        if (tl == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    // WP == kWpDk1t: batched DoorKey on one LDS tile (fused_fast_dk_1t); other WP < 0: -WP cells per
    // thread on the batched XYD direction-major path (fused_fast_xyd_soa_xn)
    constexpr bool DK1T = WP == kWpDk1t;
    constexpr bool SOA_ONLY = WP < 0;  // every negative tag runs the direction-major path alone
    constexpr bool PAIR2 = wp_is_pair(WP);
    constexpr bool DKHALF = wp_is_dkhalf(WP);
    constexpr bool SERVE_EW = wp_is_serve_ew(WP);
    constexpr int CPT = PAIR2 ? 2 : (WP < 0 && !DK1T && !DKHALF && !SERVE_EW && WP != kWpSoa ? -WP : 1);
    const bool fast = MAP == MGDP_MAP_CELL && geo.HW <= CPT * (int)blockDim.x;
    const bool soa = SOA_ONLY || (fast && !geo.pair && !geo.quad);
    if (!SERVED) copy16(cl, cells + (long long)e * geo.HWp, geo.HWp);
    if (!soa) {
        // cell-major paths use the first S entries of each (Ss-sized) tile
        if (k == 0) zero16(V0, geo.S * (int)sizeof(T));
        else copy16(V0, V + vb, geo.S * (int)sizeof(T));
    }
    if (threadIdx.x < 64) flags[threadIdx.x] = 0;
    __syncthreads();

    int cur = 0, parity = 0;
    T diff = (T)0;
    auto done = [&](int kk, double dv) {
        if (SERVED) {
            if (threadIdx.x == 0) {
#ifdef MGDP_SERVE_TRACE
                __hip_atomic_store(host_out + 15, __builtin_amdgcn_s_memtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(host_out + 9, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
                publish_tagged(host_out, kk, dv, epoch);
            }
        } else if (lone && threadIdx.x == 0) {
            publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                    (unsigned long long)kk, epoch);
        }
    };
    const T *Vfinal = nullptr;
    if constexpr (WP > 0) {  // lone XYD grid on one wave, WP cells per lane (host: B == 1, blockDim 64)
        static_assert(MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL, "one-wave path is XYD, cell mapping");
        if (SERVED || k_target < 0)
            fused_wave_xyd<T, SLIP, true, WP>(geo, cf, cl, V0, V1, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        else
            fused_wave_xyd<T, SLIP, false, WP>(geo, cf, cl, V0, V1, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;
    }
    if (SERVED || soa) {  // served lone grids are always on this path (serve_eligible): no other code in the server
        if constexpr (PAIR2) {
            static_assert(MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL, "pair path: plain XYD");
            constexpr int HWS = 128 * (kWpPair - WP);
            if (k_target < 0) fused_pair_xyd<T, true, HWS>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_pair_xyd<T, false, HWS>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else if constexpr (MODEL == MGDP_MODEL_DOORKEY && DKHALF) {
            constexpr int HWS = 64 * (kWpDkHalf - WP);
            if (k_target < 0) fused_dk_half<T, true, HWS>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_dk_half<T, false, HWS>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else if constexpr (MODEL == MGDP_MODEL_DOORKEY && DK1T) {
            if (k_target < 0) fused_fast_dk_1t<T, true>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_fast_dk_1t<T, false>(geo, cf, cl, V0, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else if constexpr (SERVE_EW) {
            static_assert(SERVED && MODEL == MGDP_MODEL_XYD && !SLIP && MAP == MGDP_MAP_CELL, "served plain XYD grid");
            // ew: 0 = this grid falls back, 1 = fused_serve_xyd (kWpServePair: fused_serve_pair), 2 = the
            // same, first solve of the grid
            bool ran = false;
            if constexpr (WP == kWpServePair) {
                if (ew) {
                    fused_serve_pair<T>(geo, cf, V0, V0 + serve_pair_tile_elems(geo.HWs, geo.W), slots, flags,
                                        V + vb, V + vb, pi + vb, k, dvl, done, *pre, ew == 2);
                    ran = true;
                }
            } else if (ew) {
                fused_serve_xyd<T>(geo, cf, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, dvl, done, *pre, ew == 2);
                ran = true;
            }
            if (!ran)
                fused_fast_xyd_soa<T, false, true>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target,
                                                   dvl, done, nullptr, nullptr, 0, pre);
        } else if constexpr (MODEL == MGDP_MODEL_XYD && CPT > 1) {
            if (k_target < 0) fused_fast_xyd_soa_xn<T, SLIP, true, CPT>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_fast_xyd_soa_xn<T, SLIP, false, CPT>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else if constexpr (MODEL == MGDP_MODEL_XYD) {
            if (SERVED || k_target < 0)
                fused_fast_xyd_soa<T, SLIP, true>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl,
                                                  done, nullptr, nullptr, 0, pre);
            else fused_fast_xyd_soa<T, SLIP, false>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else {
            // batched grids: the special-first thread -> cell map (dk_class_perm) in the unused pi region
            uint8_t *perm = (MGDP_DK_PERM && !SERVED && 2 * geo.HW + 16 + 128 <= L.pi_bytes)
                                ? reinterpret_cast<uint8_t *>(pis) : nullptr;
            if (SERVED || k_target < 0)
                fused_fast_dk_soa<T, true>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done,
                                           nullptr, nullptr, 0, pre, perm);
            else fused_fast_dk_soa<T, false>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done,
                                             nullptr, nullptr, 0, nullptr, perm);
        }
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
        return true;  // V and pi were written by their owner threads
    }
    if constexpr (SERVED || SOA_ONLY) return true;
    else {
    if (fast && MODEL == MGDP_MODEL_XYD && geo.pair) {
        int vf = 0;
        if (k_target < 0) fused_fast_xyd2<T, SLIP, true>(geo, cf, cl, V0, pis, slots, flags, k, k_target, vf, dvl, done);
        else fused_fast_xyd2<T, SLIP, false>(geo, cf, cl, V0, pis, slots, flags, k, k_target, vf, dvl, done);
        Vfinal = V0 + vf * geo.S;
    } else if (MODEL == MGDP_MODEL_XYD && MAP == MGDP_MAP_CELL && geo.quad && 4 * geo.HW <= (int)blockDim.x) {
        if (k_target < 0) fused_quad_xyd<T, SLIP, true>(geo, cf, cl, V0, V1, pis, slots, flags, k, k_target, cur, dvl, done);
        else fused_quad_xyd<T, SLIP, false>(geo, cf, cl, V0, V1, pis, slots, flags, k, k_target, cur, dvl, done);
    } else {
        while (true) {
            const T *Vin = cur ? V1 : V0;
            T *Vout = cur ? V0 : V1;
            diff = sweep_lds<T, MODEL, SLIP, MAP, true, MAP == MGDP_MAP_SA>(geo, cf, cl, Vin, Vout, pis);
            cur ^= 1;
            ++k;
            if (k_target < 0) {
                const bool more = block_any(diff >= cf.tol, flags, parity);
                parity ^= 1;
                if (!more || k >= geo.max_sweeps) break;
            } else {
                __syncthreads();
                if (k >= k_target) break;
            }
        }
        dvl = (double)block_max(diff, slots, 0);
        done(k, dvl);
        if (MAP == MGDP_MAP_CELL) {  // pi of the last sweep = argmax on V_{k-1}
            sweep_lds<T, MODEL, SLIP, MAP, false, true>(geo, cf, cl, cur ? V0 : V1, nullptr, pis);
            __syncthreads();
        }
    }
    copy16(V + vb, Vfinal ? Vfinal : (cur ? V1 : V0), geo.S * (int)sizeof(T));
    copy_pi(pi + vb, pis, geo.S);
    if (threadIdx.x == 0) {
        kenv[e] = k;
        if (geo.kexec) geo.kexec[e] = k;
        dvenv[e] = dvl;
    }
    return true;
    }
}

// WP > 0: the one-wave lone-grid variant (fused_wave_xyd), 64 threads, so its WP cells per lane
// may use the whole register file.
template <typename T, int MODEL, bool SLIP, int MAP, int WP = 0>
__global__ void __launch_bounds__(WP > 0 || wp_is_wave2(WP) || wp_is_band(WP) ? 64 : (wp_is_wave2n(WP) || wp_is_mix(WP) ? 128 : 1024), wave2_min_waves<T>(WP))
vi_fused_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, T *__restrict__ V,
                int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                unsigned long long *__restrict__ red, unsigned int *__restrict__ ticket,
                unsigned long long *__restrict__ host_out, int k_target, int fresh, int in_kernel_reduce,
                unsigned int epoch, const long long *__restrict__ k_target_dev,
                unsigned long long *__restrict__ host_mirror, unsigned long long *__restrict__ gk) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    constexpr bool kOwnLds = wp_is_wave2(WP) || wp_is_wave2n(WP) || wp_is_band(WP) || wp_is_mix(WP);  // wave2-family layouts, gk
    T *slots = reinterpret_cast<T *>(smem + (kOwnLds || wp_is_dkrow(WP) ? 0 : L.slots_off()));
    // a one-wave grid of a mixed launch: its second wave leaves before touching anything
    if constexpr (wp_is_mix(WP))
        if (threadIdx.x >= 64 && (int)blockIdx.x >= geo.nmix) return;
    // multi-GPU protocol (mgdp_vi_run_to_dev): the target sweep is the all-reduced K in device
    // memory, written by a collective ordered before this launch on the stream
    if (k_target_dev) {
        k_target = (int)k_target_dev[0];
        // mgdp_vi_run_to_dev_sync: the all-reduced word after K (the own-rule dV) goes to the host
        // with this launch's result, as two words tagged with this launch's epoch (the host waits
        // for them as for the result's)
        if (host_mirror && blockIdx.x == 0 && threadIdx.x == 0)
            publish_word2(host_mirror, (unsigned long long)k_target_dev[1], epoch);
    }
    int k;
    double dvl;
    // kWpDkRow: the wave index in an SGPR, for late_tid after the sweep loop (fused_dk_rows)
    const int wvk = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bool lone = in_kernel_reduce && gridDim.x == 1;
    const bool work = fused_grid<T, MODEL, SLIP, MAP, false, WP>(geo, cf, cells, V, pi, kenv, dvenv, host_out, k_target,
                                                                 fresh, lone, epoch,
                                                                 geo.order ? (int)geo.order[blockIdx.x] : (int)blockIdx.x,
                                                                 k, dvl, nullptr,
                                                                 kOwnLds ? gk : nullptr);
    // a launch-wide-rule launch (wave2 with gk) reduces and publishes through its own counter tree
    const bool gk_pub = kOwnLds && gk != nullptr && k_target < 0 && !k_target_dev;
    if (in_kernel_reduce && !gk_pub)
        fused_reduce(red, ticket, host_out, k, dvl, reinterpret_cast<unsigned int *>(slots + 16), epoch, work,
                     wp_is_dkrow(WP) ? late_tid(wvk) : (int)threadIdx.x);
}

// Persistent solver for a lone grid: one workgroup stays resident and serves solve requests posted
// in host-mapped memory, removing the launch and dispatch latency from every solve.  The grid is
// staged in LDS (and its topology resolved) at launch and again whenever a request carries
// kServeNewCells: the request's source word (host_cmd[1], tagged with the request's low 16 bits, so
// a source written before the request can never be paired with an older one) names the new grid's
// W*H bytes -- host-mapped staging or device memory --, which the workgroup reads with
// system-scope loads (coherent with the host and with every XCD's L2), copies into LDS and into
// the handle's HBM cells (so a later non-served launch sees the same grid).  Lane 0 of every
// polling wave reads the request word (relaxed system-scope loads, the waves staggered by s_sleep)
// and also watches the LDS word another wave may already have set.  By default only wave 0 polls
// (`pollers` = 1; the others wait at the barrier): with four staggered pollers the barrier also
// waited for the other waves' in-flight PCIe reads (measured 0.2-0.4 us per solve slower).
// poll_dma (default): the poller does not wait for its reads.  Each poll is an LDS-DMA load
// (global_load_lds_dwordx4 of the request / source pair) into a 16-B LDS mailbox, issued about
// every 60 ns, so a PCIe round trip's worth of polls is in flight and the mailbox always holds the
// latest read to return: a request is seen one round trip after it lands instead of one to two
// (one blocking read at a time put a 1.2-1.5 us sawtooth on the solve latency, by when the host
// posted relative to the poll -- tools/probe_serve.cpp with MGDP_PROBE_GAP_US).  The loads are
// asm the compiler does not track: a stray one still in flight when the request is seen writes only
// the mailbox, and the wave's next vmcnt wait (the compiler's, for its own accesses, or the one
// before the exit word) also covers it.  Request
// r (!= the last served) runs a fresh fused solve whose {k, dV} is published tagged with r.  Every
// wave leaves on the quit word, after `idle_ticks` without a request or after `life_ticks` in total
// (s_memrealtime, 100 MHz); the host relaunches the server if a request finds it gone.
constexpr int kHoutWords = 32;  // host-mapped words of a handle (mgdp_vi::h_out)
constexpr int kHoutReq = 16;    // request word; its source word follows (one 16-B pair)
constexpr int kHoutClk = 24;    // a departing server's {shader-clock cycles, 100 MHz ticks} of its life,
                                // then {100 MHz ticks inside its solves, solves served}
constexpr unsigned long long kServeQuit = ~0ull;
constexpr unsigned long long kServeNewCells = 1ull << 62;
constexpr unsigned long long kServeLast = 1ull << 61;  // request flag: leave after serving it
constexpr unsigned long long kServeSrcMask = (1ull << 48) - 1;

// One poll of the {request, source} pair (16 B of host memory, system scope) into the LDS mailbox
// `box` by LDS DMA, issued by the calling lane without waiting for it (see vi_serve_kernel).  At
// most 24 stay in flight (about 1.5 us of polls at the loop's pace; the wait is free below that).
// M0 holds the LDS address for the load and is restored after it.
__device__ __forceinline__ void poll_issue(const unsigned long long *src, unsigned long long *box) {
    const unsigned int lds = (unsigned int)(uintptr_t)box;  // low 32 bits of a shared pointer: its LDS offset
    unsigned int m0_saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off sc0 sc1\n\t"
        "s_nop 0\n\t"
        "s_mov_b32 m0, %0\n\t"
        "s_waitcnt vmcnt(24)"
        : "=&s"(m0_saved)
        : "s"(lds), "v"(src)
        : "memory");
}

// (kWpServePair: <= 4 waves by the host's serve_ew rule, so its three register sets and halo state may
// use up to 512 VGPRs per lane: no spill)
template <typename T, int MODEL, bool SLIP, int MAP, int WP = 0>
__global__ void __launch_bounds__(WP > 0 ? 64 : (WP == kWpServePair ? 256 : 1024))
vi_serve_kernel(Geo geo, Coef<T> cf, uint8_t *__restrict__ cells, T *__restrict__ V,
                int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                unsigned long long *__restrict__ host_out, const unsigned long long *__restrict__ host_cmd,
                unsigned long long served, unsigned long long idle_ticks, unsigned long long life_ticks, int pollers,
                unsigned long long exit_tag, int poll_dma) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ unsigned long long s_cmd, s_src;
    __shared__ __attribute__((aligned(16))) unsigned long long s_box[2];  // poll mailbox: {request, source}
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    uint8_t *cl = reinterpret_cast<uint8_t *>(smem + L.cells_off());
    copy16(cl, cells, geo.HWp);
    if (threadIdx.x == 0) {
        s_cmd = served;
        s_box[0] = served;
        s_box[1] = 0;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();  // shader-clock cycles
    unsigned long long t_last = t_start;
    // GPU-side time of the solves (thread 0: the poll that saw the request -> the solve's end,
    // s_memrealtime ticks already read for the idle limit, so no extra counter read per solve)
    unsigned long long t_seen = t_start, busy = 0, solves = 0;
    __syncthreads();
    // the grid stays put between kServeNewCells requests: resolve this thread's cell topology once
    typename TopoOf<T, MODEL>::type topo;
    int ew = 0;  // kWpServeEw: 0 = the grid falls back, 1 = fused_serve_xyd, 2 = the same, tiles to clear
    __shared__ int s_ew;
    auto resolve = [&]() {
        if constexpr (WP == 0 || wp_is_serve_ew(WP)) {
            const int cc = (int)threadIdx.x < geo.HW ? (int)threadIdx.x : 0;
            if constexpr (MODEL == MGDP_MODEL_XYD) topo = xyd_topo_soa<T>(cl, geo, cc);
            else topo = dk_topo_soa(cl, geo, cc);
        }
        if constexpr (WP == kWpServePair && MODEL == MGDP_MODEL_XYD) topo.halo = serve_pair_halo(cl, geo, (int)threadIdx.x);
        if constexpr (wp_is_serve_ew(WP)) ew = serve_ew_ok(cl, geo, &s_ew) ? 2 : 0;
    };
    resolve();
    while (true) {
        if (lane == 0 && wave < pollers) {  // the other waves wait at the barrier
            for (int i = 0; i < wave; ++i) __builtin_amdgcn_s_sleep(8);  // stagger the pollers
            while (true) {
                unsigned long long cmd, src = 0;
                if (poll_dma) {
                    poll_issue(host_cmd, s_box);
                    __builtin_amdgcn_s_sleep(1);
                    cmd = __hip_atomic_load(&s_box[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    src = __hip_atomic_load(&s_box[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    cmd = __hip_atomic_load(host_cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                if (cmd != served) {
                    t_seen = now;
                    if (cmd != kServeQuit && (cmd & kServeNewCells)) {
                        // the host wrote the source word before the request word; its tag proves it
                        // belongs to this request (a stale read is simply repeated)
                        if (!poll_dma || (src >> 48) != (cmd & 0xffffull))
                            src = __hip_atomic_load(host_cmd + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        while ((src >> 48) != (cmd & 0xffffull)) {
                            if (__builtin_amdgcn_s_memrealtime() - t_start > life_ticks) { cmd = kServeQuit; break; }
                            src = __hip_atomic_load(host_cmd + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                        __hip_atomic_store(&s_src, src & kServeSrcMask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    __hip_atomic_store(&s_cmd, cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (__hip_atomic_load(&s_cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != served) break;
                if (now - t_last > idle_ticks || now - t_start > life_ticks) {
                    __hip_atomic_store(&s_cmd, kServeQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (!poll_dma) __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        const unsigned long long cmd = s_cmd;
        if (cmd == kServeQuit) break;
#ifdef MGDP_SERVE_TRACE
        if (threadIdx.x == 0) {  // s_memtime counts shader-clock cycles, s_memrealtime 100 MHz ticks
            __hip_atomic_store(host_out + 14, __builtin_amdgcn_s_memtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_out + 8, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#endif
        if (cmd & kServeNewCells) {  // restage the grid named by the request
            const uint8_t *src = reinterpret_cast<const uint8_t *>(s_src);
            for (int i = threadIdx.x; i < geo.HW; i += blockDim.x) {
                const uint8_t b = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                cl[i] = b;
                cells[i] = b;
            }
            __syncthreads();
            resolve();
        }
        int k;
        double dvl;
        if (!fused_grid<T, MODEL, SLIP, MAP, true, WP>(geo, cf, cells, V, pi, kenv, dvenv, host_out, -1, 1, true,
                                                   (unsigned int)cmd, 0, k, dvl,
                                                   (WP == 0 || wp_is_serve_ew(WP)) ? &topo : nullptr, nullptr, ew) &&
            threadIdx.x == 0)
            publish_tagged(host_out, k, dvl, (unsigned int)cmd);
        if (ew == 2) ew = 1;  // the tiles' pads stay +0 until the next grid
        served = cmd;
        t_last = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            busy += t_last - t_seen;
            ++solves;
        }
        if (cmd & kServeLast) break;
        // Every wave is past s_cmd and the LDS tiles before the next request: an LDS-only barrier.
        // The V / pi stores of this solve stay in flight while the next request is polled (a
        // __syncthreads would drain them first); the host reads V / pi only after server_stop
        // has drained the stream.
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // Leaving: every wave's V / pi stores complete, then one system-scope release tells the host
    // (server_stop without a drain waits for this word instead of the stream's completion signal).
    // The word is this launch's own tag, so an earlier server's late exit store can never satisfy
    // the wait for a later one.
    // The launch's shader-clock cycles and 100 MHz ticks go out with it (kHoutClk): the host turns
    // them into the clock the server ran at (mgdp_vi_serve_clock), at no cost per solve.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(host_out + kHoutClk, __builtin_amdgcn_s_memtime() - c_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 1, __builtin_amdgcn_s_memrealtime() - t_start, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 2, busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 3, solves, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + 11, exit_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Persistent server for a resident batch (round 6): the resident one-wave batch (fused_wave2_xyd,
// B <= the kernel's resident capacity, deterministic XYD grids) stays on the device between
// solves, so a solve costs a request word instead of a launch, a dispatch of B workgroups, their
// cells copy and the end-of-kernel release.  Every request is a full solve from
// V_0 = 0 with the in-launch reduction (GkCtx) publishing {kmax, dV, kmin} tagged with the request
// exactly as a launch does; nothing is carried from one request to the next but the grids' cells
// in LDS.  Lane 0 of workgroup 0 (the forwarder) polls the host's request word (LDS-DMA mailbox,
// as vi_serve_kernel) and forwards it to `copies` device words, one per 128-B line (tag of this launch in bits
// 32..47, the request's epoch in the low 32 bits, kServeLast kept, kBreqQuit to leave); every
// other wave polls that word at agent scope with s_sleep between polls and at priority 0 (the
// waves still sweeping get the issue slots).  Only the forwarder decides to leave (quit word,
// idle or life limit); the others leave on its quit word, or after the life limit plus a grace
// period, so every wave reaches the exit.  The last wave out (a two-level exit counter) writes the exit
// word, as a lone server does.
constexpr unsigned long long kBreqQuit = 1ull << 63;
constexpr int kBreqCopies = 64;                                       // request lines (workgroup w polls w % copies)
constexpr int kBreqExit = kBreqCopies * 16;                           // exit counters: 64 shard lines, then the top line
constexpr int kBreqExitShards = 64;
constexpr int kBreqWords = kBreqExit + (kBreqExitShards + 1) * 16;
constexpr unsigned long long kBserveGraceTicks = 100000000ull;        // 1 s at 100 MHz
__device__ __forceinline__ unsigned long long rfl64(unsigned long long x) {
    const unsigned int lo = __builtin_amdgcn_readfirstlane((unsigned int)x);
    const unsigned int hi = __builtin_amdgcn_readfirstlane((unsigned int)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
// Waves per SIMD the server is compiled for: those of the fused kernel's wave2 instantiation of the
// same P (its resident capacity; fp32 P = 3: 5 instead of 7, which spilled).  Inside the request loop
// the compiler spent 25-60 % more VGPRs on the same sweep loop (fp32 P = 6: 173 vs 115 -- half the
// grids resident); with the lane index opaque per request (fused_wave2_xyd OPQ) and this bound,
// every instantiation fits without scratch.
template <typename T>
__host__ __device__ constexpr int bserve_min_waves(int P) {
    return sizeof(T) == 4 ? (P <= 2 ? 8 : P <= 4 ? 5 : P <= 6 ? 4 : 3)
                          : (P == 1 ? 8 : P == 2 ? 5 : P == 3 ? 4 : P == 4 ? 3 : P <= 7 ? 2 : 1);
}
#ifndef MGDP_BSERVE_MINW  // A/B builds: 0 = the compiler's choice (wave2_min_waves)
#define MGDP_BSERVE_MINW 1
#endif
#ifndef MGDP_BSERVE_PRIO  // A/B builds: 0 = no s_setprio (polling waves at the solving waves' priority)
#define MGDP_BSERVE_PRIO 1
#endif
#ifndef MGDP_BSERVE_OPQ  // A/B builds: 0 = the lane index as threadIdx.x in the request loop's solve
#define MGDP_BSERVE_OPQ 1
#endif
// MULTI: the launch has fewer workgroups than grids (a batch past the resident capacity, MGDP_BSERVE=2):
// its own instantiation, so the resident loop keeps its registers.
template <typename T, int P, bool MULTI = false>
__global__ void __launch_bounds__(64, MGDP_BSERVE_MINW ? bserve_min_waves<T>(P) : wave2_min_waves<T>(kWpWave2 - P))
vi_bserve_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, T *__restrict__ V,
                 int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                 unsigned long long *__restrict__ host_out, const unsigned long long *__restrict__ host_cmd,
                 unsigned long long *__restrict__ breq, unsigned long long *__restrict__ gk, unsigned long long served,
                 unsigned long long idle_ticks, unsigned long long life_ticks, unsigned long long exit_tag, int copies,
                 int nap, int wait_pub, int prio_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ __attribute__((aligned(16))) unsigned long long s_box[2];  // the forwarder's poll mailbox
    const int lane = (int)threadIdx.x;
    constexpr bool multi = MULTI;  // past the resident capacity: several grids per workgroup
    const int e = multi ? 0 : (geo.order ? (int)geo.order[blockIdx.x] : (int)blockIdx.x);
    uint8_t *cl = smem + 256;
    if (!multi) copy16(cl, cells + (long long)e * geo.HWp, geo.HWp);
    T *tile = reinterpret_cast<T *>(smem + wave2_tile_off(geo.HWp));
    const bool fwd = blockIdx.x == 0;
    const unsigned long long tg = (exit_tag & 0xffffull) << 32;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();
    unsigned long long t_last = t_start, busy = 0, solves = 0;
    if (fwd && lane == 0) {
        s_box[0] = served;
        s_box[1] = 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS accesses are in order
    const long long vb = (long long)e * geo.S;
    while (true) {
        unsigned long long cmd;
        if (MGDP_BSERVE_PRIO) __builtin_amdgcn_s_setprio(0);
        if (fwd) {
            unsigned long long c = served;
            // Host polls are PCIe reads the forwarder keeps in flight (up to 24, LDS DMA); while other grids
            // of the request still sweep they would hold its CU's memory path (trace build: the grids
            // that finished 15-18 us after the rest).  So first wait, at agent scope, for the request's
            // publication (gk_exit's device copy of the epoch); the host posts the next one only after it.
            if (wait_pub && solves > 0) {
                while (__hip_atomic_load(gk + kGkTop2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       (served & 0xffffffffull)) {
                    if (__builtin_amdgcn_s_memrealtime() - t_start > life_ticks) break;
                    __builtin_amdgcn_s_sleep(4);
                }
                t_last = __builtin_amdgcn_s_memrealtime();  // the idle limit counts from the publication
            }
            if (lane == 0) {
                while (true) {
                    poll_issue(host_cmd, s_box);
                    __builtin_amdgcn_s_sleep(1);
                    c = __hip_atomic_load(&s_box[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (c != served) break;
                    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                    if (now - t_last > idle_ticks || now - t_start > life_ticks) {
                        c = kServeQuit;
                        break;
                    }
                }
            }
            cmd = rfl64(c);
            const unsigned long long dw =
                cmd == kServeQuit ? (tg | kBreqQuit) : (tg | (cmd & 0xffffffffull) | (cmd & kServeLast));
            if (lane < copies) {
#ifdef MGDP_BSERVE_TRACE  // trace build: the forwarder's request-seen stamp beside each copy
                __hip_atomic_store(breq + lane * 16 + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#endif
                __hip_atomic_store(breq + lane * 16, dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            unsigned long long dw;
            const unsigned long long *word = breq + (blockIdx.x % (unsigned)copies) * 16u;
            while (true) {  // the whole wave loads the word (one request): no divergent loop
                dw = rfl64(__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if ((dw & (0xffffull << 32)) == tg &&
                    ((dw & kBreqQuit) || (dw & 0xffffffffull) != (served & 0xffffffffull)))
                    break;
                if (__builtin_amdgcn_s_memrealtime() - t_start > life_ticks + kBserveGraceTicks) {
                    dw = tg | kBreqQuit;
                    break;
                }
                for (int i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(10);
            }
            cmd = (dw & kBreqQuit) ? kServeQuit : ((dw & 0xffffffffull) | (dw & kServeLast));
        }
        if (cmd == kServeQuit) break;
        if (MGDP_BSERVE_PRIO) {
            // the first prio_n workgroups hold the dispatch order's longest grids (MGDP_BSERVE_PRIO_FRAC)
            if ((int)blockIdx.x < prio_n) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(1);
        }
        const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
        int k = 0;
        double dvl = 0.0;
        auto done = [](int, double) {};
        if constexpr (MULTI) {
            // More grids than workgroups: this workgroup solves the dispatch order's positions
            // blockIdx.x, + G, + 2G, ... (round-robin over the longest-first order), each from V_0 = 0
            // with its cells staged in turn, and arrives ONCE at the counter tree with its grids'
            // {min, max} sweeps and max dV (a per-grid arrival would hold the wave on its ticket's round
            // trip before every next grid).
            int kmn = 0x7fffffff, kmx = 0;
            double dvm = 0.0;
            for (int i = (int)blockIdx.x; i < geo.B; i += (int)gridDim.x) {
                const int eg = geo.order ? (int)geo.order[i] : i;
                const long long vg = (long long)eg * geo.S;
                copy16(cl, cells + (long long)eg * geo.HWp, geo.HWp);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // one wave: the cells are in place
                int kg = 0;
                double dg = 0.0;
                fused_wave2_xyd<T, true, P, true, (bool)MGDP_BSERVE_OPQ>(geo, cf, cl, tile, V + vg, V + vg, pi + vg, kg, -1,
                                                                        dg, done, GkCtx{});
                if (lane == 0) {
                    kenv[eg] = kg;
                    if (geo.kexec) geo.kexec[eg] = kg;
                    dvenv[eg] = dg;
#ifdef MGDP_BSERVE_DEBUG_WG  // diagnostics build: which workgroup and iteration solved each grid
                    if (geo.kexec) geo.kexec[eg] = (int)blockIdx.x | (((i - (int)blockIdx.x) / (int)gridDim.x) << 20);
#endif
                }
                kmn = min(kmn, kg);
                kmx = max(kmx, kg);
                dvm = dg > dvm ? dg : dvm;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gk_exit<true>(GkCtx{gk, (unsigned int)cmd, (int)blockIdx.x, (int)gridDim.x, host_out}, kmx, dvm,
                          MGDP_BSERVE_OPQ ? late_tid(0) : lane, kmn);
            k = kmx;
        } else {
            fused_wave2_xyd<T, true, P, true, (bool)MGDP_BSERVE_OPQ>(geo, cf, cl, tile, V + vb, V + vb, pi + vb, k, -1, dvl,
                                                                    done, GkCtx{gk, (unsigned int)cmd, e, geo.B, host_out});
        }
        if (lane == 0 && !multi) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
#ifdef MGDP_BSERVE_TRACE  // trace build: this grid's start / end after the forwarder saw the request,
                          // 10 ns ticks in the low / high 16 bits of its executed-sweeps word
            const unsigned long long t0 = __hip_atomic_load(breq + (blockIdx.x % (unsigned)copies) * 16u + 1,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long a = t_seen - t0 < 0xffffull ? t_seen - t0 : 0xffffull;
            const unsigned long long b = t1 - t0 < 0xffffull ? t1 - t0 : 0xffffull;
            if (geo.kexec) geo.kexec[e] = (int)(a | (b << 16));
#endif
        }
        served = cmd;
        t_last = __builtin_amdgcn_s_memrealtime();
        busy += t_last - t_seen;
        ++solves;
        if (cmd & kServeLast) break;
    }
    // Leaving: this wave's stores complete (the exit V / pi stores are write-through, the clock words
    // system-scope: drained means written), then the exit counters; the last wave out resets them and
    // writes the launch's exit word.  Waves leaving after a kServeLast request do it while that
    // request's long grids still sweep, so (tools/probe_bserve.py, the last request's wall): no wave
    // but the last fences (a system-scope release writes back the L2: +35-60 us), and the count is a
    // two-level tree like the solve's (64 shard lines, then a top line) -- 8192 atomics on one word
    // serialised at ~10 ns each ahead of the request's own publication: +82 us.
    if (lane == 0 && fwd) {
        __hip_atomic_store(host_out + kHoutClk, __builtin_amdgcn_s_memtime() - c_start, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 1, __builtin_amdgcn_s_memrealtime() - t_start, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 2, busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_out + kHoutClk + 3, solves, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
        const unsigned int G = gridDim.x;
        const unsigned int nsh = G < (unsigned)kBreqExitShards ? G : (unsigned)kBreqExitShards;
        const unsigned int sh = blockIdx.x % nsh;
        const unsigned long long size = G / nsh + (sh < G % nsh ? 1u : 0u);
        unsigned long long *cnt = breq + kBreqExit + sh * 16u, *top = breq + kBreqExit + kBreqExitShards * 16;
        if (__hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == size - 1ull) {
            __hip_atomic_store(cnt, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(top, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1ull) {
                __hip_atomic_store(top, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(host_out + 11, exit_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// The fused solve with the SURVEY 8(f) item-3 options (ND = NoDeath lava, HMODE = finite horizon
// 1 / with pi_t 2): one workgroup per grid on the direction-major one-thread-per-cell path only
// (the host enforces MGDP_MAP_CELL and no pair / quad steps when options are set).
template <typename T, int MODEL, bool SLIP, bool ND, int HMODE>
__global__ void __launch_bounds__(1024)
vi_fused_opts_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, T *__restrict__ V,
                     int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                     unsigned long long *__restrict__ red, unsigned int *__restrict__ ticket,
                     unsigned long long *__restrict__ host_out, int k_target, int fresh, int in_kernel_reduce,
                     unsigned int epoch, const T *__restrict__ rgoal, int8_t *__restrict__ pi_t) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    T *V0 = reinterpret_cast<T *>(smem);
    T *V1 = reinterpret_cast<T *>(smem + L.v_bytes);
    uint8_t *cl = reinterpret_cast<uint8_t *>(smem + L.cells_off());
    T *slots = reinterpret_cast<T *>(smem + L.slots_off());
    uint8_t *flags = reinterpret_cast<uint8_t *>(smem + L.flags_off());
    const int e = blockIdx.x;
    int k = fresh ? 0 : kenv[e];
    double dvl = fresh ? 0.0 : dvenv[e];
    // fixed-point completion (fused_grid); not for a finite horizon, whose sweeps depend on the step
    if (HMODE == 0 && k_target > k && k > 0 && dvl == 0.0) {
        if (threadIdx.x == 0) kenv[e] = k_target;
        k = k_target;
    }
    const bool work = k_target < 0 ? (!(k > 0 && dvl < geo.tol) && k < geo.max_sweeps) : (k < k_target);
    const bool lone = in_kernel_reduce && gridDim.x == 1;
    if (work) {
        const long long vb = (long long)e * geo.S;
        copy16(cl, cells + (long long)e * geo.HWp, geo.HWp);
        if (threadIdx.x < 64) flags[threadIdx.x] = 0;
        __syncthreads();
        auto done = [&](int kk, double dv) {
            if (lone && threadIdx.x == 0)
                publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                        (unsigned long long)kk, epoch);
        };
        int8_t *pit = HMODE == 2 ? pi_t + vb : nullptr;
        const long long pstride = (long long)geo.B * geo.S;
        if constexpr (MODEL == MGDP_MODEL_XYD) {
            if constexpr (HMODE == 0) {
                if (k_target < 0)
                    fused_fast_xyd_soa<T, SLIP, true, ND, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb,
                                                                 k, k_target, dvl, done, rgoal, pit, pstride);
                else
                    fused_fast_xyd_soa<T, SLIP, false, ND, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb,
                                                                  k, k_target, dvl, done, rgoal, pit, pstride);
            } else {  // finite horizon: exactly k_target = H sweeps
                fused_fast_xyd_soa<T, SLIP, false, ND, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb,
                                                              k, k_target, dvl, done, rgoal, pit, pstride);
            }
        } else {
            if constexpr (HMODE == 0) {
                if (k_target < 0)
                    fused_fast_dk_soa<T, true, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k,
                                                      k_target, dvl, done, rgoal, pit, pstride);
                else
                    fused_fast_dk_soa<T, false, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k,
                                                       k_target, dvl, done, rgoal, pit, pstride);
            } else {
                fused_fast_dk_soa<T, false, HMODE>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k,
                                                   k_target, dvl, done, rgoal, pit, pstride);
            }
        }
        if (threadIdx.x == 0) {
            kenv[e] = k;
            if (geo.kexec) geo.kexec[e] = k;
            dvenv[e] = dvl;
        }
    }
    if (in_kernel_reduce)
        fused_reduce(red, ticket, host_out, k, dvl, reinterpret_cast<unsigned int *>(slots + 16), epoch, work,
                     (int)threadIdx.x);
}

// Dispatch order from the cells (round 6): a proxy for the sweep at which each grid's own rule stops,
// computed once per cells load, so the longest grids start first from a handle's FIRST solve on.
// For a deterministic grid that stop is the longest shortest path to the goal (plus one sweep), so the
// proxy is a breadth-first depth over cells (moves only, no turns): XYD, the farthest walkable cell
// from a goal; DoorKey, the larger of that (doors and keys passable) and the farthest cell of the
// key's side (door shut) from the key plus the key's distance to the goal (fetch the key, then the
// goal).  Spearman rank correlation with the own-rule stopping sweep over reference-generated grids
// (orc_vi_fp): FourRooms 0.985, LavaS11N5 0.873, DoorKey-16 0.994.  Results never
// depend on it.  One 64-lane workgroup per grid, level-synchronous BFS in LDS (a lane's LDS accesses
// are ordered and a cell at level L+1 is only set next to one at level L, so no barrier is needed).
constexpr int kDepthMaxHW = 1024;
__device__ __forceinline__ int depth_bfs(const uint8_t *cl, uint16_t *dist, int HW, int W, int src_type,
                                         bool dk_open) {
    const int lane = threadIdx.x;
    constexpr uint16_t kUnseen = 0xffff;
    auto passable = [&](int t) { return dk_open ? (xyd_free(t) || t == T_DOOR || t == T_KEY) : xyd_free(t); };
    for (int c = lane; c < HW; c += 64) dist[c] = cl[c] == src_type ? 0 : kUnseen;
    int level = 0, maxd = 0;
    while (true) {
        bool grew = false;
        for (int c = lane; c < HW; c += 64) {
            if (dist[c] != kUnseen || !passable(cl[c])) continue;
            const bool nb = (c >= W && dist[c - W] == level) || (c + W < HW && dist[c + W] == level) ||
                            (c % W != 0 && dist[c - 1] == level) || (c % W != W - 1 && dist[c + 1] == level);
            if (nb) {
                dist[c] = (uint16_t)(level + 1);
                grew = true;
            }
        }
        if (__ballot(grew) == 0ull) break;
        maxd = ++level;
    }
    return maxd;
}
__global__ void __launch_bounds__(64) vi_depth_kernel(Geo geo, const uint8_t *__restrict__ cells, int model,
                                                      int32_t *__restrict__ depth) {
    __shared__ uint8_t cl[kDepthMaxHW];
    __shared__ uint16_t d1[kDepthMaxHW], d2[kDepthMaxHW];
    const int b = blockIdx.x, HW = geo.HW, W = geo.W;
    for (int c = threadIdx.x; c < HW; c += 64) cl[c] = cells[(long long)b * geo.HWp + c];
    int proxy = depth_bfs(cl, d1, HW, W, T_GOAL, model == MGDP_MODEL_DOORKEY);
    if (model == MGDP_MODEL_DOORKEY) {
        // the key's distance to the goal (doors and keys passable: d1), then the key side's depth
        int kd = 0x7fffffff;
        for (int c = threadIdx.x; c < HW; c += 64)
            if (cl[c] == T_KEY && d1[c] != 0xffff) kd = min(kd, (int)d1[c]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) kd = min(kd, __shfl_xor(kd, o));
        const int side = depth_bfs(cl, d2, HW, W, T_KEY, false);
        if (kd != 0x7fffffff) proxy = max(proxy, side + kd);
    }
    if (threadIdx.x == 0) depth[b] = proxy;
}

// The sharded protocol's gate (mgdp_vi_run_to_dev_sync): kdv = the all-reduced {K, E}, written by
// the collective ordered before this launch.  E == 0: every grid everywhere is at an exact fixed
// point, so the result is {K, dV 0, K}; else kmin = kGateMore asks the host for run_to(K).
constexpr unsigned long long kGateMore = 0xffffffffull;
__global__ void __launch_bounds__(64) vi_gate_kernel(const long long *__restrict__ kdv,
                                                     unsigned long long *__restrict__ host_out, unsigned int epoch) {
    if (threadIdx.x == 0) {
        const unsigned long long K = (unsigned long long)kdv[0], E = (unsigned long long)kdv[1];
        publish_word2(host_out + 12, E, epoch);  // six tagged words, no drain between them
        publish(host_out, K, 0ull, E == 0 ? K : kGateMore, epoch);
    }
}

// Large batches: one workgroup reduces the per-grid (kenv, dvenv) into host-mapped memory (a
// single arrival ticket shared by tens of thousands of workgroups would serialise on one address).
__global__ void __launch_bounds__(1024)
vi_reduce_kernel(const int32_t *__restrict__ kenv, const double *__restrict__ dvenv, int B,
                 unsigned long long *__restrict__ host_out, unsigned int epoch) {
    __shared__ unsigned long long sk[16], sd[16], sn[16];
    unsigned long long km = 0, dm = 0, kn = 0x7fffffffull;
    auto fold = [&](int k, double d) {
        km = max(km, (unsigned long long)k);
        kn = min(kn, (unsigned long long)k);
        dm = max(dm, (unsigned long long)__double_as_longlong(d));
    };
    // 16-B loads, U of them in flight per thread before any is folded: one workgroup streaming
    // 12 B per grid is latency-bound (the one-load-per-iteration loop took 24 us for 65536 grids)
    constexpr int U = 4;
    const int B4 = B / 4;  // kenv / dvenv come from hipMalloc: 16-B aligned
    const int4 *k4 = reinterpret_cast<const int4 *>(kenv);
    const double2 *d2 = reinterpret_cast<const double2 *>(dvenv);
    const int step = (int)blockDim.x;
    for (int base = threadIdx.x; base < B4; base += U * step) {
        int4 kk[U];
        double2 da[U], db[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = min(base + u * step, B4 - 1);  // clamped re-reads are harmless for max/min
            kk[u] = k4[i];
            da[u] = d2[2 * i];
            db[u] = d2[2 * i + 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fold(kk[u].x, da[u].x);
            fold(kk[u].y, da[u].y);
            fold(kk[u].z, db[u].x);
            fold(kk[u].w, db[u].y);
        }
    }
    for (int i = 4 * B4 + (int)threadIdx.x; i < B; i += step) fold(kenv[i], dvenv[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        km = max(km, (unsigned long long)__shfl_xor(km, o));
        dm = max(dm, (unsigned long long)__shfl_xor(dm, o));
        kn = min(kn, (unsigned long long)__shfl_xor(kn, o));
    }
    if ((threadIdx.x & 63) == 0) { sk[threadIdx.x >> 6] = km; sd[threadIdx.x >> 6] = dm; sn[threadIdx.x >> 6] = kn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { km = max(km, sk[i]); dm = max(dm, sd[i]); kn = min(kn, sn[i]); }
        publish(host_out, km, dm, kn, epoch);
    }
}

// The same reduction over kRedShards workgroups (one shard each, so no two workgroups share an
// atomic address), the last arrival folding the shards and publishing -- fused_reduce's protocol,
// whose shards and ticket are idle when the fused launch does not reduce (B > inkernel_max).
__global__ void __launch_bounds__(256)
vi_reduce_multi_kernel(const int32_t *__restrict__ kenv, const double *__restrict__ dvenv, int B,
                       unsigned long long *__restrict__ red, unsigned int *__restrict__ ticket,
                       unsigned long long *__restrict__ host_out, unsigned int epoch) {
    __shared__ unsigned long long sk[4], sd[4], sn[4];
    __shared__ unsigned int last;
    unsigned long long km = 0, dm = 0, kn = 0x7fffffffull;
    auto fold = [&](int k, double d) {
        km = max(km, (unsigned long long)k);
        kn = min(kn, (unsigned long long)k);
        dm = max(dm, (unsigned long long)__double_as_longlong(d));
    };
    constexpr int U = 4;
    const int B4 = B / 4;
    const int4 *k4 = reinterpret_cast<const int4 *>(kenv);
    const double2 *d2 = reinterpret_cast<const double2 *>(dvenv);
    const int step = (int)(blockDim.x * gridDim.x);
    for (int base = (int)(blockIdx.x * blockDim.x + threadIdx.x); base < B4; base += U * step) {
        int4 kk[U];
        double2 da[U], db[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = min(base + u * step, B4 - 1);  // clamped re-reads are harmless for max/min
            kk[u] = k4[i];
            da[u] = d2[2 * i];
            db[u] = d2[2 * i + 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fold(kk[u].x, da[u].x);
            fold(kk[u].y, da[u].y);
            fold(kk[u].z, db[u].x);
            fold(kk[u].w, db[u].y);
        }
    }
    if (blockIdx.x == 0)
        for (int i = 4 * B4 + (int)threadIdx.x; i < B; i += (int)blockDim.x) fold(kenv[i], dvenv[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        km = max(km, (unsigned long long)__shfl_xor(km, o));
        dm = max(dm, (unsigned long long)__shfl_xor(dm, o));
        kn = min(kn, (unsigned long long)__shfl_xor(kn, o));
    }
    if ((threadIdx.x & 63) == 0) { sk[threadIdx.x >> 6] = km; sd[threadIdx.x >> 6] = dm; sn[threadIdx.x >> 6] = kn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { km = max(km, sk[i]); dm = max(dm, sd[i]); kn = min(kn, sn[i]); }
        unsigned long long *r = red + (blockIdx.x & (kRedShards - 1)) * 4;
        const unsigned long long a = __hip_atomic_fetch_max(r + 0, km, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_fetch_max(r + 1, dm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c = __hip_atomic_fetch_min(r + 2, kn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" :: "v"(a), "v"(b), "v"(c) : "memory");
        const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x < 64) {  // every shard's updates returned before its ticket add
        unsigned long long *r = red + threadIdx.x * 4;
        unsigned long long x = __hip_atomic_exchange(r + 0, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long y = __hip_atomic_exchange(r + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long z = __hip_atomic_exchange(r + 2, 0x7fffffffull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            x = max(x, (unsigned long long)__shfl_xor(x, o));
            y = max(y, (unsigned long long)__shfl_xor(y, o));
            z = min(z, (unsigned long long)__shfl_xor(z, o));
        }
        if (threadIdx.x == 0) {
            __hip_atomic_exchange(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            publish(host_out, x, y, z, epoch);
        }
    }
}

// Early exit of a speculatively enqueued sweep: the previous sweep already met the rule.
__device__ __forceinline__ bool prev_sweep_converged(const unsigned long long *shards, int k, double tol) {
    if (k <= 1) return false;
    const unsigned long long *prev = shards + (long long)(k - 2) * 8;
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) m = fmax(m, __longlong_as_double((long long)prev[i]));
    return m < tol;
}

// ------------------------------------------------------------------------------------------------
// One Jacobi sweep (index k, 1-based) of every grid, V double-buffered in HBM.  A workgroup
// stages a group of `m` consecutive grids (their V rows and cells are contiguous in HBM) into LDS
// with 16-B loads -- the LDS tile of the neighbourhood --, updates them from LDS and writes the
// new rows back with 16-B stores; m > 1 keeps more bytes in flight per load phase and amortises
// the barriers.  check_prev: skip when the previous sweep's global max|dV| was already < tol.
// POLICY: evaluate only, write pi.
// ------------------------------------------------------------------------------------------------
constexpr int kSweepBlock = 256;

__host__ __device__ inline int sweep_smem_bytes(int S, int HWp, int tsize, int m) {
    return 2 * m * S * tsize + m * ((S + 15) / 16 * 16) + m * HWp + 256;
}

template <typename T, int MODEL, bool SLIP, int MAP, bool POLICY>
__global__ void __launch_bounds__(kSweepBlock)
vi_sweep_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, const T *__restrict__ Vin,
                T *__restrict__ Vout, int8_t *__restrict__ pi, unsigned long long *__restrict__ shards,
                int k, int check_prev, int m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if (check_prev && prev_sweep_converged(shards, k, geo.tol)) return;
    const int vbytes = geo.S * (int)sizeof(T), pib = (geo.S + 15) / 16 * 16;
    T *Vi = reinterpret_cast<T *>(smem);
    T *Vo = reinterpret_cast<T *>(smem + m * vbytes);
    int8_t *pis = reinterpret_cast<int8_t *>(smem + 2 * m * vbytes);
    uint8_t *cl = reinterpret_cast<uint8_t *>(smem + 2 * m * vbytes + m * pib);
    T *slots = reinterpret_cast<T *>(smem + 2 * m * vbytes + m * pib + m * geo.HWp);
    const int ngroups = (geo.B + m - 1) / m;

    T acc = (T)0;
    for (int gidx = blockIdx.x; gidx < ngroups; gidx += gridDim.x) {
        const int e0 = gidx * m;
        const int me = min(m, geo.B - e0);
        const long long vb = (long long)e0 * geo.S;
        __syncthreads();  // the previous group's LDS tile is no longer read
        copy16(cl, cells + (long long)e0 * geo.HWp, me * geo.HWp);
        copy16_nt_in(Vi, Vin + vb, me * vbytes);
        __syncthreads();
        for (int j = 0; j < me; ++j)
            acc = vmax(acc, sweep_lds<T, MODEL, SLIP, MAP, !POLICY, POLICY || MAP == MGDP_MAP_SA>(
                                geo, cf, cl + j * geo.HWp, Vi + j * geo.S, Vo + j * geo.S, pis + j * pib));
        __syncthreads();
        if (!POLICY) {
            copy16_nt_out(Vout + vb, Vo, me * vbytes);
        } else {
            for (int j = 0; j < me; ++j) copy_pi(pi + vb + (long long)j * geo.S, pis + j * pib, geo.S);
        }
    }
    if (!POLICY) {
        const T bdv = block_max(acc, slots, 0);
        if (threadIdx.x == 0 && shards)
            atomicMax(shards + (long long)(k - 1) * 8 + (blockIdx.x & 7),
                      (unsigned long long)__double_as_longlong((double)bdv));
    }
}

// ------------------------------------------------------------------------------------------------
// Register-pipelined HBM sweep (one thread per cell, HW <= blockDim = HWs): a workgroup walks its
// grids e = blockIdx.x + i*gridDim.x.  Each thread loads its own cell's V row (16 B XYD, 64 B
// DoorKey fp32, coalesced) and a dword of cell bytes DEPTH grids ahead into registers, so the HBM
// reads of the next grids are in flight while the current one is computed and stored; at the top
// of an iteration the registers are written to the direction-major LDS tile (the neighbourhood
// the front-cell reads need, bank-conflict free), the thread keeps its own values in registers and
// stores its new row straight to HBM.  LDS is only the neighbour exchange: no output staging.
// Same backups and |dV| as vi_sweep_kernel (bit-identical); pi stays with vi_sweep_kernel<POLICY>.
// ------------------------------------------------------------------------------------------------
template <typename T, int MODEL>
struct PipeRow {
    static constexpr int NV = MODEL == MGDP_MODEL_XYD ? 1 : 4;  // V4 per cell
    V4<T> v[NV];
    uint32_t cw;  // cell bytes 4c .. 4c+3 (threads c < HWp/4)
};

__host__ __device__ inline int sweep_pipe_smem_bytes(int S, int HW, int HWs, int HWp, int tsize) {
    return S / HW * HWs * tsize + HWp + 256;
}

// V is streamed once per sweep (Vin read, Vout written; the next sweep's Vin is the whole
// 553 MB array again, far past the 256 MB MALL), so the loads and stores are nontemporal:
// bit 0 stores, bit 1 loads.  Measured on empty16x65536 (profiles/r01_sweep_nt/): 107.8 µs
// plain, 101.5 µs stores only, 98.0 µs both.
#ifndef MGDP_SWEEP_NT
#define MGDP_SWEEP_NT 3
#endif
template <typename T>
__device__ __forceinline__ void st_v4(V4<T> *dst, const V4<T> &v) {
    if (MGDP_SWEEP_NT & 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v.v[j], &dst->v[j]);
    } else {
        *dst = v;
    }
}
template <typename T>
__device__ __forceinline__ V4<T> ld_v4(const V4<T> *src) {
    if (MGDP_SWEEP_NT & 2) {
        V4<T> v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v.v[j] = __builtin_nontemporal_load(&src->v[j]);
        return v;
    }
    return *src;
}

template <typename T, int MODEL, bool SLIP, int DEPTH>
__global__ void __launch_bounds__(1024)
vi_sweep_pipe_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, const T *__restrict__ Vin,
                     T *__restrict__ Vout, unsigned long long *__restrict__ shards, int k, int check_prev) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if (check_prev && prev_sweep_converged(shards, k, geo.tol)) return;
    using Row = PipeRow<T, MODEL>;
    constexpr int NV = Row::NV;
    const int HWs = geo.HWs;
    T *Vt = reinterpret_cast<T *>(smem);
    uint8_t *cl = smem + (size_t)geo.Ss * sizeof(T);
    T *slots = reinterpret_cast<T *>(smem + (size_t)geo.Ss * sizeof(T) + geo.HWp);
    const int c = threadIdx.x;
    const bool own_cell = c < geo.HW;
    const bool cell_word = c < (geo.HWp >> 2);
    const int cc = own_cell ? c : 0;
    const int stride = gridDim.x;

    // Unconditional loads (clamped addresses: past the last grid, idle threads re-read a valid row
    // whose values are never used), so the loop body is straight-line and the compiler's vmcnt
    // waits count the DEPTH-1 younger fetches instead of draining them.
    const int cw_idx = cell_word ? c : 0;
    auto fetch = [&](int e, Row &r) {
        const long long ee = e < geo.B ? e : geo.B - 1;
        const V4<T> *src = reinterpret_cast<const V4<T> *>(Vin + ee * geo.S + (long long)cc * 4 * NV);
#pragma unroll
        for (int q = 0; q < NV; ++q) r.v[q] = ld_v4(src + q);
        r.cw = reinterpret_cast<const uint32_t *>(cells + ee * geo.HWp)[cw_idx];
    };
    Row rows[DEPTH];
#pragma unroll
    for (int s = 0; s < DEPTH; ++s) fetch(blockIdx.x + s * stride, rows[s]);
    T acc = (T)0;
    auto step = [&](int e, Row &r) {
        // stage this grid's rows; every thread is past the previous grid's LDS reads (barrier below)
        if (MODEL == MGDP_MODEL_XYD) {
#pragma unroll
            for (int d = 0; d < 4; ++d) Vt[d * HWs + c] = r.v[0].v[d];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) *reinterpret_cast<V4<T> *>(Vt + (q * HWs + c) * 4) = r.v[q];
        }
        if (cell_word) reinterpret_cast<uint32_t *>(cl)[c] = r.cw;
        __syncthreads();
        // refill in place, DEPTH grids ahead: r is dead once staged (the thread's own values are read
        // back from the tile), so the loads need no register copies and stay in flight during this
        // grid's work
        fetch(e + DEPTH * stride, r);
        Row own;
        if (MODEL == MGDP_MODEL_XYD) {
#pragma unroll
            for (int d = 0; d < 4; ++d) own.v[0].v[d] = Vt[d * HWs + c];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) own.v[q] = *reinterpret_cast<const V4<T> *>(Vt + (q * HWs + c) * 4);
        }
        T *dst = Vout + (long long)e * geo.S + (long long)c * 4 * NV;
        if (MODEL == MGDP_MODEL_XYD) {
            const XydTopo<T> tp = xyd_topo_soa<T>(cl, geo, cc);
            T nbv[4];
            xyd_load_nb(tp, Vt, nbv);
            V4<T> out;
            uint32_t pk;
            const T dv = xyd_step<T, SLIP, false>(tp, cf, own.v[0], nbv, out, pk);
            if (own_cell) {
                st_v4(reinterpret_cast<V4<T> *>(dst), out);
                acc = vmax(acc, dv);
            }
        } else {
            const DkTopo tp = dk_topo_soa(cl, geo, cc);
            V4<T> nbs[4];
            dk_load_nb(tp, Vt, nbs);
            T in[16], outv[16];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) in[4 * q + j] = own.v[q].v[j];
            uint32_t pk[4];
            const T dv = dk_step<T, false>(tp, cf, in, nbs, outv, pk);
            if (own_cell) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_v4(reinterpret_cast<V4<T> *>(dst) + q, V4<T>{{outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]}});
                acc = vmax(acc, dv);
            }
        }
        __syncthreads();  // the tile is rewritten by the next grid
    };
    int e = blockIdx.x;
    bool more = true;
    while (more) {  // the register slots rotate: slot j holds the grid DEPTH strides ahead of it
#pragma unroll
        for (int j = 0; j < DEPTH; ++j) {
            if (e >= geo.B) { more = false; break; }
            step(e, rows[j]);
            e += stride;
        }
    }
    const T bdv = block_max(acc, slots, 0);
    if (threadIdx.x == 0 && shards)
        atomicMax(shards + (long long)(k - 1) * 8 + (blockIdx.x & 7), (unsigned long long)__double_as_longlong((double)bdv));
}

}  // namespace mgdp
