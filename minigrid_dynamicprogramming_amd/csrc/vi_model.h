// vi_model.h -- the DP model on the device: geometry, per-cell topology, the Bellman
// backups (XYD / DoorKey), wave and block reductions, convergence flags.
// Part of the single translation unit vi.hip (included in order: vi_model.h, vi_loops.h,
// vi_kernels.h); see vi.hip for the DP semantics and the data layout.
#pragma once

namespace mgdp {

struct Geo {
    int B, W, H, HW, HWp, S;
    int HWs, Ss;  // direction-major LDS tiles: cell stride HWs = round_up(HW, 64) (one slot per thread), Ss = S/HW*HWs
    int off[4];  // cell offset of the front cell for dir 0..3 (+x, +y, -x, -y)
    int max_sweeps;
    int nbuf;    // LDS V buffers of the fused kernel: 2, or 3 for the two-sweep XYD step
    int quad;    // fused XYD: 4 threads per cell (one per direction) instead of one
    int pair;    // fused XYD: two-sweep step
    double tol;
    int32_t *kexec;  // per grid: the sweep index it last computed (mgdp_vi_get_grid_sweeps); nullptr = off
    // Learned dispatch (round 5): when the same grids are solved again, workgroup b takes grid
    // order[b] (longest previous solve first) and a grid whose previous solve ran >= kprio[i]
    // sweeps raises its waves' issue priority to 3 - i (nullptr / 0: off).  Results do not depend
    // on either: grids are independent.
    const int32_t *order;
    int kprio[3];
    // Mixed wave counts (round 5, fused_mix tags): the first nmix workgroups of the learned order
    // (the grids whose previous solve ran longest) take two waves per grid, the rest one.
    int nmix;
    // The batch fits the one-wave kernel's resident capacity: its own-rule launches write their exit
    // V / pi through the L2 (fused_wave2_xyd WT, store_v4_exit)
    int wt;
};

template <typename T>
struct Coef {
    T g, p, c;  // gamma, slip keep-prob, (1-p)/6   (all rounded to T once on the host)
    T tol;      // smallest T >= tol: for x of type T, x >= tol (T)  <=>  (double)x >= tol
    T dc;       // NoDeath: reward for entering lava (the wrapper's death_cost)
};

template <typename T>
struct alignas(4 * sizeof(T)) V4 {
    T v[4];
};
template <typename T>
struct alignas(2 * sizeof(T)) V2 {
    T v[2];
};

__device__ __forceinline__ bool xyd_free(int t) { return t == T_EMPTY || t == T_FLOOR; }
__device__ __forceinline__ bool dk_walk(int t, int hk, int dop) {
    return t == T_EMPTY || t == T_FLOOR || (t == T_DOOR && dop) || (t == T_KEY && hk);
}

// All values handled here are finite and >= +0 (V in [0, 1], rewards in {0, 1}), so max() is
// order-independent and equal to the oracle's "strictly greater replaces" scan, and
// |a - b| equals the oracle's (a > b ? a - b : b - a) bit for bit.
template <typename T>
__device__ __forceinline__ T tmax(T a, T b) { return a > b ? a : b; }
__device__ __forceinline__ float vmax(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double vmax(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ float vabs(float a) { return fabsf(a); }
__device__ __forceinline__ double vabs(double a) { return fabs(a); }

// DPP move of a 32/64-bit value (all lanes active).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float lane_read(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ double lane_read(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Wave max of non-negative values: DPP within rows of 16 lanes (quad swaps, half-row and row
// mirrors), then the four row results by readlane -- no LDS round trips.
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
    v = tmax(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
    v = tmax(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
    v = tmax(v, dpp_mov<0x141>(v));  // row_half_mirror
    v = tmax(v, dpp_mov<0x140>(v));  // row_mirror
    return tmax(tmax(lane_read(v, 0), lane_read(v, 16)), tmax(lane_read(v, 32), lane_read(v, 48)));
}

// The thread index re-derived after a long loop: the wave index (workgroup-uniform, an SGPR the
// caller took before the loop) * 64 + the lane from v_mbcnt.  The mbcnt is asm, so the compiler
// cannot substitute the thread-index VGPR kept from before the loop: a kernel whose loop needs
// every VGPR then keeps no per-thread index live across it (the batched DoorKey loop at 80 VGPRs
// spilled it to scratch).
__device__ __forceinline__ int late_tid(int wave_s) {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return (wave_s << 6) | l;
}

// Block-wide max with ONE barrier; slots = [2][16] alternating by parity so that consecutive
// calls never race (a slot set is rewritten only after every thread passed the next barrier).
// tid: the caller's thread index (late_tid after a long loop).
template <typename T>
__device__ __forceinline__ T block_max_tid(T v, T *slots, int parity, int tid) {
    v = wave_max(v);
    const int w = tid >> 6;
    if ((tid & 63) == 0) slots[parity * 16 + w] = v;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    T m = slots[parity * 16];
    for (int i = 1; i < nw; ++i) m = tmax(m, slots[parity * 16 + i]);
    return m;
}
template <typename T>
__device__ __forceinline__ T block_max(T v, T *slots, int parity) { return block_max_tid(v, slots, parity, (int)threadIdx.x); }

// Block-wide OR of a predicate with ONE barrier: one byte flag per wave, two parities.
__device__ __forceinline__ bool block_any(bool p, uint8_t *flags, int parity) {
    const unsigned long long b = __ballot(p);
    if ((threadIdx.x & 63) == 0) flags[parity * 16 + (threadIdx.x >> 6)] = b != 0ull;
    __syncthreads();
    const uint4 f = *reinterpret_cast<const uint4 *>(flags + parity * 16);
    return (f.x | f.y | f.z | f.w) != 0u;
}

// Split form of block_any for loops that test the PREVIOUS sweep's flags right after the
// barrier, in parallel with the next sweep's LDS reads: flag_write before the barrier,
// flags_any after it (same two-parity protocol).
__device__ __forceinline__ void flag_write(bool p, uint8_t *flags, int parity) {
    const unsigned long long b = __ballot(p);
    if ((threadIdx.x & 63) == 0) flags[parity * 16 + (threadIdx.x >> 6)] = b != 0ull;
}
__device__ __forceinline__ bool flags_any(const uint8_t *flags, int parity) {
    if (blockDim.x <= 256)  // <= 4 waves: their flag bytes are one dword
        return *reinterpret_cast<const uint32_t *>(flags + parity * 16) != 0u;
    const uint4 f = *reinterpret_cast<const uint4 *>(flags + parity * 16);
    return (f.x | f.y | f.z | f.w) != 0u;
}

// ------------------------------------------------------------------------------------------------
// Per-cell topology.  Cell types never change during a solve, so a thread that owns a cell can
// resolve its transition structure once (from LDS or HBM) and keep it in registers for every
// sweep.  The update code below is branch-free: every case is a select on these registers.
// ------------------------------------------------------------------------------------------------
template <typename T>
struct XydTopo {
    int valid;       // agent may stand here (empty / floor)
    uint32_t term;   // bit d: forward from dir d enters a terminal cell (goal / lava)
    int nbi[4];      // V index read by forward from dir d (own state when blocked / terminal / invalid)
    T tq[4];         // terminal forward value: 1 (goal, R = 1) or 0 (lava)
    uint32_t lavaF;  // NoDeath: bit d = forward from dir d enters (walkable, non-terminal) lava
    uint32_t halo;   // served pair loop (serve_pair_halo): bit 0 the halo cell is walkable, bit 1 a goal ahead of it
};

template <typename T, bool ND = false>
__device__ __forceinline__ XydTopo<T> xyd_topo(const uint8_t *cl, const Geo &geo, int c) {
    XydTopo<T> tp;
    // NoDeath (wrappers.py:799-872): the agent may stand on lava; entering it is not terminal
    tp.valid = xyd_free(cl[c]) || (ND && cl[c] == T_LAVA);
    tp.term = 0;
    tp.lavaF = 0;
    tp.halo = 0;
    // Branch-free (selects only, every LDS byte read unconditional): it runs once per grid-sweep
    // in the HBM sweep kernels.
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int cfr = tp.valid ? c + geo.off[d] : c;  // valid cells are interior (closed border)
        const int tf0 = cl[cfr];
        const int tf = tp.valid ? tf0 : T_WALL;
        const bool goal = tf == T_GOAL, lava = tf == T_LAVA;
        const bool enter = xyd_free(tf) || (ND && lava);  // forward reads the front cell's state
        tp.term |= (uint32_t)(goal || (!ND && lava)) << d;
        tp.lavaF |= (uint32_t)(ND && lava) << d;
        tp.tq[d] = goal ? (T)1 : (T)0;
        tp.nbi[d] = (enter ? cfr : c) * 4 + d;
    }
    return tp;
}

// One cell of the XYD model: own = V_{k-1} of the cell's 4 states (registers), front values read
// from Vin.  Q_det: left/right/self (= pickup/drop/toggle/done) = g*V, forward per
// minigrid_env.py:546-553.  Invalid cells have own = 0 and all reads pointing at themselves, so
// they compute exactly 0.  Returns max |dV|; with WRITE_PI also packs the 4 argmax lanes.
template <typename T>
__device__ __forceinline__ void xyd_load_nb(const XydTopo<T> &tp, const T *Vin, T (&nbv)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) nbv[d] = Vin[tp.nbi[d]];
}

// ND: NoDeath lava (entering it: Q = death_cost + g*V[lava state]); FH: finite horizon, the goal
// reward of this sweep is rg (the exact _reward() of its step_count) instead of 1.
template <typename T, bool SLIP, bool WRITE_PI, bool ND = false, bool FH = false>
__device__ __forceinline__ T xyd_step(const XydTopo<T> &tp, const Coef<T> &cf, const V4<T> &own,
                                      const T (&nbv)[4], V4<T> &out, uint32_t &pk, T rg = (T)1) {
    if (!SLIP && !WRITE_PI) {
        // Deterministic value-only form.  Rounding is monotone and g >= 0, V >= 0, so
        //   max_a fl(g * x_a) = fl(g * max_a x_a)   and   max(., 0) is the identity:
        // V'[d] = max(fl(g_eff * max(V[d-1], V[d], V[d+1], F[d])), tq[d]) with F[d] the value
        // forward reads (own V[d] when blocked / terminal), tq[d] = 1 for a goal ahead, 0
        // otherwise (lava: Q = 0), and g_eff = 0 for absorbing cells (V' = +0).  Bit-identical to
        // the per-action form below (which the policy pass keeps).  NoDeath: the lava move
        // carries a reward, so it is its own candidate fl(dc + fl(g * F[d])); V >= 0 still holds
        // (turning in place is always worth g*V >= 0), so max with 0 stays the identity.
        const T ge = tp.valid ? cf.g : (T)0;
        T f[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) f[d] = (ND && ((tp.lavaF >> d) & 1u)) ? own.v[d] : nbv[d];
        const T m02 = vmax(own.v[0], own.v[2]), m13 = vmax(own.v[1], own.v[3]);
        const T m[4] = {vmax(vmax(own.v[0], m13), f[0]), vmax(vmax(own.v[1], m02), f[1]),
                        vmax(vmax(own.v[2], m13), f[2]), vmax(vmax(own.v[3], m02), f[3])};
        T dv = (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            T best = vmax(ge * m[d], FH ? tp.tq[d] * rg : tp.tq[d]);
            if (ND) best = vmax(best, ((tp.lavaF >> d) & 1u) ? cf.dc + cf.g * nbv[d] : (T)0);
            out.v[d] = best;
            dv = vmax(dv, vabs(best - own.v[d]));
        }
        pk = 0;
        return dv;
    }
    T gv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) gv[d] = cf.g * own.v[d];
    T dv = (T)0;
    pk = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const T qM = (ND && ((tp.lavaF >> d) & 1u)) ? cf.dc + cf.g * nbv[d] : cf.g * nbv[d];
        const T qF = ((tp.term >> d) & 1u) ? (FH ? tp.tq[d] * rg : tp.tq[d]) : qM;
        const T qL = gv[(d + 3) & 3], qR = gv[(d + 1) & 3], qS = gv[d];
        T a0 = qL, a1 = qR, a2 = qF, a3 = qS;  // Q of actions 0..3 (4..6 equal action 3)
        if (SLIP) {
            T s6 = qL + qR;
            s6 = s6 + qF;
            s6 = s6 + qS;
            s6 = s6 + qS;
            s6 = s6 + qS;
            const T tail = cf.c * s6;
            a0 = cf.p * qL + tail;
            a1 = cf.p * qR + tail;
            a2 = cf.p * qF + tail;
            a3 = cf.p * qS + tail;
        }
        T best;
        if (WRITE_PI) {
            int arg = 0;
            best = a0;
            if (a1 > best) { best = a1; arg = 1; }
            if (a2 > best) { best = a2; arg = 2; }
            if (a3 > best) { best = a3; arg = 3; }
            pk |= (uint32_t)(uint8_t)(tp.valid ? arg : -1) << (8 * d);
        } else {
            best = vmax(vmax(a0, a1), vmax(a2, a3));
        }
        best = tp.valid ? best : (T)0;  // slip mixes in constants; absorbing states stay 0
        out.v[d] = best;
        dv = vmax(dv, vabs(best - own.v[d]));
    }
    return dv;
}

// DoorKey cell topology: own walkability per (has_key, door_open) and, per direction, the front
// cell's kind, packed in registers.
struct DkTopo {
    uint32_t walk;   // bit (hk*2+dop): the agent may stand in this cell
    uint32_t f[4];   // per dir: bits 0-3 front walkable per (hk*2+dop), 4 goal, 5 lava, 6 key, 7 door
    int nb[4];       // V index of (front cell, dir d, has_key 0, door_open 0)
};

__device__ __forceinline__ uint32_t dk_walk_mask(int t) {
    uint32_t m = 0;
#pragma unroll
    for (int hk = 0; hk < 2; ++hk)
#pragma unroll
        for (int dop = 0; dop < 2; ++dop)
            if (dk_walk(t, hk, dop)) m |= 1u << (hk * 2 + dop);
    return m;
}

__device__ __forceinline__ DkTopo dk_topo(const uint8_t *cl, const Geo &geo, int c) {
    DkTopo tp;
    const int t = cl[c];
    tp.walk = dk_walk_mask(t);
    const bool inner = tp.walk != 0;  // walkable for some (hk, door): interior by validation
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int cfr = inner ? c + geo.off[d] : c;
        const int tf0 = cl[cfr];  // unconditional read, select below (branch-free)
        const int tf = inner ? tf0 : T_WALL;
        tp.f[d] = dk_walk_mask(tf) | (tf == T_GOAL ? 16u : 0u) | (tf == T_LAVA ? 32u : 0u) |
                  (tf == T_KEY ? 64u : 0u) | (tf == T_DOOR ? 128u : 0u);
        tp.nb[d] = cfr * 16 + d * 4;
    }
    return tp;
}

// One cell of the DoorKey product model: 16 states l = (dir*2 + has_key)*2 + door_open, action
// lanes left, right, forward, pickup, toggle (world_object.py:185-195, 244).  own = V_{k-1}.
template <typename T>
__device__ __forceinline__ void dk_load_nb(const DkTopo &tp, const T *Vin, V4<T> (&nb)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) nb[d] = *reinterpret_cast<const V4<T> *>(Vin + tp.nb[d]);
}

// FH: finite horizon, the goal reward of this sweep is rg instead of 1 (see xyd_step).
template <typename T, bool WRITE_PI, bool FH = false>
__device__ __forceinline__ T dk_step(const DkTopo &tp, const Coef<T> &cf, const T (&own)[16],
                                     const V4<T> (&nbs)[4], T (&outv)[16], uint32_t (&pk)[4], T rg = (T)1) {
    if (!WRITE_PI) {
        // Value-only form (see xyd_step): every non-terminal Q is fl(g * x) with x >= 0, so the
        // max over actions is fl(g * max x) -- one multiply per state -- and a goal ahead adds the
        // constant 1, lava the constant 0 (a no-op under max).  Bit-identical to the per-action
        // form below.
        T dv = (T)0;
#pragma unroll
        for (int q = 0; q < 4; ++q) pk[q] = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t f = tp.f[d];
            const V4<T> &nb = nbs[d];
            const bool key = f & 64u, door = f & 128u;
            const uint32_t fw = (f & 48u) ? 0u : f;  // forward reads the front state only when it is not terminal
            const T tqd = (f & 16u) ? (FH ? rg : (T)1) : (T)0;
#pragma unroll
            for (int hk = 0; hk < 2; ++hk) {
#pragma unroll
                for (int dop = 0; dop < 2; ++dop) {
                    const int l = (d * 2 + hk) * 2 + dop;
                    const int hd = hk * 2 + dop;
                    const T xS = own[l];
                    const T xL = own[(((d + 3) & 3) * 2 + hk) * 2 + dop];
                    const T xR = own[(((d + 1) & 3) * 2 + hk) * 2 + dop];
                    const T xF = ((fw >> hd) & 1u) ? nb.v[hd] : xS;
                    const T xP = (!hk && key) ? own[(d * 2 + 1) * 2 + dop] : xS;
                    const T xD = dop ? own[(d * 2 + hk) * 2 + 0] : (hk ? own[(d * 2 + hk) * 2 + 1] : xS);
                    const T xT = door ? xD : xS;
                    const T M = vmax(vmax(vmax(xL, xR), xS), vmax(vmax(xF, xP), xT));
                    const T best = ((tp.walk >> hd) & 1u) ? vmax(cf.g * M, tqd) : (T)0;
                    outv[l] = best;
                    dv = vmax(dv, vabs(best - own[l]));
                }
            }
        }
        return dv;
    }
    T gv[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) gv[l] = cf.g * own[l];
    T dv = (T)0;
#pragma unroll
    for (int q = 0; q < 4; ++q) pk[q] = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.f[d];
        const V4<T> &nb = nbs[d];
        const bool goal = f & 16u, lava = f & 32u, key = f & 64u, door = f & 128u;
#pragma unroll
        for (int hk = 0; hk < 2; ++hk) {
#pragma unroll
            for (int dop = 0; dop < 2; ++dop) {
                const int l = (d * 2 + hk) * 2 + dop;
                const int hd = hk * 2 + dop;
                const T qS = gv[l];
                const T qL = gv[(((d + 3) & 3) * 2 + hk) * 2 + dop];
                const T qR = gv[(((d + 1) & 3) * 2 + hk) * 2 + dop];
                const T qM = ((f >> hd) & 1u) ? cf.g * nb.v[hd] : qS;
                const T qF = goal ? (FH ? rg : (T)1) : (lava ? (T)0 : qM);
                const T qP = (!hk && key) ? gv[(d * 2 + 1) * 2 + dop] : qS;
                const T qD = dop ? gv[(d * 2 + hk) * 2 + 0] : (hk ? gv[(d * 2 + hk) * 2 + 1] : qS);
                const T qT = door ? qD : qS;
                const bool valid = (tp.walk >> hd) & 1u;
                T best;
                if (WRITE_PI) {
                    best = qL;
                    int arg = 0;
                    if (qR > best) { best = qR; arg = 1; }
                    if (qF > best) { best = qF; arg = 2; }
                    if (qP > best) { best = qP; arg = 3; }
                    if (qT > best) { best = qT; arg = 4; }
                    pk[l >> 2] |= (uint32_t)(uint8_t)(valid ? arg : -1) << (8 * (l & 3));
                } else {
                    best = vmax(vmax(vmax(qL, qR), vmax(qF, qP)), qT);
                }
                best = valid ? best : (T)0;
                outv[l] = best;
                dv = vmax(dv, vabs(best - own[l]));
            }
        }
    }
    return dv;
}

// Select-light value sweep of the DoorKey model (value-only form of dk_step, bit-identical).
// Invalid states hold +0 in every tile (absorbing, never written otherwise) and V >= +0, so:
//  * forward reads the front group whenever the front is walkable for SOME (has_key, door_open)
//    -- a door or key front's non-walkable states are exactly its invalid, +0 states -- and a
//    front forward never reads (wall, goal, lava, or any front of an absorbing cell) points at
//    cell 0's group, a border cell that stays +0: no per-state select, max(., +0) is a no-op;
//  * pickup (key ahead, has_key 0) and toggle (door ahead) add one candidate state each, +0 where
//    the front is neither (one select per state, only in waves with such a cell: KD);
//  * a cell walkable for only some (has_key, door_open) -- the door and key cells themselves --
//    zeroes its invalid states (one select per state, same waves); an absorbing cell's own
//    values, front read and goal flag are +0, so it yields +0 with no select;
//  * max(fl(g*M), tq) is needed only in waves with a goal ahead of some cell (GOAL).
// Every dropped candidate equals V[S] or is +0 <= V[S], and max is exact and order-free, so
// V' and the |dV| test are those of dk_step's per-state form.  ~4.5 VALU per state in plain waves
// (no key, door or goal next to any cell: most of a 16x16 grid) instead of ~11.
struct DkFast {
    uint32_t walk;   // as DkTopo
    uint32_t f[4];   // bit 4 goal ahead (walkable own cell only), 6 key ahead, 7 door ahead
    int nb[4];       // direction-major LDS index of the group forward reads (cell 0's when none)
};
__device__ __forceinline__ DkFast dk_fast_topo(const DkTopo &tp, int HWs) {  // tp: soa indices
    DkFast q;
    q.walk = tp.walk;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.f[d];
        const bool reads = tp.walk != 0u && !(f & 48u) && (f & 15u) != 0u;
        q.nb[d] = reads ? tp.nb[d] : d * HWs * 4;
        q.f[d] = tp.walk != 0u ? (f & (16u | 64u | 128u)) : 0u;
    }
    return q;
}
// wave class bits: 1 = some cell has a goal ahead, 2 = some cell has a key / door ahead or is one
__device__ __forceinline__ uint32_t dk_fast_class(const DkFast &q) {
    uint32_t goal = 0, kd = (q.walk != 0u && q.walk != 15u) ? 1u : 0u;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        goal |= (q.f[d] & 16u) ? 1u : 0u;
        kd |= (q.f[d] & 192u) ? 1u : 0u;
    }
    return goal | (kd << 1);
}

// DV = false: the value sweep only (returns 0) -- for the sweeps of a k_target loop whose |dV| is
// not reported (only the last one's is).
template <typename T, bool FH, bool GOAL, bool KD, bool DV = true>
__device__ __forceinline__ T dk_step_fast(const DkFast &tp, const Coef<T> &cf, const T (&own)[16],
                                          const V4<T> (&nbs)[4], T (&outv)[16], T rg = (T)1) {
    T df[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.f[d];
        const bool key = f & 64u, door = f & 128u;
        const T tqd = (f & 16u) ? (FH ? rg : (T)1) : (T)0;
#pragma unroll
        for (int hk = 0; hk < 2; ++hk) {
#pragma unroll
            for (int dop = 0; dop < 2; ++dop) {
                const int hd = hk * 2 + dop, l = d * 4 + hd;
                const T xS = own[l];
                T M = vmax(vmax(own[((d + 3) & 3) * 4 + hd], own[((d + 1) & 3) * 4 + hd]), vmax(xS, nbs[d].v[hd]));
                if (KD) {
                    // pickup -> (d, 1, dop); toggle -> close (dop 1: (d, hk, 0)) / unlock (hk 1, dop 0: (d, 1, 1))
                    T cand = (T)0;
                    if (!hk) cand = key ? own[d * 4 + 2 + dop] : cand;
                    if (dop) cand = door ? own[d * 4 + hk * 2] : cand;
                    else if (hk) cand = door ? own[d * 4 + 3] : cand;
                    M = vmax(M, cand);
                }
                T best = cf.g * M;
                if (GOAL) best = vmax(best, tqd);
                if (KD) best = ((tp.walk >> hd) & 1u) ? best : (T)0;
                outv[l] = best;
                df[l] = vabs(best - xS);
            }
        }
    }
    if constexpr (!DV) return (T)0;
    // max is exact and order-free: a three-input tree (v_max3) over the 16 differences
    const T a = vmax(vmax(df[0], df[1]), df[2]), b = vmax(vmax(df[3], df[4]), df[5]);
    const T c = vmax(vmax(df[6], df[7]), df[8]), e = vmax(vmax(df[9], df[10]), df[11]);
    const T h = vmax(vmax(df[12], df[13]), df[14]);
    return vmax(vmax(vmax(a, b), c), vmax(vmax(e, h), df[15]));
}

// LDS/HBM wrappers: read own values from Vin, update, write V and/or pi.
template <typename T, bool SLIP, bool WRITE_V, bool WRITE_PI>
__device__ __forceinline__ T xyd_update(const XydTopo<T> &tp, const Coef<T> &cf, const T *Vin, T *Vout,
                                        int8_t *pis, int c) {
    const V4<T> own = *reinterpret_cast<const V4<T> *>(Vin + c * 4);
    T nbv[4];
    xyd_load_nb(tp, Vin, nbv);
    V4<T> out;
    uint32_t pk;
    const T dv = xyd_step<T, SLIP, WRITE_PI>(tp, cf, own, nbv, out, pk);
    if (WRITE_V) *reinterpret_cast<V4<T> *>(Vout + c * 4) = out;
    if (WRITE_PI) *reinterpret_cast<uint32_t *>(pis + c * 4) = pk;
    return dv;
}

template <typename T, bool WRITE_V, bool WRITE_PI>
__device__ __forceinline__ T dk_update(const DkTopo &tp, const Coef<T> &cf, const T *Vin, T *Vout,
                                       int8_t *pis, int c) {
    T own[16], outv[16];
    uint32_t pk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const V4<T> x = *reinterpret_cast<const V4<T> *>(Vin + c * 16 + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) own[4 * q + j] = x.v[j];
    }
    V4<T> nbs[4];
    dk_load_nb(tp, Vin, nbs);
    const T dv = dk_step<T, WRITE_PI>(tp, cf, own, nbs, outv, pk);
    if (WRITE_V) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<V4<T> *>(Vout + c * 16 + 4 * q) =
                V4<T>{{outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]}};
    }
    if (WRITE_PI) *reinterpret_cast<uint4 *>(pis + c * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    return dv;
}

}  // namespace mgdp
