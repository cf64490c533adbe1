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
// Kernels
//   vi_fused_kernel   one workgroup per grid: cells + both V buffers + pi live in LDS for the
//                     whole solve; many sweeps per launch, one __syncthreads per sweep.
//   vi_sweep_kernel   one Jacobi sweep of every grid: per grid, V'[grid] is staged HBM->LDS (the
//                     LDS tile of the neighbourhood; the next grid's tile is prefetched into
//                     registers while the current one is computed), updated from LDS, written back.
// Thread mappings (template MAP): MGDP_MAP_CELL = one thread per cell updating its 4 (XYD) or
// 16 (DoorKey) states from 16-B LDS vectors; MGDP_MAP_SA = one thread per (state, action),
// 8 lanes per state, wave shuffle max-reduce with the lowest action index winning ties.
#include <hip/hip_ext.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <climits>
#include <limits>
#include <cstring>
#include <vector>

#include "common.h"

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

// Block-wide max with ONE barrier; slots = [2][16] alternating by parity so that consecutive
// calls never race (a slot set is rewritten only after every thread passed the next barrier).
template <typename T>
__device__ __forceinline__ T block_max(T v, T *slots, int parity) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) slots[parity * 16 + w] = v;
    __syncthreads();
    const int nw = blockDim.x >> 6;
    T m = slots[parity * 16];
    for (int i = 1; i < nw; ++i) m = tmax(m, slots[parity * 16 + i]);
    return m;
}

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
};

template <typename T, bool ND = false>
__device__ __forceinline__ XydTopo<T> xyd_topo(const uint8_t *cl, const Geo &geo, int c) {
    XydTopo<T> tp;
    // NoDeath (wrappers.py:799-872): the agent may stand on lava; entering it is not terminal
    tp.valid = xyd_free(cl[c]) || (ND && cl[c] == T_LAVA);
    tp.term = 0;
    tp.lavaF = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int cfr = c + geo.off[d];
        const int tf = tp.valid ? cl[cfr] : T_WALL;  // valid cells are interior (closed border)
        tp.tq[d] = (T)0;
        tp.nbi[d] = c * 4 + d;
        if (tf == T_GOAL) { tp.term |= 1u << d; tp.tq[d] = (T)1; }
        else if (tf == T_LAVA) {
            if (ND) { tp.lavaF |= 1u << d; tp.nbi[d] = cfr * 4 + d; }
            else tp.term |= 1u << d;
        }
        else if (xyd_free(tf)) tp.nbi[d] = cfr * 4 + d;
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
        const int tf = inner ? cl[cfr] : T_WALL;
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

// ------------------------------------------------------------------------------------------------
// (state, action) lane mapping: 8 lanes per state, lane a evaluates action a, a wave shuffle
// max-reduce over the 8 lanes keeps the lowest index among exact maxima (numpy argmax rule).
// ------------------------------------------------------------------------------------------------
template <typename T, int MODEL, bool SLIP, bool WRITE_V>
__device__ __forceinline__ T sa_sweep(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                      const T *Vin, T *Vout, int8_t *pis) {
    const int a = threadIdx.x & 7;
    const int groups = blockDim.x >> 3;
    const int S = geo.S;
    const int bound = (S + groups - 1) / groups * groups;
    const int A = MODEL == MGDP_MODEL_XYD ? 7 : 5;
    const T NEG = -INFINITY;
    T dv = (T)0;
    for (int s = threadIdx.x >> 3; s < bound; s += groups) {
        const bool inr = s < S;
        const int ss = inr ? s : 0;
        bool valid;
        T q = NEG;
        if (MODEL == MGDP_MODEL_XYD) {
            const int c = ss >> 2, d = ss & 3;
            valid = inr && xyd_free(cl[c]);
            if (valid && a < A) {
                if (a == 0) q = cf.g * Vin[c * 4 + ((d + 3) & 3)];
                else if (a == 1) q = cf.g * Vin[c * 4 + ((d + 1) & 3)];
                else if (a == 2) {
                    const int cfr = c + geo.off[d];
                    const int tf = cl[cfr];
                    if (tf == T_GOAL) q = (T)1;
                    else if (tf == T_LAVA) q = (T)0;
                    else if (xyd_free(tf)) q = cf.g * Vin[cfr * 4 + d];
                    else q = cf.g * Vin[ss];
                } else q = cf.g * Vin[ss];
            }
            if (SLIP) {
                const int base = (threadIdx.x & 63) & ~7;
                const T q0 = __shfl(q, base + 0), q1 = __shfl(q, base + 1), q2 = __shfl(q, base + 2),
                        q3 = __shfl(q, base + 3), q4 = __shfl(q, base + 4), q5 = __shfl(q, base + 5);
                T s6 = q0 + q1;
                s6 = s6 + q2;
                s6 = s6 + q3;
                s6 = s6 + q4;
                s6 = s6 + q5;
                if (valid && a < A) q = cf.p * q + cf.c * s6;
            }
        } else {
            const int c = ss >> 4, l = ss & 15, d = l >> 2, hk = (l >> 1) & 1, dop = l & 1;
            valid = inr && dk_walk(cl[c], hk, dop);
            if (valid && a < A) {
                const T *vc = Vin + c * 16;
                if (a == 0) q = cf.g * vc[(((d + 3) & 3) * 2 + hk) * 2 + dop];
                else if (a == 1) q = cf.g * vc[(((d + 1) & 3) * 2 + hk) * 2 + dop];
                else {
                    const int cfr = c + geo.off[d];
                    const int tf = cl[cfr];
                    int tgt = l;  // self loop unless the action changes the state
                    if (a == 2) {
                        if (tf == T_GOAL) tgt = -2;
                        else if (tf == T_LAVA) tgt = -3;
                        else if (dk_walk(tf, hk, dop)) tgt = -1;
                    } else if (a == 3) {
                        if (tf == T_KEY && !hk) tgt = (d * 2 + 1) * 2 + dop;
                    } else {
                        if (tf == T_DOOR) {
                            if (dop) tgt = (d * 2 + hk) * 2 + 0;
                            else if (hk) tgt = (d * 2 + hk) * 2 + 1;
                        }
                    }
                    if (tgt == -2) q = (T)1;
                    else if (tgt == -3) q = (T)0;
                    else if (tgt == -1) q = cf.g * Vin[cfr * 16 + l];
                    else q = cf.g * vc[tgt];
                }
            }
        }
        int arg = a;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const T qo = __shfl_xor(q, o);
            const int ao = __shfl_xor(arg, o);
            if (qo > q || (qo == q && ao < arg)) { q = qo; arg = ao; }
        }
        if (a == 0 && inr) {
            const T old = Vin[ss];
            const T nv = valid ? q : (T)0;
            if (WRITE_V) Vout[ss] = nv;
            pis[ss] = valid ? (int8_t)arg : (int8_t)-1;
            dv = vmax(dv, vabs(nv - old));
        }
    }
    return dv;
}

// Generic LDS sweep over all cells of one grid (topology re-read from LDS each time).
template <typename T, int MODEL, bool SLIP, int MAP, bool WRITE_V, bool WRITE_PI>
__device__ __forceinline__ T sweep_lds(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                       const T *Vin, T *Vout, int8_t *pis) {
    if (MAP == MGDP_MAP_SA) return sa_sweep<T, MODEL, SLIP, WRITE_V>(geo, cf, cl, Vin, Vout, pis);
    T dv = (T)0;
    for (int c = threadIdx.x; c < geo.HW; c += blockDim.x) {
        if (MODEL == MGDP_MODEL_XYD)
            dv = vmax(dv, xyd_update<T, SLIP, WRITE_V, WRITE_PI>(xyd_topo<T>(cl, geo, c), cf, Vin, Vout, pis, c));
        else
            dv = vmax(dv, dk_update<T, WRITE_V, WRITE_PI>(dk_topo(cl, geo, c), cf, Vin, Vout, pis, c));
    }
    return dv;
}

// 16-byte cooperative copies between HBM and LDS (bytes is a multiple of 16).
__device__ __forceinline__ void copy16(void *dst, const void *src, int bytes) {
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) d[i] = s[i];
}
__device__ __forceinline__ void zero16(void *dst, int bytes) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) d[i] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void copy_pi(int8_t *dst, const int8_t *src, int S) {
    // S is a multiple of 4, so pi rows are 4-byte aligned
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    for (int i = threadIdx.x; i < (S >> 2); i += blockDim.x) d[i] = s[i];
}

struct Smem {
    int nbuf, v_bytes, pi_bytes, cells_bytes, slot_bytes;
    __host__ __device__ int total() const { return nbuf * v_bytes + pi_bytes + cells_bytes + slot_bytes; }
    __host__ __device__ int pi_off() const { return nbuf * v_bytes; }
    __host__ __device__ int cells_off() const { return nbuf * v_bytes + pi_bytes; }
    __host__ __device__ int slots_off() const { return nbuf * v_bytes + pi_bytes + cells_bytes; }
    __host__ __device__ int flags_off() const { return slots_off() + 256; }
};

__host__ __device__ inline Smem smem_layout(int S, int HWp, int tsize, int nbuf = 2) {
    Smem m;
    m.nbuf = nbuf;
    m.v_bytes = S * tsize;  // S is a multiple of 4 -> 16-B multiple for f32, f64
    m.pi_bytes = (S + 15) / 16 * 16;
    m.cells_bytes = HWp;
    m.slot_bytes = 256 + 64;  // block_max slots [2][16] x 8 B + convergence flags [2][2][16] B
    return m;
}

constexpr int kRedShards = 64;  // fused-launch reduction shards: [64][kmax, dV bits, kmin, -]
constexpr int kInKernelReduceMaxB = 512;  // above this, a separate one-workgroup reduce kernel

// Fold this block's (k, dV) into the launch reduction.  Every access to the shards and the ticket
// is an atomic read-modify-write (performed at the device coherence point, never served from a
// possibly stale per-XCD L2 line), so no cache fences are needed: each block's shard updates
// return before its ticket add is issued, hence the block that draws the last ticket observes all
// of them; it combines the shards with exchanges that also re-arm them for the next launch, and
// publishes {kmax, dV bits, kmin} to host-mapped memory.
__device__ __forceinline__ void publish(unsigned long long *host_out, unsigned long long km,
                                        unsigned long long dv, unsigned long long kn, unsigned int epoch) {
    // The host polls host_out[3]; the three values are acknowledged (vmcnt drained) before the
    // epoch word is stored, so the host sees them first.  No L2 write-back (release) is needed:
    // V and pi are consumed only by later stream-ordered operations.
    __hip_atomic_store(host_out + 0, km, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 1, dv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 2, kn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(host_out + 3, (unsigned long long)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Persistent-server result: three 8-byte words, each tagged with the request epoch in its high half
// ({k}, {dV bits 63..32}, {dV bits 31..0}), so they may land in any order and need no drain between
// them; the host waits until all three carry its epoch.
__device__ __forceinline__ void publish_tagged(unsigned long long *host_out, int k, double dv, unsigned int epoch) {
    const unsigned long long tag = (unsigned long long)epoch << 32;
    const unsigned long long b = (unsigned long long)__double_as_longlong(dv);
    __hip_atomic_store(host_out + 5, tag | (unsigned int)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 6, tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 7, tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void fused_reduce(unsigned long long *red, unsigned int *ticket,
                                             unsigned long long *host_out, int k, double dvl,
                                             unsigned int *lds_flag, unsigned int epoch, bool published) {
    if (gridDim.x == 1) {  // a lone grid publishes directly (early, if it swept: see `done`)
        if (threadIdx.x == 0 && !published)
            publish(host_out, (unsigned long long)k, (unsigned long long)__double_as_longlong(dvl),
                    (unsigned long long)k, epoch);
        return;
    }
    if (threadIdx.x == 0) {
        unsigned long long *r = red + (blockIdx.x & (kRedShards - 1)) * 4;
        const unsigned long long a = __hip_atomic_fetch_max(r + 0, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_fetch_max(r + 1, (unsigned long long)__double_as_longlong(dvl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c = __hip_atomic_fetch_min(r + 2, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" :: "v"(a), "v"(b), "v"(c) : "memory");
        const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = t == gridDim.x - 1;
    }
    __syncthreads();
    if (*lds_flag && threadIdx.x < 64) {
        unsigned long long *r = red + threadIdx.x * 4;
        unsigned long long km = __hip_atomic_exchange(r + 0, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long dv = __hip_atomic_exchange(r + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long kn = __hip_atomic_exchange(r + 2, 0x7fffffffull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            km = max(km, (unsigned long long)__shfl_xor(km, o));
            dv = max(dv, (unsigned long long)__shfl_xor(dv, o));
            kn = min(kn, (unsigned long long)__shfl_xor(kn, o));
        }
        if (threadIdx.x == 0) {
            __hip_atomic_exchange(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            publish(host_out, km, dv, kn, epoch);
        }
    }
}

// XYD fast path with the LDS V tiles in direction-major (SoA) order, V_d[c] at d*HW + c: the four
// front-cell reads of a wave are then four unit-stride ds_read_b32 (no bank conflicts; the cell-
// major order made every read a 4-way conflict), and the cell's own update is four unit-stride
// writes.  The HBM rows stay in the ABI's cell-major order: each thread loads / stores its own cell's
// 16 B (V4) directly, and writes its 4 pi lanes directly, so no LDS transposition pass is needed.
template <typename T, bool ND = false>
__device__ __forceinline__ XydTopo<T> xyd_topo_soa(const uint8_t *cl, const Geo &geo, int c) {
    XydTopo<T> tp = xyd_topo<T, ND>(cl, geo, c);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int cell = tp.nbi[d] >> 2;  // cell-major index (cell*4 + d) -> direction-major
        tp.nbi[d] = d * geo.HWs + cell;
    }
    return tp;
}

// Options: ND = NoDeath lava; HMODE 1 = finite horizon (k_target = H sweeps,
// sweep k+1 computes V_{H-k-1} with goal reward rgoal[H-k-1]), 2 = the same keeping pi_t (per-action
// form every sweep, 4 lanes per cell stored to pit + t*pit_stride).
template <typename T, bool SLIP, bool LOCAL, bool ND = false, int HMODE = 0, typename Done>
__device__ __forceinline__ void fused_fast_xyd_soa(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                                   T *V0, T *V1, T *slots, uint8_t *flags,
                                                   const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                   int k_target, double &dvl, const Done &done,
                                                   const T *rgoal = nullptr, int8_t *pit = nullptr,
                                                   long long pit_stride = 0) {
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;  // idle threads shadow cell 0 and never write
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs;  // LDS stride: every thread (idle ones too) owns a slot, so LDS writes need no mask
    const int k_start = k;
    const XydTopo<T> tp = xyd_topo_soa<T, ND>(cl, geo, cc);
    V4<T> own;
    if (k == 0) {
        own = V4<T>{{(T)0, (T)0, (T)0, (T)0}};
    } else {
        own = *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) V0[d * HW + c] = own.v[d];
    __syncthreads();
    int cur = 0, parity = 0;
    T diff = (T)0;
    // One sweep from Vin to Vout; false = the rule stopped before it.  The ping-pong is unrolled
    // by two below, so each copy has fixed LDS addresses and a fixed flag parity.  Idle threads
    // shadow cell 0, so their |dV| equals cell 0's and needs no masking.
    auto sweep = [&](const T *Vin, T *Vout, const V4<T> &in, V4<T> &out) -> bool {
        T nbv[4];
        xyd_load_nb(tp, Vin, nbv);
        if (LOCAL) {
            if (k >= geo.max_sweeps) return false;
            if (k > k_start && !flags_any(flags, parity ^ 1)) return false;
        } else if (k >= k_target) {
            return false;
        }
        uint32_t pk;
        const T rg = HMODE ? rgoal[k_target - 1 - k] : (T)1;
        if (HMODE == 2) {
            diff = xyd_step<T, SLIP, true, ND, true>(tp, cf, in, nbv, out, pk, rg);
            if (own_cell) *reinterpret_cast<uint32_t *>(pit + (long long)(k_target - 1 - k) * pit_stride + c * 4) = pk;
        } else {
            diff = xyd_step<T, SLIP, false, ND, HMODE != 0>(tp, cf, in, nbv, out, pk, rg);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) Vout[q * HW + c] = out.v[q];
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    V4<T> alt;  // the two register sets alternate with the LDS buffers: no copies between sweeps
    while (true) {
        if (!sweep(V0, V1, own, alt)) { cur = 0; break; }
        if (!sweep(V1, V0, alt, own)) { cur = 1; own = alt; break; }
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    if (own_cell) {
        // pi of the last sweep = argmax on V_{k-1} (buffer cur ^ 1, intact); V_k is `own`
        const T *Vp = cur ? V0 : V1;
        V4<T> op;
        T nbv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) op.v[q] = Vp[q * HW + c];
        xyd_load_nb(tp, Vp, nbv);
        V4<T> tmp;
        uint32_t pk;
        xyd_step<T, SLIP, true, ND, HMODE != 0>(tp, cf, op, nbv, tmp, pk, HMODE ? rgoal[k_target - k] : (T)1);
        *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
        *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = own;
    }
}

// DoorKey fast path with the LDS tiles direction-major: the 4 (has_key, door_open) values of
// state group (c, d) are the V4 at (d*HW + c)*4, so a wave's front-cell reads and own writes are
// unit-stride 16-B accesses.  HBM rows stay cell-major (c*16 + d*4 + hk*2 + door_open).
__device__ __forceinline__ DkTopo dk_topo_soa(const uint8_t *cl, const Geo &geo, int c) {
    DkTopo tp = dk_topo(cl, geo, c);
#pragma unroll
    for (int d = 0; d < 4; ++d) tp.nb[d] = (d * geo.HWs + (tp.nb[d] >> 4)) * 4;
    return tp;
}

template <typename T, bool LOCAL, int HMODE = 0, typename Done>  // HMODE: see fused_fast_xyd_soa
__device__ __forceinline__ void fused_fast_dk_soa(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                                  T *V0, T *V1, T *slots, uint8_t *flags,
                                                  const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                  int k_target, double &dvl, const Done &done,
                                                  const T *rgoal = nullptr, int8_t *pit = nullptr,
                                                  long long pit_stride = 0) {
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs;  // LDS stride: every thread (idle ones too) owns a slot, so LDS writes need no mask
    const int k_start = k;
    const DkTopo tp = dk_topo_soa(cl, geo, cc);
    T own[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 16 + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) own[4 * q + j] = x.v[j];
        *reinterpret_cast<V4<T> *>(V0 + (q * HW + c) * 4) = x;
    }
    __syncthreads();
    int cur = 0, parity = 0;
    T diff = (T)0;
    auto sweep = [&](const T *Vin, T *Vout, const T (&in)[16], T (&outv)[16]) -> bool {  // see fused_fast_xyd_soa
        V4<T> nbs[4];
        dk_load_nb(tp, Vin, nbs);
        if (LOCAL) {
            if (k >= geo.max_sweeps) return false;
            if (k > k_start && !flags_any(flags, parity ^ 1)) return false;
        } else if (k >= k_target) {
            return false;
        }
        uint32_t pk[4];
        const T rg = HMODE ? rgoal[k_target - 1 - k] : (T)1;
        if (HMODE == 2) {
            diff = dk_step<T, true, true>(tp, cf, in, nbs, outv, pk, rg);
            if (own_cell)
                *reinterpret_cast<uint4 *>(pit + (long long)(k_target - 1 - k) * pit_stride + c * 16) =
                    make_uint4(pk[0], pk[1], pk[2], pk[3]);
        } else {
            diff = dk_step<T, false, HMODE != 0>(tp, cf, in, nbs, outv, pk, rg);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<V4<T> *>(Vout + (q * HW + c) * 4) =
                V4<T>{{outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]}};
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    T alt[16];
    while (true) {
        if (!sweep(V0, V1, own, alt)) { cur = 0; break; }
        if (!sweep(V1, V0, alt, own)) {
            cur = 1;
#pragma unroll
            for (int l = 0; l < 16; ++l) own[l] = alt[l];
            break;
        }
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    if (own_cell) {  // pi on V_{k-1} (buffer cur ^ 1); V_k is `own`
        const T *Vp = cur ? V0 : V1;
        T op[16], tmp[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const V4<T> x = *reinterpret_cast<const V4<T> *>(Vp + (q * HW + c) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) op[4 * q + j] = x.v[j];
        }
        V4<T> nbs[4];
        dk_load_nb(tp, Vp, nbs);
        uint32_t pk[4];
        dk_step<T, true, HMODE != 0>(tp, cf, op, nbs, tmp, pk, HMODE ? rgoal[k_target - k] : (T)1);
        *reinterpret_cast<uint4 *>(pig + c * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<V4<T> *>(Vg_out + c * 16 + 4 * q) = V4<T>{{own[4 * q], own[4 * q + 1], own[4 * q + 2], own[4 * q + 3]}};
    }
}

// Two-sweep step for the XYD fast path (geo.pair, three LDS buffers).  V_{k+2}[c, d] needs V_{k+1} only at
// the cell itself and at state (front(c, d), d); the thread recomputes that neighbour state with
// exactly the neighbour's own operations (bit-identical), so two Jacobi sweeps cost one barrier.
// Buffers rotate: input X = V_k, outputs Y = V_{k+1}, Z = V_{k+2}; the convergence flags of both
// sweeps are tested after the barrier, so the stopping sweep (and V_{K-1} for pi) is exact.
template <typename T>
struct Xyd2Topo {
    XydTopo<T> b;
    uint32_t nfree;   // bit d: the front cell n_d = c + off[d] is free (forward moves there)
    uint32_t n2term;  // bit d: forward from state (n_d, d) is terminal
    int nbase[4];     // V index of n_d's 4-state block (own block when not free)
    int n2i[4];       // V index read by forward from (n_d, d)
    T n2tq[4];
};

template <typename T>
__device__ __forceinline__ Xyd2Topo<T> xyd2_topo(const uint8_t *cl, const Geo &geo, int c) {
    Xyd2Topo<T> t;
    t.b = xyd_topo<T>(cl, geo, c);
    t.nfree = 0;
    t.n2term = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int n = c + geo.off[d];
        const bool nf = t.b.valid && xyd_free(cl[n]);
        t.nbase[d] = (nf ? n : c) * 4;
        t.n2i[d] = c * 4 + d;
        t.n2tq[d] = (T)0;
        if (nf) {
            t.nfree |= 1u << d;
            const int n2 = n + geo.off[d];  // n is free, hence interior
            const int tf = cl[n2];
            t.n2i[d] = n * 4 + d;
            if (tf == T_GOAL) { t.n2term |= 1u << d; t.n2tq[d] = (T)1; }
            else if (tf == T_LAVA) { t.n2term |= 1u << d; }
            else if (xyd_free(tf)) t.n2i[d] = n2 * 4 + d;
        }
    }
    return t;
}

// Value of one XYD state from its four distinct action values (the WRITE_PI = false branch of
// xyd_step, operation for operation).
template <typename T, bool SLIP>
__device__ __forceinline__ T xyd_value(const Coef<T> &cf, T qL, T qR, T qF, T qS) {
    T a0 = qL, a1 = qR, a2 = qF, a3 = qS;
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
    return vmax(vmax(a0, a1), vmax(a2, a3));
}

template <typename T, bool SLIP, bool LOCAL, typename Done>
__device__ __forceinline__ void fused_fast_xyd2(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                                T *vbase, int8_t *pis, T *slots, uint8_t *flags,
                                                int &k, int k_target, int &vfinal, double &dvl,
                                                const Done &done) {
    // buffer i = vbase + i*S: offsets from the LDS base keep every access a ds_* instruction (a
    // pointer picked from an array of buffers would degrade to flat loads/stores)
    auto buf = [&](int i) -> T * { return vbase + i * geo.S; };
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const Xyd2Topo<T> tp = xyd2_topo<T>(cl, geo, cc);
    const int limit = LOCAL ? geo.max_sweeps : k_target;
    V4<T> own = *reinterpret_cast<const V4<T> *>(buf(0) + cc * 4);
    int bx = 0, by = 1, bz = 2, last_n = 0, par = 0;
    T dA = (T)0, dB = (T)0, dfin = (T)0;
    int bfin = 0, bprev = 0, kfin = k;
    while (true) {
        // speculative loads from the buffer the next step would read
        const T *X = buf(last_n == 2 ? bz : (last_n == 1 ? by : bx));
        V4<T> nb4[4];
        T n2v[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            nb4[d] = *reinterpret_cast<const V4<T> *>(X + tp.nbase[d]);
            n2v[d] = X[tp.n2i[d]];
        }
        if (last_n > 0) {
            bool stop = false;
            if (LOCAL && !flags_any(flags + (par ^ 1) * 32, 0)) {  // first sweep of the last step converged
                stop = true; kfin = k - last_n + 1; bfin = by; bprev = bx; dfin = dA;
            } else if (LOCAL && last_n == 2 && !flags_any(flags + (par ^ 1) * 32 + 16, 0)) {
                stop = true; kfin = k; bfin = bz; bprev = by; dfin = dB;
            } else if (k >= limit) {
                stop = true; kfin = k;
                bfin = last_n == 2 ? bz : by;
                bprev = last_n == 2 ? by : bx;
                dfin = last_n == 2 ? dB : dA;
            }
            if (stop) break;
            if (last_n == 2) { const int t = bx; bx = bz; bz = by; by = t; }
            else { const int t = bx; bx = by; by = bz; bz = t; }
        }
        const int n = k + 2 <= limit ? 2 : 1;
        T nbv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) nbv[d] = ((tp.nfree >> d) & 1u) ? nb4[d].v[d] : own.v[d];
        V4<T> out1;
        uint32_t pk;
        dA = xyd_step<T, SLIP, false>(tp.b, cf, own, nbv, out1, pk);
        if (own_cell) *reinterpret_cast<V4<T> *>(buf(by) + cc * 4) = out1;
        else dA = (T)0;
        if (n == 2) {
            T nbv2[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const V4<T> &nv = nb4[d];
                const T qL = cf.g * nv.v[(d + 3) & 3], qR = cf.g * nv.v[(d + 1) & 3], qS = cf.g * nv.v[d];
                const T qF = ((tp.n2term >> d) & 1u) ? tp.n2tq[d] : cf.g * n2v[d];
                const T vn = xyd_value<T, SLIP>(cf, qL, qR, qF, qS);  // V_{k+1}[n_d, d]
                nbv2[d] = ((tp.nfree >> d) & 1u) ? vn : out1.v[d];
            }
            V4<T> out2;
            dB = xyd_step<T, SLIP, false>(tp.b, cf, out1, nbv2, out2, pk);
            if (own_cell) *reinterpret_cast<V4<T> *>(buf(bz) + cc * 4) = out2;
            else dB = (T)0;
            own = out2;
        } else {
            own = out1;
            dB = (T)0;
        }
        if (LOCAL) {
            flag_write(dA >= cf.tol, flags + par * 32, 0);
            if (n == 2) flag_write(dB >= cf.tol, flags + par * 32 + 16, 0);
        }
        __syncthreads();
        par ^= 1;
        k += n;
        last_n = n;
    }
    k = kfin;
    vfinal = bfin;
    dvl = (double)block_max(dfin, slots, 0);
    done(k, dvl);
    if (own_cell) xyd_update<T, SLIP, false, true>(tp.b, cf, buf(bprev), nullptr, pis, cc);  // pi on V_{K-1}
    __syncthreads();
}

// DPP quad permutation (lane i of each group of 4 reads lane CTRL[i]); all lanes must be active.
template <int CTRL>
__device__ __forceinline__ float quad_perm(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double quad_perm(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kQuadLeft = 0x93;   // lane d reads lane (d+3)&3: the state after turning left
constexpr int kQuadRight = 0x39;  // lane d reads lane (d+1)&3: the state after turning right

// XYD fused fast path with 4 threads per cell, one per direction (geo.quad): each lane holds its
// state's V in a register, gets the left/right-turn values from its quad by DPP (no LDS), reads
// only the forward value from LDS and writes one word.  Shorter dependency chain per sweep than
// one thread per cell; needs 4*HW <= blockDim.
template <typename T, bool SLIP, bool LOCAL, typename Done>
__device__ __forceinline__ void fused_quad_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *V0,
                                               T *V1, int8_t *pis, T *slots, uint8_t *flags, int &k,
                                               int k_target, int &cur, double &dvl, const Done &done) {
    const int c = threadIdx.x >> 2, d = threadIdx.x & 3;
    const bool own_cell = c < geo.HW;
    const int cc = own_cell ? c : 0;
    const int s = cc * 4 + d;
    const bool valid = own_cell && xyd_free(cl[cc]);
    bool term = false;
    T tq = (T)0;
    int nbi = s;
    if (valid) {
        const int cfr = cc + geo.off[d];
        const int tf = cl[cfr];
        if (tf == T_GOAL) { term = true; tq = (T)1; }
        else if (tf == T_LAVA) { term = true; }
        else if (xyd_free(tf)) nbi = cfr * 4 + d;
    }
    const int k_start = k;
    int parity = 0;
    T v = (cur ? V1 : V0)[s];
    T vprev = v;
    T diff = (T)0;
    while (true) {
        const T *Vin = cur ? V1 : V0;
        T *Vout = cur ? V0 : V1;
        const T nb = Vin[nbi];
        const T vl = quad_perm<kQuadLeft>(v), vr = quad_perm<kQuadRight>(v);
        const bool stop = LOCAL ? (k >= geo.max_sweeps || (k > k_start && !flags_any(flags, parity ^ 1)))
                                : k >= k_target;
        if (stop) break;
        const T qF = term ? tq : cf.g * nb;
        T best = xyd_value<T, SLIP>(cf, cf.g * vl, cf.g * vr, qF, cf.g * v);
        best = valid ? best : (T)0;
        diff = vabs(best - v);
        if (own_cell) Vout[s] = best;
        vprev = v;
        v = best;
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        cur ^= 1;
        ++k;
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    {   // pi of the last sweep: argmax on V_{k-1} (vprev in registers, forward from buffer cur ^ 1)
        const T *Vp = cur ? V0 : V1;
        const T nb = Vp[nbi];
        const T vl = quad_perm<kQuadLeft>(vprev), vr = quad_perm<kQuadRight>(vprev);
        const T qL = cf.g * vl, qR = cf.g * vr, qS = cf.g * vprev, qF = term ? tq : cf.g * nb;
        T a0 = qL, a1 = qR, a2 = qF, a3 = qS;
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
        int arg = 0;
        T best = a0;
        if (a1 > best) { best = a1; arg = 1; }
        if (a2 > best) { best = a2; arg = 2; }
        if (a3 > best) { best = a3; arg = 3; }
        if (own_cell) pis[s] = valid ? (int8_t)arg : (int8_t)-1;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Fused solve: blockIdx.x = grid index; the grid's cells, both V buffers and pi stay in LDS for
// every sweep of the launch.  k_target < 0: sweep until this grid's own max|dV| < tol (or
// max_sweeps); k_target >= 0: sweep until exactly k_target sweeps are done.  fresh: start from
// V_0 = 0 regardless of kenv/dvenv.  MAP_CELL with HW <= blockDim keeps each thread's cell
// topology in registers for the whole launch (no LDS cell reads inside the sweep loop).
// Sweeps are value-only (max, no argmax); the per-sweep convergence test is a block OR of
// (|dV| >= tol) (ballot + one byte per wave, one barrier); after the loop the exact max |dV| is
// reduced once and pi is extracted once from V_{k-1} (exactly what sweep k's argmax would give).
// ------------------------------------------------------------------------------------------------
// The whole fused solve of grid e by one workgroup: stage cells (and V unless fresh) in LDS, sweep
// to the local stopping rule (k_target < 0) or to k_target, extract pi, write V / pi / (k, dV) back.
// `lone`: this workgroup is the only one of the solve and publishes {k, dV} to the host as soon as
// they are known (pi extraction and the write-back then overlap the host's reaction); `served`:
// it does so in the persistent server's tagged form, and the cells are already staged in LDS.
template <typename T, int MODEL, bool SLIP, int MAP, bool SERVED = false>
__device__ __forceinline__ bool fused_grid(const Geo &geo, const Coef<T> &cf, const uint8_t *__restrict__ cells,
                                           T *__restrict__ V, int8_t *__restrict__ pi, int32_t *__restrict__ kenv,
                                           double *__restrict__ dvenv, unsigned long long *__restrict__ host_out,
                                           int k_target, int fresh, bool lone, unsigned int epoch, int e,
                                           int &k, double &dvl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    T *V0 = reinterpret_cast<T *>(smem);
    T *V1 = reinterpret_cast<T *>(smem + L.v_bytes);
    int8_t *pis = reinterpret_cast<int8_t *>(smem + L.pi_off());
    uint8_t *cl = reinterpret_cast<uint8_t *>(smem + L.cells_off());
    T *slots = reinterpret_cast<T *>(smem + L.slots_off());
    uint8_t *flags = reinterpret_cast<uint8_t *>(smem + L.flags_off());

    k = fresh ? 0 : kenv[e];
    dvl = fresh ? 0.0 : dvenv[e];
    const bool work = k_target < 0 ? (!(k > 0 && dvl < geo.tol) && k < geo.max_sweeps) : (k < k_target);
    if (!work) return false;
    const long long vb = (long long)e * geo.S;
    const bool fast = MAP == MGDP_MAP_CELL && geo.HW <= (int)blockDim.x;
    const bool soa = fast && !geo.pair && !geo.quad;
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
            if (threadIdx.x == 0) publish_tagged(host_out, kk, dv, epoch);
        } else if (lone && threadIdx.x == 0) {
            publish(host_out, (unsigned long long)kk, (unsigned long long)__double_as_longlong(dv),
                    (unsigned long long)kk, epoch);
        }
    };
    const T *Vfinal = nullptr;
    if (soa) {
        if (MODEL == MGDP_MODEL_XYD) {
            if (k_target < 0) fused_fast_xyd_soa<T, SLIP, true>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_fast_xyd_soa<T, SLIP, false>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        } else {
            if (k_target < 0) fused_fast_dk_soa<T, true>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
            else fused_fast_dk_soa<T, false>(geo, cf, cl, V0, V1, slots, flags, V + vb, V + vb, pi + vb, k, k_target, dvl, done);
        }
        if (threadIdx.x == 0) {
            kenv[e] = k;
            dvenv[e] = dvl;
        }
        return true;  // V and pi were written by their owner threads
    } else if (fast && MODEL == MGDP_MODEL_XYD && geo.pair) {
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
        dvenv[e] = dvl;
    }
    return true;
}

template <typename T, int MODEL, bool SLIP, int MAP>
__global__ void __launch_bounds__(1024)
vi_fused_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, T *__restrict__ V,
                int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                unsigned long long *__restrict__ red, unsigned int *__restrict__ ticket,
                unsigned long long *__restrict__ host_out, int k_target, int fresh, int in_kernel_reduce,
                unsigned int epoch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    T *slots = reinterpret_cast<T *>(smem + L.slots_off());
    int k;
    double dvl;
    const bool lone = in_kernel_reduce && gridDim.x == 1;
    const bool work = fused_grid<T, MODEL, SLIP, MAP>(geo, cf, cells, V, pi, kenv, dvenv, host_out, k_target, fresh,
                                                      lone, epoch, blockIdx.x, k, dvl);
    if (in_kernel_reduce) fused_reduce(red, ticket, host_out, k, dvl, reinterpret_cast<unsigned int *>(slots + 16), epoch, work);
}

// Persistent solver for a lone grid: one workgroup stays resident and serves solve requests posted
// in host-mapped memory, removing the launch and dispatch latency from every solve.  The cells
// cannot change while it is resident (every other entry point stops it first), so they are staged
// in LDS once.  Lane 0 of every wave polls the request word (relaxed system-scope loads, the waves
// staggered by s_sleep so a new request is seen a fraction of a round trip after it lands) and
// also watches the LDS word another wave may already have set.  Request r (!= the last served)
// runs a fresh fused solve whose {k, dV} is published tagged with r.  Every wave leaves on the quit
// word, after `idle_ticks` without a request or after `life_ticks` in total (s_memrealtime,
// 100 MHz); the host relaunches the server if a request finds it gone.
constexpr unsigned long long kServeQuit = ~0ull;

template <typename T, int MODEL, bool SLIP, int MAP>
__global__ void __launch_bounds__(1024)
vi_serve_kernel(Geo geo, Coef<T> cf, const uint8_t *__restrict__ cells, T *__restrict__ V,
                int8_t *__restrict__ pi, int32_t *__restrict__ kenv, double *__restrict__ dvenv,
                unsigned long long *__restrict__ host_out, const unsigned long long *__restrict__ host_cmd,
                unsigned long long served, unsigned long long idle_ticks, unsigned long long life_ticks) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ unsigned long long s_cmd;
    const Smem L = smem_layout(geo.Ss, geo.HWp, (int)sizeof(T), geo.nbuf);
    copy16(smem + L.cells_off(), cells, geo.HWp);
    if (threadIdx.x == 0) s_cmd = served;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_last = t_start;
    __syncthreads();
    while (true) {
        if (lane == 0) {
            for (int i = 0; i < wave; ++i) __builtin_amdgcn_s_sleep(8);  // stagger the pollers
            while (true) {
                const unsigned long long cmd = __hip_atomic_load(host_cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (cmd != served) {
                    __hip_atomic_store(&s_cmd, cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (__hip_atomic_load(&s_cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != served) break;
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                if (now - t_last > idle_ticks || now - t_start > life_ticks) {
                    __hip_atomic_store(&s_cmd, kServeQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        const unsigned long long cmd = s_cmd;
        if (cmd == kServeQuit) break;
        int k;
        double dvl;
        if (!fused_grid<T, MODEL, SLIP, MAP, true>(geo, cf, cells, V, pi, kenv, dvenv, host_out, -1, 1, true,
                                                   (unsigned int)cmd, 0, k, dvl) &&
            threadIdx.x == 0)
            publish_tagged(host_out, k, dvl, (unsigned int)cmd);
        served = cmd;
        t_last = __builtin_amdgcn_s_memrealtime();
        __syncthreads();  // every wave is past s_cmd and the LDS tiles before the next request
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
            dvenv[e] = dvl;
        }
    }
    if (in_kernel_reduce) fused_reduce(red, ticket, host_out, k, dvl, reinterpret_cast<unsigned int *>(slots + 16), epoch, work);
}

// Large batches: one workgroup reduces the per-grid (kenv, dvenv) into host-mapped memory (a
// single arrival ticket shared by tens of thousands of workgroups would serialise on one address).
__global__ void __launch_bounds__(1024)
vi_reduce_kernel(const int32_t *__restrict__ kenv, const double *__restrict__ dvenv, int B,
                 unsigned long long *__restrict__ host_out, unsigned int epoch) {
    __shared__ unsigned long long sk[16], sd[16], sn[16];
    unsigned long long km = 0, dm = 0, kn = 0x7fffffffull;
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
        const unsigned long long k = (unsigned long long)kenv[i];
        km = max(km, k);
        kn = min(kn, k);
        dm = max(dm, (unsigned long long)__double_as_longlong(dvenv[i]));
    }
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
        copy16(Vi, Vin + vb, me * vbytes);
        __syncthreads();
        for (int j = 0; j < me; ++j)
            acc = vmax(acc, sweep_lds<T, MODEL, SLIP, MAP, !POLICY, POLICY || MAP == MGDP_MAP_SA>(
                                geo, cf, cl + j * geo.HWp, Vi + j * geo.S, Vo + j * geo.S, pis + j * pib));
        __syncthreads();
        if (!POLICY) {
            copy16(Vout + vb, Vo, me * vbytes);
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

}  // namespace mgdp

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
    double *d_dvenv = nullptr;
    unsigned long long *d_shards = nullptr;
    unsigned long long *d_red = nullptr;    // fused reduction shards [64][4]
    unsigned int *d_ticket = nullptr;       // arrival ticket of the fused reduction
    unsigned long long *h_out = nullptr;    // host-mapped {kmax, dV bits, kmin, epoch, request}
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
    unsigned int epoch = 0; // tag of the last fused launch; its result lands in h_out[3]
    int nbuf = 2;                 // fused LDS V buffers (3 = two-sweep XYD step)
    int quad = 0;                 // fused XYD: 4 threads per cell
    int pair = 0;                 // fused XYD: two-sweep step
    int sweep_block = 256;
    int sweep_m = 1;              // grids staged per workgroup iteration (measured: m>1 no faster)
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
    std::chrono::steady_clock::time_point serve_last{};  // host time of the last served result
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
                          vi->d.B <= kInKernelReduceMaxB ? 1 : 0, ++vi->epoch, (const T *)vi->d_rgoal, vi->d_pi_t);
    MGDP_HIP(hipGetLastError());
    vi->fresh = 0;
    if (vi->d.B > kInKernelReduceMaxB) {
        hipLaunchKernelGGL(vi_reduce_kernel, dim3(1), dim3(1024), 0, vi->stream, vi->d_kenv, vi->d_dvenv, vi->d.B,
                           vi->d_hout, vi->epoch);
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

template <typename T, int MODEL, bool SLIP, int MAP>
int launch_fused_t(mgdp_vi *vi, int k_target) {
    if (vi->opts) return launch_opts<T>(vi, k_target);
    const Geo g = make_geo(vi);
    const Smem L = smem_layout(vi->Ss, vi->HWp, sizeof(T), vi->nbuf);
    auto kern = vi_fused_kernel<T, MODEL, SLIP, MAP>;
    if (L.total() > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, L.total()));
    TimedPair tp;
    if (int rc = timed_begin(vi, -1, &tp)) return rc;
    hipExtLaunchKernelGGL(kern, dim3(vi->d.B), dim3(vi->fused_block), L.total(), vi->stream, tp.a, tp.b, 0, g,
                       make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv,
                       vi->d_dvenv, vi->d_red, vi->d_ticket, vi->d_hout, k_target, vi->fresh,
                       vi->d.B <= kInKernelReduceMaxB ? 1 : 0, ++vi->epoch);
    MGDP_HIP(hipGetLastError());
    vi->fresh = 0;
    if (vi->d.B > kInKernelReduceMaxB) {
        hipLaunchKernelGGL(vi_reduce_kernel, dim3(1), dim3(1024), 0, vi->stream, vi->d_kenv, vi->d_dvenv, vi->d.B,
                           vi->d_hout, vi->epoch);
        MGDP_HIP(hipGetLastError());
    }
    return 0;
}

template <typename T, int MODEL, bool SLIP, int MAP>
int launch_serve_t(mgdp_vi *vi, unsigned int served) {
    const Geo g = make_geo(vi);
    const Smem L = smem_layout(vi->Ss, vi->HWp, sizeof(T), vi->nbuf);
    auto kern = vi_serve_kernel<T, MODEL, SLIP, MAP>;
    if (L.total() > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, L.total()));
    TimedPair tp;
    if (int rc = timed_begin(vi, -1, &tp)) return rc;
    hipExtLaunchKernelGGL(kern, dim3(1), dim3(vi->fused_block), L.total(), vi->stream, tp.a, tp.b, 0, g,
                          make_coef<T>(vi), vi->d_cells, (T *)vi->d_V[0], vi->d_pi, vi->d_kenv, vi->d_dvenv,
                          vi->d_hout, vi->d_hout + 4, (unsigned long long)served, vi->serve_idle_ticks,
                          vi->serve_life_ticks);
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

template <typename T, int MODEL, bool SLIP, int MAP>
int launch_sweep_t(mgdp_vi *vi, int k, int check_prev, bool policy) {
    const T *Vin = (const T *)vi->d_V[(k - 1) & 1];
    T *Vout = (T *)vi->d_V[k & 1];
    if (policy) return launch_sweep_kernel<T, MODEL, SLIP, MAP, true>(vi, Vin, Vout, k, 0);
    TimedPair tp;
    if (int rc = timed_begin(vi, k, &tp)) return rc;
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
    static int run(mgdp_vi *vi, int k_target) { return launch_fused_t<T, MODEL, SLIP, MAP>(vi, k_target); }
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
    // The last workgroup (or the reduce kernel) publishes {kmax, dV, kmin, epoch} to host-mapped
    // memory; the persistent server publishes three epoch-tagged words instead.  Poll them rather
    // than synchronise the stream (lower completion latency); everything else stays stream-ordered.
    // Poll the stream now and then to surface faults -- and, in serving mode, to relaunch a server
    // that left before it saw the request.
    const volatile unsigned long long *h = vi->h_out;
    const unsigned long long ep = (unsigned long long)vi->epoch;
    const bool tagged = vi->serving;
    auto ready = [&]() -> bool {
        if (!tagged) return h[3] == ep;
        return (h[5] >> 32) == ep && (h[6] >> 32) == ep && (h[7] >> 32) == ep;
    };
    int relaunches = 0;
    for (uint64_t spin = 0; !ready(); ++spin) {
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(vi->stream);
            if (q == hipSuccess) {
                if (ready()) break;
                if (tagged && relaunches < 4) {
                    ++relaunches;
                    if (int rc = dispatch<ServeF>(vi, vi->epoch - 1u)) return rc;
                    continue;
                }
                MGDP_CHECK(false, MGDP_E_HIP, "fused launch finished without publishing its result (epoch %u)", vi->epoch);
            }
            if (q != hipErrorNotReady) return hip_fail(q, "fused value-iteration launch", __FILE__, __LINE__);
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    unsigned long long km, dvb, kmin;
    if (tagged) {
        km = kmin = h[5] & 0xffffffffull;
        dvb = ((h[6] & 0xffffffffull) << 32) | (h[7] & 0xffffffffull);
    } else {
        km = h[0];
        dvb = h[1];
        kmin = h[2];
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
           vi->HW <= vi->fused_block && !vi->pair && !vi->quad;
}
// Ask a resident server to leave and drain the stream.  Every entry point that enqueues other
// work on the stream, or reads results, calls this first.
int server_stop(mgdp_vi *vi) {
    if (!vi->serving) return 0;
    __atomic_store_n(vi->h_out + 4, kServeQuit, __ATOMIC_RELEASE);
    vi->serving = false;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    return 0;
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
    ++vi->epoch;
    __atomic_store_n(vi->h_out + 4, (unsigned long long)vi->epoch, __ATOMIC_RELEASE);
    if (!vi->serving) {
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
    al((void **)&vi->d_dvenv, sizeof(double) * d.B);
    al((void **)&vi->d_shards, sizeof(unsigned long long) * 8 * (size_t)(d.max_sweeps + 1));
    al((void **)&vi->d_red, sizeof(unsigned long long) * (kRedShards * 4 + 2));
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
    if (e == hipSuccess) e = hipHostMalloc((void **)&vi->h_out, 8 * sizeof(unsigned long long),
                                           hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&vi->d_hout, vi->h_out, 0);
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
    if (const char *ev = std::getenv("MGDP_SERVE_IDLE_US"))  // s_memrealtime ticks at 100 MHz
        vi->serve_idle_ticks = (unsigned long long)std::max(1LL, std::atoll(ev)) * 100ull;
    if (const char *ev = std::getenv("MGDP_SERVE_LIFE_US"))
        vi->serve_life_ticks = (unsigned long long)std::max(1LL, std::atoll(ev)) * 100ull;
    if (vi->h_out) std::memset(vi->h_out, 0, 8 * sizeof(unsigned long long));
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
    (void)hipFree(vi->d_dvenv);
    (void)hipFree(vi->d_shards);
    (void)hipFree(vi->d_red);
    (void)hipFree(vi->d_rgoal);
    (void)hipFree(vi->d_pi_t);
    if (vi->h_out) (void)hipHostFree(vi->h_out);
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

int mgdp_vi_load_cells(mgdp_vi *vi, const uint8_t *cells) {
    MGDP_CHECK(vi && cells, MGDP_E_INVALID, "null argument");
    if (int rc = validate_cells(vi->d, cells)) return rc;
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    std::vector<uint8_t> pad((size_t)vi->d.B * vi->HWp, 0);
    for (int b = 0; b < vi->d.B; ++b) std::memcpy(&pad[(size_t)b * vi->HWp], cells + (size_t)b * vi->HW, vi->HW);
    MGDP_HIP(hipMemcpyAsync(vi->d_cells, pad.data(), pad.size(), hipMemcpyHostToDevice, vi->stream));
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    vi->cells_loaded = true;
    vi->k_done_valid = false;
    return 0;
}

int mgdp_vi_load_cells_device(mgdp_vi *vi, const uint8_t *d_cells) {
    MGDP_CHECK(vi && d_cells, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipMemcpy2DAsync(vi->d_cells, vi->HWp, d_cells, vi->HW, vi->HW, vi->d.B, hipMemcpyDeviceToDevice, vi->stream));
    vi->cells_loaded = true;
    vi->k_done_valid = false;
    return 0;
}

int mgdp_vi_reset(mgdp_vi *vi) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
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
        const bool serve = serve_eligible(vi) && vi->fresh;
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
    if (int rc = sweep_run(vi, vi->d.max_sweeps, false, nullptr)) return rc;
    *k_local_max = vi->k_done;
    return 0;
}

int mgdp_vi_run_to(mgdp_vi *vi, int32_t k_target, double *dv_out) {
    MGDP_CHECK(vi && dv_out, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(k_target >= 0 && k_target <= vi->d.max_sweeps, MGDP_E_INVALID, "k_target %d out of range", k_target);
    DeviceGuard guard(vi->d.device);
    if (vi->d.method == MGDP_METHOD_FUSED) {
        if (vi->k_min == k_target && vi->k_done_valid) {  // every grid is already there
            vi->k_done = k_target;
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
    if (int rc = mgdp_vi_reset(vi)) return rc;
    int32_t k = 0;
    if (int rc = mgdp_vi_run_local(vi, &k)) return rc;
    double dv = 0.0;
    if (int rc = mgdp_vi_run_to(vi, k, &dv)) return rc;
    while (vi->d.horizon == 0 && !(dv < vi->d.tol) && k < vi->d.max_sweeps) {  // contraction broken by rounding: global rule
        if (int rc = mgdp_vi_sweep(vi, &dv)) return rc;
        ++k;
    }
    if (int rc = mgdp_vi_finish(vi, k)) return rc;
    vi->converged = vi->d.horizon > 0 ? 1 : dv < vi->d.tol;  // a finite horizon is exact after H sweeps
    if (sweeps_out) *sweeps_out = k;
    if (dv_out) *dv_out = dv;
    if (converged_out) *converged_out = vi->converged;
    return 0;
}

int mgdp_vi_persistent(const mgdp_vi *vi, int32_t *on) {
    MGDP_CHECK(vi && on, MGDP_E_INVALID, "null argument");
    *on = serve_eligible(vi) ? 1 : 0;
    return 0;
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

int mgdp_vi_enable_timing(mgdp_vi *vi, int32_t on) {
    MGDP_CHECK(vi, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(vi->d.device);
    if (int rc = server_stop(vi)) return rc;
    MGDP_HIP(hipStreamSynchronize(vi->stream));
    if (int rc = timed_collect(vi)) return rc;  // drop launches timed before this call
    vi->timing = on != 0;
    vi->total_ms = 0.0;
    vi->launches = 0;
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
