// envs.hip -- batched MiniGridEnv.step / gen_obs on MI355X (gfx950).
//
// Restates minigrid/minigrid_env.py:520-590 (step), :592-645 (gen_obs_grid / gen_obs),
// :448-479 (get_view_exts), :235-240 (_reward); minigrid/core/grid.py:110-143 (rotate_left,
// slice), :244-268 (encode), :291-328 (process_vis); minigrid/core/world_object.py (cell
// predicates, Door.toggle :185-195, Box.toggle :291-294).  Pinned by tests/test_gpu_step.py against
// 256-step trajectories captured from the reference (tests/golden/traj_*.npz) and against the
// oracle's step() restatement on 4096-env batches.
//
// Layout in HBM (B envs of W x H):
//   cell        uint8 [B][HWp]   one-byte cell code (type, colour, state), row-major, see cell_code
//   agent       int32 [B][4]     x, y, dir, step_count
//   carry       int32 [B][2]     carried (type, colour); type 0 = nothing
//   contents    uint8 [B][HWp]   optional (mgdp_envs_set_contents): the cell code of the object a
//                                Box at that cell holds (Box(contains=...), world_object.py:272-294),
//                                0 = none; ccontents uint8 [B]: the same for a carried Box
//   max_steps   int32 [B], see uint8 [B] (see_through_walls)
// One step = one envs_step_kernel launch: 2 lanes per env (see the kernel).  The V x V view is
// never materialised: view cell (i, j) maps to world top_left - f*j + r*i (f = DIR_TO_VEC[dir],
// r = right_vec, minigrid_env.py:421-446), which equals the reference's slice + (dir+1) x
// rotate_left; process_vis runs on a 64-bit visibility mask.
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_ext.h>

#include "common.h"

namespace mgdp {

__constant__ int kDX[4] = {1, 0, -1, 0};
__constant__ int kDY[4] = {0, 1, 0, -1};

struct EnvGeo {
    int B, W, H, HWp, vs;
    uint32_t nd_mask;   // NoDeath (wrappers.py:799-872): bit t = OBJECT_TO_IDX type t is a no-death type
    double death_cost;
};

// One-byte cell code.  Grid.encode() (grid.py:244-268) gives every cell (type, colour, state) with
// type <= 10, colour <= 5 and state != 0 only for doors (WorldObj.encode returns state 0,
// Door.encode :197-213 open 0 / closed 1 / locked 2), so a cell fits a byte: type*8 + colour, or
// 0x80 | state*8 + colour for a door.  One plane instead of three cuts the bytes the view windows
// pull from HBM by 3x (the window rows are read at cache-line granularity, i.e. most of each grid).
__host__ __device__ inline uint32_t cell_code(int t, int c, int s) {
    return t == T_DOOR ? 0x80u | ((uint32_t)s << 3) | (uint32_t)c : ((uint32_t)t << 3) | (uint32_t)c;
}
__host__ __device__ inline void cell_decode(uint32_t code, int &t, int &c, int &s) {
    const bool door = (code & 0x80u) != 0;
    t = door ? (int)T_DOOR : (int)(code >> 3);
    c = (int)(code & 7u);
    s = door ? (int)((code >> 3) & 3u) : 0;
}
constexpr uint32_t kCodeWall = (uint32_t)T_WALL * 8u + (uint32_t)C_GREY;  // padding / out-of-grid filler

// MGDP_STEP_NT: bit 0 = the obs tile leaves with nontemporal stores, bit 1 = the window rows are
// read with nontemporal loads (both streams are touched once per step; past the MALL at 2^20 envs)
#ifndef MGDP_STEP_NT
#define MGDP_STEP_NT 1  // measured: obs stores nt 92.3 -> 90.8 us (2^20 envs), 10.0 -> 9.3 us (65536); nt window loads 1.7x slower
#endif
__device__ __forceinline__ void copy_out(uint8_t *dst, const uint8_t *src, int bytes) {
    // dst is 16-B aligned: a workgroup's first env is a multiple of 32 (32*147 = 4704 = 16*294)
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (bytes & 15) == 0) {
        const uint4 *s = reinterpret_cast<const uint4 *>(src);
        uint4 *d = reinterpret_cast<uint4 *>(dst);
        for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) {
            if (MGDP_STEP_NT & 1) {
                const uint4 v = s[i];
                __builtin_nontemporal_store(v.x, &d[i].x);
                __builtin_nontemporal_store(v.y, &d[i].y);
                __builtin_nontemporal_store(v.z, &d[i].z);
                __builtin_nontemporal_store(v.w, &d[i].w);
            } else {
                d[i] = s[i];
            }
        }
    } else {
        for (int i = threadIdx.x; i < bytes; i += blockDim.x) dst[i] = src[i];
    }
}

// _reward: 1 - 0.9 * (step_count / max_steps), fp64, no contraction (minigrid_env.py:240)
__device__ __forceinline__ double reward_fn(int sc, int ms) {
    const double q = (double)sc / (double)ms;
    const double t = 0.9 * q;
    return 1.0 - t;
}

constexpr int kWinRow = 8;  // bytes per staged window row (vs + 1 <= 8 columns)

// The view's vs x vs cells always cover the axis-aligned world box [bx, bx+vs) x [by, by+vs)
// (rotation only permutes them); (tlx, tly) is the view's top-left (get_view_exts, :448-479).
__device__ __forceinline__ void view_box(int ax, int ay, int d, int vs, int &tlx, int &tly, int &bx, int &by) {
    const int hs = vs / 2;
    const int fx = kDX[d], fy = kDY[d], rx = -fy, ry = fx;
    tlx = ax + fx * (vs - 1) - rx * hs;
    tly = ay + fy * (vs - 1) - ry * hs;
    bx = tlx + min(0, -fx * (vs - 1)) + min(0, rx * (vs - 1));
    by = tly + min(0, -fy * (vs - 1)) + min(0, ry * (vs - 1));
}

// One env step: MiniGridEnv.step (minigrid_env.py:520-590) on registers; the front-cell mutation
// of pickup / drop / toggle is returned (mut, nt/nc/ns) instead of written, so the caller orders it
// against the window it stages.
struct StepOut {
    int x, y, d, sc, ct, cc, stat, term, trunc, mut, fi, nt, nc, ns, op;  // op: kOp* (front-cell action)
    double r;
};
enum { kOpNone = 0, kOpPickup = 1, kOpDrop = 2, kOpToggleBox = 3 };

// Rd: cell reader, rd(x, y) -> (type, colour, state) of in-grid cell (x, y) of this env.
template <typename Rd>
__device__ __forceinline__ StepOut step_core(const EnvGeo &g, const Rd &rd, int x, int y, int d, int sc, int ct,
                                             int cc, int a, int ms) {
    // Branch-free over the action (a wave steps envs with different actions): every effect is
    // computed and selected.  step_count += 1 first (:523); an out-of-grid front cell fails before
    // the action branch (Grid.get assert, :533), an unknown action after it (:579-580).
    StepOut o{x, y, d, sc + 1, ct, cc, MGDP_OK, 0, 0, 0, 0, 0, 0, 0, kOpNone, 0.0};
    const int fx = x + kDX[d], fy = y + kDY[d];
    const bool inb = (unsigned)fx < (unsigned)g.W && (unsigned)fy < (unsigned)g.H;
    const bool act_ok = (unsigned)a <= 6u;
    o.stat = !inb ? MGDP_E_BOUNDS : !act_ok ? MGDP_E_ACTION : MGDP_OK;
    const int fi = inb ? fy * g.W + fx : 0;
    int ft, fc, fs;
    rd(inb ? fx : 0, inb ? fy : 0, ft, fc, fs);
    const bool ok = o.stat == MGDP_OK;
    const bool fnone = ft == T_EMPTY;
    // left / right (:536-541)
    o.d = !ok ? d : a == 0 ? ((d + 3) & 3) : a == 1 ? ((d + 1) & 3) : d;
    // forward (:544-553): can_overlap = Goal, Floor, Lava, open Door (world_object.py)
    const bool fwd = ok && a == 2;
    const uint32_t fb = 1u << (ft & 31);  // type bit: comparison chains are lowered to branches
    const bool overlap = ((fb & ((1u << T_GOAL) | (1u << T_FLOOR) | (1u << T_LAVA))) != 0) | ((ft == T_DOOR) & (fs == D_OPEN));
    const bool move = fwd && (fnone || overlap);
    o.x = move ? fx : x;
    o.y = move ? fy : y;
    const bool goal = fwd && ft == T_GOAL;
    o.term = goal || (fwd && ft == T_LAVA);
    if (goal) o.r = reward_fn(o.sc, ms);
    // pickup (:556-561): Key / Ball / Box, hands empty
    const bool pickup = ok & (a == 3) & ((fb & ((1u << T_KEY) | (1u << T_BALL) | (1u << T_BOX))) != 0) & (ct == 0);
    // drop (:564-568): front empty, carrying
    const bool drop = ok && a == 4 && fnone && ct != 0;
    // toggle (:571-575): Door.toggle (locked: needs the carried Key of its colour, unlocks and
    // opens; else flips is_open, world_object.py:185-195); Box.toggle -> its contents (:291-294):
    // empty here, the caller puts a held object from the contents plane in its place
    const bool tdoor = ok && a == 5 && ft == T_DOOR && (fs != D_LOCKED || (ct == T_KEY && cc == fc));
    const bool tbox = ok && a == 5 && ft == T_BOX;
    const bool clear = pickup || tbox;
    o.mut = clear || drop || tdoor;
    o.op = pickup ? kOpPickup : drop ? kOpDrop : tbox ? kOpToggleBox : kOpNone;
    o.fi = fi;
    o.nt = clear ? T_EMPTY : drop ? ct : ft;
    o.nc = clear ? 0 : drop ? cc : fc;
    o.ns = tdoor ? (fs == D_OPEN ? D_CLOSED : D_OPEN) : 0;
    o.ct = pickup ? ft : drop ? 0 : ct;
    o.cc = pickup ? fc : drop ? 0 : cc;
    if (!ok) return o;
    if (o.sc >= ms) o.trunc = 1;
    if (g.nd_mask) {  // NoDeath.step: front cell before, agent's cell after the step (never mutated)
        const bool going = a == 2 && !fnone && ((g.nd_mask >> ft) & 1u);
        int ct_now, c_now, s_now;
        rd(o.x, o.y, ct_now, c_now, s_now);
        const bool in_death = ct_now != T_EMPTY && ((g.nd_mask >> ct_now) & 1u);
        if (o.term && (going || in_death)) {
            o.term = 0;
            o.r += g.death_cost;
        }
    }
    return o;
}

// ------------------------------------------------------------------------------------------------
// envs_step_kernel: G = 2 (or 1, 4, 8: MGDP_STEP_GROUP) lanes per env, 256 / G envs per 256-thread
// workgroup, so a 65536-env batch is 2048 waves (2 per SIMD).  Per env:
//   * lane v stages row v of the window box with 3 dword loads aligned by v_alignbyte into the
//     group's LDS window.  The box is the view box after the turn (left / right change only the
//     direction), extended by one cell along the heading for forward, so it holds both possible
//     views, the front cell and the agent's next cell: one dependent HBM round trip after the
//     agent record, and the step reads LDS.  The wave executes its LDS accesses in issue order, so
//     the other lanes' rows are visible without a barrier (the group lies inside one wave);
//   * every lane runs step_core on the window (uniform per group); lane 0 alone writes the per-env
//     results and the front-cell mutation (window and HBM);
//   * lane i < vs owns view column i: its see-behind bits are OR-reduced over the group (xor
//     shuffles), process_vis runs on the 64-bit mask in bit-parallel form (process_vis_bits), and
//     the lane encodes its column -- obs bytes [3*vs*i, 3*vs*(i+1)) of the env, contiguous because
//     the obs is x-major -- into the LDS obs tile, which leaves with 16-B coalesced stores.
// Measured (DoorKey-16 x 65536 per step, profiles/r01_step/): one thread per env on three byte
// planes 49 us; 8 lanes per env 16.5 us; one byte plane + one round trip 15.7 us; 4 lanes 11.4 us;
// out-of-grid cells staged as walls + a code -> (encoding, see_behind) table in LDS: 4 lanes
// 11.1 us, 2 lanes 10.2 us.
// ------------------------------------------------------------------------------------------------
constexpr int kGroupBlock = 256;  // threads per workgroup (G lanes per env, 256 / G envs)

__device__ __forceinline__ uint32_t rev8(uint32_t v) { return __builtin_bitreverse32(v) >> 24; }

// process_vis (grid.py:291-328) on the see-behind mask sb (bit j*8+i = view cell (i, j)), one row
// per step from j = vs-1 up.  In row j the left-to-right pass visits i = 0..vs-2: a visible
// see-behind cell makes i+1 visible and marks (i, j-1), (i+1, j-1).  Bit i's value when visited is
// final for that pass (only i-1 can set it before), so the pass equals the closure of the row's
// seeds m moving up through the see-behind run p = sb & [0, vs-2]: adding the seeds x = m & p to p
// carries through each seeded run and sets the bit past its end, hence L = m | ((p + x) ^ p).  The
// right-to-left pass (i = vs-1..1) is the same closure in bit-reversed order, seeded by L.  Checked
// against the literal loop on 200k random masks for vs = 3, 5, 7 before use.
template <int VS>
__device__ __forceinline__ unsigned long long process_vis_bits(unsigned long long sb) {
    constexpr uint32_t limL = (1u << (VS - 1)) - 1u;
    constexpr uint32_t limR = ((1u << VS) - 1u) & ~1u;
    unsigned long long mask = 0;
    uint32_t up = 0;
#pragma unroll
    for (int j = VS - 1; j >= 0; --j) {
        const uint32_t m = up | (j == VS - 1 ? 1u << (VS / 2) : 0u);
        const uint32_t s = (uint32_t)(sb >> (8 * j)) & 0xffu;
        const uint32_t p = s & limL;
        const uint32_t L = m | ((p + (m & p)) ^ p);
        const uint32_t g1 = L & p;
        const uint32_t q = s & limR;
        const uint32_t Lr = rev8(L), qr = rev8(q);
        const uint32_t R = rev8(Lr | ((qr + (Lr & qr)) ^ qr));
        const uint32_t g2 = R & q;
        up = g1 | (g1 << 1) | g2 | (g2 >> 1);
        mask |= (unsigned long long)R << (8 * j);
    }
    return mask;
}

template <int G>
__device__ __forceinline__ unsigned long long group_or(unsigned long long v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o);
        hi |= (uint32_t)__shfl_xor((int)hi, o);
    }
    return ((unsigned long long)hi << 32) | lo;
}

template <int VS, int G>
__global__ void __launch_bounds__(kGroupBlock)
envs_step_kernel(EnvGeo g, uint8_t *__restrict__ CELL, int32_t *__restrict__ agent, int32_t *__restrict__ carry,
                 uint8_t *__restrict__ cont, uint8_t *__restrict__ ccont, const int32_t *__restrict__ max_steps, const uint8_t *__restrict__ see,
                 const int32_t *__restrict__ actions, uint8_t *__restrict__ obs,
                 int32_t *__restrict__ direction, double *__restrict__ reward,
                 uint8_t *__restrict__ terminated, uint8_t *__restrict__ truncated,
                 int32_t *__restrict__ status, int observe_only) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int OB = VS * VS * 3;  // obs bytes per env
    constexpr int WR = VS + 1;       // staged rows: the view box plus the forward cell
    constexpr int RB = kWinRow;
    constexpr int WD = WR * RB / 4;  // window dwords per env
    constexpr int NE = kGroupBlock / G;        // envs per workgroup
    constexpr int NR = (WR + G - 1) / G;       // window rows staged per lane
    constexpr int NC = (VS + G - 1) / G;       // view columns per lane
    const int slot = threadIdx.x / G, r = threadIdx.x % G;
    const int e0 = blockIdx.x * NE;
    const int e = e0 + slot;
    uint8_t *img = smem + slot * OB;
    uint32_t *win = reinterpret_cast<uint32_t *>(smem + round_up(NE * OB, 16)) + slot * (WD + 1);
    uint8_t *wb = reinterpret_cast<uint8_t *>(win);
    // cell code -> encoded (type | colour << 8 | state << 16) | see_behind << 24 (world_object.py:
    // not a wall, not a closed / locked door); read per view cell instead of decoding
    __shared__ uint32_t lut[256];
    {
        int t, c, st;
        cell_decode(threadIdx.x, t, c, st);  // blockDim == 256: one entry per thread
        c = t == T_EMPTY ? 0 : c;
        const bool behind = t != T_WALL && !(t == T_DOOR && st != D_OPEN);
        lut[threadIdx.x] = (uint32_t)t | ((uint32_t)c << 8) | ((uint32_t)st << 16) | ((uint32_t)behind << 24);
    }
    __syncthreads();
    if (e < g.B) {
        uint8_t *cell = CELL + (long long)e * g.HWp;
        const int4 ag = reinterpret_cast<const int4 *>(agent)[e];
        const int2 cr = reinterpret_cast<const int2 *>(carry)[e];
        const int act = observe_only ? -1 : actions[e];
        const int ms = observe_only ? 1 : max_steps[e];
        const int d1 = act == 0 ? ((ag.z + 3) & 3) : act == 1 ? ((ag.z + 1) & 3) : ag.z;
        int tlx, tly, bx, by;
        view_box(ag.x, ag.y, d1, VS, tlx, tly, bx, by);
        if (act == 2) { bx += min(kDX[ag.z], 0); by += min(kDY[ag.z], 0); }
#pragma unroll
        for (int k = 0; k < NR; ++k) {  // lane r stages window rows r, r+G, ...
            const int row = r + G * k;
            if (row < WR) {
                const int nd = g.HWp >> 2;
                const int off = (by + row) * g.W + bx;
                const int a = off >> 2;  // floor: off may be negative left of / above the grid
                const int sh = off & 3;
                const uint32_t *P = reinterpret_cast<const uint32_t *>(cell);
                uint32_t w[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) {  // clamped: out-of-grid bytes are replaced below
                    const uint32_t *pq = P + min(max(a + q, 0), nd - 1);
                    w[q] = (MGDP_STEP_NT & 2) ? __builtin_nontemporal_load(pq) : *pq;
                }
                // Out-of-grid cells of the window become grey walls: slice() fills them with Wall()
                // (grid.py:136-139), which encodes and blocks sight exactly like a grid wall, so the
                // view loops below need no bounds tests.  Bytes [lo, hi) of the row are in the grid.
                const int y = by + row;
                const int lo = min(max(-bx, 0), 8), hi = (unsigned)y < (unsigned)g.H ? min(max(g.W - bx, 0), 8) : 0;
                const unsigned long long keep = (hi > lo ? (~0ull >> (64 - 8 * (hi - lo))) << (8 * lo) : 0ull);
                const unsigned long long bytes = ((unsigned long long)__builtin_amdgcn_alignbyte(w[2], w[1], sh) << 32) |
                                                 __builtin_amdgcn_alignbyte(w[1], w[0], sh);
                const unsigned long long v = (bytes & keep) | (0x0101010101010101ull * kCodeWall & ~keep);
                win[row * 2 + 0] = (uint32_t)v;
                win[row * 2 + 1] = (uint32_t)(v >> 32);
            }
        }
        asm volatile("" ::: "memory");  // the group's rows are written before any lane reads them
        StepOut o{ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, MGDP_OK, 0, 0, 0, 0, 0, 0, 0, kOpNone, 0.0};
        if (!observe_only) {
            // cells outside the staged box are only asked for by turns (whose result ignores them)
            const auto rd = [&](int cx, int cy, int &t, int &c, int &s) {
                const int u = cx - bx, v = cy - by;
                const bool in = (unsigned)u < (unsigned)RB && (unsigned)v < (unsigned)WR;
                cell_decode(in ? wb[v * RB + u] : 0u, t, c, s);
            };
            o = step_core(g, rd, ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, act, ms);
        }
        if (o.stat == MGDP_OK) {
            int bx2, by2;
            view_box(o.x, o.y, o.d, VS, tlx, tly, bx2, by2);
            asm volatile("" ::: "memory");
            if (o.mut && r == 0) {  // the front cell as the step left it (in the view: the agent did not move)
                const int fy = o.fi / g.W, fx = o.fi - fy * g.W;
                uint8_t code = (uint8_t)cell_code(o.nt, o.nc, o.ns);
                if (cont) {  // contents plane present (a uniform test): what Boxes hold moves with them
                    uint8_t *cf = cont + (long long)e * g.HWp + o.fi;
                    if (o.op == kOpToggleBox) {  // the box is replaced by what it held (None: empty)
                        const uint8_t held = *cf;
                        code = held ? held : code;
                        *cf = 0;
                    } else if (o.op == kOpPickup) {  // a carried Box keeps its contents
                        ccont[e] = *cf;
                        *cf = 0;
                    } else if (o.op == kOpDrop) {
                        *cf = ccont[e];
                        ccont[e] = 0;
                    }
                }
                wb[(fy - by) * RB + (fx - bx)] = code;
                cell[o.fi] = code;
            }
            asm volatile("" ::: "memory");
            const int fx = kDX[o.d], fy = kDY[o.d], rx = -fy, ry = fx;
            // Lane r owns view columns i = r, r+G, ...  View cell (i, j) is world (wx0 - fx*j,
            // wy0 - fy*j) with wx0 = tlx + rx*i, wy0 = tly + ry*i: window byte ow0 - j*(8*fy + fx).
            // Every view cell lies in the staged box, and out-of-grid ones hold wall codes.
            const int dj = RB * fy + fx;
            uint32_t cv[NC][VS];
            unsigned long long sb = 0;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const int i = min(r + G * k, VS - 1);  // lanes past the view re-read column VS-1, contribute no bits
                const int ow0 = (tly + ry * i - by) * RB + (tlx + rx * i - bx);
#pragma unroll
                for (int j = 0; j < VS; ++j) {
                    cv[k][j] = lut[wb[ow0 - j * dj]];
                    if (r + G * k < VS) sb |= (unsigned long long)(cv[k][j] >> 24) << (j * 8 + i);
                }
            }
            sb = group_or<G>(sb);
            const unsigned long long mask = see[e] ? ~0ull : process_vis_bits<VS>(sb);
            const uint32_t carried = o.ct > 0 ? (uint32_t)o.ct | ((uint32_t)o.cc << 8) : (uint32_t)T_EMPTY;
#pragma unroll
            for (int k = 0; k < NC; ++k) {  // encode column i, grid.py:244-268; the carried object at (VS/2, VS-1)
                const int i = r + G * k;
                if (i < VS) {
                    uint8_t *col = img + i * VS * 3;
#pragma unroll
                    for (int j = 0; j < VS; ++j) {
                        uint32_t x = (j == VS - 1 && i == VS / 2) ? carried : cv[k][j];
                        x = (mask >> (j * 8 + i)) & 1ull ? x : 0u;
                        col[3 * j] = (uint8_t)x;
                        col[3 * j + 1] = (uint8_t)(x >> 8);
                        col[3 * j + 2] = (uint8_t)(x >> 16);
                    }
                }
            }
        } else {
            for (int k = r; k < OB; k += G) img[k] = 0;
        }
        if (r == 0) {
            if (!observe_only) {
                reinterpret_cast<int4 *>(agent)[e] = make_int4(o.x, o.y, o.d, o.sc);
                reinterpret_cast<int2 *>(carry)[e] = make_int2(o.ct, o.cc);
                reward[e] = o.r;
                terminated[e] = (uint8_t)o.term;
                truncated[e] = (uint8_t)o.trunc;
                status[e] = o.stat;
            }
            direction[e] = o.d;
        }
    }
    __syncthreads();
    const int n = min(NE, g.B - e0);
    copy_out(obs + (long long)e0 * OB, smem, n * OB);
}

}  // namespace mgdp

using namespace mgdp;

struct mgdp_envs {
    int device = 0, B = 0, W = 0, H = 0, HW = 0, HWp = 0, vs = 7;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint8_t *d_cell = nullptr, *d_see = nullptr;  // d_cell: one-byte cell codes [B][HWp]
    uint8_t *d_cont = nullptr, *d_ccont = nullptr;  // Box contents planes (mgdp_envs_set_contents), else null
    int32_t *d_agent = nullptr, *d_carry = nullptr, *d_max = nullptr, *d_act = nullptr, *d_dir = nullptr,
            *d_status = nullptr;
    uint8_t *d_obs = nullptr, *d_term = nullptr, *d_trunc = nullptr;
    double *d_rew = nullptr;
    uint32_t nd_mask = 0;
    // masked loads (auto-reset of some envs): one staging copy + envs_masked_load_kernel
    uint8_t *d_stage = nullptr;
    size_t stage_bytes = 0;
    double death_cost = -1.0;
    int group = 2;  // lanes per env in envs_step_kernel (MGDP_STEP_GROUP = 1, 2, 4 or 8; 2 measured fastest)
    // step-kernel timing (mgdp_envs_enable_timing): pooled event pairs handed to hipExtLaunchKernelGGL
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev, ev_pool;
    double total_ms = 0.0;
    long long launches = 0;
};

namespace {

int timed_collect(mgdp_envs *E) {  // after a stream sync
    for (auto &p : E->ev) {
        float ms = 0.f;
        MGDP_HIP(hipEventElapsedTime(&ms, p.first, p.second));
        E->total_ms += ms;
        E->launches += 1;
        E->ev_pool.push_back(p);
    }
    E->ev.clear();
    return 0;
}

EnvGeo env_geo(const mgdp_envs *E) { return EnvGeo{E->B, E->W, E->H, E->HWp, E->vs, E->nd_mask, E->death_cost}; }

int launch_step(mgdp_envs *E, const int32_t *d_act, uint8_t *d_obs, int32_t *d_dir, double *d_rew,
                uint8_t *d_term, uint8_t *d_trunc, int32_t *d_status, int observe_only) {
    const int ne = kGroupBlock / E->group;
    const int grid = (E->B + ne - 1) / ne;
    const int smem = (int)round_up(ne * E->vs * E->vs * 3, 16) + ne * ((E->vs + 1) * kWinRow + 4);
    auto pick = [&](auto k7, auto k5, auto k3) { return E->vs == 7 ? k7 : E->vs == 5 ? k5 : k3; };
    auto k = E->group == 8   ? pick(envs_step_kernel<7, 8>, envs_step_kernel<5, 8>, envs_step_kernel<3, 8>)
             : E->group == 4 ? pick(envs_step_kernel<7, 4>, envs_step_kernel<5, 4>, envs_step_kernel<3, 4>)
             : E->group == 1 ? pick(envs_step_kernel<7, 1>, envs_step_kernel<5, 1>, envs_step_kernel<3, 1>)
                             : pick(envs_step_kernel<7, 2>, envs_step_kernel<5, 2>, envs_step_kernel<3, 2>);
    hipEvent_t ta = nullptr, tb = nullptr;
    if (E->timing) {
        if (E->ev.size() >= 4096) {  // bound the pending pairs
            MGDP_HIP(hipStreamSynchronize(E->stream));
            if (int rc = timed_collect(E)) return rc;
        }
        std::pair<hipEvent_t, hipEvent_t> p;
        if (!E->ev_pool.empty()) {
            p = E->ev_pool.back();
            E->ev_pool.pop_back();
        } else {
            MGDP_HIP(hipEventCreate(&p.first));
            MGDP_HIP(hipEventCreate(&p.second));
        }
        E->ev.push_back(p);
        ta = p.first;
        tb = p.second;
    }
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(kGroupBlock), smem, E->stream, ta, tb, 0, env_geo(E), E->d_cell, E->d_agent,
                       E->d_carry, E->d_cont, E->d_ccont, E->d_max, E->d_see, d_act, d_obs, d_dir, d_rew, d_term, d_trunc, d_status,
                       observe_only);
    MGDP_HIP(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int mgdp_envs_create(int32_t device, int32_t B, int32_t W, int32_t H, int32_t view_size, mgdp_envs **out) {
    MGDP_CHECK(out, MGDP_E_INVALID, "null argument");
    MGDP_CHECK(B > 0 && W >= 3 && H >= 3, MGDP_E_INVALID, "bad shape B=%d W=%d H=%d", B, W, H);
    MGDP_CHECK(view_size >= 3 && view_size <= 7 && (view_size & 1), MGDP_E_INVALID,
               "agent_view_size must be odd and in [3, 7] (got %d)", view_size);
    int ndev = 0;
    MGDP_HIP(hipGetDeviceCount(&ndev));
    MGDP_CHECK(device >= 0 && device < ndev, MGDP_E_HIP, "device %d not available (%d visible)", device, ndev);
    int group = 2;
    if (const char *ev = std::getenv("MGDP_STEP_GROUP")) {
        group = std::atoi(ev);
        MGDP_CHECK(group == 1 || group == 2 || group == 4 || group == 8, MGDP_E_INVALID,
                   "MGDP_STEP_GROUP must be 1, 2, 4 or 8 (got %s)", ev);
    }
    DeviceGuard guard(device);
    mgdp_envs *E = new mgdp_envs();
    E->group = group;
    E->device = device; E->B = B; E->W = W; E->H = H; E->HW = W * H; E->HWp = (int)round_up(W * H, 16);
    E->vs = view_size;
    const size_t P = (size_t)B * E->HWp;
    hipError_t e = hipSuccess;
    auto al = [&](void **p, size_t n) { if (e == hipSuccess) e = hipMalloc(p, n); };
    al((void **)&E->d_cell, P);
    al((void **)&E->d_see, B);
    al((void **)&E->d_agent, sizeof(int32_t) * 4 * B);
    al((void **)&E->d_carry, sizeof(int32_t) * 2 * B);
    al((void **)&E->d_max, sizeof(int32_t) * B);
    al((void **)&E->d_act, sizeof(int32_t) * B);
    al((void **)&E->d_dir, sizeof(int32_t) * B);
    al((void **)&E->d_status, sizeof(int32_t) * B);
    al((void **)&E->d_obs, (size_t)B * view_size * view_size * 3);
    al((void **)&E->d_term, B); al((void **)&E->d_trunc, B);
    al((void **)&E->d_rew, sizeof(double) * B);
    if (e == hipSuccess) { e = hipStreamCreateWithFlags(&E->stream, hipStreamNonBlocking); E->own_stream = e == hipSuccess; }
    if (e == hipSuccess) e = hipMemset(E->d_cell, (int)kCodeWall, P);
    if (e == hipSuccess) e = hipMemset(E->d_agent, 0, sizeof(int32_t) * 4 * B);
    if (e == hipSuccess) e = hipMemset(E->d_carry, 0, sizeof(int32_t) * 2 * B);
    if (e != hipSuccess) {
        mgdp_envs_destroy(E);
        return hip_fail(e, "mgdp_envs_create allocation", __FILE__, __LINE__);
    }
    *out = E;
    return 0;
}

int mgdp_envs_destroy(mgdp_envs *E) {
    if (!E) return 0;
    DeviceGuard guard(E->device);
    if (E->stream) (void)hipStreamSynchronize(E->stream);
    void *ps[] = {E->d_cell, E->d_see, E->d_agent, E->d_carry, E->d_max, E->d_act,
                  E->d_dir, E->d_status, E->d_obs, E->d_term, E->d_trunc, E->d_rew, E->d_cont, E->d_ccont, E->d_stage};
    for (void *p : ps) (void)hipFree(p);
    for (auto &p : E->ev) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    for (auto &p : E->ev_pool) { (void)hipEventDestroy(p.first); (void)hipEventDestroy(p.second); }
    if (E->own_stream) (void)hipStreamDestroy(E->stream);
    delete E;
    return 0;
}

int mgdp_envs_set_nodeath(mgdp_envs *E, uint32_t type_mask, double death_cost) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    MGDP_CHECK(!(type_mask & (1u << T_GOAL)), MGDP_E_INVALID, "goal cannot be a death cell (wrappers.py:845)");
    MGDP_CHECK(!(type_mask & (1u << T_EMPTY)), MGDP_E_INVALID, "an empty cell is no object");
    E->nd_mask = type_mask;
    E->death_cost = death_cost;
    return 0;
}

int mgdp_envs_set_stream(mgdp_envs *E, void *s) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    MGDP_HIP(hipStreamSynchronize(E->stream));
    if (E->own_stream) { (void)hipStreamDestroy(E->stream); E->own_stream = false; E->stream = nullptr; }
    if (s) E->stream = (hipStream_t)s;
    else { MGDP_HIP(hipStreamCreateWithFlags(&E->stream, hipStreamNonBlocking)); E->own_stream = true; }
    return 0;
}

// A masked reset (mgdp_envs_load with a mask): the host packs every env's prepared record into one
// staging buffer, one copy takes it to the device, and this kernel writes the masked envs' cells,
// agent, carry, max_steps and see_through and clears their Box contents -- O(1) runtime calls for
// any number of envs (a per-env copy / memset loop made a 65536-env auto-reset ~300k API calls).
// Staging layout: [mask B][see B][pad to 16][cells B*HWp][agent B*4 i32][carry B*2 i32][max B i32].
__global__ void __launch_bounds__(64)
envs_masked_load_kernel(int B, int HWp, const uint8_t *__restrict__ st, uint8_t *__restrict__ cell, int32_t *__restrict__ agent,
                        int32_t *__restrict__ carry, int32_t *__restrict__ maxs, uint8_t *__restrict__ see,
                        uint8_t *__restrict__ cont, uint8_t *__restrict__ ccont) {
    const int b = blockIdx.x;
    if (!st[b]) return;
    const size_t o_cells = (size_t)((2 * B + 15) / 16 * 16);
    const uint4 *src = reinterpret_cast<const uint4 *>(st + o_cells + (size_t)b * HWp);
    uint4 *dst = reinterpret_cast<uint4 *>(cell + (size_t)b * HWp);
    for (int i = threadIdx.x; i < HWp / 16; i += blockDim.x) {
        dst[i] = src[i];
        if (cont) reinterpret_cast<uint4 *>(cont + (size_t)b * HWp)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (threadIdx.x == 0) {
        const int32_t *ag = reinterpret_cast<const int32_t *>(st + o_cells + (size_t)B * HWp);
        const int32_t *cr = ag + 4 * (size_t)B;
        const int32_t *ms = cr + 2 * (size_t)B;
        for (int j = 0; j < 4; ++j) agent[4 * b + j] = ag[4 * b + j];
        carry[2 * b] = cr[2 * b];
        carry[2 * b + 1] = cr[2 * b + 1];
        maxs[b] = ms[b];
        see[b] = st[B + b];
        if (ccont) ccont[b] = 0;
    }
}

int mgdp_envs_load(mgdp_envs *E, const uint8_t *enc, const int32_t *agent, const int32_t *max_steps,
                   const uint8_t *see_through, const uint8_t *mask) {
    MGDP_CHECK(E && enc && agent && max_steps && see_through, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(E->device);
    const int B = E->B, W = E->W, H = E->H, HWp = E->HWp;
    for (int b = 0; b < B; ++b) {
        if (mask && !mask[b]) continue;
        MGDP_CHECK(max_steps[b] > 0, MGDP_E_INVALID, "env %d: max_steps must be > 0", b);
        const int x = agent[3 * b], y = agent[3 * b + 1], d = agent[3 * b + 2];
        MGDP_CHECK(x >= 0 && y >= 0 && x < W && y < H && d >= 0 && d < 4, MGDP_E_BOUNDS,
                   "env %d: agent (%d,%d,%d) outside the grid", b, x, y, d);
    }
    // x-major (W,H,3) -> row-major one-byte cell codes (cell_code); what a byte cannot hold is an
    // encoding Grid.encode() never produces
    std::vector<uint8_t> cl((size_t)B * HWp, (uint8_t)kCodeWall);
    std::vector<int32_t> ag((size_t)B * 4), cr((size_t)B * 2, 0);
    for (int b = 0; b < B; ++b) {
        if (mask && !mask[b]) continue;
        const uint8_t *eb = enc + (size_t)b * W * H * 3;
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < H; ++y) {
                const uint8_t *c = eb + (x * H + y) * 3;
                const int t = c[0], co = t == T_EMPTY ? 0 : c[1], st = t == T_EMPTY ? 0 : c[2];
                MGDP_CHECK(t <= T_AGENT && co <= 5 && (t == T_DOOR ? st <= D_LOCKED : st == 0), MGDP_E_INVALID,
                           "env %d cell (%d,%d): encoding (%d,%d,%d) is not a Grid.encode() cell", b, x, y, t, c[1], c[2]);
                cl[(size_t)b * HWp + y * W + x] = (uint8_t)cell_code(t, co, st);
            }
        ag[4 * b] = agent[3 * b]; ag[4 * b + 1] = agent[3 * b + 1]; ag[4 * b + 2] = agent[3 * b + 2]; ag[4 * b + 3] = 0;
    }
    std::vector<int32_t> ms(max_steps, max_steps + B);
    std::vector<uint8_t> se(see_through, see_through + B);
    if (E->d_cont && !mask) {  // new grids hold no contents until mgdp_envs_set_contents says so
        MGDP_HIP(hipMemsetAsync(E->d_cont, 0, (size_t)B * HWp, E->stream));
        MGDP_HIP(hipMemsetAsync(E->d_ccont, 0, (size_t)B, E->stream));
    }
    if (!mask) {
        MGDP_HIP(hipMemcpyAsync(E->d_cell, cl.data(), cl.size(), hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_agent, ag.data(), ag.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_carry, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_max, ms.data(), ms.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_see, se.data(), se.size(), hipMemcpyHostToDevice, E->stream));
    } else {
        const size_t o_cells = (size_t)((2 * B + 15) / 16 * 16);
        const size_t need = o_cells + (size_t)B * HWp + sizeof(int32_t) * 7 * (size_t)B;
        std::vector<uint8_t> st(need, 0);
        std::memcpy(st.data(), mask, B);
        std::memcpy(st.data() + B, se.data(), B);
        std::memcpy(st.data() + o_cells, cl.data(), cl.size());
        std::memcpy(st.data() + o_cells + (size_t)B * HWp, ag.data(), ag.size() * 4);
        std::memcpy(st.data() + o_cells + (size_t)B * HWp + ag.size() * 4, cr.data(), cr.size() * 4);
        std::memcpy(st.data() + o_cells + (size_t)B * HWp + ag.size() * 4 + cr.size() * 4, ms.data(), ms.size() * 4);
        if (E->stage_bytes < need) {
            if (E->d_stage) MGDP_HIP(hipFree(E->d_stage));
            E->d_stage = nullptr;
            MGDP_HIP(hipMalloc((void **)&E->d_stage, need));
            E->stage_bytes = need;
        }
        MGDP_HIP(hipMemcpyAsync(E->d_stage, st.data(), need, hipMemcpyHostToDevice, E->stream));
        hipLaunchKernelGGL(envs_masked_load_kernel, dim3(B), dim3(64), 0, E->stream, B, HWp, E->d_stage, E->d_cell,
                           E->d_agent, E->d_carry, E->d_max, E->d_see, E->d_cont, E->d_ccont);
        MGDP_HIP(hipGetLastError());
    }
    MGDP_HIP(hipStreamSynchronize(E->stream));
    return 0;
}

int mgdp_envs_observe(mgdp_envs *E, uint8_t *obs, int32_t *direction) {
    MGDP_CHECK(E && obs, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(E->device);
    if (int rc = launch_step(E, nullptr, E->d_obs, E->d_dir, E->d_rew, E->d_term, E->d_trunc, E->d_status, 1)) return rc;
    const size_t ob = (size_t)E->B * E->vs * E->vs * 3;
    MGDP_HIP(hipMemcpyAsync(obs, E->d_obs, ob, hipMemcpyDeviceToHost, E->stream));
    if (direction) MGDP_HIP(hipMemcpyAsync(direction, E->d_dir, 4 * (size_t)E->B, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    return 0;
}

int mgdp_envs_step_device(mgdp_envs *E, const int32_t *d_actions, uint8_t *d_obs, int32_t *d_direction,
                          double *d_reward, uint8_t *d_terminated, uint8_t *d_truncated, int32_t *d_status) {
    MGDP_CHECK(E && d_actions && d_obs && d_direction && d_reward && d_terminated && d_truncated && d_status,
               MGDP_E_INVALID, "null argument");
    DeviceGuard guard(E->device);
    return launch_step(E, d_actions, d_obs, d_direction, d_reward, d_terminated, d_truncated, d_status, 0);
}

int mgdp_envs_step(mgdp_envs *E, const int32_t *actions, uint8_t *obs, int32_t *direction, double *reward,
                   uint8_t *terminated, uint8_t *truncated, int32_t *status) {
    MGDP_CHECK(E && actions, MGDP_E_INVALID, "null argument");
    DeviceGuard guard(E->device);
    const size_t B = E->B;
    MGDP_HIP(hipMemcpyAsync(E->d_act, actions, 4 * B, hipMemcpyHostToDevice, E->stream));
    if (int rc = launch_step(E, E->d_act, E->d_obs, E->d_dir, E->d_rew, E->d_term, E->d_trunc, E->d_status, 0)) return rc;
    std::vector<int32_t> st_local;
    int32_t *stat = status;
    if (!stat) { st_local.resize(B); stat = st_local.data(); }
    if (obs) MGDP_HIP(hipMemcpyAsync(obs, E->d_obs, B * E->vs * E->vs * 3, hipMemcpyDeviceToHost, E->stream));
    if (direction) MGDP_HIP(hipMemcpyAsync(direction, E->d_dir, 4 * B, hipMemcpyDeviceToHost, E->stream));
    if (reward) MGDP_HIP(hipMemcpyAsync(reward, E->d_rew, 8 * B, hipMemcpyDeviceToHost, E->stream));
    if (terminated) MGDP_HIP(hipMemcpyAsync(terminated, E->d_term, B, hipMemcpyDeviceToHost, E->stream));
    if (truncated) MGDP_HIP(hipMemcpyAsync(truncated, E->d_trunc, B, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipMemcpyAsync(stat, E->d_status, 4 * B, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    for (size_t b = 0; b < B; ++b) {
        if (stat[b] == MGDP_E_ACTION) { set_error("Unknown action: %d (env %zu)", actions[b], b); return MGDP_E_ACTION; }
        if (stat[b] == MGDP_E_BOUNDS) { set_error("env %zu: front cell outside the grid", b); return MGDP_E_BOUNDS; }
    }
    return 0;
}

int mgdp_envs_enable_timing(mgdp_envs *E, int32_t on) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    MGDP_HIP(hipStreamSynchronize(E->stream));
    if (int rc = timed_collect(E)) return rc;  // drop launches timed before this call
    E->timing = on != 0;
    E->total_ms = 0.0;
    E->launches = 0;
    return 0;
}

int mgdp_envs_kernel_time(mgdp_envs *E, double *total_ms, int64_t *launches) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    MGDP_HIP(hipStreamSynchronize(E->stream));
    if (int rc = timed_collect(E)) return rc;
    if (total_ms) *total_ms = E->total_ms;
    if (launches) *launches = (int64_t)E->launches;
    return 0;
}

int mgdp_envs_get_state(mgdp_envs *E, uint8_t *enc, int32_t *agent, int32_t *carry, int32_t *step_count) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    const int B = E->B, W = E->W, H = E->H, HWp = E->HWp;
    std::vector<int32_t> ag((size_t)B * 4);
    MGDP_HIP(hipMemcpyAsync(ag.data(), E->d_agent, ag.size() * 4, hipMemcpyDeviceToHost, E->stream));
    if (carry) MGDP_HIP(hipMemcpyAsync(carry, E->d_carry, 8 * (size_t)B, hipMemcpyDeviceToHost, E->stream));
    std::vector<uint8_t> cl;
    if (enc) {
        cl.resize((size_t)B * HWp);
        MGDP_HIP(hipMemcpyAsync(cl.data(), E->d_cell, cl.size(), hipMemcpyDeviceToHost, E->stream));
    }
    MGDP_HIP(hipStreamSynchronize(E->stream));
    for (int b = 0; b < B; ++b) {
        if (agent) { agent[3 * b] = ag[4 * b]; agent[3 * b + 1] = ag[4 * b + 1]; agent[3 * b + 2] = ag[4 * b + 2]; }
        if (step_count) step_count[b] = ag[4 * b + 3];
        if (enc) {
            uint8_t *eb = enc + (size_t)b * W * H * 3;
            for (int x = 0; x < W; ++x)
                for (int y = 0; y < H; ++y) {
                    const size_t i = (size_t)b * HWp + y * W + x;
                    uint8_t *c = eb + (x * H + y) * 3;
                    int t, co, st;
                    cell_decode(cl[i], t, co, st);
                    c[0] = (uint8_t)t; c[1] = (uint8_t)co; c[2] = (uint8_t)st;
                }
        }
    }
    return 0;
}

int mgdp_envs_set_state(mgdp_envs *E, const int32_t *agent, const int32_t *carry, const int32_t *step_count,
                        const uint8_t *mask) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    const int B = E->B;
    std::vector<int32_t> ag((size_t)B * 4), cr((size_t)B * 2);
    std::vector<uint8_t> cc((carry && E->d_ccont) ? (size_t)B : 0);  // carried Box contents
    MGDP_HIP(hipMemcpyAsync(ag.data(), E->d_agent, ag.size() * 4, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipMemcpyAsync(cr.data(), E->d_carry, cr.size() * 4, hipMemcpyDeviceToHost, E->stream));
    if (!cc.empty()) MGDP_HIP(hipMemcpyAsync(cc.data(), E->d_ccont, cc.size(), hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    for (int b = 0; b < B; ++b) {
        if (mask && !mask[b]) continue;
        if (agent) {
            MGDP_CHECK(agent[3 * b] >= 0 && agent[3 * b] < E->W && agent[3 * b + 1] >= 0 && agent[3 * b + 1] < E->H &&
                           agent[3 * b + 2] >= 0 && agent[3 * b + 2] < 4,
                       MGDP_E_BOUNDS, "env %d: agent outside the grid", b);
            ag[4 * b] = agent[3 * b]; ag[4 * b + 1] = agent[3 * b + 1]; ag[4 * b + 2] = agent[3 * b + 2];
        }
        if (step_count) ag[4 * b + 3] = step_count[b];
        if (carry) {
            cr[2 * b] = carry[2 * b]; cr[2 * b + 1] = carry[2 * b + 1];
            if (!cc.empty()) cc[b] = 0;  // a new carry holds nothing (see mgdp_envs_set_contents)
        }
    }
    MGDP_HIP(hipMemcpyAsync(E->d_agent, ag.data(), ag.size() * 4, hipMemcpyHostToDevice, E->stream));
    MGDP_HIP(hipMemcpyAsync(E->d_carry, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, E->stream));
    if (!cc.empty()) MGDP_HIP(hipMemcpyAsync(E->d_ccont, cc.data(), cc.size(), hipMemcpyHostToDevice, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    return 0;
}

// Box(contains=...) (world_object.py:272-294): toggle puts the held object in the box's cell,
// pickup carries the box with it, drop puts it back.  Contents are (type, colour, state) triples in
// Grid.encode() layout, type <= 1 (unseen / empty) = nothing held; each must be a cell code (see
// cell_code) and sit on a Box cell of the current grid; a carried one needs a carried Box.
int mgdp_envs_set_contents(mgdp_envs *E, const uint8_t *contents, const int32_t *carry_contents) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    const int B = E->B, W = E->W, H = E->H, HWp = E->HWp;
    std::vector<uint8_t> cl((size_t)B * HWp);
    std::vector<int32_t> cr((size_t)B * 2);
    MGDP_HIP(hipMemcpyAsync(cl.data(), E->d_cell, cl.size(), hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipMemcpyAsync(cr.data(), E->d_carry, cr.size() * 4, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    auto code_of = [](int t, int c, int s, uint8_t &out) -> bool {  // a held object's cell code
        if (t <= T_EMPTY) { out = 0; return true; }
        if (t == T_AGENT || c > 5 || (t == T_DOOR ? s > D_LOCKED : s != 0)) return false;
        out = (uint8_t)cell_code(t, c, s);
        return true;
    };
    std::vector<uint8_t> co, cc;
    if (contents) {
        co.assign((size_t)B * HWp, 0);
        for (int b = 0; b < B; ++b)
            for (int x = 0; x < W; ++x)
                for (int y = 0; y < H; ++y) {
                    const uint8_t *c = contents + ((size_t)b * W * H + x * H + y) * 3;
                    uint8_t code;
                    MGDP_CHECK(code_of(c[0], c[1], c[2], code), MGDP_E_INVALID,
                               "env %d cell (%d,%d): contents (%d,%d,%d) is not an object encoding", b, x, y, c[0], c[1], c[2]);
                    const size_t i = (size_t)b * HWp + y * W + x;
                    int t, col, st;
                    cell_decode(cl[i], t, col, st);
                    MGDP_CHECK(code == 0 || t == T_BOX, MGDP_E_INVALID, "env %d cell (%d,%d): contents on a non-box cell", b, x, y);
                    co[i] = code;
                }
    }
    if (carry_contents) {
        cc.assign((size_t)B, 0);
        for (int b = 0; b < B; ++b) {
            const int32_t *c = carry_contents + 3 * b;
            uint8_t code;
            MGDP_CHECK(c[0] >= 0 && c[1] >= 0 && c[2] >= 0 && code_of(c[0], c[1], c[2], code), MGDP_E_INVALID,
                       "env %d: carried contents (%d,%d,%d) is not an object encoding", b, c[0], c[1], c[2]);
            MGDP_CHECK(code == 0 || cr[2 * b] == T_BOX, MGDP_E_INVALID, "env %d: contents for a carried non-box", b);
            cc[b] = code;
        }
    }
    if (!E->d_cont) {
        hipError_t e = hipMalloc((void **)&E->d_cont, (size_t)B * HWp);
        if (e == hipSuccess) e = hipMalloc((void **)&E->d_ccont, (size_t)B);
        if (e == hipSuccess) e = hipMemsetAsync(E->d_cont, 0, (size_t)B * HWp, E->stream);
        if (e == hipSuccess) e = hipMemsetAsync(E->d_ccont, 0, (size_t)B, E->stream);
        if (e != hipSuccess) {
            (void)hipFree(E->d_cont);
            (void)hipFree(E->d_ccont);
            E->d_cont = E->d_ccont = nullptr;
            return hip_fail(e, "mgdp_envs_set_contents allocation", __FILE__, __LINE__);
        }
    }
    if (contents) MGDP_HIP(hipMemcpyAsync(E->d_cont, co.data(), co.size(), hipMemcpyHostToDevice, E->stream));
    if (carry_contents) MGDP_HIP(hipMemcpyAsync(E->d_ccont, cc.data(), cc.size(), hipMemcpyHostToDevice, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    return 0;
}

int mgdp_envs_get_contents(mgdp_envs *E, uint8_t *contents, int32_t *carry_contents) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    const int B = E->B, W = E->W, H = E->H, HWp = E->HWp;
    std::vector<uint8_t> co((size_t)B * HWp, 0), cc((size_t)B, 0);
    if (E->d_cont) {
        MGDP_HIP(hipMemcpyAsync(co.data(), E->d_cont, co.size(), hipMemcpyDeviceToHost, E->stream));
        MGDP_HIP(hipMemcpyAsync(cc.data(), E->d_ccont, cc.size(), hipMemcpyDeviceToHost, E->stream));
        MGDP_HIP(hipStreamSynchronize(E->stream));
    }
    auto put = [](uint8_t code, int &t, int &c, int &s) {
        if (code == 0) { t = c = s = 0; return; }
        cell_decode(code, t, c, s);
    };
    for (int b = 0; b < B; ++b) {
        int t, c, s;
        if (contents)
            for (int x = 0; x < W; ++x)
                for (int y = 0; y < H; ++y) {
                    put(co[(size_t)b * HWp + y * W + x], t, c, s);
                    uint8_t *o = contents + ((size_t)b * W * H + x * H + y) * 3;
                    o[0] = (uint8_t)t; o[1] = (uint8_t)c; o[2] = (uint8_t)s;
                }
        if (carry_contents) {
            put(cc[b], t, c, s);
            carry_contents[3 * b] = t; carry_contents[3 * b + 1] = c; carry_contents[3 * b + 2] = s;
        }
    }
    return 0;
}

}  // extern "C"
