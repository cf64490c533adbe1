// envs.hip -- batched MiniGridEnv.step / gen_obs on MI355X (gfx950).
//
// Restates minigrid/minigrid_env.py:520-590 (step), :592-645 (gen_obs_grid / gen_obs),
// :448-479 (get_view_exts), :235-240 (_reward); minigrid/core/grid.py:110-143 (rotate_left,
// slice), :244-268 (encode), :291-328 (process_vis); minigrid/core/world_object.py (cell
// predicates, Door.toggle :185-195, Box.toggle :291-294).  Pinned by tests/test_gpu_step.py against
// 256-step trajectories captured from the reference (tests/golden/traj_*.npz).
//
// Layout in HBM (B envs of W x H):
//   ty, co, st  uint8 [B][HWp]   OBJECT_TO_IDX / COLOR_TO_IDX / door state per cell, row-major
//   agent       int32 [B][4]     x, y, dir, step_count
//   carry       int32 [B][2]     carried (type, colour); type 0 = nothing
//   max_steps   int32 [B], see uint8 [B] (see_through_walls)
// One thread per env.  The V x V view is never materialised: view cell (i, j) maps to world
// top_left - f*j + r*i (f = DIR_TO_VEC[dir], r = right_vec, minigrid_env.py:421-446), which equals
// the reference's slice + (dir+1) x rotate_left; process_vis runs on a 64-bit visibility mask.
// Observations are assembled in LDS and leave with 16-byte coalesced stores.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"

namespace mgdp {

__constant__ int kDX[4] = {1, 0, -1, 0};
__constant__ int kDY[4] = {0, 1, 0, -1};

struct EnvGeo {
    int B, W, H, HWp, vs;
    uint32_t nd_mask;   // NoDeath (wrappers.py:799-872): bit t = OBJECT_TO_IDX type t is a no-death type
    double death_cost;
};

constexpr int kStepBlock = 64;  // envs per workgroup; obs staging = 64 * 147 B (16-B multiple)

__device__ __forceinline__ bool see_behind(int t, int s) {
    if (t == T_WALL) return false;
    if (t == T_DOOR) return s == D_OPEN;
    return true;
}

// gen_obs for one env into `img` (vs*vs*3 bytes, x-major [i][j][3]) in LDS.
__device__ void gen_obs_one(const EnvGeo &g, const uint8_t *ty, const uint8_t *co, const uint8_t *st,
                            int ax, int ay, int d, int ct, int cc, bool see_through, uint8_t *img) {
    const int vs = g.vs, hs = vs / 2;
    const int fx = kDX[d], fy = kDY[d];
    const int rx = -fy, ry = fx;
    const int tlx = ax + fx * (vs - 1) - rx * hs;
    const int tly = ay + fy * (vs - 1) - ry * hs;
    // see-behind mask, bit (j*8 + i)
    unsigned long long sb = 0, mask = 0;
    for (int j = 0; j < vs; ++j)
        for (int i = 0; i < vs; ++i) {
            const int wx = tlx - fx * j + rx * i, wy = tly - fy * j + ry * i;
            bool s = false;  // out of bounds -> Wall (grid.py:136-139)
            if (wx >= 0 && wy >= 0 && wx < g.W && wy < g.H) {
                const int idx = wy * g.W + wx;
                s = see_behind(ty[idx], st[idx]);
            }
            if (s) sb |= 1ull << (j * 8 + i);
        }
    if (see_through) {
        mask = ~0ull;
    } else {  // process_vis, grid.py:291-328, literal loop order
        mask = 1ull << ((vs - 1) * 8 + hs);
        for (int j = vs - 1; j >= 0; --j) {
            for (int i = 0; i < vs - 1; ++i) {
                const unsigned long long b = 1ull << (j * 8 + i);
                if (!(mask & b) || !(sb & b)) continue;
                mask |= b << 1;
                if (j > 0) mask |= (b << 1 >> 8) | (b >> 8);
            }
            for (int i = vs - 1; i >= 1; --i) {
                const unsigned long long b = 1ull << (j * 8 + i);
                if (!(mask & b) || !(sb & b)) continue;
                mask |= b >> 1;
                if (j > 0) mask |= (b >> 1 >> 8) | (b >> 8);
            }
        }
    }
    // encode, grid.py:244-268 (None -> (1,0,0), hidden -> (0,0,0)); carried object at (hs, vs-1)
    for (int i = 0; i < vs; ++i)
        for (int j = 0; j < vs; ++j) {
            uint8_t *o = img + (i * vs + j) * 3;
            int t = 0, c = 0, s = 0;
            if (mask & (1ull << (j * 8 + i))) {
                if (i == hs && j == vs - 1) {
                    if (ct > 0) { t = ct; c = cc; } else { t = T_EMPTY; }
                } else {
                    const int wx = tlx - fx * j + rx * i, wy = tly - fy * j + ry * i;
                    if (wx >= 0 && wy >= 0 && wx < g.W && wy < g.H) {
                        const int idx = wy * g.W + wx;
                        t = ty[idx];
                        if (t != T_EMPTY) { c = co[idx]; s = st[idx]; }
                    } else {
                        t = T_WALL; c = C_GREY;
                    }
                }
            }
            o[0] = (uint8_t)t; o[1] = (uint8_t)c; o[2] = (uint8_t)s;
        }
}

__device__ __forceinline__ void copy_out(uint8_t *dst, const uint8_t *src, int bytes) {
    // dst is 16-B aligned when the block starts at a multiple of kStepBlock envs (147*64 = 9408)
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (bytes & 15) == 0) {
        const uint4 *s = reinterpret_cast<const uint4 *>(src);
        uint4 *d = reinterpret_cast<uint4 *>(dst);
        for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) d[i] = s[i];
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

// ------------------------------------------------------------------------------------------------
// Windowed gen_obs.  The view's vs x vs cells always cover an axis-aligned world box
// [bx, bx+vs) x [by, by+vs) (rotation only permutes them), so the thread stages that box of the
// three planes into its own LDS window with 3*vs*3 independent dword loads (all in flight at
// once; byte-aligned with v_alignbyte so window cell (u, v) is byte u of row v) instead of ~5*vs*vs
// dependent byte loads from HBM, and the visibility and encode passes read LDS.  Rows outside the
// grid are loaded from a clamped address and never read (bounds are tested in world coordinates,
// exactly as gen_obs_one does).  Bit-identical to gen_obs_one.
// ------------------------------------------------------------------------------------------------
constexpr int kWinRow = 8;                    // bytes per staged window row (vs <= 7)
__host__ __device__ constexpr int win_stride(int vs) { return 3 * vs * kWinRow + 4; }  // odd dword count

__device__ __forceinline__ void view_box(int ax, int ay, int d, int vs, int &tlx, int &tly, int &bx, int &by) {
    const int hs = vs / 2;
    const int fx = kDX[d], fy = kDY[d], rx = -fy, ry = fx;
    tlx = ax + fx * (vs - 1) - rx * hs;
    tly = ay + fy * (vs - 1) - ry * hs;
    bx = tlx + min(0, -fx * (vs - 1)) + min(0, rx * (vs - 1));
    by = tly + min(0, -fy * (vs - 1)) + min(0, ry * (vs - 1));
}

template <int VS>
__device__ __forceinline__ void stage_window(const EnvGeo &g, const uint8_t *ty, const uint8_t *co, const uint8_t *st,
                                             int bx, int by, uint32_t *win) {
    const int nd = g.HWp >> 2;
    const uint32_t *P[3] = {reinterpret_cast<const uint32_t *>(ty), reinterpret_cast<const uint32_t *>(co),
                            reinterpret_cast<const uint32_t *>(st)};
    uint32_t w[3][VS][3];
#pragma unroll
    for (int v = 0; v < VS; ++v) {
        const int o = (by + v) * g.W + bx;
        const int a = o >> 2;  // floor(o / 4): o may be negative left of / above the grid
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int idx = min(max(a + q, 0), nd - 1);  // only bytes of in-grid cells are ever read
#pragma unroll
            for (int p = 0; p < 3; ++p) w[p][v][q] = P[p][idx];
        }
    }
#pragma unroll
    for (int v = 0; v < VS; ++v) {
        const int sh = ((by + v) * g.W + bx) & 3;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            win[(p * VS + v) * 2 + 0] = __builtin_amdgcn_alignbyte(w[p][v][1], w[p][v][0], sh);
            win[(p * VS + v) * 2 + 1] = __builtin_amdgcn_alignbyte(w[p][v][2], w[p][v][1], sh);
        }
    }
}

// gen_obs_one on the staged window `wb` (plane p, row v, column u at wb[(p*vs + v)*8 + u]).
__device__ void gen_obs_win(const EnvGeo &g, const uint8_t *wb, int tlx, int tly, int bx, int by, int d, int ct,
                            int cc, bool see_through, uint8_t *img) {
    const int vs = g.vs, hs = vs / 2;
    const int fx = kDX[d], fy = kDY[d];
    const int rx = -fy, ry = fx;
    const uint8_t *WT = wb, *WC = wb + vs * kWinRow, *WS = wb + 2 * vs * kWinRow;
    unsigned long long sb = 0, mask = 0;
    for (int j = 0; j < vs; ++j)
        for (int i = 0; i < vs; ++i) {
            const int wx = tlx - fx * j + rx * i, wy = tly - fy * j + ry * i;
            bool s = false;  // out of bounds -> Wall (grid.py:136-139)
            if (wx >= 0 && wy >= 0 && wx < g.W && wy < g.H) {
                const int o = (wy - by) * kWinRow + (wx - bx);
                s = see_behind(WT[o], WS[o]);
            }
            if (s) sb |= 1ull << (j * 8 + i);
        }
    if (see_through) {
        mask = ~0ull;
    } else {  // process_vis, grid.py:291-328, literal loop order
        mask = 1ull << ((vs - 1) * 8 + hs);
        for (int j = vs - 1; j >= 0; --j) {
            for (int i = 0; i < vs - 1; ++i) {
                const unsigned long long b = 1ull << (j * 8 + i);
                if (!(mask & b) || !(sb & b)) continue;
                mask |= b << 1;
                if (j > 0) mask |= (b << 1 >> 8) | (b >> 8);
            }
            for (int i = vs - 1; i >= 1; --i) {
                const unsigned long long b = 1ull << (j * 8 + i);
                if (!(mask & b) || !(sb & b)) continue;
                mask |= b >> 1;
                if (j > 0) mask |= (b >> 1 >> 8) | (b >> 8);
            }
        }
    }
    for (int i = 0; i < vs; ++i)
        for (int j = 0; j < vs; ++j) {
            uint8_t *o = img + (i * vs + j) * 3;
            int t = 0, c = 0, s = 0;
            if (mask & (1ull << (j * 8 + i))) {
                if (i == hs && j == vs - 1) {
                    if (ct > 0) { t = ct; c = cc; } else { t = T_EMPTY; }
                } else {
                    const int wx = tlx - fx * j + rx * i, wy = tly - fy * j + ry * i;
                    if (wx >= 0 && wy >= 0 && wx < g.W && wy < g.H) {
                        const int w = (wy - by) * kWinRow + (wx - bx);
                        t = WT[w];
                        if (t != T_EMPTY) { c = WC[w]; s = WS[w]; }
                    } else {
                        t = T_WALL; c = C_GREY;
                    }
                }
            }
            o[0] = (uint8_t)t; o[1] = (uint8_t)c; o[2] = (uint8_t)s;
        }
}

// One env step: MiniGridEnv.step (minigrid_env.py:520-590) on registers; the front-cell mutation
// of pickup / drop / toggle is returned (mut, nt/nc/ns) instead of written, so the caller orders it
// against the window staging.
struct StepOut {
    int x, y, d, sc, ct, cc, stat, term, trunc, mut, fi, nt, nc, ns;
    double r;
};

__device__ __forceinline__ StepOut step_one(const EnvGeo &g, const uint8_t *ty, const uint8_t *co, const uint8_t *st,
                                            int x, int y, int d, int sc, int ct, int cc, int a, int ms) {
    // Branch-free over the action (a wave steps envs with different actions): every effect is
    // computed and selected.  step_count += 1 first (:523); an out-of-grid front cell fails before
    // the action branch (Grid.get assert, :533), an unknown action after it (:579-580).
    StepOut o{x, y, d, sc + 1, ct, cc, MGDP_OK, 0, 0, 0, 0, 0, 0, 0, 0.0};
    const int fx = x + kDX[d], fy = y + kDY[d];
    const bool inb = (unsigned)fx < (unsigned)g.W && (unsigned)fy < (unsigned)g.H;
    const bool act_ok = (unsigned)a <= 6u;
    o.stat = !inb ? MGDP_E_BOUNDS : !act_ok ? MGDP_E_ACTION : MGDP_OK;
    const int fi = inb ? fy * g.W + fx : 0;
    const int ft = ty[fi], fc = co[fi], fs = st[fi];
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
    // opens; else flips is_open, world_object.py:185-195); Box(contains=None).toggle -> empty
    const bool tdoor = ok && a == 5 && ft == T_DOOR && (fs != D_LOCKED || (ct == T_KEY && cc == fc));
    const bool tbox = ok && a == 5 && ft == T_BOX;
    const bool clear = pickup || tbox;
    o.mut = clear || drop || tdoor;
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
        const int ct_now = ty[o.y * g.W + o.x];
        const bool in_death = ct_now != T_EMPTY && ((g.nd_mask >> ct_now) & 1u);
        if (o.term && (going || in_death)) {
            o.term = 0;
            o.r += g.death_cost;
        }
    }
    return o;
}

template <bool WIN>
__global__ void __launch_bounds__(kStepBlock)
envs_step_kernel(EnvGeo g, uint8_t *__restrict__ TY, uint8_t *__restrict__ CO, uint8_t *__restrict__ ST,
                 int32_t *__restrict__ agent, int32_t *__restrict__ carry,
                 const int32_t *__restrict__ max_steps, const uint8_t *__restrict__ see,
                 const int32_t *__restrict__ actions, uint8_t *__restrict__ obs,
                 int32_t *__restrict__ direction, double *__restrict__ reward,
                 uint8_t *__restrict__ terminated, uint8_t *__restrict__ truncated,
                 int32_t *__restrict__ status, int observe_only) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int obs_bytes = g.vs * g.vs * 3;
    const int e0 = blockIdx.x * kStepBlock;
    const int e = e0 + threadIdx.x;
    uint8_t *img = smem + threadIdx.x * obs_bytes;
    uint32_t *win = reinterpret_cast<uint32_t *>(smem + round_up(kStepBlock * obs_bytes, 16) +
                                                 threadIdx.x * win_stride(g.vs));
    if (e < g.B) {
        uint8_t *ty = TY + (long long)e * g.HWp;
        uint8_t *co = CO + (long long)e * g.HWp;
        uint8_t *st = ST + (long long)e * g.HWp;
        const int4 ag = reinterpret_cast<const int4 *>(agent)[e];
        const int2 cr = reinterpret_cast<const int2 *>(carry)[e];
        StepOut o{ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, MGDP_OK, 0, 0, 0, 0, 0, 0, 0, 0.0};
        if (!observe_only) o = step_one(g, ty, co, st, ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, actions[e], max_steps[e]);
        if (!WIN && o.mut) { ty[o.fi] = (uint8_t)o.nt; co[o.fi] = (uint8_t)o.nc; st[o.fi] = (uint8_t)o.ns; }
        if (o.stat == MGDP_OK) {
            if (WIN) {
                int tlx, tly, bx, by;
                view_box(o.x, o.y, o.d, g.vs, tlx, tly, bx, by);
                if (g.vs == 7) stage_window<7>(g, ty, co, st, bx, by, win);
                else if (g.vs == 5) stage_window<5>(g, ty, co, st, bx, by, win);
                else stage_window<3>(g, ty, co, st, bx, by, win);
                uint8_t *wb = reinterpret_cast<uint8_t *>(win);
                if (o.mut) {  // the front cell (in the view: the agent did not move) as the step left it
                    const int w = (o.fi / g.W - by) * kWinRow + (o.fi % g.W - bx);
                    wb[w] = (uint8_t)o.nt; wb[g.vs * kWinRow + w] = (uint8_t)o.nc; wb[2 * g.vs * kWinRow + w] = (uint8_t)o.ns;
                    ty[o.fi] = (uint8_t)o.nt; co[o.fi] = (uint8_t)o.nc; st[o.fi] = (uint8_t)o.ns;
                }
                gen_obs_win(g, wb, tlx, tly, bx, by, o.d, o.ct, o.cc, see[e] != 0, img);
            } else {
                gen_obs_one(g, ty, co, st, o.x, o.y, o.d, o.ct, o.cc, see[e] != 0, img);
            }
        } else {
            for (int i = 0; i < obs_bytes; ++i) img[i] = 0;
        }
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
    __syncthreads();
    const int n = min(kStepBlock, g.B - e0);
    copy_out(obs + (long long)e0 * obs_bytes, smem, n * obs_bytes);
}

// ------------------------------------------------------------------------------------------------
// Lane-group step kernel (the default): kGroup = 8 lanes per env, 32 envs per 256-thread
// workgroup, so a 65536-env batch is 8192 waves (8 per SIMD) instead of 1024 one-thread-per-env
// waves whose dependent HBM and LDS latencies nothing could hide.  Per env:
//   * every lane of the group runs step_one on the same (broadcast) loads; lane 0 alone writes
//     the per-env results and the front-cell mutation;
//   * lane v < vs stages row v of the view box (3 planes, dword loads aligned with v_alignbyte)
//     into the group's LDS window; the wave executes its LDS accesses in issue order, so the other
//     lanes' rows are visible to the reads below without a barrier (the group is inside one wave);
//   * lane i < vs owns view column i: its see-behind bits are OR-reduced over the group (xor
//     shuffles), process_vis runs on the 64-bit mask in bit-parallel form (process_vis_bits), and
//     the lane encodes its column -- obs bytes [3*vs*i, 3*vs*(i+1)) of the env, contiguous because
//     the obs is x-major -- into the LDS obs tile, which leaves with 16-B coalesced stores.
// Bit-identical to envs_step_kernel (tests/test_gpu_step.py runs both against the reference's
// trajectories and the oracle).
// ------------------------------------------------------------------------------------------------
constexpr int kGroup = 8;
constexpr int kGroupBlock = 256;
constexpr int kGroupEnvs = kGroupBlock / kGroup;

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

__device__ __forceinline__ unsigned long long group_or(unsigned long long v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int o = 1; o < kGroup; o <<= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o);
        hi |= (uint32_t)__shfl_xor((int)hi, o);
    }
    return ((unsigned long long)hi << 32) | lo;
}

template <int VS>
__global__ void __launch_bounds__(kGroupBlock)
envs_step_group_kernel(EnvGeo g, uint8_t *__restrict__ TY, uint8_t *__restrict__ CO, uint8_t *__restrict__ ST,
                       int32_t *__restrict__ agent, int32_t *__restrict__ carry,
                       const int32_t *__restrict__ max_steps, const uint8_t *__restrict__ see,
                       const int32_t *__restrict__ actions, uint8_t *__restrict__ obs,
                       int32_t *__restrict__ direction, double *__restrict__ reward,
                       uint8_t *__restrict__ terminated, uint8_t *__restrict__ truncated,
                       int32_t *__restrict__ status, int observe_only) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int OB = VS * VS * 3;            // obs bytes per env
    constexpr int WD = 3 * VS * 2;             // window dwords per env (3 planes x VS rows x 8 B)
    constexpr int RB = kWinRow;                // window row bytes
    const int slot = threadIdx.x / kGroup, r = threadIdx.x % kGroup;
    const int e0 = blockIdx.x * kGroupEnvs;
    const int e = e0 + slot;
    uint8_t *img = smem + slot * OB;
    uint32_t *win = reinterpret_cast<uint32_t *>(smem + round_up(kGroupEnvs * OB, 16)) + slot * (WD + 1);
    const uint8_t *wb = reinterpret_cast<const uint8_t *>(win);
    if (e < g.B) {
        uint8_t *ty = TY + (long long)e * g.HWp;
        uint8_t *co = CO + (long long)e * g.HWp;
        uint8_t *st = ST + (long long)e * g.HWp;
        const int4 ag = reinterpret_cast<const int4 *>(agent)[e];
        const int2 cr = reinterpret_cast<const int2 *>(carry)[e];
        StepOut o{ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, MGDP_OK, 0, 0, 0, 0, 0, 0, 0, 0.0};
        if (!observe_only) o = step_one(g, ty, co, st, ag.x, ag.y, ag.z, ag.w, cr.x, cr.y, actions[e], max_steps[e]);
        if (o.stat == MGDP_OK) {
            int tlx, tly, bx, by;
            view_box(o.x, o.y, o.d, VS, tlx, tly, bx, by);
            if (r < VS) {  // lane r stages window row r
                const int nd = g.HWp >> 2;
                const int off = (by + r) * g.W + bx;
                const int a = off >> 2;  // floor: off may be negative left of / above the grid
                const int sh = off & 3;
                const uint32_t *P[3] = {reinterpret_cast<const uint32_t *>(ty), reinterpret_cast<const uint32_t *>(co),
                                        reinterpret_cast<const uint32_t *>(st)};
                uint32_t w[3][3];
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int q = 0; q < 3; ++q) w[p][q] = P[p][min(max(a + q, 0), nd - 1)];  // only in-grid bytes are read
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    win[(p * VS + r) * 2 + 0] = __builtin_amdgcn_alignbyte(w[p][1], w[p][0], sh);
                    win[(p * VS + r) * 2 + 1] = __builtin_amdgcn_alignbyte(w[p][2], w[p][1], sh);
                }
            }
            asm volatile("" ::: "memory");
            if (o.mut && r == 0) {  // the front cell as the step left it (in the view: the agent did not move)
                const int fy = o.fi / g.W, fx = o.fi - fy * g.W;
                const int w = (fy - by) * RB + (fx - bx);
                uint8_t *wm = reinterpret_cast<uint8_t *>(win);
                wm[w] = (uint8_t)o.nt; wm[VS * RB + w] = (uint8_t)o.nc; wm[2 * VS * RB + w] = (uint8_t)o.ns;
                ty[o.fi] = (uint8_t)o.nt; co[o.fi] = (uint8_t)o.nc; st[o.fi] = (uint8_t)o.ns;
            }
            asm volatile("" ::: "memory");
            const int fx = kDX[o.d], fy = kDY[o.d], rx = -fy, ry = fx;
            const int i = r;
            // Column i's world cells (wx0 - fx*j, wy0 - fy*j), read branch-free: an out-of-grid
            // cell reads window byte 0 and is then replaced (out of bounds -> Wall, grid.py:136-139).
            const int wx0 = tlx + rx * i, wy0 = tly + ry * i;
            uint32_t tv[VS], cv[VS], sv[VS];
            bool inb[VS];
            unsigned long long sb = 0;
#pragma unroll
            for (int j = 0; j < VS; ++j) {
                const int wx = wx0 - fx * j, wy = wy0 - fy * j;
                inb[j] = i < VS && (unsigned)wx < (unsigned)g.W && (unsigned)wy < (unsigned)g.H;
                const int ow = inb[j] ? (wy - by) * RB + (wx - bx) : 0;
                tv[j] = wb[ow]; cv[j] = wb[VS * RB + ow]; sv[j] = wb[2 * VS * RB + ow];
                // see_behind as bit tests (comparison chains are lowered to branches)
                const uint32_t tb = 1u << (tv[j] & 31u);
                const bool behind = !(tb & (1u << T_WALL)) & !((tb & (1u << T_DOOR)) && sv[j] != D_OPEN);
                sb |= (unsigned long long)(inb[j] && behind) << (j * 8 + (i & 7));
            }
            sb = group_or(sb);
            const unsigned long long mask = see[e] ? ~0ull : process_vis_bits<VS>(sb);
            if (i < VS) {  // encode column i, grid.py:244-268; the carried object at (VS/2, VS-1)
                uint8_t *col = img + i * VS * 3;
                const bool centre_col = i == VS / 2;
#pragma unroll
                for (int j = 0; j < VS; ++j) {
                    uint32_t t = inb[j] ? tv[j] : (uint32_t)T_WALL;
                    uint32_t c = inb[j] ? (tv[j] == T_EMPTY ? 0u : cv[j]) : (uint32_t)C_GREY;
                    uint32_t s = inb[j] && tv[j] != T_EMPTY ? sv[j] : 0u;
                    if (j == VS - 1 && centre_col) {
                        t = o.ct > 0 ? (uint32_t)o.ct : (uint32_t)T_EMPTY;
                        c = o.ct > 0 ? (uint32_t)o.cc : 0u;
                        s = 0;
                    }
                    const bool vis = (mask >> (j * 8 + i)) & 1ull;
                    col[3 * j] = (uint8_t)(vis ? t : 0u);
                    col[3 * j + 1] = (uint8_t)(vis ? c : 0u);
                    col[3 * j + 2] = (uint8_t)(vis ? s : 0u);
                }
            }
        } else if (r < VS) {
            for (int k = 0; k < 3 * VS; ++k) img[r * VS * 3 + k] = 0;
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
    const int n = min(kGroupEnvs, g.B - e0);
    copy_out(obs + (long long)e0 * OB, smem, n * OB);
}

}  // namespace mgdp

using namespace mgdp;

struct mgdp_envs {
    int device = 0, B = 0, W = 0, H = 0, HW = 0, HWp = 0, vs = 7;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint8_t *d_ty = nullptr, *d_co = nullptr, *d_st = nullptr, *d_see = nullptr;
    int32_t *d_agent = nullptr, *d_carry = nullptr, *d_max = nullptr, *d_act = nullptr, *d_dir = nullptr,
            *d_status = nullptr;
    uint8_t *d_obs = nullptr, *d_term = nullptr, *d_trunc = nullptr;
    double *d_rew = nullptr;
    uint32_t nd_mask = 0;
    double death_cost = -1.0;
    // step kernel: 0 = envs_step_group_kernel (8 lanes per env, default), 1 = envs_step_kernel with
    // the staged window, 2 = envs_step_kernel with per-cell HBM byte loads (gen_obs_one).
    // MGDP_STEP_KERNEL=group|thread|thread_bytes selects one (measured alternatives, all tested).
    int kmode = 0;
};

namespace {

EnvGeo env_geo(const mgdp_envs *E) { return EnvGeo{E->B, E->W, E->H, E->HWp, E->vs, E->nd_mask, E->death_cost}; }

int launch_step(mgdp_envs *E, const int32_t *d_act, uint8_t *d_obs, int32_t *d_dir, double *d_rew,
                uint8_t *d_term, uint8_t *d_trunc, int32_t *d_status, int observe_only) {
    if (E->kmode == 0) {
        const int grid = (E->B + kGroupEnvs - 1) / kGroupEnvs;
        const int smem = (int)round_up(kGroupEnvs * E->vs * E->vs * 3, 16) + kGroupEnvs * (3 * E->vs * 2 + 1) * 4;
        auto k = E->vs == 7 ? envs_step_group_kernel<7> : E->vs == 5 ? envs_step_group_kernel<5> : envs_step_group_kernel<3>;
        hipLaunchKernelGGL(k, dim3(grid), dim3(kGroupBlock), smem, E->stream, env_geo(E),
                           E->d_ty, E->d_co, E->d_st, E->d_agent, E->d_carry, E->d_max, E->d_see, d_act,
                           d_obs, d_dir, d_rew, d_term, d_trunc, d_status, observe_only);
    } else {
        const int grid = (E->B + kStepBlock - 1) / kStepBlock;
        const int smem = (int)round_up(kStepBlock * E->vs * E->vs * 3, 16) + kStepBlock * win_stride(E->vs);
        hipLaunchKernelGGL(E->kmode == 1 ? envs_step_kernel<true> : envs_step_kernel<false>, dim3(grid), dim3(kStepBlock), smem, E->stream, env_geo(E),
                           E->d_ty, E->d_co, E->d_st, E->d_agent, E->d_carry, E->d_max, E->d_see, d_act,
                           d_obs, d_dir, d_rew, d_term, d_trunc, d_status, observe_only);
    }
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
    int kmode = 0;
    if (const char *ev = std::getenv("MGDP_STEP_KERNEL")) {
        const std::string m(ev);
        MGDP_CHECK(m == "group" || m == "thread" || m == "thread_bytes", MGDP_E_INVALID,
                   "MGDP_STEP_KERNEL must be group, thread or thread_bytes (got %s)", ev);
        kmode = m == "group" ? 0 : m == "thread" ? 1 : 2;
    }
    DeviceGuard guard(device);
    mgdp_envs *E = new mgdp_envs();
    E->device = device; E->B = B; E->W = W; E->H = H; E->HW = W * H; E->HWp = (int)round_up(W * H, 16);
    E->vs = view_size;
    E->kmode = kmode;
    const size_t P = (size_t)B * E->HWp;
    hipError_t e = hipSuccess;
    auto al = [&](void **p, size_t n) { if (e == hipSuccess) e = hipMalloc(p, n); };
    al((void **)&E->d_ty, P); al((void **)&E->d_co, P); al((void **)&E->d_st, P);
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
    if (e == hipSuccess) e = hipMemset(E->d_ty, T_WALL, P);
    if (e == hipSuccess) e = hipMemset(E->d_co, C_GREY, P);
    if (e == hipSuccess) e = hipMemset(E->d_st, 0, P);
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
    void *ps[] = {E->d_ty, E->d_co, E->d_st, E->d_see, E->d_agent, E->d_carry, E->d_max, E->d_act,
                  E->d_dir, E->d_status, E->d_obs, E->d_term, E->d_trunc, E->d_rew};
    for (void *p : ps) (void)hipFree(p);
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
    // x-major (W,H,3) -> row-major planes
    std::vector<uint8_t> ty((size_t)B * HWp, T_WALL), co((size_t)B * HWp, C_GREY), st((size_t)B * HWp, 0);
    std::vector<int32_t> ag((size_t)B * 4), cr((size_t)B * 2, 0);
    for (int b = 0; b < B; ++b) {
        if (mask && !mask[b]) continue;
        const uint8_t *eb = enc + (size_t)b * W * H * 3;
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < H; ++y) {
                const uint8_t *c = eb + (x * H + y) * 3;
                const size_t i = (size_t)b * HWp + y * W + x;
                ty[i] = c[0];
                co[i] = c[0] == T_EMPTY ? 0 : c[1];
                st[i] = c[0] == T_EMPTY ? 0 : c[2];
            }
        ag[4 * b] = agent[3 * b]; ag[4 * b + 1] = agent[3 * b + 1]; ag[4 * b + 2] = agent[3 * b + 2]; ag[4 * b + 3] = 0;
    }
    std::vector<int32_t> ms(max_steps, max_steps + B);
    std::vector<uint8_t> se(see_through, see_through + B);
    if (!mask) {
        MGDP_HIP(hipMemcpyAsync(E->d_ty, ty.data(), ty.size(), hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_co, co.data(), co.size(), hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_st, st.data(), st.size(), hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_agent, ag.data(), ag.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_carry, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_max, ms.data(), ms.size() * 4, hipMemcpyHostToDevice, E->stream));
        MGDP_HIP(hipMemcpyAsync(E->d_see, se.data(), se.size(), hipMemcpyHostToDevice, E->stream));
    } else {
        for (int b = 0; b < B; ++b) {
            if (!mask[b]) continue;
            const size_t o = (size_t)b * HWp;
            MGDP_HIP(hipMemcpyAsync(E->d_ty + o, &ty[o], HWp, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_co + o, &co[o], HWp, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_st + o, &st[o], HWp, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_agent + 4 * b, &ag[4 * b], 16, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_carry + 2 * b, &cr[2 * b], 8, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_max + b, &ms[b], 4, hipMemcpyHostToDevice, E->stream));
            MGDP_HIP(hipMemcpyAsync(E->d_see + b, &se[b], 1, hipMemcpyHostToDevice, E->stream));
        }
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

int mgdp_envs_get_state(mgdp_envs *E, uint8_t *enc, int32_t *agent, int32_t *carry, int32_t *step_count) {
    MGDP_CHECK(E, MGDP_E_INVALID, "null handle");
    DeviceGuard guard(E->device);
    const int B = E->B, W = E->W, H = E->H, HWp = E->HWp;
    std::vector<int32_t> ag((size_t)B * 4);
    MGDP_HIP(hipMemcpyAsync(ag.data(), E->d_agent, ag.size() * 4, hipMemcpyDeviceToHost, E->stream));
    if (carry) MGDP_HIP(hipMemcpyAsync(carry, E->d_carry, 8 * (size_t)B, hipMemcpyDeviceToHost, E->stream));
    std::vector<uint8_t> ty, co, st;
    if (enc) {
        ty.resize((size_t)B * HWp); co.resize(ty.size()); st.resize(ty.size());
        MGDP_HIP(hipMemcpyAsync(ty.data(), E->d_ty, ty.size(), hipMemcpyDeviceToHost, E->stream));
        MGDP_HIP(hipMemcpyAsync(co.data(), E->d_co, co.size(), hipMemcpyDeviceToHost, E->stream));
        MGDP_HIP(hipMemcpyAsync(st.data(), E->d_st, st.size(), hipMemcpyDeviceToHost, E->stream));
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
                    c[0] = ty[i]; c[1] = co[i]; c[2] = st[i];
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
    MGDP_HIP(hipMemcpyAsync(ag.data(), E->d_agent, ag.size() * 4, hipMemcpyDeviceToHost, E->stream));
    MGDP_HIP(hipMemcpyAsync(cr.data(), E->d_carry, cr.size() * 4, hipMemcpyDeviceToHost, E->stream));
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
        if (carry) { cr[2 * b] = carry[2 * b]; cr[2 * b + 1] = carry[2 * b + 1]; }
    }
    MGDP_HIP(hipMemcpyAsync(E->d_agent, ag.data(), ag.size() * 4, hipMemcpyHostToDevice, E->stream));
    MGDP_HIP(hipMemcpyAsync(E->d_carry, cr.data(), cr.size() * 4, hipMemcpyHostToDevice, E->stream));
    MGDP_HIP(hipStreamSynchronize(E->stream));
    return 0;
}

}  // extern "C"
