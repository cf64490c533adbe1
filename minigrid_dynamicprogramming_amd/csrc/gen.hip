// gen.hip -- batched reset(seed) grid generation on the GPU.
//
// One thread per env builds the grid that reference reset(seed) builds: gymnasium seeds the env
// with np_random(seed) = numpy Generator(PCG64(SeedSequence(seed))) (gymnasium/utils/seeding.py;
// reference minigrid_env.py:119-157) and each family's _gen_grid draws from it in a fixed order:
//   EMPTY      empty.py:97-114           FOURROOMS  fourrooms.py:79-128
//   CROSSING   crossing.py:122-184       DOORKEY    doorkey.py:75-100
//   LAVAGAP    lavagap.py:101-136        DISTSHIFT  distshift.py:99-121
// with the MiniGridEnv helpers _rand_int (:242-254), place_obj (:308-367) and place_agent
// (:378-390).  numpy's algorithms are restated below and pinned by tests against numpy itself
// (raw PCG64 output, Generator.integers / shuffle / choice) and against the reference's grid
// digests (tests/golden/digests*.json):
//   SeedSequence(entropy).generate_state(4, uint64)  -- numpy/random/bit_generator.pyx
//   PCG64 (XSL-RR 128/64, set_seed = srandom_r(state=w0:w1, seq=w2:w3)), next_uint32 hands out the
//     low then the high half of one 64-bit output (numpy/random/src/pcg64)
//   Generator.integers(lo, hi) for int64: range r = hi-lo-1; r == 0 -> lo without a draw; else
//     Lemire's bounded method on next_uint32 with the (2^32 - 1 - r) % (r + 1) rejection threshold
//   Generator.shuffle(list): for i = n-1..1: swap(i, random_interval(i)), random_interval = masked
//     next_uint32 rejection
//   Generator.choice(range(a, b)) = a + integers(0, b - a)
// The grid is staged in LDS per thread and written out with coalesced stores, as the reference's
// x-major Grid.encode() (type, colour, state) -- the layout mgdp_envs_load takes -- and/or as
// row-major type codes (the layout mgdp_vi_load_cells_device takes).
#include "common.h"

namespace mgdp {
namespace {

// COLOR_TO_IDX, constants.py:11-20
enum : uint8_t { C_RED = 0, C_GREEN = 1, C_YELLOW = 4 };

struct U128 {
    uint64_t hi, lo;
};

__device__ __forceinline__ U128 mul128(U128 a, U128 b) {  // mod 2^128
    U128 r;
    r.lo = a.lo * b.lo;
    r.hi = __umul64hi(a.lo, b.lo) + a.lo * b.hi + a.hi * b.lo;
    return r;
}
__device__ __forceinline__ U128 add128(U128 a, U128 b) {
    U128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1u : 0u);
    return r;
}

// SeedSequence(seed).generate_state(4, np.uint64), pool size 4, no spawn key.
__device__ void seedseq_state(uint64_t seed, uint64_t (&out)[4]) {
    constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
    constexpr uint32_t MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
    uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int nent = (seed >> 32) ? 2 : 1;  // _int_to_uint32_array: little-endian words, 0 -> [0]
    uint32_t hc = INIT_A;
    auto hashmix = [&](uint32_t v) {
        v ^= hc;
        hc *= MULT_A;
        v *= hc;
        v ^= v >> 16;
        return v;
    };
    auto mix = [](uint32_t x, uint32_t y) {
        uint32_t r = MIX_L * x - MIX_R * y;
        r ^= r >> 16;
        return r;
    };
    uint32_t pool[4];
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < nent ? ent[i] : 0u);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
    uint32_t h = INIT_B;
    uint32_t w[8];
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= h;
        h *= MULT_B;
        v *= h;
        v ^= v >> 16;
        w[i] = v;
    }
    for (int i = 0; i < 4; ++i) out[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

struct Pcg64 {
    U128 state, inc;
    uint32_t buf;
    bool has32;

    __device__ void step() {
        const U128 mult{0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
        state = add128(mul128(state, mult), inc);
    }
    __device__ explicit Pcg64(uint64_t seed) {
        uint64_t v[4];
        seedseq_state(seed, v);
        const U128 initstate{v[0], v[1]}, initseq{v[2], v[3]};
        inc = U128{(initseq.hi << 1) | (initseq.lo >> 63), (initseq.lo << 1) | 1u};
        state = U128{0, 0};
        step();
        state = add128(state, initstate);
        step();
        has32 = false;
        buf = 0;
    }
    __device__ uint64_t next64() {
        step();
        const uint64_t x = state.hi ^ state.lo;
        const unsigned rot = (unsigned)(state.hi >> 58);
        return (x >> rot) | (x << ((64u - rot) & 63u));
    }
    __device__ uint32_t next32() {
        if (has32) {
            has32 = false;
            return buf;
        }
        const uint64_t n = next64();
        has32 = true;
        buf = (uint32_t)(n >> 32);
        return (uint32_t)n;
    }
    // Generator.integers(lo, hi) (int64, hi exclusive, hi - lo <= 2^32)
    __device__ int integers(int lo, int hi) {
        const uint32_t rng = (uint32_t)(hi - lo - 1);
        if (rng == 0) return lo;
        const uint32_t excl = rng + 1u;
        uint64_t m = (uint64_t)next32() * excl;
        uint32_t left = (uint32_t)m;
        if (left < excl) {
            const uint32_t thr = (0xFFFFFFFFu - rng) % excl;
            while (left < thr) {
                m = (uint64_t)next32() * excl;
                left = (uint32_t)m;
            }
        }
        return lo + (int)(m >> 32);
    }
    // random_interval(max), the draw of Generator.shuffle on lists
    __device__ int interval(int mx) {
        if (mx == 0) return 0;
        uint32_t mask = (uint32_t)mx;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = next32() & mask) > (uint32_t)mx) {
        }
        return (int)v;
    }
};

constexpr int kGenBlock = 64;
constexpr long long kMaxTries = 1 << 20;  // rejection cap (the reference loops without bound)

// One env's grid in LDS: 3 planes of W*H bytes (type, colour, state), x-major like Grid.encode.
struct GridL {
    uint8_t *g;
    int W, H;
    __device__ uint8_t type(int x, int y) const { return g[(x * H + y) * 3]; }
    __device__ void set(int x, int y, uint8_t t, uint8_t c, uint8_t s) {
        uint8_t *p = g + (x * H + y) * 3;
        p[0] = t;
        p[1] = c;
        p[2] = s;
    }
    __device__ void clear(int x, int y) { set(x, y, T_EMPTY, 0, 0); }
    __device__ void wall(int x, int y) { set(x, y, T_WALL, C_GREY, 0); }
    __device__ void obstacle(int x, int y, int t) {
        if (t == T_LAVA) set(x, y, T_LAVA, C_RED, 0);
        else wall(x, y);
    }
    __device__ void horz_wall(int x, int y, int len) {
        for (int i = 0; i < len; ++i) wall(x + i, y);
    }
    __device__ void vert_wall(int x, int y, int len, int t = T_WALL) {
        for (int j = 0; j < len; ++j) obstacle(x, y + j, t);
    }
    __device__ void wall_rect(int x, int y, int w, int h) {
        horz_wall(x, y, w);
        horz_wall(x, y + h - 1, w);
        vert_wall(x, y, h);
        vert_wall(x + w - 1, y, h);
    }
};

struct Agent {
    int x = -1, y = -1, dir = 0;
    bool ok = true;
};

// place_obj (minigrid_env.py:308-367): rejection-sample a cell inside top/size that is empty and
// not the agent's; returns false when the cap is hit.
__device__ bool place_obj(Pcg64 &r, GridL &g, const Agent &a, int tx, int ty, int sx, int sy, int &px, int &py) {
    tx = max(tx, 0);
    ty = max(ty, 0);
    for (long long n = 0; n < kMaxTries; ++n) {
        px = r.integers(tx, min(tx + sx, g.W));
        py = r.integers(ty, min(ty + sy, g.H));
        if (g.type(px, py) != T_EMPTY) continue;
        if (px == a.x && py == a.y) continue;
        return true;
    }
    return false;
}
// place_agent (:378-390)
__device__ void place_agent(Pcg64 &r, GridL &g, Agent &a, int tx, int ty, int sx, int sy) {
    a.x = a.y = -1;
    int px = 0, py = 0;
    a.ok = a.ok && place_obj(r, g, a, tx, ty, sx, sy, px, py);
    a.x = px;
    a.y = py;
    a.dir = r.integers(0, 4);
}

__device__ void gen_empty(Pcg64 &r, GridL &g, Agent &a, const mgdp_gen_desc &d) {
    g.wall_rect(0, 0, g.W, g.H);
    g.set(g.W - 2, g.H - 2, T_GOAL, C_GREEN, 0);
    if (d.random_start) place_agent(r, g, a, 0, 0, g.W, g.H);
    else { a.x = 1; a.y = 1; a.dir = 0; }
}

__device__ void gen_fourrooms(Pcg64 &r, GridL &g, Agent &a) {
    const int W = g.W, H = g.H;
    g.horz_wall(0, 0, W);
    g.horz_wall(0, H - 1, W);
    g.vert_wall(0, 0, H);
    g.vert_wall(W - 1, 0, H);
    const int rw = W / 2, rh = H / 2;
    for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 2; ++i) {
            const int xL = i * rw, yT = j * rh, xR = xL + rw, yB = yT + rh;
            if (i + 1 < 2) {
                g.vert_wall(xR, yT, rh);
                g.clear(xR, r.integers(yT + 1, yB));
            }
            if (j + 1 < 2) {
                g.horz_wall(xL, yB, rw);
                g.clear(r.integers(xL + 1, xR), yB);
            }
        }
    place_agent(r, g, a, 0, 0, W, H);
    int gx = 0, gy = 0;
    a.ok = a.ok && place_obj(r, g, a, 0, 0, W, H, gx, gy);
    g.set(gx, gy, T_GOAL, C_GREEN, 0);
}

__device__ void gen_crossing(Pcg64 &r, GridL &g, Agent &a, const mgdp_gen_desc &d) {
    const int W = g.W, H = g.H;
    g.wall_rect(0, 0, W, H);
    a.x = 1;
    a.y = 1;
    a.dir = 0;
    g.set(W - 2, H - 2, T_GOAL, C_GREEN, 0);
    // rivers = [(v, i) for i in range(2, H-2, 2)] + [(h, j) for j in range(2, W-2, 2)]; code = dir*64 + pos
    int rivers[32];
    int n = 0;
    for (int i = 2; i < H - 2; i += 2) rivers[n++] = 0 * 64 + i;
    for (int j = 2; j < W - 2; j += 2) rivers[n++] = 1 * 64 + j;
    for (int i = n - 1; i >= 1; --i) {
        const int j = r.interval(i);
        const int t = rivers[i]; rivers[i] = rivers[j]; rivers[j] = t;
    }
    const int nc = min(d.num_crossings, n);
    int rv[16], rh[16], nv = 0, nh = 0;
    for (int k = 0; k < nc; ++k) {
        if (rivers[k] < 64) rv[nv++] = rivers[k];
        else rh[nh++] = rivers[k] - 64;
    }
    auto sort = [](int *x, int m) {
        for (int i = 1; i < m; ++i)
            for (int j = i; j > 0 && x[j - 1] > x[j]; --j) { const int t = x[j]; x[j] = x[j - 1]; x[j - 1] = t; }
    };
    sort(rv, nv);
    sort(rh, nh);
    for (int i = 1; i < W - 1; ++i)
        for (int k = 0; k < nh; ++k) g.obstacle(i, rh[k], d.obstacle);
    for (int k = 0; k < nv; ++k)
        for (int j = 1; j < H - 1; ++j) g.obstacle(rv[k], j, d.obstacle);
    // path = [h] * len(rivers_v) + [v] * len(rivers_h), shuffled
    int path[32];
    int np = 0;
    for (int k = 0; k < nv; ++k) path[np++] = 1;  // h
    for (int k = 0; k < nh; ++k) path[np++] = 0;  // v
    for (int i = np - 1; i >= 1; --i) {
        const int j = r.interval(i);
        const int t = path[i]; path[i] = path[j]; path[j] = t;
    }
    int lv[18], lh[18];
    lv[0] = 0;
    for (int k = 0; k < nv; ++k) lv[k + 1] = rv[k];
    lv[nv + 1] = H - 1;
    lh[0] = 0;
    for (int k = 0; k < nh; ++k) lh[k + 1] = rh[k];
    lh[nh + 1] = W - 1;
    int ri = 0, rj = 0;
    for (int k = 0; k < np; ++k) {
        int i, j;
        if (path[k] == 1) {  // h
            i = lv[ri + 1];
            j = r.integers(lh[rj] + 1, lh[rj + 1]);  // choice(range(...))
            ++ri;
        } else {
            i = r.integers(lv[ri] + 1, lv[ri + 1]);
            j = lh[rj + 1];
            ++rj;
        }
        g.clear(i, j);
    }
}

__device__ void gen_doorkey(Pcg64 &r, GridL &g, Agent &a) {
    const int W = g.W, H = g.H;
    g.wall_rect(0, 0, W, H);
    g.set(W - 2, H - 2, T_GOAL, C_GREEN, 0);
    const int split = r.integers(2, W - 2);
    g.vert_wall(split, 0, H);
    place_agent(r, g, a, 0, 0, split, H);
    const int door = r.integers(1, W - 2);
    g.set(split, door, T_DOOR, C_YELLOW, D_LOCKED);
    int kx = 0, ky = 0;
    a.ok = a.ok && place_obj(r, g, a, 0, 0, split, H, kx, ky);
    g.set(kx, ky, T_KEY, C_YELLOW, 0);
}

__device__ void gen_lavagap(Pcg64 &r, GridL &g, Agent &a, const mgdp_gen_desc &d) {
    const int W = g.W, H = g.H;
    g.wall_rect(0, 0, W, H);
    a.x = 1;
    a.y = 1;
    a.dir = 0;
    g.set(W - 2, H - 2, T_GOAL, C_GREEN, 0);
    const int gx = r.integers(2, W - 2);
    const int gy = r.integers(1, H - 1);
    g.vert_wall(gx, 1, H - 2, d.obstacle);
    g.clear(gx, gy);
}

__device__ void gen_distshift(GridL &g, Agent &a, const mgdp_gen_desc &d) {
    const int W = g.W, H = g.H;
    g.wall_rect(0, 0, W, H);
    g.set(W - 2, 1, T_GOAL, C_GREEN, 0);
    for (int i = 0; i < W - 6; ++i) {
        g.set(3 + i, 1, T_LAVA, C_RED, 0);
        g.set(3 + i, d.strip2_row, T_LAVA, C_RED, 0);
    }
    a.x = 1;
    a.y = 1;
    a.dir = 0;
}

__global__ void __launch_bounds__(kGenBlock)
gen_grids_kernel(mgdp_gen_desc d, long long seed0, int B, uint8_t *__restrict__ enc, uint8_t *__restrict__ cells,
                 int32_t *__restrict__ agent) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int W = d.W, H = d.H, cellb = W * H * 3;
    const int rec = (cellb + 3) & ~3;  // per-thread LDS record, 4-B aligned
    const int b0 = blockIdx.x * kGenBlock;
    const int b = b0 + threadIdx.x;
    GridL g{smem + threadIdx.x * rec, W, H};
    if (b < B) {
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < H; ++y) g.clear(x, y);
        Pcg64 r((uint64_t)(seed0 + b));
        Agent a;
        switch (d.family) {
            case MGDP_GEN_EMPTY: gen_empty(r, g, a, d); break;
            case MGDP_GEN_FOURROOMS: gen_fourrooms(r, g, a); break;
            case MGDP_GEN_CROSSING: gen_crossing(r, g, a, d); break;
            case MGDP_GEN_DOORKEY: gen_doorkey(r, g, a); break;
            case MGDP_GEN_LAVAGAP: gen_lavagap(r, g, a, d); break;
            default: gen_distshift(g, a, d); break;
        }
        if (agent) {
            agent[b * 3 + 0] = a.ok ? a.x : -1;
            agent[b * 3 + 1] = a.ok ? a.y : -1;
            agent[b * 3 + 2] = a.ok ? a.dir : -1;
        }
    }
    __syncthreads();
    // coalesced write-out of the block's consecutive env records
    const int nb = min(kGenBlock, B - b0);
    if (enc) {
        const long long base = (long long)b0 * cellb;
        const int total = nb * cellb;
        if (rec == cellb && (total & 15) == 0 && (base & 15) == 0) {  // records are contiguous: 16-B copy
            const uint4 *s = reinterpret_cast<const uint4 *>(smem);
            uint4 *o = reinterpret_cast<uint4 *>(enc + base);
            for (int i = threadIdx.x; i < (total >> 4); i += kGenBlock) o[i] = s[i];
        } else {
            for (int i = threadIdx.x; i < total; i += kGenBlock) {
                const int e = i / cellb, o = i - e * cellb;
                enc[base + i] = smem[e * rec + o];
            }
        }
    }
    if (cells) {  // row-major type codes
        const long long base = (long long)b0 * W * H;
        const int total = nb * W * H;
        for (int i = threadIdx.x; i < total; i += kGenBlock) {
            const int e = i / (W * H), o = i - e * (W * H), y = o / W, x = o - y * W;
            cells[base + i] = smem[e * rec + (x * H + y) * 3];
        }
    }
}

int validate(const mgdp_gen_desc *d, int B) {
    MGDP_CHECK(d, MGDP_E_INVALID, "null descriptor");
    MGDP_CHECK(d->family >= MGDP_GEN_EMPTY && d->family <= MGDP_GEN_DISTSHIFT, MGDP_E_INVALID, "unknown family %d", d->family);
    MGDP_CHECK(B > 0, MGDP_E_INVALID, "B must be > 0");
    MGDP_CHECK(d->W >= 5 && d->H >= 5 && d->W <= 32 && d->H <= 32, MGDP_E_INVALID, "grid %dx%d outside 5..32", d->W, d->H);
    if (d->family == MGDP_GEN_CROSSING) {
        MGDP_CHECK(d->W % 2 == 1 && d->H % 2 == 1, MGDP_E_INVALID, "Crossing needs odd sizes (crossing.py:123)");
        MGDP_CHECK(d->obstacle == T_LAVA || d->obstacle == T_WALL, MGDP_E_INVALID, "obstacle must be lava or wall");
        MGDP_CHECK(d->num_crossings >= 0, MGDP_E_INVALID, "num_crossings must be >= 0");
    }
    if (d->family == MGDP_GEN_LAVAGAP)
        MGDP_CHECK(d->obstacle == T_LAVA || d->obstacle == T_WALL, MGDP_E_INVALID, "obstacle must be lava or wall");
    if (d->family == MGDP_GEN_FOURROOMS) MGDP_CHECK(d->W == 19 && d->H == 19, MGDP_E_INVALID, "FourRooms is 19x19");
    if (d->family == MGDP_GEN_DISTSHIFT)
        MGDP_CHECK(d->strip2_row > 0 && d->strip2_row < d->H - 1, MGDP_E_INVALID, "strip2_row out of the grid");
    return 0;
}

}  // namespace
}  // namespace mgdp

using namespace mgdp;

extern "C" {

int mgdp_gen_grids(const mgdp_gen_desc *desc, int32_t device, void *stream, int64_t seed0, int32_t B,
                   uint8_t *enc, uint8_t *cells, int32_t *agent) {
    if (int rc = validate(desc, B)) return rc;
    MGDP_CHECK(seed0 >= 0, MGDP_E_INVALID, "seeds must be >= 0");
    DeviceGuard guard(device);
    MGDP_CHECK(guard.ok, MGDP_E_HIP, "hipSetDevice(%d) failed", device);
    const int rec = (desc->W * desc->H * 3 + 3) & ~3;
    const int smem = rec * kGenBlock;
    if (smem > 64 * 1024) MGDP_HIP(hipFuncSetAttribute((const void *)gen_grids_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    hipLaunchKernelGGL(gen_grids_kernel, dim3((B + kGenBlock - 1) / kGenBlock), dim3(kGenBlock), smem,
                       (hipStream_t)stream, *desc, (long long)seed0, B, enc, cells, agent);
    MGDP_HIP(hipGetLastError());
    return 0;
}

int mgdp_gen_grids_host(const mgdp_gen_desc *desc, int32_t device, int64_t seed0, int32_t B, uint8_t *enc,
                        uint8_t *cells, int32_t *agent) {
    if (int rc = validate(desc, B)) return rc;
    DeviceGuard guard(device);
    MGDP_CHECK(guard.ok, MGDP_E_HIP, "hipSetDevice(%d) failed", device);
    const size_t ne = (size_t)B * desc->W * desc->H * 3, nc = (size_t)B * desc->W * desc->H, na = (size_t)B * 3;
    uint8_t *de = nullptr, *dc = nullptr;
    int32_t *da = nullptr;
    hipError_t e = hipSuccess;
    if (enc) e = hipMalloc(&de, ne);
    if (e == hipSuccess && cells) e = hipMalloc(&dc, nc);
    if (e == hipSuccess && agent) e = hipMalloc(&da, na * sizeof(int32_t));
    int rc = e == hipSuccess ? 0 : hip_fail(e, "mgdp_gen_grids_host allocation", __FILE__, __LINE__);
    if (!rc) rc = mgdp_gen_grids(desc, device, nullptr, seed0, B, de, dc, da);
    if (!rc && enc && (e = hipMemcpy(enc, de, ne, hipMemcpyDeviceToHost)) != hipSuccess) rc = hip_fail(e, "copy enc", __FILE__, __LINE__);
    if (!rc && cells && (e = hipMemcpy(cells, dc, nc, hipMemcpyDeviceToHost)) != hipSuccess) rc = hip_fail(e, "copy cells", __FILE__, __LINE__);
    if (!rc && agent && (e = hipMemcpy(agent, da, na * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
        rc = hip_fail(e, "copy agent", __FILE__, __LINE__);
    if (!rc) {
        e = hipDeviceSynchronize();
        if (e != hipSuccess) rc = hip_fail(e, "mgdp_gen_grids_host", __FILE__, __LINE__);
    }
    (void)hipFree(de);
    (void)hipFree(dc);
    (void)hipFree(da);
    if (!rc && agent)
        for (size_t i = 0; i < (size_t)B; ++i)
            MGDP_CHECK(agent[i * 3 + 2] >= 0, MGDP_E_INVALID, "env %zu: rejection sampling hit its cap", i);
    return rc;
}

}  // extern "C"
