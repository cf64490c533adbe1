// Latency floor of one lone-grid sweep's LDS/barrier chain on one workgroup (MI355X).
// Build: hipcc -O3 -ffp-contract=off -Xarch_device -fno-honor-nans -Xarch_device -fno-slp-vectorize --offload-arch=gfx950 -o tools/probe_sweep_chain tools/probe_sweep_chain.hip
// Each variant runs ITERS iterations of a loop body shaped like one sweep of the served
// 4-wave solver (fused_fast_xyd_soa) and reports shader cycles (s_memtime) per iteration:
//   0 barrier only
//   1 one ds_write_b32, lgkmcnt(0), barrier, one dependent ds_read_b32
//   2 four ds_write_b32 + flag byte, barrier, four ds_read_b32 + 16-B flag read (the served loop)
//   3 as 2 plus the served loop's VALU (one-multiply backup, |dV| max, flag test)
//   4 as 3 with the east/west fronts from DPP row rotates: two writes, two reads + flag
//   5 as 3 without the stop test (no flag write/read)
//   6 as 4 without the stop test
//   7 as 3 with a constant flag byte (no ballot: the write does not wait for |dV|)
//   8 as 3 without the flag read and test (the ballot and flag write kept)
//   9 as 3 with the flags read as one dword (4 waves: 4 bytes) instead of 16 bytes
//  10 as 9, flag byte cleared by lane 0 at the sweep's start and set by every lane whose |dV| >= tol
//  11 as 9, flag byte cleared at the sweep's start, set by lane 0 under a branch on the wave's vcc
//  12 as 11 with the DPP east/west fronts
//  13 as 9 with the flag of sweep k written after barrier k (at sweep k+1's start, from the ballot
//     kept in a register) and read at sweep k+2's start: the write waits for nothing
//  14 as 13 with the DPP east/west fronts
//  15 TWO sweeps per barrier (round 6): 4 planes written per pair, the N/S fronts of the pair's second
//     sweep from the first sweep's lanes +-16 by ds_bpermute (one halo value per boundary lane from
//     3 extra LDS reads), both sweeps' ballots in one flag byte; clock64 per PAIR / 2 reported
//  16 as 15 with the +-16 lane shifts by v_permlane16_swap / v_permlane32_swap (VALU, no LDS)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

constexpr int ITERS = 4096;

__device__ __forceinline__ float dpp_row_shr1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_row_shl1(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x101, 0xf, 0xf, false));
}

// lane l <- lane l + 16 (rows 0..2 of the wave's four 16-lane rows; row 3 takes `edge`)
__device__ __forceinline__ float shift_up16_pl(float x, float edge, int row) {
    const unsigned int u = __float_as_uint(x);
    auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);   // r[0] = (X0,X0,X2,X2), r[1] = (X1,X1,X3,X3)
    auto q = __builtin_amdgcn_permlane32_swap(r[0], r[0], false, false);  // q[1] = (X2,X2,X2,X2)
    const float b = __uint_as_float(r[1]), x2 = __uint_as_float(q[1]);
    return row == 3 ? edge : (row == 1 ? x2 : b);
}
// lane l <- lane l - 16 (rows 1..3; row 0 takes `edge`)
__device__ __forceinline__ float shift_down16_pl(float x, float edge, int row) {
    const unsigned int u = __float_as_uint(x);
    auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);   // r[0] = (Y0,Y0,Y2,Y2), r[1] = (Y1,Y1,Y3,Y3)
    auto q = __builtin_amdgcn_permlane32_swap(r[1], r[1], false, false);  // q[0] = (Y1,Y1,Y1,Y1)
    const float a = __uint_as_float(r[0]), y1 = __uint_as_float(q[0]);
    return row == 0 ? edge : (row == 2 ? y1 : a);
}

template <int V>
__global__ __launch_bounds__(256) void chain(float *out, long long *cyc, float g, float tol) {
    __shared__ float tiles[2][4 * 256];
    __shared__ unsigned char flags[32];
    const int c = threadIdx.x;
    for (int i = c; i < 4 * 256; i += 256) tiles[0][i] = tiles[1][i] = 0.0f;
    if (c < 32) flags[c] = 1;
    __syncthreads();
    float own[4] = {0.f, 0.f, 0.f, 0.f};
    const bool goal = c == 200;
    const int nb[4] = {(c + 1) & 255, 256 + ((c + 16) & 255), 512 + ((c + 255) & 255), 768 + ((c + 240) & 255)};
    int parity = 0;
    unsigned char late = 1;
    bool more = true;
    const long long t0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (V == 15 || V == 16) {
            if (it & 1) continue;  // one pair per two iterations
            const float *tin = tiles[parity];
            float *tout = tiles[parity ^ 1];
            const int lane = c & 63, row = lane >> 4;
            const unsigned int fl = *reinterpret_cast<const unsigned int *>(flags + (parity ^ 1) * 16);
            const float fS = tin[nb[1]], fN = tin[nb[3]];
            const bool bottom = row == 3;
            const int hc = bottom ? (c + 16) & 255 : (c + 240) & 255;
            const float h0 = tin[hc], h2 = tin[512 + hc];
            const float hf = bottom ? tin[256 + ((hc + 16) & 255)] : tin[768 + ((hc + 240) & 255)];
            const float hs = bottom ? fS : fN;
            float o[4], dm1 = 0.f;
            {
                const float f[4] = {dpp_row_shl1(own[0]), fS, dpp_row_shr1(own[2]), fN};
                const float a = fmaxf(own[0], own[2]), b = fmaxf(own[1], own[3]);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const float m = fmaxf(fmaxf((d & 1) ? a : b, own[d]), f[d]);
                    o[d] = fmaxf(g * m, goal ? 1.0f : 0.0f);
                    dm1 = fmaxf(dm1, fabsf(o[d] - own[d]));
                }
            }
            const float hv = fmaxf(g * fmaxf(fmaxf(h0, h2), fmaxf(hs, hf)), goal ? 1.0f : 0.0f);
            float S2, N2;
            if constexpr (V == 15) {
                S2 = bottom ? hv : __int_as_float(__builtin_amdgcn_ds_bpermute(((c + 16) & 63) * 4, __float_as_int(o[1])));
                N2 = row == 0 ? hv : __int_as_float(__builtin_amdgcn_ds_bpermute(((c + 48) & 63) * 4, __float_as_int(o[3])));
            } else {
                S2 = shift_up16_pl(o[1], hv, row);
                N2 = shift_down16_pl(o[3], hv, row);
            }
            float o2[4], dm2 = 0.f;
            {
                const float f[4] = {dpp_row_shl1(o[0]), S2, dpp_row_shr1(o[2]), N2};
                const float a = fmaxf(o[0], o[2]), b = fmaxf(o[1], o[3]);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const float m = fmaxf(fmaxf((d & 1) ? a : b, o[d]), f[d]);
                    o2[d] = fmaxf(g * m, goal ? 1.0f : 0.0f);
                    dm2 = fmaxf(dm2, fabsf(o2[d] - o[d]));
                }
            }
            if (it > 0 && fl == 0u) more = false;
#pragma unroll
            for (int d = 0; d < 4; ++d) tout[d * 256 + c] = o2[d];
            const unsigned int bits = (__ballot(dm1 >= tol) != 0ull ? 1u : 0u) | (__ballot(dm2 >= tol) != 0ull ? 2u : 0u);
            if ((c & 63) == 0) flags[parity * 16 + (c >> 6)] = bits;
#pragma unroll
            for (int d = 0; d < 4; ++d) own[d] = o2[d];
            parity ^= 1;
            __syncthreads();
        } else if constexpr (V == 0) {
            __syncthreads();
        } else if constexpr (V == 1) {
            tiles[it & 1][c] = own[0];
            __syncthreads();
            own[0] = tiles[it & 1][(c + 1) & 255] + 1.0f;
        } else {
            constexpr bool DPP = V == 4 || V == 6 || V == 12 || V == 14;
            constexpr bool CLR = V >= 10 && V <= 12;
            constexpr bool LATE = V >= 13;
            constexpr bool TEST = V != 5 && V != 6;
            constexpr bool READ = TEST && V != 8;
            const float *tin = tiles[parity];
            float *tout = tiles[parity ^ 1];
            float f[4];
            unsigned int fl = 1;
            if (READ) {
                if (V >= 9) {
                    fl = *reinterpret_cast<const unsigned int *>(flags + (parity ^ 1) * 16);
                } else {
                    const uint4 x = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
                    fl = x.x | x.y | x.z | x.w;
                }
            }
            if (CLR && (c & 63) == 0) flags[parity * 16 + (c >> 6)] = 0;
            if (LATE && (c & 63) == 0) flags[parity * 16 + (c >> 6)] = late;
            if (DPP) {
                f[0] = dpp_row_shl1(own[0]);
                f[2] = dpp_row_shr1(own[2]);
                f[1] = tin[nb[1]];
                f[3] = tin[nb[3]];
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) f[d] = tin[nb[d]];
            }
            float o[4], dm = 0.f;
            if constexpr (V == 2) {
#pragma unroll
                for (int d = 0; d < 4; ++d) o[d] = f[d];
                dm = o[0];
            } else {
                const float a = fmaxf(own[0], own[2]), b = fmaxf(own[1], own[3]);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const float m = fmaxf(fmaxf((d & 1) ? a : b, own[d]), f[d]);
                    o[d] = fmaxf(g * m, goal ? 1.0f : 0.0f);
                    dm = fmaxf(dm, fabsf(o[d] - own[d]));
                }
            }
            if (READ && it > 0 && fl == 0u) more = false;
            if (DPP) {
                tout[256 + c] = o[1];
                tout[768 + c] = o[3];
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) tout[d * 256 + c] = o[d];
            }
            if (LATE) {
                late = __ballot(dm >= tol) != 0ull ? 1 : 0;
            } else if (TEST) {
                if constexpr (V == 10) {
                    if (dm >= tol) flags[parity * 16 + (c >> 6)] = 1;
                } else if constexpr (V >= 11) {
                    if (__ballot(dm >= tol) != 0ull && (c & 63) == 0) flags[parity * 16 + (c >> 6)] = 1;
                } else {
                    const bool any = V == 7 ? true : __ballot(dm >= tol) != 0ull;
                    if ((c & 63) == 0) flags[parity * 16 + (c >> 6)] = any ? 1 : 0;
                }
            }
#pragma unroll
            for (int d = 0; d < 4; ++d) own[d] = o[d];
            parity ^= 1;
            __syncthreads();
        }
    }
    const long long t1 = clock64(), r1 = wall_clock64();
    out[c] = own[0] + own[1] + own[2] + own[3] + (more ? 0.f : 1.f);
    if (c == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r1 - r0;
    }
}

template <int V>
void run(float *d_out, long long *d_cyc) {
    chain<V><<<1, 256>>>(d_out, d_cyc, 0.99f, 1e-6f);  // warm
    CHECK(hipDeviceSynchronize());
    long long best = -1, rt = 0;
    for (int r = 0; r < 5; ++r) {
        chain<V><<<1, 256>>>(d_out, d_cyc, 0.99f, 1e-6f);
        CHECK(hipDeviceSynchronize());
        long long c[2];
        CHECK(hipMemcpy(c, d_cyc, sizeof c, hipMemcpyDeviceToHost));
        if (best < 0 || c[0] < best) {
            best = c[0];
            rt = c[1];
        }
    }
    // wall_clock64 runs at 100 MHz
    std::printf("{\"variant\": %d, \"clock64_per_iter\": %.1f, \"ns_per_iter\": %.2f}\n", V, (double)best / ITERS,
                (double)rt * 10.0 / ITERS);
}

int main() {
    float *d_out;
    long long *d_cyc;
    CHECK(hipMalloc(&d_out, 256 * sizeof(float)));
    CHECK(hipMalloc(&d_cyc, 2 * sizeof(long long)));
    run<0>(d_out, d_cyc);
    run<1>(d_out, d_cyc);
    run<2>(d_out, d_cyc);
    run<3>(d_out, d_cyc);
    run<4>(d_out, d_cyc);
    run<5>(d_out, d_cyc);
    run<6>(d_out, d_cyc);
    run<7>(d_out, d_cyc);
    run<8>(d_out, d_cyc);
    run<9>(d_out, d_cyc);
    run<10>(d_out, d_cyc);
    run<11>(d_out, d_cyc);
    run<12>(d_out, d_cyc);
    run<13>(d_out, d_cyc);
    run<14>(d_out, d_cyc);
    run<15>(d_out, d_cyc);
    run<16>(d_out, d_cyc);
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_cyc));
    return 0;
}
