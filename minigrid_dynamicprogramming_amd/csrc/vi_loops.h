// vi_loops.h -- the sweep loops of one workgroup: (state, action) lanes, LDS staging,
// the fused direction-major loops, the two-sweep and four-threads-per-cell XYD loops, the launch
// reduction and host publication.
// Part of the single translation unit vi.hip (included in order: vi_model.h, vi_loops.h,
// vi_kernels.h); see vi.hip for the DP semantics and the data layout.
#pragma once

// MGDP_RUNTO_DV_ALL=1 (A/B builds): k_target loops compute |dV| on every sweep, not only the last.
// MGDP_DK_DEAD=0 (A/B builds): batched DoorKey waves of absorbing cells only do the full sweep.
#ifndef MGDP_DK_DEAD
#define MGDP_DK_DEAD 1
#endif
#ifndef MGDP_RUNTO_DV_ALL
#define MGDP_RUNTO_DV_ALL 0
#endif

namespace mgdp {
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
// The same copy with nontemporal HBM accesses, for V streamed once per launch (HBM -> LDS loads,
// LDS -> HBM stores): the lines are not kept in L2/MALL for a re-read that never comes.
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void copy16_nt_in(void *dst, const void *src, int bytes) {
    const u32x4_nt *s = reinterpret_cast<const u32x4_nt *>(src);
    u32x4_nt *d = reinterpret_cast<u32x4_nt *>(dst);
    for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) d[i] = __builtin_nontemporal_load(s + i);
}
__device__ __forceinline__ void copy16_nt_out(void *dst, const void *src, int bytes) {
    const u32x4_nt *s = reinterpret_cast<const u32x4_nt *>(src);
    u32x4_nt *d = reinterpret_cast<u32x4_nt *>(dst);
    for (int i = threadIdx.x; i < (bytes >> 4); i += blockDim.x) __builtin_nontemporal_store(s[i], d + i);
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
    if (epoch == 0) {
        // a device buffer (the multi-GPU protocol's / the chained solve's): raw {kmax, dV bits, kmin,
        // 0}, read by stream-ordered launches and collectives only
        __hip_atomic_store(host_out + 0, km, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(host_out + 1, dv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(host_out + 2, kn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(host_out + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // The host-mapped words: four 8-byte words, each tagged with the launch epoch in its high half
    // ({kmax}, {dV bits 63..32}, {dV bits 31..0}, {kmin}), so they may land in any order and need
    // no drain between them -- one PCIe write latency to the host instead of two (round 4 stored
    // the values, drained them, then the epoch word).  The host waits until all four carry its
    // epoch.  No L2 write-back (release) is needed: V and pi are consumed only by later
    // stream-ordered operations.
    const unsigned long long tag = (unsigned long long)epoch << 32;
    __hip_atomic_store(host_out + 0, tag | (km & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 1, tag | (dv >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 2, tag | (dv & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host_out + 3, tag | (kn & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A 64-bit value for the host as two epoch-tagged words (the run_to mirror of the protocol's E)
__device__ __forceinline__ void publish_word2(unsigned long long *w, unsigned long long v, unsigned int epoch) {
    const unsigned long long tag = (unsigned long long)epoch << 32;
    __hip_atomic_store(w + 0, tag | (v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(w + 1, tag | (v & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// A grid's exit stores (its V row and pi words), `wt`: written through the XCD L2 (agent-scope
// relaxed stores: sc1).  Plain stores leave the batch's V / pi dirty in the L2s, and the launch's
// end-of-kernel release writes them back after its last wave (MI355X_MICROARCH.md, boundary row:
// + bytes / 6 TB/s); written through, they reach memory while the other grids still sweep.  Measured
// (profiles/r05_wt/): a resident batch's kernel 1-2 % shorter (FourRooms x 4096 45.0 -> 44.0 us,
// LavaS11N5 x 8192 27.5 -> 27.1), a batch past residency 6 % longer (the waves queued behind the
// write-through stores): fused_wave2_xyd writes through in the launches with the in-launch reduction
// (resident batches), its own instantiation.  MGDP_WT_EXIT=0 (A/B builds): never.
#ifndef MGDP_WT_EXIT
#define MGDP_WT_EXIT 1
#endif
template <typename T>
__device__ __forceinline__ void store_v4_exit(T *p, const V4<T> &v, bool wt) {
    if (MGDP_WT_EXIT && wt) {
        unsigned long long *q = reinterpret_cast<unsigned long long *>(p);
        if constexpr (sizeof(T) == 4) {
            // one 16-B store, as the plain form (two 8-B atomic stores re-paired the loop's registers:
            // +5 VALU per two sweeps at P = 2); its vmcnt is not tracked by the compiler, which only
            // makes a later wait of its own more conservative (vector memory returns in order).
            // The s_nop 1 INSIDE the string is the store-data hazard's wait states: the compiler does not
            // pad an asm store, and its next VALU may overwrite the data registers before a store of more
            // than 8 bytes has read them (cdna_hip_programming.md §5.7; found in round 6, where the batch
            // server's multi-grid loop reused them at once: the first dword of 4-lane groups stored stale)
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v x = {v.v[0], v.v[1], v.v[2], v.v[3]};
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
        } else {
#pragma unroll
            for (int d = 0; d < 4; ++d)
                __hip_atomic_store(q + d, (unsigned long long)__double_as_longlong(v.v[d]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        *reinterpret_cast<V4<T> *>(p) = v;
    }
}
__device__ __forceinline__ void store_pi_exit(int8_t *p, uint32_t pk, bool wt) {
    if (MGDP_WT_EXIT && wt)
        __hip_atomic_store(reinterpret_cast<uint32_t *>(p), pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *reinterpret_cast<uint32_t *>(p) = pk;
}

__device__ __forceinline__ void fused_reduce(unsigned long long *red, unsigned int *ticket,
                                             unsigned long long *host_out, int k, double dvl,
                                             unsigned int *lds_flag, unsigned int epoch, bool published, int tid) {
    if (gridDim.x == 1) {  // a lone grid publishes directly (early, if it swept: see `done`)
        if (tid == 0 && !published)
            publish(host_out, (unsigned long long)k, (unsigned long long)__double_as_longlong(dvl),
                    (unsigned long long)k, epoch);
        return;
    }
    if (tid == 0) {
        unsigned long long *r = red + (blockIdx.x & (kRedShards - 1)) * 4;
        const unsigned long long a = __hip_atomic_fetch_max(r + 0, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_fetch_max(r + 1, (unsigned long long)__double_as_longlong(dvl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long c = __hip_atomic_fetch_min(r + 2, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" :: "v"(a), "v"(b), "v"(c) : "memory");
        const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = t == gridDim.x - 1;
    }
    __syncthreads();
    if (*lds_flag && tid < 64) {
        unsigned long long *r = red + tid * 4;
        unsigned long long km = __hip_atomic_exchange(r + 0, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long dv = __hip_atomic_exchange(r + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long kn = __hip_atomic_exchange(r + 2, 0x7fffffffull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            km = max(km, (unsigned long long)__shfl_xor(km, o));
            dv = max(dv, (unsigned long long)__shfl_xor(dv, o));
            kn = min(kn, (unsigned long long)__shfl_xor(kn, o));
        }
        if (tid == 0) {
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
                                                   long long pit_stride = 0, const XydTopo<T> *pre = nullptr) {
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;  // idle threads shadow cell 0 and never write
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs;  // LDS stride: every thread (idle ones too) owns a slot, so LDS writes need no mask
    const int k_start = k;
    // pre: the topology the persistent server resolved once per residency (cells cannot change)
    const XydTopo<T> tp = pre ? *pre : xyd_topo_soa<T, ND>(cl, geo, cc);
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
    // The stop test of the previous sweep (LOCAL) is read before this sweep's neighbour values
    // (LDS returns in order) but consulted only after this sweep's arithmetic, so it is off the
    // critical path; a sweep past the stopping point computes into the register set the caller
    // discards and writes nothing.
    auto sweep = [&](const T *Vin, T *Vout, const V4<T> &in, V4<T> &out) -> bool {
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);  // the previous sweep's flags (all 16 bytes: no branch on the wave count)
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        T nbv[4];
        xyd_load_nb(tp, Vin, nbv);
        uint32_t pk;
        const T rg = HMODE ? rgoal[k_target - 1 - k] : (T)1;
        T d;
        if (HMODE == 2) {
            d = xyd_step<T, SLIP, true, ND, true>(tp, cf, in, nbv, out, pk, rg);
            if (own_cell) *reinterpret_cast<uint32_t *>(pit + (long long)(k_target - 1 - k) * pit_stride + c * 4) = pk;
        } else {
            d = xyd_step<T, SLIP, false, ND, HMODE != 0>(tp, cf, in, nbv, out, pk, rg);
        }
        if (LOCAL) {
            asm volatile("" ::"v"(d));  // keep the arithmetic ahead of the test (no sinking past it)
            if (k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        }
        diff = d;
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

// The served lone deterministic XYD grid (vi_serve_kernel, WP = kWpServeEw): fused_fast_xyd_soa's
// sweep with a shorter per-sweep chain for a latency-bound workgroup of <= 4 waves.
//  * East / west fronts by DPP: cell c +- 1 is lane +- 1 of the same wave (wave_shl / wave_shr,
//    0 shifted in at the wave's ends), so only planes 1 and 3 (south / north fronts) go through
//    LDS: two ds_write and two ds_read per sweep instead of four each.  Fronts are geometric, as in
//    fused_wave2_xyd: a front the agent cannot enter is an invalid state holding +0, and V >= +0,
//    so max(., +0) is the identity and no per-direction select is needed.  The shifted-in 0 is
//    exact unless a wave's first or last cell is valid AND its west / east neighbour (another
//    wave's) is valid too: the caller checks that once per grid (serve_ew_ok) and otherwise runs
//    fused_fast_xyd_soa.
//  * The previous sweep's stop flags are one dword (<= 4 waves), no OR chain.
//  * Three register sets rotate (unrolled by 6 with the two LDS tiles), so the sweep the rule stops
//    leaves V_{k-1} intact in registers: the pi pass takes its own values there, its east / west
//    fronts by the same DPP shifts and its north / south fronts from the V_{k-1} tile.
// Same backups (one-multiply form), same rule and the same per-action pi pass as fused_fast_xyd_soa:
// bit-identical V, pi, sweep count and dV.  LDS: each tile = [pad][plane 1][pad][plane 3][pad]
// (serve_ew_tile_elems), carved from the two V buffers of the usual layout.
__host__ __device__ inline int serve_ew_padw(int W) { return (W + 15) / 16 * 16; }
__host__ __device__ inline int serve_ew_tile_elems(int HWs, int W) { return 2 * HWs + 3 * serve_ew_padw(W); }

template <typename T>
__device__ __forceinline__ T dpp_shl1_zero(T v) {  // lane i <- lane i+1; lane 63 <- +0
    if constexpr (sizeof(T) == 4) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, true));
    } else {
        const long long b = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xF, 0xF, true);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xF, 0xF, true);
        return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
}
template <typename T>
__device__ __forceinline__ T dpp_shr1_zero(T v) {  // lane i <- lane i-1; lane 0 <- +0
    if constexpr (sizeof(T) == 4) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, true));
    } else {
        const long long b = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, true);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xF, 0xF, true);
        return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
}

// Whole workgroup (uniform result): may the grid run fused_serve_xyd?  Every wave's first / last
// cell must not have a valid west / east neighbour in another wave (see above).  `word`: an LDS
// int the call may use.
__device__ __forceinline__ bool serve_ew_ok(const uint8_t *cl, const Geo &geo, int *word) {
    const int c = threadIdx.x, lane = c & 63;
    bool bad = false;
    if (c < geo.HW && xyd_free(cl[c])) {
        if (lane == 63 && c + 1 < geo.HW && xyd_free(cl[c + 1])) bad = true;
        if (lane == 0 && c > 0 && xyd_free(cl[c - 1])) bad = true;
    }
    if (threadIdx.x == 0) *word = 0;
    __syncthreads();
    if (bad) *word = 1;
    __syncthreads();
    const bool ok = *word == 0;
    __syncthreads();
    return ok;
}

// zero_tiles: clear both tiles first (the pads must hold +0); the server does it once per grid, as
// nothing else writes the pads while the grid stays (a solve rewrites tile 0's planes only).
template <typename T, typename Done>
__device__ __forceinline__ void fused_serve_xyd(const Geo &geo, const Coef<T> &cf, T *T0, T *T1, T *slots,
                                                uint8_t *flags, const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                double &dvl, const Done &done, const XydTopo<T> &tp,
                                                bool zero_tiles) {
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs, W = geo.W, padw = serve_ew_padw(W);
    const T ge = tp.valid ? cf.g : (T)0;
    // plane 1 (V of direction 1) of cell x at tile[padw + x], plane 3 at tile[2 * padw + HW + x]
    const int o1 = padw + c, o3 = 2 * padw + HW + c;
    T A[4], B[4], C[4];
    {
        V4<T> x = V4<T>{{(T)0, (T)0, (T)0, (T)0}};
        if (k != 0) x = *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) A[d] = own_cell ? x.v[d] : (T)0;
    }
    if (zero_tiles) {
        const int te = serve_ew_tile_elems(HW, W);
        for (int i = c; i < te; i += blockDim.x) {  // pads (and planes) of both tiles start at +0
            T0[i] = (T)0;
            T1[i] = (T)0;
        }
        __syncthreads();
    }
    B[0] = B[1] = B[2] = B[3] = (T)0;
    C[0] = C[1] = C[2] = C[3] = (T)0;
    T0[o1] = A[1];
    T0[o3] = A[3];
    __syncthreads();
    T diff = (T)0;
    // par: this sweep's flag parity, a constant at each unrolled call (the flag addresses fold to
    // immediate offsets); a sweep at loop position p has parity p & 1
    uint8_t *const fwave = flags + (threadIdx.x >> 6);
    const bool lane0 = (threadIdx.x & 63) == 0;
    // test: whether this sweep consults the previous sweep's flags (all but the first: the first is
    // peeled off the loop, so no sweep of the loop tests k > k_start)
    // cap: whether this sweep checks max_sweeps (every sweep does: a second, unchecked copy of the
    // six unrolled sweeps for blocks with six to spare measured 8.2 vs 5.6 us per solve -- the
    // server's code then overflows the instruction cache)
    auto sweep = [&](const T *Vin, T *Vout, const T (&in)[4], T (&out)[4], const int par, auto test, auto cap) -> bool {
        if (decltype(cap)::value && k >= geo.max_sweeps) return false;
        const uint32_t fl = *reinterpret_cast<const uint32_t *>(flags + (par ^ 1) * 16);
        const T fS = Vin[o1 + W], fN = Vin[o3 - W];
        const T fE = dpp_shl1_zero(in[0]), fW = dpp_shr1_zero(in[2]);
        const T m02 = vmax(in[0], in[2]), m13 = vmax(in[1], in[3]);
        const T m[4] = {vmax(vmax(in[0], m13), fE), vmax(vmax(in[1], m02), fS), vmax(vmax(in[2], m13), fW),
                        vmax(vmax(in[3], m02), fN)};
        T dm = (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            out[d] = vmax(ge * m[d], tp.tq[d]);
            dm = vmax(dm, vabs(out[d] - in[d]));
        }
        asm volatile("" ::"v"(dm));  // keep the arithmetic ahead of the test (no sinking past it)
        if (decltype(test)::value && fl == 0u) return false;
        diff = dm;
        Vout[o1] = out[1];
        Vout[o3] = out[3];
        const bool any = __ballot(dm >= cf.tol) != 0ull;
        if (lane0) fwave[par * 16] = any;
        __syncthreads();
        ++k;
        return true;
    };
    // on the stopping sweep: which register set holds V_k (`pos`: the set the stopped sweep read)
    int pos;
    using Yes = std::integral_constant<bool, true>;
    using No = std::integral_constant<bool, false>;
    // k_start's sweep has no previous sweep to test (a resumed solve's first one included)
    if (!sweep(T0, T1, A, B, 0, No{}, Yes{})) {
        pos = 0;
    } else {
        while (true) {
            if (!sweep(T1, T0, B, C, 1, Yes{}, Yes{})) { pos = 1; break; }
            if (!sweep(T0, T1, C, A, 0, Yes{}, Yes{})) { pos = 2; break; }
            if (!sweep(T1, T0, A, B, 1, Yes{}, Yes{})) { pos = 3; break; }
            if (!sweep(T0, T1, B, C, 0, Yes{}, Yes{})) { pos = 4; break; }
            if (!sweep(T1, T0, C, A, 1, Yes{}, Yes{})) { pos = 5; break; }
            if (!sweep(T0, T1, A, B, 0, Yes{}, Yes{})) { pos = 0; break; }
        }
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    // V_k = the stopped sweep's input set, V_{k-1} = the set before it (element selects: a pointer
    // to one of the sets would put them in scratch); the V_{k-1} tile = the stopped sweep's output
    // tile (positions 0, 2, 4 write T1)
    const int sk = pos % 3, sp = (pos + 2) % 3;
    T vk[4], vp[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        vk[d] = sk == 0 ? A[d] : (sk == 1 ? B[d] : C[d]);
        vp[d] = sp == 0 ? A[d] : (sp == 1 ? B[d] : C[d]);
    }
    const T *Tp = (pos & 1) ? T0 : T1;
    const T pE = dpp_shl1_zero(vp[0]), pW = dpp_shr1_zero(vp[2]);
    if (own_cell) {
        // forward reads the front state when the agent can enter it, else its own (xyd_step's nbv)
        const T geo_f[4] = {pE, Tp[o1 + W], pW, Tp[o3 - W]};
        T nbv[4];
        V4<T> op;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            op.v[d] = vp[d];
            const bool enter = tp.nbi[d] != d * HW + c;
            nbv[d] = enter ? geo_f[d] : vp[d];
        }
        V4<T> tmp;
        uint32_t pk;
        xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
        *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
        *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = V4<T>{{vk[0], vk[1], vk[2], vk[3]}};
    }
}

// The served lone deterministic XYD grid, TWO sweeps per workgroup barrier (vi_serve_kernel,
// WP = kWpServePair; grids on <= 4 waves whose wave edges pass serve_ew_ok).  Round 6.  A lone grid's
// sweep is latency-bound: its LDS write -> s_barrier -> LDS read round trip and the stop test's
// ballot / flag byte around it cost more than the arithmetic (tools/probe_sweep_chain.hip,
// profiles/r06_dist/: 449 cycles per sweep with the round trip, 289 without the stop test).  Here a
// workgroup barrier closes every second sweep:
//  * The pair reads V_k from the input tile (all four planes are kept in LDS): its own cell's north /
//    south fronts as fused_serve_xyd, and the values its NEIGHBOURS' sweep k+1 needs for the two
//    planes this cell's sweep k+2 reads: plane 1 of cell c + W (planes 0, 1, 2 there and plane 1 of
//    c + 2W) and plane 3 of cell c - W (planes 0, 2, 3 there and plane 3 of c - 2W).  So each lane
//    computes sweep k+1 of its own cell (fused_serve_xyd's arithmetic) and those two neighbour values
//    (the same max of the same four V_k values, the same multiply and goal select as their owners:
//    bit-identical), and sweep k+2 needs nothing from another lane but its east / west fronts, by
//    DPP as in fused_serve_xyd: no cross-wave (or cross-lane LDS) exchange inside the pair.
//  * Sweep k+2 then writes its four planes; each wave's two ballots (|dV| >= tol of sweeps k+1 and
//    k+2, a bit also 0 at the max_sweeps cap) go into one flag byte, and the barrier closes the pair.
//  * The next pair tests both bits behind its first sweep's arithmetic (the flag dword travels with
//    the data reads; that sweep writes only the set that held V_{k-2}; testing before it measured
//    slower: the test's scalar chain then sits in front of every pair's VALU work): stop after sweep
//    k-1 (V_{k-1} = the last pair's middle set, pi from V_{k-2}: the last pair's input tile, all four
//    planes, untouched) or after sweep k (V_k = its output set, pi from the middle set, whose north /
//    south fronts are the last pair's two neighbour values).  So the rule, the cap (a pair may
//    compute past it: discarded), the reported dV (the block max of the stopping sweep's |dV|) and
//    pi (argmax on V_{K-1}, lowest index on ties) are fused_serve_xyd's, bit for bit.
//  * The solve's first call computes one sweep (its first half is the identity), so the pairs cover
//    sweeps (k_start + 2, k_start + 3), ...: a stop on a pair's second sweep costs the next pair's
//    first-sweep arithmetic only, a stop on its first sweep that and the pair's second sweep
//    (Empty-16's 29 sweeps from 0 end on a second sweep).
//  * Three register sets rotate (in, middle, out) with the two tiles: the loop is unrolled by six
//    pairs.  LDS: two tiles of four planes, each [pad][HWs cells][pad], pad = round_up(2W, 16), the
//    host sizes the V buffers for them (serve_pair_tile_elems).
// Requires k < max_sweeps on entry (fused_grid only calls with work to do).
__host__ __device__ inline int serve_pair_pad(int W) { return (2 * W + 15) / 16 * 16; }
__host__ __device__ inline int serve_pair_plane(int HWs, int W) { return HWs + 2 * serve_pair_pad(W); }
__host__ __device__ inline int serve_pair_tile_elems(int HWs, int W) { return 4 * serve_pair_plane(HWs, W); }

// The pair loop's neighbour topology of thread t (resolved once per grid by the server): bit 0 the
// cell t + W is walkable, bit 1 a goal lies south of it (its plane 1 is then max(., 1)); bits 2 / 3
// the same for t - W and north.  Cells outside the grid: 0 (their value is +0, the geometric front).
__device__ __forceinline__ uint32_t serve_pair_halo(const uint8_t *cl, const Geo &geo, int t) {
    const int W = geo.W;
    uint32_t h = 0;
    const int s = t + W, n = t - W;  // a walkable cell is interior: its own fronts are in the grid
    if (t < geo.HW && s < geo.HW && xyd_free(cl[s])) h |= 1u | (cl[s + W] == T_GOAL ? 2u : 0u);
    if (t < geo.HW && n >= 0 && xyd_free(cl[n])) h |= 4u | (cl[n - W] == T_GOAL ? 8u : 0u);
    return h;
}

template <typename T, typename Done>
__device__ __forceinline__ void fused_serve_pair(const Geo &geo, const Coef<T> &cf, T *T0, T *T1, T *slots,
                                                 uint8_t *flags, const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                 double &dvl, const Done &done, const XydTopo<T> &tp,
                                                 bool zero_tiles) {
    const int c = threadIdx.x, lane = c & 63;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int W = geo.W, PL = serve_pair_plane(geo.HWs, W);
    k = __builtin_amdgcn_readfirstlane(k);  // uniform: the sweep count in an SGPR
    const int o0 = serve_pair_pad(W) + c;  // plane d of this cell at d * PL + o0
    const T ge = tp.valid ? cf.g : (T)0;
    T tq[4];  // the goal rewards in registers for the loop (the server's topology may live in memory)
#pragma unroll
    for (int d = 0; d < 4; ++d) tq[d] = tp.tq[d];
    // the neighbours' topology: cell c + W (its plane 1), cell c - W (its plane 3)
    const T geS = (tp.halo & 1u) ? cf.g : (T)0, tqS = (tp.halo & 2u) ? (T)1 : (T)0;
    const T geN = (tp.halo & 4u) ? cf.g : (T)0, tqN = (tp.halo & 8u) ? (T)1 : (T)0;
    T A[4], B[4], C[4];
    {
        V4<T> x = V4<T>{{(T)0, (T)0, (T)0, (T)0}};
        if (k != 0) x = *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) A[d] = own_cell ? x.v[d] : (T)0;
    }
    if (zero_tiles) {
        const int te = 4 * PL;
        for (int i = c; i < te; i += blockDim.x) {  // pads (and planes) of both tiles start at +0
            T0[i] = (T)0;
            T1[i] = (T)0;
        }
        __syncthreads();
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        B[d] = (T)0;
        C[d] = (T)0;
        T0[d * PL + o0] = A[d];
    }
    __syncthreads();
    uint8_t *const fwave = flags + (threadIdx.x >> 6);
    const bool lane0 = lane == 0;
    // the last pair's |dV| of its two sweeps and its middle set's north / south fronts
    T dm1p = (T)0, dm2p = (T)0, vSp = (T)0, vNp = (T)0;
    int stop = 0;  // 1: K = k - 1, 2: K = k
    // one sweep of this lane's cell from its own values and its four geometric fronts (fused_serve_xyd's)
    auto step = [&](const T (&in)[4], const T fE, const T fS, const T fW, const T fN, T (&out)[4]) -> T {
        const T m02 = vmax(in[0], in[2]), m13 = vmax(in[1], in[3]);
        const T m[4] = {vmax(vmax(in[0], m13), fE), vmax(vmax(in[1], m02), fS), vmax(vmax(in[2], m13), fW),
                        vmax(vmax(in[3], m02), fN)};
        T dm = (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            out[d] = vmax(ge * m[d], tq[d]);
            dm = vmax(dm, vabs(out[d] - in[d]));
        }
        return dm;
    };
    // par: this pair's flag slot (a constant at each unrolled call); test: whether a previous pair exists.
    // The sets rotate so that `mid` held V_{k-2} (dead: its planes are in Tout) and `out` holds the last
    // pair's middle set V_{k-1} until the test has passed.  half (the solve's first call): the first
    // sweep is the identity (mid = in, its neighbours' values read from the tile): ONE sweep.
    auto pair = [&](const T *Tin, T *Tout, const T (&in)[4], T (&mid)[4], T (&out)[4], const int par,
                    auto test, auto half) -> bool {
        constexpr bool HALF = decltype(half)::value;
        const uint32_t fl = *reinterpret_cast<const uint32_t *>(flags + (par ^ 1) * 16);
        const T fS = Tin[PL + o0 + W], fN = Tin[3 * PL + o0 - W];
        T dm1 = (T)0, vS, vN;
        if (HALF) {
#pragma unroll
            for (int d = 0; d < 4; ++d) mid[d] = in[d];
            vS = fS;
            vN = fN;
        } else {
            const T s0 = Tin[o0 + W], s2 = Tin[2 * PL + o0 + W], sf = Tin[PL + o0 + 2 * W];
            const T n0 = Tin[o0 - W], n2 = Tin[2 * PL + o0 - W], nf = Tin[3 * PL + o0 - 2 * W];
            dm1 = step(in, dpp_shl1_zero(in[0]), fS, dpp_shr1_zero(in[2]), fN, mid);
            // sweep k+1 of plane 1 of c + W and plane 3 of c - W (their owners' arithmetic)
            vS = vmax(geS * vmax(vmax(s0, s2), vmax(fS, sf)), tqS);
            vN = vmax(geN * vmax(vmax(n0, n2), vmax(fN, nf)), tqN);
            asm volatile("" ::"v"(vS), "v"(vN));  // reads and arithmetic ahead of the test (not sunk past it)
        }
        // the last pair's sweeps k - 1 and k (a bit is 0 when that sweep's |dV| < tol everywhere in the
        // wave or it reached max_sweeps)
        if (decltype(test)::value) {
            if ((fl & 0x01010101u) == 0u) { stop = 1; return false; }
            if ((fl & 0x02020202u) == 0u) { stop = 2; return false; }
        }
        const T dm2 = step(mid, dpp_shl1_zero(mid[0]), vS, dpp_shr1_zero(mid[2]), vN, out);
#pragma unroll
        for (int d = 0; d < 4; ++d) Tout[d * PL + o0] = out[d];
        constexpr int n = HALF ? 1 : 2;  // sweeps this call computes
        const uint32_t bits = (HALF || (__ballot(dm1 >= cf.tol) != 0ull && k + 1 < geo.max_sweeps) ? 1u : 0u) |
                              (__ballot(dm2 >= cf.tol) != 0ull && k + n < geo.max_sweeps ? 2u : 0u);
        if (lane0) fwave[par * 16] = (uint8_t)bits;
        dm1p = dm1;
        dm2p = dm2;
        vSp = vS;
        vNp = vN;
        __syncthreads();
        k += n;
        return true;
    };
    using Yes = std::integral_constant<bool, true>;
    using No = std::integral_constant<bool, false>;
    // p: the loop position of the pair that stopped, before its second sweep.  Its sets (in, out) by
    // p % 3: (C, B), (B, A), (A, C) -- `in` = V_k, `out` = V_{k-1} (the last pair's middle set) -- and its
    // output tile (T0 for even p) still holds V_{k-2}, the last pair's input.
    int p;
    pair(T0, T1, A, B, C, 0, No{}, Yes{});
    while (true) {
        if (!pair(T1, T0, C, A, B, 1, Yes{}, No{})) { p = 0; break; }
        if (!pair(T0, T1, B, C, A, 0, Yes{}, No{})) { p = 1; break; }
        if (!pair(T1, T0, A, B, C, 1, Yes{}, No{})) { p = 2; break; }
        if (!pair(T0, T1, C, A, B, 0, Yes{}, No{})) { p = 3; break; }
        if (!pair(T1, T0, B, C, A, 1, Yes{}, No{})) { p = 4; break; }
        if (!pair(T0, T1, A, B, C, 0, Yes{}, No{})) { p = 5; break; }
    }
    const T diff = stop == 1 ? dm1p : dm2p;
    if (stop == 1) k -= 1;
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    // element selects (a pointer to one of the sets would put them in scratch)
    const int r = p % 3;
    T vk_[4], vk1[4];  // V_k, V_{k-1}
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        vk_[d] = r == 0 ? C[d] : (r == 1 ? B[d] : A[d]);
        vk1[d] = r == 0 ? B[d] : (r == 1 ? A[d] : C[d]);
    }
    const T *Tp = (p & 1) ? T1 : T0;  // V_{k-2}, all four planes
    // V_K and V_{K-1}, and V_{K-1}'s fronts
    T vk[4], vp[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        vk[d] = stop == 1 ? vk1[d] : vk_[d];
        vp[d] = stop == 1 ? Tp[d * PL + o0] : vk1[d];
    }
    const T pS = stop == 1 ? Tp[PL + o0 + W] : vSp;
    const T pN = stop == 1 ? Tp[3 * PL + o0 - W] : vNp;
    const T pE = dpp_shl1_zero(vp[0]), pW = dpp_shr1_zero(vp[2]);
    if (own_cell) {
        // forward reads the front state when the agent can enter it, else its own (xyd_step's nbv)
        const T geo_f[4] = {pE, pS, pW, pN};
        const int HWs = geo.HWs;
        T nbv[4];
        V4<T> op;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            op.v[d] = vp[d];
            const bool enter = tp.nbi[d] != d * HWs + c;
            nbv[d] = enter ? geo_f[d] : vp[d];
        }
        V4<T> tmp;
        uint32_t pk;
        xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
        *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
        *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = V4<T>{{vk[0], vk[1], vk[2], vk[3]}};
    }
}

// Batched XYD grids with N cells per thread (cells t + j*blockDim, j < N; HWs = N * blockDim): the
// same sweep as fused_fast_xyd_soa on 1/N of the waves, so the per-sweep fixed work of a wave (flag
// read, address set-up, ballot, barrier) is paid once per N cells.  Plain deterministic / slip
// model only (the options kernel keeps one cell per thread).
template <typename T, bool SLIP, bool LOCAL, int N, typename Done>
__device__ __forceinline__ void fused_fast_xyd_soa_xn(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                                      T *V0, T *V1, T *slots, uint8_t *flags,
                                                      const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                      int k_target, double &dvl, const Done &done) {
    const int HW = geo.HWs;
    int c[N];
    XydTopo<T> tp[N];
    V4<T> own[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        c[j] = (int)(threadIdx.x + j * blockDim.x);
        const int cc = c[j] < geo.HW ? c[j] : 0;  // idle slots shadow cell 0 and never write HBM
        tp[j] = xyd_topo_soa<T>(cl, geo, cc);
        own[j] = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) V0[d * HW + c[j]] = own[j].v[d];
    }
    const int k_start = k;
    __syncthreads();
    int cur = 0, parity = 0;
    T diff = (T)0;
    auto sweep = [&](const T *Vin, T *Vout, const V4<T> (&in)[N], V4<T> (&out)[N]) -> bool {  // see fused_fast_xyd_soa
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        T nbv[N][4];
#pragma unroll
        for (int j = 0; j < N; ++j) xyd_load_nb(tp[j], Vin, nbv[j]);
        uint32_t pk;
        T d = (T)0;
#pragma unroll
        for (int j = 0; j < N; ++j) d = vmax(d, xyd_step<T, SLIP, false>(tp[j], cf, in[j], nbv[j], out[j], pk));
        if (LOCAL) {
            asm volatile("" ::"v"(d));
            if (k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        }
        diff = d;
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) Vout[q * HW + c[j]] = out[j].v[q];
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    V4<T> alt[N];
    while (true) {
        if (!sweep(V0, V1, own, alt)) { cur = 0; break; }
        if (!sweep(V1, V0, alt, own)) {
            cur = 1;
#pragma unroll
            for (int j = 0; j < N; ++j) own[j] = alt[j];
            break;
        }
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    const T *Vp = cur ? V0 : V1;  // V_{k-1}: pi of the last sweep is the argmax on it
#pragma unroll
    for (int j = 0; j < N; ++j) {
        if (c[j] < geo.HW) {
            V4<T> op, tmp;
            T nbv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) op.v[q] = Vp[q * HW + c[j]];
            xyd_load_nb(tp[j], Vp, nbv);
            uint32_t pk;
            xyd_step<T, SLIP, true>(tp[j], cf, op, nbv, tmp, pk);
            *reinterpret_cast<uint32_t *>(pig + c[j] * 4) = pk;
            *reinterpret_cast<V4<T> *>(Vg_out + c[j] * 4) = own[j];
        }
    }
}

// Batched deterministic XYD grids, two ADJACENT cells per thread (c0 = 2t, c0 + 1) and a
// compile-time plane stride HWS (= 2 * blockDim): the direction-major tiles then hold a thread's two
// values of a plane side by side, so each plane is one ds_write_b64 and its two front reads one
// ds_read2_b32, and every LDS address is one of three per-thread bases (the thread's slot, and
// that slot +-W rows) plus an immediate.  Forward reads the GEOMETRIC front cell: a front the
// agent cannot enter (wall, door, key, goal, lava) is an invalid state whose V is +0 in every tile
// (absorbing, V' = fl(0 * m) = +0), and V >= +0, so max(..., +0) is the identity and the value
// equals fused_fast_xyd_soa's (which reads the own state instead); a goal ahead still adds its
// constant 1 (only in waves that have one).  Same rule, same flags, same pi pass (the per-action
// form on the usual topology), bit-identical V, pi and sweep counts.
template <typename T, bool LOCAL, int HWS, typename Done>
__device__ __forceinline__ void fused_pair_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *V0,
                                               T *slots, uint8_t *flags, const T *Vg, T *Vg_out, int8_t *pig,
                                               int &k, int k_target, double &dvl, const Done &done) {
    struct alignas(2 * sizeof(T)) P2 { T a, b; };
    T *const V1 = V0 + 4 * HWS;  // smem_layout: V1 follows V0 (Ss = 4 * HWs)
    const int c0 = 2 * (int)threadIdx.x;
    const int lane = (int)threadIdx.x & 63;
    const int W = geo.W;
    const bool even_w = (W & 1) == 0;
    T ge[2];
    uint32_t goal = 0;  // bit 4j + d: a goal is ahead of cell c0 + j in direction d
    T own[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = c0 + j;
        const int cc = c < geo.HW ? c : 0;  // idle slots shadow cell 0 (a wall) and never write HBM
        const bool valid = xyd_free(cl[cc]);
        ge[j] = valid ? cf.g : (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            goal |= (uint32_t)(valid && cl[valid ? cc + geo.off[d] : cc] == T_GOAL) << (4 * j + d);
        const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) own[j][d] = x.v[d];
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) *reinterpret_cast<P2 *>(V0 + d * HWS + c0) = P2{own[0][d], own[1][d]};
    const bool goal_wave = __builtin_amdgcn_ballot_w64(goal != 0u) != 0ull;
    const int k_start = k;
    __syncthreads();
    int parity = 0;
    T diff = (T)0;
    // `out` is assigned only when the sweep commits, so after the loop the other register set
    // still holds V_{k-1} (the pi pass needs its planes 0 / 2, which the tiles keep only at edges)
    auto sweep = [&](const T *Vin, T *Vout, const T (&in)[2][4], T (&out)[2][4]) -> bool {
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        // geometric fronts: +1, +W, -1, -W in planes 0..3.  East / west stay in registers: the pair
        // holds each other's, the lanes beside it hold the rest (DPP wave shifts); only the two
        // wave-edge lanes read them from the tile, which the lanes at the other side of the edge
        // wrote (below).  North / south: one 8-byte read per plane when W is even (aligned,
        // conflict-free), two 4-byte reads otherwise.
        T F[2][4];
        F[0][0] = in[1][0];
        F[1][2] = in[0][2];
        F[1][0] = dpp_mov<0x130>(in[0][0]);  // wave_shl:1 -- lane i gets lane i+1's
        F[0][2] = dpp_mov<0x138>(in[1][2]);  // wave_shr:1 -- lane i gets lane i-1's
        if (lane == 63) F[1][0] = Vin[0 * HWS + c0 + 2];
        if (lane == 0) F[0][2] = Vin[2 * HWS + c0 - 1];
        if (even_w) {
            const P2 s = *reinterpret_cast<const P2 *>(Vin + 1 * HWS + c0 + W);
            const P2 n = *reinterpret_cast<const P2 *>(Vin + 3 * HWS + c0 - W);
            F[0][1] = s.a; F[1][1] = s.b;
            F[0][3] = n.a; F[1][3] = n.b;
        } else {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                F[j][1] = Vin[1 * HWS + c0 + j + W];
                F[j][3] = Vin[3 * HWS + c0 + j - W];
            }
        }
        T d = (T)0;
        T o[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const T m02 = vmax(in[j][0], in[j][2]), m13 = vmax(in[j][1], in[j][3]);
            const T m[4] = {vmax(vmax(in[j][0], m13), F[j][0]), vmax(vmax(in[j][1], m02), F[j][1]),
                            vmax(vmax(in[j][2], m13), F[j][2]), vmax(vmax(in[j][3], m02), F[j][3])};
#pragma unroll
            for (int q = 0; q < 4; ++q) o[j][q] = ge[j] * m[q];
        }
        // the goal's reward max(fl(g * m), 1) is exactly 1 (values are <= 1): a select (uniform
        // branch: few waves have one)
        if (goal_wave) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) o[j][q] = ((goal >> (4 * j + q)) & 1u) ? (T)1 : o[j][q];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) d = vmax(d, vabs(o[j][q] - in[j][q]));
        if (LOCAL) {
            asm volatile("" ::"v"(d));
            if (k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        }
        diff = d;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) out[j][q] = o[j][q];
        *reinterpret_cast<P2 *>(Vout + 1 * HWS + c0) = P2{out[0][1], out[1][1]};
        *reinterpret_cast<P2 *>(Vout + 3 * HWS + c0) = P2{out[0][3], out[1][3]};
        if (lane == 0) Vout[0 * HWS + c0] = out[0][0];           // read by the previous wave's lane 63
        if (lane == 63) Vout[2 * HWS + c0 + 1] = out[1][2];      // read by the next wave's lane 0
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    T alt[2][4], prev[2][4];
    int cur = 0;
    while (true) {
        if (!sweep(V0, V1, own, alt)) {
            cur = 0;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) prev[j][q] = alt[j][q];
            break;
        }
        if (!sweep(V1, V0, alt, own)) {
            cur = 1;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    prev[j][q] = own[j][q];
                    own[j][q] = alt[j][q];
                }
            break;
        }
    }
    // V_{k-1}'s tile: complete planes 0 / 2 (nobody reads it until the pi pass; block_max's
    // barrier orders these writes before it)
    T *Vp = cur ? V0 : V1;
    *reinterpret_cast<P2 *>(Vp + 0 * HWS + c0) = P2{prev[0][0], prev[1][0]};
    *reinterpret_cast<P2 *>(Vp + 2 * HWS + c0) = P2{prev[0][2], prev[1][2]};
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = c0 + j;
        if (c < geo.HW) {
            const XydTopo<T> tp = xyd_topo_soa<T>(cl, geo, c);
            V4<T> op, tmp;
            T nbv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) op.v[q] = Vp[q * HWS + c];
            xyd_load_nb(tp, Vp, nbv);
            uint32_t pk;
            xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
            *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
            *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = V4<T>{{own[j][0], own[j][1], own[j][2], own[j][3]}};
        }
    }
}

// Batched deterministic XYD grids, ONE wave per grid (cells j*64 + lane, j < P), no workgroup
// barrier: a wave's LDS instructions execute in issue order, so one tile suffices -- sweep k reads
// its north / south fronts (V_{k-1}) and only then overwrites them with V_k.  East / west fronts
// never touch LDS: cell c +- 1 is the neighbouring lane of the same block (DPP wave rotates), or
// at a block edge the other end of the next / previous block (the same rotate of that block's
// register); the first and last cell of the grid are border walls, whose fronts do not matter.
// The tile keeps only planes 1 (read at c + W) and 3 (read at c - W), with zero pads of padw
// cells on both sides, so it is 2 * 64 * P values per grid instead of two 4-plane tiles -- a
// Empty-16 grid needs 2.3 KB of LDS, not 8.5.  Forward reads the geometric front as in
// fused_pair_xyd (invalid states hold +0); the stop rule is the wave's ballot.  Same backups,
// rule and pi pass as fused_fast_xyd_soa: bit-identical V, pi and sweep counts.
// LDS: [slots 256 B][cells HWp][tile: pad | plane 3 (64P) | plane 1 (64P) | pad] (wave2_* below).
__host__ __device__ inline int wave2_padw(int W) { return (W + 15) / 16 * 16; }
__host__ __device__ inline int wave2_tile_off(int HWp) { return 256 + (HWp + 15) / 16 * 16; }
__host__ __device__ inline int wave2_smem_bytes(int HWp, int W, int P, int tsize) {
    return wave2_tile_off(HWp) + (2 * 64 * P + 2 * wave2_padw(W)) * tsize;
}
// In-launch reduction of an own-rule launch (mgdp_vi_solve / run_local on a one-wave batch that is
// resident at once; the host picks it then, else the reduce kernel follows the launch).  Each grid
// wave, at its own stopping sweep k_e, stores {k_e, dV} to its slots and draws a ticket of one of
// 256 shard counters (by e % 256, each counter on its own 128-B line, so at most B / 256 arrivals
// contend per line); a shard's last arrival folds its grids' slots into the shard's slots and draws
// a ticket of the top counter, whose last arrival folds the shards and publishes {kmax, dV bits,
// kmin}.  Slots are stored and loaded agent-scope (sc1) and every store is drained before
// the ticket that announces it (MI355X_MICROARCH.md: inter-workgroup hand-off).  No grid waits for
// another: a grid whose own rule stopped at an EXACT fixed point (|dV| = 0) is complete for every
// later sweep index (fixed-point completion, see fused_grid), so the global rule needs no K here.
struct GkCtx {
    unsigned long long *buf;  // gk_words(B) u64: counters, shard slots, grid slots (layout below)
    unsigned int epoch;
    int e;                    // grid (workgroup) index
    int B;                    // grids in the launch
    unsigned long long *pub;  // where the launch's {kmax, dV bits, kmin} go (host-mapped: epoch-tagged; device: raw)
};
constexpr int kGkShards = 256;
constexpr int kGkLine = 16;                                    // u64 words per 128-B line
constexpr int kGkCnt2 = 0;                                     // [256 shard counter lines][top line]
constexpr int kGkTop2 = kGkCnt2 + kGkShards * kGkLine;
constexpr int kGkSxMin = kGkTop2 + kGkLine;                    // int32 [256] shard min reported sweeps
constexpr int kGkSxMax = kGkSxMin + kGkShards / 2;             // int32 [256] shard max reported sweeps
constexpr int kGkSxDv = kGkSxMax + kGkShards / 2;              // u64 [256] shard max dV bits
__host__ __device__ inline int gk_kr_off(int B) { (void)B; return kGkSxDv + kGkShards; }  // int32 [B] sweeps,
__host__ __device__ inline int gk_dv_off(int B) { return gk_kr_off(B) + (B + 1) / 2; }     // u64 [B] dV bits
__host__ __device__ inline int gk_kn_off(int B) { return gk_dv_off(B) + B; }               // int32 [B] min sweeps (KMIN)
__host__ __device__ inline int gk_words(int B) { return gk_kn_off(B) + (B + 1) / 2; }

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// The whole wave, once it has its final answer: the launch's {kmax, dV, kmin} reduced over the
// counter tree, the last exit publishing it -- the reduce kernel a batch launch otherwise needs,
// folded into the launch.
// KMIN (the batch server's workgroups past the resident capacity, one arrival per workgroup for all
// its grids): the entry reports a {min, max} sweep pair, k_min_rep its min.
template <bool KMIN = false>
__device__ __forceinline__ void gk_exit(const GkCtx &g, int k_rep, double dv, int lane_in = -1, int k_min_rep = 0) {
    const int lane = lane_in >= 0 ? lane_in : (int)threadIdx.x & 63;
    int *kr = reinterpret_cast<int *>(g.buf + gk_kr_off(g.B));
    int *kn = KMIN ? reinterpret_cast<int *>(g.buf + gk_kn_off(g.B)) : kr;
    unsigned long long *dvr = g.buf + gk_dv_off(g.B);
    int *smin = reinterpret_cast<int *>(g.buf + kGkSxMin);
    int *smax = reinterpret_cast<int *>(g.buf + kGkSxMax);
    unsigned long long *sdv = g.buf + kGkSxDv;
    const int nsh = g.B < kGkShards ? g.B : kGkShards;
    const int s = g.e % nsh;
    const int size = g.B / nsh + (s < g.B % nsh ? 1 : 0);
    unsigned long long t = 0;
    if (lane == 0) {
        __hip_atomic_store(kr + g.e, k_rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (KMIN) __hip_atomic_store(kn + g.e, k_min_rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dvr + g.e, (unsigned long long)__double_as_longlong(dv), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t = __hip_atomic_fetch_add(g.buf + kGkCnt2 + s * kGkLine, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (__builtin_amdgcn_readfirstlane((unsigned int)t) != (unsigned int)(size - 1)) return;
    int mn = 0x7fffffff, mx = 0;
    unsigned long long dm = 0;
    for (int i = lane; i < size; i += 64) {
        const int x = __hip_atomic_load(kr + s + i * nsh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long y = __hip_atomic_load(dvr + s + i * nsh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mn = min(mn, KMIN ? __hip_atomic_load(kn + s + i * nsh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : x);
        mx = max(mx, x);
        dm = y > dm ? y : dm;
    }
    mn = wave_min_i(mn);
    mx = wave_max_i(mx);
    dm = wave_max_u64(dm);
    unsigned long long t2 = 0;
    if (lane == 0) {
        __hip_atomic_exchange(g.buf + kGkCnt2 + s * kGkLine, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(smin + s, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(smax + s, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sdv + s, dm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t2 = __hip_atomic_fetch_add(g.buf + kGkTop2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (__builtin_amdgcn_readfirstlane((unsigned int)t2) != (unsigned int)(nsh - 1)) return;
    mn = 0x7fffffff;
    mx = 0;
    dm = 0;
    for (int i = lane; i < nsh; i += 64) {
        mn = min(mn, __hip_atomic_load(smin + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        mx = max(mx, __hip_atomic_load(smax + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const unsigned long long y = __hip_atomic_load(sdv + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dm = y > dm ? y : dm;
    }
    mn = wave_min_i(mn);
    mx = wave_max_i(mx);
    dm = wave_max_u64(dm);
    if (lane == 0) {
        __hip_atomic_exchange(g.buf + kGkTop2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        publish(g.pub, (unsigned long long)mx, dm, (unsigned long long)mn, g.epoch);
        // the same epoch in device memory (the top counter's line): the resident batch server's forwarder
        // waits on it before polling the host for the next request
        __hip_atomic_store(g.buf + kGkTop2 + 1, (unsigned long long)g.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#ifndef MGDP_WAVE2_PREFETCH  // A/B builds: 1 = fused_wave2_xyd reads the next sweep's fronts early
#define MGDP_WAVE2_PREFETCH 0   // measured neutral (profiles/r05_pf/) and +9 VGPRs at P = 4
#endif
#ifndef MGDP_WAVE2_PK  // A/B builds: 1 = fused_wave2_xyd's multiplies and |dV| differences as packed fp32 pairs
#define MGDP_WAVE2_PK 0
#endif
#ifndef MGDP_WAVE2_DVTREE  // A/B builds: 1 = fused_wave2_xyd folds |dV| as a v_max3 tree
#define MGDP_WAVE2_DVTREE 0   // measured neutral (profiles/r05_tree/) and +9 VGPRs at P = 2, 4 (81 -> 90: 6 -> 5 waves)
#endif
// max of |x_i| over N values as a tree of v_max3 (depth log3 N instead of a running max's N / 2:
// max is exact and order-free, so the result is the same bits)
template <int N, typename T>
__device__ __forceinline__ T tree_max3(const T *x) {
    if constexpr (N == 1) {
        return x[0];
    } else if constexpr (N == 2) {
        return vmax(x[0], x[1]);
    } else if constexpr (N == 3) {
        return vmax(vmax(x[0], x[1]), x[2]);
    } else {
        constexpr int M = (N + 2) / 3;
        T y[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const int a = 3 * i;
            y[i] = a + 2 < N ? vmax(vmax(x[a], x[a + 1]), x[a + 2]) : (a + 1 < N ? vmax(x[a], x[a + 1]) : x[a]);
        }
        return tree_max3<M, T>(y);
    }
}
template <int B> struct WaveBuf { static constexpr int value = B; };
// WT: write the exit stores through the L2 (store_v4_exit; the caller instantiates it for the launches
// with the in-launch reduction, i.e. resident batches)
// OPQ (the resident batch server, which calls this once per request in its request loop): the lane
// index is re-derived per call by an asm the compiler cannot hoist, so nothing computed from it
// (tile and V addresses, cell indices) is moved out of the request loop and held live across it.
template <typename T, bool LOCAL, int P, bool WT = false, bool OPQ = false, typename Done>
__device__ __forceinline__ void fused_wave2_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *tile,
                                                const T *Vg, T *Vg_out, int8_t *pig, int &k, int k_target,
                                                double &dvl, const Done &done, const GkCtx gk = GkCtx{}) {
    static_assert(P >= 1 && P <= 8, "goal bits: 4 per cell, 32 per lane");
    const int lane = OPQ ? late_tid(0) : (int)threadIdx.x;
    const int W = geo.W, padw = wave2_padw(W);
    // k came from a per-grid word in memory (a VGPR); it is wave-uniform, so count sweeps in an SGPR
    // (the loop's k < max_sweeps test and increment are then scalar instructions, not VALU)
    k = __builtin_amdgcn_readfirstlane(k);
    T *const N3 = tile + padw;           // plane 3 (V of direction 3) of cell c at N3[c]
    T *const S1 = tile + padw + 64 * P;  // plane 1 of cell c at S1[c]
    T ge[P];
    uint32_t goal = 0;
    T own[P][4];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int c = j * 64 + lane;
        const int cc = c < geo.HW ? c : 0;  // idle slots shadow cell 0 (a wall) and never write HBM
        const bool valid = xyd_free(cl[cc]);
        ge[j] = valid ? cf.g : (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            goal |= (uint32_t)(valid && cl[valid ? cc + geo.off[d] : cc] == T_GOAL) << (4 * j + d);
        const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) own[j][d] = x.v[d];
        N3[c] = own[j][3];
        S1[c] = own[j][1];
    }
    for (int i = lane; i < padw; i += 64) {
        tile[i] = (T)0;
        tile[padw + 128 * P + i] = (T)0;
    }
    asm volatile("" ::: "memory");
    // per 64-cell block: does any of its cells have a goal ahead (a uniform branch per block; a
    // grid's goal touches one or two blocks)
    uint32_t goal_blocks = 0;
#pragma unroll
    for (int j = 0; j < P; ++j)
        goal_blocks |= (__builtin_amdgcn_ballot_w64(((goal >> (4 * j)) & 15u) != 0u) != 0ull ? 1u : 0u) << j;
    T diff = (T)0;
    // The north / south fronts of the sweep about to run.  With MGDP_WAVE2_PREFETCH a sweep reads the
    // next sweep's right after storing its own planes, so the LDS round trip overlaps its |dV|
    // reduction, stop ballot and branch instead of opening the next sweep (the reads of a sweep
    // that turns out to be the last are simply unused).
    T FS[P], FN[P];
    auto read_fronts = [&]() {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            FS[j] = S1[j * 64 + lane + W];
            FN[j] = N3[j * 64 + lane - W];
        }
    };
    if (MGDP_WAVE2_PREFETCH) read_fronts();
    // One sweep in -> out; returns whether another follows (the caller ran at least one: fused_grid
    // only calls with work to do).  The stop test ends the sweep that decides it, so at an exit the
    // sweep's own operands are V_{k-1} (in) and V_k (out) -- no loop-carried copy of V_{k-1}.
    auto sweep = [&](const T (&in)[P][4], T (&out)[P][4]) -> bool {
        if (!MGDP_WAVE2_PREFETCH) read_fronts();
        T R[P], L[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            R[j] = dpp_mov<0x134>(in[j][0]);  // wave_rol:1 -- lane i gets lane (i+1) mod 64
            L[j] = dpp_mov<0x13C>(in[j][2]);  // wave_ror:1 -- lane i gets lane (i-1) mod 64
        }
        T o[P][4];
        T dm = (T)0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const T FE = (j + 1 < P && lane == 63) ? R[j + 1] : R[j];
            const T FW = (j > 0 && lane == 0) ? L[j - 1] : L[j];
            const T m02 = vmax(in[j][0], in[j][2]), m13 = vmax(in[j][1], in[j][3]);
            const T m[4] = {vmax(vmax(in[j][0], m13), FE), vmax(vmax(in[j][1], m02), FS[j]),
                            vmax(vmax(in[j][2], m13), FW), vmax(vmax(in[j][3], m02), FN[j])};
            if constexpr (MGDP_WAVE2_PK && sizeof(T) == 4) {  // two packed multiplies (v_pk_mul_f32)
                typedef float f2 __attribute__((ext_vector_type(2)));
                const f2 g2 = {ge[j], ge[j]};
                const f2 a = f2{m[0], m[1]} * g2, b = f2{m[2], m[3]} * g2;
                o[j][0] = a.x;
                o[j][1] = a.y;
                o[j][2] = b.x;
                o[j][3] = b.y;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) o[j][q] = ge[j] * m[q];
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            if ((goal_blocks >> j) & 1u) {  // the goal's reward max(fl(g * m), 1) is exactly 1 (values are <= 1): a select
#pragma unroll
                for (int q = 0; q < 4; ++q) o[j][q] = ((goal >> (4 * j + q)) & 1u) ? (T)1 : o[j][q];
            }
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            S1[j * 64 + lane] = o[j][1];
            N3[j * 64 + lane] = o[j][3];
        }
        asm volatile("" ::: "memory");
        if (MGDP_WAVE2_PREFETCH) read_fronts();  // LDS is in order per wave: after this sweep's stores
        // a k_target loop reports |dV| of its last sweep only (a uniform branch)
        if (LOCAL || MGDP_RUNTO_DV_ALL || k + 1 == k_target) {
            if (MGDP_WAVE2_DVTREE) {
                T ad[4 * P];
#pragma unroll
                for (int j = 0; j < P; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) ad[4 * j + q] = vabs(o[j][q] - in[j][q]);
                dm = tree_max3<4 * P, T>(ad);
            } else if constexpr (MGDP_WAVE2_PK && sizeof(T) == 4) {  // packed differences (v_pk_add_f32)
                typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const f2 a = f2{o[j][0], o[j][1]} - f2{in[j][0], in[j][1]};
                    const f2 b = f2{o[j][2], o[j][3]} - f2{in[j][2], in[j][3]};
                    dm = vmax(vmax(dm, vabs(a.x)), vabs(a.y));
                    dm = vmax(vmax(dm, vabs(b.x)), vabs(b.y));
                }
            } else {
#pragma unroll
                for (int j = 0; j < P; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) dm = vmax(dm, vabs(o[j][q] - in[j][q]));
            }
        }
        diff = dm;
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) out[j][q] = o[j][q];
        ++k;
        if (LOCAL) return k < geo.max_sweeps && __ballot(dm >= cf.tol) != 0ull;
        return k < k_target;
    };
    // Exit work (reduction, publication, pi pass, V store) on cur = V_k, prv = V_{k-1}.
    auto finish = [&](const T (&cur)[P][4], const T (&prv)[P][4]) {
        dvl = (double)wave_max(diff);
        if (LOCAL && gk.buf != nullptr) gk_exit(gk, k, dvl, OPQ ? late_tid(0) : lane);  // this launch's reduction and its publication
        done(k, dvl);
        // pi of the last sweep = argmax on V_{k-1} (`prv`), per action with the usual topology
#pragma unroll
        for (int j = 0; j < P; ++j) {
            S1[j * 64 + lane] = prv[j][1];
            N3[j * 64 + lane] = prv[j][3];
        }
        asm volatile("" ::: "memory");
        T R[P], L[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            R[j] = dpp_mov<0x134>(prv[j][0]);
            L[j] = dpp_mov<0x13C>(prv[j][2]);
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int c = j * 64 + lane;
            const T front[4] = {(j + 1 < P && lane == 63) ? R[j + 1] : R[j], S1[c + W],
                                (j > 0 && lane == 0) ? L[j - 1] : L[j], N3[c - W]};
            if (c < geo.HW) {
                const XydTopo<T> tp = xyd_topo<T>(cl, geo, c);
                V4<T> op, tmp;
                T nbv[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    op.v[d] = prv[j][d];
                    nbv[d] = (tp.nbi[d] >> 2) != c ? front[d] : prv[j][d];  // blocked / terminal: own state
                }
                uint32_t pk;
                xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
                store_pi_exit(pig + c * 4, pk, WT);
                store_v4_exit(Vg_out + c * 4, V4<T>{{cur[j][0], cur[j][1], cur[j][2], cur[j][3]}}, WT);
            }
        }
    };
    // Two sweeps per iteration with fixed roles (own -> alt -> own); each exit runs the exit work
    // on its own roles.
    T alt[P][4];
    while (true) {
        if (!sweep(own, alt)) {
            finish(alt, own);
            return;
        }
        if (!sweep(alt, own)) {
            finish(own, alt);
            return;
        }
    }
}

// Batched deterministic XYD grids, one wave per grid, COLUMN BANDS (round 5): lane l = b*W + x owns
// the HB cells (b*HB + j, x), j < HB, of column x in band b (nb = 64 / W bands of HB = ceil(H / nb)
// rows).  A cell's north / south fronts are then the lane's own registers (the next / previous
// slot) except across band edges, and its east / west fronts the neighbouring lanes (DPP wave
// shifts; x = 0 and x = W - 1 are border walls, whose fronts do not matter), so a sweep moves two
// values between lanes (ds_bpermute: the band-edge fronts) and touches no LDS tile at all --
// fused_wave2_xyd's row-major blocks read 2P and write 2P LDS words per sweep, a round trip on
// every sweep's critical path that left FourRooms x 4096 (4 waves per SIMD) stalled half the time.
// Same one-multiply backup, geometric fronts (invalid states hold +0), goal reward, ballot stop
// rule, uncommitted last sweep and per-action pi pass as fused_wave2_xyd: bit-identical V, pi and
// sweep counts.  Grids with W <= 64 and ceil(H / (64 / W)) <= 8.
template <typename T>
__device__ __forceinline__ T lane_shfl(T v, int src) {  // lane src's v (ds_bpermute, no LDS memory)
    if constexpr (sizeof(T) == 4) {
        return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
    } else {
        const long long b = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b), hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
        return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
}
__host__ __device__ inline int band_rows(int W, int H) { return W > 64 ? 0 : (H + 64 / W - 1) / (64 / W); }

template <typename T, bool LOCAL, int HB, typename Done>
__device__ __forceinline__ void fused_band_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, const T *Vg,
                                               T *Vg_out, int8_t *pig, int &k, int k_target, double &dvl,
                                               const Done &done, const GkCtx gk = GkCtx{}) {
    static_assert(HB >= 1 && HB <= 8, "goal bits: 4 per cell, 32 per lane");
    const int lane = (int)threadIdx.x;
    k = __builtin_amdgcn_readfirstlane(k);  // uniform: the sweep count in an SGPR
    const int W = geo.W, nb = 64 / W;
    const int band = lane / W, x = lane - band * W;
    const bool lane_on = band < nb;
    const int up = lane >= W ? lane - W : lane, dn = lane + W < 64 ? lane + W : lane;  // band-edge partners
    T ge[HB];
    uint32_t goal = 0;
    int cix[HB];
    T own[HB][4];
#pragma unroll
    for (int j = 0; j < HB; ++j) {
        const int row = band * HB + j;
        const bool on = lane_on && row < geo.H;
        const int c = on ? row * W + x : -1;
        cix[j] = c;
        const int cc = on ? c : 0;  // idle slots shadow cell 0 (a wall) and never write HBM
        const bool valid = xyd_free(cl[cc]);
        ge[j] = valid ? cf.g : (T)0;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            goal |= (uint32_t)(valid && cl[valid ? cc + geo.off[d] : cc] == T_GOAL) << (4 * j + d);
        const V4<T> v = (k == 0 || !on) ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) own[j][d] = v.v[d];
    }
    uint32_t goal_slots = 0;  // per slot j: does any lane's cell have a goal ahead (a uniform branch)
#pragma unroll
    for (int j = 0; j < HB; ++j)
        goal_slots |= (__builtin_amdgcn_ballot_w64(((goal >> (4 * j)) & 15u) != 0u) != 0ull ? 1u : 0u) << j;
    const int k_start = k;
    bool more = true;
    T diff = (T)0;
    // the four geometric fronts of every slot from a register set
    auto fronts = [&](const T (&in)[HB][4], T (&FE)[HB], T (&FS)[HB], T (&FW)[HB], T (&FN)[HB]) {
        const T s_edge = lane_shfl(in[0][1], dn);       // south of slot HB-1: next band's slot 0, plane 1
        const T n_edge = lane_shfl(in[HB - 1][3], up);  // north of slot 0: previous band's slot HB-1, plane 3
#pragma unroll
        for (int j = 0; j < HB; ++j) {
            FE[j] = dpp_shl1_zero(in[j][0]);
            FW[j] = dpp_shr1_zero(in[j][2]);
            FS[j] = j + 1 < HB ? in[j + 1][1] : s_edge;
            FN[j] = j > 0 ? in[j - 1][3] : n_edge;
        }
    };
    auto sweep = [&](const T (&in)[HB][4], T (&out)[HB][4]) -> bool {  // `out` written only on commit
        if (LOCAL) {
            if (k >= geo.max_sweeps || (k > k_start && !more)) return false;
        } else if (k >= k_target) {
            return false;
        }
        T FE[HB], FS[HB], FW[HB], FN[HB];
        fronts(in, FE, FS, FW, FN);
        T o[HB][4];
#pragma unroll
        for (int j = 0; j < HB; ++j) {
            const T m02 = vmax(in[j][0], in[j][2]), m13 = vmax(in[j][1], in[j][3]);
            const T m[4] = {vmax(vmax(in[j][0], m13), FE[j]), vmax(vmax(in[j][1], m02), FS[j]),
                            vmax(vmax(in[j][2], m13), FW[j]), vmax(vmax(in[j][3], m02), FN[j])};
#pragma unroll
            for (int q = 0; q < 4; ++q) o[j][q] = ge[j] * m[q];
        }
#pragma unroll
        for (int j = 0; j < HB; ++j) {
            if ((goal_slots >> j) & 1u) {  // the goal's reward max(fl(g * m), 1) is exactly 1 (values are <= 1): a select
#pragma unroll
                for (int q = 0; q < 4; ++q) o[j][q] = ((goal >> (4 * j + q)) & 1u) ? (T)1 : o[j][q];
            }
        }
        T dm = (T)0;
        if (LOCAL || MGDP_RUNTO_DV_ALL || k + 1 == k_target) {  // a k_target loop: |dV| of its last sweep only
#pragma unroll
            for (int j = 0; j < HB; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) dm = vmax(dm, vabs(o[j][q] - in[j][q]));
        }
        diff = dm;
        if (LOCAL) more = __ballot(dm >= cf.tol) != 0ull;
#pragma unroll
        for (int j = 0; j < HB; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) out[j][q] = o[j][q];
        ++k;
        return true;
    };
    T alt[HB][4], prev[HB][4];
    while (true) {
        if (!sweep(own, alt)) {
#pragma unroll
            for (int j = 0; j < HB; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) prev[j][q] = alt[j][q];
            break;
        }
        if (!sweep(alt, own)) {
#pragma unroll
            for (int j = 0; j < HB; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    prev[j][q] = own[j][q];
                    own[j][q] = alt[j][q];
                }
            break;
        }
    }
    dvl = (double)wave_max(diff);
    if (LOCAL && gk.buf != nullptr) gk_exit(gk, k, dvl);  // this launch's reduction and its publication
    done(k, dvl);
    // pi of the last sweep = argmax on V_{k-1} (`prev`), per action with the usual topology
    T FE[HB], FS[HB], FW[HB], FN[HB];
    fronts(prev, FE, FS, FW, FN);
#pragma unroll
    for (int j = 0; j < HB; ++j) {
        const int c = cix[j];
        if (c >= 0) {
            const XydTopo<T> tp = xyd_topo<T>(cl, geo, c);
            const T front[4] = {FE[j], FS[j], FW[j], FN[j]};
            V4<T> op, tmp;
            T nbv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                op.v[d] = prev[j][d];
                nbv[d] = (tp.nbi[d] >> 2) != c ? front[d] : prev[j][d];  // blocked / terminal: own state
            }
            uint32_t pk;
            xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
            *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
            *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = V4<T>{{own[j][0], own[j][1], own[j][2], own[j][3]}};
        }
    }
}

// Batched deterministic XYD grids on TWO waves per grid (fused_wave2n_xyd): wave w owns blocks
// w*PW .. w*PW + PW - 1 of the P = 2*PW 64-cell blocks, so a grid's sweep is two chains of PW
// blocks instead of one of P -- for batches too small to fill the GPU with one wave per grid
// (FourRooms x 4096: 4096 waves on 1024 SIMDs).  The waves meet at one barrier per sweep: V_k's
// planes 1 / 3 alternate between two tiles (sweep k reads tile (k - k_start) & 1, writes the
// other), the two east / west values that cross the wave boundary (plane 0 of wave 1's first
// cell, plane 2 of wave 0's last cell) go through two LDS words per tile, and each wave's stop
// ballot through a flag word per tile, read with the next sweep's fronts -- so both waves take
// the same stop decision.  Arithmetic, rule and pi pass as fused_wave2_xyd: bit-identical results.
// LDS: [slots 256 B][cells HWp][tile 0][tile 1][edges 4 T | dV 2 T | flags 4 u32] (wave2n_*).
__host__ __device__ inline int wave2n_tile_elems(int W, int P) { return 2 * 64 * P + 2 * wave2_padw(W); }
__host__ __device__ inline int wave2n_smem_bytes(int HWp, int W, int P, int tsize) {
    return wave2_tile_off(HWp) + 2 * wave2n_tile_elems(W, P) * tsize + 64;
}
// A mixed launch (kWpMix): P blocks on one wave or 2 * ceil(P / 2) on two, the larger layout
__host__ __device__ inline int mix_smem_bytes(int HWp, int W, int P, int tsize) {
    const int a = wave2_smem_bytes(HWp, W, P, tsize), b = wave2n_smem_bytes(HWp, W, 2 * ((P + 1) / 2), tsize);
    return a > b ? a : b;
}

template <typename T, bool LOCAL, int PW, typename Done>
__device__ __forceinline__ void fused_wave2n_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *tile,
                                                 const T *Vg, T *Vg_out, int8_t *pig, int &k, int k_target,
                                                 double &dvl, const Done &done, const GkCtx gk = GkCtx{}) {
    static_assert(PW >= 1 && PW <= 8, "goal bits: 4 per cell, 32 per lane");
    constexpr int P = 2 * PW;
    const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
    k = __builtin_amdgcn_readfirstlane(k);  // uniform: the sweep count in an SGPR
    const int W = geo.W, padw = wave2_padw(W);
    const int TS = wave2n_tile_elems(W, P);
    T *const edge = tile + 2 * TS;  // [tile][0: plane 0 of cell 64 PW, 1: plane 2 of cell 64 PW - 1]
    T *const dvx = edge + 4;        // [wave] |dV| of the last sweep
    uint32_t *const flag = reinterpret_cast<uint32_t *>(reinterpret_cast<unsigned char *>(edge) + 48);  // [tile][wave]
    T ge[PW];
    uint32_t goal = 0;
    T own[PW][4];
    {
        T *const N3 = tile + padw, *const S1 = tile + padw + 64 * P;
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int c = (w * PW + j) * 64 + lane;
            const int cc = c < geo.HW ? c : 0;  // idle slots shadow cell 0 (a wall) and never write HBM
            const bool valid = xyd_free(cl[cc]);
            ge[j] = valid ? cf.g : (T)0;
#pragma unroll
            for (int d = 0; d < 4; ++d)
                goal |= (uint32_t)(valid && cl[valid ? cc + geo.off[d] : cc] == T_GOAL) << (4 * j + d);
            const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
            for (int d = 0; d < 4; ++d) own[j][d] = x.v[d];
            N3[c] = own[j][3];
            S1[c] = own[j][1];
        }
        if (w == 1 && lane == 0) edge[0] = own[0][0];
        if (w == 0 && lane == 63) edge[1] = own[PW - 1][2];
        for (int i = (int)threadIdx.x; i < padw; i += 128) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                tile[t * TS + i] = (T)0;
                tile[t * TS + padw + 128 * P + i] = (T)0;
            }
        }
    }
    uint32_t goal_blocks = 0;
#pragma unroll
    for (int j = 0; j < PW; ++j)
        goal_blocks |= (__builtin_amdgcn_ballot_w64(((goal >> (4 * j)) & 15u) != 0u) != 0ull ? 1u : 0u) << j;
    __syncthreads();
    T diff = (T)0;
    // sweep k_start + i reads tile i & 1 and writes the other (b: compile-time in the unrolled pair).
    // As fused_wave2_xyd: the stop test ends the sweep that decides it (both waves' flags, read
    // right after its barrier), so at an exit V_{k-1} is the sweep's own input set.
    auto sweep = [&](auto bc, const T (&in)[PW][4], T (&out)[PW][4]) -> bool {
        constexpr int b = decltype(bc)::value;
        const T *const N3r = tile + b * TS + padw, *const S1r = N3r + 64 * P;
        T *const N3w = tile + (b ^ 1) * TS + padw, *const S1w = N3w + 64 * P;
        T FS[PW], FN[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int c = (w * PW + j) * 64 + lane;
            FS[j] = S1r[c + W];
            FN[j] = N3r[c - W];
        }
        const T eE = edge[2 * b], eW = edge[2 * b + 1];
        T R[PW], L[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            R[j] = dpp_mov<0x134>(in[j][0]);  // wave_rol:1 -- lane i gets lane (i+1) mod 64
            L[j] = dpp_mov<0x13C>(in[j][2]);  // wave_ror:1 -- lane i gets lane (i-1) mod 64
        }
        T o[PW][4];
        T dm = (T)0;
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            // across the wave boundary: wave 0's last cell and wave 1's first cell through LDS
            const T FE = lane == 63 ? (j + 1 < PW ? R[j + 1] : (w == 0 ? eE : R[j])) : R[j];
            const T FW = lane == 0 ? (j > 0 ? L[j - 1] : (w == 1 ? eW : L[j])) : L[j];
            const T m02 = vmax(in[j][0], in[j][2]), m13 = vmax(in[j][1], in[j][3]);
            const T m[4] = {vmax(vmax(in[j][0], m13), FE), vmax(vmax(in[j][1], m02), FS[j]),
                            vmax(vmax(in[j][2], m13), FW), vmax(vmax(in[j][3], m02), FN[j])};
#pragma unroll
            for (int q = 0; q < 4; ++q) o[j][q] = ge[j] * m[q];
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            if ((goal_blocks >> j) & 1u) {  // the goal's reward max(fl(g * m), 1) is exactly 1 (values are <= 1): a select
#pragma unroll
                for (int q = 0; q < 4; ++q) o[j][q] = ((goal >> (4 * j + q)) & 1u) ? (T)1 : o[j][q];
            }
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int c = (w * PW + j) * 64 + lane;
            S1w[c] = o[j][1];
            N3w[c] = o[j][3];
        }
        if (w == 1 && lane == 0) edge[2 * (b ^ 1)] = o[0][0];
        if (w == 0 && lane == 63) edge[2 * (b ^ 1) + 1] = o[PW - 1][2];
        if (LOCAL || MGDP_RUNTO_DV_ALL || k + 1 == k_target) {
#pragma unroll
            for (int j = 0; j < PW; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) dm = vmax(dm, vabs(o[j][q] - in[j][q]));
        }
        diff = dm;
        if (LOCAL) {
            const bool more_w = __ballot(dm >= cf.tol) != 0ull;
            if (lane == 0) flag[2 * (b ^ 1) + w] = more_w ? 1u : 0u;
        }
#pragma unroll
        for (int j = 0; j < PW; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) out[j][q] = o[j][q];
        ++k;
        __syncthreads();  // this sweep's tile, edges and flags before anyone reads them
        if (LOCAL) return k < geo.max_sweeps && (flag[2 * (b ^ 1)] | flag[2 * (b ^ 1) + 1]) != 0u;
        return k < k_target;
    };
    // the exit work on cur = V_k, prv = V_{k-1} (each exit with its own roles)
    auto finish = [&](const T (&cur)[PW][4], const T (&prv)[PW][4]) {
        {
            const T dw = wave_max(diff);
            if (lane == 0) dvx[w] = dw;
        }
        __syncthreads();  // both waves' |dV|; past this no sweep reads a tile
        dvl = (double)vmax(dvx[0], dvx[1]);
        if (LOCAL && gk.buf != nullptr && w == 0) gk_exit(gk, k, dvl);  // the launch's reduction (one wave per grid)
        done(k, dvl);
        // pi of the last sweep = argmax on V_{k-1} (`prv`), per action with the usual topology
        T *const N3 = tile + padw, *const S1 = tile + padw + 64 * P;
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int c = (w * PW + j) * 64 + lane;
            S1[c] = prv[j][1];
            N3[c] = prv[j][3];
        }
        if (w == 1 && lane == 0) edge[0] = prv[0][0];
        if (w == 0 && lane == 63) edge[1] = prv[PW - 1][2];
        __syncthreads();
        const T eE = edge[0], eW = edge[1];
        T R[PW], L[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            R[j] = dpp_mov<0x134>(prv[j][0]);
            L[j] = dpp_mov<0x13C>(prv[j][2]);
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int c = (w * PW + j) * 64 + lane;
            const T front[4] = {lane == 63 ? (j + 1 < PW ? R[j + 1] : (w == 0 ? eE : R[j])) : R[j], S1[c + W],
                                lane == 0 ? (j > 0 ? L[j - 1] : (w == 1 ? eW : L[j])) : L[j], N3[c - W]};
            if (c < geo.HW) {
                const XydTopo<T> tp = xyd_topo<T>(cl, geo, c);
                V4<T> op, tmp;
                T nbv[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    op.v[d] = prv[j][d];
                    nbv[d] = (tp.nbi[d] >> 2) != c ? front[d] : prv[j][d];  // blocked / terminal: own state
                }
                uint32_t pk;
                xyd_step<T, false, true>(tp, cf, op, nbv, tmp, pk);
                *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
                *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = V4<T>{{cur[j][0], cur[j][1], cur[j][2], cur[j][3]}};
            }
        }
    };
    T alt[PW][4];
    while (true) {
        if (!sweep(WaveBuf<0>{}, own, alt)) {
            finish(alt, own);
            return;
        }
        if (!sweep(WaveBuf<1>{}, alt, own)) {
            finish(own, alt);
            return;
        }
    }
}

// Lone XYD grid on ONE wave, P cells per lane (cell j*64 + lane, same direction-major tiles with
// HWs = 64*P).  A wave's LDS instructions execute in issue order, so the writes of sweep k are
// seen by the reads of sweep k+1 without a workgroup barrier, and the stopping rule is the wave's
// ballot -- no flag round trip through LDS.  The compiler fence keeps the program order of the
// two sweeps' LDS accesses (cross-lane dependencies it cannot see).  Same arithmetic, same rule
// and same final pi pass as fused_fast_xyd_soa.
template <typename T, bool SLIP, bool LOCAL, int P, typename Done>
__device__ __forceinline__ void fused_wave_xyd(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *V0, T *V1,
                                               const T *Vg, T *Vg_out, int8_t *pig, int &k, int k_target,
                                               double &dvl, const Done &done) {
    const int lane = threadIdx.x;
    const int HW = geo.HWs;
    const int k_start = k;
    XydTopo<T> tp[P];
    V4<T> own[P], alt[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int c = j * 64 + lane;
        const int cc = c < geo.HW ? c : 0;  // idle slots shadow cell 0 and never write HBM
        tp[j] = xyd_topo_soa<T>(cl, geo, cc);
        if (k == 0) own[j] = V4<T>{{(T)0, (T)0, (T)0, (T)0}};
        else own[j] = *reinterpret_cast<const V4<T> *>(Vg + cc * 4);
#pragma unroll
        for (int d = 0; d < 4; ++d) V0[d * HW + c] = own[j].v[d];
    }
    asm volatile("" ::: "memory");
    bool more = true;
    T diff = (T)0;
    auto sweep = [&](const T *Vin, T *Vout, const V4<T> (&in)[P], V4<T> (&out)[P]) -> bool {
        T nbv[P][4];
#pragma unroll
        for (int j = 0; j < P; ++j) xyd_load_nb(tp[j], Vin, nbv[j]);
        if (LOCAL) {
            if (k >= geo.max_sweeps) return false;
            if (k > k_start && !more) return false;
        } else if (k >= k_target) {
            return false;
        }
        T dm = (T)0;
        uint32_t pk;
#pragma unroll
        for (int j = 0; j < P; ++j) dm = vmax(dm, xyd_step<T, SLIP, false>(tp[j], cf, in[j], nbv[j], out[j], pk));
#pragma unroll
        for (int j = 0; j < P; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) Vout[q * HW + j * 64 + lane] = out[j].v[q];
        asm volatile("" ::: "memory");
        diff = dm;
        if (LOCAL) more = __ballot(dm >= cf.tol) != 0ull;
        ++k;
        return true;
    };
    int cur;
    while (true) {
        if (!sweep(V0, V1, own, alt)) { cur = 0; break; }
        if (!sweep(V1, V0, alt, own)) {
            cur = 1;
#pragma unroll
            for (int j = 0; j < P; ++j) own[j] = alt[j];
            break;
        }
    }
    dvl = (double)wave_max(diff);
    done(k, dvl);
    const T *Vp = cur ? V0 : V1;  // V_{k-1}: pi of the last sweep is the argmax on it
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int c = j * 64 + lane;
        if (c < geo.HW) {
            V4<T> op, tmp;
            T nbv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) op.v[q] = Vp[q * HW + c];
            xyd_load_nb(tp[j], Vp, nbv);
            uint32_t pk;
            xyd_step<T, SLIP, true>(tp[j], cf, op, nbv, tmp, pk);
            *reinterpret_cast<uint32_t *>(pig + c * 4) = pk;
            *reinterpret_cast<V4<T> *>(Vg_out + c * 4) = own[j];
        }
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

// Thread -> cell map of a batched DoorKey grid that puts the "special" cells first (stable): those
// with a goal, key or door ahead or a key / door under them, whose waves take the longer value
// sweep (dk_step_fast's GOAL / KD forms, up to 1.7x the VALU work of the plain form).  With the
// <= ~10 special cells of a DoorKey grid in one wave, the other waves all run the plain form
// (row-major, 2.7 of a 16x16 grid's 4 waves had some special cell, 2.1 the KD form; 200 seeds).
// The LDS tiles and HBM rows stay indexed by cell: only which thread owns which cell changes, so V,
// pi and the sweep count are untouched.  Absorbing cells (walls, the goal: no walkable state) go
// last, so the 74 of a DoorKey-16 grid fill its fourth wave, which then skips the arithmetic
// (fused_fast_dk_soa's `wdead`).  Whole block (two barriers); `perm`: 2*HW bytes of LDS, `cnt`:
// 32 ints.  Returns this thread's cell (threads past HW keep their index: idle slots).
__device__ __forceinline__ int dk_class_perm(const uint8_t *cl, const Geo &geo, int16_t *perm, int *cnt) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = (int)(blockDim.x >> 6);
    bool special = false, walk = false;
    if (t < geo.HW) {
        const DkFast q = dk_fast_topo(dk_topo_soa(cl, geo, t), geo.HWs);
        special = dk_fast_class(q) != 0u;
        walk = q.walk != 0u;
    }
    const unsigned long long bs = __builtin_amdgcn_ballot_w64(special);
    const unsigned long long bp = __builtin_amdgcn_ballot_w64(walk && !special);
    const unsigned long long bv = __builtin_amdgcn_ballot_w64(t < geo.HW);
    if (lane == 0) {
        cnt[w] = __popcll(bs);
        cnt[16 + w] = __popcll(bp);
    }
    __syncthreads();
    int before_s = 0, before_p = 0, total_s = 0, total_p = 0;
    for (int i = 0; i < nw; ++i) {
        if (i < w) {
            before_s += cnt[i];
            before_p += cnt[16 + i];
        }
        total_s += cnt[i];
        total_p += cnt[16 + i];
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (t < geo.HW) {
        // the waves before w hold 64*w cells; those not special or plain are absorbing
        const int before_a = 64 * w - before_s - before_p;
        const int dest = special ? before_s + __popcll(bs & lt)
                         : walk  ? total_s + before_p + __popcll(bp & lt)
                                 : total_s + total_p + before_a + __popcll(bv & ~bs & ~bp & lt);
        perm[dest] = (int16_t)t;
    }
    __syncthreads();
    return t < geo.HW ? (int)perm[t] : t;
}

// perm_lds: with an LDS scratch (see dk_class_perm; 2*HW + 128 bytes), threads take the cells of
// the special-first map; nullptr keeps thread t on cell t.
template <typename T, bool LOCAL, int HMODE = 0, typename Done>  // HMODE: see fused_fast_xyd_soa
__device__ __forceinline__ void fused_fast_dk_soa(const Geo &geo, const Coef<T> &cf, const uint8_t *cl,
                                                  T *V0, T *V1, T *slots, uint8_t *flags,
                                                  const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                                  int k_target, double &dvl, const Done &done,
                                                  const T *rgoal = nullptr, int8_t *pit = nullptr,
                                                  long long pit_stride = 0, const DkTopo *pre = nullptr,
                                                  uint8_t *perm_lds = nullptr) {
    const int c = perm_lds ? dk_class_perm(cl, geo, reinterpret_cast<int16_t *>(perm_lds),
                                           reinterpret_cast<int *>(perm_lds + (2 * geo.HW + 15) / 16 * 16))
                           : (int)threadIdx.x;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs;  // LDS stride: every thread (idle ones too) owns a slot, so LDS writes need no mask
    const int k_start = k;
    const DkTopo tp = pre ? *pre : dk_topo_soa(cl, geo, cc);  // pre: see fused_fast_xyd_soa
    // Value sweeps use dk_step_fast, specialised per wave (a uniform branch) on whether any of
    // its cells has a goal ahead (bit 0) or a key / door ahead or under it (bit 1).
    const DkFast tpf = dk_fast_topo(tp, HW);
    const uint32_t cls = dk_fast_class(tpf);
    const uint32_t wcls = (__builtin_amdgcn_ballot_w64(cls & 1u) ? 1u : 0u) | (__builtin_amdgcn_ballot_w64(cls & 2u) ? 2u : 0u);
    // A wave of absorbing cells only (idle slots read cell 0, a border wall): every value it owns
    // is +0 in both tiles and stays +0 (dk_step_fast yields exactly +0 there), so its value sweeps
    // store +0 with no arithmetic and no front reads.  The special-first map packs a DoorKey-16
    // grid's absorbing cells into its fourth wave.
    const bool wdead = MGDP_DK_DEAD && __builtin_amdgcn_ballot_w64(tp.walk != 0u) == 0ull;
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
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);  // the previous sweep's flags (all 16 bytes: no branch on the wave count)
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        V4<T> nbs[4];
        uint32_t pk[4];
        const T rg = HMODE ? rgoal[k_target - 1 - k] : (T)1;
        T d;
        if (HMODE != 2 && wdead) {
#pragma unroll
            for (int l = 0; l < 16; ++l) outv[l] = (T)0;
            d = (T)0;
        } else if (HMODE != 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) nbs[q] = *reinterpret_cast<const V4<T> *>(Vin + tpf.nb[q]);
            // a k_target loop reports |dV| of its last sweep only: the others skip the differences
            if (LOCAL || MGDP_RUNTO_DV_ALL || k + 1 == k_target) {
                if (wcls == 0u) d = dk_step_fast<T, HMODE != 0, false, false>(tpf, cf, in, nbs, outv, rg);
                else if (wcls == 1u) d = dk_step_fast<T, HMODE != 0, true, false>(tpf, cf, in, nbs, outv, rg);
                else d = dk_step_fast<T, HMODE != 0, true, true>(tpf, cf, in, nbs, outv, rg);
            } else {
                if (wcls == 0u) d = dk_step_fast<T, HMODE != 0, false, false, false>(tpf, cf, in, nbs, outv, rg);
                else if (wcls == 1u) d = dk_step_fast<T, HMODE != 0, true, false, false>(tpf, cf, in, nbs, outv, rg);
                else d = dk_step_fast<T, HMODE != 0, true, true, false>(tpf, cf, in, nbs, outv, rg);
            }
        } else {
            dk_load_nb(tp, Vin, nbs);
            d = dk_step<T, true, true>(tp, cf, in, nbs, outv, pk, rg);
            if (own_cell)
                *reinterpret_cast<uint4 *>(pit + (long long)(k_target - 1 - k) * pit_stride + c * 16) =
                    make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
        if (LOCAL) {
            asm volatile("" ::"v"(d));  // keep the arithmetic ahead of the test (no sinking past it)
            if (k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        }
        diff = d;
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

// Batched DoorKey grids of width 16 (DoorKey-16x16: BASELINE config 5), one thread per cell, grid
// ROWS as the unit of the thread -> cell map.  Why (round 5): fused_fast_dk_soa keeps the LDS tiles
// indexed by cell while the special-first map hands threads scattered cells, so a 16-lane
// ds_read_b128 group or an 8-lane ds_write_b128 group hits one bank slot with several addresses:
// SQ_LDS_BANK_CONFLICT was 51 % of the LDS-array cycles (profiles/r04_counters/
// summary_doorkey65536.json; tools/dk_bank_sim.py predicts 55 % for that map, 0 for this one).
//  * Lane l of wave w owns cell (row[4w + l/16], l % 16): whole rows move, so a DPP row of 16 lanes is
//    one grid row and the lanes of any 16-lane read group / 8-lane write group own cells of distinct
//    x (mod 16 / mod 8): every tile access below is conflict-free.  Rows are ordered by the wave
//    class their cells need (key / door ahead or under, goal ahead; dk_step_fast's KD / GOAL
//    forms), so the special rows share as few waves as possible, and fully absorbing rows go last.
//  * East / west fronts come from lane +- 1 by DPP (wave_shl / wave_shr, +0 shifted in at the wave's
//    ends): x = 0 and x = 15 are border walls, whose fronts do not matter (ge = 0 below), so only
//    planes 1 and 3 (south / north fronts) go through LDS: two ds_read_b128 and two ds_write_b128
//    per thread and sweep instead of four each (fused_serve_xyd's scheme for DoorKey's V4 groups).
//  * Fronts are geometric: a front state the agent cannot enter is an invalid state holding +0 and
//    V >= +0 (dk_step_fast's argument); the own cell's walkability enters as ge = g or 0, so an
//    absorbing cell yields +0 with no select.
//  * The stop test of sweep k is read right after its barrier, before sweep k+1's arithmetic (the
//    batched loop has other waves to hide it), so when the rule stops, the two register sets hold
//    V_k and V_{k-1} and the tile sweep k read still holds V_{k-1}'s planes: the pi pass (dk_step's
//    per-action form, lowest index on ties) reads its own values and east / west fronts from the
//    V_{k-1} set and its north / south fronts from that tile.
// Same candidates per state, same rule, same pi: V, pi, the stopping sweep and dV are bit-identical
// to fused_fast_dk_soa / the oracle.  LDS (dkrow_*): [slots 256][flags 64][row map 128][cells HWp]
// [tile 0: plane 1 | plane 3][tile 1: ...], each plane PL = HWs + 32 V4 entries, cell c at 16 + c
// (16 zero entries either side: the border rows' north / south reads land there).
__host__ __device__ inline int dkrow_cells_off() { return 256 + 64 + 128; }
__host__ __device__ inline int dkrow_tile_off(int HWp) { return dkrow_cells_off() + (HWp + 15) / 16 * 16; }
__host__ __device__ inline int dkrow_plane(int HWs) { return HWs + 32; }  // V4 entries per plane
__host__ __device__ inline int dkrow_smem_bytes(int HWp, int HWs, int tsize) {
    return dkrow_tile_off(HWp) + 2 * 2 * dkrow_plane(HWs) * 4 * tsize;
}

// Value sweep of one DoorKey cell from geometric fronts (fE / fW: the east / west neighbours' plane
// 0 / 2 values, fS / fN: the south / north neighbours' plane 1 / 3 groups).  Candidates per state as
// dk_step_fast (left, right, self, forward; KD: pickup / toggle targets), one multiply.  KD waves:
//  * pickup (key ahead, has_key 0) and unlocking (a closed door ahead, has_key 1, door_open 0) only
//    apply where the geometric front is an invalid, +0 state (the key cell without the key, the door
//    cell shut), so their target REPLACES the front value (one select, no extra max); only closing
//    an open door (door_open 1: the open door ahead is walkable) is an extra candidate;
//  * the cell's own invalid states (the key / door cells themselves) take ge4[hd] = 0 instead of g,
//    so they yield +0 without a select.
// GOAL waves: a state whose forward move enters the goal is worth exactly 1 where the agent can be
// (the oracle's max(fl(g * M), 1) with fl(g * M) <= g < 1, every value being <= 1) and +0 where it
// cannot, so one select replaces the reward's max (and, in KD waves, the walkability mask the max
// needed): `one` = 1 / 0 per (has_key, door_open) in KD waves, 1 otherwise.
template <typename T, bool GOAL, bool KD, bool DV>
__device__ __forceinline__ T dk_rows_step(uint32_t walk, const uint32_t (&f)[4], uint32_t gdirs, T ge,
                                          const T (&ge4)[4], const T (&in)[16], const T (&fE)[4], const V4<T> &fS,
                                          const T (&fW)[4], const V4<T> &fN, T (&out)[16]) {
    T df[16];
#pragma unroll
    for (int hd = 0; hd < 4; ++hd) {
        const T m02 = vmax(in[hd], in[8 + hd]), m13 = vmax(in[4 + hd], in[12 + hd]);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int l = d * 4 + hd;
            T F = d == 0 ? fE[hd] : (d == 1 ? fS.v[hd] : (d == 2 ? fW[hd] : fN.v[hd]));
            const T xS = in[l];
            const bool key = f[d] & 64u, door = f[d] & 128u;
            if (KD) {
                if (hd == 0) F = key ? in[d * 4 + 2] : F;   // (hk 0, dop 0): pickup -> (hk 1, dop 0)
                if (hd == 1) F = key ? in[d * 4 + 3] : F;   // (hk 0, dop 1): pickup -> (hk 1, dop 1)
                if (hd == 2) F = door ? in[d * 4 + 3] : F;  // (hk 1, dop 0): unlock -> (hk 1, dop 1)
            }
            T M = vmax(vmax((d & 1) ? m02 : m13, xS), F);
            if (KD && (hd & 1)) M = vmax(M, door ? in[d * 4 + (hd >> 1) * 2] : (T)0);  // close -> (hk, 0)
            out[l] = (KD ? ge4[hd] : ge) * M;
        }
    }
    if (GOAL) {  // per direction, a wave-uniform branch (a wave holds one to three of the goal's neighbours)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            if ((gdirs >> d) & 1u) {
#pragma unroll
                for (int hd = 0; hd < 4; ++hd)
                    out[d * 4 + hd] = (f[d] & 16u) ? (KD ? (((walk >> hd) & 1u) ? (T)1 : (T)0) : (T)1) : out[d * 4 + hd];
            }
        }
    }
    if constexpr (!DV) return (T)0;
#pragma unroll
    for (int l = 0; l < 16; ++l) df[l] = vabs(out[l] - in[l]);
    const T a = vmax(vmax(df[0], df[1]), df[2]), b = vmax(vmax(df[3], df[4]), df[5]);
    const T c = vmax(vmax(df[6], df[7]), df[8]), e = vmax(vmax(df[9], df[10]), df[11]);
    const T h = vmax(vmax(df[12], df[13]), df[14]);
    return vmax(vmax(vmax(a, b), c), vmax(vmax(e, h), df[15]));
}

// HWS_C: the workgroup size (HWs) when known at compile time (kWpDkRow16), else 0
template <typename T, bool LOCAL, int HWS_C = 0, typename Done>
__device__ __forceinline__ void fused_dk_rows(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *tiles,
                                              T *slots, uint8_t *flags, uint8_t *rowmap, const T *Vg, T *Vg_out,
                                              int8_t *pig, int &k, int k_target, double &dvl, const Done &done,
                                              int &t_late) {
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // the wave index, an SGPR (late_tid after the loop)
    const bool lane0 = lane == 0;
    const int HW = geo.HW, HWs = HWS_C ? HWS_C : (int)blockDim.x, PL = dkrow_plane(HWs);
    k = __builtin_amdgcn_readfirstlane(k);  // uniform: the sweep count in an SGPR (as fused_wave2_xyd)
    const int nrow = HWs >> 4;  // row slots (rows past H are idle; <= 64: HWs <= 1024)
    // 1. Row classes from the identity map (thread t on cell t): bit 1 KD, bit 0 GOAL, bit 2 walkable.
    {
        uint32_t key = 0;
        if (t < HW) {
            const DkTopo tp0 = dk_topo(cl, geo, t);
            const DkFast q0 = dk_fast_topo(tp0, 0);
            key = (dk_fast_class(q0) & 2u ? 8u : 0u) | (dk_fast_class(q0) & 1u ? 4u : 0u) | (tp0.walk != 0u ? 2u : 0u) |
                  1u;  // 1: a real row (rows past H sort last)
        }
        const unsigned long long b3 = __builtin_amdgcn_ballot_w64(key & 8u), b2 = __builtin_amdgcn_ballot_w64(key & 4u);
        const unsigned long long b1 = __builtin_amdgcn_ballot_w64(key & 2u), b0 = __builtin_amdgcn_ballot_w64(key & 1u);
        if ((lane & 15) == 0) {
            const int sh = lane;  // this lane's 16-lane row segment
            const uint32_t rk = (((b3 >> sh) & 0xFFFFull) ? 8u : 0u) | (((b2 >> sh) & 0xFFFFull) ? 4u : 0u) |
                                (((b1 >> sh) & 0xFFFFull) ? 2u : 0u) | (((b0 >> sh) & 0xFFFFull) ? 1u : 0u);
            rowmap[64 + (t >> 4)] = (uint8_t)rk;
        }
        if (t < 64) flags[t] = 0;
        // the LDS tiles start at +0 (pads included): nothing else writes the pads
        V4<T> *tv = reinterpret_cast<V4<T> *>(tiles);
        for (int i = t; i < 4 * PL; i += HWs) tv[i] = V4<T>{{(T)0, (T)0, (T)0, (T)0}};
        __syncthreads();
        if (t < nrow) {  // stable rank, larger class first
            const uint32_t mine = rowmap[64 + t];
            int rank = 0;
            for (int r = 0; r < nrow; ++r) {
                const uint32_t o = rowmap[64 + r];
                rank += (o > mine || (o == mine && r < t)) ? 1 : 0;
            }
            rowmap[rank] = (uint8_t)t;
        }
        __syncthreads();
    }
    const int row = rowmap[t >> 4];
    const int c = row * 16 + (t & 15);
    const bool own_cell = c < HW;
    const int cc = own_cell ? c : 0;  // idle threads shadow cell 0 (a border wall): they compute +0
    const DkTopo tp = dk_topo(cl, geo, cc);
    const DkFast q = dk_fast_topo(tp, 0);
    // the directions in which some cell of this wave has the goal ahead (wave-uniform)
    uint32_t gdirs = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) gdirs |= (__builtin_amdgcn_ballot_w64((q.f[d] & 16u) != 0u) != 0ull ? 1u : 0u) << d;
    const uint32_t cls = dk_fast_class(q);
    const uint32_t wcls = (__builtin_amdgcn_ballot_w64(cls & 1u) ? 1u : 0u) | (__builtin_amdgcn_ballot_w64(cls & 2u) ? 2u : 0u);
    const T ge = tp.walk != 0u ? cf.g : (T)0;
    T ge4[4];  // per (has_key, door_open): g where the agent may stand, else 0
#pragma unroll
    for (int hd = 0; hd < 4; ++hd) ge4[hd] = ((tp.walk >> hd) & 1u) ? cf.g : (T)0;
    T *const T0 = tiles, *const T1 = tiles + 2 * PL * 4;
    const int o1 = (16 + c) * 4, o3 = (PL + 16 + c) * 4;  // own entries of planes 1 / 3 (T units)
    T A[16], Bv[16];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
        const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 16 + 4 * qd);
#pragma unroll
        for (int j = 0; j < 4; ++j) A[4 * qd + j] = own_cell ? x.v[j] : (T)0;
    }
    *reinterpret_cast<V4<T> *>(T0 + o1) = V4<T>{{A[4], A[5], A[6], A[7]}};
    *reinterpret_cast<V4<T> *>(T0 + o3) = V4<T>{{A[12], A[13], A[14], A[15]}};
    __syncthreads();
    T diff = (T)0;
    // at the stop: pos 0 = V_k in A, V_{k-1} in Bv and tile 1; pos 1 = V_k in Bv, V_{k-1} in A and tile 0
    int pos = 0;
    // One sweep loop per wave form (the class is wave-uniform and fixed for the launch): the loop
    // body is straight-line code, so the two register sets keep their registers across sweeps (a
    // class switch inside the loop made the compiler merge the forms' outputs with copies).  Every
    // loop takes the same barriers and the same (block-uniform) stop decisions.
    auto run = [&](auto goal_c, auto kd_c) {
        constexpr bool GOAL = decltype(goal_c)::value, KD = decltype(kd_c)::value;
        // One sweep in -> out; returns whether another follows (fused_grid calls with work to do, so
        // the first always runs).  The stop test ends the sweep that decides it, right after its
        // barrier: the exits then find V_{k-1} in the sweep's own input set (no copy of it carried
        // through the loop -- round 4's test at the next sweep's start cost 12-24 VGPR moves per sweep).
        auto sweep = [&](const T *Tin, T *Tout, const T (&in)[16], T (&out)[16], const int par) -> bool {
            const V4<T> fS = *reinterpret_cast<const V4<T> *>(Tin + o1 + 64);  // cell c + 16, plane 1
            const V4<T> fN = *reinterpret_cast<const V4<T> *>(Tin + o3 - 64);  // cell c - 16, plane 3
            T fE[4], fW[4];
#pragma unroll
            for (int hd = 0; hd < 4; ++hd) {
                fE[hd] = dpp_shl1_zero(in[hd]);
                fW[hd] = dpp_shr1_zero(in[8 + hd]);
            }
            T d;
            if (LOCAL) d = dk_rows_step<T, GOAL, KD, true>(tp.walk, q.f, gdirs, ge, ge4, in, fE, fS, fW, fN, out);
            else if (k + 1 == k_target) d = dk_rows_step<T, GOAL, KD, true>(tp.walk, q.f, gdirs, ge, ge4, in, fE, fS, fW, fN, out);
            else d = dk_rows_step<T, GOAL, KD, false>(tp.walk, q.f, gdirs, ge, ge4, in, fE, fS, fW, fN, out);
            diff = d;
            *reinterpret_cast<V4<T> *>(Tout + o1) = V4<T>{{out[4], out[5], out[6], out[7]}};
            *reinterpret_cast<V4<T> *>(Tout + o3) = V4<T>{{out[12], out[13], out[14], out[15]}};
            if (LOCAL) {
                const unsigned long long b = __ballot(d >= cf.tol);
                if (lane0) flags[par * 16 + wv] = b != 0ull;
            }
            __syncthreads();
            ++k;
            if (LOCAL) {
                if (k >= geo.max_sweeps) return false;
                // this sweep's flags (<= 4 waves: one dword; else 16 bytes)
                if (HWs <= 256) return *reinterpret_cast<const uint32_t *>(flags + par * 16) != 0u;
                const uint4 f4 = *reinterpret_cast<const uint4 *>(flags + par * 16);
                return (f4.x | f4.y | f4.z | f4.w) != 0u;
            }
            return k < k_target;
        };
        while (true) {
            if (!sweep(T0, T1, A, Bv, 0)) { pos = 1; break; }
            if (!sweep(T1, T0, Bv, A, 1)) { pos = 0; break; }
        }
    };
    using Yes = std::integral_constant<bool, true>;
    using No = std::integral_constant<bool, false>;
    if (wcls == 0u) run(No{}, No{});
    else if (wcls == 1u) run(Yes{}, No{});
    else run(Yes{}, Yes{});
    const int t2 = late_tid(wv);
    t_late = t2;
    dvl = (double)block_max_tid(diff, slots, 0, t2);
    done(k, dvl);
    // The pi pass re-derives the thread's cell and topology from LDS (row map and cells are still
    // there) instead of keeping them live across the sweep loop: at 6 waves per SIMD (80 VGPRs) the
    // loop leaves no room for them, and the compiler spilled them to scratch -- 76 B per thread
    // stored to memory once per launch, 0.85 GB of the DoorKey-16 x 65536 launch's HBM writes
    // (round-5 verdict).  The opaque copy of the thread index keeps the compiler from reusing the
    // values computed before the loop.
    const int c2 = rowmap[t2 >> 4] * 16 + (t2 & 15);
    const bool own2 = c2 < HW;
    const DkTopo tp2 = dk_topo(cl, geo, own2 ? c2 : 0);
    const int p1 = (16 + c2) * 4, p3 = (PL + 16 + c2) * 4;
    T vk[16], vp[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) {
        vk[l] = pos ? Bv[l] : A[l];
        vp[l] = pos ? A[l] : Bv[l];
    }
    const T *Tp = pos ? T0 : T1;
    V4<T> nbs[4];
#pragma unroll
    for (int hd = 0; hd < 4; ++hd) {
        nbs[0].v[hd] = dpp_shl1_zero(vp[hd]);
        nbs[2].v[hd] = dpp_shr1_zero(vp[8 + hd]);
    }
    nbs[1] = *reinterpret_cast<const V4<T> *>(Tp + p1 + 64);
    nbs[3] = *reinterpret_cast<const V4<T> *>(Tp + p3 - 64);
    if (own2) {
        // V_k leaves first, so its registers are free for the per-action pi pass
#pragma unroll
        for (int qd = 0; qd < 4; ++qd)
            *reinterpret_cast<V4<T> *>(Vg_out + c2 * 16 + 4 * qd) = V4<T>{{vk[4 * qd], vk[4 * qd + 1], vk[4 * qd + 2], vk[4 * qd + 3]}};
        T tmp[16];
        uint32_t pk[4];
        dk_step<T, true>(tp2, cf, vp, nbs, tmp, pk);
        *reinterpret_cast<uint4 *>(pig + c2 * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
}

// Batched DoorKey grids with each cell's 16 states split over two threads by has_key: the first
// HWs threads (whole waves) own (cell, has_key 0), the next HWs threads (cell, has_key 1), 8 states
// (dir, door_open) each.  Per thread that halves the values held per register set (own, the next
// sweep's, the four front pairs), which is what capped fused_fast_dk_soa at 4 waves per SIMD
// (107 VGPRs); the workgroup doubles to 2*HWs threads.  has_key is wave-uniform, so the half's
// transition form is a uniform branch.  Only pickup (has_key 0, key ahead -> the same (dir,
// door_open) with has_key 1) crosses the halves: it reads the other half's values of its own cell
// from the input tile (same bits as that thread's registers), only in waves with a key / door.
// LDS tiles: value (x, d, hk, dop) at ((hk*4 + d)*HWs + x)*2 + dop, so a thread's front pair and
// own pairs are unit-stride 8-B accesses.  Same candidates per state as dk_step_fast / dk_step
// (max is exact and order-free; the pi pass keeps dk_step's action order), so V, pi and the
// stopping sweep are bit-identical.
struct DkHalf {
    uint32_t walk;  // as DkTopo
    uint32_t fp;    // byte d: DkFast::f[d] (goal / key / door ahead), packed to save registers
    int nb[4];      // LDS index of the front pair forward reads (cell 0's when none)
};
template <typename T, bool HK0, bool FH, bool GOAL, bool KD>
__device__ __forceinline__ T dkh_step_fast(const DkHalf &tp, const Coef<T> &cf, const T (&own)[8], const T (&oth)[8],
                                           const V2<T> (&nbs)[4], T (&outv)[8], T rg = (T)1) {
    constexpr int hk = HK0 ? 0 : 1;
    T dv = (T)0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.fp >> (8 * d);
        const bool key = f & 64u, door = f & 128u;
        const T tqd = (f & 16u) ? (FH ? rg : (T)1) : (T)0;
#pragma unroll
        for (int dop = 0; dop < 2; ++dop) {
            const int hd = hk * 2 + dop, l = d * 2 + dop;
            const T xS = own[l];
            T M = vmax(vmax(own[((d + 3) & 3) * 2 + dop], own[((d + 1) & 3) * 2 + dop]), vmax(xS, nbs[d].v[dop]));
            if (KD) {  // pickup -> (d, 1, dop); toggle -> close (dop 1: (d, hk, 0)) / unlock (hk 1, dop 0: (d, 1, 1))
                T cand = (T)0;
                if (!hk) cand = key ? oth[l] : cand;
                if (dop) cand = door ? own[d * 2] : cand;
                else if (hk) cand = door ? own[d * 2 + 1] : cand;
                M = vmax(M, cand);
            }
            T best = cf.g * M;
            if (GOAL) best = vmax(best, tqd);
            if (KD) best = ((tp.walk >> hd) & 1u) ? best : (T)0;
            outv[l] = best;
            dv = vmax(dv, vabs(best - xS));  // running max: two live temporaries, not eight
        }
    }
    return dv;
}

// pi of one half (dk_step's WRITE_PI form restricted to has_key = hk): pk[d] = the 2 lanes' bytes
template <typename T>
__device__ __forceinline__ void dkh_pi(const DkTopo &tp, const Coef<T> &cf, int hk, const T (&own)[8], const T (&oth)[8],
                                       const V2<T> (&nbs)[4], uint32_t (&pk)[4]) {
    T gv[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) gv[l] = cf.g * own[l];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.f[d];
        const bool goal = f & 16u, lava = f & 32u, key = f & 64u, door = f & 128u;
        pk[d] = 0;
#pragma unroll
        for (int dop = 0; dop < 2; ++dop) {
            const int l = d * 2 + dop, hd = hk * 2 + dop;
            const T qS = gv[l];
            const T qL = gv[((d + 3) & 3) * 2 + dop];
            const T qR = gv[((d + 1) & 3) * 2 + dop];
            const T qM = ((f >> hd) & 1u) ? cf.g * nbs[d].v[dop] : qS;
            const T qF = goal ? (T)1 : (lava ? (T)0 : qM);
            const T qP = (!hk && key) ? cf.g * oth[l] : qS;
            const T qD = dop ? gv[d * 2] : (hk ? gv[d * 2 + 1] : qS);
            const T qT = door ? qD : qS;
            T best = qL;
            int arg = 0;
            if (qR > best) { best = qR; arg = 1; }
            if (qF > best) { best = qF; arg = 2; }
            if (qP > best) { best = qP; arg = 3; }
            if (qT > best) { best = qT; arg = 4; }
            const bool valid = (tp.walk >> hd) & 1u;
            pk[d] |= (uint32_t)(uint8_t)(valid ? arg : -1) << (8 * dop);
        }
    }
}

// HW: the plane stride geo.HWs (a multiple of 64, so has_key is uniform per wave) known at compile
// time: every tile / plane offset is an instruction immediate, and a thread keeps one LDS address
// per front cell instead of one per (tile, plane) pair.
template <typename T, bool LOCAL, int HW, typename Done>
__device__ __forceinline__ void fused_dk_half(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *V0,
                                              T *slots, uint8_t *flags, const T *Vg, T *Vg_out, int8_t *pig, int &k,
                                              int k_target, double &dvl, const Done &done) {
    T *V1 = V0 + 16 * HW;  // = smem_layout's second tile (Ss = 16 * HWs)
    const int hk = (int)threadIdx.x >= HW ? 1 : 0;
    const int c = threadIdx.x - hk * HW;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int k_start = k;
    auto tix = [&](int x, int d, int h) { return ((h * 4 + d) * HW + x) * 2; };
    DkHalf tpf;  // front pair read by forward (cell 0's when none; see dk_fast_topo)
    uint32_t cls;
    {
    const DkTopo tp = dk_topo(cl, geo, cc);  // (resolved again for the pi pass: fewer live registers)
    DkFast q;
    q.walk = tpf.walk = tp.walk;
    tpf.fp = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t f = tp.f[d];
        const bool reads = tp.walk != 0u && !(f & 48u) && (f & 15u) != 0u;
        tpf.nb[d] = tix(reads ? (tp.nb[d] >> 4) : 0, d, hk);
        q.f[d] = tp.walk != 0u ? (f & (16u | 64u | 128u)) : 0u;
        tpf.fp |= q.f[d] << (8 * d);
    }
    cls = dk_fast_class(q);
    }
    const uint32_t wcls = (__builtin_amdgcn_ballot_w64(cls & 1u) ? 1u : 0u) | (__builtin_amdgcn_ballot_w64(cls & 2u) ? 2u : 0u);
    T own[8];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const V2<T> x = k == 0 ? V2<T>{{(T)0, (T)0}} : *reinterpret_cast<const V2<T> *>(Vg + cc * 16 + d * 4 + hk * 2);
        own[2 * d] = x.v[0];
        own[2 * d + 1] = x.v[1];
        *reinterpret_cast<V2<T> *>(V0 + tix(c, d, hk)) = x;
    }
    __syncthreads();
    int cur = 0, parity = 0;
    T diff = (T)0;
    auto sweep = [&](const T *Vin, T *Vout, const T (&in)[8], T (&outv)[8]) -> bool {
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        V2<T> nbs[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) nbs[d] = *reinterpret_cast<const V2<T> *>(Vin + tpf.nb[d]);
        T d;
        if (wcls == 0u) {
            const T (&none)[8] = in;  // unused without KD
            d = hk ? dkh_step_fast<T, false, false, false, false>(tpf, cf, in, none, nbs, outv)
                   : dkh_step_fast<T, true, false, false, false>(tpf, cf, in, none, nbs, outv);
        } else if (wcls == 1u) {
            const T (&none)[8] = in;
            d = hk ? dkh_step_fast<T, false, false, true, false>(tpf, cf, in, none, nbs, outv)
                   : dkh_step_fast<T, true, false, true, false>(tpf, cf, in, none, nbs, outv);
        } else if (hk) {
            d = dkh_step_fast<T, false, false, true, true>(tpf, cf, in, in, nbs, outv);
        } else {
            T oth[8];  // the has_key-1 half's V_k of this cell (pickup)
#pragma unroll
            for (int dd = 0; dd < 4; ++dd) {
                const V2<T> x = *reinterpret_cast<const V2<T> *>(Vin + tix(c, dd, 1));
                oth[2 * dd] = x.v[0];
                oth[2 * dd + 1] = x.v[1];
            }
            d = dkh_step_fast<T, true, false, true, true>(tpf, cf, in, oth, nbs, outv);
        }
        if (LOCAL) {
            asm volatile("" ::"v"(d));  // keep the arithmetic ahead of the test (no sinking past it)
            if (k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        }
        diff = d;
#pragma unroll
        for (int dd = 0; dd < 4; ++dd)
            *reinterpret_cast<V2<T> *>(Vout + tix(c, dd, hk)) = V2<T>{{outv[2 * dd], outv[2 * dd + 1]}};
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    T alt[8];
    while (true) {
        if (!sweep(V0, V1, own, alt)) { cur = 0; break; }
        if (!sweep(V1, V0, alt, own)) {
            cur = 1;
#pragma unroll
            for (int l = 0; l < 8; ++l) own[l] = alt[l];
            break;
        }
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    if (own_cell) {  // V_k (`own`) out first (frees its registers), then pi on V_{k-1} (buffer cur ^ 1)
#pragma unroll
        for (int d = 0; d < 4; ++d)
            *reinterpret_cast<V2<T> *>(Vg_out + c * 16 + d * 4 + hk * 2) = V2<T>{{own[2 * d], own[2 * d + 1]}};
        const DkTopo tp = dk_topo(cl, geo, cc);
        const T *Vp = cur ? V0 : V1;
        T op[8], oth[8];
        V2<T> nbs[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const V2<T> x = *reinterpret_cast<const V2<T> *>(Vp + tix(c, d, hk));
            const V2<T> y = *reinterpret_cast<const V2<T> *>(Vp + tix(c, d, 1));
            op[2 * d] = x.v[0];
            op[2 * d + 1] = x.v[1];
            oth[2 * d] = y.v[0];
            oth[2 * d + 1] = y.v[1];
            nbs[d] = *reinterpret_cast<const V2<T> *>(Vp + tix(tp.nb[d] >> 4, d, hk));
        }
        uint32_t pk[4];
        dkh_pi<T>(tp, cf, hk, op, oth, nbs, pk);
#pragma unroll
        for (int d = 0; d < 4; ++d) *reinterpret_cast<uint16_t *>(pig + c * 16 + d * 4 + hk * 2) = (uint16_t)pk[d];
    }
}

// Batched DoorKey grids on ONE LDS tile (fp32): the two 16 KB tiles of fused_fast_dk_soa cap a CU
// at 4 resident 16x16 grids, one tile at 8.  A sweep reads the neighbours' V_k from the tile,
// passes a barrier (every read is done), tests the previous sweep's stop flags (read before the
// barrier, so the test waits for nothing), computes V_{k+1} and overwrites the tile, then passes
// the usual barrier: two barriers per sweep, same arithmetic.  The own cell's V_{k-1} and the
// neighbour values it met stay in the alternating register sets, which is what the final pi pass
// (argmax on V_{k-1}) needs; a sweep stopped by the test computes nothing.
template <typename T, bool LOCAL, typename Done>
__device__ __forceinline__ void fused_fast_dk_1t(const Geo &geo, const Coef<T> &cf, const uint8_t *cl, T *Vt,
                                                 T *slots, uint8_t *flags, const T *Vg, T *Vg_out, int8_t *pig,
                                                 int &k, int k_target, double &dvl, const Done &done) {
    const int c = threadIdx.x;
    const int cc = c < geo.HW ? c : 0;
    const bool own_cell = c < geo.HW;
    const int HW = geo.HWs;
    const int k_start = k;
    const DkTopo tp = dk_topo_soa(cl, geo, cc);
    T a[16], b[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const V4<T> x = k == 0 ? V4<T>{{(T)0, (T)0, (T)0, (T)0}} : *reinterpret_cast<const V4<T> *>(Vg + cc * 16 + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) a[4 * q + j] = x.v[j];
        *reinterpret_cast<V4<T> *>(Vt + (q * HW + c) * 4) = x;
    }
    __syncthreads();
    int parity = 0;
    T diff = (T)0;
    V4<T> na[4], nb[4];
    auto sweep = [&](const T (&in)[16], T (&outv)[16], V4<T> (&nbs)[4]) -> bool {
        if (LOCAL ? k >= geo.max_sweeps : k >= k_target) return false;
        uint4 fl = make_uint4(0u, 0u, 0u, 0u);
        if (LOCAL) fl = *reinterpret_cast<const uint4 *>(flags + (parity ^ 1) * 16);
        dk_load_nb(tp, Vt, nbs);
        __syncthreads();  // every read of V_k is done before the tile is overwritten
        if (LOCAL && k > k_start && (fl.x | fl.y | fl.z | fl.w) == 0u) return false;
        uint32_t pk[4];
        diff = dk_step<T, false>(tp, cf, in, nbs, outv, pk);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<V4<T> *>(Vt + (q * HW + c) * 4) =
                V4<T>{{outv[4 * q], outv[4 * q + 1], outv[4 * q + 2], outv[4 * q + 3]}};
        if (LOCAL) flag_write(diff >= cf.tol, flags, parity);
        __syncthreads();
        parity ^= 1;
        ++k;
        return true;
    };
    int last = 0;  // 0: the last committed sweep was a -> b with na; 1: b -> a with nb (one always commits)
    while (true) {
        if (!sweep(a, b, na)) break;
        last = 0;
        if (!sweep(b, a, nb)) break;
        last = 1;
    }
    dvl = (double)block_max(diff, slots, 0);
    done(k, dvl);
    if (own_cell) {  // pi on V_{k-1}: the last committed sweep's input set and the neighbours it read
        T tmp[16];
        uint32_t pk[4];
        if (last == 0) dk_step<T, true>(tp, cf, a, na, tmp, pk);
        else dk_step<T, true>(tp, cf, b, nb, tmp, pk);
        *reinterpret_cast<uint4 *>(pig + c * 16) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // V_k (element selects: a pointer to either set would put both in scratch)
            V4<T> x;
#pragma unroll
            for (int j = 0; j < 4; ++j) x.v[j] = last == 0 ? b[4 * q + j] : a[4 * q + j];
            *reinterpret_cast<V4<T> *>(Vg_out + c * 16 + 4 * q) = x;
        }
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
}  // namespace mgdp
