/*
 * mgdp.h -- C ABI of the MI355X Minigrid step / value-iteration engine (libmgdp.so).
 *
 * The reference (Farama Minigrid 2.3.1, /root/reference) is pure Python: its operator surface is
 * the gymnasium.Env plugin MiniGridEnv (minigrid/minigrid_env.py:24) registered under the
 * "gymnasium.envs" entry point (pyproject.toml:47-48 -> minigrid/__init__.py:23).  This header is
 * the native boundary behind that surface.  Each entry point cites the reference interface it
 * replaces.  The reference has no value-iteration code; the mgdp_vi_* entry
 * points implement the build-defined DP of DESIGN.md "A9" whose transition is the reference step().
 *
 * Conventions
 *   - Plain C types only; no C++ or Python types cross this boundary.
 *   - Every function returns int: MGDP_OK (0) or a negative MGDP_E_* code; mgdp_last_error()
 *     returns a thread-local message for the last failure on the calling thread.
 *   - The caller owns host buffers; the library owns the device buffers of a handle.  Entry points
 *     named *_device take device pointers and run asynchronously on the handle's stream.
 *   - A handle is bound to one HIP device and is not thread-safe (like MiniGridEnv,
 *     tests/test_envs.py:42-43).  Multi-GPU = one process and one handle per GPU.
 *   - Grid cells use the reference codes OBJECT_TO_IDX / COLOR_TO_IDX / door state
 *     (minigrid/core/constants.py:20-46).  "cells" arrays are row-major [y][x] like Grid.grid
 *     (minigrid/core/grid.py:35,72); "enc" arrays are the x-major [x][y][3] layout of
 *     Grid.encode() (minigrid/core/grid.py:244-268).
 */
#ifndef MGDP_H
#define MGDP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGDP_ABI_VERSION 12

enum {
    MGDP_OK = 0,
    MGDP_E_INVALID = -1,     /* bad argument                             (Python: ValueError)      */
    MGDP_E_HIP = -2,         /* HIP runtime failure / no device          (Python: RuntimeError)    */
    MGDP_E_UNSUPPORTED = -3, /* grid contents outside the selected model (Python: ValueError)      */
    MGDP_E_ACTION = -4,      /* "Unknown action", minigrid_env.py:579-580 (Python: ValueError)      */
    MGDP_E_BOUNDS = -5,      /* grid access out of range, grid.py:66-77  (Python: AssertionError)  */
};

/* ---------------------------------------------------------------------------------------------- */
/* Library                                                                                          */
/* ---------------------------------------------------------------------------------------------- */
const char *mgdp_last_error(void);
int mgdp_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int mgdp_device_count(int32_t *n);
/* Restrict the CALLING thread to the CPUs of `device`'s NUMA node (sysfs local_cpulist, within the
 * thread's current affinity); *ncpus_out = the CPUs kept, 0 if the node is unknown or none of its
 * CPUs is allowed (the affinity is then left unchanged).  Call it before mgdp_vi_create on the
 * thread that will solve: a served lone-grid solve polls host memory, and its latency depends on
 * which socket the polling thread and the handle's host-mapped words live on (ABI 6). */
int mgdp_pin_host_thread(int32_t device, int32_t *ncpus_out);

/* ---------------------------------------------------------------------------------------------- */
/* Value iteration over batches of grids (build-defined DP; transition = MiniGridEnv.step,          */
/* minigrid_env.py:520-583).  DESIGN.md "A9" fixes every convention:                                */
/*   MGDP_MODEL_XYD      s = (y*W + x)*4 + dir, A = 7 (Discrete(7), minigrid_env.py:63);             */
/*                       cells in {empty, wall, floor, goal, lava} (Empty/FourRooms/LavaCrossing)   */
/*   MGDP_MODEL_DOORKEY  s = (((y*W + x)*4 + dir)*2 + has_key)*2 + door_open, A = 5 lanes            */
/*                       (left, right, forward, pickup, toggle; doorkey.py:25-33); exactly one       */
/*                       door and one key of its colour                                             */
/*   R = 1 on entering the goal (terminal), lava terminal with R = 0; absorbing states V = 0, pi=-1 */
/*   Jacobi V_{k+1} = max_a Q_k, lowest action index wins ties; stop after sweep k when             */
/*   max |V_k - V_{k-1}| over all grids of the run < tol (one global rule, also across GPUs).       */
/*   slip_p >= 0 applies StochasticActionWrapper (wrappers.py:775-796) transition probabilities     */
/*   (XYD only): Q = p*Qd[a] + ((1-p)/6) * (((((Qd0+Qd1)+Qd2)+Qd3)+Qd4)+Qd5).                       */
/* ---------------------------------------------------------------------------------------------- */
enum { MGDP_MODEL_XYD = 0, MGDP_MODEL_DOORKEY = 1 };
enum { MGDP_F32 = 0, MGDP_F64 = 1 };
enum {
    MGDP_METHOD_FUSED = 0, /* LDS-resident: one workgroup per grid runs many sweeps on chip        */
    MGDP_METHOD_SWEEP = 1, /* one launch per Jacobi sweep, V double-buffered in HBM                */
};
enum {
    MGDP_MAP_CELL = 0, /* one thread per grid cell updates that cell's 4 (or 16) states            */
    MGDP_MAP_SA = 1,   /* one thread per (state, action), 8 lanes per state, wave max-reduce      */
};
/* DP options from the reference's own semantics (fused + MGDP_MAP_CELL only):
 *   lava_mode MGDP_LAVA_NODEATH: NoDeath(no_death_types=("lava",), death_cost), wrappers.py:799-872
 *     -- lava cells are states, entering lava gives R = death_cost and does not terminate (XYD).
 *   horizon H > 0: finite-horizon DP over step_count t = 0..H-1 (H = the env's max_steps):
 *     V_H = 0, V_t = max_a Q_t with the exact time-dependent goal reward of _reward()
 *     (minigrid_env.py:235-240; step_count is incremented before it, :522; truncation at
 *     step_count >= max_steps, :582-583, is V_H = 0).  Exactly H backward sweeps, no stopping
 *     rule; V / pi report t = 0; flag MGDP_KEEP_POLICY_T keeps pi_t for every t. */
enum { MGDP_LAVA_TERMINAL = 0, MGDP_LAVA_NODEATH = 1 };
enum { MGDP_KEEP_POLICY_T = 1 };

typedef struct {
    int32_t model;      /* MGDP_MODEL_*                                                            */
    int32_t dtype;      /* MGDP_F32 | MGDP_F64: arithmetic and storage type of V                    */
    int32_t method;     /* MGDP_METHOD_*                                                           */
    int32_t mapping;    /* MGDP_MAP_*                                                              */
    int32_t B, W, H;    /* grids in this handle and their size                                     */
    int32_t max_sweeps; /* hard cap on sweeps                                                      */
    int32_t device;     /* HIP device ordinal                                                      */
    int32_t reserved;
    double gamma;       /* discount                                                                */
    double tol;         /* stopping threshold on max|V_k - V_{k-1}|                                 */
    double slip_p;      /* < 0: deterministic; else keep-action probability (XYD only)            */
    int32_t horizon;    /* 0: discounted, stopping rule; H > 0: finite horizon (see above)         */
    int32_t lava_mode;  /* MGDP_LAVA_TERMINAL | MGDP_LAVA_NODEATH                                 */
    int32_t flags;      /* MGDP_KEEP_POLICY_T                                                      */
    int32_t reserved2;
    double death_cost;  /* NoDeath reward for entering lava (the wrapper's death_cost)             */
} mgdp_vi_desc;

typedef struct mgdp_vi mgdp_vi;

int mgdp_vi_create(const mgdp_vi_desc *desc, mgdp_vi **out);
int mgdp_vi_destroy(mgdp_vi *vi);
/* Launch on this hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream. */
int mgdp_vi_set_stream(mgdp_vi *vi, void *hip_stream);
/* Upload B*H*W row-major OBJECT_TO_IDX cell codes (host).  Validates them against the model:
 * MGDP_E_UNSUPPORTED if a cell type is outside the model or a border cell is walkable.  With a
 * persistent lone-grid server resident (see mgdp_vi_solve) the grid is staged in host-mapped
 * memory and handed to the server with the next request: no stream drain, no relaunch. */
int mgdp_vi_load_cells(mgdp_vi *vi, const uint8_t *cells);
/* Same from device memory (already validated by the caller).  On the handle's own stream a
 * resident lone-grid server reads the bytes itself with its next request: they must then be
 * complete before the call and stay valid and unchanged until the next solve returns (or, if no
 * solve follows, until the next call that uses the handle's stream).  On a caller-bound stream
 * (mgdp_vi_set_stream) they are copied on that stream, ordered after the caller's earlier work. */
int mgdp_vi_load_cells_device(mgdp_vi *vi, const uint8_t *d_cells);

/* Whole solve on one device: V_0 = 0, sweeps until the global rule stops.  Synchronous.
 * A lone grid (B = 1, fused, MGDP_MAP_CELL) is served by a persistent workgroup that stays
 * resident on the handle's stream between solves (no launch per solve); it leaves on any other
 * call that uses the stream, after 100 us without a request, or after 2 s.  MGDP_PERSISTENT=0 in
 * the environment (read at create) turns it off. */
int mgdp_vi_solve(mgdp_vi *vi, int32_t *sweeps_out, double *dv_out, int32_t *converged_out);
/* mgdp_vi_solve, after which a persistent lone-grid server leaves at once instead of idling out
 * (the caller has no further solve for now); the next solve relaunches it.  Same results. */
int mgdp_vi_solve_last(mgdp_vi *vi, int32_t *sweeps_out, double *dv_out, int32_t *converged_out);
/* *on = 1 if mgdp_vi_solve on this handle goes through the persistent server. */
int mgdp_vi_persistent(const mgdp_vi *vi, int32_t *on);
/* Name of the kernel mgdp_vi_kernel_time times on this handle (as rocprofv3 lists it): vi_serve_kernel,
 * vi_fused_kernel, vi_fused_opts_kernel, vi_sweep_pipe_kernel or vi_sweep_kernel; NULL on error. */
const char *mgdp_vi_kernel_name(const mgdp_vi *vi);
/* Which loop of that kernel the handle runs (ABI 11), e.g. "serve_ew", "wave2", "dk_rows", "dk_half",
 * "dk_soa", "sweep_pipe" (DESIGN.md section 4 names each); NULL on error.  Diagnostics and tests. */
const char *mgdp_vi_variant(const mgdp_vi *vi);

/* Multi-device protocol: every rank calls
 *   mgdp_vi_reset -> mgdp_vi_run_local(&k_local) -> mgdp_vi_local_result(&k, &dv_own, &k_min)
 *   -> all-reduce(MAX) {k, dv_own} -> mgdp_vi_run_to(K, &dv)
 *   -> [only if the all-reduced dv_own != 0] all-reduce(MAX) dv;
 *   while (dv >= tol && k < max_sweeps) { mgdp_vi_sweep(&dv); all-reduce; } -> mgdp_vi_finish(K).
 * Because each grid's Jacobi trajectory is independent of the others, this yields exactly the
 * V_K of the single global rule.  dv_own = 0 everywhere means every grid ended its own rule at an
 * exact fixed point (V_k == V_{k-1} bit for bit; a sweep is a function of V alone), so every later
 * sweep changes nothing and dV at K is 0 on every rank: one all-reduce per solve then suffices. */
int mgdp_vi_reset(mgdp_vi *vi);
/* Each grid sweeps until its own max|dV| < tol (or max_sweeps); returns max sweeps over grids. */
int mgdp_vi_run_local(mgdp_vi *vi, int32_t *k_local_max);
/* The last launch's reduction: max / min sweeps over the grids and the max|dV| of their last sweeps
 * (after mgdp_vi_run_local: each grid's own stopping sweep). */
int mgdp_vi_local_result(const mgdp_vi *vi, int32_t *k_max, double *dv, int32_t *k_min);
/* Continue every grid to exactly k_target sweeps; dv_out = max over grids of |dV| at sweep k. */
int mgdp_vi_run_to(mgdp_vi *vi, int32_t k_target, double *dv_out);
/* One more Jacobi sweep of every grid (all at the same sweep index); dv_out as above. */
int mgdp_vi_sweep(mgdp_vi *vi, double *dv_out);
/* Extract pi from the last sweep and publish sweeps/converged for mgdp_vi_get_*. */
int mgdp_vi_finish(mgdp_vi *vi, int32_t sweeps);
/* Checkpoint / resume (ABI 7; fused method, no horizon): continue a solve that stopped at sweep k
 * before converging (a max_sweeps cap) from its state {V_k (B*S values of the handle's dtype, as
 * mgdp_vi_get_values returns them), k, dV_k} -- on a handle of the same grids and parameters
 * whose max_sweeps exceeds k (a solve capped at max_sweeps resumes on a handle with a larger cap,
 * not on the capped one).  Jacobi is memoryless given V_k: the result (global stopping sweep, V,
 * pi, dV) is bit-identical to the uninterrupted solve.  k in [1, max_sweeps); dV >= tol (a
 * converged checkpoint is final: its pi is not rebuildable from V_k).  The C ABI cannot tell
 * whose V it is given: the Python checkpoint carries the grids' digest and the parameters and
 * ValueIteration.resume refuses a mismatch. */
int mgdp_vi_resume(mgdp_vi *vi, const void *V, int32_t k, double dv, int32_t *sweeps_out, double *dv_out,
                   int32_t *converged_out);

/* The same protocol with no host round trip between its steps (fused method, no horizon / lava
 * options; distributed.py drives it over RCCL).  d_pub / d_k are caller-owned DEVICE int64 buffers
 * ordered on the handle's stream (mgdp_vi_set_stream):
 *   mgdp_vi_reset -> mgdp_vi_run_local_dev(p) -> all-reduce(MAX) p[0..1] on the stream
 *   -> mgdp_vi_run_to_dev_sync(p, &K, &dv, &dv_own)   (one wait on host-mapped words)
 *   -> [only if dv_own != 0: p[5] <- dv, all-reduce(MAX) p[5], host read]
 *   -> mgdp_vi_set_result(K, dv) -> (rare fallback: mgdp_vi_sweep + host all-reduces) -> finish.
 * A launch writes d_pub[0..3] = {max sweeps over the shard's grids, max|dV| as IEEE-754 bits
 * (non-negative doubles order like their bits), min sweeps, 0} (a device buffer carries no epoch); run_local_dev only
 * enqueues. */
int mgdp_vi_run_local_dev(mgdp_vi *vi, int64_t *d_pub);
/* Every grid to exactly the sweep *d_k (read on the device when the launch starts); enqueue only. */
int mgdp_vi_run_to_dev(mgdp_vi *vi, const int64_t *d_k, int64_t *d_pub);
/* Every grid to exactly K = d_kdv[0] (read on the device); waits for the launch's result on the
 * host without a stream synchronisation: k_out = K, dv_out = this shard's max|dV| at sweep K,
 * dv_rule_out = d_kdv[1] read as a double (the all-reduced own-rule dV of run_local_dev). */
int mgdp_vi_run_to_dev_sync(mgdp_vi *vi, const int64_t *d_kdv, int32_t *k_out, double *dv_out,
                            double *dv_rule_out);
/* Hand the all-reduced K and dV back to the handle (every grid is at sweep K). */
int mgdp_vi_set_result(mgdp_vi *vi, int32_t k, double dv);

/* The sharded solve behind the C ABI (ABI 11): the same protocol with its collectives issued by the
 * library on a communicator it owns -- RCCL over xGMI (librccl, loaded at the first mgdp_comm_* call:
 * MGDP_RCCL_LIB, else the copy already mapped into the process, e.g. PyTorch's, else librccl.so.1).
 * Bootstrap: one rank calls mgdp_comm_unique_id and hands the 128 bytes to every rank through any
 * side channel (a torch.distributed store, MPI, a file); every rank then calls mgdp_comm_create with
 * its rank and device.  One communicator per process and device, shared by its handles. */
typedef struct mgdp_comm mgdp_comm;
/* 0 when librccl can be loaded in this process (ABI 12).  A local check with no communication: every
 * rank calls it and the ranks agree (e.g. a MIN all-reduce of the flags over their bootstrap group)
 * BEFORE any of them calls mgdp_comm_unique_id / mgdp_comm_create, which are collective (a failure
 * inside ncclCommInitRank itself leaves the other ranks waiting and cannot be recovered from). */
int mgdp_comm_available(void);
int mgdp_comm_unique_id(uint8_t *id_out /* 128 bytes */);
int mgdp_comm_create(const uint8_t *id /* 128 bytes */, int32_t nranks, int32_t rank, int32_t device,
                     mgdp_comm **out);
/* The host communicator (ABI 12): the same collectives through a shared-memory segment of this host,
 * /dev/shm<name> (name = "/..." with no other "/"), for ranks that cannot form an RCCL communicator
 * -- several ranks on ONE GPU, which RCCL refuses -- e.g. tests of mgdp_vi_solve_sharded at world > 1
 * on a one-GPU box.  Each device all-reduce becomes a stream synchronisation, a host MAX and a copy
 * back (a test and rehearsal path, not the xGMI one).  Every rank opens the segment (created
 * zero-filled by the first); the caller picks a name no earlier run used and removes the file once
 * every rank has opened it (the mappings stay valid).  A collective waits at most 120 s for its
 * peers, then fails with MGDP_E_INVALID. */
int mgdp_comm_create_host(const char *name, int32_t nranks, int32_t rank, int32_t device, mgdp_comm **out);
int mgdp_comm_destroy(mgdp_comm *comm);
/* Synchronous MAX all-reduce of n int64 host values in place (for ranks that drive the protocol from
 * the host: an empty shard, the sweep method, DP options -- they join the same collectives). */
int mgdp_comm_allreduce_max(mgdp_comm *comm, int64_t *vals, int32_t n);
/* All-reduces issued on the communicator so far, its size and this process's rank. */
int mgdp_comm_stats(const mgdp_comm *comm, int64_t *allreduces, int32_t *nranks, int32_t *rank);
/* Host waits on the GPU so far (ABI 12): one per sharded solve (its run_to result), one per dV(K) or
 * fallback-sweep all-reduce and per mgdp_comm_allreduce_max, and with the host kind one more per
 * device all-reduce; kind: 0 RCCL, 1 host. */
int mgdp_comm_host_waits(const mgdp_comm *comm, int64_t *waits, int32_t *kind);
/* One sharded solve of this rank's handle (fused method, no horizon / lava options), every rank of
 * the communicator at once: reset -> run_local_dev -> MAX all-reduce of {K, own-rule dV bits} on the
 * handle's stream -> gate / run_to(K) with one host wait on host-mapped words -> [only if the
 * all-reduced own-rule dV != 0: MAX all-reduce of dV(K)] -> rounding-level fallback sweeps, each
 * with one all-reduce -> finish.  Host-driven peers issue the same collectives in the same order
 * through mgdp_comm_allreduce_max: {k, dV bits} (2 words), then dV(K) bits (1 word) only if the
 * all-reduced dV bits are non-zero, then one word per fallback sweep while dV >= tol and
 * k < max_sweeps.  Results as mgdp_vi_solve (V and pi of the global rule, bit-identical to one global
 * Jacobi loop over every rank's grids).  Sharded solves of several handles on one communicator must
 * not overlap (one host thread calling them in turn): they share its device protocol words. */
int mgdp_vi_solve_sharded(mgdp_vi *vi, mgdp_comm *comm, int32_t *sweeps_out, double *dv_out,
                          int32_t *converged_out);

/* Results (host).  V: B*S of float or double per dtype; pi: B*S int8 (-1 = absorbing state). */
int mgdp_vi_get_values(mgdp_vi *vi, void *V);
int mgdp_vi_get_policy(mgdp_vi *vi, int8_t *pi);
/* Finite horizon with MGDP_KEEP_POLICY_T: pi_t as H*B*S int8, t-major (pi_t[t][b][s]). */
int mgdp_vi_get_policy_t(mgdp_vi *vi, int8_t *pi_t);
/* Per-sweep global max|dV| (method SWEEP only; fused runs record only the last): n <= max_sweeps */
int mgdp_vi_get_dv_trace(mgdp_vi *vi, double *trace, int32_t n);
/* Sweeps each grid executed (ABI 9; ABI 11: on every path), B int32: the sweep index each grid's
 * last computed sweep reached.  A grid whose own rule stopped at an exact fixed point (|dV| = 0)
 * reports that sweep -- its V and pi are those of every later sweep, so the global rule's remaining
 * sweeps are not executed for it (fixed-point completion), and a later run_to only moves its
 * protocol sweep count, not this one -- any other grid the sweep it was taken to (the global K).
 * The sweep method reports K for every grid. */
int mgdp_vi_get_grid_sweeps(mgdp_vi *vi, int32_t *k);
/* Device pointers of the handle's V (current) and pi buffers, for zero-copy consumers. */
int mgdp_vi_device_buffers(mgdp_vi *vi, void **d_V, void **d_pi);
int mgdp_vi_num_states(const mgdp_vi_desc *desc, int64_t *S);

/* Complete all work of the handle: a resident lone-grid server is asked to leave and the stream
 * is drained (V / pi of the last solve are in HBM).  Every result getter does this implicitly. */
int mgdp_vi_synchronize(mgdp_vi *vi);
/* HIP-event timing of the dominant kernel (fused solve or sweep), on the stream it runs on. */
int mgdp_vi_enable_timing(mgdp_vi *vi, int32_t on);
int mgdp_vi_kernel_time(mgdp_vi *vi, double *total_ms, int64_t *launches);
/* Clock of the persistent lone-grid servers (vi_serve_kernel) that ran since enable_timing: each
 * launch reports its shader-clock cycles (s_memtime) and 100 MHz ticks (s_memrealtime) when it
 * leaves; sclk_mhz = cycles / time, server_us = their summed lifetimes; solve_us = the mean
 * GPU-side time of their solves (the poll that saw a request -> the solve's end), over `solves`.
 * 0 launches: no server ran.  A diagnostic (the bench line reports it); no cost per solve. */
int mgdp_vi_serve_clock(mgdp_vi *vi, double *sclk_mhz, double *server_us, int64_t *launches, double *solve_us,
                        int64_t *solves);

/* ---------------------------------------------------------------------------------------------- */
/* Batched env stepping: the gymnasium Env reset()/step() surface (minigrid_env.py:119-157,         */
/* :520-590, gen_obs :592-645) for B envs resident on one device.                                  */
/* ---------------------------------------------------------------------------------------------- */
typedef struct mgdp_envs mgdp_envs;

/* view_size: agent_view_size (odd, 3..7, minigrid_env.py:66-68). */
int mgdp_envs_create(int32_t device, int32_t B, int32_t W, int32_t H, int32_t view_size,
                     mgdp_envs **out);
int mgdp_envs_destroy(mgdp_envs *envs);
int mgdp_envs_set_stream(mgdp_envs *envs, void *hip_stream);
/* NoDeath(env, no_death_types, death_cost) (wrappers.py:799-872) applied inside the step: bit t of
 * type_mask = OBJECT_TO_IDX type t is a no-death type (goal is refused); 0 = off. */
int mgdp_envs_set_nodeath(mgdp_envs *envs, uint32_t type_mask, double death_cost);
/* reset(): upload grids + agent of the envs whose mask byte is 1 (mask NULL = all).
 * enc: B*W*H*3 x-major (Grid.encode()), agent: B*3 (x, y, dir), max_steps: B,
 * see_through: B (see_through_walls, minigrid_env.py:41,103).  step_count and carrying reset to 0. */
int mgdp_envs_load(mgdp_envs *envs, const uint8_t *enc, const int32_t *agent,
                   const int32_t *max_steps, const uint8_t *see_through, const uint8_t *mask);
/* gen_obs() of every env without stepping (the reset() observation). obs: B*V*V*3, dir: B. */
int mgdp_envs_observe(mgdp_envs *envs, uint8_t *obs, int32_t *direction);
/* step(actions) for all B envs (host buffers).  reward fp64 (_reward, minigrid_env.py:235-240).
 * Returns MGDP_E_ACTION / MGDP_E_BOUNDS if any env failed; status (B, may be NULL) says which. */
int mgdp_envs_step(mgdp_envs *envs, const int32_t *actions, uint8_t *obs, int32_t *direction,
                   double *reward, uint8_t *terminated, uint8_t *truncated, int32_t *status);
/* Device-pointer variant, asynchronous on the handle's stream; status per env in d_status. */
int mgdp_envs_step_device(mgdp_envs *envs, const int32_t *d_actions, uint8_t *d_obs,
                          int32_t *d_direction, double *d_reward, uint8_t *d_terminated,
                          uint8_t *d_truncated, int32_t *d_status);
/* HIP-event timing of the step kernel launches (begin/end timestamps of each dispatch, as the
 * rocprofv3 kernel trace reports them); kernel_time synchronises the stream and returns the total
 * since enable_timing. */
int mgdp_envs_enable_timing(mgdp_envs *envs, int32_t on);
int mgdp_envs_kernel_time(mgdp_envs *envs, double *total_ms, int64_t *launches);
/* Read back env state: enc B*W*H*3 (x-major), agent B*3, carry B*2 (type,color; 0 = none),
 * step_count B.  Any pointer may be NULL. */
int mgdp_envs_get_state(mgdp_envs *envs, uint8_t *enc, int32_t *agent, int32_t *carry,
                        int32_t *step_count);
/* Overwrite agent (B*3), carry (B*2) and step_count (B) of the masked envs (NULL = unchanged).
 * A new carry clears that env's carried Box contents (set them again with set_contents). */
int mgdp_envs_set_state(mgdp_envs *envs, const int32_t *agent, const int32_t *carry,
                        const int32_t *step_count, const uint8_t *mask);
/* Box(contains=...) (ABI 10; world_object.py:272-294, replaces the `contains` attribute of the
 * reference's Box): what each Box cell holds, contents B*W*H*3 (x-major (type, colour, state) like
 * Grid.encode(); type 0 / 1 = holds nothing), and what a carried Box holds, carry_contents B*3
 * (NULL = unchanged).  Toggling a Box puts its contents in its cell (None: empty), pickup carries
 * them with the Box, drop puts them back.  A held object must be a Grid.encode() cell on a Box cell
 * (a carried one needs a carried Box); one level: a held Box holds nothing.  mgdp_envs_load clears
 * the loaded envs' contents.  The step kernel touches the contents planes only once they exist. */
int mgdp_envs_set_contents(mgdp_envs *envs, const uint8_t *contents, const int32_t *carry_contents);
/* Read back contents (B*W*H*3) and carry_contents (B*3); zeros where nothing is held. */
int mgdp_envs_get_contents(mgdp_envs *envs, uint8_t *contents, int32_t *carry_contents);

/* ---------------------------------------------------------------------------------------------- */
/* Batched reset(seed) grid generation on the GPU.  Env b gets seed seed0 + b */
/* and the grid/agent reference reset(seed) produces: np_random(seed) = numpy                     */
/* Generator(PCG64(SeedSequence(seed))) drawn in each family's _gen_grid order (empty.py:97-114,   */
/* fourrooms.py:79-128, crossing.py:122-184, doorkey.py:75-100, lavagap.py:101-136,               */
/* distshift.py:99-121; helpers minigrid_env.py:242-390).                                          */
/* ---------------------------------------------------------------------------------------------- */
enum {
    MGDP_GEN_EMPTY = 0, MGDP_GEN_FOURROOMS = 1, MGDP_GEN_CROSSING = 2, MGDP_GEN_DOORKEY = 3,
    MGDP_GEN_LAVAGAP = 4, MGDP_GEN_DISTSHIFT = 5,
};
typedef struct {
    int32_t family;        /* MGDP_GEN_*                                                           */
    int32_t W, H;          /* grid size (FourRooms 19; Crossing odd; 5..32)                         */
    int32_t num_crossings; /* CROSSING                                                             */
    int32_t obstacle;      /* CROSSING / LAVAGAP: OBJECT_TO_IDX of the obstacle (9 lava, 2 wall)    */
    int32_t random_start;  /* EMPTY: agent_start_pos=None -> place_agent()                          */
    int32_t strip2_row;    /* DISTSHIFT                                                            */
    int32_t reserved;
} mgdp_gen_desc;
/* Device buffers (any may be NULL): enc B*W*H*3 uint8 (x-major Grid.encode(): type, colour,
 * state -- what mgdp_envs_load takes), cells B*H*W uint8 row-major type codes (what
 * mgdp_vi_load_cells_device takes), agent B*3 int32 (x, y, dir; dir -1 if rejection sampling hit
 * its cap).  Asynchronous on `stream` (a hipStream_t; NULL = the default stream). */
int mgdp_gen_grids(const mgdp_gen_desc *desc, int32_t device, void *hip_stream, int64_t seed0, int32_t B,
                   uint8_t *enc, uint8_t *cells, int32_t *agent);
/* Same into host buffers (synchronous). */
int mgdp_gen_grids_host(const mgdp_gen_desc *desc, int32_t device, int64_t seed0, int32_t B, uint8_t *enc,
                        uint8_t *cells, int32_t *agent);

#ifdef __cplusplus
}
#endif

#endif /* MGDP_H */
