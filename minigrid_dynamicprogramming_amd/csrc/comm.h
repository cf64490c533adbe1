// comm.h -- the library's communicator for the sharded solve (RCCL over xGMI, loaded at run time).
// See include/mgdp.h (mgdp_comm_*, mgdp_vi_solve_sharded).
#pragma once

#include "common.h"

namespace mgdp {
// MAX all-reduce of n int64 words of device memory, in place, enqueued on `stream`.
int comm_allreduce_max_dev(mgdp_comm *c, int64_t *d, size_t n, hipStream_t stream);
// The communicator's device protocol buffer: int64[16] of device memory ([0..7] the protocol's words:
// {K, dV bits, kmin, 0}, [5] = dV(K) bits; [8..15] host-driven staging), and a pinned host word for
// the one-word collectives.
int64_t *comm_proto(mgdp_comm *c);
int64_t *comm_host_word(mgdp_comm *c);
int comm_device(const mgdp_comm *c);
// One host wait on the GPU made on the communicator's behalf (mgdp_comm_host_waits).
void comm_note_host_wait(mgdp_comm *c);
}  // namespace mgdp
