// Device-buffer collectives of a vh_comm (comm.hip), for other translation units of the
// library (the groupby partition exchange in hashagg.hip).  All enqueue on the library
// stream; callers hold comm_mutex() for a sequence of them.
#pragma once
#include <mutex>

#include "common.hpp"

struct vh_comm;

namespace vh {
int comm_rank(const vh_comm *c);
int comm_world(const vh_comm *c);
int comm_device(const vh_comm *c);  // the GPU the communicator was created on
std::mutex &comm_mutex(vh_comm *c);
void comm_allreduce_dev(vh_comm *c, void *buf, uint64_t count, int dtype, int op);
void comm_allgather_dev(vh_comm *c, const void *send, void *recv, uint64_t bytes);
// send / recv: per-rank segments back to back in rank order, sizes in bytes
void comm_alltoallv_dev(vh_comm *c, const void *send, const uint64_t *send_bytes, void *recv,
                        const uint64_t *recv_bytes);
}  // namespace vh
