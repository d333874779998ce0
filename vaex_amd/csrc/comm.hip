// Multi-GPU exchange of libvaexhip, bound to RCCL directly (no PyTorch): one process per
// GPU, a communicator created from a unique id the caller distributes (vaex_amd/comm.py
// hands rank 0's id to the other ranks over its host channel), every collective enqueued
// on the library stream.
//
// What crosses the links:
//   * dense grids (C2 / C4 row shards): one in-place all-reduce per aggregator grid --
//     SUM for count / sum / moment grids, MIN / MAX for min / max grids (the reference's
//     Aggregator::reduce, superagg.cpp:160-167,205-212,252-259,354-361); AggFirst needs the
//     (value, order) pair: both grids are all-gathered and reduced on the device with the
//     AggFirst rule (superagg.cpp:470-480; ranks in order, so ties keep the lower rank);
//   * groupby partitions (C5): vh_hashagg_exchange (hashagg.hip) -- the hash-partition
//     all-to-all of group rows built on vh_comm_alltoallv below.
// Dtypes RCCL has no reduction for (16-bit integers) are all-gathered and reduced on the
// device instead.
//
// Loopback communicators (vh_comm_loopback): N virtual ranks in one process on one GPU, one
// host thread per rank.  Each collective is a rendezvous of the N threads; the last to
// arrive moves every rank's bytes with device copies on the library stream (all-gather,
// all-to-all), and an all-reduce is an all-gather plus the rank-order device fold
// (k_fold_ranks) -- so the device-side code around the collectives (the AggFirst rank
// rule, the all-to-all segment math, the groupby fold of received rows) runs with N ranks'
// data on a one-GPU box.  A mismatched collective or a rank that never arrives (60 s) fails
// every rank instead of hanging.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>

#include "comm.hpp"
#include "engine.hpp"

using namespace vh;

namespace vh {

#define VH_NCCL(expr)                                                                          \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess)                                                                 \
            ::vh::fail(VH_ERR_RUNTIME, std::string("RCCL error '") + ncclGetErrorString(r_) + \
                                           "' in " #expr);                                     \
    } while (0)

static bool nccl_dtype(int d, ncclDataType_t *out) {
    switch (d) {
    case VH_F64: *out = ncclFloat64; return true;
    case VH_F32: *out = ncclFloat32; return true;
    case VH_I64: *out = ncclInt64; return true;
    case VH_U64: *out = ncclUint64; return true;
    case VH_I32: *out = ncclInt32; return true;
    case VH_U32: *out = ncclUint32; return true;
    case VH_I8: *out = ncclInt8; return true;
    case VH_U8: case VH_BOOL: *out = ncclUint8; return true;
    default: return false;  // 16-bit integers: no RCCL reduction type
    }
}

static ncclRedOp_t nccl_op(int op) {
    switch (op) {
    case VH_OP_SUM: return ncclSum;
    case VH_OP_MIN: return ncclMin;
    case VH_OP_MAX: return ncclMax;
    }
    fail(VH_ERR_ARG, "unknown reduction op");
}

// fold the world all-gathered copies (world x n, rank-major) into out[n] with op
template <typename T> __global__ void k_fold_ranks(const T *all, uint64_t n, int world, int op, T *out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        T acc = all[i];
        for (int r = 1; r < world; r++) {
            const T v = all[(uint64_t)r * n + i];
            if (op == VH_OP_SUM) acc = (T)(acc + v);
            else if (op == VH_OP_MIN) acc = v < acc ? v : acc;
            else acc = acc < v ? v : acc;
        }
        out[i] = acc;
    }
}

// AggFirst across ranks: the value of the smallest order, earlier rank on ties
// (AggFirst::reduce, superagg.cpp:470-480, applied to parts in rank order)
template <typename T>
__global__ void k_first_ranks(const T *vals, const T *ords, uint64_t n, int world, T *v_out, T *o_out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        T v = vals[i], o = ords[i];
        for (int r = 1; r < world; r++) {
            const T o2 = ords[(uint64_t)r * n + i];
            if (o2 < o) {
                o = o2;
                v = vals[(uint64_t)r * n + i];
            }
        }
        v_out[i] = v;
        o_out[i] = o;
    }
}

}  // namespace vh

namespace vh {

// ---- loopback group: N virtual ranks of one process -----------------------------------
enum LoopOp { LOOP_ALLGATHER = 1, LOOP_ALLTOALLV = 2 };

struct LoopGroup {
    explicit LoopGroup(int w) : world(w), slot(w) {}
    struct Slot {
        const void *send = nullptr;
        void *recv = nullptr;
        uint64_t bytes = 0;
        std::vector<uint64_t> sb, rb;  // all-to-all segment sizes
    };
    const int world;
    int device = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, op = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::string err;  // the last round's failure, raised on every rank
    std::vector<Slot> slot;
};

static void loop_perform(LoopGroup &g) {
    hipStream_t st = stream();
    const int W = g.world;
    if (g.op == LOOP_ALLGATHER) {
        const uint64_t b = g.slot[0].bytes;
        for (int r = 1; r < W; r++)
            if (g.slot[r].bytes != b) fail(VH_ERR_ARG, "loopback all-gather: ranks pass different sizes");
        if (b)
            for (int d = 0; d < W; d++)
                for (int s = 0; s < W; s++)
                    VH_HIP(hipMemcpyAsync(static_cast<char *>(g.slot[d].recv) + (uint64_t)s * b, g.slot[s].send, b,
                                          hipMemcpyDeviceToDevice, st));
    } else {
        // rank s's segment d (offset: its sizes before d) -> rank d's segment s
        for (int s = 0; s < W; s++)
            for (int d = 0; d < W; d++)
                if (g.slot[s].sb[d] != g.slot[d].rb[s])
                    fail(VH_ERR_ARG, "loopback all-to-all: rank " + std::to_string(s) + " sends " +
                                         std::to_string(g.slot[s].sb[d]) + " bytes to rank " + std::to_string(d) +
                                         ", which expects " + std::to_string(g.slot[d].rb[s]));
        for (int s = 0; s < W; s++) {
            uint64_t so = 0;
            for (int d = 0; d < W; d++) {
                uint64_t ro = 0;
                for (int q = 0; q < s; q++) ro += g.slot[d].rb[q];
                if (g.slot[s].sb[d])
                    VH_HIP(hipMemcpyAsync(static_cast<char *>(g.slot[d].recv) + ro,
                                          static_cast<const char *>(g.slot[s].send) + so, g.slot[s].sb[d],
                                          hipMemcpyDeviceToDevice, st));
                so += g.slot[s].sb[d];
            }
        }
    }
    VH_HIP(hipGetLastError());
    VH_HIP(hipStreamSynchronize(st));  // every rank's buffers are final when the round ends
}

// one collective round: post this rank's arguments, the last rank to arrive performs it
static void loop_round(LoopGroup &g, int rank, int op, LoopGroup::Slot mine) {
    std::unique_lock<std::mutex> lk(g.mu);
    if (g.broken) fail(VH_ERR_RUNTIME, "loopback communicator is broken by an earlier failure: " + g.err);
    if (g.arrived == 0) g.op = op;
    else if (g.op != op) {
        g.broken = true;
        g.err = "loopback: ranks called different collectives";
        g.cv.notify_all();
        fail(VH_ERR_RUNTIME, g.err);
    }
    g.slot[rank] = std::move(mine);
    const uint64_t my_gen = g.gen;
    if (++g.arrived == g.world) {
        g.err.clear();
        try {
            loop_perform(g);
        } catch (const std::exception &e) {
            g.err = e.what();
        }
        g.arrived = 0;
        g.gen++;
        g.cv.notify_all();
    } else if (!g.cv.wait_for(lk, std::chrono::seconds(60), [&] { return g.gen != my_gen || g.broken; })) {
        g.broken = true;
        g.err = "loopback: not every rank reached the collective within 60 s";
        g.cv.notify_all();
    }
    if (g.broken) fail(VH_ERR_RUNTIME, g.err);
    if (!g.err.empty()) fail(VH_ERR_RUNTIME, g.err);
}

}  // namespace vh

struct vh_comm {
    ncclComm_t comm = nullptr;
    std::shared_ptr<vh::LoopGroup> loop;  // loopback rank (no RCCL communicator)
    int rank = 0, world = 1, device = 0;
    std::mutex mu;          // one collective sequence at a time per communicator
    DevBuf stage, gather;   // host-buffer staging / all-gather scratch
};

namespace vh {

int comm_rank(const vh_comm *c) { return c->rank; }
int comm_world(const vh_comm *c) { return c->world; }
int comm_device(const vh_comm *c) { return c->device; }

void comm_allreduce_dev(vh_comm *c, void *buf, uint64_t count, int dtype, int op) {
    if (!count) return;
    ncclDataType_t t;
    if (!c->loop && nccl_dtype(dtype, &t)) {
        VH_NCCL(ncclAllReduce(buf, buf, count, t, nccl_op(op), c->comm, stream()));
        return;
    }
    // no RCCL type (or a loopback group): all-gather the copies, fold them in rank order on
    // the device
    const int isz = dtype_itemsize(dtype);
    c->gather.ensure((uint64_t)isz * count * c->world);
    comm_allgather_dev(c, buf, c->gather.ptr, (uint64_t)isz * count);
    VH_DISPATCH_DTYPE(dtype, T, if constexpr (!std::is_same_v<T, vbool>) {
        hipLaunchKernelGGL(k_fold_ranks<T>, dim3(blocks_for(count, 256)), dim3(256), 0, stream(),
                           c->gather.as<T>(), count, c->world, op, static_cast<T *>(buf));
    } else {
        hipLaunchKernelGGL(k_fold_ranks<uint8_t>, dim3(blocks_for(count, 256)), dim3(256), 0, stream(),
                           c->gather.as<uint8_t>(), count, c->world, op, static_cast<uint8_t *>(buf));
    });
    VH_HIP(hipGetLastError());
}

void comm_allgather_dev(vh_comm *c, const void *send, void *recv, uint64_t bytes) {
    if (c->loop) {
        LoopGroup::Slot s;
        s.send = send;
        s.recv = recv;
        s.bytes = bytes;
        loop_round(*c->loop, c->rank, LOOP_ALLGATHER, std::move(s));
        return;
    }
    if (!bytes) return;
    VH_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, c->comm, stream()));
}

void comm_alltoallv_dev(vh_comm *c, const void *send, const uint64_t *send_bytes, void *recv,
                        const uint64_t *recv_bytes) {
    if (c->loop) {
        LoopGroup::Slot s;
        s.send = send;
        s.recv = recv;
        s.sb.assign(send_bytes, send_bytes + c->world);
        s.rb.assign(recv_bytes, recv_bytes + c->world);
        loop_round(*c->loop, c->rank, LOOP_ALLTOALLV, std::move(s));
        return;
    }
    VH_NCCL(ncclGroupStart());
    uint64_t so = 0, ro = 0;
    for (int r = 0; r < c->world; r++) {
        if (send_bytes[r])
            VH_NCCL(ncclSend(static_cast<const char *>(send) + so, send_bytes[r], ncclUint8, r, c->comm, stream()));
        if (recv_bytes[r])
            VH_NCCL(ncclRecv(static_cast<char *>(recv) + ro, recv_bytes[r], ncclUint8, r, c->comm, stream()));
        so += send_bytes[r];
        ro += recv_bytes[r];
    }
    VH_NCCL(ncclGroupEnd());
}

std::mutex &comm_mutex(vh_comm *c) { return c->mu; }

}  // namespace vh

extern "C" {

int vh_comm_unique_id(void *out) {
    VH_API_BEGIN
    ncclUniqueId id;
    VH_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    VH_API_END
}

int vh_comm_init(const void *id, int world, int rank, vh_comm **out) {
    VH_API_BEGIN
    if (world < 1 || rank < 0 || rank >= world) fail(VH_ERR_ARG, "comm: rank out of range");
    auto c = std::make_unique<vh_comm>();
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    c->rank = rank;
    c->world = world;
    c->device = current_device();
    VH_NCCL(ncclCommInitRank(&c->comm, world, uid, rank));
    *out = c.release();
    VH_API_END
}

int vh_comm_loopback(int world, vh_comm **out) {
    VH_API_BEGIN
    if (world < 1 || world > 64) fail(VH_ERR_ARG, "comm: loopback world must be 1..64");
    auto g = std::make_shared<LoopGroup>(world);
    g->device = current_device();
    std::vector<std::unique_ptr<vh_comm>> cs;
    for (int r = 0; r < world; r++) {
        cs.push_back(std::make_unique<vh_comm>());
        cs.back()->loop = g;
        cs.back()->rank = r;
        cs.back()->world = world;
        cs.back()->device = g->device;
    }
    for (int r = 0; r < world; r++) out[r] = cs[r].release();
    VH_API_END
}

int vh_comm_destroy(vh_comm *c) {
    VH_API_BEGIN
    if (c) {
        DeviceScope ds(c->device);
        (void)hipStreamSynchronize(stream());
        if (c->comm) (void)ncclCommDestroy(c->comm);
        delete c;
        host_cache_trim();  // the end of a distributed run: release the locked host memory
    }
    VH_API_END
}

int vh_comm_allreduce(vh_comm *c, void *buf, uint64_t count, int dtype, int op, int loc) {
    VH_API_BEGIN
    DeviceScope ds(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    const int isz = dtype_itemsize(dtype);
    loc = resolve_loc(buf, loc);
    void *d = buf;
    if (loc == VH_LOC_HOST && count) {
        c->stage.ensure((uint64_t)isz * count);
        VH_HIP(hipMemcpyAsync(c->stage.ptr, buf, (uint64_t)isz * count, hipMemcpyHostToDevice, stream()));
        d = c->stage.ptr;
    }
    comm_allreduce_dev(c, d, count, dtype, op);
    if (loc == VH_LOC_HOST && count)
        VH_HIP(hipMemcpyAsync(buf, d, (uint64_t)isz * count, hipMemcpyDeviceToHost, stream()));
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_comm_allgather(vh_comm *c, const void *send, void *recv, uint64_t bytes, int loc) {
    VH_API_BEGIN
    DeviceScope ds(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    loc = resolve_loc(send, loc);
    if (loc == VH_LOC_HOST) {
        DevBuf s, r;
        s.ensure(std::max<uint64_t>(bytes, 1));
        r.ensure(std::max<uint64_t>(bytes * c->world, 1));
        VH_HIP(hipMemcpyAsync(s.ptr, send, bytes, hipMemcpyHostToDevice, stream()));
        comm_allgather_dev(c, s.ptr, r.ptr, bytes);
        VH_HIP(hipMemcpyAsync(recv, r.ptr, bytes * c->world, hipMemcpyDeviceToHost, stream()));
        VH_HIP(hipStreamSynchronize(stream()));
    } else {
        comm_allgather_dev(c, send, recv, bytes);
        VH_HIP(hipStreamSynchronize(stream()));
    }
    VH_API_END
}

int vh_comm_alltoallv(vh_comm *c, const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes,
                      int loc) {
    VH_API_BEGIN
    DeviceScope ds(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    uint64_t st = 0, rt = 0;
    for (int r = 0; r < c->world; r++) {
        st += send_bytes[r];
        rt += recv_bytes[r];
    }
    loc = resolve_loc(send, loc);
    if (loc == VH_LOC_HOST) {
        DevBuf s, r;
        s.ensure(std::max<uint64_t>(st, 1));
        r.ensure(std::max<uint64_t>(rt, 1));
        if (st) VH_HIP(hipMemcpyAsync(s.ptr, send, st, hipMemcpyHostToDevice, stream()));
        comm_alltoallv_dev(c, s.ptr, send_bytes, r.ptr, recv_bytes);
        if (rt) VH_HIP(hipMemcpyAsync(recv, r.ptr, rt, hipMemcpyDeviceToHost, stream()));
    } else {
        comm_alltoallv_dev(c, send, send_bytes, recv, recv_bytes);
    }
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_comm_barrier(vh_comm *c) {
    VH_API_BEGIN
    DeviceScope ds(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    c->stage.ensure(8);
    VH_HIP(hipMemsetAsync(c->stage.ptr, 0, 8, stream()));
    comm_allreduce_dev(c, c->stage.ptr, 1, VH_I64, VH_OP_SUM);
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

int vh_comm_agg_allreduce(vh_comm *c, vh_agg *a) {
    VH_API_BEGIN
    DeviceScope ds(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    std::lock_guard<std::mutex> glk(a->grid->mu);
    const uint64_t L = a->grid->length1d;
    switch (a->kind) {
    case VH_AGG_COUNT: case VH_AGG_SUM: case VH_AGG_SUM_MOMENT:
        comm_allreduce_dev(c, a->g.ptr, L, a->grid_dtype, VH_OP_SUM);
        break;
    case VH_AGG_MIN: case VH_AGG_MAX:
        comm_allreduce_dev(c, a->g.ptr, L, a->dtype, a->kind == VH_AGG_MIN ? VH_OP_MIN : VH_OP_MAX);
        break;
    case VH_AGG_FIRST: {
        const int isz = dtype_itemsize(a->dtype);
        const uint64_t b = (uint64_t)isz * L;
        c->gather.ensure(2 * b * c->world);
        char *gv = c->gather.as<char>(), *go = gv + b * c->world;
        comm_allgather_dev(c, a->g.ptr, gv, b);
        comm_allgather_dev(c, a->g2.ptr, go, b);
        VH_DISPATCH_DTYPE(a->dtype, T, if constexpr (!std::is_same_v<T, vbool>) {
            hipLaunchKernelGGL(k_first_ranks<T>, dim3(blocks_for(L, 256)), dim3(256), 0, stream(),
                               reinterpret_cast<const T *>(gv), reinterpret_cast<const T *>(go), L, c->world,
                               a->g.as<T>(), a->g2.as<T>());
        } else {
            fail(VH_ERR_ARG, "comm: AggFirst of bool");
        });
        VH_HIP(hipGetLastError());
        break;
    }
    default:
        fail(VH_ERR_ARG, "comm: AggNUnique grids are not additive (merge their value sets instead)");
    }
    VH_HIP(hipStreamSynchronize(stream()));
    VH_API_END
}

}  // extern "C"
