// bfsx_comm.cpp -- the exchange layer of the 1-D partitioned BFS (multi-GPU).
//
// The reference's only data exchange is Spark's hash-partitioned shuffle inside reduceByKey
// (BfsSpark.java:90), which moves whole serialised Vertex objects every level.  Here a level moves
// only what the partition boundary needs:
//   top-down   owner-routed (vertex, parent) pairs: all-to-all of counts, then all-to-allv of pairs
//   bottom-up  the frontier bitmap slices: all-gather into one global bitmap
//   every level all-reduce of the level counters (n_f, m_f, m_u): termination (BfsSpark.java:117)
//              and Beamer's direction switch, identical on every rank
// Two implementations of the same stream-ordered device-buffer interface:
//   RcclComm        one process per GPU, RCCL over xGMI (collectives enqueued on the BFS stream, so
//                   the host waits only where it needs a count)
//   LocalGroupComm  P ranks as P host threads of ONE process (same or different devices), exchanging
//                   by device copies -- the same level loop, testable on a single GPU
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>

#include "bfsx_internal.h"
#include "exchange_plan.h"

namespace bfsx {

#define BFSX_NCCL_TRY(call)                                                                          \
    do {                                                                                             \
        ncclResult_t r_ = (call);                                                                    \
        if (r_ != ncclSuccess) return ::bfsx::fail(BFSX_E_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

namespace {

// ---- RCCL ---------------------------------------------------------------------------------------
class RcclComm final : public Comm {
  public:
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    int allreduce_sum(int64_t *d_buf, int n, hipStream_t st) override {
        BFSX_NCCL_TRY(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclInt64, ncclSum, comm, st));
        return BFSX_OK;
    }
    int alltoall1(const int64_t *d_send, int64_t *d_recv, hipStream_t st) override {
        if (nranks < 2) return BFSX_OK; // the own entry is not exchanged (Comm::alltoall1)
        BFSX_NCCL_TRY(ncclGroupStart());
        for (int p = 0; p < nranks; p++) {
            if (p == rank) continue;
            BFSX_NCCL_TRY(ncclSend(d_send + p, 1, ncclInt64, p, comm, st));
            BFSX_NCCL_TRY(ncclRecv(d_recv + p, 1, ncclInt64, p, comm, st));
        }
        BFSX_NCCL_TRY(ncclGroupEnd());
        return BFSX_OK;
    }
    int alltoallv(const unsigned long long *d_send, const int64_t *scount, const int64_t *sdispl, unsigned long long *d_recv,
                  const int64_t *rcount, const int64_t *rdispl, hipStream_t st) override {
        std::vector<P2pOp> ops;
        alltoallv_ops(nranks, scount, sdispl, rcount, rdispl, ops);
        if (ops.empty()) return BFSX_OK;
        BFSX_NCCL_TRY(ncclGroupStart());
        for (const P2pOp &o : ops) {
            if (o.send) BFSX_NCCL_TRY(ncclSend(d_send + o.offset, (size_t)o.count, ncclUint64, o.peer, comm, st));
            else BFSX_NCCL_TRY(ncclRecv(d_recv + o.offset, (size_t)o.count, ncclUint64, o.peer, comm, st));
        }
        BFSX_NCCL_TRY(ncclGroupEnd());
        return BFSX_OK;
    }
    int allgather(const unsigned long long *d_in, int64_t n, unsigned long long *d_out, hipStream_t st) override {
        BFSX_NCCL_TRY(ncclAllGather(d_in, d_out, (size_t)n, ncclUint64, comm, st));
        return BFSX_OK;
    }
};

// ---- in-process group -----------------------------------------------------------------------------
struct LocalGroup {
    int nranks;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const void *> ptr;     // one posted device pointer per rank
    std::vector<std::vector<int64_t>> vals; // one posted host vector per rank
    explicit LocalGroup(int p) : nranks(p), ptr(p, nullptr), vals(p) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

class LocalGroupComm final : public Comm {
  public:
    std::shared_ptr<LocalGroup> grp;
    // Every exchange: drain my stream (my inputs are final), post, barrier, pull from the peers with
    // device copies on my stream, drain it, barrier (peers may reuse their buffers afterwards).
    int allreduce_sum(int64_t *d_buf, int n, hipStream_t st) override {
        std::vector<int64_t> mine(n);
        BFSX_HIP_TRY(hipMemcpyAsync(mine.data(), d_buf, n * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->vals[rank] = mine;
        grp->barrier();
        std::vector<int64_t> sum(n, 0);
        for (int p = 0; p < nranks; p++)
            for (int i = 0; i < n; i++) sum[i] += grp->vals[p][i];
        grp->barrier();
        BFSX_HIP_TRY(hipMemcpyAsync(d_buf, sum.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    int alltoall1(const int64_t *d_send, int64_t *d_recv, hipStream_t st) override {
        std::vector<int64_t> mine(nranks);
        BFSX_HIP_TRY(hipMemcpyAsync(mine.data(), d_send, nranks * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->vals[rank] = mine;
        grp->barrier();
        std::vector<int64_t> got(nranks);
        for (int p = 0; p < nranks; p++) got[p] = grp->vals[p][rank];
        grp->barrier();
        BFSX_HIP_TRY(hipMemcpyAsync(d_recv, got.data(), nranks * sizeof(int64_t), hipMemcpyHostToDevice, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    int alltoallv(const unsigned long long *d_send, const int64_t *scount, const int64_t *sdispl, unsigned long long *d_recv,
                  const int64_t *rcount, const int64_t *rdispl, hipStream_t st) override {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->ptr[rank] = d_send;
        grp->vals[rank].assign(sdispl, sdispl + nranks);
        grp->barrier();
        for (int p = 0; p < nranks; p++) {
            if (rcount[p] <= 0) continue;
            const unsigned long long *src = static_cast<const unsigned long long *>(grp->ptr[p]) + grp->vals[p][rank];
            BFSX_HIP_TRY(hipMemcpyAsync(d_recv + rdispl[p], src, rcount[p] * sizeof(unsigned long long), hipMemcpyDefault, st));
        }
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->barrier();
        (void)scount;
        return BFSX_OK;
    }
    int allgather(const unsigned long long *d_in, int64_t n, unsigned long long *d_out, hipStream_t st) override {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->ptr[rank] = d_in;
        grp->barrier();
        for (int p = 0; p < nranks; p++)
            BFSX_HIP_TRY(hipMemcpyAsync(d_out + p * n, grp->ptr[p], n * sizeof(unsigned long long), hipMemcpyDefault, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->barrier();
        return BFSX_OK;
    }
};

} // namespace

} // namespace bfsx

using namespace bfsx;

extern "C" {

int bfsx_comm_unique_id(uint8_t *id) {
    if (!id) return fail(BFSX_E_ARG, "null id");
    static_assert(sizeof(ncclUniqueId) == BFSX_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    BFSX_NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return BFSX_OK;
}

int bfsx_comm_init(bfsx_ctx *ctx, int rank, int nranks, const uint8_t *id) {
    if (!ctx || !id || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        return fail(BFSX_E_ARG, "bad argument");
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    auto c = std::make_unique<RcclComm>();
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    BFSX_NCCL_TRY(ncclCommInitRank(&c->comm, nranks, u, rank));
    ctx->comm.reset(c.release());
    return BFSX_OK;
}

int bfsx_comm_local_group(bfsx_ctx **ctxs, int nranks) {
    if (!ctxs || nranks < 1 || nranks > 64) return fail(BFSX_E_ARG, "bad argument");
    for (int r = 0; r < nranks; r++)
        if (!ctxs[r]) return fail(BFSX_E_ARG, "null ctx");
    auto grp = std::make_shared<LocalGroup>(nranks);
    for (int r = 0; r < nranks; r++) {
        auto c = std::make_unique<LocalGroupComm>();
        c->rank = r;
        c->nranks = nranks;
        c->grp = grp;
        ctxs[r]->comm.reset(c.release());
    }
    return BFSX_OK;
}

} // extern "C"
