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
//   RcclComm        one rank per GPU, RCCL over xGMI (collectives enqueued on the BFS stream, so the host
//                   waits only where it needs a count): one process per GPU (bfsx_comm_init) or one host
//                   thread per GPU of one process (a clique, bfsx_init_group)
//   LocalGroupComm  P ranks as P host threads of ONE process (same or different devices), exchanging
//                   by device copies -- the same level loop, testable on a single GPU
//
// Failure handling (bfsx_internal.h, Comm): Spark re-runs a lost task from its lineage; a level-synchronous
// loop cannot, so a rank that fails makes every rank fail instead of leaving its peers inside a collective:
//   LocalGroupComm  an abort flag in the group wakes every waiter; barriers give up after timeout_ms;
//                   option check_collectives compares every rank's (op, level) at each collective
//   RcclComm        a node-local shared-memory board (one per communicator, named after the unique id)
//                   carries the failing rank, its level and its message to the peers' host waits, which
//                   ncclCommAbort their own communicators; the board also holds every rank's pid, so a rank
//                   whose process died is noticed too; ranks on other nodes fall back to timeout_ms
#include <rccl/rccl.h>

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "bfsx_internal.h"
#include "exchange_plan.h"

namespace bfsx {

#define BFSX_NCCL_TRY(call)                                                                          \
    do {                                                                                             \
        ncclResult_t r_ = (call);                                                                    \
        if (r_ != ncclSuccess) return ::bfsx::fail(BFSX_E_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

const char *comm_op_name(int op) {
    switch (op) {
    case kOpAllreduce: return "all-reduce";
    case kOpAlltoall1: return "count all-to-all";
    case kOpAlltoallv: return "all-to-allv";
    case kOpAllgather: return "all-gather";
    default: return "?";
    }
}

namespace {

std::string level_name(int tag) {
    return tag >= 0 ? "level " + std::to_string(tag) : tag == -1 ? std::string("setup") : std::string("the end of the loop");
}

constexpr int kBoardRanks = 64;

// The abort board of one communicator: written once by the first rank that fails, read by every peer's host
// waits.  In shared memory for the ranks of one node (one process per GPU), in the heap for a clique.
struct Board {
    std::atomic<uint32_t> state; // 0 live, 1 being written, 2 aborted
    int32_t rank, code, tag;
    int32_t pid[kBoardRanks];
    char msg[496];
};

// Returns false when this call did not write it (another rank's abort came first).
bool board_write(Board *b, int rank, int code, int tag, const std::string &msg) {
    uint32_t expect = 0;
    if (!b->state.compare_exchange_strong(expect, 1u, std::memory_order_acq_rel)) return false;
    b->rank = rank;
    b->code = code;
    b->tag = tag;
    std::snprintf(b->msg, sizeof(b->msg), "%s", msg.c_str());
    b->state.store(2u, std::memory_order_release);
    return true;
}

// The first abort's description; waits (bounded) for a writer that is mid-way.
std::string board_read(const Board *b, int *rank_out) {
    for (int i = 0; i < 1000000 && b->state.load(std::memory_order_acquire) != 2u; i++) std::this_thread::yield();
    if (b->state.load(std::memory_order_acquire) != 2u) {
        *rank_out = -1;
        return "a peer rank failed (its message was not written)";
    }
    *rank_out = b->rank;
    return "peer rank " + std::to_string(b->rank) + " failed at " + level_name(b->tag) + ": " + b->msg;
}

uint64_t fnv1a(const uint8_t *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

// ---- RCCL ---------------------------------------------------------------------------------------
class RcclComm final : public Comm {
  public:
    ncclComm_t comm = nullptr;
    std::shared_ptr<Board> board; // null: no board (only the deadline notices a failed peer)
    bool dead = false;
    std::string dead_msg;
    int64_t last_check_ns = 0;
    unsigned long long *d_seq = nullptr; // check_collectives: the all-gathered (op, level) words
    int device = 0;

    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
        if (d_seq) (void)hipFree(d_seq);
    }
    bool failed() const override { return dead; }

    // the communicator is torn down (ncclCommAbort: RCCL's kernels still waiting on a peer exit) and every later
    // call fails with msg
    void die(const std::string &msg) {
        if (dead) return;
        dead = true;
        dead_msg = msg;
        if (comm) {
            (void)ncclCommAbort(comm);
            comm = nullptr;
        }
    }
    int dead_error() const { return fail(BFSX_E_RCCL, dead_msg); }

    void abort(int code, const std::string &msg) override {
        if (dead) return;
        if (board && !board_write(board.get(), rank, code, tag, msg)) {
            int r = -1;
            die(board_read(board.get(), &r)); // a peer's abort came first: that is the cause
            return;
        }
        die("this rank failed at " + level_name(tag) + ": " + msg + " (communicator aborted)");
    }

    int poll(int64_t t0, const char *what) override {
        if (dead) return dead_error();
        if (board && board->state.load(std::memory_order_acquire) != 0u) {
            int r = -1;
            die(board_read(board.get(), &r));
            return dead_error();
        }
        const int64_t now = now_ns();
        if (now - last_check_ns < 20000000ll) return BFSX_OK; // the slower checks every 20 ms
        last_check_ns = now;
        ncclResult_t ae = ncclSuccess;
        if (comm && ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            abort(BFSX_E_RCCL, std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
            return dead_error();
        }
        if (board) {
            const int me = (int)getpid();
            for (int p = 0; p < nranks && p < kBoardRanks; p++) {
                const int pid = board->pid[p];
                if (p == rank || pid <= 0 || pid == me) continue;
                if (kill(pid, 0) != 0 && errno == ESRCH) {
                    abort(BFSX_E_RCCL, "peer rank " + std::to_string(p) + " (pid " + std::to_string(pid) +
                                           ") exited without finishing " + what);
                    return dead_error();
                }
            }
        }
        if (timeout_ms > 0 && now - t0 > timeout_ms * 1000000ll) {
            abort(BFSX_E_RCCL, "rank " + std::to_string(rank) + " timed out after " + std::to_string(timeout_ms) +
                                   " ms waiting in " + what + " at " + level_name(tag) +
                                   " (a peer rank failed without signalling, died, or issued a different collective)");
            return dead_error();
        }
        return BFSX_OK;
    }

    // entry check of every collective: fail at once once any rank aborted
    int live() {
        if (dead) return dead_error();
        if (board && board->state.load(std::memory_order_acquire) != 0u) {
            int r = -1;
            die(board_read(board.get(), &r));
            return dead_error();
        }
        if (!comm) return fail(BFSX_E_RCCL, "communicator not initialised");
        return BFSX_OK;
    }

    // option check_collectives: all-gather every rank's (op, level) and compare before the collective
    int seq_guard(int op, hipStream_t st) {
        if (!check_seq) return BFSX_OK;
        if (!d_seq) BFSX_HIP_TRY(hipMalloc(&d_seq, (kBoardRanks + 1) * sizeof(unsigned long long)));
        const unsigned long long mine = ((unsigned long long)(uint32_t)op << 32) | (uint32_t)tag;
        // two fills instead of a copy from pageable memory, which could block the host behind a pending collective
        BFSX_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d_seq, (int)(uint32_t)mine, 1, st));
        BFSX_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)((uint32_t *)d_seq + 1), (int)(uint32_t)(mine >> 32), 1, st));
        BFSX_NCCL_TRY(ncclAllGather(d_seq, d_seq + 1, 1, ncclUint64, comm, st));
        std::vector<unsigned long long> all(nranks);
        if (int e = comm_fetch(this, st, all.data(), d_seq + 1, nranks * sizeof(unsigned long long),
                               "the collective-sequence check"))
            return e;
        for (int p = 0; p < nranks; p++)
            if (all[p] != mine) {
                const std::string m = "collective mismatch: rank " + std::to_string(rank) + " is in " + comm_op_name(op) +
                                      " at " + level_name(tag) + ", rank " + std::to_string(p) + " in " +
                                      comm_op_name((int)(all[p] >> 32)) + " at " + level_name((int)(int32_t)all[p]);
                abort(BFSX_E_RCCL, m);
                return fail(BFSX_E_RCCL, m);
            }
        return BFSX_OK;
    }

    int allreduce_sum(int64_t *d_buf, int n, hipStream_t st) override {
        if (int e = live()) return e;
        if (int e = seq_guard(kOpAllreduce, st)) return e;
        BFSX_NCCL_TRY(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclInt64, ncclSum, comm, st));
        return BFSX_OK;
    }
    int alltoall1(const int64_t *d_send, int64_t *d_recv, hipStream_t st) override {
        if (int e = live()) return e;
        if (int e = seq_guard(kOpAlltoall1, st)) return e;
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
        if (int e = live()) return e;
        if (int e = seq_guard(kOpAlltoallv, st)) return e;
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
        if (int e = live()) return e;
        if (int e = seq_guard(kOpAllgather, st)) return e;
        BFSX_NCCL_TRY(ncclAllGather(d_in, d_out, (size_t)n, ncclUint64, comm, st));
        return BFSX_OK;
    }
};

// Connect every peer channel the level loop uses (all-reduce, all-gather, point-to-point to every peer) right
// after init, on the caller's stream: RCCL connects lazily inside the first call that needs a channel, and a
// peer that failed before that call would leave this rank blocked inside RCCL's connection setup, where no
// host wait of ours can notice the abort.  Also a smoke test of the collectives before any graph work.
int warm_up(RcclComm *c, hipStream_t st) {
    int64_t *d = nullptr;
    BFSX_HIP_TRY(hipMalloc(&d, (3 * kBoardRanks + 2) * sizeof(int64_t)));
    struct Free {
        int64_t *p;
        ~Free() { (void)hipFree(p); }
    } fr{d};
    const int P = c->nranks;
    std::vector<int64_t> h(3 * kBoardRanks + 2, 0);
    h[0] = 1;
    for (int p = 0; p < P; p++) h[2 + p] = c->rank; // alltoall1 send: my rank to everyone
    BFSX_HIP_TRY(hipMemcpyAsync(d, h.data(), h.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
    if (int e = c->allreduce_sum(d, 1, st)) return e;
    if (int e = c->alltoall1(d + 2, d + 2 + kBoardRanks, st)) return e;
    if (int e = c->allgather(reinterpret_cast<const unsigned long long *>(d + 1), 1,
                             reinterpret_cast<unsigned long long *>(d + 2 + 2 * kBoardRanks), st))
        return e;
    if (int e = comm_fetch(c, st, h.data(), d, h.size() * sizeof(int64_t), "the communicator warm-up")) return e;
    if (h[0] != P) return fail(BFSX_E_RCCL, "communicator warm-up: all-reduce returned " + std::to_string(h[0]));
    for (int p = 0; p < P; p++)
        if (p != c->rank && h[2 + kBoardRanks + p] != p)
            return fail(BFSX_E_RCCL, "communicator warm-up: count all-to-all returned a wrong value from rank " +
                                         std::to_string(p));
    return BFSX_OK;
}

// ---- in-process group -----------------------------------------------------------------------------
struct LocalGroup {
    int nranks;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const void *> ptr;          // one posted device pointer per rank
    std::vector<std::vector<int64_t>> vals; // one posted host vector per rank
    std::vector<uint64_t> seq;              // check_collectives: (op << 32 | level) per rank
    bool aborted = false;
    int abort_rank = -1, abort_tag = 0;
    std::string abort_msg;
    explicit LocalGroup(int p) : nranks(p), ptr(p, nullptr), vals(p), seq(p, 0) {}

    int peer_error(int rank) const {
        if (abort_rank == rank)
            return fail(BFSX_E_RCCL, "this rank failed at " + level_name(abort_tag) + ": " + abort_msg +
                                         " (group aborted)");
        return fail(BFSX_E_RCCL, "peer rank " + std::to_string(abort_rank) + " failed at " + level_name(abort_tag) +
                                     ": " + abort_msg);
    }
    void abort_locked(int rank, int tag, const std::string &msg) {
        if (aborted) return;
        aborted = true;
        abort_rank = rank;
        abort_tag = tag;
        abort_msg = msg;
        cv.notify_all();
    }
    void abort(int rank, int tag, const std::string &msg) {
        std::lock_guard<std::mutex> lk(mu);
        abort_locked(rank, tag, msg);
    }
    // BFSX_OK once every rank arrived; BFSX_E_RCCL when the group was (or gets) aborted or the wait outlives
    // timeout_ms (which aborts it: a rank that never arrives failed without aborting, or diverged)
    int barrier(int rank, int tag, int64_t timeout_ms, const char *what) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return peer_error(rank);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            arrived = 0;
            generation++;
            cv.notify_all();
            return BFSX_OK;
        }
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : (int64_t)1 << 40);
        while (generation == gen && !aborted) {
            if (cv.wait_until(lk, deadline) == std::cv_status::timeout && generation == gen && !aborted)
                abort_locked(rank, tag,
                             "rank " + std::to_string(rank) + " timed out after " + std::to_string(timeout_ms) +
                                 " ms waiting for its peers in " + what +
                                 " (a peer rank failed without aborting the group, or issued a different collective)");
        }
        if (generation != gen) return BFSX_OK;
        return peer_error(rank);
    }
};

class LocalGroupComm final : public Comm {
  public:
    std::shared_ptr<LocalGroup> grp;
    bool failed() const override {
        std::lock_guard<std::mutex> lk(grp->mu);
        return grp->aborted;
    }
    void abort(int code, const std::string &msg) override {
        (void)code;
        grp->abort(rank, tag, msg);
    }
    int poll(int64_t t0, const char *what) override {
        {
            std::lock_guard<std::mutex> lk(grp->mu);
            if (grp->aborted) return grp->peer_error(rank);
        }
        if (timeout_ms > 0 && now_ns() - t0 > timeout_ms * 1000000ll) {
            const std::string m = "rank " + std::to_string(rank) + " timed out after " + std::to_string(timeout_ms) +
                                  " ms waiting in " + what;
            grp->abort(rank, tag, m);
            return fail(BFSX_E_RCCL, m);
        }
        return BFSX_OK;
    }
    // posts (op, level), then the first barrier of the collective; with check_collectives every rank compares
    // the posted words (they stay put until the collective's second barrier)
    int enter(int op, const char *what) {
        grp->seq[rank] = ((uint64_t)(uint32_t)op << 32) | (uint32_t)tag;
        if (int e = grp->barrier(rank, tag, timeout_ms, what)) return e;
        if (!check_seq) return BFSX_OK;
        for (int p = 0; p < nranks; p++)
            if (grp->seq[p] != grp->seq[rank]) {
                const std::string m = "collective mismatch: rank " + std::to_string(rank) + " is in " + comm_op_name(op) +
                                      " at " + level_name(tag) + ", rank " + std::to_string(p) + " in " +
                                      comm_op_name((int)(grp->seq[p] >> 32)) + " at " +
                                      level_name((int)(int32_t)(uint32_t)grp->seq[p]);
                grp->abort(rank, tag, m);
                return fail(BFSX_E_RCCL, m);
            }
        return BFSX_OK;
    }
    int leave(const char *what) { return grp->barrier(rank, tag, timeout_ms, what); }

    // Every exchange: drain my stream (my inputs are final), post, barrier, pull from the peers with
    // device copies on my stream, drain it, barrier (peers may reuse their buffers afterwards).
    int allreduce_sum(int64_t *d_buf, int n, hipStream_t st) override {
        std::vector<int64_t> mine(n);
        BFSX_HIP_TRY(hipMemcpyAsync(mine.data(), d_buf, n * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->vals[rank] = mine;
        if (int e = enter(kOpAllreduce, "an all-reduce")) return e;
        std::vector<int64_t> sum(n, 0);
        for (int p = 0; p < nranks; p++)
            for (int i = 0; i < n; i++) sum[i] += grp->vals[p][i];
        if (int e = leave("an all-reduce")) return e;
        BFSX_HIP_TRY(hipMemcpyAsync(d_buf, sum.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    int alltoall1(const int64_t *d_send, int64_t *d_recv, hipStream_t st) override {
        std::vector<int64_t> mine(nranks);
        BFSX_HIP_TRY(hipMemcpyAsync(mine.data(), d_send, nranks * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->vals[rank] = mine;
        if (int e = enter(kOpAlltoall1, "a count all-to-all")) return e;
        std::vector<int64_t> got(nranks);
        for (int p = 0; p < nranks; p++) got[p] = grp->vals[p][rank];
        if (int e = leave("a count all-to-all")) return e;
        BFSX_HIP_TRY(hipMemcpyAsync(d_recv, got.data(), nranks * sizeof(int64_t), hipMemcpyHostToDevice, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    int alltoallv(const unsigned long long *d_send, const int64_t *scount, const int64_t *sdispl, unsigned long long *d_recv,
                  const int64_t *rcount, const int64_t *rdispl, hipStream_t st) override {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->ptr[rank] = d_send;
        grp->vals[rank].assign(sdispl, sdispl + nranks);
        if (int e = enter(kOpAlltoallv, "an all-to-allv")) return e;
        int rc = BFSX_OK;
        for (int p = 0; p < nranks && !rc; p++) {
            if (rcount[p] <= 0) continue;
            const unsigned long long *src = static_cast<const unsigned long long *>(grp->ptr[p]) + grp->vals[p][rank];
            const hipError_t he = hipMemcpyAsync(d_recv + rdispl[p], src, rcount[p] * sizeof(unsigned long long),
                                                 hipMemcpyDefault, st);
            if (he != hipSuccess) rc = fail(BFSX_E_HIP, std::string("all-to-allv copy: ") + hipGetErrorString(he));
        }
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = fail(BFSX_E_HIP, "all-to-allv copies failed");
        // the peers' buffers stay untouched until every rank has copied: leave even after a failed copy (the
        // caller's comm_guard then aborts the group)
        if (int e = leave("an all-to-allv")) return rc ? rc : e;
        (void)scount;
        return rc;
    }
    int allgather(const unsigned long long *d_in, int64_t n, unsigned long long *d_out, hipStream_t st) override {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        grp->ptr[rank] = d_in;
        if (int e = enter(kOpAllgather, "an all-gather")) return e;
        int rc = BFSX_OK;
        for (int p = 0; p < nranks && !rc; p++) {
            const hipError_t he = hipMemcpyAsync(d_out + p * n, grp->ptr[p], n * sizeof(unsigned long long),
                                                 hipMemcpyDefault, st);
            if (he != hipSuccess) rc = fail(BFSX_E_HIP, std::string("all-gather copy: ") + hipGetErrorString(he));
        }
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = fail(BFSX_E_HIP, "all-gather copies failed");
        if (int e = leave("an all-gather")) return rc ? rc : e;
        return rc;
    }
};

void apply_options(Comm *c, const bfsx_ctx *ctx) {
    c->timeout_ms = ctx->opt.comm_timeout_ms;
    c->check_seq = ctx->opt.check_collectives;
}

} // namespace

Comm::~Comm() {
    if (pinned) (void)hipHostFree(pinned);
    for (void *p : pinned_retired) (void)hipHostFree(p);
}

int comm_fetch(Comm *cm, hipStream_t st, void *dst, const void *d_src, size_t bytes, const char *what) {
    if (!cm) {
        BFSX_HIP_TRY(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    if (bytes > cm->pinned_bytes) {
        // the stream may still run a collective, and hipHostFree would wait for it outside comm_sync's polling
        // (a failed peer would then hang this rank): the old buffer is retired, freed with the communicator
        if (cm->pinned) cm->pinned_retired.push_back(cm->pinned);
        cm->pinned = nullptr;
        cm->pinned_bytes = 0;
        const size_t cap = std::max<size_t>(bytes, 4096);
        BFSX_HIP_TRY(hipHostMalloc(&cm->pinned, cap, hipHostMallocDefault));
        cm->pinned_bytes = cap;
    }
    BFSX_HIP_TRY(hipMemcpyAsync(cm->pinned, d_src, bytes, hipMemcpyDeviceToHost, st));
    if (int e = comm_sync(cm, st, what)) {
        // the copy may still be queued behind the failed collective: the buffer is left to it (a few KiB
        // leaked once per failed communicator) instead of being freed under a pending transfer
        cm->pinned = nullptr;
        cm->pinned_bytes = 0;
        return e;
    }
    std::memcpy(dst, cm->pinned, bytes);
    return BFSX_OK;
}

int comm_sync(Comm *cm, hipStream_t st, const char *what) {
    if (!cm) {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        return BFSX_OK;
    }
    const int64_t t0 = now_ns();
    for (uint64_t spin = 0;; spin++) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return BFSX_OK;
        if (e != hipErrorNotReady) return fail(BFSX_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
        if (int rc = cm->poll(t0, what)) return rc;
        if (spin > 256) std::this_thread::yield();
    }
}

int comm_guard(Comm *cm, int rc) {
    const bool agreed = cm && cm->agreed;
    if (cm) cm->agreed = false;
    if (rc && cm && !agreed && !cm->failed()) {
        const std::string msg = last_error(); // abort() may overwrite the thread's message
        cm->abort(rc, msg);
        set_error(msg);
    }
    return rc;
}

// Options that live on the communicator (comm_timeout_ms, check_collectives) follow the context's.
void comm_sync_options(bfsx_ctx *ctx) {
    if (ctx && ctx->comm) apply_options(ctx->comm.get(), ctx);
}

// One process, one host thread per rank, rank r on ctxs[r]->device.  Distinct devices: an RCCL clique
// (ncclCommInitAll, xGMI); otherwise (ranks sharing a device, which RCCL refuses) the in-process group.
int comm_clique(bfsx_ctx **ctxs, int nranks, bool rccl) {
    if (!rccl) return bfsx_comm_local_group(ctxs, nranks);
    std::vector<int> devs(nranks);
    for (int r = 0; r < nranks; r++) devs[r] = ctxs[r]->device;
    std::vector<ncclComm_t> comms(nranks, nullptr);
    BFSX_NCCL_TRY(ncclCommInitAll(comms.data(), nranks, devs.data()));
    auto board = std::make_shared<Board>();
    board->state.store(0u);
    for (int r = 0; r < nranks; r++) {
        auto c = std::make_unique<RcclComm>();
        c->rank = r;
        c->nranks = nranks;
        c->comm = comms[r];
        c->board = board;
        c->device = ctxs[r]->device;
        apply_options(c.get(), ctxs[r]);
        ctxs[r]->comm.reset(c.release());
    }
    // warm-up: every rank on its own thread (the collectives of a clique block until all ranks issued them)
    std::vector<int> rcs(nranks, BFSX_OK);
    std::vector<std::string> msgs(nranks);
    std::vector<std::thread> th;
    for (int r = 0; r < nranks; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(ctxs[r]->device);
            rcs[r] = comm_guard(ctxs[r]->comm.get(), warm_up(static_cast<RcclComm *>(ctxs[r]->comm.get()), ctxs[r]->stream));
            msgs[r] = last_error();
        });
    for (auto &t : th) t.join();
    for (int r = 0; r < nranks; r++)
        if (rcs[r]) return fail(rcs[r], "rank " + std::to_string(r) + ": " + msgs[r]);
    return BFSX_OK;
}

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
    if (!ctx || !id || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks || !ctx->ranks.empty())
        return fail(BFSX_E_ARG, "bad argument");
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    auto c = std::make_unique<RcclComm>();
    c->rank = rank;
    c->nranks = nranks;
    c->device = ctx->device;
    apply_options(c.get(), ctx);
    // the node-local abort board, opened by every rank BEFORE the collective init: once any rank's
    // ncclCommInitRank returns, every rank has it mapped, so the name is unlinked right after (nothing is
    // left in /dev/shm, whatever happens to the processes later)
    char name[64];
    std::snprintf(name, sizeof(name), "/bfsx-%016llx", (unsigned long long)fnv1a(id, BFSX_COMM_ID_BYTES));
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd >= 0) {
        void *m = MAP_FAILED;
        if (ftruncate(fd, sizeof(Board)) == 0)
            m = mmap(nullptr, sizeof(Board), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m != MAP_FAILED) {
            Board *b = static_cast<Board *>(m);
            b->pid[rank] = (int32_t)getpid();
            c->board = std::shared_ptr<Board>(b, [](Board *p) { munmap(p, sizeof(Board)); });
        }
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t ir = ncclCommInitRank(&c->comm, nranks, u, rank);
    (void)shm_unlink(name);
    if (ir != ncclSuccess) return fail(BFSX_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(ir));
    if (int e = comm_guard(c.get(), warm_up(c.get(), ctx->stream))) return e;
    ctx->comm.reset(c.release());
    return BFSX_OK;
}

int bfsx_comm_local_group(bfsx_ctx **ctxs, int nranks) {
    if (!ctxs || nranks < 1 || nranks > 64) return fail(BFSX_E_ARG, "bad argument");
    for (int r = 0; r < nranks; r++)
        if (!ctxs[r] || !ctxs[r]->ranks.empty()) return fail(BFSX_E_ARG, "null or group ctx");
    auto grp = std::make_shared<LocalGroup>(nranks);
    for (int r = 0; r < nranks; r++) {
        auto c = std::make_unique<LocalGroupComm>();
        c->rank = r;
        c->nranks = nranks;
        c->grp = grp;
        apply_options(c.get(), ctxs[r]);
        ctxs[r]->comm.reset(c.release());
    }
    return BFSX_OK;
}

} // extern "C"
