// bfsx_internal.h -- shared declarations of the MI355X BFS engine (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/bfsx.h"

namespace bfsx {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
const std::string &last_error(); // the calling thread's message (bfsx_last_error)

#define BFSX_STR2(x) #x
#define BFSX_STR(x) BFSX_STR2(x)
// the message names the call and its source line: an asynchronous device fault surfaces at the next
// checked call, and the line tells which one that was
#define BFSX_HIP_TRY(call)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return ::bfsx::fail(e_ == hipErrorOutOfMemory ? BFSX_E_OOM : BFSX_E_HIP,         \
                                std::string(#call) + " [" + __FILE__ ":" BFSX_STR(__LINE__) "]: " + \
                                    hipGetErrorString(e_));                                  \
    } while (0)

struct Options {
    int direction = BFSX_DIR_AUTO;
    int alpha = 20;             // top-down -> bottom-up when m_f > m_u / alpha (re-tuned on scale 26 with the
                                // two-stage bottom-up: 20 vs 30 = +2%, within run-to-run noise of 10..45)
    int beta = 24;              // bottom-up -> top-down when n_f < n / beta (and shrinking)
    int64_t pull_min_edges = (int64_t)1 << 16; // push -> pull needs at least this many frontier edges (and n/512)
    uint32_t hub_degree = 64;   // degree above which a frontier vertex goes to the multi-workgroup bin
    bool persist = true;        // narrow top-down frontiers run many levels per launch (K3p)
    bool vis_front = true;      // single device: a pull level after a push / hybrid / K3p level reads vis as its frontier
    bool persist_front = true;  // a BFS's first K3p launch that stops for a pull level also leaves the bitmap frontier
    bool push_log = true;       // single device: per-level push winners go to the push log, not the packed state
    bool hub_lds_skip = true;   // single device: the hub bin skips targets an LDS snapshot of the hubs' visited bits marks
    int persist_blocks = 0;     // K3p workgroups (0: auto, three per four CUs)
    int offset_bits = 0;        // traversal row-offset width: 0 = uint32 when nnz < 2^32, else int64; 64 = int64
    bool degree_order = true;   // rows ordered by neighbour degree (desc) instead of id (asc)
    bool relabel = true;        // vertices renumbered by degree (desc) at build, inside every rank's id range
    int hub_bits = -1;          // bottom-up hub probe domain: -1 auto, 0 off, b = 2^b hubs
    int bu_unroll = 4;          // bottom-up candidates per lane per round (4 or 2)
    bool bu_pipeline = true;    // bottom-up: the next round's top1 loads overlap this round (kU = 4)
    int bu_sparse = 64;          // single device: pull levels with <= n/bu_sparse unvisited candidates run k_bu_sparse (0 off)
    bool bu_lds_prefix = true;  // pull kernels: the frontier bits of the 2^16 lowest (highest-degree) ids in LDS
    int64_t slot_pairs = -1;    // partitioned push levels with a global m_f up to this: fixed exchange slots (-1: auto)
    // partitioned: ids of degree above big_degree (at most big_cap per rank) are listed with their degree
    // on every rank (read at a graph's first partitioned BFS; see dist_big_list)
    int64_t big_degree = 4096;
    bool leaf_skip = true;      // single device: a pull level's degree-1 discoveries stay out of the next push queue
    int64_t big_cap = (int64_t)1 << 20;
    int hybrid = 1;             // hybrid levels (hub pull + non-hub push): 0 off, 1 auto (cost model), 2 force
    int hybrid_pct = 125;       // auto: hybrid when the frontier's hub edges exceed this % of the unvisited count
    int64_t build_chunk = (int64_t)1 << 30; // CSR build: raw adjacency entries per sort/dedup chunk
    int persist_abort_at = -1;  // test hook: K3p aborts at this level of its launch (-1: never)
    int64_t persist_dmax = 512; // K3p: longer rows are heavy (swept by the whole grid); a host frontier holding one stays out
    bool poison_queues = false; // test hook: fill the frontier queues and hub list with 0xFF before every BFS
    bool bu_force_spill = false; // diagnostic: the partitioned pull kernel in a spilling (8 waves/SIMD) build
    int test_overread = -1;     // test hook: that top-down level's kernels read one queue entry past the tail
    bool check_retired = false; // test hook: the partitioned loop fails if a launch or exchange uses a retired buffer
    int sparse_exchange = 1;    // partitioned pull levels: small global frontiers exchanged as id lists (0 off, 1 auto, 2 on)
    int64_t comm_timeout_ms = 120000; // partitioned path: a host wait on the peers fails after this long
    bool check_collectives = false;   // debug: every collective checks that all ranks are in the same (op, level)
    int fail_rank = -1, fail_level = -1; // test hook (fault injection): that rank fails at that level of the loop
    bool comm_timing = false;   // partitioned: hipEvents around every collective of the level loop (bfsx_comm_times)
    int race_probe = 0;         // test hook: k_td's queue init late behind stale LDS (1), and without its barrier (2)
    int64_t slot_force = -1;    // test hook: fixed-slot push levels use slots of this many pairs (the store guard fires)
};

// ---- bfsx_comm.cpp: exchange layer of the partitioned BFS ---------------------------------
// Stream-ordered collectives on device buffers (RCCL, or an in-process group of host threads).
//
// Failure handling ("A failed rank fails every rank"): a collective loop is only as live as its
// slowest rank, so a rank that leaves a collective call with an error calls abort() (comm_guard below), which
// makes every peer's pending and later collectives fail with BFSX_E_RCCL "peer rank r failed ...": the
// in-process group wakes its waiters; RCCL ranks signal each other through a node-local shared-memory board
// and ncclCommAbort their communicators.  Every host wait of the partitioned path polls for that (poll(), from
// post_wait and comm_sync) and gives up after `timeout_ms` (a rank that died or diverged without signalling).
// An aborted communicator stays failed, like an aborted NCCL communicator.
enum CommOp : int { kOpAllreduce = 1, kOpAlltoall1 = 2, kOpAlltoallv = 3, kOpAllgather = 4 };
const char *comm_op_name(int op);
struct Comm {
    int rank = 0, nranks = 1;
    int tag = -1;                // the partitioned loop's level (-1: setup, -2: after the loop): names a collective
    int64_t timeout_ms = 120000; // option comm_timeout_ms: a host wait on the peers fails after this long
    bool check_seq = false;      // option check_collectives: every collective compares (op, level) across the ranks
    bool agreed = false;         // the error being returned was reached by every rank at the same point: no abort
    void *pinned = nullptr;      // comm_fetch's bounce buffer (page-locked host memory)
    size_t pinned_bytes = 0;
    // bounce buffers replaced by a larger fetch: freed with the communicator, never while a collective may still
    // be queued on the stream (hipHostFree waits for the device, outside the polled host waits)
    std::vector<void *> pinned_retired;
    virtual ~Comm();
    virtual int allreduce_sum(int64_t *d_buf, int n, hipStream_t st) = 0;              // in place
    // one value per rank; d_recv[rank] (the value a rank sends itself) may be left unwritten
    virtual int alltoall1(const int64_t *d_send, int64_t *d_recv, hipStream_t st) = 0;
    virtual int alltoallv(const unsigned long long *d_send, const int64_t *scount, const int64_t *sdispl, unsigned long long *d_recv,
                          const int64_t *rcount, const int64_t *rdispl, hipStream_t st) = 0; // host counts
    virtual int allgather(const unsigned long long *d_in, int64_t n, unsigned long long *d_out, hipStream_t st) = 0;
    // This rank failed with (code, msg): every peer's pending and later collectives fail.  Idempotent; a no-op
    // when a peer's abort is what failed this rank.
    virtual void abort(int code, const std::string &msg) = 0;
    // Between spins of a host wait that started at t0_ns (steady clock): BFSX_OK, or BFSX_E_RCCL with the
    // message set once any rank aborted or the wait outlived timeout_ms (which aborts the group).
    virtual int poll(int64_t t0_ns, const char *what) = 0;
    virtual bool failed() const = 0; // aborted (by this rank or a peer): every call fails
};
int64_t now_ns();
// hipStreamSynchronize for the partitioned path: polls the communicator while the stream drains
int comm_sync(Comm *cm, hipStream_t st, const char *what);
// Device -> host copy of a collective's result: through cm's page-locked bounce buffer, then comm_sync.  A copy
// straight into pageable memory blocks the host until the stream reaches it, outside comm_sync's polling: a rank
// whose peer failed would wait there for a collective that never completes.
int comm_fetch(Comm *cm, hipStream_t st, void *dst, const void *d_src, size_t bytes, const char *what);
// After a collective entry point returned rc on this rank: abort the group when rc is this rank's own error
// (not a peer's abort it merely observed), so no peer waits for it.  Returns rc.
int comm_guard(Comm *cm, int rc);
void comm_sync_options(bfsx_ctx *ctx); // the context's comm_timeout_ms / check_collectives onto its communicator
// ranks ctxs[0..n) of one process, one host thread each: an RCCL clique over their (distinct) devices, or the
// in-process group (rccl = false)
int comm_clique(bfsx_ctx **ctxs, int nranks, bool rccl);

// ---- kernels_build.hip -------------------------------------------------------------------
// Builds the CSR (sorted, de-duplicated neighbour sets, self-loops kept once) from device tuple
// arrays.  Takes ownership of nothing; d_u/d_v stay owned by the caller.
// Rows are built for the global id range [lo, lo + nv) only (lo = 0, nv = all for one device);
// nv_global sizes the sort keys and the degree table of the degree-ordered rows.
// relabel_chunk > 0 (with degree_order): vertices renumbered by degree, descending, inside every id range
// [r*relabel_chunk, (r+1)*relabel_chunk) (one range on one device, the ranks' ranges on a partition);
// *d_perm = this rank's slice of the permutation (local internal row of original local id i) and
// *d_inv = the whole inverse (original id of global internal id x) are set, else left untouched.
int build_csr_device(hipStream_t stream, int64_t nv, const uint32_t *d_u, const uint32_t *d_v, int64_t m,
                     bool degree_order, int64_t relabel_chunk, int64_t **d_row_off, uint32_t **d_col, int64_t *nnz,
                     uint32_t **d_tuple_cnt, uint32_t **d_perm, uint32_t **d_inv, int64_t lo = 0,
                     int64_t nv_global = -1);
// Row-chunk size (raw adjacency entries) of the CSR build's sort/dedup/ordering passes, calling thread.
void set_build_chunk(int64_t entries);
int kronecker_generate(hipStream_t stream, int scale, int edgefactor, uint64_t seed, uint32_t *d_u,
                       uint32_t *d_v);
// ---- kernels_parse.hip: GPU tokenizer of the algs4 edge lines (after the two header lines) -----
// body/n: host bytes of the edge lines; first_lineno: file line number of the first of them.  On success
// the tuples are device arrays of length *m (caller frees); errors match the host parser's.
int parse_algs4_device(hipStream_t st, const char *body, size_t n, int64_t nv, int64_t first_lineno, uint32_t **d_u,
                       uint32_t **d_v, int64_t *m);
// The same CSR built straight from the Kronecker counter stream (rows of global ids [lo, lo+nv_local)).
int build_csr_kronecker(hipStream_t stream, int scale, int edgefactor, uint64_t seed, bool degree_order,
                        int64_t relabel_chunk, int64_t **d_row_off, uint32_t **d_col, int64_t *nnz,
                        uint32_t **d_tuple_cnt, uint32_t **d_perm, uint32_t **d_inv, int64_t lo, int64_t nv_local);

// D2H copy of a relabelled graph's CSR in ORIGINAL ids (rows of original ids, entries mapped back;
// each row keeps its degree-descending order).  row_off[nv+1] / col[nnz] host, either may be null.
int export_csr_original(hipStream_t stream, int64_t nv, int64_t nnz, const int64_t *d_row_off, const uint32_t *d_col,
                        const uint32_t *d_perm, const uint32_t *d_inv, int64_t *row_off, uint32_t *col);
// ---- the BFS kernel families (bfs_core.h; kernels_{push,pull,persist,level,dist}.hip) -------------
struct BfsWorkspace;
int bfs_run(bfsx_graph *g, int64_t source, bfsx_stats *stats);
int bfs_mcomp(bfsx_graph *g, int64_t *m_comp, int64_t *reached);
int64_t bfs_persist_fallbacks(const bfsx_graph *g); // BFS runs re-run without K3p after a barrier abort
int bfs_copy_result(bfsx_graph *g, int32_t *dist_out, int64_t *parent_out);
// device time (ms) of the most recent copy's unpack kernel (state + level records -> original-id dist/parent); -1: none
double bfs_last_unpack_ms(const bfsx_graph *g);
// its first part: the push log scattered and the pull records folded into the per-vertex state (the result in
// internal ids); -1 when the last copy took the scatter path (graphs without the relabel)
double bfs_last_resolve_ms(const bfsx_graph *g);
void bfs_comm_times(const bfsx_graph *g, double *ms, int64_t *count); // option comm_timing: last partitioned BFS
// multi-GPU level primitives (kernels_dist.hip), driven by bfsx_dist_* in bfsx_api.cpp
int dist_begin(bfsx_graph *g, int64_t source, int64_t *deg_local, int64_t deg_known = -1);
int dist_frontier_info(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local, int *in_queue);
int dist_td_expand(bfsx_graph *g, unsigned long long *d_send, int64_t send_cap, int64_t *send_counts);
int dist_td_claim(bfsx_graph *g, const unsigned long long *d_recv, int64_t n);
int dist_frontier_slice(bfsx_graph *g, unsigned long long *d_slice);
int dist_bu_step(bfsx_graph *g, const unsigned long long *d_front_global);
int dist_level_end(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local);
int dist_finish(bfsx_graph *g);
// the whole partitioned level loop with the exchanges through ctx->comm (collective over the ranks)
int dist_bfs_run(bfsx_graph *g, int64_t source, bfsx_stats *stats);
void bfs_workspace_free(BfsWorkspace *ws);
// packed state (parent << 32 | dist) of the most recent BFS (device; null before the first one).  Valid after
// bfs_resolve: a single-device BFS leaves its pull levels' discoveries in their level records (4-B parents +
// one bitmap per pull level) until then.
const unsigned long long *bfs_state(const bfsx_graph *g);
int bfs_resolve(bfsx_graph *g);
// ---- kernels_validate.hip: Graph500-style validation of the most recent result --------------------
// res = {violating vertices, smallest violating id (-1: none), reached, adjacency entries checked};
// collective on a partitioned graph.  stt: packed states of the local rows to check (device), null =
// the most recent BFS (source < 0: its source).
int bfs_validate(bfsx_graph *g, int64_t source, const unsigned long long *stt, int64_t res[4]);

} // namespace bfsx

struct bfsx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bfsx::Options opt;
    int num_cus = 256;
    std::unique_ptr<bfsx::Comm> comm; // partitioned path: set by bfsx_comm_init / bfsx_comm_local_group
    // a group context (bfsx_init_group): one rank context per rank, driven by one host thread each inside every
    // call on the group; the group itself holds no stream or communicator
    std::vector<bfsx_ctx *> ranks;
};

struct bfsx_graph {
    bfsx_ctx *ctx = nullptr;
    int64_t nv = 0, nnz = 0, m = 0; // nv = rows held here (all vertices unless partitioned)
    // 1-D partition (multi-GPU): this rank holds rows of global ids [v_lo, v_lo + nv); chunk ids per
    // rank (multiple of 64); adjacency entries are global ids.  Single device: v_lo = 0, nranks = 1.
    int64_t nv_global = 0, v_lo = 0, chunk = 0;
    int rank = 0, nranks = 1;
    int64_t *d_row_off = nullptr; // [nv+1]
    uint32_t *d_col = nullptr;    // [nnz]
    uint32_t *d_tuple_cnt = nullptr; // [nv]: input tuples whose first endpoint is v (m_comp)
    // degree-descending relabel (option "relabel", inside every rank's id range): every device array is indexed by the
    // internal id; perm[original] = internal, inv[internal] = original.  Null: internal = original.
    uint32_t *d_perm = nullptr, *d_inv = nullptr;
    bfsx::BfsWorkspace *ws = nullptr;
    // a graph of a group context: rank r's partition (rows of global ids [r*chunk, ...)) in parts[r]; the group
    // graph's own fields hold nv_global / nnz (sum) / m and nothing is on a device under it directly
    std::vector<bfsx_graph *> parts;
    // host memo of the immutable per-source lookups a BFS start reads back from the device (each a synchronous
    // 4-16 B copy, ~10 us of host time): original -> internal id, internal id -> its row bounds.  Bounded.
    std::unordered_map<int64_t, int64_t> perm_memo;
    std::unordered_map<int64_t, std::pair<int64_t, int64_t>> row_memo;
    // most recent BFS
    int64_t last_source = -1;
    double last_t_bfs_ms = 0.0; // device time of the most recent BFS (source init -> finalize)
    std::vector<double> level_cum_ms;
    std::vector<int32_t> level_dirs;
    std::vector<bfsx_level_stat> level_stats;
};
