// kernels_dist.hip -- the 1-D partitioned level loop (multi-GPU): owner-routed pair exchange of
// the push levels, frontier all-gather / id exchange of the pull levels, the all-reduced level close -- the
// replacement of Spark's reduceByKey shuffle (BfsSpark.java:90) -- and the level primitives the test suite's
// protocol driver steps through.
#include "bfs_core.h"

namespace bfsx {

namespace {

// Multi-GPU: claim the (v, parent) pairs other ranks routed to this rank's vertices.
template <class OffT>
__global__ __launch_bounds__(kBS) void k_claim_remote(const u64 *__restrict__ pairs, u64 npairs,
                                                      const OffT *__restrict__ row_off, u64 *vis,
                                                      u64 *__restrict__ stt, uint32_t *__restrict__ qout,
                                                      LevelSlot *ring, int level, uint32_t lo, u64 slot,
                                                      uint32_t nrows, u64 *err, int64_t *sums, u64 *ctr, int nctr,
                                                      u64 *arrive, int rank, int nranks, u64 *__restrict__ plog,
                                                      u64 qcap) {
    LevelSlot *cn = ring + (level + 1) % 3;
    __shared__ LogQueue q; // plog (the push log's segment of this level): winners as (vertex, parent) pairs
    using Q = LogQueue;
    bq_init(q);
    __syncthreads();
    const int32_t nd = level + 1;
    u64 acc_mf = 0, attempts = 0, acc_dmax = 0;
    // slot > 0: the P fixed slots of [count, slot pairs] (small levels); npairs = (P - 1) * slot, the peers' slots
    for (u64 i0 = (u64)blockIdx.x * kBS; i0 < npairs; i0 += (u64)gridDim.x * kBS) {
        const u64 i = i0 + threadIdx.x;
        bool win = false;
        uint32_t vl = 0, parent = 0;
        bool have = i < npairs;
        u64 at = i;
        if (have && slot) { // npairs = (P - 1) * slot: the peers' slots (the own one is not exchanged, plan_slots)
            const u64 pp = i / slot, k = i - pp * slot;
            const u64 p = pp + (pp >= (u64)rank ? 1u : 0u);
            const u64 base = p * (slot + 1);
            have = k < pairs[base];
            at = base + 1 + k;
        }
        if (have) {
            const u64 pr = pairs[at];
            vl = (uint32_t)(pr >> 32) - lo;
            if (id_ok(vl, nrows, err) && claim(vl, vis, attempts)) {
                win = true;
                parent = (uint32_t)pr;
                if (!plog) stt[vl] = pack_state(parent, nd);
                const u64 dg = (u64)(row_off[vl + 1] - row_off[vl]);
                acc_mf += dg;
                acc_dmax = dg > acc_dmax ? dg : acc_dmax;
            }
        }
        q_push(q, win, vl, parent);
        __syncthreads();
        if (q.n > Q::kCap - (uint32_t)kBS) q_flush(q, qout, plog, &cn->qtail, qcap, err);
    }
    q_flush(q, qout, plog, &cn->qtail, qcap, err);
    shard_add(cn, 0, acc_mf, 0, attempts, 0, acc_dmax);
    if (!sums) return;
    // the level close in the last workgroup to arrive (no k_level_sums dispatch): every wave's queue and
    // shard atomics have returned or drained before the one agent-scope arrival add
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1ull;
    __syncthreads();
    if (s_last) level_sums(cn, 1, sums, ctr, nctr, rank, nranks, err);
}

// Multi-GPU: stable bucketing of remote pairs by owning rank (P <= kMaxRanks).  Two passes over the
// pairs: per-workgroup destination histograms (LDS atomics), then one reservation atomic per
// (workgroup, destination) and LDS-ranked scatter.


// n_cap: the pairs `pairs` holds (a tail past it was guarded by rq_flush and is not read); a pair whose destination
// is not a rank is reported (kSiteSlotDest) and left out.
__global__ __launch_bounds__(kBS) void k_bucket_count(const u64 *__restrict__ pairs, const u64 *__restrict__ d_n,
                                                      u64 n_cap, uint32_t chunk, int nranks, u64 *__restrict__ dcount,
                                                      u64 *err) {
    __shared__ uint32_t s_h[kMaxRanks];
    const uint64_t n = min(*d_n, n_cap);
    for (int d = threadIdx.x; d < nranks; d += kBS) s_h[d] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBS) {
        const uint32_t d = (uint32_t)(pairs[i] >> 32) / chunk;
        if (idx_ok(d, (u64)nranks, err, kSiteSlotDest)) atomicAdd(&s_h[d], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nranks; d += kBS)
        if (s_h[d]) atomicAdd(&dcount[d], (u64)s_h[d]);
}

// Small top-down levels (fixed per-destination slots of [count, cap pairs], so the exchange needs no count
// all-to-all and no host round trip before the pairs move) are bucketed by the push kernels themselves
// (rq_flush in slot mode, slot_headers_if_last); the counted exchange below buckets in two passes.
__global__ __launch_bounds__(kBS) void k_bucket_scatter(const u64 *__restrict__ pairs, const u64 *__restrict__ d_n,
                                                        u64 n_cap, uint32_t chunk, int nranks,
                                                        const u64 *__restrict__ dcount, u64 *__restrict__ dcursor,
                                                        u64 *__restrict__ out, u64 out_cap, u64 *err) {
    __shared__ uint32_t s_h[kMaxRanks];
    __shared__ u64 s_base[kMaxRanks];
    const uint64_t n = min(*d_n, n_cap);
    for (uint64_t i0 = (uint64_t)blockIdx.x * kBS; i0 < n; i0 += (uint64_t)gridDim.x * kBS) {
        for (int d = threadIdx.x; d < nranks; d += kBS) s_h[d] = 0;
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        u64 pr = 0;
        uint32_t d = 0, r = 0;
        bool ok = false;
        if (i < n) {
            pr = pairs[i];
            d = (uint32_t)(pr >> 32) / chunk;
            ok = d < (uint32_t)nranks; // reported by k_bucket_count
            if (ok) r = atomicAdd(&s_h[d], 1u);
        }
        __syncthreads();
        for (int k = threadIdx.x; k < nranks; k += kBS) {
            if (s_h[k]) {
                u64 off = 0; // exclusive prefix of the destination totals
                for (int j = 0; j < k; j++) off += dcount[j];
                s_base[k] = off + atomicAdd(&dcursor[k], (u64)s_h[k]);
            }
        }
        __syncthreads();
        if (ok && idx_ok(s_base[d] + r, out_cap, err, kSiteBucket)) out[s_base[d] + r] = pr;
        __syncthreads();
    }
}

// The ids of a slice (original ids, slice-relative) whose degree exceeds thr, appended as (global id << 32 |
// degree) to out[0..cap); *cnt counts all of them (a count above cap means the list overflowed).
__global__ __launch_bounds__(kBS) void k_select_big(const uint32_t *__restrict__ deg, int64_t chunk, uint32_t thr,
                                                    int64_t v_lo, u64 *__restrict__ out, u64 cap, u64 *cnt) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < chunk; v += (int64_t)gridDim.x * kBS) {
        const uint32_t d = deg[v];
        if (d > thr) {
            const u64 i = atomicAdd(cnt, 1ull);
            if (i < cap) out[i] = ((u64)(v_lo + v) << 32) | d;
        }
    }
}
// Sparse frontier exchange (partitioned pull levels): local row ids -> global ids (u64 words of the send
// buffer), and the received global ids -> the global frontier bitmap (zeroed before).
__global__ __launch_bounds__(kBS) void k_ids_global(const uint32_t *__restrict__ ids, u64 n, uint32_t lo,
                                                    u64 *__restrict__ out) {
    for (u64 i = (u64)blockIdx.x * kBS + threadIdx.x; i < n; i += (u64)gridDim.x * kBS) out[i] = (u64)ids[i] + lo;
}
__global__ __launch_bounds__(kBS) void k_ids_to_bitmap(const u64 *__restrict__ ids, u64 n, u64 *bm) {
    for (u64 i = (u64)blockIdx.x * kBS + threadIdx.x; i < n; i += (u64)gridDim.x * kBS) {
        const u64 v = ids[i];
        atomicOr(bm + (v >> 6), 1ull << (v & 63u));
    }
}

#ifdef BFSX_DIAG
// Option race_probe (diagnostic): fill the LDS of every CU with 0x01010101 words, so that a push workgroup reading its
// queue counts before they are zeroed reads 16,843,009 (event (d)).
__global__ __launch_bounds__(kBS) void k_lds_poison() {
    __shared__ uint32_t s[8192]; // 32 KiB; several resident workgroups per CU cover its LDS
    for (int i = threadIdx.x; i < 8192; i += kBS) s[i] = 0x01010101u;
    __syncthreads();
    if (s[threadIdx.x ^ 1] == 0u) s[0] = 1u; // keeps the stores
}
#endif

// Multi-GPU host reads without a D2H copy + stream synchronise: one wave copies two device ranges into
// mapped pinned host memory and then publishes a sequence number the host spins on (as publish_if_last).
__global__ void k_post(const u64 *__restrict__ a, int na, const u64 *__restrict__ b, int nb, u64 *post, u64 seq) {
    for (int i = threadIdx.x; i < na + nb; i += blockDim.x) post[1 + i] = i < na ? a[i] : b[i - na];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) *(volatile u64 *)post = seq;
}

// Multi-GPU level close: one workgroup sums the level's counter shards into
//   out[0..6] = local {n_f, m_f, m_u, scanned, rows/claims, stage2, walked}   out[8..10] = copy of {n_f, m_f, m_u}
// (the copy is all-reduced in place; the local half stays for the per-level record), and zeroes the
// next top-down level's exchange counters `ctr` (nothing reads them after this level's claim kernel).
__global__ void k_level_sums(const LevelSlot *__restrict__ slot, int topdown, int64_t *__restrict__ out,
                             u64 *__restrict__ ctr, int nctr, int rank, int nranks, const u64 *err) {
    level_sums(slot, topdown, out, ctr, nctr, rank, nranks, err);
}

} // namespace

// Post `na` words at a and `nb` at b to the host (in order) and wait for them; out gets na + nb words.  The
// partitioned loop passes its communicator: the wait then also ends (BFSX_E_RCCL) when a peer rank aborted or
// the wait outlived the communicator's deadline (Comm::poll), instead of spinning behind a collective that
// will never complete.
int post_wait(BfsWorkspace *ws, hipStream_t st, const u64 *a, int na, const u64 *b, int nb, u64 *out,
              Comm *cm, const char *what) {
    hipLaunchKernelGGL(k_post, dim3(1), dim3(64), 0, st, a, na, b, nb, ws->d_post, ++ws->post_seq);
    BFSX_LAUNCHED(st);
    const volatile u64 *seq = ws->h_post;
    const int64_t t0 = cm ? now_ns() : 0;
    for (uint64_t spin = 1; *seq != ws->post_seq; spin++) {
        if (cm && (spin & 0xFFF) == 0)
            if (int rc = cm->poll(t0, what)) return rc;
        if ((spin & 0xFFFF) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e != hipSuccess && e != hipErrorNotReady)
                return fail(BFSX_E_HIP, std::string("exchange: ") + hipGetErrorString(e));
            if (e == hipSuccess && *seq != ws->post_seq) return fail(BFSX_E_HIP, "exchange counts were not posted");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    for (int i = 0; i < na + nb; i++) out[i] = ((const volatile u64 *)ws->h_post)[1 + i];
    return BFSX_OK;
}

// ==== multi-GPU level primitives (1-D partition) ====================================================
// The product runs the partitioned level loop natively (dist_bfs_run below, exchanges through
// bfsx_comm.cpp).  The primitives here step the same kernels one level at a time for the test suite's
// protocol driver (tests/dist_driver.py, include/bfsx_levels.h), which owns the exchange buffers and
// passes their device pointers in:
//   begin -> per level { td_expand -> all-to-all(pairs) -> td_claim | frontier_slice -> all-gather ->
//   bu_step } -> level_end (local counts; the caller all-reduces) -> finish.
namespace {

inline Part make_part(bfsx_graph *g, BfsWorkspace *ws) {
    Part p{};
    p.lo = (uint32_t)g->v_lo;
    p.chunk = (uint32_t)g->chunk;
    p.rank = (uint32_t)g->rank;
    p.remote = ws->remote;
    p.remote_tail = ws->d_dist_ctr;
    p.remote_cap = (u64)ws->remote_cap;
    p.nrows = (uint32_t)g->nv;
    p.err = ws->d_err;
    p.nranks = (uint32_t)g->nranks;
    return p;
}

int dist_ws(bfsx_graph *g) {
    int rc = ws_alloc(g);
    if (rc) return rc;
    if (!g->ws->d_dist_ctr) BFSX_HIP_TRY(hipMalloc(&g->ws->d_dist_ctr, kCtrWords * sizeof(u64)));
    // the push log (nv entries: a vertex is discovered once), before the first collective of the first BFS
    if (g->ctx->opt.push_log && !g->ws->plog)
        BFSX_HIP_TRY(hipMalloc(&g->ws->plog, (size_t)std::max<int64_t>(g->nv, 1) * sizeof(u64)));
    if (!g->ws->h_post) {
        BFSX_HIP_TRY(hipHostMalloc(&g->ws->h_post, kPostWords * sizeof(u64),
                                   hipHostMallocMapped | hipHostMallocCoherent));
        BFSX_HIP_TRY(hipHostGetDevicePointer((void **)&g->ws->d_post, g->ws->h_post, 0));
        g->ws->h_post[0] = 0;
        g->ws->post_seq = 0;
    }
    return BFSX_OK;
}

int dist_level_events(BfsWorkspace *ws, int level) {
    while ((int)ws->ev_level.size() <= level) {
        hipEvent_t e0, e1;
        BFSX_HIP_TRY(hipEventCreate(&e0));
        BFSX_HIP_TRY(hipEventCreate(&e1));
        ws->ev_begin.push_back(e0);
        ws->ev_level.push_back(e1);
    }
    return BFSX_OK;
}

} // namespace

// deg_known >= 0: the source's degree (the native loop reads its host degree table), so the owner
// needs no D2H read of its row bounds
int dist_begin(bfsx_graph *g, int64_t source, int64_t *deg_local, int64_t deg_known) {
    if (source < 0 || source >= g->nv_global) return fail(BFSX_E_RANGE, "source vertex outside the graph");
    int rc = dist_ws(g);
    if (rc) return rc;
    BfsWorkspace *ws = g->ws;
    hipStream_t st = g->ctx->stream;
    const bool owned = source >= g->v_lo && source < g->v_lo + g->nv;
    int64_t sl = owned ? source - g->v_lo : -1; // local internal row of the source
    if (owned && g->d_perm) {
        uint32_t x = 0;
        BFSX_HIP_TRY(hipMemcpy(&x, g->d_perm + sl, sizeof(x), hipMemcpyDeviceToHost));
        sl = (int64_t)x;
    }
    int64_t deg = 0;
    if (owned && deg_known >= 0) {
        deg = deg_known;
    } else if (owned) {
        int64_t so[2];
        BFSX_HIP_TRY(hipMemcpy(so, g->d_row_off + sl, sizeof(so), hipMemcpyDeviceToHost));
        deg = so[1] - so[0];
    }
    if (BFSX_DIAG_ON && g->ctx->opt.poison_queues) // test hook (see bfs_run_impl)
        for (uint32_t *q : {ws->qa, ws->qb, ws->hubs})
            BFSX_HIP_TRY(hipMemsetAsync(q, 0xFF, (size_t)std::max<int64_t>(g->nv, 1) * sizeof(uint32_t), st));
    BFSX_HIP_TRY(hipEventRecord(ws->ev_start, st));
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    hipLaunchKernelGGL(k_init, dim3(clamp_grid((ws->nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0, st,
                       owned ? (uint32_t)sl : 0xFFFFFFFFu, (uint32_t)(g->v_lo + sl), ws->prev_source, ws->dead, ws->nwords,
                       ws->st, ws->vis, ws->qa, ws->ring);
    BFSX_LAUNCHED(st);
    ws->prev_source = sl;
    // no pull-level records and no push log yet: the level primitives (tests/dist_driver.py) store packed states
    // only, and the native loop (dist_bfs_run) keeps its pull levels' records through its own RecLog.  A push log
    // left pending by an earlier one-device BFS on this workspace must not be scattered over this result.
    ws->n_prec = 0;
    ws->log_n = 0;
    ws->log_end.clear();
    ws->log_nd.clear();
    ws->logs_pending = false;
    ws->resolved = true;
    ws->d_level = 0;
    ws->d_dir = BFSX_DIR_TOPDOWN;
    ws->d_in_queue = true;
    ws->d_nf = owned ? 1 : 0;
    ws->d_mf = deg;
    g->level_dirs.clear();
    g->level_cum_ms.clear();
    g->level_stats.clear();
    // the result's source as the validator sees it: its global internal id on the owner; on the other
    // ranks of a relabelled partition nv_global, which names no row (only the owner knows the mapping)
    g->last_source = (owned || !g->d_perm) ? (owned ? g->v_lo + sl : source) : g->nv_global;
    *deg_local = deg;
    return BFSX_OK;
}

int dist_frontier_info(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local, int *in_queue) {
    if (!g->ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    *nf_local = g->ws->d_nf;
    *mf_local = g->ws->d_mf;
    *in_queue = g->ws->d_in_queue ? 1 : 0;
    return BFSX_OK;
}

int dist_td_expand(bfsx_graph *g, u64 *d_send, int64_t send_cap, int64_t *send_counts) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    hipStream_t st = g->ctx->stream;
    const int level = ws->d_level, P = g->nranks;
    if (int rc2 = dist_level_events(ws, level)) return rc2;
    BFSX_HIP_TRY(hipEventRecord(ws->ev_begin[level], st));
    if (!ws->d_in_queue) { // frontier held as a local bitmap slice (after a bottom-up level)
        BFSX_HIP_TRY(hipMemsetAsync(ws->d_cursor, 0, sizeof(u64), st));
        const int64_t per_block_min = (int64_t)kBS * kCompactWords;
        const unsigned gb = clamp_grid((ws->nwords + per_block_min - 1) / per_block_min, 256);
        const int64_t wpb = ((ws->nwords + gb - 1) / gb + per_block_min - 1) / per_block_min * per_block_min;
        hipLaunchKernelGGL(k_bitmap_to_queue, dim3(gb), dim3(kBS), 0, st, ws->front, ws->nwords, wpb, ws->qa,
                           ws->d_cursor, ws->nwords * 64);
        BFSX_LAUNCHED(st);
        ws->d_in_queue = true;
    }
    // remote pairs <= adjacency entries of the local frontier
    const int64_t need = std::max<int64_t>(ws->d_mf, 1);
    if (need > ws->remote_cap) {
        if (ws->remote) ws->retired.push_back({ws->remote, (size_t)ws->remote_cap * sizeof(u64)});
        ws->remote = nullptr;
        ws->remote_cap = std::max<int64_t>(need, 2 * ws->remote_cap);
        BFSX_HIP_TRY(hipMalloc(&ws->remote, ws->remote_cap * sizeof(u64)));
    }
    if (send_cap < ws->d_mf) return fail(BFSX_E_ARG, "send buffer smaller than the local frontier's m_f");
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_dist_ctr, 0, kCtrHead * sizeof(u64), st));
    const Part pt = make_part(g, ws);
    if (int e = launch_td<true>(g, ws, ws->d_nf, ws->d_mf, -1, level, pt)) return e;
    u64 n_remote = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&n_remote, ws->d_dist_ctr, sizeof(n_remote), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    u64 *dcount = ws->d_dist_ctr + 1, *dcursor = ws->d_dist_ctr + 1 + kMaxRanks;
    if (n_remote > 0) {
        const unsigned gbk = clamp_grid(((int64_t)n_remote + kBS - 1) / kBS, 1024);
        hipLaunchKernelGGL(k_bucket_count, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                           (u64)ws->remote_cap, (uint32_t)g->chunk, P, dcount, ws->d_err);
        BFSX_LAUNCHED(st);
        hipLaunchKernelGGL(k_bucket_scatter, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                           (u64)ws->remote_cap, (uint32_t)g->chunk, P, dcount, dcursor, d_send, (u64)send_cap,
                           ws->d_err);
        BFSX_LAUNCHED(st);
    }
    std::vector<u64> h(P, 0);
    BFSX_HIP_TRY(hipMemcpyAsync(h.data(), dcount, P * sizeof(u64), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    for (int p = 0; p < P; p++) send_counts[p] = (int64_t)h[p];
    ws->d_dir = BFSX_DIR_TOPDOWN;
    return BFSX_OK;
}

int dist_td_claim(bfsx_graph *g, const u64 *d_recv, int64_t n) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    if (n <= 0) return BFSX_OK;
    hipStream_t st = g->ctx->stream;
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    const dim3 grid(clamp_grid((n + kBS - 1) / kBS, cap));
    if (ws->off32)
        hipLaunchKernelGGL(k_claim_remote<uint32_t>, grid, dim3(kBS), 0, st, d_recv, (u64)n, ws->off32, ws->vis,
                           ws->st, ws->qb, ws->ring, ws->d_level, (uint32_t)g->v_lo, (u64)0, (uint32_t)g->nv, ws->d_err,
                           nullptr, nullptr, 0, nullptr, g->rank, g->nranks, nullptr, (u64)g->nv);
    else
        hipLaunchKernelGGL(k_claim_remote<int64_t>, grid, dim3(kBS), 0, st, d_recv, (u64)n, g->d_row_off,
                           ws->vis, ws->st, ws->qb, ws->ring, ws->d_level, (uint32_t)g->v_lo, (u64)0, (uint32_t)g->nv, ws->d_err,
                           nullptr, nullptr, 0, nullptr, g->rank, g->nranks, nullptr, (u64)g->nv);
    BFSX_LAUNCHED(st);
    return BFSX_OK;
}

int dist_frontier_slice(bfsx_graph *g, u64 *d_slice) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    hipStream_t st = g->ctx->stream;
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    if (int rc2 = dist_level_events(ws, ws->d_level)) return rc2;
    BFSX_HIP_TRY(hipEventRecord(ws->ev_begin[ws->d_level], st));
    if (ws->d_in_queue) {
        BFSX_HIP_TRY(hipMemsetAsync(d_slice, 0, ws->nwords * sizeof(u64), st));
        hipLaunchKernelGGL(k_queue_to_bitmap, dim3(clamp_grid((ws->d_nf + kBS - 1) / kBS, cap)), dim3(kBS), 0, st,
                           ws->qa, (uint32_t)ws->d_nf, d_slice, (uint32_t)g->nv, ws->d_err);
        BFSX_LAUNCHED(st);
    } else {
        BFSX_HIP_TRY(hipMemcpyAsync(d_slice, ws->front, ws->nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
    }
    BFSX_HIP_TRY(hipStreamSynchronize(st)); // the caller hands the slice to a collective next
    return BFSX_OK;
}

int dist_bu_step(bfsx_graph *g, const u64 *d_front_global) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    if (int e = launch_bu<true>(g, ws, d_front_global, ws->next, nullptr, ws->d_level)) return e;
    ws->d_dir = BFSX_DIR_BOTTOMUP;
    ws->d_in_queue = false;
    return BFSX_OK;
}

int dist_level_end(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    hipStream_t st = g->ctx->stream;
    const int level = ws->d_level;
    if (int rc2 = dist_level_events(ws, level)) return rc2;
    BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
    BFSX_HIP_TRY(hipMemcpyAsync(ws->h_slot, ws->ring + (level + 1) % 3, sizeof(LevelSlot), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    const SlotSums s = sum_slot(ws->h_slot);
    const bool td = ws->d_dir == BFSX_DIR_TOPDOWN;
    const int64_t nf_new = td ? (int64_t)ws->h_slot->qtail : s.nf;
    bfsx_level_stat ls{};
    ls.direction = ws->d_dir;
    ls.level = level;
    ls.frontier_in = ws->d_nf;
    ls.frontier_out = nf_new;
    ls.mf_in = ws->d_mf;
    ls.scanned = s.sc;
    ls.claims = s.cl;
    ls.stage2 = s.s2;
    ls.walked = s.wk;
    ls.explicit_parents = s.ex;
    g->level_stats.push_back(ls);
    g->level_dirs.push_back(ws->d_dir);
    if (td) std::swap(ws->qa, ws->qb);
    else std::swap(ws->front, ws->next);
    ws->d_in_queue = td;
    ws->d_nf = nf_new;
    ws->d_mf = s.mf;
    ws->d_level = level + 1;
    *nf_local = nf_new;
    *mf_local = s.mf;
    return BFSX_OK;
}

int dist_finish(bfsx_graph *g) {
    BfsWorkspace *ws = g->ws;
    if (!ws) return fail(BFSX_E_ARG, "bfsx_dist_begin first");
    hipStream_t st = g->ctx->stream;
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    {
        const unsigned wb = clamp_grid((ws->nwords + kBS - 1) / kBS, cap);
        hipLaunchKernelGGL(k_finalize, dim3(wb), dim3(kBS), 0, st, ws->vis, ws->nwords, ws->st);
    }
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipEventRecord(ws->ev_end, st));
    BFSX_HIP_TRY(hipEventSynchronize(ws->ev_end));
    if (int e = check_queue_guard(ws)) return e;
    {
        float ms = 0.f;
        BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_start, ws->ev_end));
        g->last_t_bfs_ms = ms;
    }
    for (int k = 0; k < 4; k++) {
        ws->comm_ms[k] = 0.0;
        ws->comm_n[k] = 0;
    }
    for (int i = 0; i < ws->n_comm; i++) { // option comm_timing (CommSpan): every span has completed by ev_end
        float ms = 0.f;
        const int k = ws->comm_kind[i];
        if (k >= 0 && k < 4 && hipEventElapsedTime(&ms, ws->ev_comm[2 * i], ws->ev_comm[2 * i + 1]) == hipSuccess) {
            ws->comm_ms[k] += ms;
            ws->comm_n[k]++;
        }
    }
    const int levels = ws->d_level;
    g->level_cum_ms.resize(levels);
    for (int l = 0; l < levels; l++) {
        float t = 0.f, k = 0.f;
        BFSX_HIP_TRY(hipEventElapsedTime(&t, ws->ev_start, ws->ev_level[l]));
        BFSX_HIP_TRY(hipEventElapsedTime(&k, ws->ev_begin[l], ws->ev_level[l]));
        g->level_cum_ms[l] = t;
        if (l < (int)g->level_stats.size()) {
            g->level_stats[l].cum_ms = t;
            g->level_stats[l].kernel_ms = k;
        }
    }
    return BFSX_OK;
}

// ==== multi-GPU native level loop ===================================================================
// The same level-synchronous loop as bfs_run, over a 1-D partition, with every exchange enqueued on
// the BFS stream through ctx->comm (RCCL or the in-process group).  Host waits per level: one for a
// bottom-up level (the all-reduced counters), two for a top-down level (+ the pair counts that size
// the grouped send/recv).  Distances are level-synchronous, so they are bit-identical to bfs_run's.
namespace {

// BFSX_TRACE: the device ranges of this rank's buffers at every push level of the partitioned loop (to match
// against a fault address or a runtime log)
void trace_buffers(const bfsx_graph *g, const BfsWorkspace *ws, int level) {
    const int64_t nv = std::max<int64_t>(g->nv, 1), nw = ws->nwords;
    const struct {
        const char *name;
        const void *p;
        int64_t bytes;
    } b[] = {{"row_off", g->d_row_off, (nv + 1) * 8},    {"col", g->d_col, g->nnz * 4},
             {"off32", ws->off32, (nv + 1) * 4},         {"st", ws->st, nv * 8},
             {"vis", ws->vis, nw * 8},                   {"front", ws->front, nw * 8},
             {"next", ws->next, nw * 8},                 {"dead", ws->dead, nw * 8},
             {"qa", ws->qa, nv * 4},                     {"qb", ws->qb, nv * 4},
             {"hubs", ws->hubs, nv * 4},                 {"top1", ws->top1, nv * 4},
             {"rest", ws->rest, nv * 16},                {"ring", ws->ring, 3 * (int64_t)sizeof(LevelSlot)},
             {"remote", ws->remote, ws->remote_cap * 8}, {"sendbuf", ws->sendbuf, ws->send_cap * 8},
             {"recvbuf", ws->recvbuf, ws->recv_cap * 8}, {"fglob", ws->fglob, ws->fglob_words * 8},
             {"dist_ctr", ws->d_dist_ctr, kCtrWords * 8}, {"post", ws->d_post, kPostWords * 8},
             {"err", ws->d_err, kErrWords * 8},                   {"pub", ws->d_pub, (int64_t)sizeof(Published)}};
    for (const auto &x : b)
        fprintf(stderr, "[bfsx] rank %d level %d buffer %-8s [0x%llx, 0x%llx)\n", g->rank, level, x.name,
                (unsigned long long)(uintptr_t)x.p, (unsigned long long)((uintptr_t)x.p + x.bytes));
}

// Option comm_timing: an event pair around one collective of the level loop on the BFS stream (bfsx_comm_times).
// The end event is recorded when the scope ends, also on an early error return.
struct CommSpan {
    bfsx_graph *g;
    BfsWorkspace *ws;
    int idx = -1;
    CommSpan(bfsx_graph *g_, BfsWorkspace *ws_, int op) : g(g_), ws(ws_) {
        if (!g->ctx->opt.comm_timing) return;
        const int k = ws->n_comm;
        while ((int)ws->ev_comm.size() < 2 * (k + 1)) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return;
            ws->ev_comm.push_back(e);
        }
        if ((int)ws->comm_kind.size() <= k) ws->comm_kind.resize(k + 1);
        ws->comm_kind[k] = op - 1;
        if (hipEventRecord(ws->ev_comm[2 * k], g->ctx->stream) != hipSuccess) return;
        idx = k;
        ws->n_comm = k + 1;
    }
    ~CommSpan() {
        if (idx >= 0) (void)hipEventRecord(ws->ev_comm[2 * idx + 1], g->ctx->stream);
    }
};

int grow(BfsWorkspace *ws, u64 *&buf, int64_t &cap, int64_t need) {
    if (need <= cap) return BFSX_OK;
    if (buf) ws->retired.push_back({buf, (size_t)cap * sizeof(u64)}); // freed with the workspace (BfsWorkspace::retired)
    buf = nullptr;
    cap = std::max<int64_t>(need, cap + cap / 2);
    BFSX_HIP_TRY(hipMalloc(&buf, cap * sizeof(u64)));
    return BFSX_OK;
}

// Option check_retired (test hook): fail when a buffer pointer the next launches or exchanges use lies inside a
// retired buffer (BfsWorkspace::retired) -- the debug assertion behind DESIGN.md 4, event (b): no kernel
// argument, copy source or LocalGroup posting of the partitioned loop refers to a replaced buffer.
int check_live(const bfsx_graph *g, const BfsWorkspace *ws, int level, const char *where,
               std::initializer_list<std::pair<const char *, const void *>> ptrs) {
    if (!g->ctx->opt.check_retired) return BFSX_OK;
    for (const auto &x : ptrs) {
        const uintptr_t a = (uintptr_t)x.second;
        if (!a) continue;
        for (const auto &r : ws->retired)
            if (a >= (uintptr_t)r.p && a < (uintptr_t)r.p + r.bytes)
                return fail(BFSX_E_HIP, std::string("check_retired: ") + where + " at level " + std::to_string(level) +
                                            " uses " + x.first + ", which lies inside a retired buffer");
    }
    return BFSX_OK;
}

// Once per graph (collective): the ORIGINAL ids of degree > big_degree with their degrees, all-gathered into
// a sorted host list (u64 id << 32 | degree).  It replaces a table of every id's degree (4 B per id: 4 GiB
// per rank at scale 30); a Kronecker graph has few such ids (options big_degree = 4096 and big_cap = 2^20
// ids per rank, else the list overflows and source degrees stay unknown).
int dist_big_list(bfsx_graph *g, BfsWorkspace *ws, Comm *cm) {
    hipStream_t st = g->ctx->stream;
    const int64_t thr = g->ctx->opt.big_degree;
    const u64 cap = (u64)g->ctx->opt.big_cap;
    const int P = g->nranks;
    // Collective: every rank takes part in both all-gathers whatever happens locally.  Everything that can
    // fail on one rank (allocations, the selection kernels) happens before the first one, and a failed rank
    // posts the count ~0, so that all ranks leave together with the same error.
    // the temporaries are retired into the workspace, not freed here (see BfsWorkspace::retired)
    struct Bufs {
        std::vector<BfsWorkspace::Retired> &sink;
        size_t chunk, cap, P;
        uint32_t *slice = nullptr;
        u64 *sel = nullptr, *cnt = nullptr, *all = nullptr;
        ~Bufs() {
            if (slice) sink.push_back({slice, chunk * sizeof(uint32_t)});
            if (sel) sink.push_back({sel, cap * sizeof(u64)});
            if (cnt) sink.push_back({cnt, (1 + kMaxRanks) * sizeof(u64)});
            if (all) sink.push_back({all, P * cap * sizeof(u64)});
        }
    } b{ws->retired, (size_t)g->chunk, (size_t)cap, (size_t)P};
    BFSX_HIP_TRY(hipMalloc(&b.cnt, (1 + kMaxRanks) * sizeof(u64)));
    bool ok = hipMalloc(&b.slice, g->chunk * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&b.sel, cap * sizeof(u64)) == hipSuccess &&
              hipMalloc(&b.all, (size_t)P * cap * sizeof(u64)) == hipSuccess &&
              hipMemsetAsync(b.cnt, 0, sizeof(u64), st) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_slice_degrees, dim3(clamp_grid((g->chunk + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                           g->d_row_off, g->d_perm, g->nv, g->chunk, b.slice);
        hipLaunchKernelGGL(k_select_big, dim3(clamp_grid((g->chunk + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                           b.slice, g->chunk, (uint32_t)thr, g->v_lo, b.sel, cap, b.cnt);
        ok = hipGetLastError() == hipSuccess;
    }
    if (!ok) {
        (void)hipGetLastError();
        const u64 bad = ~0ull;
        BFSX_HIP_TRY(hipMemcpyAsync(b.cnt, &bad, sizeof(bad), hipMemcpyHostToDevice, st));
    }
    if (int e = cm->allgather(b.cnt, 1, b.cnt + 1, st)) return e;
    std::vector<u64> counts(P, 0);
    if (int e = comm_fetch(cm, st, counts.data(), b.cnt + 1, P * sizeof(u64), "the degree-list all-gather")) return e;
    u64 maxc = 0;
    bool over = false;
    for (int p = 0; p < P; p++) {
        if (counts[p] == ~0ull)
            return fail(BFSX_E_OOM, "degree list of the partitioned loop: rank " + std::to_string(p) +
                                        " could not allocate or select its ids");
        maxc = std::max(maxc, counts[p]);
        over = over || counts[p] > cap;
    }
    const u64 mine = counts[g->rank];
    if (std::getenv("BFSX_TRACE"))
        fprintf(stderr, "[bfsx] rank %d: %llu ids of degree > %lld\n", g->rank, (unsigned long long)mine, (long long)thr);
    ws->h_big.clear();
    ws->big_overflow = over;
    if (!over) {
        maxc = std::max<u64>(maxc, 1);
        BFSX_HIP_TRY(hipMemsetAsync(b.sel + mine, 0xFF, (maxc - mine) * sizeof(u64), st));
        if (int e = cm->allgather(b.sel, (int64_t)maxc, b.all, st)) return e;
        std::vector<u64> h(P * maxc);
        if (int e = comm_fetch(cm, st, h.data(), b.all, h.size() * sizeof(u64), "the degree-list all-gather")) return e;
        for (u64 x : h)
            if (x != ~0ull) ws->h_big.push_back(x);
        std::sort(ws->h_big.begin(), ws->h_big.end());
    }
    ws->big_thr = thr;
    return BFSX_OK;
}

// level close: local sums + all-reduce of (n_f, m_f, m_u); returns [0..4] local, [8..10] global
int dist_level_close(bfsx_graph *g, BfsWorkspace *ws, bool td, int64_t out[kCtrSums16], bool summed) {
    hipStream_t st = g->ctx->stream;
    const int level = ws->d_level;
    int64_t *sums = reinterpret_cast<int64_t *>(ws->d_dist_ctr + kCtrSums);
    if (!summed) {
        hipLaunchKernelGGL(k_level_sums, dim3(1), dim3(64), 0, st, ws->ring + (level + 1) % 3, td ? 1 : 0, sums,
                           ws->d_dist_ctr, kCtrHead, g->rank, g->nranks, ws->d_err);
        BFSX_LAUNCHED(st);
    }
    BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
    Comm *cm = g->ctx->comm.get();
    {
        CommSpan span(g, ws, kOpAllreduce);
        if (int e = cm->allreduce_sum(sums + 8, 4 + g->nranks, st)) return e;
    }
    return post_wait(ws, st, reinterpret_cast<const u64 *>(sums), 12 + g->nranks, nullptr, 0,
                     reinterpret_cast<u64 *>(out), cm, "a level close");
}

// Option sparse_exchange: a pull level's global frontier travels as an id list when it holds fewer than n/128
// vertices (auto; 8 B per id against the n/8-byte bitmap all-gather), always (on, P > 1) or never (off).  The
// per-rank sizes come from the last level close; identical on every rank.
bool sparse_exchange(const bfsx_graph *g, int64_t nf_global, const std::vector<int64_t> &rank_nf) {
    const int mode = g->ctx->opt.sparse_exchange;
    if (g->nranks < 2 || mode == 0 || (int)rank_nf.size() != g->nranks) return false;
    return mode == 2 || nf_global * 128 < g->nv_global;
}

// The largest global m_f a push level exchanges through fixed slots (option slot_pairs; auto: a rank sends its
// P - 1 peers a slot of m_f + 1 words each whether it fills them or not, so the bound keeps that under 1 MiB --
// 16,384 pairs at P = 8 as before round 5, 131,072 at P = 2 -- and at P = 1, where nothing is sent, any level of up
// to 2^22 edges saves the count exchange and its host wait)
int64_t slot_pairs_for(const bfsx_graph *g) {
    const int64_t o = g->ctx->opt.slot_pairs;
    if (o >= 0) return o;
    const int64_t P = g->nranks;
    return P <= 1 ? ((int64_t)1 << 22) : std::max<int64_t>(16384, ((int64_t)1 << 20) / (8 * (P - 1)));
}

int dist_bfs_impl(bfsx_graph *g, int64_t source, bfsx_stats *stats, Comm *cm) {
    cm->tag = -1;
    if (g->ctx->opt.fail_rank == g->rank && g->ctx->opt.fail_level == -2) // test hook: before any collective
        return fail(BFSX_E_HIP, "fault injection: rank " + std::to_string(g->rank) + " fails before the first collective");
    int rc = dist_ws(g);
    if (rc) return rc;
    BfsWorkspace *ws = g->ws;
    if ((rc = ensure_hub_row_lim(g, ws))) return rc; // pull levels count their discoveries below it
    hipStream_t st = g->ctx->stream;
    const Options &opt = g->ctx->opt;
    const int P = g->nranks;
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    if (int e = grow(ws, ws->fglob, ws->fglob_words, ws->nwords * P)) return e;
    int64_t *sums = reinterpret_cast<int64_t *>(ws->d_dist_ctr + kCtrSums);
    int64_t h[kCtrSums16];
    if (ws->nnz_global < 0) { // once per graph
        h[0] = g->nnz;
        BFSX_HIP_TRY(hipMemcpyAsync(sums + 8, h, sizeof(int64_t), hipMemcpyHostToDevice, st));
        if (int e = cm->allreduce_sum(sums + 8, 1, st)) return e;
        if (int e = comm_fetch(cm, st, h, sums + 8, sizeof(int64_t), "the adjacency-count all-reduce")) return e;
        ws->nnz_global = h[0];
    }
    if (ws->big_thr < 0) {
        if (int e = dist_big_list(g, ws, cm)) return e; // once per graph (collective)
    }
    if (source < 0 || source >= g->nv_global) return fail(BFSX_E_RANGE, "source vertex outside the graph");
    // The first level's global m_f is the source's degree, which only its owner holds.  Every rank looks
    // the source up in the all-gathered list of ids with degree > big_thr: a listed source's degree is
    // exact; any other source has degree <= big_thr, a bound that sizes the level's fixed exchange slots
    // just as well (no rank sends more pairs than the source has edges).  An overflowed list leaves the
    // degree unknown: the level takes the counted exchange.  Decided identically on every rank.
    int64_t deg = -1, mf = 0;
    if (!ws->big_overflow) {
        const auto it = std::lower_bound(ws->h_big.begin(), ws->h_big.end(), (u64)source << 32);
        if (it != ws->h_big.end() && (int64_t)(*it >> 32) == source) deg = (int64_t)(*it & 0xFFFFFFFFull);
        mf = deg >= 0 ? deg : ws->big_thr;
    } else {
        mf = slot_pairs_for(g) + 1;
    }
    int64_t deg_local = 0;
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_dist_ctr, 0, kCtrHead * sizeof(u64), st)); // before the timed region
    // (dist_begin clears a stale push log of an earlier one-device BFS on this workspace)
    if ((rc = dist_begin(g, source, &deg_local, deg))) return rc;

    int dir = (opt.direction == BFSX_DIR_BOTTOMUP) ? BFSX_DIR_BOTTOMUP : BFSX_DIR_TOPDOWN;
    const bool owner = source >= g->v_lo && source < g->v_lo + g->nv;
    // the local frontier's largest degree (-1: unknown): at most hub_degree means the next push level needs no
    // hub bin (k_td_hubs is not launched).  After a push level the kernels' d_max; after a pull level
    // hub_degree when it found no vertex below hub_row_lim (the rows that can exceed hub_degree)
    int64_t dmax_local = owner ? deg_local : 0;
    // m_u: an unlisted source's degree (<= big_thr of ~10^9 entries) is left in it until the first pull
    // level recounts m_u exactly; it only feeds Beamer's switch
    int64_t nf = 1, prev_nf = 0, mu = ws->nnz_global - std::max<int64_t>(deg, 0), examined = 0;
    // m_u of this rank's unvisited rows.  A pull level reports the exact m_u it leaves (the degree sum
    // of its unvisited candidates), so the m_f of the frontier it found is the m_u it consumed: no
    // per-discovery degree read in the pull kernel.  Before the first pull level the count still holds
    // the isolated self-loop-only rows' entries, which can only over-state that m_f (a safe bound for
    // the next push level's pair buffers).
    int64_t mu_local = g->nnz - (owner ? deg_local : 0);
    int64_t visited_local = owner ? 1 : 0;
    int td_levels = 0, bu_levels = 0;
    // the local bitmap frontier: ws->front after a push -> pull conversion, the last pull level's record after a
    // pull level; pull levels store 4-B parents plus their record, as on one device (RecLog, BfsWorkspace::par)
    const u64 *bmf = ws->front;
    RecLog recs(g, ws);
    std::vector<int64_t> rank_nf; // every rank's frontier size after the last level close (all-reduced)
    int64_t nf_core = -1;         // after a pull level: its local discoveries below leaf_lo (-1: unknown)
    ExchangePlan plan;
    std::vector<u64> hc(2 * kMaxRanks);
    ws->n_comm = 0; // comm_timing: this BFS's collectives
    for (;;) {
        const int level = ws->d_level;
        cm->tag = level;
        if (opt.fail_rank == g->rank && opt.fail_level == level) // test hook: this rank fails mid-BFS
            return fail(BFSX_E_HIP, "fault injection: rank " + std::to_string(g->rank) + " fails at level " +
                                        std::to_string(level));
        if (opt.direction == BFSX_DIR_AUTO && level > 0) {
            // Beamer's rule, plus the exchange cost: a top-down level ships up to 8*m_f*(P-1)/P bytes of
            // (vertex, parent) pairs, a bottom-up level all-gathers an n/8-byte bitmap -- pull as soon as
            // the pairs would outweigh the bitmap
            const bool pairs_heavy = P > 1 && mf * 64 * (P - 1) > g->nv_global * P;
            if (dir == BFSX_DIR_TOPDOWN) {
                if (mf > mu / std::max(opt.alpha, 1) || pairs_heavy) dir = BFSX_DIR_BOTTOMUP;
            } else if (nf < g->nv_global / std::max(opt.beta, 1) && nf < prev_nf && !pairs_heavy) {
                dir = BFSX_DIR_TOPDOWN;
            }
        }
        if (int e = dist_level_events(ws, level)) return e;
        BFSX_HIP_TRY(hipEventRecord(ws->ev_begin[level], st));
        const bool td = dir == BFSX_DIR_TOPDOWN;
        bool summed = false; // the level's last kernel already closed the level (k_claim_remote)
        u64 *plog = nullptr; // a push level's push-log segment
        int64_t nq = ws->d_nf; // the push queue's length
        if (td) {
            if (!ws->d_in_queue) { // local bitmap slice -> queue
                // leaf skip (as on one device): after a pull level the discoveries at local ids >= leaf_lo have
                // one adjacency entry, their parent, and sweep nothing; the queue holds the nf_core others (the
                // pull kernel counted them)
                const bool skip = opt.leaf_skip && nf_core >= 0 && ws->leaf_lo < g->nv;
                const int64_t lim = skip ? ws->leaf_lo : ws->nwords * 64;
                const int64_t cw = (lim + 63) / 64;
                BFSX_HIP_TRY(hipMemsetAsync(ws->d_cursor, 0, sizeof(u64), st));
                const int64_t per_block_min = (int64_t)kBS * kCompactWords;
                const unsigned gb = clamp_grid(std::max<int64_t>((cw + per_block_min - 1) / per_block_min, 1), 256);
                const int64_t wpb = ((cw + gb - 1) / gb + per_block_min - 1) / per_block_min * per_block_min;
                hipLaunchKernelGGL(k_bitmap_to_queue, dim3(gb), dim3(kBS), 0, st, bmf, cw, wpb, ws->qa,
                                   ws->d_cursor, lim);
                BFSX_LAUNCHED(st);
                if (skip) nq = nf_core;
                ws->d_in_queue = true;
            }
            // remote pairs <= adjacency entries of the local frontier
            const int64_t need = std::max<int64_t>(ws->d_mf, 1);
            if (need > ws->remote_cap) {
                if (ws->remote) ws->retired.push_back({ws->remote, (size_t)ws->remote_cap * sizeof(u64)});
                ws->remote = nullptr;
                ws->remote_cap = std::max<int64_t>(need, 2 * ws->remote_cap);
                BFSX_HIP_TRY(hipMalloc(&ws->remote, ws->remote_cap * sizeof(u64)));
            }
            if (int e = grow(ws, ws->sendbuf, ws->send_cap, need)) return e;
            // the exchange counters are zero: dist_bfs_run zeroes them before the first level, every
            // level's close (k_claim_remote's last workgroup or k_level_sums) after its exchange
            Part pt = make_part(g, ws);
            static const bool trace_bufs = std::getenv("BFSX_TRACE") != nullptr;
            if (trace_bufs) trace_buffers(g, ws, level);
            u64 *dcount = ws->d_dist_ctr + 1, *dcursor = ws->d_dist_ctr + 1 + kMaxRanks;
            // pair count read on the device: the grid is sized by its upper bound, the local m_f
            const unsigned gbk = clamp_grid((need + kBS - 1) / kBS, 1024);
            int64_t slot = 0, ro = 0; // slot > 0: fixed-slot exchange
            if (mf <= slot_pairs_for(g)) {
                // small level: no rank sends more than the global m_f pairs to any peer, so every peer gets
                // a fixed slot [count, m_f pairs] -- one exchange, no count all-to-all, no host wait.  The push
                // kernels write the pairs into the slots themselves; the last one's last workgroup writes the
                // counts (dcount, unused by the slot exchange, counts its arrivals)
                slot = std::max<int64_t>(mf, 1);
                if (BFSX_DIAG_ON && opt.slot_force > 0) slot = opt.slot_force; // test hook: a slot bound too small
                if (int e = grow(ws, ws->sendbuf, ws->send_cap, P * (slot + 1))) return e;
                if (int e = grow(ws, ws->recvbuf, ws->recv_cap, P * (slot + 1))) return e;
                pt.slot_out = ws->sendbuf;
                pt.slot_cap = (u64)slot;
                pt.slot_cursor = dcursor;
                pt.slot_arrive = dcount;
                plan_slots(P, slot, plan, g->rank); // the own slot stays empty and is not exchanged
                ro = (int64_t)(P - 1) * slot; // candidate entries the claim kernel reads: the peers' slots
            }
            if (int e = check_live(g, ws, level, "push kernels",
                                   {{"queue in", ws->qa}, {"queue out", ws->qb}, {"hubs", ws->hubs}, {"vis", ws->vis},
                                    {"state", ws->st}, {"remote", pt.remote}, {"slot_out", pt.slot_out},
                                    {"counters", ws->d_dist_ctr}, {"front", ws->front}}))
                return e;
            // the push log (option push_log, as on one device): this level's winners, local claims and remote ones
            // alike, are (vertex, parent) pairs at their queue positions in the log segment [log_n, log_n + n_f)
            plog = opt.push_log ? ws->plog + ws->log_n : nullptr;
#ifdef BFSX_DIAG
            if (opt.race_probe) { // test hook: stale LDS + a late queue init (k_td)
                hipLaunchKernelGGL(k_lds_poison, dim3(g->ctx->num_cus * 8), dim3(kBS), 0, st);
                BFSX_LAUNCHED(st);
                pt.probe = (uint32_t)opt.race_probe;
            }
#endif
            if (int e = launch_td<true>(g, ws, nq, ws->d_mf, dmax_local, level, pt, false, nullptr, 0, nullptr, plog))
                return e;
            if (!slot) {
                hipLaunchKernelGGL(k_bucket_count, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                                   (u64)ws->remote_cap, (uint32_t)g->chunk, P, dcount, ws->d_err);
                BFSX_LAUNCHED(st);
                hipLaunchKernelGGL(k_bucket_scatter, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                                   (u64)ws->remote_cap, (uint32_t)g->chunk, P, dcount, dcursor, ws->sendbuf,
                                   (u64)ws->send_cap, ws->d_err);
                BFSX_LAUNCHED(st);
                u64 *drecv = ws->d_dist_ctr + kCtrRecv;
                {
                    CommSpan span(g, ws, kOpAlltoall1);
                    if (int e = cm->alltoall1(reinterpret_cast<int64_t *>(dcount), reinterpret_cast<int64_t *>(drecv), st))
                        return e;
                }
                if (int e = post_wait(ws, st, dcount, P, drecv, P, hc.data(), cm, "a pair-count exchange")) return e;
                hc[P + g->rank] = 0; // alltoall1 does not exchange the own entry (no pairs route to it)
                plan_counted(P, hc.data(), hc.data() + P, plan);
                ro = plan.recv_total;
                if (int e = grow(ws, ws->recvbuf, ws->recv_cap, std::max<int64_t>(ro, 1))) return e;
            }
            if (int e = check_live(g, ws, level, "pair exchange + claim",
                                   {{"sendbuf", ws->sendbuf}, {"recvbuf", ws->recvbuf}, {"remote", ws->remote}}))
                return e;
            {
                CommSpan span(g, ws, kOpAlltoallv);
                if (int e = cm->alltoallv(ws->sendbuf, plan.scount.data(), plan.sdispl.data(), ws->recvbuf,
                                          plan.rcount.data(), plan.rdispl.data(), st))
                    return e;
            }
            if (ro > 0) { // its last workgroup closes the level (the sums k_level_sums would compute)
                const dim3 grid(clamp_grid((ro + kBS - 1) / kBS, cap));
                const u64 qcap = (u64)std::max<int64_t>(plog ? g->nv - ws->log_n : g->nv, 0); // as the push kernels'
                u64 *arrive = ws->d_dist_ctr + kCtrHead - 1;
                if (ws->off32)
                    hipLaunchKernelGGL(k_claim_remote<uint32_t>, grid, dim3(kBS), 0, st, ws->recvbuf, (u64)ro,
                                       ws->off32, ws->vis, ws->st, ws->qb, ws->ring, level, (uint32_t)g->v_lo,
                                       (u64)slot, (uint32_t)g->nv, ws->d_err, sums, ws->d_dist_ctr, kCtrHead, arrive,
                                       g->rank, g->nranks, plog, qcap);
                else
                    hipLaunchKernelGGL(k_claim_remote<int64_t>, grid, dim3(kBS), 0, st, ws->recvbuf, (u64)ro,
                                       g->d_row_off, ws->vis, ws->st, ws->qb, ws->ring, level, (uint32_t)g->v_lo,
                                       (u64)slot, (uint32_t)g->nv, ws->d_err, sums, ws->d_dist_ctr, kCtrHead, arrive,
                                       g->rank, g->nranks, plog, qcap);
                BFSX_LAUNCHED(st);
                summed = true;
            }
            td_levels++;
        } else if (sparse_exchange(g, nf, rank_nf)) {
            // a small global frontier travels as an id list (4-8 B per id instead of the n/8-byte bitmap
            // all-gather): every rank sends its ids to every rank, then sets them in the global bitmap
            const int64_t mine = ws->d_nf;
            if (int e = grow(ws, ws->sendbuf, ws->send_cap, std::max<int64_t>(mine, 1))) return e;
            if (int e = grow(ws, ws->recvbuf, ws->recv_cap, std::max<int64_t>(nf, 1))) return e;
            const uint32_t *ids = ws->qa;
            if (!ws->d_in_queue) { // the last pull level's record -> local ids
                BFSX_HIP_TRY(hipMemsetAsync(ws->d_cursor, 0, sizeof(u64), st));
                const int64_t per_block_min = (int64_t)kBS * kCompactWords;
                const unsigned gb = clamp_grid((ws->nwords + per_block_min - 1) / per_block_min, 256);
                const int64_t wpb = ((ws->nwords + gb - 1) / gb + per_block_min - 1) / per_block_min * per_block_min;
                hipLaunchKernelGGL(k_bitmap_to_queue, dim3(gb), dim3(kBS), 0, st, bmf, ws->nwords, wpb, ws->qb,
                                   ws->d_cursor, ws->nwords * 64);
                BFSX_LAUNCHED(st);
                ids = ws->qb;
            }
            if (mine > 0) {
                hipLaunchKernelGGL(k_ids_global, dim3(clamp_grid((mine + kBS - 1) / kBS, cap)), dim3(kBS), 0, st, ids,
                                   (u64)mine, (uint32_t)g->v_lo, ws->sendbuf);
                BFSX_LAUNCHED(st);
            }
            plan_broadcast(P, mine, rank_nf.data(), plan);
            u64 *rec = nullptr;
            if (int e = recs.take(&rec)) return e;
            if (int e = check_live(g, ws, level, "sparse frontier exchange + pull kernel",
                                   {{"sendbuf", ws->sendbuf}, {"recvbuf", ws->recvbuf}, {"fglob", ws->fglob},
                                    {"record", rec}, {"vis", ws->vis}, {"parents", ws->par}}))
                return e;
            {
                CommSpan span(g, ws, kOpAlltoallv);
                if (int e = cm->alltoallv(ws->sendbuf, plan.scount.data(), plan.sdispl.data(), ws->recvbuf,
                                          plan.rcount.data(), plan.rdispl.data(), st))
                    return e;
            }
            BFSX_HIP_TRY(hipMemsetAsync(ws->fglob, 0, (size_t)ws->nwords * P * sizeof(u64), st));
            if (plan.recv_total > 0) {
                hipLaunchKernelGGL(k_ids_to_bitmap, dim3(clamp_grid((plan.recv_total + kBS - 1) / kBS, cap)), dim3(kBS),
                                   0, st, ws->recvbuf, (u64)plan.recv_total, ws->fglob);
                BFSX_LAUNCHED(st);
            }
            ws->d_in_queue = false;
            if (int e = launch_bu<false>(g, ws, ws->fglob, rec, ws->par, level)) return e;
            recs.done(level + 1);
            bmf = rec;
            bu_levels++;
        } else {
            if (ws->d_in_queue) { // after a push level: the visited slice stands for the frontier slice
                // (every visited vertex an unvisited one can touch is in the frontier: kernels_level.hip, bfs_run;
                // globally the same, so the all-gathered visited slices serve the pull kernel as the frontier)
                BFSX_HIP_TRY(hipMemcpyAsync(ws->front, ws->vis, ws->nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
                bmf = ws->front;
                ws->d_in_queue = false;
            }
            u64 *rec = nullptr;
            if (int e = recs.take(&rec)) return e;
            if (int e = check_live(g, ws, level, "frontier all-gather + pull kernel",
                                   {{"front", bmf}, {"fglob", ws->fglob}, {"record", rec}, {"vis", ws->vis},
                                    {"parents", ws->par}}))
                return e;
            {
                CommSpan span(g, ws, kOpAllgather);
                if (int e = cm->allgather(bmf, ws->nwords, ws->fglob, st)) return e;
            }
            if (int e = launch_bu<false>(g, ws, ws->fglob, rec, ws->par, level)) return e; // m_f from m_u (below)
            recs.done(level + 1);
            bmf = rec;
            bu_levels++;
        }
        if (int e = dist_level_close(g, ws, td, h, summed)) return e;
        if (h[11 + P] != 0) { // a queue guard fired on some rank(s) this level: every rank fails here, together
            std::string who;
            for (int r = 0; r < P; r++)
                if ((uint64_t)h[11 + P] >> r & 1ull) who += (who.empty() ? "" : ", ") + std::to_string(r);
            std::string mine;
            if (check_queue_guard(ws)) mine = " (this rank: " + last_error() + ")";
            cm->agreed = true; // every rank leaves here with this error: the communicator stays usable
            return fail(BFSX_E_HIP, "device guard (queue id / store bound) fired at level " + std::to_string(level) +
                                        " on rank(s) " + who + mine);
        }
        static const bool trace = std::getenv("BFSX_TRACE") != nullptr;
        if (trace)
            fprintf(stderr, "[bfsx] rank %d level %d %s: nf %lld -> %lld (global %lld)\n", g->rank, level,
                    td ? "push" : "pull", (long long)ws->d_nf, (long long)h[0], (long long)h[8]);
        // per-level record (local counts) and state advance
        bfsx_level_stat ls{};
        ls.direction = dir;
        ls.level = level;
        ls.frontier_in = ws->d_nf;
        ls.frontier_out = h[0];
        ls.mf_in = ws->d_mf;
        ls.unvisited_in = g->nv - visited_local - ws->n_dead;
        ls.scanned = h[3];
        ls.claims = h[4];
        ls.stage2 = h[5];
        ls.walked = h[6];
        ls.explicit_parents = td ? 0 : h[0]; // a partition's pull levels store every parent explicitly
        g->level_stats.push_back(ls);
        g->level_dirs.push_back(dir);
        examined += h[3];
        visited_local += h[0];
        if (td) std::swap(ws->qa, ws->qb);
        if (plog && h[0] > 0) { // the level's local winners are log entries [log_n, log_n + n_f)
            ws->log_n += h[0];
            ws->log_end.push_back(ws->log_n);
            ws->log_nd.push_back(level + 1);
        }
        dmax_local = td ? h[7] : (h[7] == 0 ? (int64_t)opt.hub_degree : -1);
        nf_core = td ? -1 : h[1]; // a pull level's local discoveries below leaf_lo (k_bu counts them in m_f)
        rank_nf.assign(h + 11, h + 11 + P);
        ws->d_dir = dir;
        ws->d_in_queue = td;
        ws->d_nf = h[0];
        ws->d_level = level + 1;
        prev_nf = nf;
        nf = h[8];
        if (td) { // the push kernels and the claims sum the degrees of what they discover
            ws->d_mf = h[1];
            mf = h[9];
            mu -= mf;
            mu_local -= h[1];
        } else { // the pull kernel reports the m_u it leaves: what it found held the difference
            ws->d_mf = std::max<int64_t>(mu_local - h[2], 0);
            mf = std::max<int64_t>(mu - h[10], 0);
            mu = h[10];
            mu_local = h[2];
        }
        if (nf == 0) break;
    }
    cm->tag = -2;
    recs.finish();
    if (ws->log_n > 0) { // scattered into st by bfs_resolve / the unpack, outside the timed region
        ws->logs_pending = true;
        ws->resolved = false;
    }
    if ((rc = dist_finish(g))) return rc;
    if (stats) {
        *stats = bfsx_stats{};
        stats->levels = ws->d_level;
        stats->topdown_levels = td_levels;
        stats->bottomup_levels = bu_levels;
        stats->edges_examined = examined;
        float ms = 0.f;
        BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_start, ws->ev_end));
        stats->t_bfs_ms = ms;
        int64_t m = 0, r = 0;
        if ((rc = bfs_mcomp(g, &m, &r))) return rc;
        h[0] = m;
        h[1] = r;
        BFSX_HIP_TRY(hipMemcpyAsync(sums + 8, h, 2 * sizeof(int64_t), hipMemcpyHostToDevice, st));
        if (int e = cm->allreduce_sum(sums + 8, 2, st)) return e;
        if (int e = comm_fetch(cm, st, h, sums + 8, 2 * sizeof(int64_t), "the m_comp all-reduce")) return e;
        stats->m_comp = h[0];
        stats->reached = h[1];
    }
    return BFSX_OK;
}

} // namespace

// The partitioned BFS, collective: a rank that fails aborts the group (comm_guard), so every rank returns an
// error instead of waiting for it inside a collective ("A failed rank fails every rank").
int dist_bfs_run(bfsx_graph *g, int64_t source, bfsx_stats *stats) {
    Comm *cm = g->ctx->comm.get();
    if (!cm) return fail(BFSX_E_ARG, "no communicator on this context (bfsx_comm_init / bfsx_comm_local_group)");
    if (cm->nranks != g->nranks || cm->rank != g->rank)
        return fail(BFSX_E_ARG, "graph partition does not match the communicator's rank/size");
    if (cm->failed()) return cm->poll(now_ns(), "a BFS on an aborted communicator");
    // argument errors are the same on every rank (every rank passes the same source): no abort
    if (source < 0 || source >= g->nv_global) return fail(BFSX_E_RANGE, "source vertex outside the graph");
    comm_sync_options(g->ctx);
    return comm_guard(cm, dist_bfs_impl(g, source, stats, cm));
}


} // namespace bfsx
