// bfs_core.h -- shared core of the BFS kernels (not part of the C-ABI): the per-graph device workspace, the
// level counter slots, the wave/workgroup helpers every kernel family uses, the frontier-conversion and record
// kernels more than one level loop launches, and the host entry points the kernel families export to the loops.
//
// The kernel families (one translation unit each) replace the reference's per-level Spark job
// (BfsSpark.java:61-118):
//   kernels_push.hip     mapper (:66-87) GRAY u emits (n, d+1) for n in N(u) -> top-down push k_td / k_td_hubs;
//                        the reducer (:90-108, min distance / darkest colour) is fused into it as an atomicOr
//                        claim on the visited bitmap (every contender of a level carries the same level+1, so
//                        the min is race-free and exact)
//   kernels_pull.hip     (no reference analogue) bottom-up pull k_bu / k_bu_sparse, Beamer's direction switch
//   kernels_persist.hip  K3p: many narrow push levels per launch (high-diameter graphs, BreadthFirstPaths.java:33)
//   kernels_level.hip    the single-device level loop, collect + contains("GRAY") (:110-117) as a device counter
//                        slot published to mapped host memory, the workspace, the result unpack
//   kernels_dist.hip     the 1-D partitioned level loop (multi-GPU, the shuffle of :90 as RCCL exchanges)
// State: one packed 64-bit word per vertex, st[v] = parent << 32 | dist (dist INT32_MAX = WHITE, the
// reference's Integer.MAX_VALUE; parent 0xFFFFFFFF = none), so a discovery is ONE 8-byte store instead
// of two scattered 4-byte stores; the visited bitmap u64[n/64] (BLACK|GRAY, pre-set for isolated
// vertices); the frontier as a queue u32[] (top-down) or a bitmap u64[] (bottom-up).
// Row offsets are read as uint32 when the graph's adjacency has < 2^32 entries (half the bytes of the
// int64 CSR offsets on every vertex probe), as int64 otherwise; every traversal kernel is templated on it.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <initializer_list>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "bfsx_internal.h"
#include "exchange_plan.h"

namespace bfsx {

// Diagnostic build (libbfsx_diag.so, -DBFSX_DIAG): the test hooks (poison_queues, test_overread, bu_force_spill's
// spilling pull kernel, persist_abort_at, check_retired, fail_at) and the encoded hub probe domain of graphs built
// without the relabel are compiled only there; the product library refuses those options.
#ifdef BFSX_DIAG
constexpr bool BFSX_DIAG_ON = true;
#else
constexpr bool BFSX_DIAG_ON = false;
#endif

using u64 = unsigned long long;

constexpr int kBS = 256;
constexpr int kWaves = kBS / 64;
constexpr int kShards = 64; // stat counters are spread over 64 lines: a single device-scope counter hit
                            // by every workgroup costs ~12 ns per arrival (MI355X_MICROARCH fan-in row)
constexpr u64 kUnreached = 0xFFFFFFFF7FFFFFFFull; // parent = 0xFFFFFFFF (-1), dist = INT32_MAX

__device__ __host__ inline u64 pack_state(uint32_t parent, int32_t d) { return ((u64)parent << 32) | (uint32_t)d; }

struct alignas(64) StatShard {
    u64 nf;      // vertices in the produced frontier (bottom-up)
    u64 mf;      // sum of their degrees (Beamer m_f; top-down levels and the multi-GPU bottom-up step)
    u64 scanned; // adjacency entries read (algorithmic-bytes accounting)
    u64 claims;  // top-down atomicOr claims attempted (diagnostics)
    u64 mu;      // bottom-up: degree sum of the candidates left unvisited (Beamer m_u, exact)
    u64 stage2;  // bottom-up: candidates that loaded rest[] (stage A2, 16 B each)
    u64 walked;  // bottom-up: adjacency entries read from col in phase B (4 B each)
    u64 nhub;    // bottom-up, single device: vertices found below hub_row_lim (the only possible hubs)
    u64 expl;    // discoveries that stored an explicit 4-B parent (provenance code kCodeExplicit; bytes accounting)
    u64 dmax;    // top-down: largest degree in the produced frontier (skips the hub bin when <= hub_deg)
};
constexpr int kStatFields = 9; // summed fields, in declaration order (dmax is a max)

// Counters of one level.  Level L reads slot L%3 (its own frontier, already on the host), accumulates
// the frontier it produces into slot (L+1)%3 and zeroes slot (L+2)%3: no per-level memset.
struct alignas(64) DoneShard {
    u64 n;
    u64 pad[7];
};
constexpr int kDoneShards = 8; // arrival counters of publish_if_last, one line each (blockIdx % 8)

struct LevelSlot {
    u64 qtail; // top-down next-queue allocation cursor (= frontier size produced)
    u64 nhub;  // top-down hub-list length
    u64 done;  // shards of the publishing kernel whose workgroups have all finished (publish_if_last)
    u64 pad[5];
    StatShard sh[kShards];
    DoneShard dsh[kDoneShards]; // finished workgroups of the publishing kernel, per blockIdx % 8
};
constexpr int kSlotWords = (int)(sizeof(LevelSlot) / sizeof(u64));

// K3p (persistent top-down, below): per-level records and the grid-barrier state of one launch.
constexpr uint32_t kPersistNf = 8192; // widest frontier a K3p level may produce and still continue
constexpr int kPersistLevels = 1024;  // levels per launch

struct alignas(64) PersistRec {
    u64 qtail, mf, dmax, scanned, claims, t_end, mfh, pad; // mfh: degree sum of the hubs discovered
};
constexpr int kRecWords = 7; // per-workgroup record words of a K3p level

struct alignas(128) PersistCtl {
    u64 abort; // raised by a workgroup whose poll timed out or whose segment would overflow
    u64 pad[15];
};
// host-visible result of one launch (mapped pinned memory, written by workgroup 0)
struct alignas(64) PersistOut {
    u64 levels, abort, t0, done; // done: set by workgroup 0 once levels / abort / the records are final
    u64 front;                   // the launch stopped for Beamer's rule and left its last frontier as a bitmap too
    u64 pad[3];
    PersistRec rec[kPersistLevels];
};

// A level's counter sums as the host reads them (mapped pinned memory, written by publish_if_last).
struct alignas(64) Published {
    u64 seq;
    int64_t qtail, nf, mf, sc, cl, mu, dmax, stage2, walked, nhub, expl;
};

struct BfsWorkspace {
    int64_t nv = 0, nwords = 0;
    u64 *st = nullptr;                  // packed parent << 32 | dist
    // Pull levels (single device) store only a 4-B parent, par[v]; their discoveries are the level's record
    // bitmap prec[k] (the `next` bitmap k_bu writes anyway, kept per level instead of swapped), which gives
    // them distance prec_lvl[k] + 1.  st[v] of such a vertex is stale until bfs_resolve (or the fused unpack)
    // reads the records -- outside the timed region, like the unpack to original ids.
    uint32_t *par = nullptr;
    // how each pull discovery's parent is named (kCodeTop1 .. kCodeExplicit); single device only (null on a
    // partition, whose pull levels store every parent explicitly)
    uint8_t *pcode = nullptr;
    // the original ids of top1 / rest (relabelled graphs; the unpack's parents of code 0-3 without an inv gather),
    // built at the first unpack when the device has room for them (else the unpack maps through inv)
    uint32_t *otop1 = nullptr;
    uint4 *orest = nullptr;
    bool orig_nbrs_tried = false;
    std::vector<u64 *> prec;            // record pool (grown on demand, kept across BFS runs)
    std::vector<int32_t> prec_nd;       // distance of record k's vertices (its level + 1), last BFS
    int n_prec = 0;                     // records of the last BFS
    bool resolved = true;               // st holds every reached vertex's state (no record or log pending)
    // Push log (single device, round 4): the winners of a per-level push level (k_td / k_td_hubs, not K3p) are
    // written as vertex | parent << 32 at their next-frontier queue positions -- coalesced through the LDS
    // queue -- instead of one scattered 8-B state store each.  Level k's entries are plog[log_end[k-1],
    // log_end[k]) with distance log_nd[k]; bfs_resolve / the unpack scatter them into st (apply_logs), outside
    // the timed region like the pull records.
    u64 *plog = nullptr;                // nv entries (a vertex is discovered once)
    int64_t log_n = 0;                  // entries of the last BFS
    std::vector<int64_t> log_end;
    std::vector<int32_t> log_nd;
    bool logs_pending = false;          // entries not yet scattered into st
    int64_t *d_log_meta = nullptr;      // device copy of log_end + log_nd for k_resolve_log
    int64_t log_meta_cap = 0;
    uint32_t *off32 = nullptr;          // uint32 copy of the row offsets (nnz < 2^32), else null
    u64 *vis = nullptr, *front = nullptr, *next = nullptr;
    // single device (option vis_front): the second visited buffer.  A pull level whose frontier is the visited
    // bitmap itself (after a push, hybrid or K3p level) reads vis and writes vis | its discoveries into
    // bu_vis_out (= vis2, one-shot, consumed by the next pull launch); the loop then swaps vis and vis2
    u64 *vis2 = nullptr, *bu_vis_out = nullptr;
    u64 *dead = nullptr;                // isolated vertices + padding (initial visited bitmap)
    int64_t n_dead = 0;                 // isolated vertices (excluding padding)
    uint32_t *top1 = nullptr;           // first (highest-degree) neighbour of every vertex (+ kDeg1 flag)
    uint4 *rest = nullptr;              // {2nd, 3rd, 4th neighbour, degree} of every vertex (k_bu stage A2)
    uint32_t top1_flag = 0;             // kDeg1 when every global id < 2^31, else 0 (flag unused)
    // hub-encoded probe domain of the bottom-up kernel (single device; see k_bu): the hub_k highest-degree
    // vertices, their frontier bits gathered into a small bitmap per bottom-up level
    int64_t hub_k = 0;                  // 0: off
    uint32_t *hub_id = nullptr;         // [hub_k] global id of hub h (degree descending)
    uint32_t hub_tdeg = 0xFFFFFFFFu;    // the hubs are exactly the vertices of degree >= hub_tdeg
    // relabelled graph (ids in degree order): the hubs of the hybrid levels are the ids below hub_lim and
    // need no encoded domain (their frontier bits are already the first hub_lim/64 words of the bitmap)
    uint32_t hub_lim = 0;
    // every id >= leaf_lo has at most one adjacency entry (on a relabelled graph the degree-1 tail): a
    // discovered leaf's only neighbour is its parent, so a push level after a pull level leaves the
    // leaves of its bitmap frontier out of its queue (option leaf_skip)
    int64_t leaf_lo = 0;
    // every id >= hub_row_lim has at most hub_deg adjacency entries (the id of the last row with more, + 1;
    // on a relabelled graph a short prefix): a pull level that found no vertex below it hands the next
    // push level a frontier without hubs (no hub bin, K3p-eligible).  Recomputed when hub_degree changes.
    int64_t hub_row_lim = -1;
    uint32_t hub_row_deg = 0;
    uint32_t *colh = nullptr;           // [nnz] col with hub entries encoded kHubBit | h
    u64 *hfront = nullptr;              // [ceil(hub_k/64)] frontier bits of the hubs
    uint32_t *qa = nullptr, *qb = nullptr, *hubs = nullptr;
    // result staging of bfsx_bfs / bfsx_result (one word per original id: parent << 32 | dist, or int32 dist
    // only): its own buffer, allocated at the first copy -- never the frontier queues, whose stale words must
    // not be result data and whose result data must not be frontier ids -- and two pinned host chunks the D2H
    // copy streams through while host threads split them into the caller's arrays
    u64 *out64 = nullptr;
    // the unpack's phase-1 words (k_unpack_live: parent_original << 32 | dist per INTERNAL id): the push log's
    // buffer once the log is scattered (single device), else rtmp, allocated at the first copy
    u64 *rtmp = nullptr;
    // every id >= iso_lo names an empty row (1 + the largest non-empty row): on a relabelled graph the isolated
    // tail of the degree order, half the ids of a scale-26 Kronecker graph
    int64_t iso_lo = 0;
    int out_mode = 0;        // out64's fill: 0 none, 1 packed words, 2 int32 distances (isolated ids keep it)
    int64_t out_dirty = -1;  // an isolated vertex whose out64 entry the last unpack overwrote (it was the source)
    u64 *h_stage = nullptr;
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    hipEvent_t ev_unpack0 = nullptr, ev_unpack1 = nullptr, ev_unpack_mid = nullptr;
    double last_unpack_ms = -1.0;       // device time of the most recent unpack (state -> original-id arrays)
    double last_resolve_ms = -1.0;      // its internal-id part: push log + records folded into st (-1: none)
    // mapped pinned word: 0, or 1 << 32 | id of the first out-of-range id a queue consumer met (id_ok)
    u64 *h_err = nullptr, *d_err = nullptr;
    LevelSlot *ring = nullptr;          // device, 3 slots
    LevelSlot *h_slot = nullptr;        // pinned host mirror of one slot
    Published *h_pub = nullptr, *d_pub = nullptr; // mapped pinned level counters (host / device view)
    // K3p (persistent top-down): output segments, workgroup records, barrier state (device) and the
    // launch result (mapped pinned host memory)
    u64 *persist_seg = nullptr;         // K3p segments: 2 parities x G x kRegion entries of 16 B
    u64 *persist_brec = nullptr;
    u64 *persist_hseg = nullptr;        // heavy-row regions: 2 parities x G x kHeavyPer x {row start, v | deg << 32}
    void *persist_ctl = nullptr, *h_pout = nullptr, *d_pout = nullptr;
    int persist_grid = 0;       // workgroups (<= one per CU, all co-resident)
    size_t persist_lds = 0;     // dynamic LDS per workgroup (keeps one workgroup per CU)
    size_t persist_lds_light = 0; // the same for the instantiation without heavy rows
    // the graph has a row longer than persist_dmax (heavy_thr: the persist_dmax that was checked; -1 none)
    bool heavy_rows = true;
    int64_t heavy_thr = -1;
    u64 persist_bar = 0;        // K3p levels run since the records were last zeroed (the record tag base)
    bool persist_reset = true;  // persist_ctl and the records must be zeroed before the next launch
    bool persist_off = false;   // K3p cannot run on this device (occupancy check failed)
    int64_t persist_fallbacks = 0; // BFS runs re-run without K3p after a barrier abort
    double clock_khz = 100000.0; // device wall-clock rate
    u64 pub_seq = 0;
    u64 *d_cursor = nullptr;            // bitmap -> queue compaction cursor
    u64 *d_red = nullptr;               // reductions (m_comp, reached)
    int64_t prev_source = -1;
    // multi-GPU level state (bfsx_dist_*)
    u64 *remote = nullptr;              // unbucketed remote pairs
    int64_t remote_cap = 0;
    u64 *d_dist_ctr = nullptr;          // kCtrWords: [0] remote tail, then count, cursor, recv count, sums
    u64 *h_post = nullptr, *d_post = nullptr; // mapped pinned: [0] sequence, [1..] words posted by k_post
    u64 post_seq = 0;
    u64 *sendbuf = nullptr, *recvbuf = nullptr, *fglob = nullptr; // native exchange buffers
    int64_t send_cap = 0, recv_cap = 0, fglob_words = 0;
    int64_t nnz_global = -1;
    // partitioned: the ORIGINAL ids whose degree exceeds big_thr, sorted, with their degrees (u64 id << 32 |
    // degree), all-gathered once per graph; every other id has degree <= big_thr (see dist_bfs_run)
    std::vector<u64> h_big;
    int64_t big_thr = -1;               // -1: not built; the slot_pairs option the list was built for
    bool big_overflow = false;          // more than big_cap such ids on a rank: source degrees unknown (counted level 0)
    int d_level = 0, d_dir = BFSX_DIR_TOPDOWN;
    bool d_in_queue = true;
    int64_t d_nf = 0, d_mf = 0;
    hipEvent_t ev_start = nullptr, ev_end = nullptr;
    std::vector<hipEvent_t> ev_begin, ev_level; // per level: before / after its kernels
    // Device buffers replaced while the partitioned loop runs (grown exchange buffers, the degree-list
    // temporaries): freed with the workspace, never in the middle of the loop.  The ranks of an in-process
    // group share one device, and a hipFree issued by one rank while the others' kernels ran coincided with
    // device memory faults in those kernels ("Wrong-result events", event (b)).
    struct Retired {
        const void *p;
        size_t bytes;
    };
    std::vector<Retired> retired;
    // option comm_timing: event pairs around the level loop's collectives of the last partitioned BFS, their kind
    // (CommOp - 1) and the per-kind sums bfsx_comm_times reads
    std::vector<hipEvent_t> ev_comm;
    std::vector<int> comm_kind;
    int n_comm = 0;
    double comm_ms[4] = {0, 0, 0, 0};
    int64_t comm_n[4] = {0, 0, 0, 0};
};

// Debug aid (environment BFSX_SYNC_LAUNCH=1): synchronise the stream after every launch, so an asynchronous
// device fault surfaces at the launch that caused it (BFSX_HIP_TRY's message names the source line), while the
// other streams -- the other ranks of an in-process group -- keep running concurrently.
inline bool sync_launch() {
    static const bool on = std::getenv("BFSX_SYNC_LAUNCH") != nullptr;
    return on;
}
#define BFSX_LAUNCHED(stream)                                                                                   \
    do {                                                                                                        \
        BFSX_HIP_TRY(hipGetLastError());                                                                        \
        if (::bfsx::sync_launch()) BFSX_HIP_TRY(hipStreamSynchronize(stream));                                  \
    } while (0)

__device__ inline unsigned lane_id() { return threadIdx.x & 63u; }

__device__ inline uint32_t wave_incl_scan(uint32_t x) {
    const unsigned lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= (unsigned)d) x += y;
    }
    return x;
}

__device__ inline u64 wave_sum(u64 x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    return x;
}

__device__ inline void zero_slot(LevelSlot *ring, int level) {
    if (blockIdx.x == 0) {
        u64 *p = reinterpret_cast<u64 *>(ring + (level + 2) % 3);
        for (int i = threadIdx.x; i < kSlotWords; i += kBS) p[i] = 0ull;
    }
}

// Block-uniform: reduce the per-thread stat values over the workgroup; threads 0..6 add them to this
// workgroup's shard of the level's counters.  Order: nf, mf, scanned, claims, mu, stage2, walked.
__device__ inline u64 wave_max(u64 x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const u64 y = __shfl_xor(x, d);
        x = y > x ? y : x;
    }
    return x;
}
__device__ inline uint32_t wave_max32(uint32_t x) { // one lane exchange per step where u64 takes two
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t y = __shfl_xor(x, d);
        x = y > x ? y : x;
    }
    return x;
}

__device__ inline void shard_add(LevelSlot *slot, u64 nf, u64 mf, u64 scanned, u64 claims, u64 mu, u64 dmax = 0,
                                 u64 stage2 = 0, u64 walked = 0, u64 nhub = 0, u64 expl = 0) {
    __shared__ u64 s_red[kStatFields][kWaves];
    __shared__ u64 s_dmax[kWaves];
    dmax = wave_max(dmax);
    if (lane_id() == 0) s_dmax[threadIdx.x >> 6] = dmax;
    u64 v[kStatFields] = {nf, mf, scanned, claims, mu, stage2, walked, nhub, expl};
    const unsigned wave = threadIdx.x >> 6;
#pragma unroll
    for (int f = 0; f < kStatFields; f++) {
        v[f] = wave_sum(v[f]);
        if (lane_id() == 0) s_red[f][wave] = v[f];
    }
    __syncthreads();
    if (threadIdx.x < kStatFields) {
        u64 t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) t += s_red[threadIdx.x][w];
        if (t) atomicAdd(reinterpret_cast<u64 *>(&slot->sh[blockIdx.x % kShards]) + threadIdx.x, t);
    } else if (threadIdx.x == kStatFields) {
        u64 t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) t = s_dmax[w] > t ? s_dmax[w] : t;
        if (t) atomicMax(&slot->sh[blockIdx.x % kShards].dmax, t);
    }
}

// ---- level counters -> host: the sums of the level's stat shards are published into mapped pinned host
// memory with a sequence number the host spins on (a D2H copy + stream synchronise costs ~15 us per
// level on MI355X).  The LAST workgroup of the level's last kernel publishes (a separate one-wave kernel cost ~6-9 us
// per level: its dependent-dispatch gap plus the kernel).  Every workgroup fences its
// shard / queue atomics and arrives on the slot's `done` counter; the one that arrives last reads the
// shards back with device-scope loads (they were updated by device-scope atomics, which bypass the XCD
// L2s) and writes the record to mapped host memory.  Block-uniform; pub == null: no-op.
__device__ inline void publish_if_last(LevelSlot *slot, Published *pub, u64 seq) {
    if (!pub) return;
    __shared__ int s_last;
    // hand-off without fences (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1
    // table): every wave drains its own shard / queue atomics (device-scope atomics are performed at the
    // memory side), a barrier, then ONE agent-scope add per workgroup whose returned value names the
    // last arriver, which reads the shards back with sc1 loads.  A __threadfence() here writes back the
    // XCD's L2 in every workgroup (buffer_wbl2): it doubled the BFS time.
    // The arrivals are sharded (blockIdx % 8, one line each; the last of a shard adds to `done`): ~1,500
    // workgroups on one counter queue ~12 ns each at the memory side, which a tail of simultaneous
    // finishers would pay in full.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned G = gridDim.x, sh = blockIdx.x % kDoneShards;
        const u64 n_sh = (G - sh + kDoneShards - 1) / kDoneShards; // workgroups of this shard
        int last = __hip_atomic_fetch_add(&slot->dsh[sh].n, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   n_sh - 1ull;
        if (last)
            last = __hip_atomic_fetch_add(&slot->done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (u64)min(G, (unsigned)kDoneShards) - 1ull;
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x < 64) {
        const unsigned lane = threadIdx.x;
        const u64 *sh = reinterpret_cast<const u64 *>(&slot->sh[lane]);
        auto ld = [](const u64 *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        const u64 nf = wave_sum(ld(sh + 0)), mf = wave_sum(ld(sh + 1)), sc = wave_sum(ld(sh + 2)),
                  cl = wave_sum(ld(sh + 3)), mu = wave_sum(ld(sh + 4)), s2 = wave_sum(ld(sh + 5)),
                  wk = wave_sum(ld(sh + 6)), nh = wave_sum(ld(sh + 7)), ex = wave_sum(ld(sh + 8)),
                  dmax = wave_max(ld(sh + 9));
        static_assert(offsetof(StatShard, expl) == 8 * sizeof(u64) && offsetof(StatShard, dmax) == 9 * sizeof(u64),
                      "publish_if_last reads the shard fields by position");
        const u64 qt = ld(&slot->qtail);
        if (lane == 0) {
            // mapped host memory (uncached): the record's stores complete before the sequence number's
            volatile Published *vp = pub;
            vp->stage2 = (int64_t)s2;
            vp->walked = (int64_t)wk;
            vp->nhub = (int64_t)nh;
            vp->expl = (int64_t)ex;
            vp->qtail = (int64_t)qt;
            vp->nf = (int64_t)nf;
            vp->mf = (int64_t)mf;
            vp->sc = (int64_t)sc;
            vp->cl = (int64_t)cl;
            vp->mu = (int64_t)mu;
            vp->dmax = (int64_t)dmax;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            vp->seq = seq;
        }
    }
}

// ---- store guards (round 6) ----------------------------------------------------------------------
// Every computed global index of the push / exchange path is checked against its buffer's capacity before the
// store.  A violation is not written: it is reported in the workspace's mapped error words (err[0] = 2 << 32 |
// site, err[1] = index, err[2] = bound) and fails the BFS -- on a partition at the level close, on every rank
// together (level_sums' guard bit) -- instead of becoming a wild store.  One compare per flush or per pair.
enum GuardSite : uint32_t {
    kSiteSlot = 1,     // rq_flush: a pair's position in its destination's fixed exchange slot
    kSiteSlotDest = 2, // rq_flush / bucketing: a pair's destination rank
    kSiteRemote = 3,   // rq_flush: the counted exchange's remote-pair buffer
    kSiteHubs = 4,     // k_td: the hub list
    kSiteQueue = 5,    // q_flush: the next-frontier queue / push-log segment
    kSiteBucket = 6,   // k_bucket_scatter: the send buffer
};
constexpr int kErrWords = 4; // mapped error words: [0] code, [1] index, [2] bound
__device__ inline bool idx_ok(u64 i, u64 bound, u64 *err, uint32_t site) {
    if (i < bound) return true;
    if (err) {
        volatile u64 *e = reinterpret_cast<volatile u64 *>(err);
        e[1] = i;
        e[2] = bound;
        __threadfence_system();
        e[0] = 0x200000000ull | site;
    }
    return false;
}

// ---- block-level output queue ------------------------------------------------------------------
// Winners are appended to an LDS buffer (LDS atomics) and flushed to the global next-frontier queue
// with ONE global atomic per flush (~kQCap winners): a single device counter hit by every wave
// serialises at the memory side (measured 2.4 G edges/s on scale 26 with per-wave appends).
constexpr int kQCap = 4096;

template <int kCapT>
struct BlockQueueT {
    static constexpr uint32_t kCap = kCapT;
    uint32_t buf[kCapT];
    uint32_t n;
    uint32_t gbase;
};
using BlockQueue = BlockQueueT<kQCap>;
// Single-device push kernels: winners are queued with their parent (vertex | parent << 32, same LDS bytes as
// BlockQueue); a flush writes the next frontier's ids and, with a push log, the pairs at the same positions.
template <int kCapT>
struct LogQueueT {
    static constexpr uint32_t kCap = kCapT;
    u64 buf[kCapT];
    uint32_t n;
    uint32_t gbase;
};
using LogQueue = LogQueueT<kQCap / 2>;
// the partitioned push kernels queue (vertex, parent) pairs too, so that their winners go to the push log like one
// device's (round 5); they also hold a remote-pair queue
using DistQueue = LogQueueT<kQCap / 2>;

// All 64 lanes of every wave call this (wave-uniform control flow).
template <class Q>
__device__ inline void bq_push(Q &q, bool win, uint32_t v) {
    const u64 mask = __ballot(win);
    if (mask == 0) return;
    const unsigned lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&q.n, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (win) q.buf[base + __popcll(mask & ((1ull << lane) - 1ull))] = v;
}

// Block-uniform: every thread calls after a __syncthreads().
template <class Q>
__device__ inline void bq_flush(Q &q, uint32_t *__restrict__ qout, u64 *qtail) {
    const uint32_t n = q.n;
    if (n == 0) return;
    if (threadIdx.x == 0) q.gbase = (uint32_t)atomicAdd(qtail, (u64)n);
    __syncthreads();
    const uint32_t gb = q.gbase;
    for (uint32_t i = threadIdx.x; i < n; i += kBS) qout[gb + i] = q.buf[i];
    __syncthreads();
    if (threadIdx.x == 0) q.n = 0;
    __syncthreads();
}

template <class Q>
__device__ inline void bq_init(Q &q) {
    if (threadIdx.x == 0) q.n = 0;
}

// The push kernels' queue calls for either queue type (the id-only queue ignores the parent and the log).
template <int C>
__device__ inline void q_push(BlockQueueT<C> &q, bool win, uint32_t v, uint32_t) {
    bq_push(q, win, v);
}
template <int C>
__device__ inline void q_push(LogQueueT<C> &q, bool win, uint32_t v, uint32_t parent) {
    const u64 mask = __ballot(win);
    if (mask == 0) return;
    const unsigned lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&q.n, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (win) q.buf[base + __popcll(mask & ((1ull << lane) - 1ull))] = (u64)v | ((u64)parent << 32);
}
template <int C>
__device__ inline void q_flush(BlockQueueT<C> &q, uint32_t *__restrict__ qout, u64 *, u64 *qtail, u64 = ~0ull,
                               u64 * = nullptr) {
    bq_flush(q, qout, qtail);
}
// qcap / err: the entries the output queue (and the push-log segment) hold; a flush that would pass them is
// reported (kSiteQueue) and dropped instead of written
template <int C>
__device__ inline void q_flush(LogQueueT<C> &q, uint32_t *__restrict__ qout, u64 *__restrict__ plog, u64 *qtail,
                               u64 qcap = ~0ull, u64 *err = nullptr) {
    const uint32_t n = q.n;
    if (n == 0) return;
    if (threadIdx.x == 0) q.gbase = (uint32_t)atomicAdd(qtail, (u64)n);
    __syncthreads();
    const uint32_t gb = q.gbase;
    if (lane_id() == 0) (void)idx_ok((u64)gb + n - 1u, qcap, err, kSiteQueue); // every wave checks what it stores
    for (uint32_t i = threadIdx.x; i < n && (u64)gb + n <= qcap; i += kBS) {
        const u64 e = q.buf[i];
        qout[gb + i] = (uint32_t)e;
        if (plog) plog[gb + i] = e;
    }
    __syncthreads();
    if (threadIdx.x == 0) q.n = 0;
    __syncthreads();
}

// ---- K3: top-down push, degree-binned -----------------------------------------------------------
// Two bins, chosen per frontier vertex by degree:
//   k_td       vertex groups: a workgroup takes 256 frontier vertices of degree <= hub_deg, scans
//              their degrees in LDS and sweeps the union of their rows edge-parallel (a thread finds
//              its row by binary search in the LDS scan), kItems edges per thread per step so that
//              several independent loads are in flight.
//   k_td_hubs  multi-workgroup bin: vertices of degree > hub_deg are appended to a hub list; every
//              workgroup loads a batch of hubs into LDS, scans their degrees and sweeps an equal
//              share of the batch's edges, so a single huge row or thousands of medium rows are
//              spread evenly over the whole grid.
constexpr int kItems = 4;
constexpr int kHubBatch = 1024;

__device__ inline bool claim(uint32_t v, u64 *vis, u64 &attempts) {
    const u64 bit = 1ull << (v & 63u);
    u64 *w = vis + (v >> 6);
    if (*w & bit) return false; // bits are only ever set: a stale line can only under-report
    attempts++;
    return !(atomicOr(w, bit) & bit);
}

// The hub set of the hybrid levels (bfs_run): on a relabelled graph (ids in degree order) the ids below
// `lim`, otherwise the vertices of degree >= `tdeg` (the encoded pull domain's members).  Off: {~0, 0}.
struct HubSet {
    uint32_t tdeg;
    uint32_t lim;
};
__device__ inline bool is_hub(const HubSet &h, uint32_t v, u64 deg) { return v < h.lim || deg >= (u64)h.tdeg; }

// 1-D partition of the vertex ids (multi-GPU path): this rank owns global ids [lo, lo+chunk) and
// stores their rows; adjacency entries stay global.  Single-GPU graphs use lo = 0, one rank.
struct Part {
    uint32_t lo;     // first owned global id
    uint32_t chunk;  // ids per rank (multiple of 64)
    uint32_t rank;
    uint32_t nrows;  // rows held here: every queued id must be below it (id_ok)
    u64 *remote;      // (v << 32 | parent) pairs for vertices owned elsewhere
    u64 *remote_tail; // their allocation cursor
    u64 remote_cap;   // entries `remote` holds (kSiteRemote)
    u64 qcap;         // entries the push kernels' next-frontier queue and push-log segment hold (kSiteQueue)
    u64 *err;         // mapped host word: set when a queue holds an id >= nrows (null: unchecked)
    uint32_t nranks;
    uint32_t probe;   // diagnostic build, option race_probe: 1 delay, 2 delay + no queue-init barrier (k_td)
    // small partitioned push levels (fixed-slot exchange): remote pairs go straight into the send buffer's
    // per-destination slots [count, slot_cap pairs] (slot_cap 0: into `remote` for the counted exchange);
    // the level's last push kernel has slot_arrive set: its last workgroup writes the slot counts
    u64 *slot_out;
    u64 slot_cap;
    u64 *slot_cursor;
    u64 *slot_arrive;
};

// Queue-entry guard.  Every kernel that reads vertex ids out of a frontier queue, the hub list or an
// exchange buffer checks them against the rows it holds before using them as an index: a stale or
// poisoned entry (a consumer reading past a queue's tail) is reported to the host (bfs_run fails with
// BFSX_E_HIP) and skipped, instead of becoming a wild row_off / col / state access.  One compare per
// frontier vertex; the store happens only on a bad id.
__device__ inline bool id_ok(uint32_t u, uint32_t nrows, u64 *err) {
    if (u < nrows) return true;
    if (err) *reinterpret_cast<volatile u64 *>(err) = 0x100000000ull | u;
    return false;
}

// Remote pairs, LDS-buffered like the local queue (multi-GPU path only).
constexpr int kRCap = 1024;
constexpr int kMaxRanks = 64;
struct RemoteQueue {
    u64 buf[kRCap];
    u64 gbase; // 64-bit: a forced top-down level at scale 30 can route more than 2^32 pairs
    uint32_t n;
    uint32_t h[kMaxRanks]; // slot mode: this flush's pairs per destination, then their slot bases
    u64 base[kMaxRanks];
};

__device__ inline void rq_push(RemoteQueue &q, bool send, u64 pair) {
    const u64 mask = __ballot(send);
    if (mask == 0) return;
    const unsigned lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&q.n, (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (send) q.buf[base + __popcll(mask & ((1ull << lane) - 1ull))] = pair;
}

__device__ inline void rq_flush(RemoteQueue &q, const Part &pt) {
    const uint32_t n = q.n;
    if (n == 0) return;
    if (pt.slot_cap) {
        // fixed-slot exchange: an LDS histogram by destination, ONE reservation atomic per (workgroup,
        // destination) on the slot cursors, then every pair to its slot (no separate bucketing pass)
        constexpr int kPer = kRCap / kBS;
        for (int d = threadIdx.x; d < kMaxRanks; d += kBS) q.h[d] = 0u;
        __syncthreads();
        uint32_t r[kPer], dst[kPer]; // dst = kMaxRanks: no slot (past the queue, or a guarded destination)
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + (uint32_t)k * kBS;
            const uint32_t d = i < n ? (uint32_t)(q.buf[i] >> 32) / pt.chunk : 0u;
            dst[k] = (i < n && idx_ok(d, pt.nranks, pt.err, kSiteSlotDest)) ? d : (uint32_t)kMaxRanks;
            r[k] = dst[k] < (uint32_t)kMaxRanks ? atomicAdd(&q.h[dst[k]], 1u) : 0u;
        }
        __syncthreads();
        for (int d = threadIdx.x; d < kMaxRanks; d += kBS)
            if (q.h[d]) q.base[d] = atomicAdd(&pt.slot_cursor[d], (u64)q.h[d]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + (uint32_t)k * kBS;
            // the slot bound is the host's per-peer bound on this level's pairs (the global m_f, kernels_dist.hip)
            if (dst[k] < (uint32_t)kMaxRanks && idx_ok(q.base[dst[k]] + r[k], pt.slot_cap, pt.err, kSiteSlot))
                pt.slot_out[(u64)dst[k] * (pt.slot_cap + 1) + 1 + q.base[dst[k]] + r[k]] = q.buf[i];
        }
        __syncthreads();
        if (threadIdx.x == 0) q.n = 0;
        __syncthreads();
        return;
    }
    if (threadIdx.x == 0) q.gbase = atomicAdd(pt.remote_tail, (u64)n);
    __syncthreads();
    const u64 gb = q.gbase;
    // the remote buffer holds the local frontier's m_f pairs (the host's bound, kernels_dist.hip)
    if (lane_id() == 0) (void)idx_ok(gb + n - 1u, pt.remote_cap, pt.err, kSiteRemote);
    for (uint32_t i = threadIdx.x; i < n && gb + n <= pt.remote_cap; i += kBS) pt.remote[gb + i] = q.buf[i];
    __syncthreads();
    if (threadIdx.x == 0) q.n = 0;
    __syncthreads();
}

// Slot mode, the level's last push kernel: the last workgroup to arrive writes every destination's pair
// count into its slot header (the cursors are device-scope atomics whose values have all returned:
// fence-free hand-off as in publish_if_last).  Block-uniform.
__device__ inline void slot_headers_if_last(const Part &pt) {
    if (!pt.slot_arrive) return;
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(pt.slot_arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1ull;
    __syncthreads();
    if (!s_last) return;
    for (uint32_t p = threadIdx.x; p < pt.nranks; p += kBS)
        pt.slot_out[(u64)p * (pt.slot_cap + 1)] =
            __hip_atomic_load(&pt.slot_cursor[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Multi-GPU level close (k_level_sums below, or the last workgroup of k_claim_remote): the level's counter
// shards summed into out[0..6] = local {n_f, m_f, m_u, scanned, rows/claims, stage2, walked}, out[8..10] = copy
// of {n_f, m_f, m_u} (all-reduced in place), and the next level's exchange counters `ctr` zeroed.
//   out[7] = local d_max of the produced frontier (top-down) or local vertices found below hub_row_lim
//   (bottom-up): either tells the next push level whether it needs the hub bin.
//   out[11 + r], r < nranks: this rank's n_f in its own slot, 0 elsewhere -- all-reduced with out[8..10], every
//   rank learns every rank's frontier size (the sparse frontier exchange's receive counts).
//   out[11 + nranks]: bit `rank` set when this rank's queue guard (id_ok, `err`) has fired -- all-reduced too, so
//   every rank leaves the loop at the same level with the same error instead of the failing rank alone (the
//   guard used to be read only after the loop, between the last level close and the m_comp all-reduce: a
//   rank-local early return that left its peers inside that all-reduce, DESIGN.md 4, event (c)).
// One wave (threads 0..63) of the calling workgroup; the shards are read with agent-scope loads, so a
// last-arriving workgroup of the level's last kernel can run it (k_claim_remote) as well as k_level_sums.
__device__ inline void level_sums(const LevelSlot *__restrict__ slot, int topdown, int64_t *__restrict__ out,
                                  u64 *__restrict__ ctr, int nctr, int rank, int nranks, const u64 *err) {
    if (threadIdx.x >= 64) return;
    const unsigned lane = threadIdx.x;
    auto ld = [](const u64 *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // top-down: the pairs this rank shipped = the sum of the per-destination cursors (slot or counted
    // exchange), read before the counters are zeroed; recorded as the level's `walked`
    const u64 shipped = (topdown && nctr >= 1 + 2 * kMaxRanks) ? wave_sum(ld(ctr + 1 + kMaxRanks + lane)) : 0ull;
    for (int i = lane; i < nctr; i += 64) ctr[i] = 0ull;
    const StatShard &sh = slot->sh[lane];
    u64 t[7] = {wave_sum(ld(&sh.nf)),      wave_sum(ld(&sh.mf)),     wave_sum(ld(&sh.mu)),
                wave_sum(ld(&sh.scanned)), wave_sum(ld(&sh.claims)), wave_sum(ld(&sh.stage2)),
                wave_sum(ld(&sh.walked))};
    const u64 dmax = wave_max(ld(&sh.dmax)), nhub = wave_sum(ld(&sh.nhub));
    if (topdown) {
        t[0] = ld(&slot->qtail);
        t[6] = shipped;
    }
    if (lane == 0) {
        for (int i = 0; i < 7; i++) out[i] = (int64_t)t[i];
        for (int i = 0; i < 3; i++) out[8 + i] = (int64_t)t[i];
        out[7] = (int64_t)(topdown ? dmax : nhub);
        for (int r = 0; r < nranks; r++) out[11 + r] = r == rank ? (int64_t)t[0] : 0;
        const u64 e = err ? __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
        out[11 + nranks] = e ? (int64_t)(1ull << rank) : 0; // distinct bits: the all-reduced sum is their OR
    }
}
// multi-GPU counter block: [0] remote tail | count[64] | cursor[64] | arrivals | recv count[64] | level sums[16 + 64]
constexpr int kCtrHead = 2 + 2 * kMaxRanks; // zeroed per level (the last word: k_claim_remote's arrivals)
constexpr int kCtrRecv = kCtrHead;
constexpr int kCtrSums = kCtrHead + kMaxRanks;
// level sums: [0..10] as level_sums writes them, [11, 11 + P) per-rank n_f, [11 + P] the ranks whose queue guard fired
constexpr int kCtrSums16 = 16 + kMaxRanks;
constexpr int kCtrWords = kCtrSums + kCtrSums16;
constexpr int kPostWords = 1 + 2 * kMaxRanks + 16; // mapped host words of k_post: sequence + posted values
static_assert(12 + kMaxRanks <= kCtrSums16, "level sums overrun their block");
static_assert(12 + kMaxRanks <= kPostWords - 1, "a level close posts 12 + P words");
static_assert(2 * kMaxRanks <= kPostWords - 1, "a count exchange posts 2P words");

// top1 flag and hub-domain encoding of the pull kernels (kernels_pull.hip, the workspace set-up)
constexpr uint32_t kDeg1 = 0x80000000u;
constexpr uint32_t kHubBit = 0x40000000u; // hub encoding needs every global id < 2^30
constexpr uint32_t kHubMask = kHubBit - 1u;

struct SlotSums {
    int64_t nf = 0, mf = 0, sc = 0, cl = 0, mu = 0, s2 = 0, wk = 0, nh = 0, ex = 0;
};

// ---- host entry points of the kernel families (definitions in the .hip file named) ----------------
// kernels_level.hip
unsigned clamp_grid(int64_t blocks, unsigned cap);
int hub_setup(bfsx_graph *g, BfsWorkspace *ws);
int ws_alloc(bfsx_graph *g);
Part single_part(const bfsx_graph *g, const BfsWorkspace *ws);
int check_queue_guard(BfsWorkspace *ws);
int ensure_hub_row_lim(bfsx_graph *g, BfsWorkspace *ws);
int wait_published(BfsWorkspace *ws, hipStream_t st);
SlotSums sum_slot(const LevelSlot *s);
int64_t bu_floor(const bfsx_graph *g, const BfsWorkspace *ws);
int apply_logs(bfsx_graph *g, BfsWorkspace *ws, hipEvent_t ev = nullptr);
// kernels_push.hip: one top-down level (k_td, plus k_td_hubs for the frontier rows above hub_degree)
inline HubSet hub_set(const BfsWorkspace *ws) { return HubSet{ws->hub_k > 0 ? ws->hub_tdeg : 0xFFFFFFFFu, ws->hub_lim}; }
inline bool has_hubs(const BfsWorkspace *ws) { return ws->hub_k > 0 || ws->hub_lim > 0; }
template <bool kDist>
int launch_td(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t mf, int64_t dmax, int level, const Part &pt,
              bool skip_hubs = false, Published *pub = nullptr, u64 seq = 0, uint32_t *par = nullptr,
              u64 *plog = nullptr);
// kernels_pull.hip: one bottom-up level; the hub sweep of a hybrid level; the sparse pull of the tail levels
template <bool kMf>
int launch_bu(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level,
              Published *pub = nullptr, u64 seq = 0);
int launch_bu_hubonly(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level);
int launch_bu_sparse(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level,
                     uint32_t qlim, Published *pub, u64 seq);
// kernels_persist.hip: K3p
int ensure_heavy_rows(bfsx_graph *g, BfsWorkspace *ws);
int persist_blocks(const bfsx_ctx *ctx);
int persist_setup(bfsx_graph *g, BfsWorkspace *ws);
bool persist_fits(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t dmax, bool heavy_src = false);
int persist_td(bfsx_graph *g, BfsWorkspace *ws, int level, int64_t nf, int64_t mu, u64 *front, uint32_t h0_v = 0,
               uint32_t h0_deg = 0, int64_t h0_beg = 0);
constexpr int kPersistAborted = -1000; // internal: K3p aborted (barrier timeout); bfs_run retries without it
// kernels_dist.hip
int post_wait(BfsWorkspace *ws, hipStream_t st, const u64 *a, int na, const u64 *b, int nb, u64 *out,
              Comm *cm = nullptr, const char *what = "a level close");

// ---- pull-level records (single device, BfsWorkspace::par) ----------------------------------------
// At most kMaxRec records per BFS; a BFS with more pull levels folds its records into st mid-BFS (k_resolve).
constexpr int kMaxRec = 32;
struct RecSet {
    const u64 *bm[kMaxRec];
    int32_t nd[kMaxRec]; // distance of the record's vertices (its level + 1)
    int n;
};

// How a pull level found a vertex's parent (round 5; BfsWorkspace::pcode, one byte per vertex): the parent is
// the vertex's first row entry (top1), its 2nd / 3rd / 4th (rest .x / .y / .z) -- the entries the pull kernel
// probed first, which top1 / rest already hold -- or the explicit 4-B parent in par (a row walk, the push half of
// a hybrid level, the encoded hub domain).  A discovery thus writes one byte where it wrote a 4-B parent; the
// result's resolution reads the parent back from top1 / rest (or, in original ids, from otop1 / orest).
constexpr uint8_t kCodeTop1 = 0, kCodeExplicit = 4;
struct ParSrc {
    const uint32_t *par;   // explicit parents
    const uint8_t *code;   // provenance codes
    const uint32_t *top1;  // first row entry (flag bits in fmask)
    const uint4 *rest;     // 2nd..4th row entries (+ degree)
    uint32_t fmask;
};
inline ParSrc par_src(const BfsWorkspace *ws) { return ParSrc{ws->par, ws->pcode, ws->top1, ws->rest, ws->top1_flag}; }
__device__ __forceinline__ uint32_t record_parent(const ParSrc &ps, int64_t v) {
    if (!ps.code) return ps.par[v]; // a partition's pull levels store every parent explicitly
    const uint8_t c = ps.code[v];
    if (c == kCodeTop1) return ps.top1[v] & ~ps.fmask;
    if (c < kCodeExplicit) {
        const uint4 r = ps.rest[v];
        return c == 1 ? r.x : c == 2 ? r.y : r.z;
    }
    return ps.par[v];
}

// state of internal vertex i: st[i], unless a record holds i (its parent is then recorded by ps).  Lanes of
// consecutive i share their record words (one broadcast load per wave and record).
__device__ __forceinline__ u64 rec_state(const u64 *__restrict__ stt, const ParSrc &ps, const RecSet &rs, int64_t i) {
    for (int r = 0; r < rs.n; r++)
        if ((rs.bm[r][i >> 6] >> (i & 63)) & 1ull) return pack_state(record_parent(ps, i), rs.nd[r]);
    return stt[i];
}

// ---- kernels more than one level loop launches (internal linkage: one copy per translation unit; a unit that
// launches none of them drops its copies) ----
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace {

// ---- K2: BFS init: visited bitmap <- dead mask (+ the source bit), source state, counter slots ------
// s: local row of the source (0xFFFFFFFF: the source is owned by another rank); sglob: its global id.
__global__ __launch_bounds__(kBS) void k_init(uint32_t s, uint32_t sglob, int64_t prev, const u64 *__restrict__ dead,
                                              int64_t nwords, u64 *stt, u64 *__restrict__ vis, uint32_t *q,
                                              LevelSlot *ring) {
    const int64_t sw = s != 0xFFFFFFFFu ? (int64_t)(s >> 6) : -1;
    for (int64_t w = (int64_t)blockIdx.x * kBS + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBS)
        vis[w] = dead[w] | (w == sw ? 1ull << (s & 63u) : 0ull);
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        // a previous isolated source is pre-visited (dead mask) so k_finalize never resets it
        if (prev >= 0 && ((dead[prev >> 6] >> (prev & 63)) & 1ull)) stt[prev] = kUnreached;
        if (s != 0xFFFFFFFFu) {
            stt[s] = pack_state(sglob, 0);
            q[0] = s;
        }
    }
    zero_slot(ring, -2); // slot 0
    zero_slot(ring, -1); // slot 1
}

// ---- K4: frontier representation changes -------------------------------------------------------
__global__ __launch_bounds__(kBS) void k_queue_to_bitmap(const uint32_t *__restrict__ q, uint32_t qlen, u64 *bm,
                                                         uint32_t nrows, u64 *err) {
    for (uint32_t i = blockIdx.x * kBS + threadIdx.x; i < qlen; i += gridDim.x * kBS) {
        const uint32_t v = q[i];
        if (id_ok(v, nrows, err)) atomicOr(bm + (v >> 6), 1ull << (v & 63u));
    }
}

// The same with the queue length read on the device (the top-down half of a hybrid level appends to
// the queue; its length is known to the host only after the level is published).
// Publishes the level (hybrid levels end with it).
__global__ __launch_bounds__(kBS) void k_queue_to_bitmap_dev(const uint32_t *__restrict__ q, LevelSlot *cn, u64 *bm,
                                                             Published *pub, u64 seq, uint32_t nrows, u64 *err) {
    const uint32_t n = (uint32_t)cn->qtail;
    for (uint32_t i = blockIdx.x * kBS + threadIdx.x; i < n; i += gridDim.x * kBS) {
        const uint32_t v = q[i];
        if (id_ok(v, nrows, err)) atomicOr(bm + (v >> 6), 1ull << (v & 63u));
    }
    publish_if_last(cn, pub, seq);
}

// Ballot/popcount compaction of a bitmap into a queue.  A workgroup owns a contiguous range of words
// (kCompactWords per thread, coalesced), counts its set bits, scans the per-thread counts in LDS and
// reserves its output range with ONE atomic; the grid is kept small (<= 256 workgroups) so the
// reservation counter sees a few hundred arrivals, not one per wave.
constexpr int kCompactWords = 16;

// lim: ids >= lim are left out (the leaves of leaf_skip); nwords covers them at most by one word.
__global__ __launch_bounds__(kBS) void k_bitmap_to_queue(const u64 *__restrict__ bm, int64_t nwords,
                                                         int64_t words_per_block, uint32_t *__restrict__ q,
                                                         u64 *cursor, int64_t lim) {
    __shared__ uint32_t s_wsum[kWaves];
    __shared__ uint32_t s_base;
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const int64_t wb = (int64_t)blockIdx.x * words_per_block;
    const int64_t we = min(nwords, wb + words_per_block);
    for (int64_t w0 = wb; w0 < we; w0 += (int64_t)kBS * kCompactWords) {
        u64 x[kCompactWords];
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < kCompactWords; i++) {
            const int64_t w = w0 + (int64_t)i * kBS + tid;
            x[i] = w < we ? bm[w] : 0ull;
            if (w * 64 + 64 > lim) x[i] &= w * 64 >= lim ? 0ull : (1ull << (lim - w * 64)) - 1ull;
            c += (uint32_t)__popcll(x[i]);
        }
        const uint32_t inc = wave_incl_scan(c);
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        uint32_t woff = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            woff += (w < (int)wave) ? s_wsum[w] : 0u;
            total += s_wsum[w];
        }
        if (tid == 0) s_base = total ? (uint32_t)atomicAdd(cursor, (u64)total) : 0u;
        __syncthreads();
        uint32_t p = s_base + woff + inc - c;
#pragma unroll
        for (int i = 0; i < kCompactWords; i++) {
            u64 y = x[i];
            const int64_t w = w0 + (int64_t)i * kBS + tid;
            while (y) {
                const int b = __ffsll((long long)y) - 1;
                q[p++] = (uint32_t)(w * 64 + b);
                y &= y - 1ull;
            }
        }
        __syncthreads();
    }
}

// After the last level: vertices left unvisited in this BFS (and not isolated) become WHITE again
// (INT32_MAX, no parent), so the per-BFS init never rewrites the whole state array (isolated vertices
// keep the value written once when the workspace is created).
__global__ __launch_bounds__(kBS) void k_finalize(const u64 *__restrict__ vis, int64_t nwords, u64 *__restrict__ stt) {
    for (int64_t w = (int64_t)blockIdx.x * kBS + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBS) {
        u64 u = ~vis[w];
        while (u) {
            const int b = __ffsll((long long)u) - 1;
            stt[w * 64 + b] = kUnreached;
            u &= u - 1ull;
        }
    }
}

__global__ __launch_bounds__(kBS) void k_fill64(u64 *__restrict__ p, int64_t n, u64 val) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) p[i] = val;
}

// *out = 1 + the largest row id with more than `thr` adjacency entries (0: none).  thr = 1: leaf_lo;
// thr = hub_degree: hub_row_lim, below which every row of more than hub_degree entries lies
__global__ __launch_bounds__(kBS) void k_rows_above(const int64_t *__restrict__ row_off, int64_t nv, int64_t thr,
                                                    u64 *out) {
    u64 m = 0;
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS)
        if (row_off[v + 1] - row_off[v] > thr) m = (u64)v + 1;
    for (int d = 32; d >= 1; d >>= 1) {
        const u64 o = __shfl_xor(m, d);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63u) == 0 && m) atomicMax(out, m);
}

// Degrees of this rank's rows as uint32, padded with 0 to `chunk` entries (the all-gather slice); with
// `perm` (a relabelled partition's slice of the permutation) in ORIGINAL id order.
__global__ __launch_bounds__(kBS) void k_slice_degrees(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ perm,
                                                       int64_t nv, int64_t chunk, uint32_t *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < chunk; v += (int64_t)gridDim.x * kBS) {
        const int64_t r = (perm && v < nv) ? (int64_t)perm[v] : v;
        out[v] = v < nv ? (uint32_t)(row_off[r + 1] - row_off[r]) : 0u;
    }
}
} // namespace

namespace {

// The push log into st (apply_logs): entry i of the log belongs to the first segment s with end[s] > i and
// gets distance nd[s] (meta = end[0..nseg) then nd[0..nseg)).  Outside the timed region.
__global__ __launch_bounds__(kBS) void k_resolve_log(const u64 *__restrict__ plog, int64_t n,
                                                     const int64_t *__restrict__ meta, int nseg, u64 *__restrict__ stt) {
    const int64_t *end = meta, *nd = meta + nseg;
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        int lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (end[mid] > i) hi = mid;
            else lo = mid + 1;
        }
        const u64 e = plog[i];
        stt[(uint32_t)e] = pack_state((uint32_t)(e >> 32), (int32_t)nd[lo]);
    }
}

// st[v] = (par[v], nd_r) for every vertex v of every record r (the validator's and m_comp's view of a result;
// a BFS with more than kMaxRec pull levels).  One wave per bitmap word, lane = bit: a word's par loads and state
// stores are one coalesced access each.
__global__ __launch_bounds__(kBS) void k_resolve(RecSet rs, int64_t nwords, ParSrc ps, u64 *__restrict__ stt) {
    const unsigned lane = lane_id();
    const int64_t nwaves = ((int64_t)gridDim.x * kBS) >> 6;
    for (int64_t w = ((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6; w < nwords; w += nwaves) {
        for (int r = 0; r < rs.n; r++) {
            const u64 m = rs.bm[r][w];
            if (m == 0ull) continue; // wave-uniform
            if ((m >> lane) & 1ull) {
                const int64_t v = w * 64 + lane;
                stt[v] = pack_state(record_parent(ps, v), rs.nd[r]);
            }
        }
    }
}


} // namespace
#pragma clang diagnostic pop

// The pull-level records of one BFS (BfsWorkspace::par): every pull level writes its discoveries into a fresh
// bitmap of the pool; a BFS with more than kMaxRec pull levels folds them into st (k_resolve) and starts over.
struct RecLog {
    bfsx_graph *g;
    BfsWorkspace *ws;
    int n = 0;
    int32_t nd[kMaxRec];
    RecLog(bfsx_graph *g_, BfsWorkspace *ws_) : g(g_), ws(ws_) {
        ws->n_prec = 0;
        ws->resolved = true;
    }
    RecSet set() const {
        RecSet rs{};
        rs.n = n;
        for (int r = 0; r < n; r++) {
            rs.bm[r] = ws->prec[r];
            rs.nd[r] = nd[r];
        }
        return rs;
    }
    // the record the next pull level writes (the frontier it reads, a former record, is never the one returned)
    int take(u64 **out) {
        hipStream_t st = g->ctx->stream;
        if (n == kMaxRec) {
            hipLaunchKernelGGL(k_resolve, dim3(clamp_grid((ws->nwords * 64 + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                               set(), ws->nwords, par_src(ws), ws->st);
            BFSX_LAUNCHED(st);
            n = 0;
        }
        while ((int)ws->prec.size() <= n) {
            u64 *b = nullptr;
            BFSX_HIP_TRY(hipMalloc(&b, ws->nwords * sizeof(u64)));
            ws->prec.push_back(b);
        }
        *out = ws->prec[n];
        return BFSX_OK;
    }
    void done(int32_t dist) { nd[n++] = dist; } // the record just written holds the vertices at distance dist
    void finish() {
        ws->n_prec = n;
        ws->prec_nd.assign(nd, nd + n);
        ws->resolved = n == 0;
    }
};

} // namespace bfsx
