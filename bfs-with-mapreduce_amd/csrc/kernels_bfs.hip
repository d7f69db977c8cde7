// kernels_bfs.hip -- the BFS hot path on the GPU (gfx950, wave64).
//
// Replaces the reference's per-level Spark job (BfsSpark.java:61-118):
//   mapper   (:66-87)  GRAY u emits (n, d+1) for n in N(u)          -> K3 top-down push (k_td, k_td_hubs)
//   reducer  (:90-108) min distance / darkest colour per vertex id  -> fused: atomicOr claim on the
//                      visited bitmap; the single winner writes dist = level+1 (every contender of a
//                      level carries the same level+1, so the min is race-free and exact)
//   collect + contains("GRAY") (:110-117)                            -> K4 frontier count in a sharded
//                      device counter slot, read back as one small D2H per level
//   (no reference analogue)                                          -> K5 bottom-up pull (k_bu) with
//                      Beamer's direction-optimising switch
// State: one packed 64-bit word per vertex, st[v] = parent << 32 | dist (dist INT32_MAX = WHITE, the
// reference's Integer.MAX_VALUE; parent 0xFFFFFFFF = none), so a discovery is ONE 8-byte store instead
// of two scattered 4-byte stores; the visited bitmap u64[n/64] (BLACK|GRAY, pre-set for isolated
// vertices); the frontier as a queue u32[] (top-down) or a bitmap u64[] (bottom-up).
// Row offsets are read as uint32 when the graph's adjacency has < 2^32 entries (half the bytes of the
// int64 CSR offsets on every vertex probe), as int64 otherwise; every traversal kernel is templated on it.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <initializer_list>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "bfsx_internal.h"
#include "exchange_plan.h"

namespace bfsx {

namespace {

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
    u64 dmax;    // top-down: largest degree in the produced frontier (skips the hub bin when <= hub_deg)
};
constexpr int kStatFields = 8; // summed fields, in declaration order (dmax is a max)

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

// A level's counter sums as the host reads them (mapped pinned memory, written by publish_if_last).
struct alignas(64) Published {
    u64 seq;
    int64_t qtail, nf, mf, sc, cl, mu, dmax, stage2, walked, nhub;
};

} // namespace

struct BfsWorkspace {
    int64_t nv = 0, nwords = 0;
    u64 *st = nullptr;                  // packed parent << 32 | dist
    // Pull levels (single device) store only a 4-B parent, par[v]; their discoveries are the level's record
    // bitmap prec[k] (the `next` bitmap k_bu writes anyway, kept per level instead of swapped), which gives
    // them distance prec_lvl[k] + 1.  st[v] of such a vertex is stale until bfs_resolve (or the fused unpack)
    // reads the records -- outside the timed region, like the unpack to original ids.
    uint32_t *par = nullptr;
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
    // the unpack's phase-1 words (k_resolve_all: parent_original << 32 | dist per INTERNAL id): the push log's
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
};

namespace {

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
                                 u64 stage2 = 0, u64 walked = 0, u64 nhub = 0) {
    __shared__ u64 s_red[kStatFields][kWaves];
    __shared__ u64 s_dmax[kWaves];
    dmax = wave_max(dmax);
    if (lane_id() == 0) s_dmax[threadIdx.x >> 6] = dmax;
    u64 v[kStatFields] = {nf, mf, scanned, claims, mu, stage2, walked, nhub};
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
                  wk = wave_sum(ld(sh + 6)), nh = wave_sum(ld(sh + 7)), dmax = wave_max(ld(sh + 8));
        const u64 qt = ld(&slot->qtail);
        if (lane == 0) {
            // mapped host memory (uncached): the record's stores complete before the sequence number's
            volatile Published *vp = pub;
            vp->stage2 = (int64_t)s2;
            vp->walked = (int64_t)wk;
            vp->nhub = (int64_t)nh;
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
// the partitioned push kernels also hold a remote-pair queue: half-size queues keep 4 workgroups per CU
using DistQueue = BlockQueueT<kQCap / 2>;
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
__device__ inline void q_flush(BlockQueueT<C> &q, uint32_t *__restrict__ qout, u64 *, u64 *qtail) {
    bq_flush(q, qout, qtail);
}
template <int C>
__device__ inline void q_flush(LogQueueT<C> &q, uint32_t *__restrict__ qout, u64 *__restrict__ plog, u64 *qtail) {
    const uint32_t n = q.n;
    if (n == 0) return;
    if (threadIdx.x == 0) q.gbase = (uint32_t)atomicAdd(qtail, (u64)n);
    __syncthreads();
    const uint32_t gb = q.gbase;
    for (uint32_t i = threadIdx.x; i < n; i += kBS) {
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
    u64 *err;         // mapped host word: set when a queue holds an id >= nrows (null: unchecked)
    uint32_t nranks;
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
        uint32_t r[kPer], dst[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + (uint32_t)k * kBS;
            dst[k] = i < n ? (uint32_t)(q.buf[i] >> 32) / pt.chunk : 0u;
            r[k] = i < n ? atomicAdd(&q.h[dst[k]], 1u) : 0u;
        }
        __syncthreads();
        for (int d = threadIdx.x; d < kMaxRanks; d += kBS)
            if (q.h[d]) q.base[d] = atomicAdd(&pt.slot_cursor[d], (u64)q.h[d]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t i = threadIdx.x + (uint32_t)k * kBS;
            if (i < n) pt.slot_out[(u64)dst[k] * (pt.slot_cap + 1) + 1 + q.base[dst[k]] + r[k]] = q.buf[i];
        }
        __syncthreads();
        if (threadIdx.x == 0) q.n = 0;
        __syncthreads();
        return;
    }
    if (threadIdx.x == 0) q.gbase = atomicAdd(pt.remote_tail, (u64)n);
    __syncthreads();
    const u64 gb = q.gbase;
    for (uint32_t i = threadIdx.x; i < n; i += kBS) pt.remote[gb + i] = q.buf[i];
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

// Sweep edges [x_begin, x_end) of a segment table (scan/beg/u in LDS, n entries; u = local row id)
// in steps of kBS*kItems.  Block-uniform.  kDist: targets owned by another rank become remote pairs.
// par != null (the push half of a hybrid level): a winner's parent also goes to the 4-B parent array, because the
// level's discoveries are merged into the pull half's level record, whose vertices take their parent from there.
template <bool kDist, class OffT, class ScanT, class Q>
__device__ inline void sweep_segments(const ScanT *s_scan, const int64_t *s_beg, const uint32_t *s_u, int n,
                                      uint64_t x_begin, uint64_t x_end, const OffT *__restrict__ row_off,
                                      const uint32_t *__restrict__ col, u64 *vis, u64 *__restrict__ stt,
                                      uint32_t *__restrict__ par, int32_t nd, Q &q, uint32_t *__restrict__ qout, u64 *qtail,
                                      const Part &pt, RemoteQueue *rq, u64 &acc_mf, u64 &attempts, u64 &acc_dmax,
                                      HubSet hs, u64 &acc_mfh, u64 &acc_nh, u64 *__restrict__ plog) {
    for (uint64_t x0 = x_begin; x0 < x_end; x0 += (uint64_t)kBS * kItems) {
        uint32_t v[kItems], pu[kItems];
        bool valid[kItems];
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            const uint64_t x = x0 + (uint64_t)k * kBS + threadIdx.x;
            valid[k] = x < x_end;
            v[k] = 0;
            pu[k] = 0;
            if (valid[k]) {
                int lo = 0, hi = n - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((uint64_t)s_scan[mid] <= x) lo = mid;
                    else hi = mid - 1;
                }
                v[k] = col[s_beg[lo] + (int64_t)(x - (uint64_t)s_scan[lo])];
                pu[k] = s_u[lo] + pt.lo; // global id of the frontier vertex
            }
        }
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            bool win = false, send = false;
            uint32_t vl = v[k];
            if (kDist) {
                send = valid[k] && (v[k] / pt.chunk) != pt.rank;
                vl = v[k] - pt.lo;
            }
            if (valid[k] && !send && claim(vl, vis, attempts)) {
                win = true;
                // the push log (single device) or the hybrid level's parent array + record carry the result;
                // else the packed state
                if (par) par[vl] = pu[k];
                else if (!plog) stt[vl] = pack_state(pu[k], nd);
                const u64 dg = (u64)(row_off[vl + 1] - row_off[vl]);
                acc_mf += dg;
                acc_dmax = dg > acc_dmax ? dg : acc_dmax;
                if (is_hub(hs, v[k], dg)) { // a hub of the hybrid levels (bfs_run)
                    acc_mfh += dg;
                    acc_nh += 1;
                }
            }
            q_push(q, win, vl, pu[k]);
            if (kDist) rq_push(*rq, send, ((u64)v[k] << 32) | pu[k]);
        }
        __syncthreads();
        if (q.n > Q::kCap - (uint32_t)(kBS * kItems)) q_flush(q, qout, plog, qtail);
        if (kDist && rq->n > (uint32_t)(kRCap - kBS * kItems)) rq_flush(*rq, pt);
    }
}

template <bool kDist, class OffT>
__global__ __launch_bounds__(kBS) void k_td(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const uint32_t *__restrict__ qin, uint32_t qlen,
                                            uint32_t *__restrict__ qout, u64 *vis, u64 *__restrict__ stt,
                                            uint32_t *__restrict__ par, LevelSlot *ring, int level, uint32_t hub_deg,
                                            uint32_t *__restrict__ hubs, Part pt, int gsz, HubSet hs,
                                            HubSet skip, Published *pub, u64 seq, u64 *__restrict__ plog) {
    LevelSlot *cn = ring + (level + 1) % 3;
    zero_slot(ring, level);
    __shared__ uint32_t s_scan[kBS + 1];
    __shared__ int64_t s_beg[kBS];
    __shared__ uint32_t s_u[kBS];
    __shared__ uint32_t s_wsum[kWaves];
    __shared__ typename std::conditional<kDist, DistQueue, LogQueue>::type q;
    __shared__ typename std::conditional<kDist, RemoteQueue, char>::type rq_storage;
    RemoteQueue *rq = kDist ? reinterpret_cast<RemoteQueue *>(&rq_storage) : nullptr;
    bq_init(q);
    if (kDist && threadIdx.x == 0) rq->n = 0;
    const int32_t nd = level + 1;
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    u64 acc_mf = 0, attempts = 0, scanned = 0, acc_dmax = 0, acc_mfh = 0, acc_nh = 0;
    // gsz (<= kBS) frontier vertices per workgroup and step: a narrow frontier spreads over more
    // workgroups, so each sweeps its rows in one step instead of several dependent ones
    for (uint32_t base = blockIdx.x * gsz; base < qlen; base += gridDim.x * gsz) {
        const uint32_t i = base + tid;
        uint32_t deg = 0, u = 0;
        int64_t beg = 0;
        if ((int)tid < gsz && i < qlen && id_ok(qin[i], pt.nrows, pt.err)) {
            u = qin[i];
            beg = (int64_t)row_off[u];
            int64_t d = (int64_t)row_off[u + 1] - beg;
            if (d == 1 && level > 0) {
                // a discovered vertex with one neighbour: that neighbour is the parent it was found
                // from (visited), so its row holds nothing to claim -- the frontier a pull level hands to
                // a push level is mostly such leaves
                d = 0;
            } else if (is_hub(skip, u + pt.lo, (u64)d)) { // hybrid level: the pull hub sweep covers this vertex
                d = 0;
            } else if (d > (int64_t)hub_deg) {
                hubs[atomicAdd(&cn->nhub, 1ull)] = u;
                d = 0;
            }
            deg = (uint32_t)d;
        }
        const uint32_t inc = wave_incl_scan(deg);
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        uint32_t woff = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            const uint32_t t = s_wsum[w];
            woff += (w < (int)wave) ? t : 0u;
            total += t;
        }
        s_scan[tid] = woff + inc - deg;
        s_beg[tid] = beg;
        s_u[tid] = u;
        if (tid == 0) {
            s_scan[kBS] = total;
            scanned += total;
        }
        __syncthreads();
        sweep_segments<kDist>(s_scan, s_beg, s_u, gsz, 0, total, row_off, col, vis, stt, par, nd, q, qout, &cn->qtail, pt, rq,
                              acc_mf, attempts, acc_dmax, hs, acc_mfh, acc_nh, plog);
        __syncthreads();
    }
    q_flush(q, qout, plog, &cn->qtail);
    if (kDist) rq_flush(*rq, pt);
    // top-down: stage2 = degree sum of the hub-domain vertices discovered, walked = their number
    shard_add(cn, 0, acc_mf, scanned, attempts, 0, acc_dmax, acc_mfh, acc_nh);
    publish_if_last(cn, pub, seq);
    if (kDist) slot_headers_if_last(pt);
}

template <bool kDist, class OffT>
__global__ __launch_bounds__(kBS) void k_td_hubs(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                                 const uint32_t *__restrict__ hubs, uint32_t *__restrict__ qout,
                                                 u64 *vis, u64 *__restrict__ stt, uint32_t *__restrict__ par,
                                                 LevelSlot *ring, int level,
                                                 Part pt, HubSet hs, Published *pub, u64 seq, u64 *__restrict__ plog) {
    LevelSlot *cn = ring + (level + 1) % 3;
    __shared__ u64 s_scan[kHubBatch + 1];
    __shared__ int64_t s_beg[kHubBatch];
    __shared__ uint32_t s_u[kHubBatch];
    __shared__ u64 s_tsum[kBS];
    __shared__ typename std::conditional<kDist, DistQueue, LogQueue>::type q;
    __shared__ typename std::conditional<kDist, RemoteQueue, char>::type rq_storage;
    RemoteQueue *rq = kDist ? reinterpret_cast<RemoteQueue *>(&rq_storage) : nullptr;
    bq_init(q);
    if (kDist && threadIdx.x == 0) rq->n = 0;
    const uint32_t nh = (uint32_t)cn->nhub;
    const int32_t nd = level + 1;
    const unsigned tid = threadIdx.x;
    constexpr int kPer = kHubBatch / kBS;
    u64 acc_mf = 0, attempts = 0, scanned = 0, acc_dmax = 0, acc_mfh = 0, acc_nh = 0;
    __syncthreads();
    for (uint32_t h0 = 0; h0 < nh; h0 += kHubBatch) {
        const int hb = (int)min((uint32_t)kHubBatch, nh - h0);
        // thread tid owns batch entries [tid*kPer, tid*kPer+kPer): load degrees, local sum
        u64 d[kPer], local = 0;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int idx = (int)tid * kPer + k;
            d[k] = 0;
            if (idx < hb) {
                const uint32_t u = hubs[h0 + idx];
                const bool ok = id_ok(u, pt.nrows, pt.err);
                const int64_t b = ok ? (int64_t)row_off[u] : 0;
                d[k] = ok ? (u64)((int64_t)row_off[u + 1] - b) : 0ull;
                s_beg[idx] = b;
                s_u[idx] = ok ? u : 0u;
            }
            local += d[k];
        }
        s_tsum[tid] = local;
        __syncthreads();
        // block inclusive scan of the per-thread sums (Hillis-Steele in LDS)
        for (int off = 1; off < kBS; off <<= 1) {
            const u64 add = tid >= (unsigned)off ? s_tsum[tid - off] : 0ull;
            __syncthreads();
            s_tsum[tid] += add;
            __syncthreads();
        }
        u64 run = s_tsum[tid] - local;
        const u64 total = s_tsum[kBS - 1];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int idx = (int)tid * kPer + k;
            s_scan[idx] = (idx < hb) ? run : total;
            run += d[k];
        }
        if (tid == 0) s_scan[kHubBatch] = total;
        __syncthreads();
        // this workgroup's equal share of the batch's edges
        const uint64_t x_begin = total * blockIdx.x / gridDim.x, x_end = total * (blockIdx.x + 1) / gridDim.x;
        if (tid == 0) scanned += x_end - x_begin;
        sweep_segments<kDist>(s_scan, s_beg, s_u, hb, x_begin, x_end, row_off, col, vis, stt, par, nd, q, qout, &cn->qtail, pt,
                              rq, acc_mf, attempts, acc_dmax, hs, acc_mfh, acc_nh, plog);
        __syncthreads();
    }
    q_flush(q, qout, plog, &cn->qtail);
    if (kDist) rq_flush(*rq, pt);
    shard_add(cn, 0, acc_mf, scanned, attempts, 0, acc_dmax, acc_mfh, acc_nh);
    publish_if_last(cn, pub, seq);
    if (kDist) slot_headers_if_last(pt);
}

// ---- K3p: persistent top-down for narrow frontiers --------------------------------------------------
// High-diameter graphs (largeG: >= 567 levels, BreadthFirstPaths.java:33) run hundreds of levels whose
// frontiers hold a few thousand vertices: per level, two launches, the host round trip and a
// chain of single-counter atomics cost more than the work.  One launch of at most one workgroup per
// CU runs such levels back to back, with no same-address atomic on the level's critical path:
//   * workgroup b takes the frontier slice [nf*b/G, nf*(b+1)/G) and sweeps its rows edge-parallel
//     (as k_td); the vis word and the target's row offsets are loaded together, so a win costs no
//     further round trip;
//   * winners go straight to b's own output segment (kRegion slots of {row start, vertex | degree}; LDS
//     counter, no global cursor), written through L2 (`sc1` stores), and b's level record {n, m_f,
//     scanned, claims, d_max};
//   * the records are the grid barrier (round 3): every word carries the level's 16-bit tag, and thread t
//     of every workgroup polls workgroup t's record until it holds the tag -- so the arrival and the record
//     read are one round trip (an arrival counter plus a separate record read cost the largeG stand-in
//     1.5 us per level).  Every workgroup then scans the counts into segment offsets and takes the same
//     decision: continue, or stop when the BFS ends, the next frontier is no longer narrow (n_f >
//     kPersistNf, or a slice could hold more than kRegion edges), Beamer's rule asks for bottom-up or
//     the level budget is used up.  On stop every workgroup copies its segment into the contiguous
//     queue the per-level kernels read.
// Hand-off form (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table): every
// handed-off byte (segment entries, records) is stored `sc1` and loaded `sc1`; every wave waits
// vmcnt(0) before the workgroup barrier behind which one lane writes the tagged record; the poll is an
// `sc1` load of every record's tagged words.  Visited words are claimed by device atomics (a stale plain
// pre-check can only under-report a set bit), the state array is read only after the launch.
constexpr uint32_t kRegion = 16384; // output slots per workgroup and level parity
struct alignas(128) PersistCtl {
    u64 abort; // raised by a workgroup whose poll timed out or whose segment would overflow
    u64 pad[15];
};
// host-visible result of one launch (mapped pinned memory, written by workgroup 0)
struct alignas(64) PersistOut {
    u64 levels, abort, t0, done, pad[4]; // done: set by workgroup 0 once levels / abort / the records are final
    PersistRec rec[kPersistLevels];
};

__device__ inline void st_sc1(u64 *p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline u64 ld_sc1(const u64 *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }


// Heavy rows inside K3p (round 3).  A frontier vertex with more than `heavy_deg` entries is not swept by the
// one workgroup whose slice holds it: the workgroup that discovers it records it in its own heavy region
// (row start, vertex, degree; at most kHeavyPer per workgroup and level -- more stay light), and at the next
// level every workgroup loads the whole heavy table (at most kHeavyMax rows) into LDS and sweeps an equal
// 1/G share of its edges, exactly as the per-level hub bin (k_td_hubs) spreads hub rows.  So a narrow level
// whose few vertices hold hundreds of thousands of edges -- a BFS's first and second levels -- runs inside
// the launch instead of costing two launches and a host round trip each.  The first level's heavy row (the
// source) comes from the host (h0_*).
constexpr uint32_t kHeavyPer = 32;
constexpr uint32_t kHeavyMax = 1024;

// One step of K3p's sweep: kBS * kItems edges [x0, x_end) of a segment table (scan / row start / vertex, n
// rows).  Winners store their state; light ones (<= heavy_deg entries, or a full heavy region) go to the
// workgroup's segment, heavy ones to its heavy region (see k_td_persist).  Block-uniform.
template <class OffT, bool kHeavy>
__device__ __forceinline__ void persist_step(uint32_t x0, uint32_t x_end, const uint32_t *t_scan, const int64_t *t_beg,
                                             const uint32_t *t_u, int n, const OffT *__restrict__ row_off,
                                             const uint32_t *__restrict__ col, u64 *vis, u64 *__restrict__ stt,
                                             int32_t nd, HubSet hs, u64 heavy_deg, u64 *sout,
                                             u64 *hout, uint32_t &s_n, uint32_t &s_hn, PersistCtl *ctl, u64 &acc_mf,
                                             u64 &attempts, u64 &acc_dmax, u64 &acc_mfh, u64 &acc_eh, u64 &acc_dmh) {
    const unsigned tid = threadIdx.x, lane = tid & 63u;
    uint32_t v[kItems], pu[kItems];
    bool valid[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const uint32_t x = x0 + (uint32_t)k * kBS + tid;
        valid[k] = x < x_end;
        v[k] = 0;
        pu[k] = 0;
        if (valid[k]) {
            int lo = 0, hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (t_scan[mid] <= x) lo = mid;
                else hi = mid - 1;
            }
            v[k] = col[t_beg[lo] + (int64_t)(x - t_scan[lo])];
            pu[k] = t_u[lo];
        }
    }
    // the visited word and the target's row bounds in one round trip
    u64 wv[kItems];
    int64_t r0[kItems], r1[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        wv[k] = valid[k] ? vis[v[k] >> 6] : ~0ull;
        r0[k] = valid[k] ? (int64_t)row_off[v[k]] : 0;
        r1[k] = valid[k] ? (int64_t)row_off[v[k] + 1] : 0;
    }
    // every item's claim in flight before any result is used (a ballot per item would wait out one atomic
    // round trip per item in turn)
    u64 old[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const u64 bit = 1ull << (v[k] & 63u);
        old[k] = bit;
        if (!(wv[k] & bit)) {
            attempts++;
            old[k] = atomicOr(vis + (v[k] >> 6), bit);
        }
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const bool win = !(old[k] & (1ull << (v[k] & 63u)));
        const u64 dg = win ? (u64)(r1[k] - r0[k]) : 0ull;
        bool heavy = false;
        if (win) {
            stt[v[k]] = pack_state(pu[k], nd);
            if (kHeavy && dg > heavy_deg) { // a heavy row: this workgroup's heavy region, if it has room
                const uint32_t hp = atomicAdd(&s_hn, 1u);
                if (hp < kHeavyPer) {
                    st_sc1(hout + 2 * hp, (u64)r0[k]);
                    st_sc1(hout + 2 * hp + 1, (u64)v[k] | (dg << 32));
                    heavy = true;
                }
            }
        }
        const bool light = win && !heavy;
        acc_mf += dg;
        acc_mfh += is_hub(hs, v[k], dg) ? dg : 0ull;
        acc_eh += heavy ? dg : 0ull;
        const u64 dl = light ? dg : 0ull, dh = heavy ? dg : 0ull;
        acc_dmax = dl > acc_dmax ? dl : acc_dmax;
        acc_dmh = dh > acc_dmh ? dh : acc_dmh;
        const u64 mask = __ballot(light);
        if (mask) {
            const int leader = __ffsll((long long)mask) - 1;
            uint32_t pos = 0;
            if ((int)lane == leader) pos = atomicAdd(&s_n, (uint32_t)__popcll(mask));
            pos = __shfl(pos, leader) + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
            if (light) {
                if (pos < kRegion) { // the entry carries its row bounds: the next level needs no row_off load
                    st_sc1(sout + 2 * pos, (u64)r0[k]);
                    st_sc1(sout + 2 * pos + 1, (u64)v[k] | (dg << 32));
                }
                else st_sc1(&ctl->abort, 1ull); // cannot happen: slices are bounded on entry
            }
        }
    }
}

// K3p's end for the host: every record / count store of workgroup 0 drained and made visible system-wide before
// the flag (PersistOut lives in mapped pinned host memory).
__device__ inline void persist_done(PersistOut *out) {
    __threadfence_system();
    *reinterpret_cast<volatile u64 *>(&out->done) = 1ull;
}

// alpha <= 0: no direction switch (direction forced top-down).  q0: the first level's (light) frontier
// (contiguous); seg: 2 parities x G segments of kRegion; brec: 2 parities x G records (kRecWords); hseg: 2
// parities x G heavy regions of kHeavyPer entries {row start, vertex | degree << 32}; qfinal: the last
// frontier, contiguous (light entries, then heavy ones).  bar0: barrier rounds completed by earlier launches.
// kHeavy = false: the instantiation for graphs without a row longer than persist_dmax (no heavy table, no
// heavy regions): the heavy machinery costs a largeG-class level ~2 us (19.1 vs 17.0 us per level).
template <class OffT, bool kHeavy>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_td_persist(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                                    const uint32_t *__restrict__ q0, uint32_t nf0, u64 *seg,
                                                    u64 *brec, uint32_t *__restrict__ qfinal, u64 *vis,
                                                    u64 *__restrict__ stt, LevelSlot *ring, int level0, int64_t mu0,
                                                    int alpha, int max_levels, u64 bar0, PersistCtl *ctl,
                                                    PersistOut *out, HubSet hs, int64_t bu_floor,
                                                    int inject_abort, u64 heavy_deg, uint32_t nrows, u64 *err,
                                                    u64 *hseg, uint32_t h0_v, uint32_t h0_deg, int64_t h0_beg) {
    extern __shared__ char s_dyn[]; // sized by the host so that one workgroup fills a CU's LDS share
    __shared__ uint32_t s_off[kBS + 1];
    __shared__ uint32_t s_hoff[kBS + 1];
    __shared__ uint32_t s_scan[kBS + 1];
    __shared__ int64_t s_beg[kBS];
    __shared__ uint32_t s_u[kBS];
    __shared__ uint32_t s_wsum[kWaves];
    __shared__ u64 s_red[9][kWaves];
    __shared__ uint32_t s_n, s_hn;
    constexpr uint32_t kHT = kHeavy ? kHeavyMax : 1u; // the heavy table's LDS (none without heavy rows)
    __shared__ uint32_t s_hv[kHT];
    __shared__ int64_t s_hb[kHT];
    __shared__ uint32_t s_hscan[kHT + 1];
    (void)s_dyn;
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const unsigned G = gridDim.x, b = blockIdx.x;
    if (b == 0) {
        // the per-level kernels that follow expect clean counter slots (each zeroes two levels ahead)
        u64 *p = reinterpret_cast<u64 *>(ring);
        for (int i = tid; i < 3 * kSlotWords; i += kBS) p[i] = 0ull;
        if (tid == 0) out->t0 = (u64)wall_clock64();
    }
    uint32_t nf = nf0, nh_in = h0_deg ? 1u : 0u;
    u64 eh_in = h0_deg;
    int64_t mu = mu0;
    for (int it = 0;; it++) {
        // segments of 16-B entries {row start, vertex | degree << 32}
        const u64 *sin = seg + (size_t)((it + 1) & 1) * G * kRegion * 2; // previous level's segments
        u64 *sout = seg + ((size_t)(it & 1) * G * kRegion + (size_t)b * kRegion) * 2;
        const u64 *hin = hseg + (size_t)((it + 1) & 1) * G * kHeavyPer * 2;   // previous level's heavy regions
        u64 *hout = hseg + ((size_t)(it & 1) * G + b) * kHeavyPer * 2;          // this workgroup's
        u64 *rout = brec + (size_t)(it & 1) * G * kRecWords;
        const u64 tag = ((bar0 + (u64)it + 1) & 0xFFFFull) << 48; // this level's record tag (never 0)
        const int32_t nd = level0 + it + 1;
        if (tid == 0) {
            s_n = 0;
            s_hn = 0;
        }
        u64 acc_mf = 0, attempts = 0, scanned = 0, acc_dmax = 0, acc_mfh = 0, acc_eh = 0, acc_dmh = 0;
        // this level's heavy table (every workgroup holds all of it)
        if (kHeavy && nh_in) {
            uint32_t d[kHeavyMax / kBS];
            uint32_t local = 0;
#pragma unroll
            for (int k = 0; k < (int)(kHeavyMax / kBS); k++) {
                const uint32_t t = tid * (kHeavyMax / kBS) + (uint32_t)k;
                d[k] = 0;
                if (t < nh_in) {
                    uint32_t v = h0_v;
                    int64_t beg = h0_beg;
                    d[k] = h0_deg;
                    if (it > 0) { // region r of heavy index t: the last with s_hoff[r] <= t
                        int lo = 0, hi = (int)G - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (s_hoff[mid] <= t) lo = mid;
                            else hi = mid - 1;
                        }
                        const u64 *e = hin + ((size_t)lo * kHeavyPer + (t - s_hoff[lo])) * 2;
                        beg = (int64_t)ld_sc1(e);
                        const u64 w = ld_sc1(e + 1);
                        v = (uint32_t)w;
                        d[k] = (uint32_t)(w >> 32);
                    }
                    s_hv[t] = v;
                    s_hb[t] = beg;
                }
                local += d[k];
            }
            const uint32_t inc = wave_incl_scan(local);
            if (lane == 63) s_wsum[wave] = inc;
            __syncthreads();
            uint32_t run = inc - local;
            for (int w = 0; w < (int)wave; w++) run += s_wsum[w];
#pragma unroll
            for (int k = 0; k < (int)(kHeavyMax / kBS); k++) {
                s_hscan[tid * (kHeavyMax / kBS) + (uint32_t)k] = run;
                run += d[k];
            }
            if (tid == kBS - 1) s_hscan[kHeavyMax] = run;
        }
        // nf <= kPersistNf and b < kBS: the products fit 32 bits (no 64-bit division on the critical path)
        const uint32_t vb = nf * b / G, ve = nf * (b + 1) / G;
        __syncthreads();
        // light rows: this workgroup's slice of the frontier, its rows swept by this workgroup
        for (uint32_t base = vb; base < ve; base += kBS) {
            const uint32_t i = base + tid;
            const int n = (int)min((uint32_t)kBS, ve - base);
            uint32_t deg = 0, u = 0;
            int64_t beg = 0;
            if (i < ve) {
                if (it == 0) {
                    u = q0[i];
                    if (!id_ok(u, nrows, err)) u = 0xFFFFFFFFu;
                } else { // segment s of frontier index i: the last with s_off[s] <= i
                    int lo = 0, hi = (int)G - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (s_off[mid] <= i) lo = mid;
                        else hi = mid - 1;
                    }
                    const u64 *e = sin + ((size_t)lo * kRegion + (i - s_off[lo])) * 2;
                    beg = (int64_t)ld_sc1(e);
                    const u64 w = ld_sc1(e + 1);
                    u = (uint32_t)w;
                    deg = (uint32_t)(w >> 32);
                }
                if (it == 0) {
                    if (u != 0xFFFFFFFFu) {
                        beg = (int64_t)row_off[u];
                        deg = (uint32_t)((int64_t)row_off[u + 1] - beg);
                    } else {
                        u = 0; // a rejected q0 entry: an empty row
                    }
                }
            }
            const uint32_t inc = wave_incl_scan(deg);
            if (lane == 63) s_wsum[wave] = inc;
            __syncthreads();
            uint32_t woff = 0, total = 0;
#pragma unroll
            for (int w = 0; w < kWaves; w++) {
                const uint32_t t = s_wsum[w];
                woff += (w < (int)wave) ? t : 0u;
                total += t;
            }
            s_scan[tid] = woff + inc - deg;
            s_beg[tid] = beg;
            s_u[tid] = u;
            if (tid == 0) scanned += total;
            __syncthreads();
            for (uint32_t x0 = 0; x0 < total; x0 += kBS * kItems)
                persist_step<OffT, kHeavy>(x0, total, s_scan, s_beg, s_u, n, row_off, col, vis, stt, nd, hs, heavy_deg, sout, hout, s_n,
                             s_hn, ctl, acc_mf, attempts, acc_dmax, acc_mfh, acc_eh, acc_dmh);
            __syncthreads();
        }
        // heavy rows: this workgroup's 1/G share of the heavy table's edges
        if (kHeavy && nh_in) {
            const uint32_t xb = (uint32_t)(eh_in * b / G), xe = (uint32_t)(eh_in * (b + 1) / G);
            if (tid == 0) scanned += xe - xb;
            for (uint32_t x0 = xb; x0 < xe; x0 += kBS * kItems)
                persist_step<OffT, kHeavy>(x0, xe, s_hscan, s_hb, s_hv, (int)nh_in, row_off, col, vis, stt, nd, hs, heavy_deg, sout,
                             hout, s_n, s_hn, ctl, acc_mf, attempts, acc_dmax, acc_mfh, acc_eh, acc_dmh);
        }
        // test hook (option "persist_abort_at"): every workgroup takes the abort path at this level, as a
        // grid-barrier timeout would, and the host re-runs the BFS without K3p
        if (it == inject_abort) {
            if (b == 0 && tid == 0) {
                out->abort = 1;
                out->levels = (u64)it;
                persist_done(out);
            }
            return;
        }
        // this workgroup's level record: {n | light d_max << 32, m_f, scanned, claims, m_f(hubs),
        // heavy n | heavy d_max << 32, heavy edges}
        {
            const u64 v0 = wave_sum(acc_mf), v1 = wave_sum(scanned), v2 = wave_sum(attempts), v3 = wave_max(acc_dmax),
                      v4 = wave_sum(acc_mfh), v5 = wave_sum(acc_eh), v6 = wave_max(acc_dmh);
            if (lane == 0) {
                s_red[0][wave] = v0;
                s_red[1][wave] = v1;
                s_red[2][wave] = v2;
                s_red[3][wave] = v3;
                s_red[4][wave] = v4;
                s_red[5][wave] = v5;
                s_red[6][wave] = v6;
            }
            // the record is the arrival: every wave's segment / heavy-region / claim traffic must have
            // completed before thread 0 writes it
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                u64 a = 0, c = 0, d = 0, m = 0, h = 0, e = 0, mh = 0;
                for (int w = 0; w < kWaves; w++) {
                    a += s_red[0][w];
                    c += s_red[1][w];
                    d += s_red[2][w];
                    m = s_red[3][w] > m ? s_red[3][w] : m;
                    h += s_red[4][w];
                    e += s_red[5][w];
                    mh = s_red[6][w] > mh ? s_red[6][w] : mh;
                }
                const u64 nh = min(s_hn, kHeavyPer);
                // every word carries the level's 16-bit tag (bits 48..63): the words are the barrier
                constexpr u64 k24 = (1ull << 24) - 1, k48 = (1ull << 48) - 1;
                u64 *r = rout + kRecWords * b;
                st_sc1(r + 0, (u64)s_n | (min(m, k24) << 24) | tag);
                st_sc1(r + 1, min(a, k48) | tag);
                st_sc1(r + 2, min(c, k48) | tag);
                st_sc1(r + 3, min(d, k48) | tag);
                st_sc1(r + 4, min(h, k48) | tag);
                if (kHeavy) {
                    st_sc1(r + 5, nh | (min(mh, k24) << 24) | tag);
                    st_sc1(r + 6, min(e, k48) | tag);
                }
            }
        }
        // Barrier and record exchange in one: thread t < G polls workgroup t's record until every word
        // carries this level's tag (no arrival counter, no separate record read after it).  d_max values
        // are clamped to 2^24 - 1: any value above kRegion stops the launch anyway.
        u64 r_n = 0, r_dm = 0, r_mf = 0, r_sc = 0, r_cl = 0, r_mfh = 0, r_nh = 0, r_dmh = 0, r_eh = 0;
        {
            __shared__ int s_ok;
            if (tid == 0) s_ok = 1;
            __syncthreads();
            constexpr u64 k24 = (1ull << 24) - 1, k48 = (1ull << 48) - 1;
            const u64 *rr = rout + kRecWords * tid;
            u64 w[kRecWords] = {0, 0, 0, 0, 0, 0, 0};
            constexpr int kw = kHeavy ? kRecWords : 5;
            for (uint32_t spin = 0;; spin++) {
                // poll the first word alone while waiting (1/kw of the traffic), then the others once
                bool ok = true;
                if (tid < G) {
                    w[0] = ld_sc1(rr);
                    ok = (w[0] & ~k48) == tag;
                }
                if (__all(ok)) {
                    if (tid < G) {
#pragma unroll
                        for (int i = 1; i < kw; i++) w[i] = ld_sc1(rr + i);
#pragma unroll
                        for (int i = 1; i < kw; i++) ok = ok && (w[i] & ~k48) == tag;
                    }
                    if (__all(ok)) break;
                }
                if (ld_sc1(&ctl->abort)) {
                    s_ok = 0;
                    break;
                }
                if (spin > (1u << 22)) {
                    if (lane == 0) st_sc1(&ctl->abort, 1ull);
                    s_ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            // a workgroup whose segment overflowed (its record's count exceeds kRegion; it also raised ctl->abort)
            // makes every workgroup take the abort path at THIS level, before any s_off is built from that count
            if (tid < G && (w[0] & k24) > (u64)kRegion) s_ok = 0;
            __syncthreads();
            if (!s_ok) {
                if (b == 0 && tid == 0) {
                    out->abort = 1;
                    out->levels = (u64)it;
                    persist_done(out);
                }
                return;
            }
            if (tid < G) {
                r_n = w[0] & k24;
                r_dm = (w[0] >> 24) & k24;
                r_mf = w[1] & k48;
                r_sc = w[2] & k48;
                r_cl = w[3] & k48;
                r_mfh = w[4] & k48;
                if (kHeavy) {
                    r_nh = w[5] & k24;
                    r_dmh = (w[5] >> 24) & k24;
                    r_eh = w[6] & k48;
                }
            }
        }
        // what every workgroup needs for the offsets and the stop decision; the statistics only workgroup 0
        // publishes (scanned, claims, hub m_f, heavy d_max) are reduced there alone (the level's critical path)
        const bool stats = b == 0;
        const uint32_t inc = wave_incl_scan((uint32_t)r_n), hinc = kHeavy ? wave_incl_scan((uint32_t)r_nh) : 0u;
        const u64 smf = wave_sum(r_mf), seh = kHeavy ? wave_sum(r_eh) : 0ull;
        const u64 sdm = wave_max32((uint32_t)r_dm); // d_max values are clamped to 24 bits
        u64 ssc = 0, scl = 0, smfh = 0, sdmh = 0;
        if (stats) {
            ssc = wave_sum(r_sc);
            scl = wave_sum(r_cl);
            smfh = wave_sum(r_mfh);
            sdmh = kHeavy ? wave_max(r_dmh) : 0ull;
        }
        __shared__ uint32_t s_hw[kWaves];
        __syncthreads(); // s_red / s_wsum reuse
        if (lane == 63) {
            s_wsum[wave] = inc;
            s_hw[wave] = hinc;
        }
        if (lane == 0) {
            s_red[0][wave] = smf;
            s_red[1][wave] = ssc;
            s_red[2][wave] = scl;
            s_red[3][wave] = sdm;
            s_red[4][wave] = smfh;
            s_red[5][wave] = seh;
            s_red[6][wave] = sdmh;
        }
        __syncthreads();
        uint32_t woff = 0, nf_new = 0, hoff = 0, nh_new = 0;
        u64 mf_new = 0, sc_new = 0, cl_new = 0, dm_new = 0, mfh_new = 0, eh_new = 0, dmh_new = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            woff += (w < (int)wave) ? s_wsum[w] : 0u;
            nf_new += s_wsum[w];
            hoff += (w < (int)wave) ? s_hw[w] : 0u;
            nh_new += s_hw[w];
            mf_new += s_red[0][w];
            dm_new = s_red[3][w] > dm_new ? s_red[3][w] : dm_new;
            eh_new += s_red[5][w];
            if (stats) {
                sc_new += s_red[1][w];
                cl_new += s_red[2][w];
                mfh_new += s_red[4][w];
                dmh_new = s_red[6][w] > dmh_new ? s_red[6][w] : dmh_new;
            }
        }
        const uint32_t my_n = (uint32_t)r_n, my_nh = (uint32_t)r_nh;
        s_off[tid] = woff + inc - my_n; // entries past G: unused
        s_hoff[tid] = hoff + hinc - my_nh;
        if (tid == 0) {
            s_off[kBS] = nf_new;
            s_hoff[kBS] = nh_new;
        }
        const uint32_t nf_all = nf_new + nh_new;
        if (b == 0 && tid == 0) {
            PersistRec &r = out->rec[it];
            r.qtail = nf_all;
            r.mf = mf_new;
            r.dmax = dm_new > dmh_new ? dm_new : dmh_new;
            r.scanned = sc_new;
            r.claims = cl_new;
            r.mfh = mfh_new;
            r.t_end = (u64)wall_clock64();
            out->levels = (u64)(it + 1);
        }
        mu -= (int64_t)mf_new;
        // stop when the BFS ends, the light frontier is no longer narrow, the heavy table would overflow, a
        // workgroup's share (light slice + heavy edges) could overflow its segment, Beamer asks for
        // bottom-up, or the level budget is used up
        // (Beamer's m_f > m_u / alpha as a product: the same decision as the host's for m_u >= 0, without a
        // 64-bit division on every workgroup's critical path)
        const bool beamer = alpha > 0 && (mu >= 0 ? (int64_t)mf_new * alpha > mu : (int64_t)mf_new > mu / alpha);
        const bool stop = nf_all == 0 || nf_new > kPersistNf || nh_new > kHeavyMax ||
                          (u64)((nf_new + G - 1) / G) * dm_new + (kHeavy ? (eh_new + G - 1) / G : 0ull) > (u64)kRegion ||
                          (beamer && (int64_t)mf_new > bu_floor) ||
                          it + 1 >= max_levels;
        __syncthreads();
        // the host reads the counts as soon as they are final (a mapped flag, no stream synchronise: that cost ~13 us
        // per launch); the hand-back below is stream-ordered before the next kernel anyway
        if (stop && b == 0 && tid == 0) persist_done(out);
        if (stop) { // hand the frontier back contiguous: the light entries, then the heavy ones
            const uint32_t nb = (b + 1 < G ? s_off[b + 1] : nf_new) - s_off[b], ob = s_off[b];
            for (uint32_t i = tid; i < nb; i += kBS) qfinal[ob + i] = (uint32_t)ld_sc1(sout + 2 * i + 1);
            const uint32_t hb = (b + 1 < G ? s_hoff[b + 1] : nh_new) - s_hoff[b], hbase = nf_new + s_hoff[b];
            for (uint32_t i = tid; i < hb; i += kBS) qfinal[hbase + i] = (uint32_t)ld_sc1(hout + 2 * i + 1);
            return;
        }
        nf = nf_new;
        nh_in = nh_new;
        eh_in = eh_new;
    }
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
// Multi-GPU: claim the (v, parent) pairs other ranks routed to this rank's vertices.
template <class OffT>
__global__ __launch_bounds__(kBS) void k_claim_remote(const u64 *__restrict__ pairs, u64 npairs,
                                                      const OffT *__restrict__ row_off, u64 *vis,
                                                      u64 *__restrict__ stt, uint32_t *__restrict__ qout,
                                                      LevelSlot *ring, int level, uint32_t lo, u64 slot,
                                                      uint32_t nrows, u64 *err, int64_t *sums, u64 *ctr, int nctr,
                                                      u64 *arrive, int rank, int nranks) {
    LevelSlot *cn = ring + (level + 1) % 3;
    __shared__ BlockQueue q;
    bq_init(q);
    __syncthreads();
    const int32_t nd = level + 1;
    u64 acc_mf = 0, attempts = 0, acc_dmax = 0;
    // slot > 0: npairs = P * slot entries in P fixed slots of [count, slot pairs] (small levels)
    for (u64 i0 = (u64)blockIdx.x * kBS; i0 < npairs; i0 += (u64)gridDim.x * kBS) {
        const u64 i = i0 + threadIdx.x;
        bool win = false;
        uint32_t vl = 0;
        bool have = i < npairs;
        u64 at = i;
        if (have && slot) { // the own slot is not exchanged (plan_slots): skipped
            const u64 p = i / slot, k = i - p * slot;
            const u64 base = p * (slot + 1);
            have = p != (u64)rank && k < pairs[base];
            at = base + 1 + k;
        }
        if (have) {
            const u64 pr = pairs[at];
            vl = (uint32_t)(pr >> 32) - lo;
            if (id_ok(vl, nrows, err) && claim(vl, vis, attempts)) {
                win = true;
                stt[vl] = pack_state((uint32_t)pr, nd);
                const u64 dg = (u64)(row_off[vl + 1] - row_off[vl]);
                acc_mf += dg;
                acc_dmax = dg > acc_dmax ? dg : acc_dmax;
            }
        }
        bq_push(q, win, vl);
        __syncthreads();
        if (q.n > (uint32_t)(kQCap - kBS)) bq_flush(q, qout, &cn->qtail);
    }
    bq_flush(q, qout, &cn->qtail);
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


__global__ __launch_bounds__(kBS) void k_bucket_count(const u64 *__restrict__ pairs, const u64 *__restrict__ d_n,
                                                      uint32_t chunk, int nranks, u64 *__restrict__ dcount) {
    __shared__ uint32_t s_h[kMaxRanks];
    const uint64_t n = *d_n;
    for (int d = threadIdx.x; d < nranks; d += kBS) s_h[d] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBS)
        atomicAdd(&s_h[(uint32_t)(pairs[i] >> 32) / chunk], 1u);
    __syncthreads();
    for (int d = threadIdx.x; d < nranks; d += kBS)
        if (s_h[d]) atomicAdd(&dcount[d], (u64)s_h[d]);
}

// Small top-down levels (fixed per-destination slots of [count, cap pairs], so the exchange needs no count
// all-to-all and no host round trip before the pairs move) are bucketed by the push kernels themselves
// (rq_flush in slot mode, slot_headers_if_last); the counted exchange below buckets in two passes.
__global__ __launch_bounds__(kBS) void k_bucket_scatter(const u64 *__restrict__ pairs, const u64 *__restrict__ d_n,
                                                        uint32_t chunk, int nranks, const u64 *__restrict__ dcount,
                                                        u64 *__restrict__ dcursor, u64 *__restrict__ out) {
    __shared__ uint32_t s_h[kMaxRanks];
    __shared__ u64 s_base[kMaxRanks];
    const uint64_t n = *d_n;
    for (uint64_t i0 = (uint64_t)blockIdx.x * kBS; i0 < n; i0 += (uint64_t)gridDim.x * kBS) {
        for (int d = threadIdx.x; d < nranks; d += kBS) s_h[d] = 0;
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        u64 pr = 0;
        uint32_t d = 0, r = 0;
        if (i < n) {
            pr = pairs[i];
            d = (uint32_t)(pr >> 32) / chunk;
            r = atomicAdd(&s_h[d], 1u);
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
        if (i < n) out[s_base[d] + r] = pr;
        __syncthreads();
    }
}

// ---- K5: bottom-up pull --------------------------------------------------------------------------
// A wave owns 64 consecutive words of the visited bitmap (4096 vertices): one coalesced 512-B load
// brings them into registers (lane k holds word w0+k).  The unvisited vertices of the group are
// compacted lane-densely -- a wave prefix of per-word popcounts gives every word its first rank, and
// each round every word writes the ids of its unvisited bits ranked inside the round into an LDS
// list -- so every lane works on a live candidate whether the level leaves half the vertices
// unvisited or one in a hundred.  Then two phases per round of kBuU*64 candidates:
//   A  every lane takes kBuU candidates at once: kBuU coalesced top1[v] loads (v's highest-degree
//      neighbour), then kBuU independent frontier-bit probes -- the whole round costs two memory
//      round trips instead of two per candidate.  Hits are done: no row offset is ever read for them.
//   B  the misses (compacted into LDS with a ballot) walk the rest of their rows, 8 entries per step.
//      A miss whose row holds only top1 (kDeg1 flag in top1) is settled in A without a row read.
// Found bits are OR-ed into a per-wave LDS copy of the 64 next-frontier words and written back
// coalesced with the visited words.  Single GPU: m_f of the new frontier is not needed (a bottom-up
// level is only ever followed by the n_f test), so the level accumulates the exact m_u instead --
// the degree sum of the candidates it leaves unvisited, which it reads anyway.  kMf (multi-GPU)
// also accumulates m_f, the size bound of the next top-down exchange.
// kHubs (single device): every frontier-bit probe of the level is a random 8-B access into an n/8-byte
// bitmap (8 MiB at scale 26: twice an XCD's L2, so most probes are served by the Infinity Cache).  The
// probes concentrate on high-degree vertices: top1 IS a vertex's highest-degree neighbour and rows are
// degree-ordered.  So the hub_k highest-degree vertices get a second, dense id h: `colh` (a copy of col)
// and top1 carry kHubBit | h for hub entries, and a kernel before each bottom-up level gathers the
// hubs' frontier bits into `hfront` (hub_k bits: 256 KiB at scale 26, L2-resident on every XCD).  A
// hub probe reads hfront, any other probe reads front; the parent of a hub hit is hub_id[h].
// kU: candidates per lane per round (4 at 6 waves/SIMD, or 2 at 8 waves/SIMD; option "bu_unroll")
constexpr uint32_t kDeg1 = 0x80000000u;
constexpr uint32_t kHubBit = 0x40000000u; // hub encoding needs every global id < 2^30
constexpr uint32_t kHubMask = kHubBit - 1u;

// word holding the frontier bit of probe id x (bit x & 63: a hub index keeps the id's low 6 bits)
template <bool kHubs>
__device__ inline const u64 *probe_word(const u64 *__restrict__ front, const u64 *__restrict__ hfront, uint32_t x) {
    if (kHubs) {
        const bool hb = (x & kHubBit) != 0u;
        return (hb ? hfront : front) + ((x & (hb ? kHubMask : 0xFFFFFFFFu)) >> 6);
    }
    return front + (x >> 6);
}
template <bool kHubs>
__device__ inline uint32_t probe_id(const uint32_t *__restrict__ hub_id, uint32_t x) {
    return (kHubs && (x & kHubBit)) ? hub_id[x & kHubMask] : x;
}

// frontier bit of probe id x (32-bit probe word: one VGPR per probe in flight)
template <bool kHubs>
__device__ inline uint32_t probe_bit(const u64 *__restrict__ front, const u64 *__restrict__ hfront, uint32_t x) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(probe_word<kHubs>(front, hfront, x));
    return (w[(x >> 5) & 1u] >> (x & 31u)) & 1u;
}

// Whether adjacency entry x names a hub of the hybrid levels: the encoded domain's bit, or (relabelled
// graph, plain ids) an id below the hub limit.
template <bool kHubs>
__device__ inline bool hub_entry(uint32_t x, uint32_t lim) {
    return kHubs ? (x & kHubBit) != 0u : x < lim;
}

// Hub sweep (hybrid levels): only hub entries are probed; a non-hub entry reads as "not in frontier"
// without a memory access (the frontier's non-hub vertices are expanded top-down in the same level).
template <bool kHubs, bool kHubOnly>
__device__ inline uint32_t probe_hub(const u64 *__restrict__ front, const u64 *__restrict__ hfront, uint32_t x,
                                     uint32_t lim) {
    if (kHubOnly && !hub_entry<kHubs>(x, lim)) return 0u;
    return probe_bit<kHubs>(front, hfront, x);
}

// Second stage of phase A (see below): rest[v] = {c1, c2, c3, deg} -- the 2nd..4th neighbours of v in
// row order (the last one repeated for rows shorter than 4, so every slot is a real neighbour) and
// its degree (saturated at 2^32-1).  A miss on top1 probes c1..c3 at once from this one 16-B load;
// only rows longer than 4 without a hit there walk their row (phase B, from entry 4).
// kPipe: the next round's top1 loads are issued right after this round's frontier probes, so they
// overlap the probes, stage A2 and phase B instead of opening the next round (one dependent memory
// latency fewer per round; a half-group of dense candidates runs up to 8 rounds).
constexpr uint32_t kPrefIds = 1u << 16; // LDS frontier prefix: 8 KiB per workgroup
// A 64-word group's candidates are listed in kBuParts parts (kBuCand LDS slots per wave).  Round 4 measured 4 parts
// (22.8 KiB of LDS) at 5 and 6 waves per SIMD and 8 parts at 6: the pull kernel got 3-9% slower each time (fewer
// candidates per round), so 2 parts (31 KiB, 5 waves per SIMD) stay.
constexpr int kBuParts = 2;
constexpr uint32_t kBuCand = 64u * 64u / (uint32_t)kBuParts;
// The ids whose frontier bits the pull kernel reads from LDS: the first `ids` ids of each of `nseg` id
// ranges of 2^shift ids (one range on one device, shift >= 32 = the whole id space; a partition's
// ranks' ranges).  ids = 0: off.
struct PrefixSpec {
    uint32_t ids, nseg, shift, pad;
};
// A pull level's discovery: the 4-B parent only (the level's record bitmap gives the distance, BfsWorkspace::par;
// one device and the partitioned loop alike); par_out == null: the packed state.
__device__ __forceinline__ void settle_state(u64 *__restrict__ stt, uint32_t *__restrict__ par_out, uint32_t v,
                                             uint32_t parent, int32_t nd) {
    if (par_out) par_out[v] = parent;
    else stt[v] = pack_state(parent, nd);
}

// kSpill: a diagnostic instantiation compiled for 8 waves per SIMD (64 VGPRs), so it spills to scratch --
// option bu_force_spill, the round-2 "spilling pull kernel + concurrent in-process ranks" experiment.
template <class OffT, bool kMf, bool kHubs, int kU, bool kHubOnly, bool kPipe, bool kSpill = false>
__device__ __forceinline__ void k_bu_body(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const uint32_t *__restrict__ top1, const uint4 *__restrict__ rest,
                                            const u64 *__restrict__ front, u64 *__restrict__ next,
                                            u64 *__restrict__ vis, u64 *__restrict__ stt, uint32_t *__restrict__ par_out,
                                            LevelSlot *ring, int level,
                                            int64_t nwords, uint32_t fmask, const u64 *__restrict__ hfront,
                                            const uint32_t *__restrict__ hub_id, uint32_t hub_lim, uint32_t leaf_lo,
                                            PrefixSpec pf, Published *pub, u64 seq, uint32_t hub_row_lim) {
    LevelSlot *cn = ring + (level + 1) % 3;
    zero_slot(ring, level);
    __shared__ u64 s_nx[kWaves][64];
    // phase B's rows; the hub sweep (kHubOnly) carries them over rounds until a full 64-lane batch is ready
    __shared__ uint32_t s_miss[kWaves][(64 * kU) + (kHubOnly ? 64 : 0)];
    __shared__ uint16_t s_cand[kWaves][kBuCand]; // candidate offsets (v - group base) of one part of the group
    // the frontier bits of the first pf.ids ids of every id range (the highest-degree vertices of a
    // relabelled graph, where most probes land) copied to LDS once per workgroup; pf.ids = 0: off
    __shared__ uint32_t s_pref[kPrefIds / 32];
    {
        const uint32_t *front32 = reinterpret_cast<const uint32_t *>(front);
        const uint32_t wps = pf.ids / 32u; // words per range
        for (uint32_t i = threadIdx.x; i < wps * pf.nseg; i += kBS) {
            const uint32_t seg = i / wps;
            s_pref[i] = front32[((size_t)seg << (pf.shift - 5)) + (i - seg * wps)];
        }
        __syncthreads();
    }
    auto fword = [&](uint32_t x) -> uint32_t { // 32-bit frontier word of probe id x
        const uint32_t seg = pf.shift >= 32 ? 0u : (x >> pf.shift);
        const uint32_t off = pf.shift >= 32 ? x : (x & ((1u << pf.shift) - 1u));
        if (off < pf.ids) return s_pref[seg * (pf.ids >> 5) + (off >> 5)];
        return reinterpret_cast<const uint32_t *>(probe_word<kHubs>(front, hfront, x))[(x >> 5) & 1u];
    };
    auto fbit = [&](uint32_t x) -> uint32_t {
        if (kHubOnly && !hub_entry<kHubs>(x, hub_lim)) return 0u;
        return (fword(x) >> (x & 31u)) & 1u;
    };
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const int32_t nd = level + 1;
    // per-lane counters fit 32 bits (a lane sees a few hundred candidates per launch); widened at the end
    uint32_t acc_nf = 0, acc_mf = 0, acc_sc = 0, acc_mu = 0, acc_rows = 0, acc_s2 = 0, acc_wk = 0, acc_nh = 0;
    const int64_t wstride = (int64_t)gridDim.x * kWaves * 64;
    for (int64_t w0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; w0 < nwords; w0 += wstride) {
        const int64_t wl = w0 + lane;
        const u64 vwl = wl < nwords ? vis[wl] : ~0ull;
        const u64 unv = ~vwl;
        const uint32_t c = (uint32_t)__popcll(unv);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = __shfl(incl, 63);
        if (total == 0) { // wave-uniform: every vertex of the group visited or isolated
            if (wl < nwords) next[wl] = 0ull;
            continue;
        }
        const uint32_t excl = incl - c;
        s_nx[wave][lane] = 0ull;
        __builtin_amdgcn_wave_barrier();
        const uint32_t vbase = (uint32_t)(w0 * 64);
        // the group's candidates, one part (64 / kBuParts words, <= kBuCand vertices) at a time: each word's
        // lane writes the offsets of its unvisited bits at its rank, then rounds of (64 * kU) candidates
        for (int h = 0; h < kBuParts; h++) {
            constexpr int kWp = 64 / kBuParts; // words per part
            const uint32_t hb = h ? __shfl(incl, h * kWp - 1) : 0u, he = __shfl(incl, (h + 1) * kWp - 1);
            if (hb == he) continue; // wave-uniform
            if ((int)(lane / kWp) == h) {
                u64 bits = unv;
                uint32_t idx = excl - hb;
                while (bits) {
                    s_cand[wave][idx++] = (uint16_t)(lane * 64u + (uint32_t)(__ffsll((long long)bits) - 1));
                    bits &= bits - 1ull;
                }
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t xn[kU]; // kPipe: top1 of the next round's candidates, in flight
            if (kPipe) {
#pragma unroll
                for (int k = 0; k < kU; k++) {
                    const uint32_t vk = vbase + s_cand[wave][(uint32_t)k * 64 + lane];
                    xn[k] = (hb + (uint32_t)k * 64 + lane < he) ? top1[vk] : 0u;
                }
            }
            uint32_t nmiss = 0; // wave-uniform: phase-B rows waiting in s_miss
            for (uint32_t t0 = hb; t0 < he; t0 += (64 * kU)) {
                // diagnostic kSpill build: 48 VGPRs clobbered per round leave the live state too few
                // registers under the 96 of 5 waves/SIMD, so the compiler spills it to scratch
                if constexpr (kSpill) asm volatile("" ::: "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71");
                uint32_t v[kU], x[kU];
#pragma unroll
                for (int k = 0; k < kU; k++) // past the half's end: masked below
                    v[k] = vbase + s_cand[wave][t0 - hb + (uint32_t)k * 64 + lane];
                // A1: top1 of every candidate, then its frontier bit
                const uint32_t t1 = t0 + 64 * kU; // next round
                uint32_t vn[kU];
                if (kPipe) {
#pragma unroll
                    for (int k = 0; k < kU; k++) {
                        x[k] = xn[k];
                        const uint32_t at = t1 - hb + (uint32_t)k * 64 + lane; // past the list: unused (masked below)
                        vn[k] = vbase + s_cand[wave][at < kBuCand ? at : 0u];
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < kU; k++) x[k] = (t0 + (uint32_t)k * 64 + lane < he) ? top1[v[k]] : 0u;
                }
                __builtin_amdgcn_wave_barrier();
                uint32_t pw[kU]; // the 32-bit frontier word of each candidate's top1
#pragma unroll
                for (int k = 0; k < kU; k++) {
                    const uint32_t xx = x[k] & ~fmask;
                    pw[k] = ((t0 + (uint32_t)k * 64 + lane < he) && (!kHubOnly || hub_entry<kHubs>(xx, hub_lim)))
                                ? fword(xx)
                                : 0u;
                }
                if (kPipe && t1 < he) { // wave-uniform; issued after the probes, so waiting on them does not wait on these
#pragma unroll
                    for (int k = 0; k < kU; k++) xn[k] = (t1 + (uint32_t)k * 64 + lane < he) ? top1[vn[k]] : 0u;
                }
                uint32_t fbm = 0u; // bit k: candidate k's top1 is in the frontier
#pragma unroll
                for (int k = 0; k < kU; k++) fbm |= ((pw[k] >> ((x[k] & ~fmask) & 31u)) & 1u) << k;
                // A2: misses of A1 load rest[v] (c1..c3 + degree) and probe c1..c3 together
                uint4 r[kU];
#pragma unroll
                for (int k = 0; k < kU; k++) {
                    const bool a2 = (t0 + (uint32_t)k * 64 + lane < he) && !((fbm >> k) & 1u) && !(x[k] & fmask) &&
                                    (!kHubOnly || hub_entry<kHubs>(x[k] & ~fmask, hub_lim));
                    r[k] = a2 ? rest[v[k]] : make_uint4(0u, 0u, 0u, 0u);
                    acc_s2 += a2;
                }
                uint32_t pbm = 0u; // bits 3k..3k+2: c1..c3 of candidate k in the frontier
#pragma unroll
                for (int k = 0; k < kU; k++) {
                    if (r[k].w != 0u)
                        pbm |= (fbit(r[k].x) | (fbit(r[k].y) << 1) | (fbit(r[k].z) << 2)) << (3 * k);
                }
#pragma unroll
                for (int k = 0; k < kU; k++) {
                    const bool ok = t0 + (uint32_t)k * 64 + lane < he;
                    const bool deg1 = (x[k] & fmask) != 0; // top1 was the row's only entry
                    const uint32_t deg = r[k].w;           // 0 unless A2 ran
                    bool found = false, miss = false;
                    uint32_t par = 0;
                    const uint32_t pb = (pbm >> (3 * k)) & 7u;
                    if (ok) {
                        if ((fbm >> k) & 1u) {
                            found = true;
                            par = x[k] & ~fmask;
                            acc_sc += 1;
                        } else if (deg1) {
                            acc_mu += 1;
                            acc_sc += 1;
                        } else if (kHubOnly && !hub_entry<kHubs>(x[k] & ~fmask, hub_lim)) {
                            acc_mu += 1; // no hub in the row (degree unknown here; the next pull level recounts m_u)
                            acc_sc += 1;
                        } else if (pb) {
                            found = true;
                            par = (pb & 1u) ? r[k].x : (pb & 2u) ? r[k].y : r[k].z;
                            acc_sc += 2u + (uint32_t)__ffs((int)pb) - 1u;
                        } else if (deg <= 4u || (kHubOnly && !(hub_entry<kHubs>(r[k].x, hub_lim) &&
                                                               hub_entry<kHubs>(r[k].y, hub_lim) &&
                                                               hub_entry<kHubs>(r[k].z, hub_lim)))) {
                            acc_mu += deg; // row exhausted (or, hub sweep: its hub prefix is)
                            acc_sc += deg < 4u ? deg : 4u;
                        } else {
                            miss = true;
                            acc_sc += 4;
                        }
                    }
                    if (found) {
                        settle_state(stt, par_out, v[k], probe_id<kHubs>(hub_id, par), nd);
                        atomicOr(&s_nx[wave][(v[k] - vbase) >> 6], 1ull << (v[k] & 63u));
                        acc_nf += 1;
                        if (kMf) acc_mf += deg ? deg : (uint32_t)(row_off[v[k] + 1] - row_off[v[k]]);
                        else if (!kHubOnly) { // single device: non-leaves found, and possible hubs found
                            acc_mf += v[k] < leaf_lo ? 1u : 0u;
                            acc_nh += v[k] < hub_row_lim ? 1u : 0u;
                        }
                    }
                    const u64 mm = __ballot(miss);
                    if (miss) s_miss[wave][nmiss + __popcll(mm & ((1ull << lane) - 1ull))] = v[k];
                    nmiss += (uint32_t)__popcll(mm);
                }
                __builtin_amdgcn_wave_barrier();
                // B: rows longer than 4 with no hit in their first 4 entries walk the rest, 8 per step.  The
                // hub sweep walks them in full 64-row batches only (fewer rows wait for the next round, the
                // half's last round walks the rest): hybrid levels 599 -> 546 us.  The pull levels do not
                // gain from it and their sparse levels lose (profiles/r02r/deferred_phaseB_ab.txt).
                const uint32_t nb = (!kHubOnly || t0 + 64 * kU >= he) ? nmiss : (nmiss & ~63u); // wave-uniform
                for (uint32_t m0 = 0; m0 < nb; m0 += 64) {
                    if (m0 + lane < nb) {
                        const uint32_t vv = s_miss[wave][m0 + lane];
                        const int64_t b = (int64_t)row_off[vv], e = (int64_t)row_off[vv + 1];
                        bool found = false, stop = false;
                        uint32_t par = 0;
                        int64_t j = b + 4;
                        while (!found && !stop && j < e) {
                            const int64_t left = e - j;
                            const uint32_t x0 = col[j];
                            const uint32_t x1 = left > 1 ? col[j + 1] : x0;
                            const uint32_t x2 = left > 2 ? col[j + 2] : x0;
                            const uint32_t x3 = left > 3 ? col[j + 3] : x0;
                            const uint32_t x4 = left > 4 ? col[j + 4] : x0;
                            const uint32_t x5 = left > 5 ? col[j + 5] : x0;
                            const uint32_t x6 = left > 6 ? col[j + 6] : x0;
                            const uint32_t x7 = left > 7 ? col[j + 7] : x0;
                            const uint32_t h0 = fbit(x0), h1 = fbit(x1), h2 = fbit(x2), h3 = fbit(x3);
                            const uint32_t h4 = fbit(x4), h5 = fbit(x5), h6 = fbit(x6), h7 = fbit(x7);
                            const uint32_t hm = h0 | (h1 << 1) | (h2 << 2) | (h3 << 3) | (h4 << 4) | (h5 << 5) |
                                                (h6 << 6) | (h7 << 7);
                            if (hm) {
                                found = true;
                                const int h = __ffs((int)hm) - 1;
                                par = h == 0 ? x0 : h == 1 ? x1 : h == 2 ? x2 : h == 3 ? x3 : h == 4 ? x4 : h == 5 ? x5 : h == 6 ? x6 : x7;
                                j += h + 1;
                            } else {
                                j += left < 8 ? left : 8;
                                // hub sweep: rows are degree-ordered, so past the first non-hub entry no
                                // hub follows
                                if (kHubOnly)
                                    stop = !(hub_entry<kHubs>(x0, hub_lim) && hub_entry<kHubs>(x1, hub_lim) &&
                                             hub_entry<kHubs>(x2, hub_lim) && hub_entry<kHubs>(x3, hub_lim) &&
                                             hub_entry<kHubs>(x4, hub_lim) && hub_entry<kHubs>(x5, hub_lim) &&
                                             hub_entry<kHubs>(x6, hub_lim) && hub_entry<kHubs>(x7, hub_lim));
                            }
                        }
                        acc_sc += (uint32_t)(j - b - 4);
                        acc_wk += (uint32_t)(j - b - 4);
                        acc_rows += 1;
                        if (found) {
                            settle_state(stt, par_out, vv, probe_id<kHubs>(hub_id, par), nd);
                            atomicOr(&s_nx[wave][(vv - vbase) >> 6], 1ull << (vv & 63u));
                            acc_nf += 1;
                            if (kMf) acc_mf += (uint32_t)(e - b);
                            else if (!kHubOnly) {
                                acc_mf += vv < leaf_lo ? 1u : 0u;
                                acc_nh += vv < hub_row_lim ? 1u : 0u;
                            }
                        } else {
                            acc_mu += (uint32_t)(e - b);
                        }
                    }
                }
                if (kHubOnly && nb && nb < nmiss && lane < nmiss - nb) // carry the < 64 left to the front
                    s_miss[wave][lane] = s_miss[wave][nb + lane];
                nmiss -= nb;
                __builtin_amdgcn_wave_barrier();
            }
            __builtin_amdgcn_wave_barrier(); // the next half rewrites the list
        }
        const u64 nxl = s_nx[wave][lane];
        if (wl < nwords) {
            next[wl] = nxl;
            if (nxl) vis[wl] = vwl | nxl;
        }
    }
    // claims field: rows walked (phase B)
    shard_add(cn, acc_nf, acc_mf, acc_sc, acc_rows, acc_mu, 0, acc_s2, acc_wk, acc_nh);
    publish_if_last(cn, pub, seq);
}

#define BFSX_K_BU_PARAMS                                                                                        \
    const OffT *__restrict__ row_off, const uint32_t *__restrict__ col, const uint32_t *__restrict__ top1,      \
        const uint4 *__restrict__ rest, const u64 *__restrict__ front, u64 *__restrict__ next,                  \
        u64 *__restrict__ vis, u64 *__restrict__ stt, uint32_t *__restrict__ par_out, LevelSlot *ring, int level,   \
        int64_t nwords, uint32_t fmask,                                                                        \
        const u64 *__restrict__ hfront, const uint32_t *__restrict__ hub_id, uint32_t hub_lim, uint32_t leaf_lo, \
        PrefixSpec pf, Published *pub, u64 seq, uint32_t hub_row_lim
#define BFSX_K_BU_ARGS                                                                                          \
    row_off, col, top1, rest, front, next, vis, stt, par_out, ring, level, nwords, fmask, hfront, hub_id, hub_lim,     \
        leaf_lo, pf,                                                                                           \
        pub, seq, hub_row_lim

template <class OffT, bool kMf, bool kHubs, int kU, bool kHubOnly, bool kPipe>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(5))) void k_bu(BFSX_K_BU_PARAMS) {
    k_bu_body<OffT, kMf, kHubs, kU, kHubOnly, kPipe>(BFSX_K_BU_ARGS);
}
// Diagnostic only (option bu_force_spill): the partitioned pipelined pull kernel built so that it
// spills to scratch -- the round-2 "spilling pull kernel + concurrent in-process ranks" experiment.
template <class OffT>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(5))) void k_bu_spill(BFSX_K_BU_PARAMS) {
    k_bu_body<OffT, true, false, 4, false, true, true>(BFSX_K_BU_ARGS);
}

// ---- K5s: sparse pull (the tail pull levels) -------------------------------------------------------
// A pull level whose unvisited candidates are few (a scale-26 BFS's third and later pull levels: 10^4-10^5
// candidates in a 2^20-word bitmap) spends k_bu's time in per-group latency chains: a wave takes 64 words
// at a time and runs the whole top1 -> probe -> rest -> probe -> row chain for the handful of candidates
// that group holds, group after group (~3 groups per wave at scale 26: 28 us for 46 K candidates).
// k_bu_sparse gives each wave kSparseWords consecutive words, loads them at once, gathers ALL their
// candidates into one LDS batch list and runs the chain once per 256 candidates.  The discoveries below
// qlim (the next push level's queue: the non-leaves with leaf_skip) are appended to qout directly, wave-
// aggregated, so the push level that follows needs no bitmap -> queue pass; the next-frontier and visited
// words are written back as k_bu writes them, so a pull level may follow as well.  No LDS frontier prefix:
// with this few probes the 8 KiB copy per workgroup would cost more than it saves.
// Counters: nf = every vertex found, mf = the ones queued (= qtail), nhub = the ones below hub_row_lim.
constexpr int kSparseWords = 256;      // bitmap words per wave (16,384 vertices)
constexpr uint32_t kSparseCap = 512;   // candidate batch list per wave: <= 255 carried + one window

template <class OffT>
__global__ __launch_bounds__(kBS) void k_bu_sparse(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                                   const uint32_t *__restrict__ top1, const uint4 *__restrict__ rest,
                                                   const u64 *__restrict__ front, u64 *__restrict__ next,
                                                   u64 *__restrict__ vis, u64 *__restrict__ stt,
                                                   uint32_t *__restrict__ par_out, LevelSlot *ring,
                                                   int level, int64_t nwords, uint32_t fmask, uint32_t hub_row_lim,
                                                   uint32_t qlim, uint32_t *__restrict__ qout, Published *pub,
                                                   u64 seq) {
    LevelSlot *cn = ring + (level + 1) % 3;
    zero_slot(ring, level);
    __shared__ uint32_t s_c[kWaves][kSparseCap];
    __shared__ uint32_t s_miss[kWaves][256];
    __shared__ u64 s_nx[kWaves][kSparseWords];
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const int32_t nd = level + 1;
    constexpr int kC = kSparseWords / 64;
    uint32_t acc_nf = 0, acc_q = 0, acc_sc = 0, acc_mu = 0, acc_rows = 0, acc_s2 = 0, acc_wk = 0, acc_nh = 0;
    const uint32_t *front32 = reinterpret_cast<const uint32_t *>(front);
    auto fbit = [&](uint32_t x) -> uint32_t { return (front32[x >> 5] >> (x & 31u)) & 1u; };
    int64_t wb = 0; // first word of the wave's current range
    // state word + next-frontier bit of a found vertex; wave-uniform queue append of the ones below qlim
    auto settle = [&](bool found, uint32_t v, uint32_t par) {
        if (found) {
            settle_state(stt, par_out, v, par, nd);
            atomicOr(&s_nx[wave][(int64_t)(v >> 6) - wb], 1ull << (v & 63u));
            acc_nf += 1;
            acc_nh += v < hub_row_lim ? 1u : 0u;
        }
        const bool q = found && v < qlim;
        const u64 qm = __ballot(q);
        if (qm) {
            const int leader = __ffsll((long long)qm) - 1;
            u64 base = 0;
            if ((int)lane == leader) base = atomicAdd(&cn->qtail, (u64)__popcll(qm));
            base = __shfl(base, leader);
            if (q) qout[base + __popcll(qm & ((1ull << lane) - 1ull))] = v;
            acc_q += q ? 1u : 0u;
        }
    };
    // one round over the first n (<= 256) ids of the wave's batch list: A1 (top1), A2 (rest), B (row walk)
    auto run_round = [&](uint32_t n) {
        uint32_t v[4], x[4];
        bool ok[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t i = (uint32_t)k * 64 + lane;
            ok[k] = i < n;
            v[k] = ok[k] ? s_c[wave][i] : 0u;
            x[k] = ok[k] ? top1[v[k]] : 0u;
        }
        uint32_t fbm = 0u;
#pragma unroll
        for (int k = 0; k < 4; k++) fbm |= (ok[k] ? fbit(x[k] & ~fmask) : 0u) << k;
        uint4 r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool a2 = ok[k] && !((fbm >> k) & 1u) && !(x[k] & fmask);
            r[k] = a2 ? rest[v[k]] : make_uint4(0u, 0u, 0u, 0u);
            acc_s2 += a2;
        }
        uint32_t pbm = 0u;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (r[k].w != 0u) pbm |= (fbit(r[k].x) | (fbit(r[k].y) << 1) | (fbit(r[k].z) << 2)) << (3 * k);
        uint32_t nmiss = 0; // wave-uniform
#pragma unroll
        for (int k = 0; k < 4; k++) {
            bool found = false, miss = false;
            uint32_t par = 0;
            const uint32_t pb = (pbm >> (3 * k)) & 7u, deg = r[k].w;
            if (ok[k]) {
                if ((fbm >> k) & 1u) {
                    found = true;
                    par = x[k] & ~fmask;
                    acc_sc += 1;
                } else if (x[k] & fmask) { // top1 was the row's only entry
                    acc_mu += 1;
                    acc_sc += 1;
                } else if (pb) {
                    found = true;
                    par = (pb & 1u) ? r[k].x : (pb & 2u) ? r[k].y : r[k].z;
                    acc_sc += 2u + (uint32_t)__ffs((int)pb) - 1u;
                } else if (deg <= 4u) {
                    acc_mu += deg;
                    acc_sc += deg;
                } else {
                    miss = true;
                    acc_sc += 4;
                }
            }
            settle(found, v[k], par);
            const u64 mm = __ballot(miss);
            if (miss) s_miss[wave][nmiss + __popcll(mm & ((1ull << lane) - 1ull))] = v[k];
            nmiss += (uint32_t)__popcll(mm);
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t m0 = 0; m0 < nmiss; m0 += 64) {
            bool found = false;
            uint32_t par = 0, vv = 0;
            if (m0 + lane < nmiss) {
                vv = s_miss[wave][m0 + lane];
                const int64_t b = (int64_t)row_off[vv], e = (int64_t)row_off[vv + 1];
                int64_t j = b + 4;
                while (!found && j < e) {
                    const int64_t left = e - j;
                    uint32_t xs[8];
#pragma unroll
                    for (int t = 0; t < 8; t++) xs[t] = left > t ? col[j + t] : col[j];
                    uint32_t hm = 0u;
#pragma unroll
                    for (int t = 0; t < 8; t++) hm |= fbit(xs[t]) << t;
                    if (hm) {
                        found = true;
                        const int h = __ffs((int)hm) - 1;
                        par = xs[h];
                        j += h + 1;
                    } else {
                        j += left < 8 ? left : 8;
                    }
                }
                acc_sc += (uint32_t)(j - b - 4);
                acc_wk += (uint32_t)(j - b - 4);
                acc_rows += 1;
                if (!found) acc_mu += (uint32_t)(e - b);
            }
            settle(found, vv, par);
        }
        __builtin_amdgcn_wave_barrier();
    };
    const int64_t wstride = (int64_t)gridDim.x * kWaves * kSparseWords;
    for (wb = ((int64_t)blockIdx.x * kWaves + wave) * kSparseWords; wb < nwords; wb += wstride) {
        u64 vw[kC];
#pragma unroll
        for (int c = 0; c < kC; c++) {
            const int64_t wl = wb + c * 64 + lane;
            vw[c] = wl < nwords ? vis[wl] : ~0ull;
            s_nx[wave][c * 64 + lane] = 0ull;
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t n = 0; // wave-uniform: ids waiting in the batch list
#pragma unroll
        for (int c = 0; c < kC; c++) {
            const u64 unv = ~vw[c];
            const uint32_t cnt = (uint32_t)__popcll(unv);
            const uint32_t incl = wave_incl_scan(cnt);
            const uint32_t total = __shfl(incl, 63), excl = incl - cnt;
            const uint32_t base_id = (uint32_t)((wb + c * 64 + lane) * 64);
            for (uint32_t w0 = 0; w0 < total;) { // windows of the chunk's candidates that fit the list
                const uint32_t take = min(total - w0, kSparseCap - n);
                u64 bits = unv;
                uint32_t rk = excl;
                while (bits) {
                    if (rk >= w0 && rk < w0 + take)
                        s_c[wave][n + (rk - w0)] = base_id + (uint32_t)(__ffsll((long long)bits) - 1);
                    rk++;
                    bits &= bits - 1ull;
                }
                __builtin_amdgcn_wave_barrier();
                n += take;
                w0 += take;
                while (n >= 256) { // full rounds, the rest moves to the front of the list
                    run_round(256);
                    const uint32_t left = n - 256;
                    uint32_t keep[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t i = (uint32_t)k * 64 + lane;
                        keep[k] = i < left ? s_c[wave][256 + i] : 0u;
                    }
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t i = (uint32_t)k * 64 + lane;
                        if (i < left) s_c[wave][i] = keep[k];
                    }
                    __builtin_amdgcn_wave_barrier();
                    n = left;
                }
            }
        }
        if (n) run_round(n);
#pragma unroll
        for (int c = 0; c < kC; c++) {
            const int64_t wl = wb + c * 64 + lane;
            const u64 nx = s_nx[wave][c * 64 + lane];
            if (wl < nwords) {
                next[wl] = nx;
                if (nx) vis[wl] = vw[c] | nx;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // claims field: rows walked (phase B); mf field: discoveries queued
    shard_add(cn, acc_nf, acc_q, acc_sc, acc_rows, acc_mu, 0, acc_s2, acc_wk, acc_nh);
    publish_if_last(cn, pub, seq);
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

// Frontier of a top-down level as a bitmap without one atomic per vertex: the visited bitmap after
// the level XOR its snapshot from before the level (bits are only ever set).
__global__ __launch_bounds__(kBS) void k_new_bits(const u64 *__restrict__ vis, int64_t nwords, u64 *__restrict__ snap) {
    for (int64_t w = (int64_t)blockIdx.x * kBS + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBS)
        snap[w] ^= vis[w];
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

// ---- pull-level records (single device, BfsWorkspace::par) ----------------------------------------
// At most kMaxRec records per BFS; a BFS with more pull levels folds its records into st mid-BFS (k_resolve).
constexpr int kMaxRec = 32;
struct RecSet {
    const u64 *bm[kMaxRec];
    int32_t nd[kMaxRec]; // distance of the record's vertices (its level + 1)
    int n;
};

// state of internal vertex i: st[i], unless a record holds i (its parent is then par[i]).  Lanes of consecutive
// i share their record words (one broadcast load per wave and record).
__device__ __forceinline__ u64 rec_state(const u64 *__restrict__ stt, const uint32_t *__restrict__ par,
                                         const RecSet &rs, int64_t i) {
    for (int r = 0; r < rs.n; r++)
        if ((rs.bm[r][i >> 6] >> (i & 63)) & 1ull) return pack_state(par[i], rs.nd[r]);
    return stt[i];
}

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
__global__ __launch_bounds__(kBS) void k_resolve(RecSet rs, int64_t nwords, const uint32_t *__restrict__ par,
                                                 u64 *__restrict__ stt) {
    const unsigned lane = lane_id();
    const int64_t nwaves = ((int64_t)gridDim.x * kBS) >> 6;
    for (int64_t w = ((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6; w < nwords; w += nwaves) {
        for (int r = 0; r < rs.n; r++) {
            const u64 m = rs.bm[r][w];
            if (m == 0ull) continue; // wave-uniform
            if ((m >> lane) & 1ull) {
                const int64_t v = w * 64 + lane;
                stt[v] = pack_state(par[v], rs.nd[r]);
            }
        }
    }
}

// Result extraction (outside the timed region): internal state (+ the pending records) -> one 8-byte word per
// ORIGINAL id, out[o] = parent_original << 32 | dist (one scattered store per vertex where separate dist and
// parent arrays took two), or dist only.  kRelabel: internal local row i is original vertex inv[lo + i] (a
// partition's relabel keeps it inside the rank's range [lo, lo + n)); parents are global internal ids and map
// back through the whole inv.  Isolated vertices (`dead`; half the ids of a scale-26 Kronecker graph) keep
// the unreached word the buffer was filled with once, except keep0 / keep1 (this BFS's source, the last one
// written that was isolated), so only the other half costs a scattered store.
template <bool kRelabel>
__global__ __launch_bounds__(kBS) void k_unpack(const u64 *__restrict__ stt, const uint32_t *__restrict__ par,
                                                RecSet rs, const uint32_t *__restrict__ inv, int64_t lo, int64_t n,
                                                const u64 *__restrict__ dead, int64_t keep0, int64_t keep1,
                                                u64 *__restrict__ out, int32_t *__restrict__ dist_only) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        if (((dead[i >> 6] >> (i & 63)) & 1ull) && i != keep0 && i != keep1) continue;
        const u64 s = rec_state(stt, par, rs, i);
        const uint32_t o = kRelabel ? (uint32_t)((int64_t)inv[lo + i] - lo) : (uint32_t)i;
        if (dist_only) {
            dist_only[o] = (int32_t)(uint32_t)s;
        } else {
            const uint32_t p = (uint32_t)(s >> 32);
            const uint32_t po = (!kRelabel || p == 0xFFFFFFFFu) ? p : inv[p];
            out[o] = ((u64)po << 32) | (uint32_t)s;
        }
    }
}

// The result in ORIGINAL id order (a relabelled graph), in two passes (round 5; round 4 ran one gather of
// 0.685 ms per scale-26 result whose every entry chained perm -> dead word -> one record word per pull level ->
// st or par -> inv, each a dependent gather):
//   phase 1, k_resolve_all, INTERNAL id order: one wave per 64-vertex bitmap word, lane = bit.  The word's record
//     words are broadcast loads issued together; par, st and tmp are coalesced.  A record vertex's state
//     (par[i], the record's distance) is stored into st, so st ends resolved (parents in internal ids: the
//     Graph500 kernel-2 result on the device, which the validator and m_comp read), and with tmp every live i
//     gets tmp[i] = parent_original << 32 | dist, the parent mapped through inv here, where the parents of
//     consecutive vertices are the same few hubs (inv lines stay cached).  Only the words below iso_lo (the
//     isolated tail) and the source's word are visited.
//   phase 2, k_unpack_gather: thread o reads perm[o] and copies tmp[perm[o]] into out[o] -- whole-line writes,
//     near-sequential reads (the relabel keeps original order inside a degree class) -- or writes the unreached
//     word without a load for an id of the isolated tail.
__global__ __launch_bounds__(kBS) void k_resolve_all(RecSet rs, int64_t nwords_live, int64_t src_word,
                                                     const uint32_t *__restrict__ par, u64 *__restrict__ stt,
                                                     const uint32_t *__restrict__ inv, u64 *__restrict__ tmp,
                                                     int64_t n) {
    const unsigned lane = lane_id();
    const int64_t nwaves = ((int64_t)gridDim.x * kBS) >> 6;
    const int64_t nit = nwords_live + (src_word >= nwords_live ? 1 : 0);
    for (int64_t it = ((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6; it < nit; it += nwaves) {
        const int64_t w = it < nwords_live ? it : src_word;
        int hit = -1;
#pragma unroll 4
        for (int r = 0; r < rs.n; r++) // records are disjoint: the loads are independent
            if ((rs.bm[r][w] >> lane) & 1ull) hit = r;
        const int64_t v = w * 64 + lane;
        if (v >= n) continue;
        u64 s;
        if (hit >= 0) {
            s = pack_state(par[v], rs.nd[hit]);
            stt[v] = s;
        } else {
            s = stt[v];
        }
        if (tmp) {
            const uint32_t p = (uint32_t)(s >> 32);
            tmp[v] = ((u64)(p == 0xFFFFFFFFu ? p : inv[p]) << 32) | (uint32_t)s;
        }
    }
}

__global__ __launch_bounds__(kBS) void k_unpack_gather(const u64 *__restrict__ tmp, const uint32_t *__restrict__ perm,
                                                       int64_t n, int64_t iso_lo, int64_t src, u64 *__restrict__ out,
                                                       int32_t *__restrict__ dist_only) {
    for (int64_t o = (int64_t)blockIdx.x * kBS + threadIdx.x; o < n; o += (int64_t)gridDim.x * kBS) {
        const int64_t i = (int64_t)perm[o];
        const u64 s = (i >= iso_lo && i != src) ? kUnreached : tmp[i];
        if (dist_only) dist_only[o] = (int32_t)(uint32_t)s;
        else out[o] = s;
    }
}

// Dead mask: vertices that no BFS can reach from elsewhere (degree 0, or a self-loop only) plus the
// padding bits of the last word.  The visited bitmap starts as this mask, so bottom-up waves skip
// groups that hold only visited/isolated vertices with one uniform branch.
__global__ __launch_bounds__(kBS) void k_dead_mask(const int64_t *__restrict__ row_off,
                                                   const uint32_t *__restrict__ col, int64_t nv, int64_t nwords,
                                                   uint32_t lo, u64 *__restrict__ dead) {
    const unsigned lane = lane_id();
    for (int64_t w = ((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6; w < nwords;
         w += ((int64_t)gridDim.x * kBS) >> 6) {
        const int64_t v = w * 64 + lane; // local row id; adjacency entries are global ids
        bool d = true;
        if (v < nv) {
            const int64_t b = row_off[v], e = row_off[v + 1];
            d = (e == b) || (e == b + 1 && col[b] == (uint32_t)(v + lo));
        }
        const u64 m = __ballot(d);
        if (lane == 0) dead[w] = m;
    }
}

// top1[v] = first (highest-degree) neighbour, flagged with `flag` when it is the row's only entry.
__global__ __launch_bounds__(kBS) void k_top1(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ col,
                                              int64_t nv, uint32_t flag, uint32_t *__restrict__ top1) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS) {
        const int64_t b = row_off[v], e = row_off[v + 1];
        top1[v] = (e > b) ? (col[b] | (e == b + 1 ? flag : 0u)) : (uint32_t)v;
    }
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

// rest[v] = {c1, c2, c3, deg} of row v (see k_bu); rows shorter than 4 repeat their last entry
// (a degree-1 row repeats top1: probing it again is harmless).
__global__ __launch_bounds__(kBS) void k_rest(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ col,
                                              int64_t nv, uint4 *__restrict__ rest) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS) {
        const int64_t b = row_off[v], d = row_off[v + 1] - b;
        uint4 r = make_uint4(0u, 0u, 0u, 0u);
        if (d > 0) {
            r.x = col[b + (d > 1 ? 1 : d - 1)];
            r.y = col[b + (d > 2 ? 2 : d - 1)];
            r.z = col[b + (d > 3 ? 3 : d - 1)];
            r.w = d >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)d;
        }
        rest[v] = r;
    }
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
// Hub selection: sort keys ~degree (ascending = degree descending, ties by id: the sort is stable).
__global__ __launch_bounds__(kBS) void k_hub_keys(const uint32_t *__restrict__ deg, int64_t n,
                                                  uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < n; v += (int64_t)gridDim.x * kBS) {
        keys[v] = ~deg[v];
        ids[v] = (uint32_t)v;
    }
}
__global__ __launch_bounds__(kBS) void k_count_le(const uint32_t *__restrict__ keys, int64_t n, uint32_t x, u64 *out) {
    u64 c = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) c += keys[i] <= x;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(out, c);
}
__global__ __launch_bounds__(kBS) void k_hub_index(const uint32_t *__restrict__ hub_id, int64_t k,
                                                   uint32_t *__restrict__ hidx) {
    for (int64_t h = (int64_t)blockIdx.x * kBS + threadIdx.x; h < k; h += (int64_t)gridDim.x * kBS)
        hidx[hub_id[h]] = (uint32_t)h;
}
// out[i] = hub-encoded in[i] (bits in `keep` pass through: the top1 degree-1 flag); in == out allowed
__global__ __launch_bounds__(kBS) void k_hub_encode(const uint32_t *in, int64_t n, const uint32_t *__restrict__ hidx,
                                                    uint32_t keep, uint32_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        const uint32_t x = in[i];
        const uint32_t h = hidx[x & ~keep];
        out[i] = (h != 0xFFFFFFFFu ? (kHubBit | h) : (x & ~keep)) | (x & keep);
    }
}
// Before a bottom-up level: hfront bit h = frontier bit of hub h (one lane per hub, a ballot per word).
__global__ __launch_bounds__(kBS) void k_hub_gather(const uint32_t *__restrict__ hub_id, int64_t k,
                                                    const u64 *__restrict__ front, u64 *__restrict__ hfront) {
    for (int64_t h0 = (int64_t)blockIdx.x * kBS; h0 < k; h0 += (int64_t)gridDim.x * kBS) {
        const int64_t h = h0 + threadIdx.x;
        bool bit = false;
        if (h < k) {
            const uint32_t v = hub_id[h];
            bit = (front[v >> 6] >> (v & 63u)) & 1ull;
        }
        const u64 w = __ballot(bit);
        if ((threadIdx.x & 63u) == 0 && h < k) hfront[h >> 6] = w;
    }
}

__global__ __launch_bounds__(kBS) void k_off32(const int64_t *__restrict__ row_off, int64_t n,
                                               uint32_t *__restrict__ off32) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS)
        off32[i] = (uint32_t)row_off[i];
}

__global__ __launch_bounds__(kBS) void k_popc(const u64 *__restrict__ bm, int64_t nwords, u64 *out) {
    u64 c = 0;
    for (int64_t w = (int64_t)blockIdx.x * kBS + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBS)
        c += (u64)__popcll(bm[w]);
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(out, c);
}

// m_comp (Graph500 TEPS numerator) and reached count, outside the timed region.
__global__ __launch_bounds__(kBS) void k_mcomp(const u64 *__restrict__ stt, const uint32_t *__restrict__ tcnt,
                                               int64_t nv, u64 *out) {
    u64 m = 0, r = 0;
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS) {
        if ((int32_t)(uint32_t)stt[v] != INT32_MAX) {
            m += tcnt[v];
            r += 1;
        }
    }
    m = wave_sum(m);
    r = wave_sum(r);
    if (lane_id() == 0 && (m | r)) {
        atomicAdd(out, m);
        atomicAdd(out + 1, r);
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

unsigned clamp_grid(int64_t blocks, unsigned cap) {
    if (blocks < 1) blocks = 1;
    return (unsigned)std::min<int64_t>(blocks, cap);
}

// Hub probe domain of k_bu: the hub_k highest-degree vertices of the whole graph (option "hub_bits":
// auto = the power of two >= n/1024 (measured: 2^16..2^19 hubs at scale 26 within noise, more hubs slower
// as the per-level gather grows); off for ids >= 2^30 or n < 2^16).  On a partition every rank ranks the
// global degrees and gathers the hubs' bits from the all-gathered global frontier bitmap.
int hub_setup(bfsx_graph *g, BfsWorkspace *ws) {
    const int hb = g->ctx->opt.hub_bits;
    const bool part = g->nranks > 1;
    if (hb == 0 || g->nv_global < 64) return BFSX_OK;
    if (g->d_perm) { // relabelled: hubs = the first k ids (the k highest degrees), nothing to build
        if (part) return BFSX_OK; // a partition's ranges each start with their hubs; no hybrid levels there
        int64_t k = 64;
        if (hb < 0) {
            if (g->nv < ((int64_t)1 << 16)) return BFSX_OK;
            while (k * 1024 < g->nv) k *= 2;
        } else {
            k = (int64_t)1 << hb;
        }
        ws->hub_lim = (uint32_t)std::min<int64_t>(k, g->nv);
        return BFSX_OK;
    }
    if (g->nv_global > ((int64_t)1 << 30)) return BFSX_OK;
    Comm *cm = g->ctx->comm.get();
    // a partition ranks the hubs by GLOBAL degree: the degrees are all-gathered over the communicator
    // (collective -- every rank reaches this at its first BFS); a partition driven without one (the
    // Python level-primitive driver) stays off
    if (part && (!cm || cm->nranks != g->nranks || cm->rank != g->rank)) return BFSX_OK;
    int64_t k;
    if (hb < 0) {
        if (g->nv_global < ((int64_t)1 << 16)) return BFSX_OK;
        k = 64;
        while (k * 1024 < g->nv_global) k *= 2;
    } else {
        k = (int64_t)1 << hb;
    }
    const int64_t ng = part ? g->chunk * g->nranks : g->nv; // ids ranked (a partition: padded slices)
    k = std::min<int64_t>(k, ng);
    hipStream_t st = g->ctx->stream;
    const size_t nv = (size_t)g->nv, nr = (size_t)ng;
    struct Tmp {
        void *p = nullptr;
        ~Tmp() {
            if (p) (void)hipFree(p);
        }
    } degs, slice, keys, keys2, ids, ids2, hidx, sort_tmp;
    BFSX_HIP_TRY(hipMalloc(&degs.p, nr * sizeof(uint32_t)));
    const unsigned gfill = clamp_grid(((int64_t)nr + kBS - 1) / kBS, 8192);
    if (part) {
        BFSX_HIP_TRY(hipMalloc(&slice.p, (size_t)g->chunk * sizeof(uint32_t)));
        hipLaunchKernelGGL(k_slice_degrees, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, nullptr, g->nv, g->chunk,
                           (uint32_t *)slice.p);
        BFSX_LAUNCHED(st);
        if (int e = cm->allgather((const u64 *)slice.p, g->chunk / 2, (u64 *)degs.p, st)) return e;
    } else {
        hipLaunchKernelGGL(k_slice_degrees, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, nullptr, g->nv, g->nv,
                           (uint32_t *)degs.p);
        BFSX_LAUNCHED(st);
    }
    // the encoded adjacency copy (4 B per entry) and the ranking temporaries must leave half of the free
    // device memory untouched (scale 30 on one device: the graph alone is ~150 GB), else stay off (a
    // local decision: a rank's hub domain only changes how ITS pull kernel probes)
    size_t mfree = 0, mtotal = 0;
    BFSX_HIP_TRY(hipMemGetInfo(&mfree, &mtotal));
    if ((size_t)g->nnz * 4 + nr * 20 > mfree / 2) return BFSX_OK;
    // from here on an allocation failure (e.g. ranks of an in-process group racing for one device's
    // memory) leaves the domain off instead of failing the BFS: it is an optimisation of the pull
    // kernel only, and top1 is encoded last, after every allocation has succeeded
#define HUB_ALLOC(call)                                                                          \
    do {                                                                                         \
        const hipError_t h_ = (call);                                                            \
        if (h_ == hipErrorOutOfMemory) {                                                         \
            (void)hipGetLastError();                                                             \
            for (void **p_ : {(void **)&ws->hub_id, (void **)&ws->colh, (void **)&ws->hfront})   \
                if (*p_) {                                                                       \
                    (void)hipFree(*p_);                                                          \
                    *p_ = nullptr;                                                               \
                }                                                                                \
            return BFSX_OK;                                                                      \
        }                                                                                        \
        BFSX_HIP_TRY(h_);                                                                        \
    } while (0)
    HUB_ALLOC(hipMalloc(&keys.p, nr * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&keys2.p, nr * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&ids.p, nr * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&ids2.p, nr * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_hub_keys, dim3(gfill), dim3(kBS), 0, st, (const uint32_t *)degs.p, ng, (uint32_t *)keys.p,
                       (uint32_t *)ids.p);
    BFSX_LAUNCHED(st);
    size_t tb = 0;
    BFSX_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, (uint32_t *)keys.p, (uint32_t *)keys2.p, (uint32_t *)ids.p,
                                           (uint32_t *)ids2.p, nr, 0, 32, st));
    HUB_ALLOC(hipMalloc(&sort_tmp.p, std::max<size_t>(tb, 16)));
    BFSX_HIP_TRY(rocprim::radix_sort_pairs(sort_tmp.p, tb, (uint32_t *)keys.p, (uint32_t *)keys2.p, (uint32_t *)ids.p,
                                           (uint32_t *)ids2.p, nr, 0, 32, st));
    // the hub set is closed under degree ties: every vertex of degree >= the k-th largest degree (so a
    // kernel tells a hub by its degree alone, and degree-ordered rows hold their hubs as a prefix)
    uint32_t kth = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&kth, (uint32_t *)keys2.p + (k - 1), sizeof(kth), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, sizeof(u64), st));
    hipLaunchKernelGGL(k_count_le, dim3(gfill), dim3(kBS), 0, st, (const uint32_t *)keys2.p, ng, kth, ws->d_red);
    BFSX_LAUNCHED(st);
    u64 keff = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&keff, ws->d_red, sizeof(keff), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    k = (int64_t)keff;
    HUB_ALLOC(hipMalloc(&ws->hub_id, (size_t)k * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&hidx.p, nr * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&ws->colh, (size_t)std::max<int64_t>(g->nnz, 1) * sizeof(uint32_t)));
    HUB_ALLOC(hipMalloc(&ws->hfront, (size_t)((k + 63) / 64) * sizeof(u64)));
#undef HUB_ALLOC
    ws->hub_tdeg = ~kth;
    BFSX_HIP_TRY(hipMemcpyAsync(ws->hub_id, ids2.p, (size_t)k * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    BFSX_HIP_TRY(hipMemsetAsync(hidx.p, 0xFF, nr * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_hub_index, dim3(clamp_grid((k + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st, ws->hub_id, k,
                       (uint32_t *)hidx.p);
    BFSX_LAUNCHED(st);
    hipLaunchKernelGGL(k_hub_encode, dim3(clamp_grid((g->nnz + kBS - 1) / kBS, 65536)), dim3(kBS), 0, st, g->d_col,
                       g->nnz, (const uint32_t *)hidx.p, 0u, ws->colh);
    BFSX_LAUNCHED(st);
    hipLaunchKernelGGL(k_hub_encode, dim3(clamp_grid(((int64_t)nv + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                       ws->top1, g->nv, (const uint32_t *)hidx.p, ws->top1_flag, ws->top1);
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipStreamSynchronize(st)); // the temporaries are freed on return
    ws->hub_k = k;
    return BFSX_OK;
}

int ws_alloc(bfsx_graph *g) {
    if (g->ws) return BFSX_OK;
    auto *ws = new BfsWorkspace();
    g->ws = ws;
    hipStream_t st = g->ctx->stream;
    ws->nv = g->nv;
    // a partitioned graph pads every rank's slice to chunk/64 words so that frontier slices
    // all-gather into one global bitmap
    ws->nwords = g->chunk / 64;
    const size_t nv = (size_t)std::max<int64_t>(g->nv, 1);
    BFSX_HIP_TRY(hipMalloc(&ws->st, nv * sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->par, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->vis, ws->nwords * sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->front, ws->nwords * sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->next, ws->nwords * sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->dead, ws->nwords * sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->qa, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->qb, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->hubs, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->top1, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->ring, 3 * sizeof(LevelSlot)));
    BFSX_HIP_TRY(hipHostMalloc(&ws->h_slot, sizeof(LevelSlot), hipHostMallocDefault));
    BFSX_HIP_TRY(hipHostMalloc(&ws->h_pub, sizeof(Published), hipHostMallocMapped | hipHostMallocCoherent));
    BFSX_HIP_TRY(hipHostGetDevicePointer((void **)&ws->d_pub, ws->h_pub, 0));
    ws->h_pub->seq = 0;
    BFSX_HIP_TRY(hipHostMalloc(&ws->h_err, sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent));
    BFSX_HIP_TRY(hipHostGetDevicePointer((void **)&ws->d_err, ws->h_err, 0));
    *ws->h_err = 0;
    BFSX_HIP_TRY(hipMalloc(&ws->d_cursor, sizeof(u64)));
    BFSX_HIP_TRY(hipMalloc(&ws->d_red, 3 * sizeof(u64)));
    BFSX_HIP_TRY(hipEventCreate(&ws->ev_start));
    BFSX_HIP_TRY(hipEventCreate(&ws->ev_end));
    const unsigned gfill = clamp_grid(((int64_t)nv + kBS - 1) / kBS, 8192);
    hipLaunchKernelGGL(k_fill64, dim3(gfill), dim3(kBS), 0, st, ws->st, (int64_t)nv, kUnreached);
    BFSX_LAUNCHED(st);
    // every offset (incl. row_off[nv] = nnz) fits in uint32; "offset_bits=64" keeps the int64 path (tests)
    if (g->nnz < (int64_t)0xFFFFFFFFll && g->ctx->opt.offset_bits != 64) {
        BFSX_HIP_TRY(hipMalloc(&ws->off32, (nv + 1) * sizeof(uint32_t)));
        hipLaunchKernelGGL(k_off32, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, g->nv + 1, ws->off32);
        BFSX_LAUNCHED(st);
    }
    ws->top1_flag = (g->nv_global <= ((int64_t)1 << 31)) ? kDeg1 : 0u;
    hipLaunchKernelGGL(k_top1, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, g->d_col, g->nv, ws->top1_flag, ws->top1);
    BFSX_LAUNCHED(st);
    if (int e = hub_setup(g, ws)) return e;
    BFSX_HIP_TRY(hipMalloc(&ws->rest, nv * sizeof(uint4)));
    hipLaunchKernelGGL(k_rest, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, ws->hub_k > 0 ? ws->colh : g->d_col,
                       g->nv, ws->rest);
    BFSX_LAUNCHED(st);
    hipLaunchKernelGGL(k_dead_mask, dim3(clamp_grid((ws->nwords * 64 + kBS - 1) / kBS, 4096)), dim3(kBS), 0, st,
                       g->d_row_off, g->d_col, g->nv, ws->nwords, (uint32_t)g->v_lo, ws->dead);
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, 3 * sizeof(u64), st));
    hipLaunchKernelGGL(k_popc, dim3(clamp_grid((ws->nwords + kBS - 1) / kBS, 2048)), dim3(kBS), 0, st, ws->dead,
                       ws->nwords, ws->d_red);
    BFSX_LAUNCHED(st);
    hipLaunchKernelGGL(k_rows_above, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, g->nv, (int64_t)1, ws->d_red + 1);
    BFSX_LAUNCHED(st);
    hipLaunchKernelGGL(k_rows_above, dim3(gfill), dim3(kBS), 0, st, g->d_row_off, g->nv, (int64_t)0, ws->d_red + 2);
    BFSX_LAUNCHED(st);
    u64 nd[3] = {0, 0, 0};
    BFSX_HIP_TRY(hipMemcpyAsync(nd, ws->d_red, sizeof(nd), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    ws->n_dead = (int64_t)nd[0] - (ws->nwords * 64 - g->nv); // minus padding bits
    ws->leaf_lo = (int64_t)nd[1];
    ws->iso_lo = (int64_t)nd[2];
    return BFSX_OK;
}

// The single-device "partition": every row local, queue entries checked against nv (id_ok).
Part single_part(const bfsx_graph *g, const BfsWorkspace *ws) {
    Part p{};
    p.nrows = (uint32_t)g->nv;
    p.err = ws->d_err;
    return p;
}

// After a BFS: fail if a queue consumer met an out-of-range id (the word is cleared for the next BFS).
int check_queue_guard(BfsWorkspace *ws) {
    std::atomic_thread_fence(std::memory_order_acquire);
    const u64 e = *reinterpret_cast<volatile u64 *>(ws->h_err);
    if (!e) return BFSX_OK;
    *reinterpret_cast<volatile u64 *>(ws->h_err) = 0;
    return fail(BFSX_E_HIP, "internal error: a frontier-queue consumer read vertex id " +
                                std::to_string((uint32_t)e) + ", outside the rows of this graph (stale queue entry)");
}

// ws->heavy_rows for the current persist_dmax option: does any row exceed it (K3p's heavy instantiation)?  One
// pass over the row offsets, outside any timed region.
int ensure_heavy_rows(bfsx_graph *g, BfsWorkspace *ws) {
    const int64_t thr = g->ctx->opt.persist_dmax;
    if (ws->heavy_thr == thr) return BFSX_OK;
    hipStream_t st = g->ctx->stream;
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, sizeof(u64), st));
    hipLaunchKernelGGL(k_rows_above, dim3(clamp_grid((g->nv + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st, g->d_row_off,
                       g->nv, thr, ws->d_red);
    BFSX_LAUNCHED(st);
    u64 lim = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&lim, ws->d_red, sizeof(lim), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    ws->heavy_rows = lim > 0;
    ws->heavy_thr = thr;
    return BFSX_OK;
}

// ws->hub_row_lim for the current hub_degree option (one pass over the row offsets, outside any timed region).
int ensure_hub_row_lim(bfsx_graph *g, BfsWorkspace *ws) {
    const uint32_t hd = g->ctx->opt.hub_degree;
    if (ws->hub_row_lim >= 0 && ws->hub_row_deg == hd) return BFSX_OK;
    hipStream_t st = g->ctx->stream;
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, sizeof(u64), st));
    hipLaunchKernelGGL(k_rows_above, dim3(clamp_grid((g->nv + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st, g->d_row_off,
                       g->nv, (int64_t)hd, ws->d_red);
    BFSX_LAUNCHED(st);
    u64 lim = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&lim, ws->d_red, sizeof(lim), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    ws->hub_row_lim = (int64_t)lim;
    ws->hub_row_deg = hd;
    return BFSX_OK;
}

// ---- launch helpers: one per traversal kernel, dispatching on the row-offset width -------------
HubSet hub_set(const BfsWorkspace *ws) {
    return HubSet{ws->hub_k > 0 ? ws->hub_tdeg : 0xFFFFFFFFu, ws->hub_lim};
}
bool has_hubs(const BfsWorkspace *ws) { return ws->hub_k > 0 || ws->hub_lim > 0; }

// dmax: largest degree in the frontier (< 0: unknown) -- the hub bin is skipped when no vertex exceeds
// the hub degree
// skip_hubs (hybrid level): frontier vertices of the hub domain are left to the bottom-up hub sweep.
// pub != null: the last kernel launched publishes the level's counters (seq) from its last workgroup
// plog (single device): the level's winners go to the push log as vertex | parent << 32 at their queue positions
// instead of a packed-state store (BfsWorkspace::plog)
template <bool kDist>
int launch_td(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t mf, int64_t dmax, int level, const Part &pt,
              bool skip_hubs = false, Published *pub = nullptr, u64 seq = 0, uint32_t *par = nullptr,
              u64 *plog = nullptr) {
    hipStream_t st = g->ctx->stream;
    const HubSet hs = hub_set(ws);
    const HubSet skip = skip_hubs ? hs : HubSet{0xFFFFFFFFu, 0u};
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    const uint32_t hub_deg = g->ctx->opt.hub_degree;
    int gsz = 16;
    while (gsz < kBS && (int64_t)gsz * 2 * g->ctx->num_cus < nf) gsz *= 2;
    const dim3 grid(clamp_grid((nf + gsz - 1) / gsz, cap));
    // hubs: sized by the frontier's degree sum when known (mf < 0: after a bottom-up level)
    const bool hubs = dmax >= 0 ? dmax > (int64_t)hub_deg : (mf < 0 || mf > (int64_t)hub_deg);
    const dim3 gh(mf < 0 ? cap : clamp_grid((mf + kBS * kItems - 1) / (kBS * kItems), cap));
    // slot mode: only the level's last push kernel writes the slot headers
    Part pt0 = pt;
    if (hubs) pt0.slot_arrive = nullptr;
    if (ws->off32) {
        hipLaunchKernelGGL((k_td<kDist, uint32_t>), grid, dim3(kBS), 0, st, ws->off32, g->d_col, ws->qa, (uint32_t)nf,
                           ws->qb, ws->vis, ws->st, par, ws->ring, level, hub_deg, ws->hubs, pt0, gsz, hs, skip,
                           hubs ? nullptr : pub, seq, plog);
        BFSX_LAUNCHED(st);
        if (hubs) {
            hipLaunchKernelGGL((k_td_hubs<kDist, uint32_t>), gh, dim3(kBS), 0, st, ws->off32, g->d_col, ws->hubs,
                               ws->qb, ws->vis, ws->st, par, ws->ring, level, pt, hs, pub, seq, plog);
            BFSX_LAUNCHED(st);
        }
    } else {
        hipLaunchKernelGGL((k_td<kDist, int64_t>), grid, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->qa,
                           (uint32_t)nf, ws->qb, ws->vis, ws->st, par, ws->ring, level, hub_deg, ws->hubs, pt0, gsz, hs, skip,
                           hubs ? nullptr : pub, seq, plog);
        BFSX_LAUNCHED(st);
        if (hubs) {
            hipLaunchKernelGGL((k_td_hubs<kDist, int64_t>), gh, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->hubs,
                               ws->qb, ws->vis, ws->st, par, ws->ring, level, pt, hs, pub, seq, plog);
            BFSX_LAUNCHED(st);
        }
    }
    return BFSX_OK;
}

// Frontier ids whose bits the pull kernels read from an LDS copy: the highest-degree ids of a
// relabelled graph -- on one device the first 2^16 ids, on a partition the first 2^16/P ids of every
// rank's range (its own hubs) when the ranges are powers of two.  Off for the encoded hub domain, whose
// probe ids are not plain ids.
template <bool kHubs>
PrefixSpec lds_prefix(const bfsx_graph *g, const BfsWorkspace *ws) {
    PrefixSpec off{0u, 0u, 32u, 0u};
    if (kHubs || !g->d_perm || !g->ctx->opt.bu_lds_prefix) return off;
    if (g->nranks == 1) return PrefixSpec{(uint32_t)std::min<int64_t>(kPrefIds, ws->nwords * 64) & ~63u, 1u, 32u, 0u};
    const int64_t chunk = g->chunk;
    if (chunk & (chunk - 1)) return off; // not a power of two: the range of an id would need a division
    int shift = 0;
    while (((int64_t)1 << shift) < chunk) shift++;
    const uint32_t per = (uint32_t)std::min<int64_t>(kPrefIds / g->nranks, chunk) & ~63u;
    return per ? PrefixSpec{per, (uint32_t)g->nranks, (uint32_t)shift, 0u} : off;
}

template <class OffT, bool kMf, bool kHubs, int kU, bool kHubOnly, bool kPipe, bool kSpill = false>
int launch_bu_u(bfsx_graph *g, BfsWorkspace *ws, const OffT *row_off, const u64 *front, u64 *next, uint32_t *par,
                int level, Published *pub, u64 seq) {
    hipStream_t st = g->ctx->stream;
    // persistent grid: exactly the resident workgroups (a partial second wave of workgroups would
    // leave most CUs idle at the tail of the grid-stride loop)
    static int per_cu = 0;
    if (!per_cu) {
        const void *kfn = kSpill ? reinterpret_cast<const void *>(&k_bu_spill<OffT>)
                                 : reinterpret_cast<const void *>(&k_bu<OffT, kMf, kHubs, kU, kHubOnly, kPipe>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kBS, 0) !=
                hipSuccess ||
            per_cu < 1)
            per_cu = 4;
    }
    const unsigned cap = (unsigned)(g->ctx->num_cus * per_cu);
    const dim3 grid(clamp_grid((ws->nwords + kWaves * 64 - 1) / (kWaves * 64), cap));
    if (kHubs) {
        hipLaunchKernelGGL(k_hub_gather, dim3(clamp_grid((ws->hub_k + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                           ws->hub_id, ws->hub_k, front, ws->hfront);
        BFSX_LAUNCHED(st);
    }
#define BFSX_K_BU_LAUNCH(kern)                                                                                   \
    hipLaunchKernelGGL(kern, grid, dim3(kBS), 0, st, row_off, kHubs ? ws->colh : g->d_col, ws->top1, ws->rest, front, \
                       next, ws->vis, ws->st, par, ws->ring, level, ws->nwords, ws->top1_flag, ws->hfront, ws->hub_id,  \
                       ws->hub_lim, (uint32_t)std::min<int64_t>(ws->leaf_lo, 0xFFFFFFFFll), lds_prefix<kHubs>(g, ws),  \
                       pub, seq, (uint32_t)std::min<int64_t>(ws->hub_row_lim, 0xFFFFFFFFll))
    if constexpr (kSpill) BFSX_K_BU_LAUNCH((k_bu_spill<OffT>));
    else BFSX_K_BU_LAUNCH((k_bu<OffT, kMf, kHubs, kU, kHubOnly, kPipe>));
#undef BFSX_K_BU_LAUNCH
    BFSX_LAUNCHED(st);
    return BFSX_OK;
}

template <class OffT, bool kMf, bool kHubs>
int launch_bu_t(bfsx_graph *g, BfsWorkspace *ws, const OffT *row_off, const u64 *front, u64 *next, uint32_t *par,
                int level, Published *pub, u64 seq) {
    if (g->ctx->opt.bu_unroll == 2)
        return launch_bu_u<OffT, kMf, kHubs, 2, false, false>(g, ws, row_off, front, next, par, level, pub, seq);
    if (kMf && !kHubs && g->ctx->opt.bu_force_spill) // diagnostic (see k_bu's kSpill)
        return launch_bu_u<OffT, kMf, false, 4, false, true, true>(g, ws, row_off, front, next, par, level, pub, seq);
    // kMf (partitioned) + kPipe needs more than the 96 VGPRs of 5 waves per SIMD: that instantiation runs
    // at 4 waves per SIMD (a spilling pull kernel is never an option)
    return g->ctx->opt.bu_pipeline
               ? launch_bu_u<OffT, kMf, kHubs, 4, false, true>(g, ws, row_off, front, next, par, level, pub, seq)
               : launch_bu_u<OffT, kMf, kHubs, 4, false, false>(g, ws, row_off, front, next, par, level, pub, seq);
}

// The bottom-up half of a hybrid level: candidates probe only the hubs of the frontier (single device).
int launch_bu_hubonly(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level) {
    if (ws->hub_k > 0)
        return ws->off32
                   ? launch_bu_u<uint32_t, false, true, 4, true, false>(g, ws, ws->off32, front, next, par, level, nullptr, 0)
                   : launch_bu_u<int64_t, false, true, 4, true, false>(g, ws, g->d_row_off, front, next, par, level, nullptr, 0);
    return ws->off32
               ? launch_bu_u<uint32_t, false, false, 4, true, false>(g, ws, ws->off32, front, next, par, level, nullptr, 0)
               : launch_bu_u<int64_t, false, false, 4, true, false>(g, ws, g->d_row_off, front, next, par, level, nullptr, 0);
}

// par == null: discoveries store the packed state (the partitioned loop); else the 4-B parent (single device,
// `next` is then the level's record)
template <bool kMf>
int launch_bu(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level,
              Published *pub = nullptr, u64 seq = 0) {
    if (ws->hub_k > 0) // top1 is hub-encoded: every bottom-up launch of this graph uses the hub domain
        return ws->off32 ? launch_bu_t<uint32_t, kMf, true>(g, ws, ws->off32, front, next, par, level, pub, seq)
                         : launch_bu_t<int64_t, kMf, true>(g, ws, g->d_row_off, front, next, par, level, pub, seq);
    return ws->off32 ? launch_bu_t<uint32_t, kMf, false>(g, ws, ws->off32, front, next, par, level, pub, seq)
                     : launch_bu_t<int64_t, kMf, false>(g, ws, g->d_row_off, front, next, par, level, pub, seq);
}

// The sparse pull kernel (tail levels): one wave per kSparseWords words.  The discoveries below qlim land in
// ws->qa (the next push level's queue; its length is the published qtail).
int launch_bu_sparse(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level,
                     uint32_t qlim, Published *pub, u64 seq) {
    hipStream_t st = g->ctx->stream;
    const unsigned cap = (unsigned)g->ctx->num_cus * 8u;
    const dim3 grid(clamp_grid((ws->nwords + kWaves * kSparseWords - 1) / (kWaves * kSparseWords), cap));
    const uint32_t hrl = (uint32_t)std::min<int64_t>(ws->hub_row_lim, 0xFFFFFFFFll);
    if (ws->off32)
        hipLaunchKernelGGL(k_bu_sparse<uint32_t>, grid, dim3(kBS), 0, st, ws->off32, g->d_col, ws->top1, ws->rest,
                           front, next, ws->vis, ws->st, par, ws->ring, level, ws->nwords, ws->top1_flag, hrl, qlim,
                           ws->qa, pub, seq);
    else
        hipLaunchKernelGGL(k_bu_sparse<int64_t>, grid, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->top1, ws->rest,
                           front, next, ws->vis, ws->st, par, ws->ring, level, ws->nwords, ws->top1_flag, hrl, qlim,
                           ws->qa, pub, seq);
    BFSX_LAUNCHED(st);
    return BFSX_OK;
}

struct SlotSums {
    int64_t nf = 0, mf = 0, sc = 0, cl = 0, mu = 0, s2 = 0, wk = 0, nh = 0;
};

// Spin until the level's counters of the current sequence number have landed; poll the stream now and then so a
// faulted kernel surfaces as an error instead of a hang.
int wait_published(BfsWorkspace *ws, hipStream_t st) {
    const volatile u64 *seq = &ws->h_pub->seq;
    for (uint64_t spin = 1; *seq != ws->pub_seq; spin++) {
        if ((spin & 0xFFFF) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e != hipSuccess && e != hipErrorNotReady)
                return fail(BFSX_E_HIP, std::string("level kernels: ") + hipGetErrorString(e));
            if (e == hipSuccess && *seq != ws->pub_seq) return fail(BFSX_E_HIP, "level counters were not published");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return BFSX_OK;
}

// Post `na` words at a and `nb` at b to the host (in order) and wait for them; out gets na + nb words.  The
// partitioned loop passes its communicator: the wait then also ends (BFSX_E_RCCL) when a peer rank aborted or
// the wait outlived the communicator's deadline (Comm::poll), instead of spinning behind a collective that
// will never complete.
int post_wait(BfsWorkspace *ws, hipStream_t st, const u64 *a, int na, const u64 *b, int nb, u64 *out,
              Comm *cm = nullptr, const char *what = "a level close") {
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

SlotSums sum_slot(const LevelSlot *s) {
    SlotSums r;
    for (int i = 0; i < kShards; i++) {
        r.nf += (int64_t)s->sh[i].nf;
        r.mf += (int64_t)s->sh[i].mf;
        r.sc += (int64_t)s->sh[i].scanned;
        r.cl += (int64_t)s->sh[i].claims;
        r.mu += (int64_t)s->sh[i].mu;
        r.s2 += (int64_t)s->sh[i].stage2;
        r.wk += (int64_t)s->sh[i].walked;
        r.nh += (int64_t)s->sh[i].nhub;
    }
    return r;
}

struct LevelTiming {
    int ev;        // event slot: this level's own (per-level kernels) or the K3p launch's begin event
    bool persisted;
    double rel_ms; // K3p: end of the level after the launch's start (device wall clock)
    double k_ms;   // K3p: the level's own span
};

// Beamer's top-down -> bottom-up test compares m_f with m_u / alpha, but a pull level also has a fixed
// cost -- one pass over the n/64-word visited bitmap -- that the tail of a BFS (a few thousand frontier
// edges against a few thousand unvisited ones) never recovers: 30-40 us pull levels where a push
// level takes a few.  So a push level hands over only when its frontier has more than n/512 edges.
// The smallest frontier edge count a push -> pull switch needs: a pull level costs a pass over the n/64-word
// visited bitmap plus the frontier conversions and their dispatches (60-160 us per level at the tail of a
// 1 M-vertex high-diameter BFS, against ~13 us for a K3p push level), which a frontier of a few ten thousand
// edges never recovers.  Option pull_min_edges (default 2^16: largeG stand-in 9.69 -> 7.30 ms; scale 26 keeps n/512).
int64_t bu_floor(const bfsx_graph *g, const BfsWorkspace *ws) {
    return std::max<int64_t>(ws->nwords / 8, g->ctx->opt.pull_min_edges);
}

// K3p geometry: at most one workgroup per CU and at most kBS (every workgroup reads all records).
// auto: three workgroups per four CUs.  Every workgroup polls every record at each level's barrier, and the
// slowest of G dependent chains sets the level: on the largeG stand-in 160-192 workgroups give 10.6-10.7 us per
// level against 11.1 at 256 (96: 10.8, 32: 12.1), and scale 26 is level or better
// (profiles/r04y_k3p_grid_largeg.txt, profiles/r04y_k3p_grid_scale26_ab.txt).
int persist_blocks(const bfsx_ctx *ctx) {
    const int want = ctx->opt.persist_blocks > 0 ? ctx->opt.persist_blocks : std::max(1, ctx->num_cus * 3 / 4);
    return std::max(1, std::min({want, ctx->num_cus, kBS}));
}

// Whether a top-down level of nf vertices (largest degree dmax, < 0: unknown) may start K3p: every
// workgroup's slice must fit its output segment whatever it discovers.  G is the grid the launch will
// use: fixed at the graph's first K3p launch (ws->persist_grid), the option's value before it.
// A frontier vertex's row is swept by ONE workgroup of K3p (kBS * kItems entries per dependent step), so a
// frontier holding a vertex of degree > persist_dmax goes to the per-level kernels, whose multi-workgroup
// hub bin spreads that row over the whole grid (a 5,000-entry row took 52 us in K3p, ~20 us per level).
// K3p's buffers and grid, once per workspace: the grid is the occupancy-capped one the launch will use,
// known before the first persist_fits test (round 2 checked the first launch's segment bound against the
// uncapped option value).  persist_off: K3p cannot be co-resident on this device.
int persist_setup(bfsx_graph *g, BfsWorkspace *ws) {
    if (!ws->persist_seg) {
        const int G = persist_blocks(g->ctx);
        ws->persist_grid = G;
        BFSX_HIP_TRY(hipMalloc(&ws->persist_seg, (size_t)2 * G * kRegion * 2 * sizeof(u64)));
        BFSX_HIP_TRY(hipMalloc(&ws->persist_brec, (size_t)2 * G * kRecWords * sizeof(u64)));
        BFSX_HIP_TRY(hipMalloc(&ws->persist_hseg, (size_t)2 * G * kHeavyPer * 2 * sizeof(u64)));
        BFSX_HIP_TRY(hipMalloc(&ws->persist_ctl, sizeof(PersistCtl)));
        BFSX_HIP_TRY(hipHostMalloc(&ws->h_pout, sizeof(PersistOut), hipHostMallocMapped | hipHostMallocCoherent));
        BFSX_HIP_TRY(hipHostGetDevicePointer(&ws->d_pout, ws->h_pout, 0));
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, g->ctx->device) != hipSuccess || khz <= 0)
            khz = 100000;
        ws->clock_khz = (double)khz;
        // more than half a CU's LDS per workgroup: the dispatcher can place only one per CU
        int lds_cu = 0;
        hipFuncAttributes fa{};
        // both instantiations (with and without heavy rows) get the same padding, sized by the larger static
        // LDS (the heavy one), so each one's dynamic share is set for its own static size
        const void *kfh = ws->off32 ? reinterpret_cast<const void *>(&k_td_persist<uint32_t, true>)
                                    : reinterpret_cast<const void *>(&k_td_persist<int64_t, true>);
        const void *kfl = ws->off32 ? reinterpret_cast<const void *>(&k_td_persist<uint32_t, false>)
                                    : reinterpret_cast<const void *>(&k_td_persist<int64_t, false>);
        hipFuncAttributes fl{};
        if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, g->ctx->device) ==
                hipSuccess &&
            hipFuncGetAttributes(&fa, kfh) == hipSuccess && hipFuncGetAttributes(&fl, kfl) == hipSuccess && lds_cu > 0) {
            const size_t want = (size_t)lds_cu / 2 + 1024;
            const size_t dyn = want > fa.sharedSizeBytes ? want - fa.sharedSizeBytes : 0;
            const size_t dynl = want > fl.sharedSizeBytes ? want - fl.sharedSizeBytes : 0;
            if (dyn && dynl && hipFuncSetAttribute(kfh, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn) == hipSuccess &&
                hipFuncSetAttribute(kfl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dynl) == hipSuccess) {
                ws->persist_lds = dyn;
                ws->persist_lds_light = dynl;
            }
            (void)hipGetLastError();
        }
        // the grid barrier needs every workgroup resident at once: never launch more than the occupancy
        // API says fit for either instantiation (one per CU with the LDS padding above)
        int per_cu = 0, per_cul = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfh, kBS, ws->persist_lds) != hipSuccess) per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cul, kfl, kBS, ws->persist_lds_light) != hipSuccess)
            per_cul = 0;
        (void)hipGetLastError();
        ws->persist_grid = std::min(G, std::min(per_cu, per_cul) * g->ctx->num_cus);
        if (ws->persist_grid < 1) {
            ws->persist_off = true; // cannot be co-resident: narrow levels stay per-level launches
            return BFSX_OK;
        }
    }
    return BFSX_OK;
}

// heavy_src: the frontier is the source alone (level 0, its row bounds known to the host): a row longer than
// persist_dmax enters as K3p's heavy table (spread over the whole grid) instead of keeping K3p out.
bool persist_fits(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t dmax, bool heavy_src = false) {
    const bfsx_ctx *ctx = g->ctx;
    if (!ctx->opt.persist || ws->persist_off || nf <= 0 || nf > (int64_t)kPersistNf || dmax < 0) return false;
    const bool heavy = heavy_src && nf == 1 && dmax > ctx->opt.persist_dmax;
    if (dmax > ctx->opt.persist_dmax && !heavy) return false;
    if (!ws->persist_seg && persist_setup(g, ws) != BFSX_OK) {
        ws->persist_off = true; // no K3p buffers: narrow levels stay per-level launches
        return false;
    }
    const int64_t G = ws->persist_grid;
    if (ws->persist_off || G < 1) return false;
    return heavy ? (dmax + G - 1) / G <= (int64_t)kRegion : ((nf + G - 1) / G) * dmax <= (int64_t)kRegion;
}

constexpr int kPersistAborted = -1000; // internal: K3p aborted (barrier timeout); bfs_run retries without it

// Run K3p from `level` (frontier of nf vertices in ws->qa; its last frontier lands in ws->qb).
// Returns the number of levels it ran (>= 1) with their records in the PersistOut, or an error.
// h0_deg > 0: the first level's frontier is the single heavy row {h0_v, h0_beg, h0_deg} (nf = 0 light).
int persist_td(bfsx_graph *g, BfsWorkspace *ws, int level, int64_t nf, int64_t mu, uint32_t h0_v = 0,
               uint32_t h0_deg = 0, int64_t h0_beg = 0) {
    hipStream_t st = g->ctx->stream;
    const Options &opt = g->ctx->opt;
    if (!ws->persist_seg || ws->persist_off) return 0; // persist_fits sets K3p up before the first launch
    // record tags are 16 bits of the monotonic level count: before they could wrap within a launch, and after
    // an abort, the records are zeroed (tag 0 is never used) and the count restarts
    if (ws->persist_reset || ws->persist_bar + (u64)kPersistLevels + 1 > 0xFFFFull) {
        BFSX_HIP_TRY(hipMemsetAsync(ws->persist_ctl, 0, sizeof(PersistCtl), st));
        BFSX_HIP_TRY(hipMemsetAsync(ws->persist_brec, 0, (size_t)2 * ws->persist_grid * kRecWords * sizeof(u64), st));
        ws->persist_bar = 0;
        ws->persist_reset = false;
    }
    auto *out = reinterpret_cast<PersistOut *>(ws->h_pout);
    out->levels = 0;
    out->abort = 0;
    out->done = 0;
    std::atomic_thread_fence(std::memory_order_release);
    const int alpha = opt.direction == BFSX_DIR_AUTO ? std::max(opt.alpha, 1) : 0;
    auto *ctl = reinterpret_cast<PersistCtl *>(ws->persist_ctl);
    auto *dout = reinterpret_cast<PersistOut *>(ws->d_pout);
    const dim3 grid(ws->persist_grid);
    // the heavy instantiation only when a row can be heavy: the graph has rows longer than persist_dmax, or
    // the source enters as one
    const bool heavy = h0_deg > 0 || ws->heavy_rows;
    auto kp32 = heavy ? &k_td_persist<uint32_t, true> : &k_td_persist<uint32_t, false>;
    auto kp64 = heavy ? &k_td_persist<int64_t, true> : &k_td_persist<int64_t, false>;
    const size_t lds = heavy ? ws->persist_lds : ws->persist_lds_light;
    if (ws->off32)
        hipLaunchKernelGGL(kp32, grid, dim3(kBS), lds, st, ws->off32, g->d_col, ws->qa,
                           (uint32_t)nf, ws->persist_seg, ws->persist_brec, ws->qb, ws->vis, ws->st, ws->ring, level,
                           mu, alpha, kPersistLevels, ws->persist_bar, ctl, dout,
                           hub_set(ws), bu_floor(g, ws), opt.persist_abort_at, (u64)opt.persist_dmax,
                           (uint32_t)g->nv, ws->d_err, ws->persist_hseg, h0_v, h0_deg, h0_beg);
    else
        hipLaunchKernelGGL(kp64, grid, dim3(kBS), lds, st, g->d_row_off, g->d_col, ws->qa,
                           (uint32_t)nf, ws->persist_seg, ws->persist_brec, ws->qb, ws->vis, ws->st, ws->ring, level,
                           mu, alpha, kPersistLevels, ws->persist_bar, ctl, dout,
                           hub_set(ws), bu_floor(g, ws), opt.persist_abort_at, (u64)opt.persist_dmax,
                           (uint32_t)g->nv, ws->d_err, ws->persist_hseg, h0_v, h0_deg, h0_beg);
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
    // spin on workgroup 0's flag; poll the stream now and then so a faulted launch surfaces as an error
    const volatile u64 *done = &out->done;
    for (uint64_t spin = 1; *done == 0; spin++) {
        if ((spin & 0xFFFF) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e != hipSuccess && e != hipErrorNotReady)
                return fail(BFSX_E_HIP, std::string("persistent top-down: ") + hipGetErrorString(e));
            if (e == hipSuccess && *done == 0) {
                ws->persist_reset = true;
                return fail(BFSX_E_HIP, "persistent top-down: the launch ended without its done flag");
            }
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (out->abort) {
        ws->persist_reset = true;
        set_error("persistent top-down: grid barrier timed out or a segment overflowed");
        return kPersistAborted;
    }
    if (out->levels < 1 || out->levels > (u64)kPersistLevels) {
        ws->persist_reset = true;
        return fail(BFSX_E_HIP, "persistent top-down: no level ran");
    }
    ws->persist_bar += out->levels;
    return (int)out->levels;
}

} // namespace

void bfs_workspace_free(BfsWorkspace *ws) {
    if (!ws) return;
    for (void *p : {(void *)ws->sendbuf, (void *)ws->recvbuf, (void *)ws->fglob, (void *)ws->persist_seg,
                    (void *)ws->persist_brec, (void *)ws->persist_hseg, ws->persist_ctl})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)ws->st, (void *)ws->off32, (void *)ws->vis, (void *)ws->front, (void *)ws->next,
                    (void *)ws->dead, (void *)ws->qa, (void *)ws->qb, (void *)ws->hubs, (void *)ws->top1, (void *)ws->rest,
                    (void *)ws->hub_id, (void *)ws->colh, (void *)ws->hfront, (void *)ws->ring, (void *)ws->d_cursor, (void *)ws->d_red, (void *)ws->remote,
                    (void *)ws->d_dist_ctr, (void *)ws->out64, (void *)ws->rtmp})
        if (p) (void)hipFree(p);
    for (const auto &r : ws->retired) (void)hipFree(const_cast<void *>(r.p));
    for (void *p : ws->prec) (void)hipFree(p);
    if (ws->par) (void)hipFree(ws->par);
    if (ws->plog) (void)hipFree(ws->plog);
    if (ws->d_log_meta) (void)hipFree(ws->d_log_meta);
    if (ws->h_err) (void)hipHostFree(ws->h_err);
    if (ws->ev_unpack0) (void)hipEventDestroy(ws->ev_unpack0);
    if (ws->ev_unpack1) (void)hipEventDestroy(ws->ev_unpack1);
    if (ws->ev_unpack_mid) (void)hipEventDestroy(ws->ev_unpack_mid);
    for (auto e : ws->ev_stage)
        if (e) (void)hipEventDestroy(e);
    if (ws->h_stage) (void)hipHostFree(ws->h_stage);
    if (ws->h_slot) (void)hipHostFree(ws->h_slot);
    if (ws->h_pub) (void)hipHostFree(ws->h_pub);
    if (ws->h_pout) (void)hipHostFree(ws->h_pout);
    if (ws->h_post) (void)hipHostFree(ws->h_post);
    if (ws->ev_start) (void)hipEventDestroy(ws->ev_start);
    if (ws->ev_end) (void)hipEventDestroy(ws->ev_end);
    for (auto e : ws->ev_level) (void)hipEventDestroy(e);
    for (auto e : ws->ev_begin) (void)hipEventDestroy(e);
    delete ws;
}

namespace {

int bfs_run_impl(bfsx_graph *g, int64_t source, bfsx_stats *stats, bool allow_persist, bool record_start);

} // namespace

// K3p's grid barrier needs all of its workgroups resident; the launch is sized by the occupancy API,
// but another context on the same device can still hold CUs.  A barrier that times out aborts the
// launch (every workgroup exits), and the BFS is re-run from its source without K3p -- the level
// loop is deterministic, so the result is the same.  The re-run keeps the first attempt's start event, so
// t_bfs covers the aborted attempt too.
int bfs_run(bfsx_graph *g, int64_t source, bfsx_stats *stats) {
    int rc = bfs_run_impl(g, source, stats, true, true);
    if (rc == kPersistAborted) {
        g->ws->persist_fallbacks++;
        rc = bfs_run_impl(g, source, stats, false, false);
    }
    return rc == kPersistAborted ? fail(BFSX_E_HIP, "persistent top-down aborted twice") : rc;
}

int64_t bfs_persist_fallbacks(const bfsx_graph *g) { return g->ws ? g->ws->persist_fallbacks : 0; }

namespace {

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
                               set(), ws->nwords, ws->par, ws->st);
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

int bfs_run_impl(bfsx_graph *g, int64_t source, bfsx_stats *stats, bool allow_persist, bool record_start) {
    if (source < 0 || source >= g->nv)
        return fail(BFSX_E_RANGE, "source vertex " + std::to_string(source) + " outside [0, " +
                                      std::to_string(g->nv) + ")");
    int rc = ws_alloc(g);
    if (rc) return rc;
    BfsWorkspace *ws = g->ws;
    if ((rc = ensure_hub_row_lim(g, ws))) return rc;
    if ((rc = ensure_heavy_rows(g, ws))) return rc;
    bfsx_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    const Options &opt = ctx->opt;
    const int64_t nv = g->nv, nwords = ws->nwords;
    const unsigned cap = (unsigned)ctx->num_cus * 8u;

    int64_t src_off[2];
    const auto rm = g->row_memo.find(source);
    if (rm != g->row_memo.end()) {
        src_off[0] = rm->second.first;
        src_off[1] = rm->second.second;
    } else {
        BFSX_HIP_TRY(hipMemcpy(src_off, g->d_row_off + source, sizeof(src_off), hipMemcpyDeviceToHost));
        if (g->row_memo.size() >= 65536) g->row_memo.clear();
        g->row_memo.emplace(source, std::make_pair(src_off[0], src_off[1]));
    }

    // push log of this BFS (BfsWorkspace::plog), allocated once per workspace
    ws->log_n = 0;
    ws->log_end.clear();
    ws->log_nd.clear();
    ws->logs_pending = false;
    if (opt.push_log && !ws->plog) BFSX_HIP_TRY(hipMalloc(&ws->plog, (size_t)std::max<int64_t>(nv, 1) * sizeof(u64)));
    const int64_t n_pre = ws->n_dead; // pre-visited non-padding ids
    if (opt.poison_queues) // test hook: a consumer that reads past a queue's tail meets 0xFFFFFFFF (id_ok)
        for (uint32_t *q : {ws->qa, ws->qb, ws->hubs})
            BFSX_HIP_TRY(hipMemsetAsync(q, 0xFF, (size_t)std::max<int64_t>(nv, 1) * sizeof(uint32_t), st));
    // ---- timed region: source init -> last level ----
    if (record_start) BFSX_HIP_TRY(hipEventRecord(ws->ev_start, st));
    hipLaunchKernelGGL(k_init, dim3(clamp_grid((nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0, st, (uint32_t)source,
                       (uint32_t)source, ws->prev_source, ws->dead, nwords, ws->st, ws->vis, ws->qa, ws->ring);
    BFSX_LAUNCHED(st);
    ws->prev_source = source;

    int dir = (opt.direction == BFSX_DIR_BOTTOMUP) ? BFSX_DIR_BOTTOMUP : BFSX_DIR_TOPDOWN;
    bool in_queue = true; // frontier currently held in ws->qa (else in ws->front)
    bool snapped = false; // ws->front holds the visited bitmap from before the last (top-down) level
    int64_t nf = 1, prev_nf = 0;
    int64_t mf = src_off[1] - src_off[0]; // degree sum of the frontier being expanded (-1: unknown)
    int64_t dmax = mf;                    // its largest degree (-1: unknown)
    int64_t mu = g->nnz;                  // Beamer m_u: adjacency entries of unvisited vertices
    // degree sum of the frontier's hub-domain vertices (-1: unknown): a top-down level whose frontier
    // degree sum sits mostly in hubs runs as a hybrid level (below)
    int64_t mfh = ((ws->hub_k > 0 && mf >= (int64_t)ws->hub_tdeg) || source < (int64_t)ws->hub_lim) ? mf : 0;
    int64_t examined = 0, visited = 1;
    // the frontier's vertices below leaf_lo (-1: unknown); set by a pull level (its k_bu counts them)
    int64_t nf_core = -1;
    // a pull level's discoveries below hub_row_lim (-1: unknown): 0 means no frontier vertex has more than
    // hub_degree entries, so the next push level needs no hub bin and may run inside K3p
    int64_t nh_found = -1;
    // the last (sparse) pull level already wrote the next push level's queue into ws->qa (nf_core ids)
    bool queue_ready = false;
    int td_levels = 0, bu_levels = 0;
    // the bitmap frontier: ws->front after a push -> pull conversion, a pull level's record after a pull level
    const u64 *bmf = ws->front;
    // pull-level records of this BFS (BfsWorkspace::par)
    RecLog recs(g, ws);
    std::vector<LevelTiming> timing;
    g->level_dirs.clear();
    g->level_cum_ms.clear();
    g->level_stats.clear();
    int level = 0;
    for (;; level++) {
        if (opt.direction == BFSX_DIR_AUTO && level > 0) {
            if (dir == BFSX_DIR_TOPDOWN) {
                if (mf > mu / std::max(opt.alpha, 1) && mf > bu_floor(g, ws)) dir = BFSX_DIR_BOTTOMUP;
            } else if (nf < nv / std::max(opt.beta, 1) && nf < prev_nf) {
                dir = BFSX_DIR_TOPDOWN;
            }
        }
        while ((int)ws->ev_level.size() <= level) {
            hipEvent_t e0, e1;
            BFSX_HIP_TRY(hipEventCreate(&e0));
            BFSX_HIP_TRY(hipEventCreate(&e1));
            ws->ev_begin.push_back(e0);
            ws->ev_level.push_back(e1);
        }
        BFSX_HIP_TRY(hipEventRecord(ws->ev_begin[level], st));
        // Hybrid level: a top-down level whose frontier is dominated (by degree sum) by hubs -- a hub root's
        // neighbourhood: a few thousand vertices with tens of millions of edges -- would push every one of
        // those edges through a random visited-bitmap probe.  Instead the unvisited vertices pull from
        // the frontier's HUBS only (k_bu hub sweep: every probe lands in the small gathered hub bitmap,
        // and a degree-ordered row stops at its first non-hub entry), and the frontier's non-hub
        // vertices are expanded top-down behind it.  Measured on scale 26 (U = 32.8 M unvisited): the
        // hybrid level costs 0.95-1.4 ms (most of it the unvisited vertices that find no frontier hub and
        // walk their whole hub prefix), the push level ~0.028 ms per million frontier edges (0.72 ms at
        // 17.6 M, 1.74 ms at 67.4 M) -- so hybrid only once the hubs' edges exceed 1.25 U.
        bool hybrid = false, sparse = false;
        u64 *bu_rec = nullptr; // a pull level's record
        if (dir == BFSX_DIR_TOPDOWN && in_queue && level > 0 && has_hubs(ws) && opt.hybrid != 0 && mfh > 0) {
            const int64_t unv = nv - visited - n_pre;
            hybrid = opt.hybrid == 2 || 100 * mfh > (int64_t)opt.hybrid_pct * unv;
        }
        if (hybrid) {
            BFSX_HIP_TRY(hipMemsetAsync(ws->front, 0, nwords * sizeof(u64), st));
            hipLaunchKernelGGL(k_queue_to_bitmap, dim3(clamp_grid((nf + kBS - 1) / kBS, cap)), dim3(kBS), 0, st, ws->qa,
                               (uint32_t)nf, ws->front, (uint32_t)g->nv, ws->d_err);
            BFSX_LAUNCHED(st);
            u64 *rec = nullptr;
            if (int e = recs.take(&rec)) return e;
            if (int e = launch_bu_hubonly(g, ws, ws->front, rec, ws->par, level)) return e; // -> rec, vis, par
            const Part pt = single_part(g, ws);
            // -> qb; its winners also store their parent in par (they join the record below)
            if (int e = launch_td<false>(g, ws, nf, mf, dmax, level, pt, true, nullptr, 0, ws->par)) return e;
            LevelSlot *cn = ws->ring + (level + 1) % 3;
            hipLaunchKernelGGL(k_queue_to_bitmap_dev, dim3(cap), dim3(kBS), 0, st, ws->qb, cn, rec, ws->d_pub,
                               ++ws->pub_seq, (uint32_t)g->nv, ws->d_err);
            BFSX_LAUNCHED(st);
            BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
            if (int e = wait_published(ws, st)) return e;
            const int64_t nf_new = ws->h_pub->nf + ws->h_pub->qtail;
            g->level_dirs.push_back(BFSX_DIR_HYBRID);
            bfsx_level_stat ls{};
            ls.direction = BFSX_DIR_HYBRID;
            ls.level = level;
            ls.frontier_in = nf;
            ls.frontier_out = nf_new;
            ls.mf_in = mf;
            ls.unvisited_in = nv - visited - n_pre;
            ls.scanned = ws->h_pub->sc;
            ls.claims = ws->h_pub->cl;
            g->level_stats.push_back(ls);
            timing.push_back({level, false, 0.0, 0.0});
            examined += ls.scanned;
            visited += nf_new;
            prev_nf = nf;
            nf = nf_new;
            // m_u: the pull half counted the candidates it left (a row without hubs counts 1), minus the
            // degree sum of what the push half then discovered among them
            mu = std::max<int64_t>(ws->h_pub->mu - ws->h_pub->mf, 0);
            mf = -1;
            dmax = -1;
            mfh = -1;
            dir = BFSX_DIR_BOTTOMUP; // the new frontier is a bitmap
            nf_core = -1;
            nh_found = -1;
            queue_ready = false;
            in_queue = false;
            snapped = false;
            bu_levels++;
            recs.done(level + 1);
            bmf = rec;
            if (nf == 0) break;
            continue;
        }
        if (dir == BFSX_DIR_BOTTOMUP && in_queue) {
            if (snapped) { // front holds the visited bitmap from before the last top-down level
                hipLaunchKernelGGL(k_new_bits, dim3(clamp_grid((nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0, st,
                                   ws->vis, nwords, ws->front);
            } else {
                BFSX_HIP_TRY(hipMemsetAsync(ws->front, 0, nwords * sizeof(u64), st));
                hipLaunchKernelGGL(k_queue_to_bitmap, dim3(clamp_grid((nf + kBS - 1) / kBS, cap)), dim3(kBS), 0, st,
                                   ws->qa, (uint32_t)nf, ws->front, (uint32_t)g->nv, ws->d_err);
            }
            BFSX_LAUNCHED(st);
            bmf = ws->front;
            in_queue = false;
        } else if (dir == BFSX_DIR_TOPDOWN && !in_queue && queue_ready) {
            // the sparse pull level queued its discoveries (the non-leaves with leaf_skip) itself
            nf = nf_core;
            if (nh_found == 0) dmax = (int64_t)opt.hub_degree; // a bound: every discovery is a short row
            in_queue = true;
        } else if (dir == BFSX_DIR_TOPDOWN && !in_queue) {
            // leaf skip: a pull level's discoveries at ids >= leaf_lo have one neighbour, their parent, so
            // they sweep nothing; the queue holds the nf_core others (the pull kernel counted them)
            const bool skip = opt.leaf_skip && nf_core >= 0 && ws->leaf_lo < nv;
            const int64_t lim = skip ? ws->leaf_lo : nwords * 64;
            const int64_t cw = (lim + 63) / 64; // words holding ids below lim
            BFSX_HIP_TRY(hipMemsetAsync(ws->d_cursor, 0, sizeof(u64), st));
            const int64_t per_block_min = (int64_t)kBS * kCompactWords;
            const unsigned gb = clamp_grid(std::max<int64_t>((cw + per_block_min - 1) / per_block_min, 1), 256);
            const int64_t wpb = ((cw + gb - 1) / gb + per_block_min - 1) / per_block_min * per_block_min;
            hipLaunchKernelGGL(k_bitmap_to_queue, dim3(gb), dim3(kBS), 0, st, bmf, cw, wpb, ws->qa,
                               ws->d_cursor, lim);
            BFSX_LAUNCHED(st);
            if (skip) nf = nf_core;
            if (nh_found == 0) dmax = (int64_t)opt.hub_degree; // a bound: every discovery is a short row
            static const bool trace = std::getenv("BFSX_TRACE") != nullptr;
            if (trace) {
                u64 qn = 0;
                BFSX_HIP_TRY(hipMemcpyAsync(&qn, ws->d_cursor, sizeof(qn), hipMemcpyDeviceToHost, st));
                BFSX_HIP_TRY(hipStreamSynchronize(st));
                fprintf(stderr, "[bfsx] level %d: bitmap -> queue %llu ids below %lld, nf %lld (skip %d)\n", level,
                        (unsigned long long)qn, (long long)lim, (long long)nf, (int)skip);
            }
            in_queue = true;
        }
        nf_core = -1;
        nh_found = -1;
        queue_ready = false;
        snapped = false;
        u64 *plog = nullptr; // this level's push-log segment (a per-level push level with push_log)
        // level 0: a source row longer than persist_dmax enters K3p as its heavy table (row bounds known)
        const bool heavy_src = level == 0 && nf == 1 && dmax > opt.persist_dmax;
        if (dir == BFSX_DIR_TOPDOWN && allow_persist && persist_fits(g, ws, nf, dmax, heavy_src)) {
            // narrow frontier: run as many levels as stay narrow inside one launch (K3p)
            const int ran = heavy_src ? persist_td(g, ws, level, 0, mu, (uint32_t)source, (uint32_t)dmax, src_off[0])
                                      : persist_td(g, ws, level, nf, mu);
            if (ran < 0) return ran;
            // ran == 0: K3p unavailable on this device (occupancy check): per-level launches below
            if (ran > 0) {
                const PersistOut &po = *reinterpret_cast<const PersistOut *>(ws->h_pout);
                for (int i = 0; i < ran; i++) {
                    const PersistRec &r = po.rec[i];
                    bfsx_level_stat ls{};
                    ls.direction = BFSX_DIR_TOPDOWN;
                    ls.level = level + i;
                    ls.frontier_in = nf;
                    ls.frontier_out = (int64_t)r.qtail;
                    ls.mf_in = (int64_t)r.scanned;
                    ls.unvisited_in = nv - visited - n_pre;
                    ls.scanned = (int64_t)r.scanned;
                    ls.claims = (int64_t)r.claims;
                    g->level_stats.push_back(ls);
                    g->level_dirs.push_back(BFSX_DIR_TOPDOWN);
                    timing.push_back({level, true, (double)(r.t_end - po.t0) / ws->clock_khz,
                                      (double)(r.t_end - (i ? po.rec[i - 1].t_end : po.t0)) / ws->clock_khz});
                    examined += ls.scanned;
                    visited += ls.frontier_out;
                    mu -= (int64_t)r.mf;
                    prev_nf = nf;
                    nf = ls.frontier_out;
                    mf = (int64_t)r.mf;
                    dmax = (int64_t)r.dmax;
                    mfh = has_hubs(ws) ? (int64_t)r.mfh : -1;
                }
                std::swap(ws->qa, ws->qb); // K3p hands its last frontier back in qb (and zeroed the ring)
                td_levels += ran;
                level += ran - 1;
                if (nf == 0) break;
                continue;
            }
        }
        if (dir == BFSX_DIR_TOPDOWN) {
            // a wide top-down level may hand over to bottom-up: snapshot the visited bitmap (8 B per 64
            // vertices) so its frontier bitmap is one XOR pass instead of one atomic per discovered vertex
            if (mf >= nwords / 4 && opt.direction == BFSX_DIR_AUTO) {
                BFSX_HIP_TRY(hipMemcpyAsync(ws->front, ws->vis, nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
                snapped = true;
            }
            const Part pt = single_part(g, ws);
            // test hook: the level's kernels read one entry past the queue's tail (the guard must catch it)
            const int64_t nf_l = level == opt.test_overread ? nf + 1 : nf;
            plog = opt.push_log ? ws->plog + ws->log_n : nullptr;
            if (int e = launch_td<false>(g, ws, nf_l, mf, dmax, level, pt, false, ws->d_pub, ++ws->pub_seq, nullptr, plog))
                return e;
            td_levels++;
        } else {
            // few unvisited candidates (the tail levels): the sparse kernel, which also queues its discoveries
            sparse = opt.bu_sparse > 0 && ws->hub_k == 0 && (nv - visited - n_pre) * opt.bu_sparse <= nwords * 64;
            if (int e = recs.take(&bu_rec)) return e;
            if (sparse) {
                const uint32_t qlim = (uint32_t)(opt.leaf_skip ? std::min<int64_t>(ws->leaf_lo, nv) : nv);
                if (int e = launch_bu_sparse(g, ws, bmf, bu_rec, ws->par, level, qlim, ws->d_pub, ++ws->pub_seq))
                    return e;
            } else if (int e = launch_bu<false>(g, ws, bmf, bu_rec, ws->par, level, ws->d_pub, ++ws->pub_seq)) {
                return e;
            }
            bu_levels++;
        }
        BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
        if (int e = wait_published(ws, st)) return e;
        SlotSums s;
        s.nf = ws->h_pub->nf;
        s.mf = ws->h_pub->mf;
        s.sc = ws->h_pub->sc;
        s.cl = ws->h_pub->cl;
        s.mu = ws->h_pub->mu;
        s.s2 = ws->h_pub->stage2;
        s.wk = ws->h_pub->walked;
        const int64_t nf_new = (dir == BFSX_DIR_TOPDOWN) ? ws->h_pub->qtail : s.nf;
        if (plog && nf_new > 0) { // the level's winners are log entries [log_n, log_n + nf_new)
            ws->log_n += nf_new;
            ws->log_end.push_back(ws->log_n);
            ws->log_nd.push_back(level + 1);
            ws->logs_pending = true;
        }
        const int rec_dir = sparse ? BFSX_DIR_BOTTOMUP_SPARSE : dir;
        g->level_dirs.push_back(rec_dir);
        bfsx_level_stat ls{};
        ls.direction = rec_dir;
        ls.level = level;
        ls.frontier_in = nf;
        ls.frontier_out = nf_new;
        ls.mf_in = (dir == BFSX_DIR_TOPDOWN) ? s.sc : mf; // top-down: the kernels count the rows they sweep
        ls.unvisited_in = nv - visited - n_pre;      // live candidates (isolated ones are pre-visited)
        ls.scanned = s.sc;
        ls.claims = s.cl;
        ls.stage2 = s.s2;
        ls.walked = s.wk;
        g->level_stats.push_back(ls);
        timing.push_back({level, false, 0.0, 0.0});
        examined += ls.scanned;
        visited += nf_new;
        prev_nf = nf;
        nf = nf_new;
        if (dir == BFSX_DIR_TOPDOWN) {
            mu -= s.mf;
            mf = s.mf;
            dmax = ws->h_pub->dmax;
            mfh = has_hubs(ws) ? s.s2 : -1; // top-down: stage2 = degree sum of the hubs discovered
            std::swap(ws->qa, ws->qb);
        } else {
            mu = s.mu; // exact: degree sum of the candidates this level left unvisited
            nf_core = s.mf; // the single-GPU bottom-up step counts its discoveries below leaf_lo here
            nh_found = ws->h_pub->nhub;
            queue_ready = sparse; // the sparse kernel counted (mf) and queued them
            mf = -1;   // not accumulated by the single-GPU bottom-up step
            dmax = -1;
            mfh = -1;
            recs.done(level + 1);
            bmf = bu_rec;
        }
        if (nf == 0) break;
    }
    // unvisited (non-isolated) vertices -> WHITE; inside the timed region
    hipLaunchKernelGGL(k_finalize, dim3(clamp_grid((nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0, st, ws->vis, nwords,
                       ws->st);
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipEventRecord(ws->ev_end, st));
    BFSX_HIP_TRY(hipEventSynchronize(ws->ev_end));
    if (int e = check_queue_guard(ws)) return e;
    recs.finish();
    if (ws->logs_pending) ws->resolved = false;
    const int levels = level + 1;
    float ms = 0.f;
    BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_start, ws->ev_end));
    g->level_cum_ms.resize(levels);
    for (int l = 0; l < levels; l++) {
        float t = 0.f, k = 0.f;
        const LevelTiming &lt = timing[l];
        if (lt.persisted) { // device clock inside the launch that started at event slot lt.ev
            BFSX_HIP_TRY(hipEventElapsedTime(&t, ws->ev_start, ws->ev_begin[lt.ev]));
            t += (float)lt.rel_ms;
            k = (float)lt.k_ms;
        } else {
            BFSX_HIP_TRY(hipEventElapsedTime(&t, ws->ev_start, ws->ev_level[l]));
            BFSX_HIP_TRY(hipEventElapsedTime(&k, ws->ev_begin[l], ws->ev_level[l]));
        }
        g->level_cum_ms[l] = t;
        g->level_stats[l].cum_ms = t;
        g->level_stats[l].kernel_ms = k;
    }
    g->last_source = source;
    g->last_t_bfs_ms = ms;
    if (stats) {
        stats->levels = levels;
        stats->topdown_levels = td_levels;
        stats->bottomup_levels = bu_levels;
        stats->t_bfs_ms = ms;
        stats->edges_examined = examined;
    }
    return BFSX_OK;
}

} // namespace

// Scatter the last BFS's push log into st (outside the timed region; no-op when nothing is pending).  ev: recorded
// after the segment table's upload, before the kernel (the unpack's timing starts there).
int apply_logs(bfsx_graph *g, BfsWorkspace *ws, hipEvent_t ev = nullptr) {
    hipStream_t st = g->ctx->stream;
    const int nseg = (int)ws->log_end.size();
    if (!ws->logs_pending || nseg == 0) {
        ws->logs_pending = false;
        if (ev) BFSX_HIP_TRY(hipEventRecord(ev, st));
        return BFSX_OK;
    }
    if (2 * nseg > ws->log_meta_cap) {
        if (ws->d_log_meta) BFSX_HIP_TRY(hipFree(ws->d_log_meta));
        ws->log_meta_cap = std::max<int64_t>(2 * nseg, 256);
        BFSX_HIP_TRY(hipMalloc(&ws->d_log_meta, ws->log_meta_cap * sizeof(int64_t)));
    }
    std::vector<int64_t> meta(ws->log_end);
    meta.insert(meta.end(), ws->log_nd.begin(), ws->log_nd.end());
    BFSX_HIP_TRY(hipMemcpyAsync(ws->d_log_meta, meta.data(), meta.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st)); // meta is a host temporary
    if (ev) BFSX_HIP_TRY(hipEventRecord(ev, st));
    hipLaunchKernelGGL(k_resolve_log, dim3(clamp_grid((ws->log_n + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st, ws->plog,
                       ws->log_n, ws->d_log_meta, nseg, ws->st);
    BFSX_LAUNCHED(st);
    ws->logs_pending = false;
    return BFSX_OK;
}

// Fold the last BFS's pull-level records and push log into st (the validator's and m_comp's view of a result;
// outside the timed region).  No-op when none is pending.
int bfs_resolve(bfsx_graph *g) {
    BfsWorkspace *ws = g->ws;
    if (!ws || ws->resolved) return BFSX_OK;
    if (int e = apply_logs(g, ws)) return e;
    hipStream_t st = g->ctx->stream;
    RecSet rs{};
    rs.n = ws->n_prec;
    for (int r = 0; r < ws->n_prec; r++) {
        rs.bm[r] = ws->prec[r];
        rs.nd[r] = ws->prec_nd[r];
    }
    hipLaunchKernelGGL(k_resolve, dim3(clamp_grid((ws->nwords * 64 + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st, rs,
                       ws->nwords, ws->par, ws->st);
    BFSX_LAUNCHED(st);
    ws->resolved = true;
    return BFSX_OK;
}

int bfs_mcomp(bfsx_graph *g, int64_t *m_comp, int64_t *reached) {
    BfsWorkspace *ws = g->ws;
    hipStream_t st = g->ctx->stream;
    if (int e = bfs_resolve(g)) return e;
    u64 h[2] = {0, 0};
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, 2 * sizeof(u64), st));
    hipLaunchKernelGGL(k_mcomp, dim3(clamp_grid((g->nv + kBS - 1) / kBS, 2048)), dim3(kBS), 0, st, ws->st,
                       g->d_tuple_cnt, g->nv, ws->d_red);
    BFSX_LAUNCHED(st);
    BFSX_HIP_TRY(hipMemcpyAsync(h, ws->d_red, sizeof(h), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    *m_comp = (int64_t)h[0];
    *reached = (int64_t)h[1];
    return BFSX_OK;
}

const unsigned long long *bfs_state(const bfsx_graph *g) { return g->ws ? g->ws->st : nullptr; }

namespace {

constexpr size_t kStageBytes = (size_t)32 << 20; // one pinned staging chunk of the result copy

// Host threads of the result copy: the job's CPU share (OMP_NUM_THREADS, as the GPU box sets it), at most 16.
int copy_threads() {
    static const int n = [] {
        int t = (int)std::thread::hardware_concurrency();
        if (const char *e = std::getenv("OMP_NUM_THREADS")) {
            const int x = std::atoi(e);
            if (x > 0) t = std::min(t > 0 ? t : x, x);
        }
        return std::max(1, std::min(t, 16));
    }();
    return n;
}

} // namespace

// The result in the caller's ids: one unpack kernel (state + pending records -> parent << 32 | dist per original
// id, or int32 dist only), then the D2H copy through two pinned 32 MiB chunks, each split by host threads into
// dist (int32) and parent (int64, -1 = none) while the next chunk is in flight (a pageable copy plus one host
// thread widening 67 M parents took 80 ms at scale 26).
int bfs_copy_result(bfsx_graph *g, int32_t *dist_out, int64_t *parent_out) {
    BfsWorkspace *ws = g->ws;
    if (!ws || g->last_source < 0) return fail(BFSX_E_ARG, "no BFS result on this graph yet");
    hipStream_t st = g->ctx->stream;
    const size_t nv = (size_t)g->nv;
    if (!ws->out64) {
        BFSX_HIP_TRY(hipMalloc(&ws->out64, std::max<size_t>(nv, 1) * sizeof(u64)));
        BFSX_HIP_TRY(hipEventCreate(&ws->ev_unpack0));
        BFSX_HIP_TRY(hipEventCreate(&ws->ev_unpack1));
        BFSX_HIP_TRY(hipEventCreate(&ws->ev_unpack_mid));
    }
    RecSet rs{};
    rs.n = ws->resolved ? 0 : ws->n_prec;
    for (int r = 0; r < rs.n; r++) {
        rs.bm[r] = ws->prec[r];
        rs.nd[r] = ws->prec_nd[r];
    }
    // dist only (int32 words) when only dist is asked for; parent << 32 | dist otherwise, also when nothing is
    // copied (a device-only materialisation of the whole result: bfsx_result with two null outputs)
    const bool packed = parent_out != nullptr || dist_out == nullptr;
    int32_t *d_dist_only = packed ? nullptr : reinterpret_cast<int32_t *>(ws->out64);
    const dim3 grid(clamp_grid(((int64_t)nv + kBS - 1) / kBS, 8192));
    const int mode = packed ? 1 : 2;
    // a relabelled graph unpacks in original id order and writes every entry (k_unpack_gather): no prefill
    const bool gather = g->d_perm != nullptr && g->d_inv != nullptr;
    if (!gather && ws->out_mode != mode) { // every entry unreached once; isolated vertices keep it from then on
        if (packed) {
            hipLaunchKernelGGL(k_fill64, grid, dim3(kBS), 0, st, ws->out64, (int64_t)nv, kUnreached);
        } else {
            hipLaunchKernelGGL(k_fill64, grid, dim3(kBS), 0, st, ws->out64, (int64_t)(nv + 1) / 2,
                               ((u64)INT32_MAX << 32) | (u64)INT32_MAX);
        }
        BFSX_LAUNCHED(st);
        ws->out_mode = mode;
        ws->out_dirty = -1;
    }
    // the source's local row (a partition's non-owning ranks: none)
    const int64_t src = (g->last_source >= g->v_lo && g->last_source < g->v_lo + g->nv) ? g->last_source - g->v_lo : -1;
    bool src_dead = false; // an isolated source's entry must be reset by the next (scatter-form) unpack
    if (src >= 0 && !gather) {
        u64 dw = 0;
        BFSX_HIP_TRY(hipMemcpyAsync(&dw, ws->dead + (src >> 6), sizeof(dw), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        src_dead = (dw >> (src & 63)) & 1ull;
    }
    if (int e = apply_logs(g, ws, ws->ev_unpack0)) return e; // the push log is part of the unpack's time
    if (gather) {
        u64 *tmp = ws->plog; // free once the log is scattered (apply_logs above)
        if (!tmp) {
            if (!ws->rtmp) BFSX_HIP_TRY(hipMalloc(&ws->rtmp, std::max<size_t>(nv, 1) * sizeof(u64)));
            tmp = ws->rtmp;
        }
        const int64_t nw_live = std::min<int64_t>((ws->iso_lo + 63) / 64, ws->nwords);
        const int64_t src_word = src >= 0 ? src / 64 : 0;
        hipLaunchKernelGGL(k_resolve_all, dim3(clamp_grid((nw_live + 1 + kWaves - 1) / kWaves, 8192)), dim3(kBS), 0, st,
                           rs, nw_live, src_word, ws->par, ws->st, g->d_inv, tmp, (int64_t)nv);
        BFSX_LAUNCHED(st);
        ws->resolved = true; // st now holds every record vertex's state too (bfs_resolve has nothing left to do)
        BFSX_HIP_TRY(hipEventRecord(ws->ev_unpack_mid, st));
        hipLaunchKernelGGL(k_unpack_gather, grid, dim3(kBS), 0, st, tmp, g->d_perm, (int64_t)nv, ws->iso_lo, src,
                           ws->out64, d_dist_only);
        ws->out_mode = 0; // every entry written: a later scatter-mode unpack must prefill again
    } else if (g->d_inv)
        hipLaunchKernelGGL(k_unpack<true>, grid, dim3(kBS), 0, st, ws->st, ws->par, rs, g->d_inv, g->v_lo, (int64_t)nv,
                           ws->dead, src, ws->out_dirty, ws->out64, d_dist_only);
    else
        hipLaunchKernelGGL(k_unpack<false>, grid, dim3(kBS), 0, st, ws->st, ws->par, rs, g->d_inv, g->v_lo,
                           (int64_t)nv, ws->dead, src, ws->out_dirty, ws->out64, d_dist_only);
    BFSX_LAUNCHED(st);
    ws->out_dirty = src_dead ? src : -1;
    BFSX_HIP_TRY(hipEventRecord(ws->ev_unpack1, st));
    if (dist_out || parent_out) {
        if (!ws->h_stage) {
            BFSX_HIP_TRY(hipHostMalloc(&ws->h_stage, 2 * kStageBytes, hipHostMallocDefault));
            BFSX_HIP_TRY(hipEventCreateWithFlags(&ws->ev_stage[0], hipEventDisableTiming));
            BFSX_HIP_TRY(hipEventCreateWithFlags(&ws->ev_stage[1], hipEventDisableTiming));
        }
        const size_t esz = packed ? sizeof(u64) : sizeof(int32_t);
        const size_t per = kStageBytes / esz; // elements per chunk
        const size_t nchunk = (nv + per - 1) / per;
        const char *src = reinterpret_cast<const char *>(ws->out64);
        char *stage[2] = {reinterpret_cast<char *>(ws->h_stage), reinterpret_cast<char *>(ws->h_stage) + kStageBytes};
        auto issue = [&](size_t c) -> int {
            const size_t b = c * per, n = std::min(per, nv - b);
            BFSX_HIP_TRY(hipMemcpyAsync(stage[c & 1], src + b * esz, n * esz, hipMemcpyDeviceToHost, st));
            BFSX_HIP_TRY(hipEventRecord(ws->ev_stage[c & 1], st));
            return BFSX_OK;
        };
        const int T = copy_threads();
        std::vector<std::thread> pool;
        pool.reserve(T);
        if (int e = issue(0)) return e;
        for (size_t c = 0; c < nchunk; c++) {
            BFSX_HIP_TRY(hipEventSynchronize(ws->ev_stage[c & 1]));
            // the chunk before this one is fully split (joined below), so its buffer takes chunk c + 1
            if (c + 1 < nchunk)
                if (int e = issue(c + 1)) return e;
            const size_t b = c * per, n = std::min(per, nv - b);
            const char *buf = stage[c & 1];
            auto split = [&, b, buf](size_t lo, size_t hi) {
                if (packed) {
                    const u64 *x = reinterpret_cast<const u64 *>(buf);
                    for (size_t i = lo; i < hi; i++) {
                        const u64 w = x[i];
                        if (dist_out) dist_out[b + i] = (int32_t)(uint32_t)w;
                        parent_out[b + i] = (int64_t)(int32_t)(uint32_t)(w >> 32); // 0xFFFFFFFF (none) -> -1
                    }
                } else {
                    std::memcpy(dist_out + b + lo, buf + lo * sizeof(int32_t), (hi - lo) * sizeof(int32_t));
                }
            };
            const size_t step = (n + T - 1) / T;
            for (int t = 1; t < T; t++) {
                const size_t lo = std::min(n, (size_t)t * step), hi = std::min(n, lo + step);
                if (lo < hi) pool.emplace_back(split, lo, hi);
            }
            split(0, std::min(n, step));
            for (auto &th : pool) th.join();
            pool.clear();
        }
    }
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    float ms = 0.f;
    BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_unpack0, ws->ev_unpack1));
    ws->last_unpack_ms = ms;
    ws->last_resolve_ms = -1.0;
    if (gather) {
        BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_unpack0, ws->ev_unpack_mid));
        ws->last_resolve_ms = ms;
    }
    return BFSX_OK;
}

double bfs_last_unpack_ms(const bfsx_graph *g) { return g->ws ? g->ws->last_unpack_ms : -1.0; }
double bfs_last_resolve_ms(const bfsx_graph *g) { return g->ws ? g->ws->last_resolve_ms : -1.0; }

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
    p.nrows = (uint32_t)g->nv;
    p.err = ws->d_err;
    p.nranks = (uint32_t)g->nranks;
    return p;
}

int dist_ws(bfsx_graph *g) {
    int rc = ws_alloc(g);
    if (rc) return rc;
    if (!g->ws->d_dist_ctr) BFSX_HIP_TRY(hipMalloc(&g->ws->d_dist_ctr, kCtrWords * sizeof(u64)));
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
    if (g->ctx->opt.poison_queues) // test hook (see bfs_run_impl)
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
                           (uint32_t)g->chunk, P, dcount);
        BFSX_LAUNCHED(st);
        hipLaunchKernelGGL(k_bucket_scatter, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                           (uint32_t)g->chunk, P, dcount, dcursor, d_send);
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
                           nullptr, nullptr, 0, nullptr, g->rank, g->nranks);
    else
        hipLaunchKernelGGL(k_claim_remote<int64_t>, grid, dim3(kBS), 0, st, d_recv, (u64)n, g->d_row_off,
                           ws->vis, ws->st, ws->qb, ws->ring, ws->d_level, (uint32_t)g->v_lo, (u64)0, (uint32_t)g->nv, ws->d_err,
                           nullptr, nullptr, 0, nullptr, g->rank, g->nranks);
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
             {"err", ws->d_err, 8},                      {"pub", ws->d_pub, (int64_t)sizeof(Published)}};
    for (const auto &x : b)
        fprintf(stderr, "[bfsx] rank %d level %d buffer %-8s [0x%llx, 0x%llx)\n", g->rank, level, x.name,
                (unsigned long long)(uintptr_t)x.p, (unsigned long long)((uintptr_t)x.p + x.bytes));
}

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
    BFSX_HIP_TRY(hipMemcpyAsync(counts.data(), b.cnt + 1, P * sizeof(u64), hipMemcpyDeviceToHost, st));
    if (int e = comm_sync(cm, st, "the degree-list all-gather")) return e;
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
        BFSX_HIP_TRY(hipMemcpyAsync(h.data(), b.all, h.size() * sizeof(u64), hipMemcpyDeviceToHost, st));
        if (int e = comm_sync(cm, st, "the degree-list all-gather")) return e;
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
    if (int e = cm->allreduce_sum(sums + 8, 4 + g->nranks, st)) return e;
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
        BFSX_HIP_TRY(hipMemcpyAsync(h, sums + 8, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        if (int e = comm_sync(cm, st, "the adjacency-count all-reduce")) return e;
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
        mf = opt.slot_pairs + 1;
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
    bool snapped = false; // ws->front holds the visited slice from before the last (top-down) level
    int td_levels = 0, bu_levels = 0;
    // the local bitmap frontier: ws->front after a push -> pull conversion, the last pull level's record after a
    // pull level; pull levels store 4-B parents plus their record, as on one device (RecLog, BfsWorkspace::par)
    const u64 *bmf = ws->front;
    RecLog recs(g, ws);
    std::vector<int64_t> rank_nf; // every rank's frontier size after the last level close (all-reduced)
    int64_t nf_core = -1;         // after a pull level: its local discoveries below leaf_lo (-1: unknown)
    ExchangePlan plan;
    std::vector<u64> hc(2 * kMaxRanks);
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
        const bool was_snapped = snapped;
        snapped = false;
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
            // a wide top-down level may hand over to bottom-up: snapshot the visited slice (see bfs_run)
            if (ws->d_mf >= ws->nwords / 4 && opt.direction == BFSX_DIR_AUTO) {
                BFSX_HIP_TRY(
                    hipMemcpyAsync(ws->front, ws->vis, ws->nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
                snapped = true;
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
            if (mf <= opt.slot_pairs) {
                // small level: no rank sends more than the global m_f pairs to any peer, so every peer gets
                // a fixed slot [count, m_f pairs] -- one exchange, no count all-to-all, no host wait.  The push
                // kernels write the pairs into the slots themselves; the last one's last workgroup writes the
                // counts (dcount, unused by the slot exchange, counts its arrivals)
                slot = std::max<int64_t>(mf, 1);
                if (int e = grow(ws, ws->sendbuf, ws->send_cap, P * (slot + 1))) return e;
                if (int e = grow(ws, ws->recvbuf, ws->recv_cap, P * (slot + 1))) return e;
                pt.slot_out = ws->sendbuf;
                pt.slot_cap = (u64)slot;
                pt.slot_cursor = dcursor;
                pt.slot_arrive = dcount;
                plan_slots(P, slot, plan, g->rank); // the own slot stays empty and is not exchanged
                ro = P * slot; // candidate entries the claim kernel reads
            }
            if (int e = check_live(g, ws, level, "push kernels",
                                   {{"queue in", ws->qa}, {"queue out", ws->qb}, {"hubs", ws->hubs}, {"vis", ws->vis},
                                    {"state", ws->st}, {"remote", pt.remote}, {"slot_out", pt.slot_out},
                                    {"counters", ws->d_dist_ctr}, {"front", ws->front}}))
                return e;
            if (int e = launch_td<true>(g, ws, nq, ws->d_mf, dmax_local, level, pt)) return e;
            if (!slot) {
                hipLaunchKernelGGL(k_bucket_count, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                                   (uint32_t)g->chunk, P, dcount);
                BFSX_LAUNCHED(st);
                hipLaunchKernelGGL(k_bucket_scatter, dim3(gbk), dim3(kBS), 0, st, ws->remote, ws->d_dist_ctr,
                                   (uint32_t)g->chunk, P, dcount, dcursor, ws->sendbuf);
                BFSX_LAUNCHED(st);
                u64 *drecv = ws->d_dist_ctr + kCtrRecv;
                if (int e = cm->alltoall1(reinterpret_cast<int64_t *>(dcount), reinterpret_cast<int64_t *>(drecv), st))
                    return e;
                if (int e = post_wait(ws, st, dcount, P, drecv, P, hc.data(), cm, "a pair-count exchange")) return e;
                hc[P + g->rank] = 0; // alltoall1 does not exchange the own entry (no pairs route to it)
                plan_counted(P, hc.data(), hc.data() + P, plan);
                ro = plan.recv_total;
                if (int e = grow(ws, ws->recvbuf, ws->recv_cap, std::max<int64_t>(ro, 1))) return e;
            }
            if (int e = check_live(g, ws, level, "pair exchange + claim",
                                   {{"sendbuf", ws->sendbuf}, {"recvbuf", ws->recvbuf}, {"remote", ws->remote}}))
                return e;
            if (int e = cm->alltoallv(ws->sendbuf, plan.scount.data(), plan.sdispl.data(), ws->recvbuf,
                                      plan.rcount.data(), plan.rdispl.data(), st))
                return e;
            if (ro > 0) { // its last workgroup closes the level (the sums k_level_sums would compute)
                const dim3 grid(clamp_grid((ro + kBS - 1) / kBS, cap));
                u64 *arrive = ws->d_dist_ctr + kCtrHead - 1;
                if (ws->off32)
                    hipLaunchKernelGGL(k_claim_remote<uint32_t>, grid, dim3(kBS), 0, st, ws->recvbuf, (u64)ro,
                                       ws->off32, ws->vis, ws->st, ws->qb, ws->ring, level, (uint32_t)g->v_lo,
                                       (u64)slot, (uint32_t)g->nv, ws->d_err, sums, ws->d_dist_ctr, kCtrHead, arrive,
                                       g->rank, g->nranks);
                else
                    hipLaunchKernelGGL(k_claim_remote<int64_t>, grid, dim3(kBS), 0, st, ws->recvbuf, (u64)ro,
                                       g->d_row_off, ws->vis, ws->st, ws->qb, ws->ring, level, (uint32_t)g->v_lo,
                                       (u64)slot, (uint32_t)g->nv, ws->d_err, sums, ws->d_dist_ctr, kCtrHead, arrive,
                                       g->rank, g->nranks);
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
            if (int e = cm->alltoallv(ws->sendbuf, plan.scount.data(), plan.sdispl.data(), ws->recvbuf,
                                      plan.rcount.data(), plan.rdispl.data(), st))
                return e;
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
            if (ws->d_in_queue) { // local queue -> bitmap slice
                if (was_snapped) { // front holds the visited slice from before the last top-down level
                    hipLaunchKernelGGL(k_new_bits, dim3(clamp_grid((ws->nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0,
                                       st, ws->vis, ws->nwords, ws->front);
                } else {
                    BFSX_HIP_TRY(hipMemsetAsync(ws->front, 0, ws->nwords * sizeof(u64), st));
                    hipLaunchKernelGGL(k_queue_to_bitmap, dim3(clamp_grid((ws->d_nf + kBS - 1) / kBS, cap)), dim3(kBS),
                                       0, st, ws->qa, (uint32_t)ws->d_nf, ws->front, (uint32_t)g->nv, ws->d_err);
                }
                BFSX_LAUNCHED(st);
                bmf = ws->front;
                ws->d_in_queue = false;
            }
            u64 *rec = nullptr;
            if (int e = recs.take(&rec)) return e;
            if (int e = check_live(g, ws, level, "frontier all-gather + pull kernel",
                                   {{"front", bmf}, {"fglob", ws->fglob}, {"record", rec}, {"vis", ws->vis},
                                    {"parents", ws->par}}))
                return e;
            if (int e = cm->allgather(bmf, ws->nwords, ws->fglob, st)) return e;
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
            return fail(BFSX_E_HIP, "queue guard fired at level " + std::to_string(level) + " on rank(s) " + who + mine);
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
        g->level_stats.push_back(ls);
        g->level_dirs.push_back(dir);
        examined += h[3];
        visited_local += h[0];
        if (td) std::swap(ws->qa, ws->qb);
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
        BFSX_HIP_TRY(hipMemcpyAsync(h, sums + 8, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        if (int e = comm_sync(cm, st, "the m_comp all-reduce")) return e;
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
