// kernels_bfs.hip -- the BFS hot path on the GPU (gfx950, wave64).
//
// Replaces the reference's per-level Spark job (BfsSpark.java:61-118):
//   mapper   (:66-87)  GRAY u emits (n, d+1) for n in N(u)          -> K3 top-down push  (k_td, k_td_hubs)
//   reducer  (:90-108) min distance / darkest colour per vertex id  -> fused: atomicOr claim on the
//                      visited bitmap; the single winner writes dist = level+1 (every contender of a
//                      level carries the same level+1, so the min is race-free and exact)
//   collect + contains("GRAY") (:110-117)                            -> K4 frontier count in a device
//                      counter ring, read back as one 64-B D2H per level
//   (no reference analogue)                                          -> K5 bottom-up pull (k_bu) with
//                      Beamer's direction-optimising switch
// State: dist int32[n] (INT32_MAX = WHITE), parent int32[n], visited bitmap u64[n/64] (BLACK|GRAY),
// frontier as a queue u32[] (top-down) or bitmap u64[] (bottom-up).
#include <algorithm>
#include <chrono>

#include "bfsx_internal.h"

namespace bfsx {

struct BfsWorkspace {
    int64_t nv = 0, nwords = 0;
    int32_t *dist = nullptr, *parent = nullptr;
    unsigned long long *vis = nullptr, *front = nullptr, *next = nullptr;
    uint32_t *qa = nullptr, *qb = nullptr, *hubs = nullptr;
    LevelCounters *ring = nullptr;   // device, 4 slots (3 ring + 1 scratch)
    LevelCounters *h_ring = nullptr; // pinned host mirror of one slot
    unsigned long long *d_red = nullptr; // reductions (m_comp, reached)
    hipEvent_t ev_start = nullptr;
    std::vector<hipEvent_t> ev_begin, ev_level; // per level: before / after its kernels
};

namespace {

constexpr int kBS = 256;
constexpr int kWaves = kBS / 64;

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

__device__ inline unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    return x;
}

// Claim vertex v in the visited bitmap.  A plain load first filters already-visited vertices (bits
// only ever get set, so a stale line can only under-report); the atomicOr decides the race.
__device__ inline bool try_claim(uint32_t v, unsigned long long *vis) {
    const unsigned long long bit = 1ull << (v & 63u);
    unsigned long long *w = vis + (v >> 6);
    if (*w & bit) return false;
    return !(atomicOr(w, bit) & bit);
}

// Wave-collective append of the winners to the next queue: one ballot, one atomic per wave.
// Must be called by all 64 lanes (wave-uniform control flow).
__device__ inline void wave_append(bool win, uint32_t v, unsigned long long vdeg, uint32_t *__restrict__ q,
                                   LevelCounters *c) {
    const unsigned long long mask = __ballot(win);
    if (mask == 0) return;
    const unsigned lane = lane_id();
    const int leader = __ffsll((long long)mask) - 1;
    const unsigned long long dsum = wave_sum(win ? vdeg : 0ull);
    uint32_t base = 0;
    if ((int)lane == leader) {
        base = (uint32_t)atomicAdd(&c->nf, (unsigned long long)__popcll(mask));
        atomicAdd(&c->mf, dsum);
    }
    base = __shfl(base, leader);
    if (win) q[base + __popcll(mask & ((1ull << lane) - 1ull))] = v;
}

__device__ inline void zero_slot(LevelCounters *ring, int level) {
    if (blockIdx.x == 0 && threadIdx.x < 8)
        reinterpret_cast<unsigned long long *>(ring + (level + 2) % 3)[threadIdx.x] = 0ull;
}

// ---- K2: source init (after memsets of dist / visited / counters) ------------------------------
__global__ void k_init_source(uint32_t s, const int64_t *__restrict__ row_off, int32_t *dist, int32_t *parent,
                              unsigned long long *vis, uint32_t *q, LevelCounters *ring) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        dist[s] = 0;
        parent[s] = (int32_t)s;
        vis[s >> 6] = 1ull << (s & 63u);
        q[0] = s;
        ring[0].nf = 1;
        ring[0].mf = (unsigned long long)(row_off[s + 1] - row_off[s]);
        ring[3].pad[0] = ring[0].mf;
    }
}

// ---- K3: top-down push, workgroup-balanced -----------------------------------------------------
// Each workgroup takes 256 frontier vertices, scans their degrees in LDS and sweeps the union of
// their adjacency rows edge-parallel (thread / wave / workgroup granularity in one pass: a thread
// finds its row by binary search in the LDS scan).  Vertices of degree > hub_deg go to the hub list
// and are swept by every workgroup in k_td_hubs (the multi-workgroup bin).
__global__ __launch_bounds__(kBS) void k_td(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const uint32_t *__restrict__ qin, uint32_t qlen,
                                            uint32_t *__restrict__ qout, unsigned long long *vis,
                                            int32_t *__restrict__ dist, int32_t *__restrict__ parent,
                                            LevelCounters *ring, int level, uint32_t hub_deg,
                                            uint32_t *__restrict__ hubs) {
    LevelCounters *cn = ring + (level + 1) % 3;
    zero_slot(ring, level);
    __shared__ uint32_t s_scan[kBS + 1];
    __shared__ int64_t s_beg[kBS];
    __shared__ uint32_t s_u[kBS];
    __shared__ uint32_t s_wsum[kWaves];
    const int32_t nd = level + 1;
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    for (uint32_t base = blockIdx.x * kBS; base < qlen; base += gridDim.x * kBS) {
        const uint32_t i = base + tid;
        uint32_t deg = 0, u = 0;
        int64_t beg = 0;
        if (i < qlen) {
            u = qin[i];
            beg = row_off[u];
            int64_t d = row_off[u + 1] - beg;
            if (d > (int64_t)hub_deg) {
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
        if (tid == 0) s_scan[kBS] = total;
        __syncthreads();
        for (uint32_t e0 = 0; e0 < total; e0 += kBS) {
            const uint32_t e = e0 + tid;
            bool win = false;
            uint32_t v = 0;
            unsigned long long vdeg = 0;
            if (e < total) {
                int lo = 0, hi = kBS - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_scan[mid] <= e) lo = mid;
                    else hi = mid - 1;
                }
                v = col[s_beg[lo] + (e - s_scan[lo])];
                if (try_claim(v, vis)) {
                    win = true;
                    dist[v] = nd;
                    parent[v] = (int32_t)s_u[lo];
                    vdeg = (unsigned long long)(row_off[v + 1] - row_off[v]);
                }
            }
            wave_append(win, v, vdeg, qout, cn);
        }
        __syncthreads();
    }
}

// Multi-workgroup bin: every workgroup sweeps a strided slice of each hub's row.
__global__ __launch_bounds__(kBS) void k_td_hubs(const int64_t *__restrict__ row_off,
                                                 const uint32_t *__restrict__ col,
                                                 const uint32_t *__restrict__ hubs, uint32_t *__restrict__ qout,
                                                 unsigned long long *vis, int32_t *__restrict__ dist,
                                                 int32_t *__restrict__ parent, LevelCounters *ring, int level) {
    LevelCounters *cn = ring + (level + 1) % 3;
    const uint32_t nh = (uint32_t)cn->nhub;
    const int32_t nd = level + 1;
    for (uint32_t h = 0; h < nh; h++) {
        const uint32_t u = hubs[h];
        const int64_t beg = row_off[u], deg = row_off[u + 1] - beg;
        for (int64_t e0 = (int64_t)blockIdx.x * kBS; e0 < deg; e0 += (int64_t)gridDim.x * kBS) {
            const int64_t e = e0 + threadIdx.x;
            bool win = false;
            uint32_t v = 0;
            unsigned long long vdeg = 0;
            if (e < deg) {
                v = col[beg + e];
                if (try_claim(v, vis)) {
                    win = true;
                    dist[v] = nd;
                    parent[v] = (int32_t)u;
                    vdeg = (unsigned long long)(row_off[v + 1] - row_off[v]);
                }
            }
            wave_append(win, v, vdeg, qout, cn);
        }
    }
}

// ---- K5: bottom-up pull --------------------------------------------------------------------------
// One wave owns one 64-vertex word of the visited bitmap: lane l handles vertex 64w+l, so the
// visited word is one broadcast load, row offsets are a coalesced 512-B read, and the new frontier
// word / visited word are written by one lane without atomics.  Each unvisited vertex scans its row
// until it finds a neighbour in the current frontier bitmap.
__global__ __launch_bounds__(kBS) void k_bu(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const unsigned long long *__restrict__ front,
                                            unsigned long long *__restrict__ next,
                                            unsigned long long *__restrict__ vis, int32_t *__restrict__ dist,
                                            int32_t *__restrict__ parent, LevelCounters *ring, int level,
                                            int64_t nwords, int64_t nv) {
    LevelCounters *cn = ring + (level + 1) % 3;
    zero_slot(ring, level);
    __shared__ unsigned long long s_nf[kWaves], s_mf[kWaves], s_sc[kWaves];
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const int32_t nd = level + 1;
    unsigned long long acc_nf = 0, acc_mf = 0, acc_sc = 0;
    for (int64_t w = (int64_t)blockIdx.x * kWaves + wave; w < nwords; w += (int64_t)gridDim.x * kWaves) {
        const unsigned long long vw = vis[w];
        const int64_t v = w * 64 + lane;
        bool found = false;
        uint32_t par = 0;
        unsigned long long deg = 0, scanned = 0;
        if (v < nv && !((vw >> lane) & 1ull)) {
            const int64_t b = row_off[v], e = row_off[v + 1];
            deg = (unsigned long long)(e - b);
            int64_t j = b;
            for (; j < e; j++) {
                const uint32_t x = col[j];
                if ((front[x >> 6] >> (x & 63u)) & 1ull) {
                    found = true;
                    par = x;
                    j++;
                    break;
                }
            }
            scanned = (unsigned long long)(j - b);
        }
        const unsigned long long fm = __ballot(found);
        if (found) {
            dist[v] = nd;
            parent[v] = (int32_t)par;
        }
        if (lane == 0) {
            next[w] = fm;
            if (fm) vis[w] = vw | fm;
        }
        acc_nf += (unsigned long long)__popcll(fm);
        acc_mf += wave_sum(found ? deg : 0ull);
        acc_sc += scanned;
    }
    acc_sc = wave_sum(acc_sc);
    if (lane == 0) {
        s_nf[wave] = acc_nf;
        s_mf[wave] = acc_mf;
        s_sc[wave] = acc_sc;
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long a = 0, b = 0, c = 0;
#pragma unroll
        for (int i = 0; i < kWaves; i++) {
            a += s_nf[i];
            b += s_mf[i];
            c += s_sc[i];
        }
        if (a) {
            atomicAdd(&cn->nf, a);
            atomicAdd(&cn->mf, b);
        }
        if (c) atomicAdd(&cn->scanned, c);
    }
}

// ---- K4: frontier representation changes -------------------------------------------------------
__global__ __launch_bounds__(kBS) void k_queue_to_bitmap(const uint32_t *__restrict__ q, uint32_t qlen,
                                                         unsigned long long *bm) {
    for (uint32_t i = blockIdx.x * kBS + threadIdx.x; i < qlen; i += gridDim.x * kBS) {
        const uint32_t v = q[i];
        atomicOr(bm + (v >> 6), 1ull << (v & 63u));
    }
}

// Ballot/popcount compaction: each lane owns one bitmap word; a wave prefix of the popcounts gives
// each lane its write offset; one atomic per wave reserves the wave's range.
__global__ __launch_bounds__(kBS) void k_bitmap_to_queue(const unsigned long long *__restrict__ bm, int64_t nwords,
                                                         uint32_t *__restrict__ q, unsigned long long *cursor) {
    const unsigned lane = lane_id();
    for (int64_t w0 = (int64_t)blockIdx.x * kBS; w0 < nwords; w0 += (int64_t)gridDim.x * kBS) {
        const int64_t w = w0 + threadIdx.x;
        unsigned long long x = (w < nwords) ? bm[w] : 0ull;
        const uint32_t c = (uint32_t)__popcll(x);
        const uint32_t inc = wave_incl_scan(c);
        const uint32_t tot = __shfl(inc, 63);
        uint32_t base = 0;
        if (lane == 63 && tot) base = (uint32_t)atomicAdd(cursor, (unsigned long long)tot);
        base = __shfl(base, 63);
        uint32_t p = base + inc - c;
        while (x) {
            const int b = __ffsll((long long)x) - 1;
            q[p++] = (uint32_t)(w * 64 + b);
            x &= x - 1ull;
        }
    }
}

// m_comp (Graph500 TEPS numerator) and reached count, outside the timed region.
__global__ __launch_bounds__(kBS) void k_mcomp(const int32_t *__restrict__ dist, const uint32_t *__restrict__ tcnt,
                                               int64_t nv, unsigned long long *out) {
    unsigned long long m = 0, r = 0;
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS) {
        if (dist[v] != INT32_MAX) {
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

unsigned clamp_grid(int64_t blocks, unsigned cap) {
    if (blocks < 1) blocks = 1;
    return (unsigned)std::min<int64_t>(blocks, cap);
}

int ws_alloc(bfsx_graph *g) {
    if (g->ws) return BFSX_OK;
    auto *ws = new BfsWorkspace();
    g->ws = ws;
    ws->nv = g->nv;
    ws->nwords = (g->nv + 63) / 64;
    const size_t nv = (size_t)std::max<int64_t>(g->nv, 1);
    BFSX_HIP_TRY(hipMalloc(&ws->dist, nv * sizeof(int32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->parent, nv * sizeof(int32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->vis, ws->nwords * sizeof(unsigned long long)));
    BFSX_HIP_TRY(hipMalloc(&ws->front, ws->nwords * sizeof(unsigned long long)));
    BFSX_HIP_TRY(hipMalloc(&ws->next, ws->nwords * sizeof(unsigned long long)));
    BFSX_HIP_TRY(hipMalloc(&ws->qa, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->qb, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->hubs, nv * sizeof(uint32_t)));
    BFSX_HIP_TRY(hipMalloc(&ws->ring, 4 * sizeof(LevelCounters)));
    BFSX_HIP_TRY(hipHostMalloc(&ws->h_ring, sizeof(LevelCounters), hipHostMallocDefault));
    BFSX_HIP_TRY(hipMalloc(&ws->d_red, 2 * sizeof(unsigned long long)));
    BFSX_HIP_TRY(hipEventCreate(&ws->ev_start));
    return BFSX_OK;
}

} // namespace

void bfs_workspace_free(BfsWorkspace *ws) {
    if (!ws) return;
    for (void *p : {(void *)ws->dist, (void *)ws->parent, (void *)ws->vis, (void *)ws->front, (void *)ws->next,
                    (void *)ws->qa, (void *)ws->qb, (void *)ws->hubs, (void *)ws->ring, (void *)ws->d_red})
        if (p) (void)hipFree(p);
    if (ws->h_ring) (void)hipHostFree(ws->h_ring);
    if (ws->ev_start) (void)hipEventDestroy(ws->ev_start);
    for (auto e : ws->ev_level) (void)hipEventDestroy(e);
    for (auto e : ws->ev_begin) (void)hipEventDestroy(e);
    delete ws;
}

int bfs_run(bfsx_graph *g, int64_t source, bfsx_stats *stats) {
    if (source < 0 || source >= g->nv)
        return fail(BFSX_E_RANGE, "source vertex " + std::to_string(source) + " outside [0, " +
                                      std::to_string(g->nv) + ")");
    int rc = ws_alloc(g);
    if (rc) return rc;
    BfsWorkspace *ws = g->ws;
    bfsx_ctx *ctx = g->ctx;
    hipStream_t st = ctx->stream;
    const Options &opt = ctx->opt;
    const int64_t nv = g->nv, nwords = ws->nwords;
    const unsigned cap = (unsigned)ctx->num_cus * 8u;

    // ---- timed region: source init -> last level ----
    BFSX_HIP_TRY(hipEventRecord(ws->ev_start, st));
    BFSX_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)ws->dist, 0x7FFFFFFF, (size_t)nv, st));
    BFSX_HIP_TRY(hipMemsetAsync(ws->vis, 0, nwords * sizeof(unsigned long long), st));
    BFSX_HIP_TRY(hipMemsetAsync(ws->ring, 0, 4 * sizeof(LevelCounters), st));
    hipLaunchKernelGGL(k_init_source, dim3(1), dim3(64), 0, st, (uint32_t)source, g->d_row_off, ws->dist,
                       ws->parent, ws->vis, ws->qa, ws->ring);
    BFSX_HIP_TRY(hipGetLastError());

    int dir = (opt.direction == BFSX_DIR_BOTTOMUP) ? BFSX_DIR_BOTTOMUP : BFSX_DIR_TOPDOWN;
    bool in_queue = true; // frontier currently held in ws->qa (else in ws->front)
    int64_t nf = 1, prev_nf = 0;
    int64_t mf = -1;      // unknown for the source frontier (no host sync before level 0)
    int64_t mu = g->nnz;  // Beamer m_u: adjacency entries of unvisited vertices
    int64_t examined = 0, visited = 1;
    int td_levels = 0, bu_levels = 0;
    g->level_dirs.clear();
    g->level_cum_ms.clear();
    g->level_stats.clear();
    int level = 0;
    for (;; level++) {
        if (opt.direction == BFSX_DIR_AUTO && level > 0) {
            if (dir == BFSX_DIR_TOPDOWN) {
                if (mf > mu / std::max(opt.alpha, 1)) dir = BFSX_DIR_BOTTOMUP;
            } else if (nf < nv / std::max(opt.beta, 1) && nf < prev_nf) {
                dir = BFSX_DIR_TOPDOWN;
            }
        }
        if ((int)ws->ev_level.size() <= level) {
            hipEvent_t e0, e1;
            BFSX_HIP_TRY(hipEventCreate(&e0));
            BFSX_HIP_TRY(hipEventCreate(&e1));
            ws->ev_begin.push_back(e0);
            ws->ev_level.push_back(e1);
        }
        BFSX_HIP_TRY(hipEventRecord(ws->ev_begin[level], st));
        if (dir == BFSX_DIR_BOTTOMUP && in_queue) {
            BFSX_HIP_TRY(hipMemsetAsync(ws->front, 0, nwords * sizeof(unsigned long long), st));
            hipLaunchKernelGGL(k_queue_to_bitmap, dim3(clamp_grid((nf + kBS - 1) / kBS, cap)), dim3(kBS), 0, st,
                               ws->qa, (uint32_t)nf, ws->front);
            BFSX_HIP_TRY(hipGetLastError());
            in_queue = false;
        } else if (dir == BFSX_DIR_TOPDOWN && !in_queue) {
            BFSX_HIP_TRY(hipMemsetAsync(&ws->ring[3].aux, 0, sizeof(unsigned long long), st));
            hipLaunchKernelGGL(k_bitmap_to_queue, dim3(clamp_grid((nwords + kBS - 1) / kBS, cap)), dim3(kBS), 0,
                               st, ws->front, nwords, ws->qa, &ws->ring[3].aux);
            BFSX_HIP_TRY(hipGetLastError());
            in_queue = true;
        }
        if (dir == BFSX_DIR_TOPDOWN) {
            hipLaunchKernelGGL(k_td, dim3(clamp_grid((nf + kBS - 1) / kBS, cap)), dim3(kBS), 0, st, g->d_row_off,
                               g->d_col, ws->qa, (uint32_t)nf, ws->qb, ws->vis, ws->dist, ws->parent, ws->ring,
                               level, opt.hub_degree, ws->hubs);
            BFSX_HIP_TRY(hipGetLastError());
            if (mf < 0 || mf > (int64_t)opt.hub_degree) {
                hipLaunchKernelGGL(k_td_hubs, dim3(cap), dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->hubs, ws->qb,
                                   ws->vis, ws->dist, ws->parent, ws->ring, level);
                BFSX_HIP_TRY(hipGetLastError());
            }
            td_levels++;
        } else {
            hipLaunchKernelGGL(k_bu, dim3(clamp_grid((nwords + kWaves - 1) / kWaves, cap)), dim3(kBS), 0, st,
                               g->d_row_off, g->d_col, ws->front, ws->next, ws->vis, ws->dist, ws->parent,
                               ws->ring, level, nwords, nv);
            BFSX_HIP_TRY(hipGetLastError());
            bu_levels++;
        }
        BFSX_HIP_TRY(hipEventRecord(ws->ev_level[level], st));
        BFSX_HIP_TRY(hipMemcpyAsync(ws->h_ring, ws->ring + (level + 1) % 3, sizeof(LevelCounters),
                                    hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        g->level_dirs.push_back(dir);
        const int64_t nf_new = (int64_t)ws->h_ring->nf, mf_new = (int64_t)ws->h_ring->mf;
        bfsx_level_stat ls{};
        ls.direction = dir;
        ls.level = level;
        ls.frontier_in = nf;
        ls.frontier_out = nf_new;
        ls.mf_in = mf;
        ls.unvisited_in = nv - visited;
        ls.scanned = (dir == BFSX_DIR_TOPDOWN) ? mf : (int64_t)ws->h_ring->scanned;
        g->level_stats.push_back(ls);
        if (dir == BFSX_DIR_TOPDOWN) examined += (mf < 0 ? 0 : mf);
        else examined += (int64_t)ws->h_ring->scanned;
        visited += nf_new;
        mu -= mf_new;
        prev_nf = nf;
        nf = nf_new;
        mf = mf_new;
        if (dir == BFSX_DIR_TOPDOWN) std::swap(ws->qa, ws->qb);
        else std::swap(ws->front, ws->next);
        if (nf == 0) break;
    }
    const int levels = level + 1;
    float ms = 0.f;
    BFSX_HIP_TRY(hipEventElapsedTime(&ms, ws->ev_start, ws->ev_level[level]));
    g->level_cum_ms.resize(levels);
    for (int l = 0; l < levels; l++) {
        float t = 0.f, k = 0.f;
        BFSX_HIP_TRY(hipEventElapsedTime(&t, ws->ev_start, ws->ev_level[l]));
        BFSX_HIP_TRY(hipEventElapsedTime(&k, ws->ev_begin[l], ws->ev_level[l]));
        g->level_cum_ms[l] = t;
        g->level_stats[l].cum_ms = t;
        g->level_stats[l].kernel_ms = k;
    }
    if (!g->level_stats.empty() && g->level_stats[0].mf_in < 0) {
        // the source's degree was written by k_init_source into the scratch slot
        unsigned long long d0 = 0;
        BFSX_HIP_TRY(hipMemcpy(&d0, &ws->ring[3].pad[0], sizeof(d0), hipMemcpyDeviceToHost));
        g->level_stats[0].mf_in = (int64_t)d0;
        if (g->level_stats[0].direction == BFSX_DIR_TOPDOWN) {
            g->level_stats[0].scanned = (int64_t)d0;
            examined += (int64_t)d0;
        }
    }
    g->last_source = source;
    if (stats) {
        stats->levels = levels;
        stats->topdown_levels = td_levels;
        stats->bottomup_levels = bu_levels;
        stats->t_bfs_ms = ms;
        stats->edges_examined = examined;
    }
    return BFSX_OK;
}

int bfs_mcomp(bfsx_graph *g, int64_t *m_comp, int64_t *reached) {
    BfsWorkspace *ws = g->ws;
    hipStream_t st = g->ctx->stream;
    unsigned long long h[2] = {0, 0};
    BFSX_HIP_TRY(hipMemsetAsync(ws->d_red, 0, 2 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_mcomp, dim3(clamp_grid((g->nv + kBS - 1) / kBS, 2048)), dim3(kBS), 0, st, ws->dist,
                       g->d_tuple_cnt, g->nv, ws->d_red);
    BFSX_HIP_TRY(hipGetLastError());
    BFSX_HIP_TRY(hipMemcpyAsync(h, ws->d_red, sizeof(h), hipMemcpyDeviceToHost, st));
    BFSX_HIP_TRY(hipStreamSynchronize(st));
    *m_comp = (int64_t)h[0];
    *reached = (int64_t)h[1];
    return BFSX_OK;
}

int bfs_copy_result(bfsx_graph *g, int32_t *dist_out, int64_t *parent_out) {
    BfsWorkspace *ws = g->ws;
    if (!ws || g->last_source < 0) return fail(BFSX_E_ARG, "no BFS result on this graph yet");
    hipStream_t st = g->ctx->stream;
    const size_t nv = (size_t)g->nv;
    std::vector<int32_t> dtmp;
    int32_t *dist = dist_out;
    if (!dist) {
        dtmp.resize(nv);
        dist = dtmp.data();
    }
    BFSX_HIP_TRY(hipMemcpyAsync(dist, ws->dist, nv * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (parent_out) {
        // int32 device parents land in the upper half of the int64 output, then widen in place
        int32_t *p32 = reinterpret_cast<int32_t *>(parent_out) + nv;
        BFSX_HIP_TRY(hipMemcpyAsync(p32, ws->parent, nv * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        BFSX_HIP_TRY(hipStreamSynchronize(st));
        for (size_t i = 0; i < nv; i++) parent_out[i] = (dist[i] == INT32_MAX) ? -1 : (int64_t)p32[i];
    } else {
        BFSX_HIP_TRY(hipStreamSynchronize(st));
    }
    return BFSX_OK;
}

} // namespace bfsx
