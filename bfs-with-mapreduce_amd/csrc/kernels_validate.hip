// kernels_validate.hip -- Graph500-style validation of a BFS result on the GPU, at full size.
//
// The north star asks for distances bit-exact against the reference and parent trees that pass
// Graph500-style validation.  The CPU oracle (oracle/oracle.c, orc_validate) checks both up to a few
// million edges; at the benchmark sizes (scale 26: 2.1 G adjacency entries; scale 30: 34 G over 8
// ranks) this kernel checks the same rules on the device, one edge-parallel pass over the CSR:
//   (1) dist[src] = 0 and parent[src] = src;
//   (2) a reached v != src has a parent p with dist[p] = dist[v] - 1, and p is in v's neighbour set
//       (the tree edge exists: Graph500 rule 3, BreadthFirstPaths.check, algs4.jar!/BreadthFirstPaths.java:171-212);
//   (3) an unreached v has no parent and no reached neighbour (the tree spans the component);
//   (4) every edge (v, w) joins two reached vertices whose distances differ by at most one.
// (1)+(2) give dist[v] >= the true distance (dist is the length of a real path), (3)+(4) give
// dist[v] <= it (induction along a shortest path), so a result that passes has EXACTLY the BFS
// distances of the graph -- the reference's per-vertex distances (BfsSpark.java:100, min over the
// level's emissions) -- and a valid BFS tree.  The parent choice itself is not compared: the
// reference's tie-break depends on Spark's shuffle order (BfsSpark.java:97).
//
// Partitioned graphs: every rank all-gathers the distances (int32 per vertex, chunk per rank) and
// checks its own rows; the error counts are all-reduced.
#include <algorithm>

#include "bfsx_internal.h"

namespace bfsx {

namespace {

using u64 = unsigned long long;
constexpr int kBS = 256;

// dist of every local row (slice of `chunk` int32, padding rows unreached)
__global__ __launch_bounds__(kBS) void k_val_dist(const u64 *__restrict__ stt, int64_t nv, int64_t chunk,
                                                  int32_t *__restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < chunk; v += (int64_t)gridDim.x * kBS)
        out[v] = v < nv ? (int32_t)(uint32_t)stt[v] : INT32_MAX;
}

// One wave per row (grid-stride).  out[0] = violating vertices, out[1] = smallest violating global id,
// out[2] = reached vertices, out[3] = adjacency entries checked.
__global__ __launch_bounds__(kBS) void k_validate(const int64_t *__restrict__ row_off, const uint32_t *__restrict__ col,
                                                  const u64 *__restrict__ stt, const int32_t *__restrict__ dglob,
                                                  int64_t nv, int64_t lo, int64_t nglob, int64_t src,
                                                  u64 *__restrict__ out) {
    const unsigned lane = threadIdx.x & 63u;
    const int64_t wave = ((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBS) >> 6;
    u64 bad_n = 0, reached = 0, edges = 0, first = ~0ull;
    for (int64_t v = wave; v < nv; v += nwaves) {
        const u64 s = stt[v];
        const int32_t dv = (int32_t)(uint32_t)s;
        const uint32_t pv = (uint32_t)(s >> 32);
        const int64_t gid = lo + v;
        const int64_t beg = row_off[v], end = row_off[v + 1];
        bool bad = false, seen_parent = false;
        if (gid == src) {
            bad = dv != 0 || (int64_t)pv != gid;
        } else if (dv == INT32_MAX) {
            bad = pv != 0xFFFFFFFFu;
        } else {
            bad = dv <= 0 || (int64_t)pv >= nglob || dglob[pv] != dv - 1;
        }
        for (int64_t e = beg + lane; e < end; e += 64) {
            const uint32_t w = col[e];
            const int32_t dw = (int64_t)w < nglob ? dglob[w] : -1;
            if (dv == INT32_MAX) {
                bad |= dw != INT32_MAX;
            } else {
                bad |= dw == INT32_MAX || dw < 0 || dw < dv - 1 || dw > dv + 1;
                seen_parent |= w == pv;
            }
        }
        if (gid != src && dv != INT32_MAX && __ballot(seen_parent) == 0) bad = true;
        bad = __ballot(bad) != 0;
        if (lane == 0) {
            bad_n += bad;
            if (bad && (u64)gid < first) first = (u64)gid;
            reached += dv != INT32_MAX;
            edges += (u64)(end - beg);
        }
    }
    if (lane == 0 && (bad_n | reached | edges)) {
        if (bad_n) {
            atomicAdd(out, bad_n);
            atomicMin(out + 1, first);
        }
        atomicAdd(out + 2, reached);
        atomicAdd(out + 3, edges);
    }
}

} // namespace

int bfs_validate(bfsx_graph *g, int64_t source, const unsigned long long *stt, int64_t res[4]) {
    if (!stt) {
        if (int e = bfs_resolve(g)) return e;
        stt = bfs_state(g);
        if (!stt || g->last_source < 0) return fail(BFSX_E_ARG, "no BFS result on this graph yet");
        if (source < 0) source = g->last_source;
    }
    // a partition's non-owning ranks of a relabelled graph pass nv_global (the source is none of their rows)
    if (source < 0 || source > (g->nranks > 1 ? g->nv_global : g->nv - 1)) return fail(BFSX_E_ARG, "source out of range");
    const bool part = g->nranks > 1;
    Comm *cm = g->ctx->comm.get();
    if (part && (!cm || cm->nranks != g->nranks || cm->rank != g->rank))
        return fail(BFSX_E_ARG, "partitioned graph: attach a communicator first (validation is collective)");
    hipStream_t st = g->ctx->stream;
    const int64_t chunk = part ? g->chunk : g->nv;
    const int64_t nglob = part ? g->chunk * g->nranks : g->nv;
    struct Buf {
        void *p = nullptr;
        ~Buf() {
            if (p) (void)hipFree(p);
        }
    } slice, glob, red;
    // the local slice is padded to an even number of int32 so it travels as u64 words
    const int64_t cpad = (chunk + 1) & ~(int64_t)1;
    BFSX_HIP_TRY(hipMalloc(&slice.p, cpad * sizeof(int32_t)));
    BFSX_HIP_TRY(hipMalloc(&red.p, 4 * sizeof(u64)));
    const unsigned gfill = (unsigned)std::min<int64_t>(std::max<int64_t>((cpad + kBS - 1) / kBS, 1), 8192);
    hipLaunchKernelGGL(k_val_dist, dim3(gfill), dim3(kBS), 0, st, stt, g->nv, cpad, (int32_t *)slice.p);
    BFSX_HIP_TRY(hipGetLastError());
    const int32_t *dglob = (const int32_t *)slice.p;
    if (part) {
        if (cpad != chunk) return fail(BFSX_E_ARG, "partition chunk must be even");
        BFSX_HIP_TRY(hipMalloc(&glob.p, nglob * sizeof(int32_t)));
        if (int e = cm->allgather((const u64 *)slice.p, chunk / 2, (u64 *)glob.p, st)) return e;
        dglob = (const int32_t *)glob.p;
    }
    const u64 init[4] = {0, ~0ull, 0, 0};
    BFSX_HIP_TRY(hipMemcpyAsync(red.p, init, sizeof(init), hipMemcpyHostToDevice, st));
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>((g->nv * 64 + kBS - 1) / kBS, 1),
                                                      (int64_t)g->ctx->num_cus * 32);
    hipLaunchKernelGGL(k_validate, dim3(grid), dim3(kBS), 0, st, g->d_row_off, g->d_col, stt, dglob, g->nv, g->v_lo,
                       nglob, source, (u64 *)red.p);
    BFSX_HIP_TRY(hipGetLastError());
    u64 h[4];
    if (int e = comm_fetch(part ? cm : nullptr, st, h, red.p, sizeof(h), "the validation's distance all-gather"))
        return e;
    res[0] = (int64_t)h[0];
    res[1] = h[1] == ~0ull ? -1 : (int64_t)h[1];
    res[2] = (int64_t)h[2];
    res[3] = (int64_t)h[3];
    if (part) {
        // one all-reduce: the three counts, and per rank its smallest bad id + 1 (0 = none) in its own
        // slot; ranks own ascending id ranges, so the first nonzero slot holds the global minimum
        int64_t *d = nullptr;
        BFSX_HIP_TRY(hipMalloc(&d, (3 + g->nranks) * sizeof(int64_t)));
        std::vector<int64_t> v(3 + g->nranks, 0);
        v[0] = res[0];
        v[1] = res[2];
        v[2] = res[3];
        v[3 + g->rank] = res[1] + 1; // 0 = none
        BFSX_HIP_TRY(hipMemcpyAsync(d, v.data(), v.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
        int e = cm->allreduce_sum(d, (int)v.size(), st);
        if (!e) e = comm_fetch(cm, st, v.data(), d, v.size() * sizeof(int64_t), "the validation's all-reduce");
        (void)hipFree(d);
        if (e) return e;
        res[0] = v[0];
        res[2] = v[1];
        res[3] = v[2];
        res[1] = -1;
        for (int r = 0; r < g->nranks; r++)
            if (v[3 + r] > 0) {
                res[1] = v[3 + r] - 1;
                break;
            }
    }
    return BFSX_OK;
}

} // namespace bfsx
