// kernels_push.hip -- top-down push levels (the reference's mapper, BfsSpark.java:66-87, with the reducer
// :90-108 fused in as a visited-bitmap claim): k_td (vertex groups of degree <= hub_degree) and k_td_hubs (the
// multi-workgroup bin of the higher-degree rows), single device and partitioned (kDist: remote targets become
// owner-routed pairs).
#include "bfs_core.h"

namespace bfsx {

namespace {

constexpr uint32_t kVisPref = 1u << 16; // ids whose visited bits the hub bin snapshots into LDS (8 KiB)

// Sweep edges [x_begin, x_end) of a segment table (scan/beg/u in LDS, n entries; u = local row id)
// in steps of kBS*kItems.  Block-uniform.  kDist: targets owned by another rank become remote pairs.
// par != null (the push half of a hybrid level): a winner's parent also goes to the 4-B parent array, because the
// level's discoveries are merged into the pull half's level record, whose vertices take their parent from there
// (provenance code kCodeExplicit in pcode).
// s_vp / vpref (the hub bin of a relabelled single-device graph, option hub_lds_skip): the visited bits of ids below
// vpref as they stood when the level began, in LDS.  A target whose bit is set there needs no global probe -- on the
// hub-core level most edges of a degree-ordered hub row start with other hubs, visited a level earlier.
__device__ __forceinline__ uint32_t vl_of(uint32_t v, const Part &pt) { return v - pt.lo; }

template <bool kDist, class OffT, class ScanT, class BegT, class Q>
__device__ inline void sweep_segments(const ScanT *s_scan, const BegT *s_beg, const uint32_t *s_u, int n,
                                      uint64_t x_begin, uint64_t x_end, const OffT *__restrict__ row_off,
                                      const uint32_t *__restrict__ col, u64 *vis, u64 *__restrict__ stt,
                                      uint32_t *__restrict__ par, uint8_t *__restrict__ pcode, int32_t nd, Q &q, uint32_t *__restrict__ qout, u64 *qtail,
                                      const Part &pt, RemoteQueue *rq, u64 &acc_mf, u64 &attempts, u64 &acc_dmax,
                                      HubSet hs, u64 &acc_mfh, u64 &acc_nh, u64 &acc_ex, u64 *__restrict__ plog,
                                      const u64 *s_vp = nullptr, uint32_t vpref = 0u) {
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
                v[k] = col[(int64_t)s_beg[lo] + (int64_t)(x - (uint64_t)s_scan[lo])];
                pu[k] = s_u[lo] + pt.lo; // global id of the frontier vertex
            }
        }
#pragma unroll
        for (int k = 0; k < kItems; k++) {
            bool win = false, send = false;
            uint32_t vl = v[k];
            if (kDist) {
                send = valid[k] && vl_of(v[k], pt) >= pt.chunk; // outside this rank's id range [lo, lo + chunk)
                vl = v[k] - pt.lo;
            }
            const bool known = vpref && vl < vpref && ((s_vp[vl >> 6] >> (vl & 63u)) & 1ull);
            if (valid[k] && !send && !known && claim(vl, vis, attempts)) {
                win = true;
                // the push log (single device) or the hybrid level's parent array + record carry the result;
                // else the packed state
                if (par) {
                    par[vl] = pu[k];
                    if (pcode) pcode[vl] = kCodeExplicit;
                    acc_ex++;
                }
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
        if (q.n > Q::kCap - (uint32_t)(kBS * kItems)) q_flush(q, qout, plog, qtail, pt.qcap, pt.err);
        if (kDist && rq->n > (uint32_t)(kRCap - kBS * kItems)) rq_flush(*rq, pt);
    }
}

template <bool kDist, class OffT>
__global__ __launch_bounds__(kBS) void k_td(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const uint32_t *__restrict__ qin, uint32_t qlen,
                                            uint32_t *__restrict__ qout, u64 *vis, u64 *__restrict__ stt,
                                            uint32_t *__restrict__ par, uint8_t *__restrict__ pcode, LevelSlot *ring,
                                            int level, uint32_t hub_deg,
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
    if (BFSX_DIAG_ON && pt.probe && threadIdx.x < 64) // option race_probe: wave 0 zeroes the counts late
        for (int i = 0; i < 64; i++) __builtin_amdgcn_s_sleep(127);
    bq_init(q);
    if (kDist && threadIdx.x == 0) rq->n = 0;
    // Every wave must see the zeroed queue counts before it reads them.  A workgroup with no frontier vertex (a
    // partitioned rank whose local frontier is empty: every non-owner at level 0) goes straight to the final
    // flushes; without this barrier waves 1-3 could read q.n / rq->n before wave 0 zeroed them -- whatever an
    // earlier kernel left in that LDS -- and flush that many stale entries to a stale base: the round-3..5
    // "illegal memory access" of the partitioned push levels (event (d)).
    if (!(BFSX_DIAG_ON && pt.probe == 2)) __syncthreads(); // race_probe=nobarrier: the rounds-3..5 code

    const int32_t nd = level + 1;
    const unsigned tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    u64 acc_mf = 0, attempts = 0, scanned = 0, acc_dmax = 0, acc_mfh = 0, acc_nh = 0, acc_ex = 0;
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
                const u64 h = atomicAdd(&cn->nhub, 1ull); // the list holds nrows ids (a vertex is queued once)
                if (idx_ok(h, pt.nrows, pt.err, kSiteHubs)) hubs[h] = u;
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
        sweep_segments<kDist>(s_scan, s_beg, s_u, gsz, 0, total, row_off, col, vis, stt, par, pcode, nd, q, qout, &cn->qtail, pt,
                              rq, acc_mf, attempts, acc_dmax, hs, acc_mfh, acc_nh, acc_ex, plog);
        __syncthreads();
    }
    q_flush(q, qout, plog, &cn->qtail, pt.qcap, pt.err);
    if (kDist) rq_flush(*rq, pt);
    // top-down: stage2 = degree sum of the hub-domain vertices discovered, walked = their number
    shard_add(cn, 0, acc_mf, scanned, attempts, 0, acc_dmax, acc_mfh, acc_nh, acc_ex);
    publish_if_last(cn, pub, seq);
    if (kDist) slot_headers_if_last(pt);
}

template <bool kDist, class OffT>
__global__ __launch_bounds__(kBS) void k_td_hubs(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                                 const uint32_t *__restrict__ hubs, uint32_t *__restrict__ qout,
                                                 u64 *vis, u64 *__restrict__ stt, uint32_t *__restrict__ par,
                                                 uint8_t *__restrict__ pcode, LevelSlot *ring, int level,
                                                 Part pt, HubSet hs, Published *pub, u64 seq, u64 *__restrict__ plog,
                                                 uint32_t vpref) {
    LevelSlot *cn = ring + (level + 1) % 3;
    // single device: the level's starting visited bits of the ids below vpref (hub_lds_skip); 8 KiB of LDS
    __shared__ typename std::conditional<kDist, char, u64[kVisPref / 64]>::type s_vp_storage;
    const u64 *s_vp = nullptr;
    if constexpr (!kDist) {
        for (uint32_t w = threadIdx.x; w < vpref / 64u; w += kBS) s_vp_storage[w] = vis[w];
        s_vp = s_vp_storage;
    } else {
        vpref = 0u;
    }
    // 32-bit row offsets (nnz < 2^32) make every edge prefix and row start of a batch fit 32 bits: half the LDS
    // of 64-bit ones, which keeps 4 workgroups per CU beside the queues (and the hub_lds_skip snapshot)
    using ScanT = typename std::conditional<sizeof(OffT) == 4, uint32_t, u64>::type;
    using BegT = typename std::conditional<sizeof(OffT) == 4, uint32_t, int64_t>::type;
    __shared__ ScanT s_scan[kHubBatch + 1];
    __shared__ BegT s_beg[kHubBatch];
    __shared__ uint32_t s_u[kHubBatch];
    __shared__ u64 s_tsum[kBS];
    __shared__ typename std::conditional<kDist, DistQueue, LogQueue>::type q;
    __shared__ typename std::conditional<kDist, RemoteQueue, char>::type rq_storage;
    RemoteQueue *rq = kDist ? reinterpret_cast<RemoteQueue *>(&rq_storage) : nullptr;
    bq_init(q);
    if (kDist && threadIdx.x == 0) rq->n = 0;
    const uint32_t nh = (uint32_t)min(cn->nhub, (u64)pt.nrows); // k_td's guard dropped any entry past nrows
    const int32_t nd = level + 1;
    const unsigned tid = threadIdx.x;
    constexpr int kPer = kHubBatch / kBS;
    u64 acc_mf = 0, attempts = 0, scanned = 0, acc_dmax = 0, acc_mfh = 0, acc_nh = 0, acc_ex = 0;
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
                s_beg[idx] = (BegT)b;
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
            s_scan[idx] = (ScanT)((idx < hb) ? run : total);
            run += d[k];
        }
        if (tid == 0) s_scan[kHubBatch] = (ScanT)total;
        __syncthreads();
        // this workgroup's equal share of the batch's edges
        const uint64_t x_begin = total * blockIdx.x / gridDim.x, x_end = total * (blockIdx.x + 1) / gridDim.x;
        if (tid == 0) scanned += x_end - x_begin;
        sweep_segments<kDist>(s_scan, s_beg, s_u, hb, x_begin, x_end, row_off, col, vis, stt, par, pcode, nd, q, qout,
                              &cn->qtail, pt, rq, acc_mf, attempts, acc_dmax, hs, acc_mfh, acc_nh, acc_ex, plog, s_vp, vpref);
        __syncthreads();
    }
    q_flush(q, qout, plog, &cn->qtail, pt.qcap, pt.err);
    if (kDist) rq_flush(*rq, pt);
    shard_add(cn, 0, acc_mf, scanned, attempts, 0, acc_dmax, acc_mfh, acc_nh, acc_ex);
    publish_if_last(cn, pub, seq);
    if (kDist) slot_headers_if_last(pt);
}

} // namespace

// dmax: largest degree in the frontier (< 0: unknown) -- the hub bin is skipped when no vertex exceeds
// the hub degree
// skip_hubs (hybrid level): frontier vertices of the hub domain are left to the bottom-up hub sweep.
// pub != null: the last kernel launched publishes the level's counters (seq) from its last workgroup
// plog (single device): the level's winners go to the push log as vertex | parent << 32 at their queue positions
// instead of a packed-state store (BfsWorkspace::plog)
template <bool kDist>
int launch_td(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t mf, int64_t dmax, int level, const Part &pt,
              bool skip_hubs, Published *pub, u64 seq, uint32_t *par,
              u64 *plog) {
    hipStream_t st = g->ctx->stream;
    uint8_t *pcode = par ? ws->pcode : nullptr;
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
    // the next-frontier queue holds nv ids; the push-log segment [log_n, nv) what is left of the log
    Part ptq = pt;
    ptq.qcap = (u64)std::max<int64_t>(plog ? g->nv - ws->log_n : g->nv, 0);
    // slot mode: only the level's last push kernel writes the slot headers
    Part pt0 = ptq;
    if (hubs) pt0.slot_arrive = nullptr;
    // the LDS snapshot of the hubs' visited bits (relabelled single-device graphs: the hubs are the lowest ids)
    const uint32_t vpref = (!kDist && g->d_perm && g->ctx->opt.hub_lds_skip)
                               ? (uint32_t)std::min<int64_t>(kVisPref, ws->nwords * 64) : 0u;
    if (ws->off32) {
        hipLaunchKernelGGL((k_td<kDist, uint32_t>), grid, dim3(kBS), 0, st, ws->off32, g->d_col, ws->qa, (uint32_t)nf,
                           ws->qb, ws->vis, ws->st, par, pcode, ws->ring, level, hub_deg, ws->hubs, pt0, gsz, hs, skip,
                           hubs ? nullptr : pub, seq, plog);
        BFSX_LAUNCHED(st);
        if (hubs) {
            hipLaunchKernelGGL((k_td_hubs<kDist, uint32_t>), gh, dim3(kBS), 0, st, ws->off32, g->d_col, ws->hubs,
                               ws->qb, ws->vis, ws->st, par, pcode, ws->ring, level, ptq, hs, pub, seq, plog, vpref);
            BFSX_LAUNCHED(st);
        }
    } else {
        hipLaunchKernelGGL((k_td<kDist, int64_t>), grid, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->qa,
                           (uint32_t)nf, ws->qb, ws->vis, ws->st, par, pcode, ws->ring, level, hub_deg, ws->hubs, pt0, gsz, hs, skip,
                           hubs ? nullptr : pub, seq, plog);
        BFSX_LAUNCHED(st);
        if (hubs) {
            hipLaunchKernelGGL((k_td_hubs<kDist, int64_t>), gh, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->hubs,
                               ws->qb, ws->vis, ws->st, par, pcode, ws->ring, level, ptq, hs, pub, seq, plog, vpref);
            BFSX_LAUNCHED(st);
        }
    }
    return BFSX_OK;
}

template int launch_td<false>(bfsx_graph *, BfsWorkspace *, int64_t, int64_t, int64_t, int, const Part &, bool,
                              Published *, u64, uint32_t *, u64 *);
template int launch_td<true>(bfsx_graph *, BfsWorkspace *, int64_t, int64_t, int64_t, int, const Part &, bool,
                             Published *, u64, uint32_t *, u64 *);

} // namespace bfsx
