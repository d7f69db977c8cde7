// kernels_persist.hip -- K3p: the persistent top-down kernel that runs many narrow push levels in one launch,
// with a grid barrier made of tagged per-workgroup level records (high-diameter graphs: largeG's >= 567 levels,
// algs4.jar!/BreadthFirstPaths.java:33), and its host side.
#include "bfs_core.h"

namespace bfsx {

namespace {

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
                                                    u64 *hseg, uint32_t h0_v, uint32_t h0_deg, int64_t h0_beg,
                                                    u64 *front, int64_t front_words) {
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
    // front != null (a BFS's first launch): should the launch stop because Beamer asks for a pull level, it also
    // leaves the pull kernel's frontier bitmap in `front`: a copy of the visited bitmap.  A pull level may take
    // every visited vertex as frontier: an unvisited vertex has no neighbour at a distance below the level's (it
    // would have been discovered), so its probes meet exactly the frontier's bits either way, in the same row order
    // -- the same parents, the same distances.  No memset, no queue -> bitmap atomics.
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
        const bool to_pull = nf_all > 0 && beamer && (int64_t)mf_new > bu_floor; // the host's switch, the same test
        const bool stop = nf_all == 0 || nf_new > kPersistNf || nh_new > kHeavyMax ||
                          (u64)((nf_new + G - 1) / G) * dm_new + (kHeavy ? (eh_new + G - 1) / G : 0ull) > (u64)kRegion ||
                          to_pull || it + 1 >= max_levels;
        __syncthreads();
        // the host reads the counts as soon as they are final (a mapped flag, no stream synchronise: that cost ~13 us
        // per launch); the hand-back below is stream-ordered before the next kernel anyway
        const bool bits = front && to_pull;
        if (stop && b == 0 && tid == 0) {
            out->front = bits ? 1ull : 0ull;
            persist_done(out);
        }
        if (stop) { // hand the frontier back contiguous: the light entries, then the heavy ones (+ the bitmap)
            // 8 loads in flight per thread before their stores (a one-element loop waits a round trip per element)
            constexpr int kCp = 8;
            // bits: the host's next level is the pull (the same test as to_pull), which reads `front`, not the queue
            const uint32_t nb = bits ? 0u : (b + 1 < G ? s_off[b + 1] : nf_new) - s_off[b], ob = s_off[b];
            for (uint32_t i0 = 0; i0 < nb; i0 += kBS * kCp) {
                uint32_t e[kCp];
#pragma unroll
                for (int k = 0; k < kCp; k++) {
                    const uint32_t i = i0 + (uint32_t)k * kBS + tid;
                    e[k] = i < nb ? (uint32_t)ld_sc1(sout + 2 * i + 1) : 0u;
                }
#pragma unroll
                for (int k = 0; k < kCp; k++) {
                    const uint32_t i = i0 + (uint32_t)k * kBS + tid;
                    if (i < nb) qfinal[ob + i] = e[k];
                }
            }
            const uint32_t hb = bits ? 0u : (b + 1 < G ? s_hoff[b + 1] : nh_new) - s_hoff[b], hbase = nf_new + s_hoff[b];
            for (uint32_t i = tid; i < hb; i += kBS) qfinal[hbase + i] = (uint32_t)ld_sc1(hout + 2 * i + 1);
            if (bits) { // every claim of the level completed before its record (vmcnt(0)); sc1 loads see them all
                const int64_t w0 = front_words * b / G, w1 = front_words * (b + 1) / G;
                for (int64_t x0 = w0; x0 < w1; x0 += (int64_t)kBS * kCp) {
                    u64 e[kCp];
#pragma unroll
                    for (int k = 0; k < kCp; k++) {
                        const int64_t w = x0 + (int64_t)k * kBS + tid;
                        e[k] = w < w1 ? ld_sc1(vis + w) : 0ull;
                    }
#pragma unroll
                    for (int k = 0; k < kCp; k++) {
                        const int64_t w = x0 + (int64_t)k * kBS + tid;
                        if (w < w1) front[w] = e[k];
                    }
                }
            }
            return;
        }
        nf = nf_new;
        nh_in = nh_new;
        eh_in = eh_new;
    }
}

} // namespace

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
bool persist_fits(bfsx_graph *g, BfsWorkspace *ws, int64_t nf, int64_t dmax, bool heavy_src) {
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


// Run K3p from `level` (frontier of nf vertices in ws->qa; its last frontier lands in ws->qb).
// Returns the number of levels it ran (>= 1) with their records in the PersistOut, or an error.
// h0_deg > 0: the first level's frontier is the single heavy row {h0_v, h0_beg, h0_deg} (nf = 0 light).
int persist_td(bfsx_graph *g, BfsWorkspace *ws, int level, int64_t nf, int64_t mu, u64 *front, uint32_t h0_v,
               uint32_t h0_deg, int64_t h0_beg) {
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
    out->front = 0;
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
                           (uint32_t)g->nv, ws->d_err, ws->persist_hseg, h0_v, h0_deg, h0_beg, front, front == ws->vis ? (int64_t)0 : ws->nwords);
    else
        hipLaunchKernelGGL(kp64, grid, dim3(kBS), lds, st, g->d_row_off, g->d_col, ws->qa,
                           (uint32_t)nf, ws->persist_seg, ws->persist_brec, ws->qb, ws->vis, ws->st, ws->ring, level,
                           mu, alpha, kPersistLevels, ws->persist_bar, ctl, dout,
                           hub_set(ws), bu_floor(g, ws), opt.persist_abort_at, (u64)opt.persist_dmax,
                           (uint32_t)g->nv, ws->d_err, ws->persist_hseg, h0_v, h0_deg, h0_beg, front, front == ws->vis ? (int64_t)0 : ws->nwords);
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

} // namespace bfsx
