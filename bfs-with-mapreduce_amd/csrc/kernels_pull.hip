// kernels_pull.hip -- bottom-up pull levels (no reference analogue: the direction-optimising half of the
// level loop that replaces BfsSpark.java:66-108): k_bu (the dense pull, and the hub sweep of a hybrid level) and
// k_bu_sparse (the tail pull levels), and their launchers.
#include "bfs_core.h"

namespace bfsx {

namespace {

#ifdef BFSX_DIAG
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
#endif

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
// A pull level's discovery: its provenance code, plus the 4-B parent when the code is explicit (the level's record
// bitmap gives the distance; BfsWorkspace::pcode / par, one device and the partitioned loop alike); par_out ==
// null: the packed state (the test suite's level primitives).
__device__ __forceinline__ void settle_state(u64 *__restrict__ stt, uint32_t *__restrict__ par_out,
                                             uint8_t *__restrict__ code_out, uint32_t v, uint32_t code,
                                             uint32_t parent, int32_t nd) {
    if (par_out) {
        if (code_out) code_out[v] = (uint8_t)code;
        if (!code_out || code == kCodeExplicit) par_out[v] = parent;
    } else {
        stt[v] = pack_state(parent, nd);
    }
}

// kSpill: a diagnostic instantiation compiled for 8 waves per SIMD (64 VGPRs), so it spills to scratch --
// option bu_force_spill, the round-2 "spilling pull kernel + concurrent in-process ranks" experiment.
template <class OffT, bool kMf, bool kHubs, int kU, bool kHubOnly, bool kPipe, bool kSpill = false>
__device__ __forceinline__ void k_bu_body(const OffT *__restrict__ row_off, const uint32_t *__restrict__ col,
                                            const uint32_t *__restrict__ top1, const uint4 *__restrict__ rest,
                                            const u64 *__restrict__ front, u64 *__restrict__ next,
                                            u64 *__restrict__ vis, u64 *__restrict__ vis_out, u64 *__restrict__ stt,
                                            uint32_t *__restrict__ par_out,
                                            uint8_t *__restrict__ code_out, LevelSlot *ring, int level,
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
    uint32_t acc_ex = 0; // discoveries with an explicit 4-B parent
    const int64_t wstride = (int64_t)gridDim.x * kWaves * 64;
    for (int64_t w0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; w0 < nwords; w0 += wstride) {
        const int64_t wl = w0 + lane;
        const u64 vwl = wl < nwords ? vis[wl] : ~0ull;
        const u64 unv = ~vwl;
        const uint32_t c = (uint32_t)__popcll(unv);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t total = __shfl(incl, 63);
        if (total == 0) { // wave-uniform: every vertex of the group visited or isolated
            if (wl < nwords) {
                next[wl] = 0ull;
                if (vis_out) vis_out[wl] = vwl;
            }
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
                    uint32_t par = 0, code = kCodeExplicit; // the encoded hub domain names every parent explicitly
                    const uint32_t pb = (pbm >> (3 * k)) & 7u;
                    if (ok) {
                        if ((fbm >> k) & 1u) {
                            found = true;
                            par = x[k] & ~fmask;
                            if (!kHubs) code = kCodeTop1;
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
                            if (!kHubs) code = (uint32_t)__ffs((int)pb); // 1, 2, 3: rest .x, .y, .z
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
                        settle_state(stt, par_out, code_out, v[k], code, probe_id<kHubs>(hub_id, par), nd);
                        atomicOr(&s_nx[wave][(v[k] - vbase) >> 6], 1ull << (v[k] & 63u));
                        acc_nf += 1;
                        if (kHubs) acc_ex += 1; // phase A names its parent by code 0-3, except the hub domain
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
                            settle_state(stt, par_out, code_out, vv, kCodeExplicit, probe_id<kHubs>(hub_id, par), nd);
                            atomicOr(&s_nx[wave][(vv - vbase) >> 6], 1ull << (vv & 63u));
                            acc_nf += 1;
                            acc_ex += 1;
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
            // vis_out (the frontier is vis itself): every word goes to the other buffer, vis stays as the level
            // found it -- another wave may still probe it
            if (vis_out) vis_out[wl] = vwl | nxl;
            else if (nxl) vis[wl] = vwl | nxl;
        }
    }
    // claims field: rows walked (phase B)
    shard_add(cn, acc_nf, acc_mf, acc_sc, acc_rows, acc_mu, 0, acc_s2, acc_wk, acc_nh, acc_ex);
    publish_if_last(cn, pub, seq);
}

#define BFSX_K_BU_PARAMS                                                                                        \
    const OffT *__restrict__ row_off, const uint32_t *__restrict__ col, const uint32_t *__restrict__ top1,      \
        const uint4 *__restrict__ rest, const u64 *__restrict__ front, u64 *__restrict__ next,                  \
        u64 *__restrict__ vis, u64 *__restrict__ vis_out, u64 *__restrict__ stt, uint32_t *__restrict__ par_out,       \
        uint8_t *__restrict__ code_out,                                                                        \
        LevelSlot *ring, int level,                                                                            \
        int64_t nwords, uint32_t fmask,                                                                        \
        const u64 *__restrict__ hfront, const uint32_t *__restrict__ hub_id, uint32_t hub_lim, uint32_t leaf_lo, \
        PrefixSpec pf, Published *pub, u64 seq, uint32_t hub_row_lim
#define BFSX_K_BU_ARGS                                                                                          \
    row_off, col, top1, rest, front, next, vis, vis_out, stt, par_out, code_out, ring, level, nwords, fmask, hfront,   \
        hub_id,                                                                                                \
        hub_lim,                                                                                               \
        leaf_lo, pf,                                                                                           \
        pub, seq, hub_row_lim

template <class OffT, bool kMf, bool kHubs, int kU, bool kHubOnly, bool kPipe>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(5))) void k_bu(BFSX_K_BU_PARAMS) {
    k_bu_body<OffT, kMf, kHubs, kU, kHubOnly, kPipe>(BFSX_K_BU_ARGS);
}
#ifdef BFSX_DIAG
// Diagnostic build only (option bu_force_spill): the partitioned pipelined pull kernel built so that it
// spills to scratch -- the round-2 "spilling pull kernel + concurrent in-process ranks" experiment.
template <class OffT>
__global__ __launch_bounds__(kBS) __attribute__((amdgpu_waves_per_eu(5))) void k_bu_spill(BFSX_K_BU_PARAMS) {
    k_bu_body<OffT, true, false, 4, false, true, true>(BFSX_K_BU_ARGS);
}
#endif

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
                                                   uint32_t *__restrict__ par_out, uint8_t *__restrict__ code_out,
                                                   LevelSlot *ring,
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
    uint32_t acc_ex = 0; // discoveries with an explicit 4-B parent
    const uint32_t *front32 = reinterpret_cast<const uint32_t *>(front);
    auto fbit = [&](uint32_t x) -> uint32_t { return (front32[x >> 5] >> (x & 31u)) & 1u; };
    int64_t wb = 0; // first word of the wave's current range
    // state word + next-frontier bit of a found vertex; wave-uniform queue append of the ones below qlim
    auto settle = [&](bool found, uint32_t v, uint32_t code, uint32_t par) {
        if (found) {
            settle_state(stt, par_out, code_out, v, code, par, nd);
            atomicOr(&s_nx[wave][(int64_t)(v >> 6) - wb], 1ull << (v & 63u));
            acc_nf += 1;
            acc_ex += code == kCodeExplicit ? 1u : 0u;
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
            uint32_t par = 0, code = kCodeExplicit;
            const uint32_t pb = (pbm >> (3 * k)) & 7u, deg = r[k].w;
            if (ok[k]) {
                if ((fbm >> k) & 1u) {
                    found = true;
                    par = x[k] & ~fmask;
                    code = kCodeTop1;
                    acc_sc += 1;
                } else if (x[k] & fmask) { // top1 was the row's only entry
                    acc_mu += 1;
                    acc_sc += 1;
                } else if (pb) {
                    found = true;
                    par = (pb & 1u) ? r[k].x : (pb & 2u) ? r[k].y : r[k].z;
                    code = (uint32_t)__ffs((int)pb);
                    acc_sc += 2u + (uint32_t)__ffs((int)pb) - 1u;
                } else if (deg <= 4u) {
                    acc_mu += deg;
                    acc_sc += deg;
                } else {
                    miss = true;
                    acc_sc += 4;
                }
            }
            settle(found, v[k], code, par);
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
            settle(found, vv, kCodeExplicit, par);
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
    shard_add(cn, acc_nf, acc_q, acc_sc, acc_rows, acc_mu, 0, acc_s2, acc_wk, acc_nh, acc_ex);
    publish_if_last(cn, pub, seq);
}

} // namespace

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
#ifdef BFSX_DIAG
        const void *kfn = kSpill ? reinterpret_cast<const void *>(&k_bu_spill<OffT>)
                                 : reinterpret_cast<const void *>(&k_bu<OffT, kMf, kHubs, kU, kHubOnly, kPipe>);
#else
        static_assert(!kSpill && !kHubs, "the spilling pull kernel and the hub domain are diagnostic builds only");
        const void *kfn = reinterpret_cast<const void *>(&k_bu<OffT, kMf, kHubs, kU, kHubOnly, kPipe>);
#endif
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kBS, 0) !=
                hipSuccess ||
            per_cu < 1)
            per_cu = 4;
    }
    const unsigned cap = (unsigned)(g->ctx->num_cus * per_cu);
    const dim3 grid(clamp_grid((ws->nwords + kWaves * 64 - 1) / (kWaves * 64), cap));
#ifdef BFSX_DIAG
    if (kHubs) {
        hipLaunchKernelGGL(k_hub_gather, dim3(clamp_grid((ws->hub_k + kBS - 1) / kBS, 8192)), dim3(kBS), 0, st,
                           ws->hub_id, ws->hub_k, front, ws->hfront);
        BFSX_LAUNCHED(st);
    }
#endif
#define BFSX_K_BU_LAUNCH(kern)                                                                                   \
    hipLaunchKernelGGL(kern, grid, dim3(kBS), 0, st, row_off, kHubs ? ws->colh : g->d_col, ws->top1, ws->rest, front, \
                       next, ws->vis, ws->bu_vis_out, ws->st, par, ws->pcode, ws->ring, level, ws->nwords,           \
                       ws->top1_flag, ws->hfront,                                                                       \
                       ws->hub_id,                                                                                      \
                       ws->hub_lim, (uint32_t)std::min<int64_t>(ws->leaf_lo, 0xFFFFFFFFll), lds_prefix<kHubs>(g, ws),  \
                       pub, seq, (uint32_t)std::min<int64_t>(ws->hub_row_lim, 0xFFFFFFFFll))
#ifdef BFSX_DIAG
    if constexpr (kSpill) BFSX_K_BU_LAUNCH((k_bu_spill<OffT>));
    else
#endif
        BFSX_K_BU_LAUNCH((k_bu<OffT, kMf, kHubs, kU, kHubOnly, kPipe>));
#undef BFSX_K_BU_LAUNCH
    ws->bu_vis_out = nullptr; // one-shot
    BFSX_LAUNCHED(st);
    return BFSX_OK;
}

template <class OffT, bool kMf, bool kHubs>
int launch_bu_t(bfsx_graph *g, BfsWorkspace *ws, const OffT *row_off, const u64 *front, u64 *next, uint32_t *par,
                int level, Published *pub, u64 seq) {
    if (g->ctx->opt.bu_unroll == 2)
        return launch_bu_u<OffT, kMf, kHubs, 2, false, false>(g, ws, row_off, front, next, par, level, pub, seq);
#ifdef BFSX_DIAG
    if (kMf && !kHubs && g->ctx->opt.bu_force_spill) // diagnostic (see k_bu's kSpill)
        return launch_bu_u<OffT, kMf, false, 4, false, true, true>(g, ws, row_off, front, next, par, level, pub, seq);
#endif
    // kMf (partitioned) + kPipe needs more than the 96 VGPRs of 5 waves per SIMD: that instantiation runs
    // at 4 waves per SIMD (a spilling pull kernel is never an option)
    return g->ctx->opt.bu_pipeline
               ? launch_bu_u<OffT, kMf, kHubs, 4, false, true>(g, ws, row_off, front, next, par, level, pub, seq)
               : launch_bu_u<OffT, kMf, kHubs, 4, false, false>(g, ws, row_off, front, next, par, level, pub, seq);
}

// The bottom-up half of a hybrid level: candidates probe only the hubs of the frontier (single device).
int launch_bu_hubonly(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level) {
#ifdef BFSX_DIAG
    if (ws->hub_k > 0)
        return ws->off32
                   ? launch_bu_u<uint32_t, false, true, 4, true, false>(g, ws, ws->off32, front, next, par, level, nullptr, 0)
                   : launch_bu_u<int64_t, false, true, 4, true, false>(g, ws, g->d_row_off, front, next, par, level, nullptr, 0);
#endif
    return ws->off32
               ? launch_bu_u<uint32_t, false, false, 4, true, false>(g, ws, ws->off32, front, next, par, level, nullptr, 0)
               : launch_bu_u<int64_t, false, false, 4, true, false>(g, ws, g->d_row_off, front, next, par, level, nullptr, 0);
}

// par == null: discoveries store the packed state (the partitioned loop); else the 4-B parent (single device,
// `next` is then the level's record)
template <bool kMf>
int launch_bu(bfsx_graph *g, BfsWorkspace *ws, const u64 *front, u64 *next, uint32_t *par, int level,
              Published *pub, u64 seq) {
#ifdef BFSX_DIAG
    if (ws->hub_k > 0) // top1 is hub-encoded: every bottom-up launch of this graph uses the hub domain
        return ws->off32 ? launch_bu_t<uint32_t, kMf, true>(g, ws, ws->off32, front, next, par, level, pub, seq)
                         : launch_bu_t<int64_t, kMf, true>(g, ws, g->d_row_off, front, next, par, level, pub, seq);
#endif
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
                           front, next, ws->vis, ws->st, par, ws->pcode, ws->ring, level, ws->nwords, ws->top1_flag, hrl,
                           qlim,
                           ws->qa, pub, seq);
    else
        hipLaunchKernelGGL(k_bu_sparse<int64_t>, grid, dim3(kBS), 0, st, g->d_row_off, g->d_col, ws->top1, ws->rest,
                           front, next, ws->vis, ws->st, par, ws->pcode, ws->ring, level, ws->nwords, ws->top1_flag, hrl,
                           qlim,
                           ws->qa, pub, seq);
    BFSX_LAUNCHED(st);
    return BFSX_OK;
}

template int launch_bu<false>(bfsx_graph *, BfsWorkspace *, const u64 *, u64 *, uint32_t *, int, Published *, u64);
template int launch_bu<true>(bfsx_graph *, BfsWorkspace *, const u64 *, u64 *, uint32_t *, int, Published *, u64);

} // namespace bfsx
