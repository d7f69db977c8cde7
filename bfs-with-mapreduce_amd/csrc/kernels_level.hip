// kernels_level.hip -- the single-device level loop (BfsSpark.java:57-118 on one GPU): the workspace, the
// loop with Beamer's direction switch and its hybrid levels, the counters published by each level's last
// workgroup (collect + contains("GRAY"), :110-117), and the result unpack to the caller's ids.
#include <rocprim/device/device_radix_sort.hpp>

#include "bfs_core.h"

namespace bfsx {

namespace {

// Result extraction (outside the timed region): internal state (+ the pending records) -> one 8-byte word per
// ORIGINAL id, out[o] = parent_original << 32 | dist (one scattered store per vertex where separate dist and
// parent arrays took two), or dist only.  kRelabel: internal local row i is original vertex inv[lo + i] (a
// partition's relabel keeps it inside the rank's range [lo, lo + n)); parents are global internal ids and map
// back through the whole inv.  Isolated vertices (`dead`; half the ids of a scale-26 Kronecker graph) keep
// the unreached word the buffer was filled with once, except keep0 / keep1 (this BFS's source, the last one
// written that was isolated), so only the other half costs a scattered store.
template <bool kRelabel>
__global__ __launch_bounds__(kBS) void k_unpack(const u64 *__restrict__ stt, ParSrc ps, RecSet rs, const uint32_t *__restrict__ inv, int64_t lo, int64_t n,
                                                const u64 *__restrict__ dead, int64_t keep0, int64_t keep1,
                                                u64 *__restrict__ out, int32_t *__restrict__ dist_only) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        if (((dead[i >> 6] >> (i & 63)) & 1ull) && i != keep0 && i != keep1) continue;
        const u64 s = rec_state(stt, ps, rs, i);
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
//   phase 1, k_unpack_live, INTERNAL id order over the live ids (below iso_lo, the isolated tail): tmp[i] =
//     parent_original << 32 | dist.  A record vertex (found by a pull level) takes its distance from the record
//     and its parent from its provenance code (ParSrc): codes 0-3 read the original-id copy of the row entry
//     the pull kernel probed (otop1 / orest, coalesced with i), code 4 the explicit parent through inv.  Other
//     vertices read st, their parent through inv.  The record words are broadcast loads (a wave's 64 lanes share
//     one), everything else coalesced except the inv lookups of push-found vertices.  st is left as it is: the
//     validator and m_comp fold the records into it when they run (bfs_resolve).
//   phase 2, k_unpack_gather: thread o reads perm[o] and copies tmp[perm[o]] into out[o] -- whole-line writes,
//     near-sequential reads (the relabel keeps original order inside a degree class) -- or writes the unreached
//     word without a load for an id of the isolated tail.
// Both passes are streams with one dependent gather per element; a grid-stride loop with one element per
// iteration leaves them latency-bound (each wave waits a whole memory round trip per element: 0.35 + 0.30 ms at
// scale 26 in a rocprof trace, against ~0.15 ms each at the streaming rate).  So every thread handles kUnpackU
// elements per step -- tiles of kBS * kUnpackU consecutive ids per workgroup, every load of a stage issued
// before the first is used.  Round 6 found that the source did not get that from hipcc: a load under a per-id
// condition became a branch followed by s_waitcnt vmcnt(0), so the stages still went one round trip per element.
// The branch-free forms (k_unpack_live4, k_unpack_gather) issue every load and select afterwards: 0.47-0.48 ->
// 0.37-0.39 ms per scale-26 result (profiles/r06ub_unpack_ab.txt), 0.35 with 16 ids per thread in the gather.
// k_unpack_live stays for a graph without the codes or the original-id copies.
#ifndef BFSX_UNPACK_U
#define BFSX_UNPACK_U 8
#endif
constexpr int kUnpackU = BFSX_UNPACK_U;
// k_unpack_gather's ids per thread and tile step (16: 0.39 -> 0.35 ms per scale-26 result against 8; 24 equal, 32
// and 4 slower: profiles/r06uu_gather_unroll_ab.txt, r06uv_gather_unroll_ab.txt)
#ifndef BFSX_GATHER_U
#define BFSX_GATHER_U 16
#endif
constexpr int kGatherU = BFSX_GATHER_U;

// otop1[v] / orest[v]: top1 / rest with their entries mapped to original ids (built once per graph, at its first
// unpack; the degree-1 flag of top1 dropped)
__global__ __launch_bounds__(kBS) void k_orig_nbrs(const uint32_t *__restrict__ top1, const uint4 *__restrict__ rest,
                                                   uint32_t fmask, const uint32_t *__restrict__ inv, int64_t n,
                                                   uint32_t *__restrict__ otop1, uint4 *__restrict__ orest) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < n; v += (int64_t)gridDim.x * kBS) {
        otop1[v] = inv[top1[v] & ~fmask];
        const uint4 r = rest[v];
        orest[v] = make_uint4(inv[r.x], inv[r.y], inv[r.z], r.w);
    }
}

__global__ __launch_bounds__(kBS) void k_unpack_live(RecSet rs, int64_t live_n, int64_t src, ParSrc ps,
                                                     const uint32_t *__restrict__ otop1,
                                                     const uint4 *__restrict__ orest, const u64 *__restrict__ stt,
                                                     const uint32_t *__restrict__ inv, u64 *__restrict__ tmp,
                                                     int64_t n) {
    constexpr int64_t kTile = (int64_t)kBS * kUnpackU;
    const unsigned lane = lane_id();
    for (int64_t t0 = (int64_t)blockIdx.x * kTile; t0 < live_n; t0 += (int64_t)gridDim.x * kTile) {
        // element j of a wave is one whole bitmap word: its record words are wave-uniform (scalar loads)
        int hit[kUnpackU];
#pragma unroll
        for (int j = 0; j < kUnpackU; j++) hit[j] = -1;
        for (int r = 0; r < rs.n; r++) { // records are disjoint
            const u64 *bm = rs.bm[r];
#pragma unroll
            for (int j = 0; j < kUnpackU; j++) {
                const int wj = __builtin_amdgcn_readfirstlane((int)((t0 + j * kBS) >> 6) + (int)(threadIdx.x >> 6));
                if ((int64_t)wj * 64 < live_n && ((bm[wj] >> lane) & 1ull)) hit[j] = r;
            }
        }
        // stage 1, issued together: a record vertex's code and the original id of its first row entry, anyone
        // else's state
        uint32_t code[kUnpackU], o1[kUnpackU];
        u64 s[kUnpackU];
#pragma unroll
        for (int j = 0; j < kUnpackU; j++) {
            const int64_t v = t0 + j * kBS + threadIdx.x;
            const bool live = v < live_n;
            // streamed once (non-temporal: keep the Infinity Cache for tmp, which k_unpack_gather reads next)
            code[j] = (live && hit[j] >= 0) ? __builtin_nontemporal_load(ps.code + v) : 0xFFu;
            o1[j] = (live && hit[j] >= 0 && otop1) ? __builtin_nontemporal_load(otop1 + v) : 0u;
            s[j] = (live && hit[j] < 0) ? __builtin_nontemporal_load(stt + v) : kUnreached;
        }
        // stage 2: the parent of every other kind -- an original id already (codes 0-3 with the copies), or an
        // internal id that goes through inv (explicit parents, st's)
        uint32_t p[kUnpackU], d[kUnpackU];
        bool mapped[kUnpackU];
#pragma unroll
        for (int j = 0; j < kUnpackU; j++) {
            const int64_t v = t0 + j * kBS + threadIdx.x;
            const uint32_t c = code[j];
            mapped[j] = false;
            if (hit[j] < 0) {
                p[j] = (uint32_t)(s[j] >> 32);
                d[j] = (uint32_t)s[j];
            } else {
                d[j] = (uint32_t)rs.nd[hit[j]];
                if (otop1 && c == kCodeTop1) {
                    p[j] = o1[j];
                    mapped[j] = true;
                } else if (otop1 && c < kCodeExplicit) {
                    const uint4 r = orest[v];
                    p[j] = c == 1 ? r.x : c == 2 ? r.y : r.z;
                    mapped[j] = true;
                } else {
                    p[j] = record_parent(ps, v);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kUnpackU; j++)
            if (!mapped[j] && p[j] != 0xFFFFFFFFu) p[j] = inv[p[j]];
#pragma unroll
        for (int j = 0; j < kUnpackU; j++) {
            const int64_t v = t0 + j * kBS + threadIdx.x;
            if (v < live_n) tmp[v] = ((u64)p[j] << 32) | d[j];
        }
    }
    // an isolated source lies in the tail the loop skips: its state (distance 0, itself as parent) is in st
    if (src >= live_n && src < n && blockIdx.x == 0 && threadIdx.x == 0) {
        const u64 s = stt[src];
        tmp[src] = ((u64)inv[(uint32_t)(s >> 32)] << 32) | (uint32_t)s;
    }
}

// 16-B non-temporal loads (the builtin takes clang vector types, not HIP's uint4)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load4(const void *p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
// k_unpack_live, branch-free (round 6): four consecutive internal ids per lane, and no load behind a per-id
// branch.  hipcc puts a branch around a conditional load and waits for every outstanding load after it
// (s_waitcnt vmcnt(0)), so the per-id `cond ? load : default` of k_unpack_live issued its loads one round trip
// at a time.  Here every load is issued, with the address of an element that needs none moved to entry 0 of its
// array (a line every wave touches: no extra HBM traffic), and the value selected afterwards.  Four ids per lane
// also make the streaming accesses wide: the codes of four ids are one 4-B load, their otop1 entries one 16-B
// load, their states two 16-B loads and their tmp words two 16-B stores.  Needs the codes and otop1 / orest
// (else k_unpack_live); a tile that crosses live_n takes k_unpack_live's per-id path.
constexpr int kLiveRecUnroll = 4; // record words loaded together (a BFS has 2-4 pull levels; more loop)
#ifndef BFSX_LIVE_G
#define BFSX_LIVE_G 2
#endif
// groups of four consecutive ids per lane and tile (1-4 within 1%: profiles/r06lg_live_groups_ab.txt)
constexpr int kLiveG = BFSX_LIVE_G;
__global__ __launch_bounds__(kBS) void k_unpack_live4(RecSet rs, int64_t live_n, int64_t src, ParSrc ps,
                                                      const uint32_t *__restrict__ otop1,
                                                      const uint4 *__restrict__ orest, const u64 *__restrict__ stt,
                                                      const uint32_t *__restrict__ inv, u64 *__restrict__ tmp,
                                                      int64_t n) {
    constexpr int64_t kTile = (int64_t)kBS * 4 * kLiveG;
    for (int64_t t0 = (int64_t)blockIdx.x * kTile; t0 < live_n; t0 += (int64_t)gridDim.x * kTile) {
        if (t0 + kTile > live_n) { // the last tile: per id (uniform branch)
            for (int64_t v = t0 + threadIdx.x; v < live_n; v += kBS) {
                int hit = -1;
                for (int r = 0; r < rs.n; r++)
                    if ((rs.bm[r][v >> 6] >> (v & 63)) & 1ull) hit = r;
                uint32_t p, d;
                bool mapped = false;
                if (hit < 0) {
                    const u64 x = stt[v];
                    p = (uint32_t)(x >> 32);
                    d = (uint32_t)x;
                } else {
                    d = (uint32_t)rs.nd[hit];
                    const uint32_t c = ps.code[v];
                    if (c == kCodeTop1) {
                        p = otop1[v];
                        mapped = true;
                    } else if (c < kCodeExplicit) {
                        const uint4 r = orest[v];
                        p = c == 1 ? r.x : c == 2 ? r.y : r.z;
                        mapped = true;
                    } else {
                        p = ps.par[v];
                    }
                }
                if (!mapped && p != 0xFFFFFFFFu) p = inv[p];
                tmp[v] = ((u64)p << 32) | d;
            }
            continue;
        }
        int64_t v0[kLiveG];
#pragma unroll
        for (int g = 0; g < kLiveG; g++) v0[g] = t0 + g * (kBS * 4) + threadIdx.x * 4;
        // stage 0: the record words (16 lanes share one), the first kLiveRecUnroll records issued together
        unsigned nib[kLiveG] = {}; // per group: ids found by some pull level
        uint32_t hd[4 * kLiveG];            // their distance (a record's level + 1; taken with the record's uniform index)
#pragma unroll
        for (int j = 0; j < 4 * kLiveG; j++) hd[j] = 0u;
        {
            u64 w[kLiveRecUnroll][kLiveG];
#pragma unroll
            for (int r = 0; r < kLiveRecUnroll; r++)
#pragma unroll
                for (int g = 0; g < kLiveG; g++) // past rs.n (maybe none: a BFS without pull levels) read st instead
                    w[r][g] = (r < rs.n ? rs.bm[r] : stt)[v0[g] >> 6];
#pragma unroll
            for (int r = 0; r < kLiveRecUnroll; r++)
#pragma unroll
                for (int g = 0; g < kLiveG; g++) {
                    const unsigned m = r < rs.n ? (unsigned)(w[r][g] >> (v0[g] & 63)) & 0xFu : 0u;
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        if ((m >> k) & 1u) hd[g * 4 + k] = (uint32_t)rs.nd[r];
                    nib[g] |= m;
                }
        }
        for (int r = kLiveRecUnroll; r < rs.n; r++) // records are disjoint
#pragma unroll
            for (int g = 0; g < kLiveG; g++) {
                const unsigned m = (unsigned)(rs.bm[r][v0[g] >> 6] >> (v0[g] & 63)) & 0xFu;
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if ((m >> k) & 1u) hd[g * 4 + k] = (uint32_t)rs.nd[r];
                nib[g] |= m;
            }
        // stage 1: codes + otop1 of groups with a record vertex, states of groups with another one
        uint32_t code4[kLiveG];
        uint4 o1[kLiveG], sa[kLiveG], sb[kLiveG];
#pragma unroll
        for (int g = 0; g < kLiveG; g++) {
            const int64_t vh = nib[g] ? v0[g] : 0, va = (~nib[g] & 3u) ? v0[g] : 0, vb = (~nib[g] & 12u) ? v0[g] : 0;
            code4[g] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(ps.code + vh));
            o1[g] = nt_load4(otop1 + vh);
            sa[g] = nt_load4(stt + va);
            sb[g] = nt_load4(stt + vb + 2);
        }
        // stage 2: orest for codes 1-3, the explicit parent for code 4
        uint32_t p[4 * kLiveG], d[4 * kLiveG];
        uint4 ro[4 * kLiveG];
        uint32_t pe[4 * kLiveG];
#pragma unroll
        for (int j = 0; j < 4 * kLiveG; j++) {
            const int g = j >> 2, k = j & 3;
            const uint32_t c = (code4[g] >> (8 * k)) & 0xFFu;
            const bool rec = (nib[g] >> k) & 1u;
            const int64_t v = v0[g] + k;
            ro[j] = orest[(rec && c != kCodeTop1 && c < kCodeExplicit) ? v : 0];
            pe[j] = ps.par[(rec && c >= kCodeExplicit) ? v : 0];
        }
        bool need_inv[4 * kLiveG];
#pragma unroll
        for (int j = 0; j < 4 * kLiveG; j++) {
            const int g = j >> 2, k = j & 3;
            const uint32_t c = (code4[g] >> (8 * k)) & 0xFFu;
            const uint4 sv = k < 2 ? sa[g] : sb[g];
            const uint32_t sp = (k & 1) ? sv.w : sv.y, sd = (k & 1) ? sv.z : sv.x;
            const uint32_t ot = k == 0 ? o1[g].x : k == 1 ? o1[g].y : k == 2 ? o1[g].z : o1[g].w;
            // masks, not a select chain: the chain became a dynamic component index into scratch
            const uint32_t orr = (ro[j].x & (0u - (uint32_t)(c == 1))) | (ro[j].y & (0u - (uint32_t)(c == 2))) |
                                 (ro[j].z & (0u - (uint32_t)(c == 3)));
            if (!((nib[g] >> k) & 1u)) {
                p[j] = sp;
                d[j] = sd;
                need_inv[j] = sp != 0xFFFFFFFFu;
            } else {
                d[j] = hd[j];
                p[j] = c == kCodeTop1 ? ot : c < kCodeExplicit ? orr : pe[j];
                need_inv[j] = c >= kCodeExplicit && pe[j] != 0xFFFFFFFFu;
            }
        }
        // stage 3: internal parents -> original ids
        uint32_t q[4 * kLiveG];
#pragma unroll
        for (int j = 0; j < 4 * kLiveG; j++) q[j] = inv[need_inv[j] ? p[j] : 0u];
#pragma unroll
        for (int j = 0; j < 4 * kLiveG; j++)
            if (need_inv[j]) p[j] = q[j];
#pragma unroll
        for (int g = 0; g < kLiveG; g++) {
            u64 *t = tmp + v0[g];
            *reinterpret_cast<uint4 *>(t) = make_uint4(d[g * 4], p[g * 4], d[g * 4 + 1], p[g * 4 + 1]);
            *reinterpret_cast<uint4 *>(t + 2) = make_uint4(d[g * 4 + 2], p[g * 4 + 2], d[g * 4 + 3], p[g * 4 + 3]);
        }
    }
    // an isolated source lies in the tail the loop skips: its state (distance 0, itself as parent) is in st
    if (src >= live_n && src < n && blockIdx.x == 0 && threadIdx.x == 0) {
        const u64 s = stt[src];
        tmp[src] = ((u64)inv[(uint32_t)(s >> 32)] << 32) | (uint32_t)s;
    }
}

// XCD-aware: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8), each with its own L2, so the
// grid is cut into 8 contiguous ranges of original ids, one per XCD.  A degree class whose members are sparse in
// the original order then shares its tmp lines inside one L2 instead of every XCD fetching each line.
constexpr int kXcds = 8;
// Phase 2.  Branch-free (round 6, see k_unpack_live4): a whole tile's perm loads are issued together and every
// tmp load is issued (an isolated id's at entry 0), then selected; the stores need no per-id test.  XCD ranges
// are whole tiles, so only a tile that crosses its range's end takes the per-id path.
template <bool kDistOnly>
__global__ __launch_bounds__(kBS) void k_unpack_gather(const u64 *__restrict__ tmp, const uint32_t *__restrict__ perm,
                                                          int64_t n, int64_t iso_lo, int64_t src, u64 *__restrict__ out,
                                                          int32_t *__restrict__ dist_only) {
    constexpr int64_t kTile = (int64_t)kBS * kGatherU;
    const int64_t per_xcd = ((n + kXcds - 1) / kXcds + kTile - 1) / kTile * kTile;
    const int64_t lo = (int64_t)(blockIdx.x % kXcds) * per_xcd, hi = std::min<int64_t>(lo + per_xcd, n);
    const int64_t step = (int64_t)(gridDim.x / kXcds) * kTile;
    for (int64_t t0 = lo + (int64_t)(blockIdx.x / kXcds) * kTile; t0 < hi; t0 += step) {
        if (t0 + kTile > hi) { // per id
            for (int64_t o = t0 + threadIdx.x; o < hi; o += kBS) {
                const int64_t i = perm[o];
                const u64 s = (i < iso_lo || i == src) ? tmp[i] : kUnreached;
                if (kDistOnly) dist_only[o] = (int32_t)(uint32_t)s;
                else out[o] = s;
            }
            continue;
        }
        uint32_t i[kGatherU];
#pragma unroll
        for (int j = 0; j < kGatherU; j++) i[j] = __builtin_nontemporal_load(perm + t0 + j * kBS + threadIdx.x);
        u64 s[kGatherU];
#pragma unroll
        for (int j = 0; j < kGatherU; j++) {
            const bool live = (int64_t)i[j] < iso_lo || (int64_t)i[j] == src;
            s[j] = tmp[live ? i[j] : 0u];
            s[j] = live ? s[j] : kUnreached;
        }
#pragma unroll
        for (int j = 0; j < kGatherU; j++) {
            const int64_t o = t0 + j * kBS + threadIdx.x;
            if (kDistOnly) __builtin_nontemporal_store((int32_t)(uint32_t)s[j], dist_only + o);
            else __builtin_nontemporal_store(s[j], out + o);
        }
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

#ifdef BFSX_DIAG // the encoded hub probe domain (graphs built with relabel=off)
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
#endif

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
    constexpr int kU = 8; // loads in flight per thread (a one-element grid-stride loop was latency-bound: 325 us)
    for (int64_t t0 = (int64_t)blockIdx.x * kBS * kU; t0 < nv; t0 += (int64_t)gridDim.x * kBS * kU) {
        u64 s[kU];
        uint32_t c[kU];
#pragma unroll
        for (int j = 0; j < kU; j++) {
            const int64_t v = t0 + j * kBS + threadIdx.x;
            s[j] = v < nv ? stt[v] : (u64)INT32_MAX;
            c[j] = v < nv ? tcnt[v] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kU; j++)
            if ((int32_t)(uint32_t)s[j] != INT32_MAX) {
                m += c[j];
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

} // namespace

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
#ifndef BFSX_DIAG
    // the encoded domain of a graph without the relabel (a dense second id per hub, a second copy of col) is
    // built by the diagnostic library only: the product relabels, which makes the hubs an id prefix
    return BFSX_OK;
#else
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
#endif
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
    if (g->nranks == 1) BFSX_HIP_TRY(hipMalloc(&ws->pcode, nv));
    BFSX_HIP_TRY(hipMalloc(&ws->vis, ws->nwords * sizeof(u64)));
    if (g->nranks == 1) BFSX_HIP_TRY(hipMalloc(&ws->vis2, ws->nwords * sizeof(u64))); // option vis_front
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
    BFSX_HIP_TRY(hipHostMalloc(&ws->h_err, kErrWords * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent));
    BFSX_HIP_TRY(hipHostGetDevicePointer((void **)&ws->d_err, ws->h_err, 0));
    for (int i = 0; i < kErrWords; i++) ws->h_err[i] = 0;
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

// After a BFS (a partition: at every level close): fail if a queue consumer met an out-of-range id (id_ok) or a
// store guard refused an index (idx_ok); the words are cleared for the next BFS.
int check_queue_guard(BfsWorkspace *ws) {
    std::atomic_thread_fence(std::memory_order_acquire);
    volatile u64 *w = reinterpret_cast<volatile u64 *>(ws->h_err);
    const u64 e = w[0], idx = w[1], bound = w[2];
    if (!e) return BFSX_OK;
    for (int i = 0; i < kErrWords; i++) w[i] = 0;
    if ((e >> 32) == 2u) {
        static const char *const site[] = {"?", "a fixed exchange slot (pairs routed to one peer)",
                                           "the destination rank of a routed pair", "the remote-pair buffer",
                                           "the hub list", "the next-frontier queue / push-log segment",
                                           "the pair send buffer"};
        const uint32_t s = (uint32_t)e;
        return fail(BFSX_E_HIP, std::string("internal error: store guard: index ") + std::to_string(idx) +
                                    " into " + (s < 7 ? site[s] : "?") + " of bound " + std::to_string(bound) +
                                    " refused (a host bound was too small; nothing was written)");
    }
    return fail(BFSX_E_HIP, "internal error: a frontier-queue consumer read vertex id " +
                                std::to_string((uint32_t)e) + ", outside the rows of this graph (stale queue entry)");
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
        r.ex += (int64_t)s->sh[i].expl;
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

void bfs_workspace_free(BfsWorkspace *ws) {
    if (!ws) return;
    for (void *p : {(void *)ws->sendbuf, (void *)ws->recvbuf, (void *)ws->fglob, (void *)ws->persist_seg,
                    (void *)ws->persist_brec, (void *)ws->persist_hseg, ws->persist_ctl})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)ws->st, (void *)ws->off32, (void *)ws->vis, (void *)ws->vis2, (void *)ws->front, (void *)ws->next,
                    (void *)ws->dead, (void *)ws->qa, (void *)ws->qb, (void *)ws->hubs, (void *)ws->top1, (void *)ws->rest,
                    (void *)ws->hub_id, (void *)ws->colh, (void *)ws->hfront, (void *)ws->ring, (void *)ws->d_cursor, (void *)ws->d_red, (void *)ws->remote,
                    (void *)ws->d_dist_ctr, (void *)ws->out64, (void *)ws->rtmp, (void *)ws->pcode, (void *)ws->otop1,
                    (void *)ws->orest})
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
    for (auto e : ws->ev_comm) (void)hipEventDestroy(e);
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
    if (BFSX_DIAG_ON && opt.poison_queues) // test hook: a consumer that reads past a queue's tail meets 0xFFFFFFFF (id_ok)
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
    // the last K3p launch stopped for a pull level and also left its frontier in ws->front (option persist_front)
    bool front_ready = false;
    // ... and that frontier is vis itself (option vis_front: the launch skipped its queue hand-back, copied nothing)
    bool front_in_vis = false;
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
        bool vis_front_lvl = false; // this pull level reads vis as its frontier (option vis_front)
        u64 *bu_rec = nullptr; // a pull level's record
        if (dir == BFSX_DIR_TOPDOWN && in_queue && level > 0 && has_hubs(ws) && opt.hybrid != 0 && mfh > 0) {
            const int64_t unv = nv - visited - n_pre;
            hybrid = opt.hybrid == 2 || 100 * mfh > (int64_t)opt.hybrid_pct * unv;
        }
        if (hybrid) {
            // the hub sweep's frontier: the visited bitmap (every visited vertex a candidate can touch is in the
            // frontier: see the pull levels below) -- read in place with vis_front (the sweep writes vis2), else a
            // copy
            const bool hv = opt.vis_front && ws->vis2;
            if (!hv) BFSX_HIP_TRY(hipMemcpyAsync(ws->front, ws->vis, nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
            u64 *rec = nullptr;
            if (int e = recs.take(&rec)) return e;
            if (hv) ws->bu_vis_out = ws->vis2;
            if (int e = launch_bu_hubonly(g, ws, hv ? ws->vis : ws->front, rec, ws->par, level)) return e; // -> rec, vis, par
            if (hv) std::swap(ws->vis, ws->vis2); // the push half claims against the sweep's result
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
            ls.explicit_parents = ws->h_pub->expl;
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
            bu_levels++;
            recs.done(level + 1);
            bmf = rec;
            if (nf == 0) break;
            continue;
        }
        if (front_ready && dir != BFSX_DIR_BOTTOMUP) // K3p left no queue: its stop test is this switch's
            return fail(BFSX_E_HIP, "internal error: the persistent launch stopped for a pull level the loop did not take");
        const bool will_sparse =
            opt.bu_sparse > 0 && ws->hub_k == 0 && (nv - visited - n_pre) * opt.bu_sparse <= nwords * 64;
        if (dir == BFSX_DIR_BOTTOMUP && in_queue && front_ready && front_in_vis && !will_sparse) {
            bmf = ws->vis; // K3p stopped for this pull level without handing its queue back (option vis_front)
            vis_front_lvl = true;
            in_queue = false;
        } else if (dir == BFSX_DIR_BOTTOMUP && in_queue && front_ready && !front_in_vis) {
            bmf = ws->front; // K3p stopped for this pull level and left the frontier in front as well
            in_queue = false;
        } else if (dir == BFSX_DIR_BOTTOMUP && in_queue) {
            // The pull level's frontier bitmap after a push level: a copy of the visited bitmap, not the frontier
            // alone.  Level-synchronous BFS: before level L every vertex at distance <= L is visited, and an
            // unvisited vertex has no neighbour at distance < L (it would have been discovered), so the only
            // visited vertices its probes can meet ARE the frontier -- the same hits in the same row order, the
            // same parents and distances -- for one 8-B copy per 64 ids instead of an atomic per frontier vertex
            // (round 6; rounds 1-5 snapshotted the bitmap before a wide push level and XOR-ed it after).
            // Option vis_front (round 6): no copy -- the dense pull kernel reads vis itself as the frontier and
            // writes vis | its discoveries into vis2 (every word), and the loop swaps the two after the launch.
            // The sparse kernel updates vis in place, so a sparse level still takes the copy.
            if (opt.vis_front && ws->vis2 && !will_sparse) {
                bmf = ws->vis;
                vis_front_lvl = true;
            } else {
                BFSX_HIP_TRY(hipMemcpyAsync(ws->front, ws->vis, nwords * sizeof(u64), hipMemcpyDeviceToDevice, st));
                bmf = ws->front;
            }
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
        front_ready = false;
        front_in_vis = false;
        u64 *plog = nullptr; // this level's push-log segment (a per-level push level with push_log)
        // level 0: a source row longer than persist_dmax enters K3p as its heavy table (row bounds known)
        const bool heavy_src = level == 0 && nf == 1 && dmax > opt.persist_dmax;
        if (dir == BFSX_DIR_TOPDOWN && allow_persist && persist_fits(g, ws, nf, dmax, heavy_src)) {
            // narrow frontier: run as many levels as stay narrow inside one launch (K3p)
            // the BFS's first launch hands a frontier that Beamer sends to a pull level back as the bitmap too
            // (with vis_front it is vis itself: the launch only skips handing its queue back, and the pull kernel
            // reads vis)
            const bool vf = opt.vis_front && ws->vis2;
            u64 *kfront = (level == 0 && opt.direction == BFSX_DIR_AUTO && opt.persist_front) ? (vf ? ws->vis : ws->front)
                                                                                               : nullptr;
            const int ran = heavy_src ? persist_td(g, ws, level, 0, mu, kfront, (uint32_t)source, (uint32_t)dmax,
                                                   src_off[0])
                                      : persist_td(g, ws, level, nf, mu, kfront);
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
                front_ready = po.front != 0;
                front_in_vis = front_ready && kfront == ws->vis;
                td_levels += ran;
                level += ran - 1;
                if (nf == 0) break;
                continue;
            }
        }
        if (dir == BFSX_DIR_TOPDOWN) {
            const Part pt = single_part(g, ws);
            // test hook: the level's kernels read one entry past the queue's tail (the guard must catch it)
            const int64_t nf_l = (BFSX_DIAG_ON && level == opt.test_overread) ? nf + 1 : nf;
            plog = opt.push_log ? ws->plog + ws->log_n : nullptr;
            if (int e = launch_td<false>(g, ws, nf_l, mf, dmax, level, pt, false, ws->d_pub, ++ws->pub_seq, nullptr, plog))
                return e;
            td_levels++;
        } else {
            // few unvisited candidates (the tail levels): the sparse kernel, which also queues its discoveries
            sparse = opt.bu_sparse > 0 && ws->hub_k == 0 && (nv - visited - n_pre) * opt.bu_sparse <= nwords * 64;
            if (int e = recs.take(&bu_rec)) return e;
            if (vis_front_lvl && sparse) return fail(BFSX_E_HIP, "internal error: a sparse pull level on the visited bitmap");
            if (sparse) {
                const uint32_t qlim = (uint32_t)(opt.leaf_skip ? std::min<int64_t>(ws->leaf_lo, nv) : nv);
                if (int e = launch_bu_sparse(g, ws, bmf, bu_rec, ws->par, level, qlim, ws->d_pub, ++ws->pub_seq))
                    return e;
            } else {
                if (vis_front_lvl) ws->bu_vis_out = ws->vis2;
                if (int e = launch_bu<false>(g, ws, bmf, bu_rec, ws->par, level, ws->d_pub, ++ws->pub_seq)) return e;
                if (vis_front_lvl) std::swap(ws->vis, ws->vis2);
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
        s.ex = ws->h_pub->expl;
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
        ls.explicit_parents = s.ex;
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
int apply_logs(bfsx_graph *g, BfsWorkspace *ws, hipEvent_t ev) {
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
                       ws->nwords, par_src(ws), ws->st);
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
    if (gather && !ws->orig_nbrs_tried) { // once per graph, outside the unpack's time
        ws->orig_nbrs_tried = true;
        // not for the encoded hub domain, whose top1 / rest are not vertex ids (its pull parents are all explicit)
        if (ws->hub_k == 0 && ws->pcode && hipMalloc(&ws->otop1, nv * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&ws->orest, nv * sizeof(uint4)) == hipSuccess) {
            hipLaunchKernelGGL(k_orig_nbrs, grid, dim3(kBS), 0, st, ws->top1, ws->rest, ws->top1_flag, g->d_inv,
                               (int64_t)nv, ws->otop1, ws->orest);
            BFSX_LAUNCHED(st);
        } else { // no room: codes 0-3 map through inv like explicit parents
            (void)hipGetLastError();
            if (ws->otop1) (void)hipFree(ws->otop1);
            ws->otop1 = nullptr;
            ws->orest = nullptr;
        }
    }
    if (int e = apply_logs(g, ws, ws->ev_unpack0)) return e; // the push log is part of the unpack's time
    if (gather) {
        u64 *tmp = ws->plog; // free once the log is scattered (apply_logs above)
        if (!tmp) {
            if (!ws->rtmp) BFSX_HIP_TRY(hipMalloc(&ws->rtmp, std::max<size_t>(nv, 1) * sizeof(u64)));
            tmp = ws->rtmp;
        }
        const int64_t live_n = std::min<int64_t>(ws->iso_lo, (int64_t)nv);
        const int64_t tile = (int64_t)kBS * kUnpackU;
        if (ws->otop1 && ws->pcode) // the branch-free pass needs the codes and the original-id copies
            hipLaunchKernelGGL(k_unpack_live4, dim3(clamp_grid((live_n + kBS * 4 * kLiveG - 1) / (kBS * 4 * kLiveG), 4096)), dim3(kBS), 0,
                               st, rs, live_n, src, par_src(ws), ws->otop1, ws->orest, ws->st, g->d_inv, tmp,
                               (int64_t)nv);
        else
            hipLaunchKernelGGL(k_unpack_live, dim3(clamp_grid((live_n + tile - 1) / tile, 4096)), dim3(kBS), 0, st,
                               rs, live_n, src, par_src(ws), ws->otop1, ws->orest, ws->st, g->d_inv, tmp, (int64_t)nv);
        BFSX_LAUNCHED(st);
        BFSX_HIP_TRY(hipEventRecord(ws->ev_unpack_mid, st));
        // a multiple of the XCD count, about one tile per workgroup
        const unsigned gx = std::max<unsigned>(
            kXcds, clamp_grid(((int64_t)nv + (int64_t)kBS * kGatherU - 1) / ((int64_t)kBS * kGatherU), 4096) / kXcds * kXcds);
        if (d_dist_only)
            hipLaunchKernelGGL(k_unpack_gather<true>, dim3(gx), dim3(kBS), 0, st, tmp, g->d_perm, (int64_t)nv,
                               ws->iso_lo, src, ws->out64, d_dist_only);
        else
            hipLaunchKernelGGL(k_unpack_gather<false>, dim3(gx), dim3(kBS), 0, st, tmp, g->d_perm, (int64_t)nv,
                               ws->iso_lo, src, ws->out64, d_dist_only);
        ws->out_mode = 0; // every entry written: a later scatter-mode unpack must prefill again
    } else if (g->d_inv)
        hipLaunchKernelGGL(k_unpack<true>, grid, dim3(kBS), 0, st, ws->st, par_src(ws), rs, g->d_inv, g->v_lo, (int64_t)nv,
                           ws->dead, src, ws->out_dirty, ws->out64, d_dist_only);
    else
        hipLaunchKernelGGL(k_unpack<false>, grid, dim3(kBS), 0, st, ws->st, par_src(ws), rs, g->d_inv, g->v_lo,
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
void bfs_comm_times(const bfsx_graph *g, double *ms, int64_t *count) {
    for (int k = 0; k < 4; k++) {
        ms[k] = g->ws ? g->ws->comm_ms[k] : 0.0;
        count[k] = g->ws ? g->ws->comm_n[k] : 0;
    }
}

} // namespace bfsx
