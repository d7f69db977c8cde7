// kernels_build.hip -- graph construction on the GPU (gfx950).
//
// Replaces GraphFileUtil.convert's symmetrise + HashSet dedup (GraphFileUtil.java:60-66, Vertex.java
// :74-76): tuples (a,b) become the neighbour sets N(a) += b, N(b) += a, with duplicates collapsed and
// a self-loop kept once.  The result is CSR: row_off int64[nv+1], col uint32[nnz], rows ascending.
//
// Pipeline (all on one HIP stream, all HBM-streaming integer work):
//   K1a count    degree histogram (atomicAdd per endpoint) + tuple count per first endpoint (m_comp)
//   K1b scan     rocPRIM exclusive scan -> row offsets
//   K1c scatter  per-row cursors (64-bit atomics) -> unsorted rows
//   K1d sort     rocPRIM segmented radix sort of every row (chunked below 2^32 entries)
//   K1e dedup    keep-flags (row head or != predecessor) -> scan -> compact -> new row offsets
// The Kronecker generator (Graph500 recipe, counter-based RNG) also lives here; a Kronecker graph is
// built straight from the counter stream (every pass regenerates its tuples, none are stored).
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>

#include "bfsx_internal.h"

namespace bfsx {

namespace {

constexpr int kBS = 256;

// raw adjacency entries per build chunk (option "build_chunk"; set per build by the calling thread)
thread_local int64_t kBuildChunk = (int64_t)1 << 30;

__global__ void k_fill_i64(int64_t *__restrict__ p, int64_t n, int64_t v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

inline unsigned grid_for(int64_t work, int64_t per_block, unsigned cap = 16384) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---- Kronecker generator ---------------------------------------------------------------------
__device__ __host__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct KronParams {
    uint64_t sh;       // mix64(seed)
    uint64_t mask;     // 2^scale - 1
    uint64_t a1, c1, a2, c2;
    int s1, s2, scale;
    uint32_t t_ab, t_an, t_cn;
};

__device__ inline uint64_t kron_perm(uint64_t x, const KronParams &p) {
    x = (x * p.a1 + p.c1) & p.mask;
    x ^= x >> p.s1;
    x = (x * p.a2 + p.c2) & p.mask;
    x ^= x >> p.s2;
    x = (x * p.a1 + p.c2) & p.mask;
    return x;
}

// Tuple k of the stream: one counter-based draw per (k, bit), then the bijective relabel.
__device__ inline void kron_tuple(const KronParams &p, int64_t k, uint32_t &u, uint32_t &v) {
    uint64_t i = 0, j = 0;
    for (int ib = 0; ib < p.scale; ib++) {
        uint64_t r = mix64((((uint64_t)k) << 6 | (uint64_t)ib) ^ p.sh);
        uint32_t r1 = (uint32_t)(r >> 32), r2 = (uint32_t)r;
        uint64_t ii = r1 > p.t_ab;
        uint64_t jj = r2 > (ii ? p.t_cn : p.t_an);
        i |= ii << ib;
        j |= jj << ib;
    }
    u = (uint32_t)kron_perm(i, p);
    v = (uint32_t)kron_perm(j, p);
}

__global__ __launch_bounds__(kBS) void k_kronecker(KronParams p, int64_t m, uint32_t *__restrict__ u,
                                                   uint32_t *__restrict__ v) {
    for (int64_t k = (int64_t)blockIdx.x * kBS + threadIdx.x; k < m; k += (int64_t)gridDim.x * kBS)
        kron_tuple(p, k, u[k], v[k]);
}

KronParams kron_params(int scale, uint64_t seed) {
    KronParams p;
    p.scale = scale;
    p.sh = mix64(seed);
    p.mask = (1ULL << scale) - 1;
    p.a1 = (mix64(seed ^ 0xA5A5A5A5A5A5A5A5ULL) | 1ULL) & p.mask;
    p.c1 = mix64(seed ^ 0x5A5A5A5A5A5A5A5AULL) & p.mask;
    p.a2 = (mix64(seed ^ 0x3C3C3C3C3C3C3C3CULL) | 1ULL) & p.mask;
    p.c2 = mix64(seed ^ 0xC3C3C3C3C3C3C3C3ULL) & p.mask;
    p.s1 = scale / 2 + 1;
    p.s2 = scale / 3 + 1;
    // A,B,C,D = .57,.19,.19,.05: ab = .76, a_norm = 57/76, c_norm = 19/24, as 2^-32 fractions
    p.t_ab = (uint32_t)((76ULL << 32) / 100ULL);
    p.t_an = (uint32_t)((57ULL << 32) / 76ULL);
    p.t_cn = (uint32_t)((19ULL << 32) / 24ULL);
    return p;
}

// Tuple sources of the build: tuples held in device arrays (files, host tuples), or regenerated on
// the fly from the Kronecker counter stream by every pass that needs them (no 8 B/tuple array: at
// scale 30 that is 137 GB per device).
struct ArraySrc {
    const uint32_t *u, *v;
    __device__ void operator()(int64_t i, uint32_t &a, uint32_t &b) const {
        a = u[i];
        b = v[i];
    }
};

struct KronSrc {
    KronParams p;
    __device__ void operator()(int64_t i, uint32_t &a, uint32_t &b) const { kron_tuple(p, i, a, b); }
};

// The same tuples with both endpoints renamed through `perm` (the degree-descending relabel below).
template <class Src>
struct PermSrc {
    Src s;
    const uint32_t *perm;
    __device__ void operator()(int64_t i, uint32_t &a, uint32_t &b) const {
        uint32_t x, y;
        s(i, x, y);
        a = perm[x];
        b = perm[y];
    }
};


// Rows are built only for global ids in [lo, lo + nv) (the whole graph on one device); indices into
// deg / tcnt / cursor are local (id - lo), adjacency entries stay global.
template <class Src>
__global__ __launch_bounds__(kBS) void k_count(Src src, int64_t m, uint32_t lo, uint32_t nv, uint32_t *__restrict__ deg,
                                               uint32_t *__restrict__ tcnt) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBS) {
        uint32_t ua, vb;
        src(i, ua, vb);
        const uint32_t a = ua - lo, b = vb - lo; // unsigned wrap: out of range -> >= nv
        if (a < nv) {
            atomicAdd(&deg[a], 1u);
            atomicAdd(&tcnt[a], 1u);
        }
        if (b < nv && a != b) atomicAdd(&deg[b], 1u);
    }
}

template <class Src>
__global__ __launch_bounds__(kBS) void k_scatter(Src src, int64_t m, uint32_t lo, uint32_t nv,
                                                 unsigned long long *__restrict__ cursor, uint32_t *__restrict__ col) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBS) {
        uint32_t a, b;
        src(i, a, b);
        if (a - lo < nv) col[atomicAdd(&cursor[a - lo], 1ull)] = b;
        if (b - lo < nv && a != b) col[atomicAdd(&cursor[b - lo], 1ull)] = a;
    }
}

// Degree of every global id over the whole tuple list (duplicates counted): the row-order key of a
// partitioned graph, whose neighbours' rows live on other ranks.
template <class Src>
__global__ __launch_bounds__(kBS) void k_count_all(Src src, int64_t m, uint32_t *__restrict__ deg) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBS) {
        uint32_t a, b;
        src(i, a, b);
        atomicAdd(&deg[a], 1u);
        if (a != b) atomicAdd(&deg[b], 1u);
    }
}

__global__ __launch_bounds__(kBS) void k_keep(const uint32_t *__restrict__ col, int64_t nnz,
                                              uint8_t *__restrict__ keep) {
    for (int64_t j = (int64_t)blockIdx.x * kBS + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * kBS) {
        if (j == 0) { keep[0] = 1; continue; }
        if (!keep[j]) keep[j] = col[j] != col[j - 1];
    }
}

__global__ __launch_bounds__(kBS) void k_compact(const uint32_t *__restrict__ col, const uint8_t *__restrict__ keep,
                                                 const int64_t *__restrict__ pos, int64_t nnz,
                                                 uint32_t *__restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * kBS + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * kBS)
        if (keep[j]) out[pos[j]] = col[j];
}

// Chunk variants (rows [r0, r1) whose raw entries are [e0, e1)): heads relative to e0, and the new row
// offsets = the chunk's output base + the rank of the row's first entry among the kept ones.
__global__ __launch_bounds__(kBS) void k_mark_heads_c(const int64_t *__restrict__ off, int64_t r0, int64_t r1,
                                                      int64_t e0, uint8_t *__restrict__ keep) {
    for (int64_t r = r0 + (int64_t)blockIdx.x * kBS + threadIdx.x; r < r1; r += (int64_t)gridDim.x * kBS) {
        const int64_t b = off[r];
        if (off[r + 1] > b) keep[b - e0] = 1;
    }
}
__global__ __launch_bounds__(kBS) void k_new_off_c(const int64_t *__restrict__ off, const int64_t *__restrict__ pos,
                                                   int64_t r0, int64_t r1, int64_t e0, int64_t obase,
                                                   int64_t *__restrict__ noff) {
    for (int64_t r = r0 + (int64_t)blockIdx.x * kBS + threadIdx.x; r < r1; r += (int64_t)gridDim.x * kBS)
        noff[r] = obase + pos[off[r] - e0];
}

struct SubBase {
    int64_t base;
    __host__ __device__ int64_t operator()(int64_t x) const { return x - base; }
};

struct U8ToI64 {
    __host__ __device__ int64_t operator()(uint8_t x) const { return (int64_t)x; }
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    T *release() {
        T *q = p;
        p = nullptr;
        return q;
    }
};

} // namespace

void set_build_chunk(int64_t entries) { kBuildChunk = std::max<int64_t>(entries, 1); }

int kronecker_generate(hipStream_t stream, int scale, int edgefactor, uint64_t seed, uint32_t *d_u,
                       uint32_t *d_v) {
    const KronParams p = kron_params(scale, seed);
    int64_t m = (int64_t)edgefactor << scale;
    hipLaunchKernelGGL(k_kronecker, dim3(grid_for(m, kBS, 32768)), dim3(kBS), 0, stream, p, m, d_u, d_v);
    BFSX_HIP_TRY(hipGetLastError());
    return BFSX_OK;
}

// Row chunks [cuts[i], cuts[i+1]) of at most `limit` entries each (a longer single row is a chunk of
// its own) and at most kChunkRows rows, from a host copy of the offsets.  The row cap: rocPRIM's
// segmented radix sort mis-sorts chunks of very many tiny segments (a relabelled scale-29/30 graph's
// tail chunk: 2^30 entries in hundreds of millions of rows of degree 1..7 moved entries between rows,
// `profiles/r02i_segsort.txt`); 2^24 rows per chunk stays far below that.
constexpr int64_t kChunkRows = (int64_t)1 << 24;
int plan_row_chunks(const std::vector<int64_t> &h_off, int64_t nv, int64_t limit, std::vector<int64_t> &cuts) {
    cuts.assign(1, 0);
    int64_t r = 0;
    while (r < nv) {
        int64_t r2 = std::upper_bound(h_off.begin() + r, h_off.begin() + nv + 1, h_off[r] + limit) - h_off.begin() - 1;
        if (r2 <= r) r2 = r + 1; // one row longer than the limit
        r2 = std::min<int64_t>(r2, r + kChunkRows);
        if (h_off[r2] - h_off[r] >= ((int64_t)1 << 31)) return fail(BFSX_E_ARG, "a single adjacency row exceeds 2^31 entries");
        r2 = std::min<int64_t>(r2, nv);
        cuts.push_back(r2);
        r = r2;
    }
    return BFSX_OK;
}

// One segmented sort of `rows` rows (offsets d_off[0..rows], entries starting at e0; n < 2^31 entries):
// keys_in[0..n) -> keys_out[0..n).
template <class K>
int sort_rows_range(hipStream_t stream, const int64_t *d_off, int64_t rows, int64_t e0, int64_t n, const K *keys_in,
                    K *keys_out, unsigned end_bit) {
    auto beg = rocprim::make_transform_iterator(d_off, SubBase{e0});
    auto end = rocprim::make_transform_iterator(d_off + 1, SubBase{e0});
    size_t tmp_bytes = 0;
    BFSX_HIP_TRY(rocprim::segmented_radix_sort_keys(nullptr, tmp_bytes, keys_in, keys_out, (unsigned)n,
                                                    (unsigned)rows, beg, end, 0, end_bit, stream));
    DevBuf<char> tmp;
    BFSX_HIP_TRY(tmp.alloc(tmp_bytes));
    BFSX_HIP_TRY(rocprim::segmented_radix_sort_keys(tmp.p, tmp_bytes, keys_in, keys_out, (unsigned)n, (unsigned)rows,
                                                    beg, end, 0, end_bit, stream));
    BFSX_HIP_TRY(hipStreamSynchronize(stream)); // tmp is freed on return
    return BFSX_OK;
}

// Key for the degree-descending row order: (UINT32_MAX - deg(nbr)) << 32 | nbr.
// gdeg (partitioned graphs): global degree table; otherwise the degree comes from the local CSR.
__global__ __launch_bounds__(kBS) void k_degree_keys(const int64_t *__restrict__ off, const uint32_t *__restrict__ col,
                                                     const uint32_t *__restrict__ gdeg, int64_t nnz,
                                                     unsigned long long *__restrict__ keys) {
    for (int64_t j = (int64_t)blockIdx.x * kBS + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * kBS) {
        const uint32_t x = col[j];
        const uint64_t d = gdeg ? (uint64_t)gdeg[x] : (uint64_t)(off[x + 1] - off[x]);
        const uint64_t dk = d >= 0xFFFFFFFFull ? 0ull : 0xFFFFFFFFull - d;
        keys[j] = (dk << 32) | x;
    }
}

__global__ __launch_bounds__(kBS) void k_low32(const unsigned long long *__restrict__ keys, int64_t nnz,
                                               uint32_t *__restrict__ col) {
    for (int64_t j = (int64_t)blockIdx.x * kBS + threadIdx.x; j < nnz; j += (int64_t)gridDim.x * kBS)
        col[j] = (uint32_t)keys[j];
}

// Re-order every row so that high-degree neighbours come first: a bottom-up probe of an unvisited
// vertex then tests the neighbour most likely to be in a large frontier first (early exit).  Row chunks
// of <= kBuildChunk entries keep the 64-bit sort keys at 16 B per CHUNK entry, not per graph entry.
int order_rows_by_degree(hipStream_t stream, const int64_t *d_off, int64_t nv, int64_t nnz, uint32_t *d_col,
                         const uint32_t *gdeg) {
    if (nnz <= 0) return BFSX_OK;
    std::vector<int64_t> h_off(nv + 1), cuts;
    BFSX_HIP_TRY(hipMemcpy(h_off.data(), d_off, (nv + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    if (int rc = plan_row_chunks(h_off, nv, kBuildChunk, cuts)) return rc;
    int64_t cap = 0;
    for (size_t c = 0; c + 1 < cuts.size(); c++) cap = std::max(cap, h_off[cuts[c + 1]] - h_off[cuts[c]]);
    DevBuf<unsigned long long> k0, k1;
    BFSX_HIP_TRY(k0.alloc(cap));
    BFSX_HIP_TRY(k1.alloc(cap));
    for (size_t c = 0; c + 1 < cuts.size(); c++) {
        const int64_t r0 = cuts[c], r1 = cuts[c + 1], e0 = h_off[r0], n = h_off[r1] - e0;
        if (n <= 0) continue;
        hipLaunchKernelGGL(k_degree_keys, dim3(grid_for(n, kBS)), dim3(kBS), 0, stream, d_off, d_col + e0, gdeg, n,
                           k0.p);
        BFSX_HIP_TRY(hipGetLastError());
        if (int rc = sort_rows_range(stream, d_off + r0, r1 - r0, e0, n, k0.p, k1.p, 64u)) return rc;
        hipLaunchKernelGGL(k_low32, dim3(grid_for(n, kBS)), dim3(kBS), 0, stream, k1.p, n, d_col + e0);
        BFSX_HIP_TRY(hipGetLastError());
    }
    BFSX_HIP_TRY(hipStreamSynchronize(stream));
    return BFSX_OK;
}

namespace {

template <class Src>
int build_rows(hipStream_t stream, int64_t nv, Src src, int64_t m, bool degree_order, int64_t **d_row_off_out,
               uint32_t **d_col_out, int64_t *nnz_out, uint32_t **d_tuple_cnt_out, int64_t lo, int64_t nv_global) {
    if (nv_global < 0) nv_global = nv;
    const bool partitioned = lo != 0 || nv != nv_global;
    DevBuf<uint32_t> deg, tcnt;
    DevBuf<int64_t> off;
    BFSX_HIP_TRY(deg.alloc(nv + 1));
    BFSX_HIP_TRY(tcnt.alloc(nv));
    BFSX_HIP_TRY(off.alloc(nv + 1));
    BFSX_HIP_TRY(hipMemsetAsync(deg.p, 0, (nv + 1) * sizeof(uint32_t), stream));
    BFSX_HIP_TRY(hipMemsetAsync(tcnt.p, 0, nv * sizeof(uint32_t), stream));
    if (m > 0) {
        hipLaunchKernelGGL(k_count<Src>, dim3(grid_for(m, kBS)), dim3(kBS), 0, stream, src, m, (uint32_t)lo,
                           (uint32_t)nv, deg.p, tcnt.p);
        BFSX_HIP_TRY(hipGetLastError());
    }
    // K1b: row offsets (int64) = exclusive scan of degrees
    {
        size_t tmp_bytes = 0;
        BFSX_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp_bytes, deg.p, off.p, (int64_t)0, (size_t)(nv + 1),
                                             rocprim::plus<int64_t>(), stream));
        DevBuf<char> tmp;
        BFSX_HIP_TRY(tmp.alloc(tmp_bytes));
        BFSX_HIP_TRY(rocprim::exclusive_scan(tmp.p, tmp_bytes, deg.p, off.p, (int64_t)0, (size_t)(nv + 1),
                                             rocprim::plus<int64_t>(), stream));
    }
    int64_t nnz_raw = 0;
    BFSX_HIP_TRY(hipMemcpyAsync(&nnz_raw, off.p + nv, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    BFSX_HIP_TRY(hipStreamSynchronize(stream));
    deg.reset();

    // K1c: scatter into per-row slots
    DevBuf<uint32_t> col;
    BFSX_HIP_TRY(col.alloc(nnz_raw));
    {
        DevBuf<int64_t> cursor;
        BFSX_HIP_TRY(cursor.alloc(nv));
        BFSX_HIP_TRY(hipMemcpyAsync(cursor.p, off.p, nv * sizeof(int64_t), hipMemcpyDeviceToDevice, stream));
        if (m > 0) {
            hipLaunchKernelGGL(k_scatter<Src>, dim3(grid_for(m, kBS)), dim3(kBS), 0, stream, src, m, (uint32_t)lo,
                               (uint32_t)nv, (unsigned long long *)cursor.p, col.p);
            BFSX_HIP_TRY(hipGetLastError());
        }
        BFSX_HIP_TRY(hipStreamSynchronize(stream));
    }

    // K1d + K1e per row chunk (<= kBuildChunk raw entries): sort the chunk's rows by neighbour id into a
    // chunk buffer, mark the first copy of every neighbour, scan, and compact the kept entries back into
    // `col` at the running output position (never past the chunk's own start: dedup only shrinks), with
    // the chunk's new row offsets.  Peak memory is the raw adjacency + ~13 B per chunk entry instead of
    // ~21 B per graph entry, so a scale-30 graph builds on one 288 GB device.  `col` keeps its raw
    // allocation (the few % of duplicates) instead of a copy to the exact size.
    DevBuf<int64_t> noff;
    BFSX_HIP_TRY(noff.alloc(nv + 1));
    int64_t nnz = 0;
    {
        std::vector<int64_t> h_off(nv + 1), cuts;
        BFSX_HIP_TRY(hipMemcpy(h_off.data(), off.p, (nv + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
        if (int rc = plan_row_chunks(h_off, nv, kBuildChunk, cuts)) return rc;
        int64_t cap = 0;
        for (size_t c = 0; c + 1 < cuts.size(); c++) cap = std::max(cap, h_off[cuts[c + 1]] - h_off[cuts[c]]);
        unsigned end_bit = 1;
        while (end_bit < 32 && (1ULL << end_bit) < (uint64_t)nv_global) end_bit++;
        DevBuf<uint32_t> col_s;
        DevBuf<uint8_t> keep;
        DevBuf<int64_t> pos;
        BFSX_HIP_TRY(col_s.alloc(cap));
        BFSX_HIP_TRY(keep.alloc(cap + 1));
        BFSX_HIP_TRY(pos.alloc(cap + 1));
        DevBuf<char> stmp;
        size_t stmp_cap = 0;
        for (size_t c = 0; c + 1 < cuts.size(); c++) {
            const int64_t r0 = cuts[c], r1 = cuts[c + 1], e0 = h_off[r0], n = h_off[r1] - e0;
            if (n > 0) {
                if (int rc = sort_rows_range(stream, off.p + r0, r1 - r0, e0, n, col.p + e0, col_s.p, end_bit))
                    return rc;
                BFSX_HIP_TRY(hipMemsetAsync(keep.p, 0, n + 1, stream));
                hipLaunchKernelGGL(k_mark_heads_c, dim3(grid_for(r1 - r0, kBS)), dim3(kBS), 0, stream, off.p, r0, r1,
                                   e0, keep.p);
                BFSX_HIP_TRY(hipGetLastError());
                hipLaunchKernelGGL(k_keep, dim3(grid_for(n, kBS)), dim3(kBS), 0, stream, col_s.p, n, keep.p);
                BFSX_HIP_TRY(hipGetLastError());
                auto in = rocprim::make_transform_iterator(keep.p, U8ToI64{});
                size_t tb = 0;
                BFSX_HIP_TRY(rocprim::exclusive_scan(nullptr, tb, in, pos.p, (int64_t)0, (size_t)(n + 1),
                                                     rocprim::plus<int64_t>(), stream));
                if (tb > stmp_cap) {
                    stmp.reset();
                    BFSX_HIP_TRY(stmp.alloc(tb));
                    stmp_cap = tb;
                }
                BFSX_HIP_TRY(rocprim::exclusive_scan(stmp.p, tb, in, pos.p, (int64_t)0, (size_t)(n + 1),
                                                     rocprim::plus<int64_t>(), stream));
                hipLaunchKernelGGL(k_compact, dim3(grid_for(n, kBS)), dim3(kBS), 0, stream, col_s.p, keep.p, pos.p, n,
                                   col.p + nnz);
                BFSX_HIP_TRY(hipGetLastError());
                hipLaunchKernelGGL(k_new_off_c, dim3(grid_for(r1 - r0, kBS)), dim3(kBS), 0, stream, off.p, pos.p, r0,
                                   r1, e0, nnz, noff.p);
                BFSX_HIP_TRY(hipGetLastError());
                int64_t kept = 0;
                BFSX_HIP_TRY(hipMemcpyAsync(&kept, pos.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
                BFSX_HIP_TRY(hipStreamSynchronize(stream));
                nnz += kept;
            } else {
                hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(r1 - r0, kBS)), dim3(kBS), 0, stream, noff.p + r0, r1 - r0,
                                   nnz);
                BFSX_HIP_TRY(hipGetLastError());
            }
        }
        BFSX_HIP_TRY(hipMemcpyAsync(noff.p + nv, &nnz, sizeof(int64_t), hipMemcpyHostToDevice, stream));
        BFSX_HIP_TRY(hipStreamSynchronize(stream));
    }
    DevBuf<uint32_t> &col_f = col;
    if (degree_order) {
        DevBuf<uint32_t> gdeg;
        if (partitioned) {
            BFSX_HIP_TRY(gdeg.alloc(nv_global));
            BFSX_HIP_TRY(hipMemsetAsync(gdeg.p, 0, nv_global * sizeof(uint32_t), stream));
            if (m > 0) {
                hipLaunchKernelGGL(k_count_all<Src>, dim3(grid_for(m, kBS)), dim3(kBS), 0, stream, src, m, gdeg.p);
                BFSX_HIP_TRY(hipGetLastError());
            }
        }
        int rc = order_rows_by_degree(stream, noff.p, nv, nnz, col_f.p, gdeg.p);
        if (rc) return rc;
    }

    *d_row_off_out = noff.release();
    *d_col_out = col_f.release();
    *d_tuple_cnt_out = tcnt.release();
    *nnz_out = nnz;
    return BFSX_OK;
}

// Degree-descending relabel keys of ids [base, base + n): ~degree (an ascending sort puts the highest
// degree first), ids.
__global__ __launch_bounds__(kBS) void k_rank_keys(const uint32_t *__restrict__ deg, int64_t base, int64_t n,
                                                   uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
        keys[i] = ~deg[base + i];
        ids[i] = (uint32_t)(base + i);
    }
}

__global__ __launch_bounds__(kBS) void k_invert(const uint32_t *__restrict__ inv, int64_t n, uint32_t *__restrict__ perm) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS)
        perm[inv[i]] = (uint32_t)i;
}

// out[i] = perm[lo + i] - lo: a rank's own slice of the permutation, as local row indices
__global__ __launch_bounds__(kBS) void k_local_perm(const uint32_t *__restrict__ perm, int64_t lo, int64_t n,
                                                    uint32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS)
        out[i] = (uint32_t)((int64_t)perm[lo + i] - lo);
}

// Relabel (rchunk > 0): the vertices are renumbered by degree, descending (tuple-endpoint degree:
// duplicates counted, a self-loop once; ties by id) INSIDE every id range [r*rchunk, (r+1)*rchunk) --
// one range on a single device, the ranks' ranges on a 1-D partition, so a vertex keeps its owner and
// a partition's routing (owner = id / chunk) is unchanged -- and the CSR is built from the renamed
// tuples.  Internal id order is then degree order within every range, so
//   - the high-degree vertices every pull probe and push claim concentrates on occupy the first lines
//     of every range of the frontier / visited bitmaps, the state array and top1/rest (cache-resident),
//     and the "hubs" of the hybrid levels (single device) are simply the ids below a limit;
//   - on one device, rows sorted ascending by internal id ARE degree-ordered (no second sort of the
//     adjacency); a partition still degree-orders its rows (their entries span every range);
//   - isolated vertices sit at the end of their range, in whole words the pull kernel skips.
// Every rank computes the whole permutation itself from the tuple stream (no exchange).  Returned:
// *d_perm_out[i] = local internal row of ORIGINAL local id lo + i (a slice of the permutation),
// *d_inv_out[x] = original id of GLOBAL internal id x (the whole inverse: parents map back through it).
template <class Src>
int build_csr_impl(hipStream_t stream, int64_t nv, Src src, int64_t m, bool degree_order, int64_t rchunk,
                   int64_t **d_row_off_out, uint32_t **d_col_out, int64_t *nnz_out, uint32_t **d_tuple_cnt_out,
                   uint32_t **d_perm_out, uint32_t **d_inv_out, int64_t lo, int64_t nv_global) {
    if (nv_global < 0) nv_global = nv;
    if (rchunk <= 0 || !degree_order)
        return build_rows(stream, nv, src, m, degree_order, d_row_off_out, d_col_out, nnz_out, d_tuple_cnt_out, lo,
                          nv_global);
    const int64_t n = nv_global;
    const bool single = lo == 0 && nv == n;
    DevBuf<uint32_t> perm, inv;
    {
        DevBuf<uint32_t> deg, keys, keys2, ids;
        BFSX_HIP_TRY(deg.alloc(n + 1));
        BFSX_HIP_TRY(hipMemsetAsync(deg.p, 0, (n + 1) * sizeof(uint32_t), stream));
        if (m > 0) {
            hipLaunchKernelGGL(k_count_all<Src>, dim3(grid_for(m, kBS)), dim3(kBS), 0, stream, src, m, deg.p);
            BFSX_HIP_TRY(hipGetLastError());
        }
        const int64_t rmax = std::min(rchunk, n);
        BFSX_HIP_TRY(keys.alloc(rmax));
        BFSX_HIP_TRY(keys2.alloc(rmax));
        BFSX_HIP_TRY(ids.alloc(rmax));
        BFSX_HIP_TRY(inv.alloc(n));
        DevBuf<char> tmp;
        size_t tmp_cap = 0;
        for (int64_t r0 = 0; r0 < n; r0 += rchunk) { // one stable sort per range (ties keep id order)
            const int64_t cnt = std::min(rchunk, n - r0);
            hipLaunchKernelGGL(k_rank_keys, dim3(grid_for(cnt, kBS)), dim3(kBS), 0, stream, deg.p, r0, cnt, keys.p,
                               ids.p);
            BFSX_HIP_TRY(hipGetLastError());
            size_t tb = 0;
            BFSX_HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, keys.p, keys2.p, ids.p, inv.p + r0, (size_t)cnt, 0, 32,
                                                   stream));
            if (tb > tmp_cap) {
                BFSX_HIP_TRY(hipStreamSynchronize(stream));
                tmp.reset();
                BFSX_HIP_TRY(tmp.alloc(tb));
                tmp_cap = tb;
            }
            BFSX_HIP_TRY(rocprim::radix_sort_pairs(tmp.p, tb, keys.p, keys2.p, ids.p, inv.p + r0, (size_t)cnt, 0, 32,
                                                   stream));
        }
        BFSX_HIP_TRY(perm.alloc(n));
        hipLaunchKernelGGL(k_invert, dim3(grid_for(n, kBS)), dim3(kBS), 0, stream, inv.p, n, perm.p);
        BFSX_HIP_TRY(hipGetLastError());
        BFSX_HIP_TRY(hipStreamSynchronize(stream)); // temporaries are freed at the end of this scope
    }
    // one device: ascending rows of internal ids are degree-descending rows, no degree-order pass
    int rc = build_rows(stream, nv, PermSrc<Src>{src, perm.p}, m, !single, d_row_off_out, d_col_out, nnz_out,
                        d_tuple_cnt_out, lo, nv_global);
    if (rc) return rc;
    if (single) {
        *d_perm_out = perm.release();
    } else { // keep only this rank's slice of the permutation
        DevBuf<uint32_t> loc;
        BFSX_HIP_TRY(loc.alloc(nv));
        if (nv > 0) {
            hipLaunchKernelGGL(k_local_perm, dim3(grid_for(nv, kBS)), dim3(kBS), 0, stream, perm.p, lo, nv, loc.p);
            BFSX_HIP_TRY(hipGetLastError());
        }
        BFSX_HIP_TRY(hipStreamSynchronize(stream));
        *d_perm_out = loc.release();
    }
    *d_inv_out = inv.release();
    return BFSX_OK;
}

} // namespace

namespace {

__global__ __launch_bounds__(kBS) void k_orig_deg(const uint32_t *__restrict__ perm, const int64_t *__restrict__ off,
                                                  int64_t nv, int64_t *__restrict__ deg) {
    for (int64_t v = (int64_t)blockIdx.x * kBS + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBS) {
        const uint32_t x = perm[v];
        deg[v] = off[x + 1] - off[x];
    }
}

// Original rows [r0, r1): one wave per row, entries mapped back to original ids, written at
// off_o[v] - e0 of the chunk buffer.
__global__ __launch_bounds__(kBS) void k_orig_rows(const uint32_t *__restrict__ perm, const uint32_t *__restrict__ inv,
                                                   const int64_t *__restrict__ off, const uint32_t *__restrict__ col,
                                                   const int64_t *__restrict__ off_o, int64_t r0, int64_t r1, int64_t e0,
                                                   uint32_t *__restrict__ out) {
    const unsigned lane = threadIdx.x & 63u;
    const int64_t nw = ((int64_t)gridDim.x * kBS) >> 6;
    for (int64_t v = r0 + (((int64_t)blockIdx.x * kBS + threadIdx.x) >> 6); v < r1; v += nw) {
        const uint32_t x = perm[v];
        const int64_t b = off[x], e = off[x + 1], o = off_o[v] - e0;
        for (int64_t j = b + lane; j < e; j += 64) out[o + (j - b)] = inv[col[j]];
    }
}

} // namespace

int export_csr_original(hipStream_t stream, int64_t nv, int64_t nnz, const int64_t *d_row_off, const uint32_t *d_col,
                        const uint32_t *d_perm, const uint32_t *d_inv, int64_t *row_off, uint32_t *col) {
    DevBuf<int64_t> deg, off_o;
    BFSX_HIP_TRY(deg.alloc(nv + 1));
    BFSX_HIP_TRY(off_o.alloc(nv + 1));
    BFSX_HIP_TRY(hipMemsetAsync(deg.p + nv, 0, sizeof(int64_t), stream));
    hipLaunchKernelGGL(k_orig_deg, dim3(grid_for(nv, kBS)), dim3(kBS), 0, stream, d_perm, d_row_off, nv, deg.p);
    BFSX_HIP_TRY(hipGetLastError());
    {
        size_t tb = 0;
        BFSX_HIP_TRY(rocprim::exclusive_scan(nullptr, tb, deg.p, off_o.p, (int64_t)0, (size_t)(nv + 1),
                                             rocprim::plus<int64_t>(), stream));
        DevBuf<char> tmp;
        BFSX_HIP_TRY(tmp.alloc(tb));
        BFSX_HIP_TRY(rocprim::exclusive_scan(tmp.p, tb, deg.p, off_o.p, (int64_t)0, (size_t)(nv + 1),
                                             rocprim::plus<int64_t>(), stream));
        BFSX_HIP_TRY(hipStreamSynchronize(stream));
    }
    std::vector<int64_t> h_own;
    int64_t *h_off = row_off;
    if (!h_off) {
        h_own.resize(nv + 1);
        h_off = h_own.data();
    }
    BFSX_HIP_TRY(hipMemcpy(h_off, off_o.p, (nv + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    if (!col || nnz <= 0) return BFSX_OK;
    // rows in chunks of <= 2^28 entries (one temporary of 1 GiB at most, whatever the graph's size)
    std::vector<int64_t> h_vec;
    if (!h_own.empty()) h_vec.swap(h_own);
    const std::vector<int64_t> &hv = h_vec.empty() ? std::vector<int64_t>(h_off, h_off + nv + 1) : h_vec;
    std::vector<int64_t> cuts;
    if (int rc = plan_row_chunks(hv, nv, (int64_t)1 << 28, cuts)) return rc;
    int64_t cap = 0;
    for (size_t c = 0; c + 1 < cuts.size(); c++) cap = std::max(cap, hv[cuts[c + 1]] - hv[cuts[c]]);
    DevBuf<uint32_t> buf;
    BFSX_HIP_TRY(buf.alloc(cap));
    for (size_t c = 0; c + 1 < cuts.size(); c++) {
        const int64_t r0 = cuts[c], r1 = cuts[c + 1], e0 = hv[r0], n = hv[r1] - e0;
        if (n <= 0) continue;
        hipLaunchKernelGGL(k_orig_rows, dim3(grid_for((r1 - r0) * 64, kBS)), dim3(kBS), 0, stream, d_perm, d_inv,
                           d_row_off, d_col, off_o.p, r0, r1, e0, buf.p);
        BFSX_HIP_TRY(hipGetLastError());
        BFSX_HIP_TRY(hipMemcpyAsync(col + e0, buf.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        BFSX_HIP_TRY(hipStreamSynchronize(stream));
    }
    return BFSX_OK;
}

int build_csr_device(hipStream_t stream, int64_t nv, const uint32_t *d_u, const uint32_t *d_v, int64_t m,
                     bool degree_order, int64_t relabel_chunk, int64_t **d_row_off, uint32_t **d_col, int64_t *nnz,
                     uint32_t **d_tuple_cnt, uint32_t **d_perm, uint32_t **d_inv, int64_t lo, int64_t nv_global) {
    return build_csr_impl(stream, nv, ArraySrc{d_u, d_v}, m, degree_order, relabel_chunk, d_row_off, d_col, nnz,
                          d_tuple_cnt, d_perm, d_inv, lo, nv_global);
}

int build_csr_kronecker(hipStream_t stream, int scale, int edgefactor, uint64_t seed, bool degree_order,
                        int64_t relabel_chunk, int64_t **d_row_off, uint32_t **d_col, int64_t *nnz,
                        uint32_t **d_tuple_cnt, uint32_t **d_perm, uint32_t **d_inv, int64_t lo, int64_t nv_local) {
    const int64_t m = (int64_t)edgefactor << scale;
    return build_csr_impl(stream, nv_local, KronSrc{kron_params(scale, seed)}, m, degree_order, relabel_chunk, d_row_off,
                          d_col, nnz, d_tuple_cnt, d_perm, d_inv, lo, (int64_t)1 << scale);
}

} // namespace bfsx
