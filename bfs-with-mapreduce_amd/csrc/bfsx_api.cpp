// bfsx_api.cpp -- the C-ABI of libbfsx.so (declared in include/bfsx.h; the test-only level primitives in
// include/bfsx_levels.h).
//
// Host side of the drop-in boundary: error plumbing, the algs4 edge-list parser with
// GraphFileUtil.convert semantics (GraphFileUtil.java:45-66), graph handles, root sampling and the
// synchronous bfsx_bfs wrapper around the device level loops (kernels_level.hip, kernels_dist.hip).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <thread>
#include <unordered_set>

#include "../../include/bfsx_levels.h"
#include "bfsx_internal.h"
#include "java_digits.h"

namespace bfsx {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

const std::string &last_error() { return g_last_error; }

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Integer.parseInt over the exact token, no trimming (Unicode decimal digits included, java_digits.h)
inline bool parse_java_int(const char *s, size_t n, int64_t &out) {
    return java_parse_int(reinterpret_cast<const unsigned char *>(s), 0, (int64_t)n, out);
}

struct MappedFile {
    const char *p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~MappedFile() {
        if (p && n) munmap((void *)p, n);
        if (fd >= 0) close(fd);
    }
};

// BufferedReader.readLine line splitting: '\n', '\r' or "\r\n" end a line; no trailing empty line.
struct LineReader {
    const char *b;
    size_t n, pos = 0;
    bool next(const char *&ls, size_t &ll) {
        if (pos >= n) return false;
        const size_t s = pos;
        const void *nl = memchr(b + s, '\n', n - s);
        size_t e = nl ? (size_t)((const char *)nl - b) : n;
        const void *cr = memchr(b + s, '\r', e - s);
        if (cr) e = (size_t)((const char *)cr - b);
        ls = b + s;
        ll = e - s;
        if (e < n) e += (b[e] == '\r' && e + 1 < n && b[e + 1] == '\n') ? 2 : 1;
        pos = e;
        return true;
    }
};

template <class T>
struct HostVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    ~HostVec() { free(p); }
    bool push(T x) {
        if (n == cap) {
            size_t nc = cap ? cap * 2 : 4096;
            T *q = (T *)realloc(p, nc * sizeof(T));
            if (!q) return false;
            p = q;
            cap = nc;
        }
        p[n++] = x;
        return true;
    }
    T *release() {
        T *q = p;
        p = nullptr;
        return q;
    }
};

// mmap a whole file (GraphFileUtil.java:46 new FileInputStream; IOException -> BFSX_E_IO)
int map_file(const char *path, MappedFile &f) {
    f.fd = open(path, O_RDONLY);
    if (f.fd < 0) return fail(BFSX_E_IO, std::string("cannot open ") + path + ": " + strerror(errno));
    struct stat sb;
    if (fstat(f.fd, &sb) != 0) return fail(BFSX_E_IO, std::string("cannot stat ") + path);
    f.n = (size_t)sb.st_size;
    if (f.n) {
        void *m = mmap(nullptr, f.n, PROT_READ, MAP_PRIVATE, f.fd, 0);
        if (m == MAP_FAILED) return fail(BFSX_E_IO, std::string("cannot map ") + path);
        f.p = (const char *)m;
        madvise(m, f.n, MADV_SEQUENTIAL);
    }
    return BFSX_OK;
}

// The two header lines (GraphFileUtil.java:48,58-59): V with Integer.parseInt, the edge count read and
// ignored.  Leaves the reader at the first edge line.
int read_algs4_header(LineReader &lr, int64_t &nv) {
    const char *ls;
    size_t ll;
    if (!lr.next(ls, ll)) return fail(BFSX_E_PARSE, "missing vertex count line (parseInt(null))");
    int64_t V;
    if (!parse_java_int(ls, ll, V)) return fail(BFSX_E_PARSE, "line 1: vertex count is not an int");
    if (V < 0) return fail(BFSX_E_PARSE, "line 1: negative vertex count (HashMap capacity)");
    nv = V > 0 ? V : 1; // vertex 0 is always created (GraphFileUtil.java:53)
    lr.next(ls, ll);    // edge count, unused
    return BFSX_OK;
}

// File -> device tuples with the GPU tokenizer (kernels_parse.hip).
int load_algs4_device(bfsx_ctx *ctx, const char *path, int64_t &nv, int64_t &m, uint32_t *&d_u, uint32_t *&d_v) {
    MappedFile f;
    if (int rc = map_file(path, f)) return rc;
    LineReader lr{f.p, f.n};
    if (int rc = read_algs4_header(lr, nv)) return rc;
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    return parse_algs4_device(ctx->stream, f.p + lr.pos, f.n - lr.pos, nv, 3, &d_u, &d_v, &m);
}

} // namespace

// Original vertex id -> the global internal id every device array is indexed by (identity without
// relabel).  v must be owned by this rank (the relabel keeps every id inside its owner's range).
int to_internal(const bfsx_graph *g, int64_t v, int64_t *out) {
    if (!g->d_perm) {
        *out = v;
        return BFSX_OK;
    }
    if (v < g->v_lo || v >= g->v_lo + g->nv) return fail(BFSX_E_ARG, "vertex not owned by this rank");
    auto &memo = const_cast<bfsx_graph *>(g)->perm_memo;
    const auto it = memo.find(v);
    if (it != memo.end()) {
        *out = it->second;
        return BFSX_OK;
    }
    uint32_t x = 0;
    BFSX_HIP_TRY(hipMemcpy(&x, g->d_perm + (v - g->v_lo), sizeof(x), hipMemcpyDeviceToHost));
    *out = g->v_lo + (int64_t)x;
    if (memo.size() >= 65536) memo.clear();
    memo.emplace(v, *out);
    return BFSX_OK;
}

// A relabelled partition's source as the validator sees it (dist_begin's convention): its global
// internal id on the owner, nv_global (no row) on the other ranks -- no collective needed.
int dist_map_source(const bfsx_graph *g, int64_t source, int64_t *out) {
    if (source >= g->v_lo && source < g->v_lo + g->nv) return to_internal(g, source, out);
    *out = g->nv_global;
    return BFSX_OK;
}

int to_original(const bfsx_graph *g, int64_t x, int64_t *out) {
    if (!g->d_inv || x < 0) {
        *out = x;
        return BFSX_OK;
    }
    uint32_t v = 0;
    BFSX_HIP_TRY(hipMemcpy(&v, g->d_inv + x, sizeof(v), hipMemcpyDeviceToHost));
    *out = (int64_t)v;
    return BFSX_OK;
}

// ---- group contexts (bfsx_init_group): N ranks of one process, one host thread per rank ------------------
// "Multi-GPU is internal: one host thread (or process) per device, with an RCCL communicator
// per ctx.  The caller sees one call."  Every call on a group context or graph runs the rank calls of the
// 1-D partitioned path (bfsx_dist_*) on one host thread per rank and returns when all have finished.
namespace {

bool is_group(const bfsx_ctx *c) { return c && !c->ranks.empty(); }
bool is_group(const bfsx_graph *g) { return g && !g->parts.empty(); }

// fn(r) on one host thread per rank (rank r's device current).  The reported error is the first rank whose
// failure is its own -- a rank that only saw a peer abort the group says "peer rank ..." -- prefixed with its rank.
int run_ranks(const std::vector<bfsx_ctx *> &ranks, const std::function<int(int)> &fn) {
    const int P = (int)ranks.size();
    std::vector<int> rc(P, BFSX_OK);
    std::vector<std::string> msg(P);
    std::vector<std::thread> th;
    th.reserve(P);
    for (int r = 0; r < P; r++)
        th.emplace_back([&, r] {
            const hipError_t he = hipSetDevice(ranks[r]->device);
            rc[r] = he != hipSuccess ? fail(BFSX_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)) : fn(r);
            if (rc[r]) msg[r] = last_error();
        });
    for (auto &t : th) t.join();
    int pick = -1;
    auto peer = [&](int r) { return msg[r].rfind("peer rank", 0) == 0; };
    for (int r = 0; r < P; r++)
        if (rc[r] && (pick < 0 || (peer(pick) && !peer(r)))) pick = r;
    if (pick < 0) return BFSX_OK;
    return fail(rc[pick], "rank " + std::to_string(pick) + ": " + msg[pick]);
}

// a group graph from every rank's partition (graph construction has no collective: a failed rank fails alone)
int group_graph(bfsx_ctx *ctx, bfsx_graph **out, const std::function<int(int, bfsx_graph **)> &make) {
    const int P = (int)ctx->ranks.size();
    std::vector<bfsx_graph *> parts(P, nullptr);
    const int rc = run_ranks(ctx->ranks, [&](int r) { return make(r, &parts[r]); });
    if (rc) {
        for (bfsx_graph *p : parts) bfsx_graph_free(p);
        return rc;
    }
    auto *g = new (std::nothrow) bfsx_graph();
    if (!g) {
        for (bfsx_graph *p : parts) bfsx_graph_free(p);
        return fail(BFSX_E_OOM, "graph");
    }
    g->ctx = ctx;
    g->parts = parts;
    g->nranks = P;
    g->nv_global = g->nv = parts[0]->nv_global;
    g->chunk = parts[0]->chunk;
    g->m = parts[0]->m;
    for (bfsx_graph *p : parts) g->nnz += p->nnz;
    *out = g;
    return BFSX_OK;
}

int group_bfs(bfsx_graph *g, int64_t source, int32_t *dist_out, int64_t *parent_out, bfsx_stats *stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (source < 0 || source >= g->nv_global)
        return fail(BFSX_E_RANGE, "source vertex " + std::to_string(source) + " outside [0, " +
                                      std::to_string(g->nv_global) + ")");
    const int P = (int)g->parts.size();
    std::vector<bfsx_stats> st(P);
    const int rc = run_ranks(g->ctx->ranks, [&](int r) {
        bfsx_graph *p = g->parts[r];
        if (int e = dist_bfs_run(p, source, stats ? &st[r] : nullptr)) return e;
        if (!dist_out && !parent_out) return BFSX_OK;
        return bfs_copy_result(p, dist_out ? dist_out + p->v_lo : nullptr, parent_out ? parent_out + p->v_lo : nullptr);
    });
    if (rc) return rc;
    g->last_source = source;
    g->last_t_bfs_ms = 0;
    for (bfsx_graph *p : g->parts) g->last_t_bfs_ms = std::max(g->last_t_bfs_ms, p->last_t_bfs_ms);
    if (stats) {
        *stats = st[0]; // levels, directions and the all-reduced m_comp / reached agree on every rank
        stats->t_bfs_ms = g->last_t_bfs_ms;
        stats->t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return BFSX_OK;
}

} // namespace

} // namespace bfsx

using namespace bfsx;

extern "C" {

int bfsx_abi_version(void) { return BFSX_ABI_VERSION; }

const char *bfsx_last_error(void) { return g_last_error.c_str(); }

void bfsx_free_host(void *p) { free(p); }

int bfsx_parse_algs4(const char *path, int64_t *nv_out, int64_t *m_out, uint32_t **u_out, uint32_t **v_out) {
    if (!path || !nv_out || !m_out || !u_out || !v_out) return fail(BFSX_E_ARG, "null argument");
    MappedFile f;
    if (int rc = map_file(path, f)) return rc;
    LineReader lr{f.p, f.n};
    const char *ls;
    size_t ll;
    int64_t nv = 0;
    if (int rc = read_algs4_header(lr, nv)) return rc;
    HostVec<uint32_t> us, vs;
    int64_t lineno = 2;
    while (lr.next(ls, ll)) { // GraphFileUtil.java:60-66, to EOF
        lineno++;
        const char *sp = (const char *)memchr(ls, ' ', ll);
        if (!sp) return fail(BFSX_E_PARSE, "line " + std::to_string(lineno) + ": expected two tokens");
        const size_t n0 = (size_t)(sp - ls);
        const char *t1 = sp + 1;
        const char *sp2 = (const char *)memchr(t1, ' ', ll - n0 - 1);
        const size_t n1 = sp2 ? (size_t)(sp2 - t1) : ll - n0 - 1;
        int64_t a, b;
        if (!parse_java_int(ls, n0, a) || !parse_java_int(t1, n1, b))
            return fail(BFSX_E_PARSE, "line " + std::to_string(lineno) + ": token is not an int");
        if (a < 0 || a >= nv || b < 0 || b >= nv)
            return fail(BFSX_E_RANGE, "line " + std::to_string(lineno) + ": vertex id outside [0," +
                                          std::to_string(nv) + ")");
        if (!us.push((uint32_t)a) || !vs.push((uint32_t)b)) return fail(BFSX_E_OOM, "out of host memory");
    }
    *nv_out = nv;
    *m_out = (int64_t)us.n;
    *u_out = us.release();
    *v_out = vs.release();
    if (!*u_out) *u_out = (uint32_t *)malloc(sizeof(uint32_t));
    if (!*v_out) *v_out = (uint32_t *)malloc(sizeof(uint32_t));
    return BFSX_OK;
}

int bfsx_init(int device, bfsx_ctx **out) {
    if (!out) return fail(BFSX_E_ARG, "null out");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return fail(BFSX_E_NODEV, "no HIP device available");
    if (device < 0 || device >= count) return fail(BFSX_E_ARG, "device ordinal out of range");
    BFSX_HIP_TRY(hipSetDevice(device));
    auto *ctx = new (std::nothrow) bfsx_ctx();
    if (!ctx) return fail(BFSX_E_OOM, "ctx");
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->num_cus = prop.multiProcessorCount;
    if (ctx->num_cus <= 0) ctx->num_cus = 256;
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return fail(BFSX_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return BFSX_OK;
}

int bfsx_init_group(int nranks, bfsx_ctx **out) {
    if (!out || nranks < 1 || nranks > 64) return fail(BFSX_E_ARG, "nranks must be in [1, 64]");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(BFSX_E_NODEV, "no HIP device available");
    const char *mode = std::getenv("BFSX_GROUP_COMM"); // rccl | local (default: rccl when the devices are distinct)
    const bool want_local = mode && !std::strcmp(mode, "local");
    if (mode && !std::strcmp(mode, "rccl") && nranks > count)
        return fail(BFSX_E_ARG, "BFSX_GROUP_COMM=rccl needs one device per rank (" + std::to_string(count) + " visible)");
    auto *gctx = new (std::nothrow) bfsx_ctx();
    if (!gctx) return fail(BFSX_E_OOM, "ctx");
    for (int r = 0; r < nranks; r++) {
        bfsx_ctx *c = nullptr;
        if (int rc = bfsx_init(r % count, &c)) {
            bfsx_finalize(gctx);
            return rc;
        }
        gctx->ranks.push_back(c);
    }
    gctx->num_cus = gctx->ranks[0]->num_cus;
    if (int rc = comm_clique(gctx->ranks.data(), nranks, nranks <= count && !want_local)) {
        const std::string msg = last_error();
        bfsx_finalize(gctx);
        return fail(rc, msg);
    }
    *out = gctx;
    return BFSX_OK;
}

int bfsx_group_size(const bfsx_ctx *ctx) { return !ctx ? BFSX_E_ARG : is_group(ctx) ? (int)ctx->ranks.size() : 1; }

void bfsx_finalize(bfsx_ctx *ctx) {
    if (!ctx) return;
    for (bfsx_ctx *c : ctx->ranks) bfsx_finalize(c);
    ctx->ranks.clear();
    (void)hipSetDevice(ctx->device);
    ctx->comm.reset();
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

static int set_option_one(bfsx_ctx *ctx, const char *key, const char *value);

int bfsx_set_option(bfsx_ctx *ctx, const char *key, const char *value) {
    if (!ctx || !key || !value) return fail(BFSX_E_ARG, "null argument");
    if (int rc = set_option_one(ctx, key, value)) return rc;
    for (bfsx_ctx *c : ctx->ranks) // a group context: every rank's
        if (int rc = set_option_one(c, key, value)) return rc;
    return BFSX_OK;
}

static int set_option_one(bfsx_ctx *ctx, const char *key, const char *value) {
    const std::string k(key), v(value);
#ifndef BFSX_DIAG
    // test hooks and diagnostics exist in the diagnostic library only (libbfsx_diag.so, built with BFSX_DIAG);
    // "off" is accepted (a no-op) so that a caller resetting them needs no special case
    for (const char *d : {"poison_queues", "test_overread", "bu_force_spill", "persist_abort_at", "check_retired", "fail_at",
                          "slot_force", "race_probe"})
        if (k == d) {
            if (v == "off") return BFSX_OK;
            return fail(BFSX_E_ARG, k + " is a test hook of the diagnostic library (libbfsx_diag.so, built with "
                                        "BFSX_DIAG); the product library does not compile it");
        }
#endif
    auto as_int = [&](int &dst) -> int {
        char *end = nullptr;
        long x = strtol(value, &end, 10);
        if (!end || *end || x <= 0 || x > (1L << 30)) return fail(BFSX_E_ARG, "bad integer for " + k);
        dst = (int)x;
        return BFSX_OK;
    };
    if (k == "direction") {
        if (v == "auto") ctx->opt.direction = BFSX_DIR_AUTO;
        else if (v == "topdown") ctx->opt.direction = BFSX_DIR_TOPDOWN;
        else if (v == "bottomup") ctx->opt.direction = BFSX_DIR_BOTTOMUP;
        else return fail(BFSX_E_ARG, "direction must be auto|topdown|bottomup");
        return BFSX_OK;
    }
    if (k == "row_order") {
        if (v == "degree") ctx->opt.degree_order = true;
        else if (v == "id") ctx->opt.degree_order = false;
        else return fail(BFSX_E_ARG, "row_order must be degree|id");
        return BFSX_OK;
    }
    if (k == "relabel") {
        if (v == "on") ctx->opt.relabel = true;
        else if (v == "off") ctx->opt.relabel = false;
        else return fail(BFSX_E_ARG, "relabel must be on|off");
        return BFSX_OK;
    }
    if (k == "alpha") return as_int(ctx->opt.alpha);
    if (k == "hybrid_pct") return as_int(ctx->opt.hybrid_pct);
    if (k == "beta") return as_int(ctx->opt.beta);
    if (k == "persist") {
        if (v == "on") ctx->opt.persist = true;
        else if (v == "off") ctx->opt.persist = false;
        else return fail(BFSX_E_ARG, "persist must be on|off");
        return BFSX_OK;
    }
    if (k == "vis_front") {
        if (v == "on") ctx->opt.vis_front = true;
        else if (v == "off") ctx->opt.vis_front = false;
        else return fail(BFSX_E_ARG, "vis_front must be on|off");
        return BFSX_OK;
    }
    if (k == "persist_front") {
        if (v == "on") ctx->opt.persist_front = true;
        else if (v == "off") ctx->opt.persist_front = false;
        else return fail(BFSX_E_ARG, "persist_front must be on|off");
        return BFSX_OK;
    }
    if (k == "hub_lds_skip") {
        if (v == "on") ctx->opt.hub_lds_skip = true;
        else if (v == "off") ctx->opt.hub_lds_skip = false;
        else return fail(BFSX_E_ARG, "hub_lds_skip must be on|off");
        return BFSX_OK;
    }
    if (k == "push_log") {
        if (v == "on") ctx->opt.push_log = true;
        else if (v == "off") ctx->opt.push_log = false;
        else return fail(BFSX_E_ARG, "push_log must be on|off");
        return BFSX_OK;
    }
    if (k == "persist_blocks") {
        if (v == "auto") {
            ctx->opt.persist_blocks = 0;
            return BFSX_OK;
        }
        return as_int(ctx->opt.persist_blocks);
    }
    if (k == "persist_abort_at") {
        if (v == "off") {
            ctx->opt.persist_abort_at = -1;
            return BFSX_OK;
        }
        char *end = nullptr;
        const long x = strtol(value, &end, 10);
        if (!end || *end || x < 0 || x > (1L << 20)) return fail(BFSX_E_ARG, "persist_abort_at must be off|level >= 0");
        ctx->opt.persist_abort_at = (int)x;
        return BFSX_OK;
    }
    if (k == "pull_min_edges") {
        char *end = nullptr;
        const long long x = std::strtoll(v.c_str(), &end, 10);
        if (!end || *end || x < 0) return fail(BFSX_E_ARG, "pull_min_edges must be an edge count >= 0");
        ctx->opt.pull_min_edges = x;
        return BFSX_OK;
    }
    if (k == "persist_dmax") {
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < 1) return fail(BFSX_E_ARG, "persist_dmax must be a degree >= 1");
        ctx->opt.persist_dmax = x;
        return BFSX_OK;
    }
    if (k == "slot_pairs") {
        if (v == "auto") {
            ctx->opt.slot_pairs = -1;
            return BFSX_OK;
        }
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < 0) return fail(BFSX_E_ARG, "slot_pairs must be auto or a pair count >= 0");
        ctx->opt.slot_pairs = x;
        return BFSX_OK;
    }
    if (k == "poison_queues") {
        if (v == "on") ctx->opt.poison_queues = true;
        else if (v == "off") ctx->opt.poison_queues = false;
        else return fail(BFSX_E_ARG, "poison_queues must be on|off");
        return BFSX_OK;
    }
    if (k == "bu_force_spill") {
        if (v == "on") ctx->opt.bu_force_spill = true;
        else if (v == "off") ctx->opt.bu_force_spill = false;
        else return fail(BFSX_E_ARG, "bu_force_spill must be on|off");
        return BFSX_OK;
    }
    if (k == "test_overread") {
        if (v == "off") {
            ctx->opt.test_overread = -1;
            return BFSX_OK;
        }
        char *end = nullptr;
        const long x = strtol(value, &end, 10);
        if (!end || *end || x < 0 || x > (1L << 20)) return fail(BFSX_E_ARG, "test_overread must be off|level >= 0");
        ctx->opt.test_overread = (int)x;
        return BFSX_OK;
    }
    if (k == "sparse_exchange") {
        if (v == "off") ctx->opt.sparse_exchange = 0;
        else if (v == "auto") ctx->opt.sparse_exchange = 1;
        else if (v == "on") ctx->opt.sparse_exchange = 2;
        else return fail(BFSX_E_ARG, "sparse_exchange must be auto|on|off");
        return BFSX_OK;
    }
    if (k == "check_retired") {
        if (v == "on") ctx->opt.check_retired = true;
        else if (v == "off") ctx->opt.check_retired = false;
        else return fail(BFSX_E_ARG, "check_retired must be on|off");
        return BFSX_OK;
    }
    if (k == "check_collectives") {
        if (v == "on") ctx->opt.check_collectives = true;
        else if (v == "off") ctx->opt.check_collectives = false;
        else return fail(BFSX_E_ARG, "check_collectives must be on|off");
        comm_sync_options(ctx);
        return BFSX_OK;
    }
    if (k == "comm_timeout_ms") {
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < 0) return fail(BFSX_E_ARG, "comm_timeout_ms must be a duration >= 0 (0: no deadline)");
        ctx->opt.comm_timeout_ms = x;
        comm_sync_options(ctx);
        return BFSX_OK;
    }
    if (k == "fail_at") { // test hook: "rank:level", "rank:setup" or "off"
        if (v == "off") {
            ctx->opt.fail_rank = ctx->opt.fail_level = -1;
            return BFSX_OK;
        }
        const size_t c = v.find(':');
        char *end = nullptr;
        const long r = c == std::string::npos ? -1 : strtol(v.substr(0, c).c_str(), &end, 10);
        if (r < 0 || r >= 64 || !end || *end) return fail(BFSX_E_ARG, "fail_at must be off|rank:level|rank:setup");
        const std::string l = v.substr(c + 1);
        long lv = -2;
        if (l != "setup") {
            lv = strtol(l.c_str(), &end, 10);
            if (l.empty() || !end || *end || lv < 0) return fail(BFSX_E_ARG, "fail_at must be off|rank:level|rank:setup");
        }
        ctx->opt.fail_rank = (int)r;
        ctx->opt.fail_level = (int)lv;
        return BFSX_OK;
    }
    if (k == "comm_timing") {
        if (v == "on") ctx->opt.comm_timing = true;
        else if (v == "off") ctx->opt.comm_timing = false;
        else return fail(BFSX_E_ARG, "comm_timing must be on|off");
        return BFSX_OK;
    }
    if (k == "race_probe") { // test hook
        if (v == "off") ctx->opt.race_probe = 0;
        else if (v == "delay") ctx->opt.race_probe = 1;
        else if (v == "nobarrier") ctx->opt.race_probe = 2;
        else return fail(BFSX_E_ARG, "race_probe must be off|delay|nobarrier");
        return BFSX_OK;
    }
    if (k == "slot_force") { // test hook: "off" or a slot size in pairs
        if (v == "off") {
            ctx->opt.slot_force = -1;
            return BFSX_OK;
        }
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < 1) return fail(BFSX_E_ARG, "slot_force must be off or a pair count >= 1");
        ctx->opt.slot_force = x;
        return BFSX_OK;
    }
    if (k == "leaf_skip") {
        if (v == "on") ctx->opt.leaf_skip = true;
        else if (v == "off") ctx->opt.leaf_skip = false;
        else return fail(BFSX_E_ARG, "leaf_skip must be on|off");
        return BFSX_OK;
    }
    if (k == "big_degree" || k == "big_cap") {
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < (k == "big_cap" ? 1 : 0) || x > 0xFFFFFFFFll)
            return fail(BFSX_E_ARG, k + " must be an integer in [" + (k == "big_cap" ? "1" : "0") + ", 2^32)");
        (k == "big_cap" ? ctx->opt.big_cap : ctx->opt.big_degree) = x;
        return BFSX_OK;
    }
    if (k == "hybrid") {
        if (v == "off") ctx->opt.hybrid = 0;
        else if (v == "auto") ctx->opt.hybrid = 1;
        else if (v == "force") ctx->opt.hybrid = 2;
        else return fail(BFSX_E_ARG, "hybrid must be auto|off|force");
        return BFSX_OK;
    }
    if (k == "bu_unroll") {
        if (v == "2") ctx->opt.bu_unroll = 2;
        else if (v == "4") ctx->opt.bu_unroll = 4;
        else return fail(BFSX_E_ARG, "bu_unroll must be 2|4");
        return BFSX_OK;
    }
    if (k == "bu_pipeline") {
        if (v == "on") ctx->opt.bu_pipeline = true;
        else if (v == "off") ctx->opt.bu_pipeline = false;
        else return fail(BFSX_E_ARG, "bu_pipeline must be on|off");
        return BFSX_OK;
    }
    if (k == "bu_sparse") {
        if (v == "off") {
            ctx->opt.bu_sparse = 0;
            return BFSX_OK;
        }
        return as_int(ctx->opt.bu_sparse);
    }
    if (k == "bu_lds_prefix") {
        if (v == "on") ctx->opt.bu_lds_prefix = true;
        else if (v == "off") ctx->opt.bu_lds_prefix = false;
        else return fail(BFSX_E_ARG, "bu_lds_prefix must be on|off");
        return BFSX_OK;
    }
    if (k == "build_chunk") {
        char *end = nullptr;
        const long long x = strtoll(value, &end, 10);
        if (!end || *end || x < 1) return fail(BFSX_E_ARG, "build_chunk must be a positive entry count");
        ctx->opt.build_chunk = x;
        return BFSX_OK;
    }
    if (k == "hub_bits") {
        if (v == "auto") ctx->opt.hub_bits = -1;
        else if (v == "off") ctx->opt.hub_bits = 0;
        else {
            int b = 0;
            if (int rc = as_int(b)) return rc;
            if (b < 1 || b > 30) return fail(BFSX_E_ARG, "hub_bits must be auto|off|1..30");
            ctx->opt.hub_bits = b;
        }
        return BFSX_OK;
    }
    if (k == "offset_bits") {
        if (v == "auto") ctx->opt.offset_bits = 0;
        else if (v == "64") ctx->opt.offset_bits = 64;
        else return fail(BFSX_E_ARG, "offset_bits must be auto|64");
        return BFSX_OK;
    }
    if (k == "hub_degree") {
        int h = 0;
        int rc = as_int(h);
        if (!rc) ctx->opt.hub_degree = (uint32_t)h;
        return rc;
    }
    return fail(BFSX_E_ARG, "unknown option " + k);
}

// rank/nranks > 1: 1-D partition -- this rank keeps the rows of global ids [rank*chunk, +chunk),
// chunk = ceil(nv / nranks) rounded up to a multiple of 64 (frontier slices are whole bitmap words).
static bfsx_graph *new_partition(bfsx_ctx *ctx, int64_t nv, int64_t m, int rank, int nranks) {
    auto *g = new (std::nothrow) bfsx_graph();
    if (!g) return nullptr;
    g->ctx = ctx;
    g->m = m;
    g->nv_global = nv;
    g->rank = rank;
    g->nranks = nranks;
    if (nranks > 1) {
        g->chunk = ((nv + nranks - 1) / nranks + 63) / 64 * 64;
        g->v_lo = std::min<int64_t>((int64_t)rank * g->chunk, nv);
        g->nv = std::min<int64_t>(g->chunk, nv - g->v_lo);
    } else {
        g->chunk = (nv + 63) / 64 * 64; // whole bitmap words, like the partitioned case
        g->v_lo = 0;
        g->nv = nv;
    }
    return g;
}

// dist: built for the partitioned loop (bfsx_dist_*).  The relabel renumbers inside every rank's id
// range (ranges of `chunk` ids; one range on one device), so ownership never changes.
static int graph_from_device_edges(bfsx_ctx *ctx, int64_t nv, uint32_t *d_u, uint32_t *d_v, int64_t m, int rank,
                                   int nranks, bfsx_graph **out, bool dist) {
    bfsx_graph *g = new_partition(ctx, nv, m, rank, nranks);
    if (!g) return fail(BFSX_E_OOM, "graph");
    set_build_chunk(ctx->opt.build_chunk);
    (void)dist;
    int rc = build_csr_device(ctx->stream, g->nv, d_u, d_v, m, ctx->opt.degree_order, ctx->opt.relabel ? g->chunk : 0,
                              &g->d_row_off, &g->d_col, &g->nnz, &g->d_tuple_cnt, &g->d_perm, &g->d_inv, g->v_lo, nv);
    if (rc) {
        delete g;
        return rc;
    }
    *out = g;
    return BFSX_OK;
}

static int graph_from_host_edges(bfsx_ctx *ctx, int64_t nv, const uint32_t *u, const uint32_t *v, int64_t m,
                                 int rank, int nranks, bfsx_graph **out, bool dist) {
    if (!ctx || !out || nv <= 0 || m < 0 || (m > 0 && (!u || !v))) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(ctx)) return fail(BFSX_E_ARG, "a group context partitions its graphs itself (bfsx_graph_from_edges)");
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) return fail(BFSX_E_ARG, "bad rank/nranks");
    if (nv > (int64_t)INT32_MAX) return fail(BFSX_E_ARG, "nv must be < 2^31 on one device");
    for (int64_t i = 0; i < m; i++)
        if ((int64_t)u[i] >= nv || (int64_t)v[i] >= nv)
            return fail(BFSX_E_RANGE, "tuple " + std::to_string(i) + " has a vertex id >= nv");
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    uint32_t *d_u = nullptr, *d_v = nullptr;
    BFSX_HIP_TRY(hipMalloc(&d_u, std::max<int64_t>(m, 1) * sizeof(uint32_t)));
    hipError_t e = hipMalloc(&d_v, std::max<int64_t>(m, 1) * sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipFree(d_u);
        return fail(BFSX_E_OOM, "device tuples");
    }
    int rc = BFSX_OK;
    if (m > 0) {
        if (hipMemcpyAsync(d_u, u, m * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(d_v, v, m * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
            rc = fail(BFSX_E_HIP, "H2D tuples");
    }
    if (!rc) rc = graph_from_device_edges(ctx, nv, d_u, d_v, m, rank, nranks, out, dist);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    return rc;
}

int bfsx_graph_from_edges(bfsx_ctx *ctx, int64_t nv, const uint32_t *u, const uint32_t *v, int64_t m,
                          bfsx_graph **out) {
    if (is_group(ctx)) {
        if (!out) return fail(BFSX_E_ARG, "null out");
        const int P = (int)ctx->ranks.size();
        return group_graph(ctx, out, [&](int r, bfsx_graph **o) {
            return graph_from_host_edges(ctx->ranks[r], nv, u, v, m, r, P, o, true);
        });
    }
    return graph_from_host_edges(ctx, nv, u, v, m, 0, 1, out, false);
}

int bfsx_dist_graph_from_edges(bfsx_ctx *ctx, int64_t nv, const uint32_t *u, const uint32_t *v, int64_t m, int rank,
                               int nranks, bfsx_graph **out) {
    return graph_from_host_edges(ctx, nv, u, v, m, rank, nranks, out, true);
}

int bfsx_dist_graph_load_algs4(bfsx_ctx *ctx, const char *path, int rank, int nranks, bfsx_graph **out) {
    if (!ctx || !path || !out || is_group(ctx)) return fail(BFSX_E_ARG, "bad argument");
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) return fail(BFSX_E_ARG, "bad rank/nranks");
    int64_t nv = 0, m = 0;
    uint32_t *d_u = nullptr, *d_v = nullptr;
    // every rank tokenizes the whole file on its own device (kernels_parse.hip) and keeps the rows it owns
    int rc = load_algs4_device(ctx, path, nv, m, d_u, d_v);
    if (rc) return rc;
    if (nv > (int64_t)INT32_MAX) rc = fail(BFSX_E_ARG, "nv must be < 2^31");
    if (!rc) rc = graph_from_device_edges(ctx, nv, d_u, d_v, m, rank, nranks, out, true);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    return rc;
}

int bfsx_graph_load_algs4(bfsx_ctx *ctx, const char *path, bfsx_graph **out) {
    if (!ctx || !path || !out) return fail(BFSX_E_ARG, "null argument");
    if (is_group(ctx)) {
        const int P = (int)ctx->ranks.size();
        return group_graph(ctx, out, [&](int r, bfsx_graph **o) {
            return bfsx_dist_graph_load_algs4(ctx->ranks[r], path, r, P, o);
        });
    }
    int64_t nv = 0, m = 0;
    uint32_t *d_u = nullptr, *d_v = nullptr;
    int rc = load_algs4_device(ctx, path, nv, m, d_u, d_v);
    if (rc) return rc;
    if (nv > (int64_t)INT32_MAX) rc = fail(BFSX_E_ARG, "nv must be < 2^31 on one device");
    if (!rc) rc = graph_from_device_edges(ctx, nv, d_u, d_v, m, 0, 1, out, false);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    return rc;
}

int bfsx_parse_algs4_gpu(bfsx_ctx *ctx, const char *path, int64_t *nv_out, int64_t *m_out, uint32_t **u_out,
                         uint32_t **v_out) {
    if (!ctx || !path || !nv_out || !m_out || !u_out || !v_out) return fail(BFSX_E_ARG, "null argument");
    if (is_group(ctx)) ctx = ctx->ranks[0];
    int64_t nv = 0, m = 0;
    uint32_t *d_u = nullptr, *d_v = nullptr;
    int rc = load_algs4_device(ctx, path, nv, m, d_u, d_v);
    if (rc) return rc;
    uint32_t *u = (uint32_t *)malloc(std::max<int64_t>(m, 1) * sizeof(uint32_t));
    uint32_t *v = (uint32_t *)malloc(std::max<int64_t>(m, 1) * sizeof(uint32_t));
    if (!u || !v) rc = fail(BFSX_E_OOM, "out of host memory");
    if (!rc && m > 0 &&
        (hipMemcpy(u, d_u, m * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(v, d_v, m * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess))
        rc = fail(BFSX_E_HIP, "D2H tuples");
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    if (rc) {
        free(u);
        free(v);
        return rc;
    }
    *nv_out = nv;
    *m_out = m;
    *u_out = u;
    *v_out = v;
    return BFSX_OK;
}

int bfsx_kronecker_edges(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, uint32_t *u, uint32_t *v) {
    if (!ctx || !u || !v || scale < 1 || scale > 31 || edgefactor < 1) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(ctx)) ctx = ctx->ranks[0];
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    const int64_t m = (int64_t)edgefactor << scale;
    uint32_t *d_u = nullptr, *d_v = nullptr;
    BFSX_HIP_TRY(hipMalloc(&d_u, m * sizeof(uint32_t)));
    if (hipMalloc(&d_v, m * sizeof(uint32_t)) != hipSuccess) {
        (void)hipFree(d_u);
        return fail(BFSX_E_OOM, "device tuples");
    }
    int rc = kronecker_generate(ctx->stream, scale, edgefactor, seed, d_u, d_v);
    if (!rc && (hipMemcpyAsync(u, d_u, m * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                hipMemcpyAsync(v, d_v, m * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                hipStreamSynchronize(ctx->stream) != hipSuccess))
        rc = fail(BFSX_E_HIP, "D2H tuples");
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    return rc;
}

static int graph_kronecker(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, int rank, int nranks,
                           bfsx_graph **out, bool dist) {
    if (!ctx || !out || scale < 1 || scale > 30 || edgefactor < 1) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(ctx)) {
        if (dist) return fail(BFSX_E_ARG, "a group context partitions its graphs itself (bfsx_graph_kronecker)");
        const int P = (int)ctx->ranks.size();
        return group_graph(ctx, out, [&](int r, bfsx_graph **o) {
            return graph_kronecker(ctx->ranks[r], scale, edgefactor, seed, r, P, o, true);
        });
    }
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) return fail(BFSX_E_ARG, "bad rank/nranks");
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    const int64_t nv = (int64_t)1 << scale;
    const int64_t m = (int64_t)edgefactor << scale;
    // built straight from the counter stream: no tuple arrays (8 B per tuple, 137 GB at scale 30)
    bfsx_graph *g = new_partition(ctx, nv, m, rank, nranks);
    if (!g) return fail(BFSX_E_OOM, "graph");
    set_build_chunk(ctx->opt.build_chunk);
    (void)dist;
    int rc = build_csr_kronecker(ctx->stream, scale, edgefactor, seed, ctx->opt.degree_order,
                                 ctx->opt.relabel ? g->chunk : 0, &g->d_row_off, &g->d_col, &g->nnz, &g->d_tuple_cnt,
                                 &g->d_perm, &g->d_inv, g->v_lo, g->nv);
    (void)hipStreamSynchronize(ctx->stream);
    if (rc) {
        delete g;
        return rc;
    }
    *out = g;
    return BFSX_OK;
}

int bfsx_graph_kronecker(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, bfsx_graph **out) {
    return graph_kronecker(ctx, scale, edgefactor, seed, 0, 1, out, false);
}

int bfsx_dist_graph_kronecker(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, int rank, int nranks,
                              bfsx_graph **out) {
    return graph_kronecker(ctx, scale, edgefactor, seed, rank, nranks, out, true);
}

int bfsx_graph_partition(const bfsx_graph *g, int64_t *nv_global, int64_t *v_lo, int64_t *nv_local, int64_t *chunk,
                         int32_t *rank, int32_t *nranks) {
    if (!g) return fail(BFSX_E_ARG, "null graph");
    if (is_group(g)) { // the whole graph, held by nranks ranks of this process
        if (nv_global) *nv_global = g->nv_global;
        if (v_lo) *v_lo = 0;
        if (nv_local) *nv_local = g->nv_global;
        if (chunk) *chunk = g->chunk;
        if (rank) *rank = 0;
        if (nranks) *nranks = (int32_t)g->parts.size();
        return BFSX_OK;
    }
    if (nv_global) *nv_global = g->nv_global;
    if (v_lo) *v_lo = g->v_lo;
    if (nv_local) *nv_local = g->nv;
    if (chunk) *chunk = g->chunk;
    if (rank) *rank = g->rank;
    if (nranks) *nranks = g->nranks;
    return BFSX_OK;
}

#define BFSX_DIST_GUARD(g)                                                                           \
    do {                                                                                             \
        if (!(g)) return fail(BFSX_E_ARG, "null graph");                                             \
        if (is_group(g)) return fail(BFSX_E_ARG, "a group graph runs its ranks itself: use bfsx_bfs"); \
        BFSX_HIP_TRY(hipSetDevice((g)->ctx->device));                                                \
    } while (0)

int bfsx_graph_degree(const bfsx_graph *g, int64_t v, int64_t *deg) {
    if (!g || !deg) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) {
        if (v < 0 || v >= g->nv_global) {
            *deg = -1;
            return BFSX_OK;
        }
        return bfsx_graph_degree(g->parts[(size_t)(v / g->chunk)], v, deg);
    }
    *deg = -1;
    if (v < g->v_lo || v >= g->v_lo + g->nv) return BFSX_OK;
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    int64_t x = 0;
    if (int rc = to_internal(g, v, &x)) return rc;
    int64_t off[2];
    BFSX_HIP_TRY(hipMemcpy(off, g->d_row_off + (x - g->v_lo), sizeof(off), hipMemcpyDeviceToHost));
    *deg = off[1] - off[0];
    return BFSX_OK;
}

int bfsx_dist_begin(bfsx_graph *g, int64_t source, int64_t *deg_local) {
    BFSX_DIST_GUARD(g);
    int64_t d = 0;
    int rc = dist_begin(g, source, &d);
    if (deg_local) *deg_local = d;
    return rc;
}

int bfsx_dist_frontier_info(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local) {
    BFSX_DIST_GUARD(g);
    int64_t a = 0, b = 0;
    int q = 0;
    int rc = dist_frontier_info(g, &a, &b, &q);
    if (nf_local) *nf_local = a;
    if (mf_local) *mf_local = b;
    return rc;
}

int bfsx_dist_td_expand(bfsx_graph *g, void *d_send, int64_t send_cap, int64_t *send_counts) {
    BFSX_DIST_GUARD(g);
    if (!send_counts || (!d_send && send_cap > 0)) return fail(BFSX_E_ARG, "bad argument");
    return dist_td_expand(g, (unsigned long long *)d_send, send_cap, send_counts);
}

int bfsx_dist_td_claim(bfsx_graph *g, const void *d_recv, int64_t n) {
    BFSX_DIST_GUARD(g);
    return dist_td_claim(g, (const unsigned long long *)d_recv, n);
}

int bfsx_dist_frontier_slice(bfsx_graph *g, void *d_slice) {
    BFSX_DIST_GUARD(g);
    if (!d_slice) return fail(BFSX_E_ARG, "null slice");
    return dist_frontier_slice(g, (unsigned long long *)d_slice);
}

int bfsx_dist_bu_step(bfsx_graph *g, const void *d_front_global) {
    BFSX_DIST_GUARD(g);
    if (!d_front_global) return fail(BFSX_E_ARG, "null frontier");
    return dist_bu_step(g, (const unsigned long long *)d_front_global);
}

int bfsx_dist_level_end(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local) {
    BFSX_DIST_GUARD(g);
    int64_t a = 0, b = 0;
    int rc = dist_level_end(g, &a, &b);
    if (nf_local) *nf_local = a;
    if (mf_local) *mf_local = b;
    return rc;
}

int bfsx_dist_finish(bfsx_graph *g) {
    BFSX_DIST_GUARD(g);
    return dist_finish(g);
}

int bfsx_dist_bfs(bfsx_graph *g, int64_t source, bfsx_stats *stats) {
    BFSX_DIST_GUARD(g);
    return dist_bfs_run(g, source, stats);
}

int bfsx_dist_mcomp(bfsx_graph *g, int64_t *m_local, int64_t *reached_local) {
    BFSX_DIST_GUARD(g);
    int64_t a = 0, b = 0;
    int rc = bfs_mcomp(g, &a, &b);
    if (m_local) *m_local = a;
    if (reached_local) *reached_local = b;
    return rc;
}

void bfsx_graph_free(bfsx_graph *g) {
    if (!g) return;
    for (bfsx_graph *p : g->parts) bfsx_graph_free(p);
    g->parts.clear();
    (void)hipSetDevice(g->ctx->device);
    bfs_workspace_free(g->ws);
    if (g->d_row_off) (void)hipFree(g->d_row_off);
    if (g->d_col) (void)hipFree(g->d_col);
    if (g->d_tuple_cnt) (void)hipFree(g->d_tuple_cnt);
    if (g->d_perm) (void)hipFree(g->d_perm);
    if (g->d_inv) (void)hipFree(g->d_inv);
    delete g;
}

int64_t bfsx_graph_nv(const bfsx_graph *g) { return g ? g->nv : -1; }
int64_t bfsx_graph_nnz(const bfsx_graph *g) { return g ? g->nnz : -1; }
int64_t bfsx_graph_m(const bfsx_graph *g) { return g ? g->m : -1; }

int bfsx_graph_csr(const bfsx_graph *g, int64_t *row_off, uint32_t *col) {
    if (!g) return fail(BFSX_E_ARG, "null graph");
    if (is_group(g)) { // the ranks' rows in id order, one after the other
        int64_t base = 0;
        for (const bfsx_graph *p : g->parts) {
            std::vector<int64_t> off((size_t)p->nv + 1);
            BFSX_HIP_TRY(hipSetDevice(p->ctx->device));
            if (int rc = bfsx_graph_csr(p, off.data(), col ? col + base : nullptr)) return rc;
            if (row_off)
                for (int64_t i = 0; i <= p->nv; i++) row_off[p->v_lo + i] = base + off[(size_t)i];
            base += off[(size_t)p->nv];
        }
        return BFSX_OK;
    }
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    if (g->d_perm) return export_csr_original(g->ctx->stream, g->nv, g->nnz, g->d_row_off, g->d_col, g->d_perm,
                                              g->d_inv, row_off, col);
    if (row_off)
        BFSX_HIP_TRY(hipMemcpyAsync(row_off, g->d_row_off, (g->nv + 1) * sizeof(int64_t), hipMemcpyDeviceToHost,
                                    g->ctx->stream));
    if (col && g->nnz)
        BFSX_HIP_TRY(
            hipMemcpyAsync(col, g->d_col, g->nnz * sizeof(uint32_t), hipMemcpyDeviceToHost, g->ctx->stream));
    BFSX_HIP_TRY(hipStreamSynchronize(g->ctx->stream));
    return BFSX_OK;
}

static int sample_roots_impl(bfsx_graph *g, int count, uint64_t seed, int64_t *roots);

int bfsx_sample_roots(bfsx_graph *g, int count, uint64_t seed, int64_t *roots) {
    if (!g || !roots || count < 0) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) {
        const int P = (int)g->parts.size();
        std::vector<std::vector<int64_t>> got(P, std::vector<int64_t>((size_t)count + 1));
        if (int rc = run_ranks(g->ctx->ranks, [&](int r) { return bfsx_sample_roots(g->parts[r], count, seed, got[r].data()); }))
            return rc;
        std::copy(got[0].begin(), got[0].begin() + count, roots);
        return BFSX_OK;
    }
    const int rc = sample_roots_impl(g, count, seed, roots);
    return g->nranks > 1 ? comm_guard(g->ctx->comm.get(), rc) : rc; // collective on a partition
}

static int sample_roots_impl(bfsx_graph *g, int count, uint64_t seed, int64_t *roots) {
    // a partitioned graph samples collectively: the owner of each candidate decides, the verdict is
    // all-reduced, so every rank returns the same roots as the single-device graph would
    const bool part = g->nranks > 1;
    Comm *cm = g->ctx->comm.get();
    if (part && (!cm || cm->nranks != g->nranks || cm->rank != g->rank))
        return fail(BFSX_E_ARG, "partitioned graph: attach a communicator first (sampling is collective)");
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    hipStream_t st = g->ctx->stream;
    struct DevFlag {
        int64_t *p = nullptr;
        ~DevFlag() {
            if (p) (void)hipFree(p);
        }
    } flag;
    if (part) BFSX_HIP_TRY(hipMalloc(&flag.p, sizeof(int64_t)));
    std::unordered_set<int64_t> seen;
    int found = 0;
    const uint64_t max_tries = 1000ull + 1000ull * (uint64_t)count;
    for (uint64_t t = 0; t < max_tries && found < count; t++) {
        const int64_t x = (int64_t)(mix64(seed + t) % (uint64_t)g->nv_global);
        if (seen.count(x)) continue;
        int64_t ok = 0;
        if (x >= g->v_lo && x < g->v_lo + g->nv) {
            int64_t xi = x; // internal id (relabelled single-device graphs)
            if (int rc = to_internal(g, x, &xi)) return rc;
            int64_t off[2];
            BFSX_HIP_TRY(hipMemcpy(off, g->d_row_off + (xi - g->v_lo), sizeof(off), hipMemcpyDeviceToHost));
            const int64_t deg = off[1] - off[0];
            ok = deg > 0;
            if (deg == 1) { // only neighbour may be a self-loop (Graph500: degree >= 1 excluding self-loops)
                uint32_t nb = 0;
                BFSX_HIP_TRY(hipMemcpy(&nb, g->d_col + off[0], sizeof(nb), hipMemcpyDeviceToHost));
                ok = (int64_t)nb != xi;
            }
        }
        if (part) {
            // fills, not pageable copies: neither may block the host behind a collective a failed peer never joins
            BFSX_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)flag.p, (int)ok, 1, st));
            BFSX_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)((uint32_t *)flag.p + 1), 0, 1, st));
            if (int e = cm->allreduce_sum(flag.p, 1, st)) return e;
            if (int e = comm_fetch(cm, st, &ok, flag.p, sizeof(ok), "root sampling")) return e;
        }
        if (!ok) continue;
        seen.insert(x);
        roots[found++] = x;
    }
    if (found < count) return fail(BFSX_E_ARG, "could not sample enough roots with degree >= 1");
    return BFSX_OK;
}

int bfsx_bfs(bfsx_graph *g, int64_t source, int32_t *dist_out, int64_t *parent_out, bfsx_stats *stats) {
    if (!g) return fail(BFSX_E_ARG, "null graph");
    if (is_group(g)) return group_bfs(g, source, dist_out, parent_out, stats);
    if (g->nranks > 1) return fail(BFSX_E_ARG, "partitioned graph: run it with bfsx_dist_bfs (collective over the ranks)");
    const auto t0 = std::chrono::steady_clock::now();
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    if (source < 0 || source >= g->nv)
        return fail(BFSX_E_RANGE, "source vertex " + std::to_string(source) + " outside [0, " + std::to_string(g->nv) +
                                      ")");
    int64_t si = source;
    if (int rc = to_internal(g, source, &si)) return rc;
    bfsx_stats local{};
    const int64_t retries0 = bfs_persist_fallbacks(g);
    int rc = bfs_run(g, si, &local);
    if (rc) return rc;
    local.persist_retries = (int32_t)(bfs_persist_fallbacks(g) - retries0);
    if (dist_out || parent_out) {
        rc = bfs_copy_result(g, dist_out, parent_out);
        if (rc) return rc;
    }
    if (stats) {
        rc = bfs_mcomp(g, &local.m_comp, &local.reached);
        if (rc) return rc;
        local.t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        *stats = local;
    }
    return BFSX_OK;
}

int bfsx_validate(bfsx_graph *g, int64_t source, int64_t *errors, int64_t *first_bad, int64_t *reached,
                  int64_t *entries) {
    if (!g) return fail(BFSX_E_ARG, "null graph");
    if (is_group(g)) {
        if (source < 0) source = g->last_source;
        const int P = (int)g->parts.size();
        std::vector<std::array<int64_t, 4>> res(P);
        if (int rc = run_ranks(g->ctx->ranks, [&](int r) {
                return bfsx_validate(g->parts[r], source, &res[r][0], &res[r][1], &res[r][2], &res[r][3]);
            }))
            return rc;
        if (errors) *errors = res[0][0]; // collective: every rank holds the all-reduced verdict
        if (first_bad) *first_bad = res[0][1];
        if (reached) *reached = res[0][2];
        if (entries) *entries = res[0][3];
        return BFSX_OK;
    }
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    int64_t res[4] = {0, -1, 0, 0};
    int64_t si = source;
    if (source >= 0 && g->nranks == 1) {
        if (source >= g->nv) return fail(BFSX_E_ARG, "source out of range");
        if (int rc = to_internal(g, source, &si)) return rc;
    } else if (source >= 0 && g->d_perm) { // relabelled partition: the owner maps the source (collective)
        if (source >= g->nv_global) return fail(BFSX_E_ARG, "source out of range");
        if (int rc = dist_map_source(g, source, &si)) return rc;
    }
    if (int rc = bfs_validate(g, si, nullptr, res)) return g->nranks > 1 ? comm_guard(g->ctx->comm.get(), rc) : rc;
    if (int rc = to_original(g, res[1], &res[1])) return rc;
    if (errors) *errors = res[0];
    if (first_bad) *first_bad = res[1];
    if (reached) *reached = res[2];
    if (entries) *entries = res[3];
    return BFSX_OK;
}

int bfsx_validate_result(bfsx_graph *g, int64_t source, const int32_t *dist, const int64_t *parent, int64_t *errors,
                         int64_t *first_bad) {
    if (!g || !dist || !parent) return fail(BFSX_E_ARG, "null argument");
    if (g->nranks > 1 || is_group(g)) return fail(BFSX_E_ARG, "partitioned graph: use bfsx_validate (collective)");
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    std::vector<unsigned long long> packed((size_t)g->nv);
    std::vector<uint32_t> perm;
    int64_t si = source;
    if (g->d_perm) { // the caller's arrays are indexed by original ids; the device checks internal ones
        if (source < 0 || source >= g->nv) return fail(BFSX_E_ARG, "source out of range");
        perm.resize((size_t)g->nv);
        BFSX_HIP_TRY(hipMemcpy(perm.data(), g->d_perm, perm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        si = perm[(size_t)source];
    }
    for (int64_t i = 0; i < g->nv; i++) {
        const int64_t p = parent[i];
        uint32_t pw = (uint32_t)p;
        if (!perm.empty() && p >= 0 && p < g->nv) pw = perm[(size_t)p];
        const size_t at = perm.empty() ? (size_t)i : (size_t)perm[(size_t)i];
        packed[at] = ((unsigned long long)pw << 32) | (uint32_t)dist[i];
    }
    unsigned long long *d = nullptr;
    BFSX_HIP_TRY(hipMalloc(&d, std::max<size_t>(packed.size(), 1) * sizeof(unsigned long long)));
    hipError_t he = hipMemcpy(d, packed.data(), packed.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
    int64_t res[4] = {0, -1, 0, 0};
    int rc = he == hipSuccess ? bfs_validate(g, si, d, res)
                              : fail(BFSX_E_HIP, std::string("validate upload: ") + hipGetErrorString(he));
    (void)hipFree(d);
    if (rc) return rc;
    if (!perm.empty() && res[1] >= 0) {
        uint32_t v = 0;
        BFSX_HIP_TRY(hipMemcpy(&v, g->d_inv + res[1], sizeof(v), hipMemcpyDeviceToHost));
        res[1] = v;
    }
    if (errors) *errors = res[0];
    if (first_bad) *first_bad = res[1];
    return BFSX_OK;
}

int bfsx_result(bfsx_graph *g, int32_t *dist_out, int64_t *parent_out) {
    if (!g) return fail(BFSX_E_ARG, "null graph");
    if (is_group(g))
        return run_ranks(g->ctx->ranks, [&](int r) {
            bfsx_graph *p = g->parts[r];
            return bfs_copy_result(p, dist_out ? dist_out + p->v_lo : nullptr, parent_out ? parent_out + p->v_lo : nullptr);
        });
    BFSX_HIP_TRY(hipSetDevice(g->ctx->device));
    return bfs_copy_result(g, dist_out, parent_out);
}

int bfsx_level_times(bfsx_graph *g, double *cum_ms, int cap) {
    if (!g || (!cum_ms && cap > 0)) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) { // per level: the slowest rank's cumulative device time
        const int n = (int)std::min<size_t>(g->parts[0]->level_cum_ms.size(), (size_t)std::max(cap, 0));
        for (int i = 0; i < n; i++) {
            cum_ms[i] = 0;
            for (const bfsx_graph *p : g->parts)
                if ((size_t)i < p->level_cum_ms.size()) cum_ms[i] = std::max(cum_ms[i], p->level_cum_ms[i]);
        }
        return n;
    }
    int n = (int)std::min<size_t>(g->level_cum_ms.size(), (size_t)std::max(cap, 0));
    for (int i = 0; i < n; i++) cum_ms[i] = g->level_cum_ms[i];
    return n;
}

int bfsx_last_bfs_ms(const bfsx_graph *g, double *ms) {
    if (!g || !ms) return fail(BFSX_E_ARG, "bad argument");
    if (g->last_source < 0) return fail(BFSX_E_ARG, "no BFS result on this graph yet");
    *ms = g->last_t_bfs_ms;
    return BFSX_OK;
}

int bfsx_persist_fallbacks(const bfsx_graph *g, int64_t *count) {
    if (!g || !count) return fail(BFSX_E_ARG, "bad argument");
    *count = bfs_persist_fallbacks(g);
    return BFSX_OK;
}

int bfsx_comm_times(const bfsx_graph *g, double *ms, int64_t *count) {
    if (!g || !ms || !count) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) { // the largest span over the ranks, per kind
        for (int k = 0; k < 4; k++) {
            ms[k] = 0.0;
            count[k] = 0;
        }
        for (const bfsx_graph *p : g->parts) {
            double m[4];
            int64_t c[4];
            bfs_comm_times(p, m, c);
            for (int k = 0; k < 4; k++) {
                ms[k] = std::max(ms[k], m[k]);
                count[k] = std::max(count[k], c[k]);
            }
        }
        return BFSX_OK;
    }
    bfs_comm_times(g, ms, count);
    return BFSX_OK;
}

int bfsx_last_unpack_ms(const bfsx_graph *g, double *ms) {
    if (!g || !ms) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) {
        *ms = -1.0;
        for (const bfsx_graph *p : g->parts) *ms = std::max(*ms, bfs_last_unpack_ms(p));
        return BFSX_OK;
    }
    *ms = bfs_last_unpack_ms(g);
    return BFSX_OK;
}

int bfsx_last_resolve_ms(const bfsx_graph *g, double *ms) {
    if (!g || !ms) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) {
        *ms = -1.0;
        for (const bfsx_graph *p : g->parts) *ms = std::max(*ms, bfs_last_resolve_ms(p));
        return BFSX_OK;
    }
    *ms = bfs_last_resolve_ms(g);
    return BFSX_OK;
}

int bfsx_level_dirs(bfsx_graph *g, int32_t *dirs, int cap) {
    if (!g || (!dirs && cap > 0)) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) return bfsx_level_dirs(g->parts[0], dirs, cap); // all-reduced: the same on every rank
    int n = (int)std::min<size_t>(g->level_dirs.size(), (size_t)std::max(cap, 0));
    for (int i = 0; i < n; i++) dirs[i] = g->level_dirs[i];
    return n;
}

int bfsx_level_stats(bfsx_graph *g, bfsx_level_stat *out, int cap) {
    if (!g || (!out && cap > 0)) return fail(BFSX_E_ARG, "bad argument");
    if (is_group(g)) { // counts summed over the ranks, times the slowest rank's
        const int n = bfsx_level_stats(g->parts[0], out, cap);
        std::vector<bfsx_level_stat> o((size_t)std::max(n, 1));
        for (size_t q = 1; q < g->parts.size(); q++) {
            const int k = std::min(n, bfsx_level_stats(g->parts[q], o.data(), n));
            for (int i = 0; i < k; i++) {
                out[i].frontier_in += o[i].frontier_in;
                out[i].frontier_out += o[i].frontier_out;
                out[i].mf_in += o[i].mf_in;
                out[i].unvisited_in += o[i].unvisited_in;
                out[i].scanned += o[i].scanned;
                out[i].claims += o[i].claims;
                out[i].stage2 += o[i].stage2;
                out[i].walked += o[i].walked;
                out[i].explicit_parents += o[i].explicit_parents;
                out[i].kernel_ms = std::max(out[i].kernel_ms, o[i].kernel_ms);
                out[i].cum_ms = std::max(out[i].cum_ms, o[i].cum_ms);
            }
        }
        return n;
    }
    int n = (int)std::min<size_t>(g->level_stats.size(), (size_t)std::max(cap, 0));
    for (int i = 0; i < n; i++) out[i] = g->level_stats[i];
    return n;
}

int bfsx_device_synchronize(bfsx_ctx *ctx) {
    if (!ctx) return fail(BFSX_E_ARG, "null ctx");
    for (bfsx_ctx *c : ctx->ranks)
        if (int rc = bfsx_device_synchronize(c)) return rc;
    if (is_group(ctx)) return BFSX_OK;
    BFSX_HIP_TRY(hipSetDevice(ctx->device));
    BFSX_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return BFSX_OK;
}

} // extern "C"
