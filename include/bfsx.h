/*
 * bfsx.h -- C-ABI of the MI355X-native BFS engine (libbfsx.so).
 *
 * The reference (NorthernDemon/BFS-with-MapReduce) has no FFI: its hot path is the per-problem-file
 * block of BfsSpark.main (src/main/java/it/unitn/bd/bfs/BfsSpark.java:55-118) -- the loader call
 * GraphFileUtil.convert (GraphFileUtil.java:45-69), then the map/reduceByKey level loop whose
 * mapper (BfsSpark.java:66-87) and reducer (BfsSpark.java:90-108) are Spark function objects.
 * Each entry point below names the reference code it replaces.  INTEGRATION.md shows the JNI /
 * Panama binding a maintainer adds to call these from BfsSpark.main.
 *
 * Conventions
 *   - Every int-returning function returns BFSX_OK (0) or a negative BFSX_E_* code; a message for
 *     the calling thread is available from bfsx_last_error().  No C++ exception crosses the ABI.
 *   - Handles are library-owned; free them with the matching *_free / bfsx_finalize.
 *   - Output arrays are caller-allocated HOST memory of length bfsx_graph_nv().
 *   - Distances: int32, INT32_MAX (2147483647) = unreachable, exactly the reference's
 *     Integer.MAX_VALUE initial distance (GraphFileUtil.java:55) that survives for WHITE vertices.
 *   - Parents: int64, -1 = unreachable, parent[source] = source.
 *   - A bfsx_ctx is used by one host thread at a time (like the single driver thread of
 *     BfsSpark.main); bfsx_bfs is synchronous.
 */
#ifndef BFSX_H
#define BFSX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5): bfsx_level_stat gained explicit_parents at its end; bfsx_init_group, bfsx_group_size,
 * bfsx_dist_graph_load_algs4 and bfsx_last_resolve_ms were added
 * 3 (round 6): bfsx_comm_times was added (no layout changed) */
#define BFSX_ABI_VERSION 3

/* Error codes.  Mapping to the reference's exceptions:
 *   E_IO    <- IOException from FileInputStream / Files.write  (GraphFileUtil.java:43,46,68)
 *   E_PARSE <- NumberFormatException / IndexOutOfBoundsException (GraphFileUtil.java:48,61-63)
 *   E_RANGE <- NullPointerException for a vertex id outside [0,V)  (GraphFileUtil.java:64-65)  */
#define BFSX_OK 0
#define BFSX_E_IO (-1)
#define BFSX_E_PARSE (-2)
#define BFSX_E_RANGE (-3)
#define BFSX_E_HIP (-4)
#define BFSX_E_RCCL (-5)
#define BFSX_E_OOM (-6)
#define BFSX_E_ARG (-7)
#define BFSX_E_NODEV (-8)

/* Traversal direction policy (bfsx_set_option "direction"). */
#define BFSX_DIR_AUTO 0     /* direction-optimising (Beamer alpha/beta switch) */
#define BFSX_DIR_TOPDOWN 1  /* push only: the reference mapper's direction (BfsSpark.java:73-79) */
#define BFSX_DIR_BOTTOMUP 2 /* pull only */
#define BFSX_DIR_HYBRID 3   /* (level records only) pull from the frontier's hubs + push from its other vertices */
#define BFSX_DIR_BOTTOMUP_SPARSE 4 /* (level records only) a pull level with few unvisited candidates, run by the
                                     * sparse pull kernel (which also queues the next push frontier) */

typedef struct bfsx_ctx bfsx_ctx;
typedef struct bfsx_graph bfsx_graph;

/* Per-BFS statistics.  levels == the number of map/reduce passes the reference runs for the same
 * graph and source (BfsSpark.java:61, ecc(source)+1), so "Elapsed time [k]" lines line up. */
typedef struct bfsx_stats {
    int32_t levels;          /* map/reduce passes = eccentricity(source) + 1 */
    int32_t topdown_levels;  /* levels run as push (queue -> queue) */
    int32_t bottomup_levels; /* levels run as pull (bitmap -> bitmap) */
    int32_t persist_retries; /* times this BFS was re-run without the persistent push kernel (barrier abort) */
    int64_t reached;         /* vertices with finite distance (BLACK at the end) */
    int64_t m_comp;          /* input edge tuples inside the source's component (TEPS numerator) */
    int64_t edges_examined;  /* sum of frontier degrees over top-down levels + probes (approximate) */
    double t_bfs_ms;         /* device time: source init -> last level complete (hipEvents) */
    double t_total_ms;       /* host wall time of the whole call incl. D2H of outputs */
} bfsx_stats;

/* Per-level record of the most recent bfsx_bfs (diagnostics and roofline accounting). */
typedef struct bfsx_level_stat {
    int32_t direction;     /* BFSX_DIR_TOPDOWN, _BOTTOMUP, _HYBRID or _BOTTOMUP_SPARSE */
    int32_t level;         /* 0-based: expands the vertices at distance `level` */
    int64_t frontier_in;   /* vertices in the frontier being expanded (GRAY before the pass) */
    int64_t frontier_out;  /* vertices discovered (GRAY after the pass) */
    int64_t mf_in;         /* sum of frontier degrees (top-down edges scanned) */
    int64_t unvisited_in;  /* WHITE vertices before the pass (bottom-up candidates) */
    int64_t scanned;       /* adjacency entries read (top-down: mf_in; bottom-up: counted) */
    int64_t claims;        /* top-down: atomic visited-bitmap claims attempted; bottom-up: rows walked past top1 */
    double kernel_ms;      /* device time of this level's kernels (hipEvents around them) */
    double cum_ms;         /* device time since source init, like the reference's Stopwatch */
    int64_t stage2;        /* bottom-up: candidates that read their 2nd..4th neighbours (16-B rest[] load) */
    int64_t walked;        /* bottom-up: adjacency entries read from the CSR past the first four (phase B);
                            * top-down on a partitioned graph: (vertex, parent) pairs this rank sent to others */
    int64_t explicit_parents; /* pull and hybrid levels: discoveries that stored a 4-B parent (the others a 1-B
                               * provenance code only: their parent is their first, 2nd, 3rd or 4th row entry) */
} bfsx_level_stat;

/* ---- library / context ---------------------------------------------------------------------- */
int bfsx_abi_version(void);
const char *bfsx_last_error(void);
/* Replaces: new JavaSparkContext(...) + spark.addJar (BfsSpark.java:50-51). device = HIP ordinal. */
int bfsx_init(int device, bfsx_ctx **out);
/* A group context: nranks ranks inside this process, rank r on HIP device r % (visible devices), one host thread
 * per rank inside every call.  Replaces the Spark cluster the reference connects to (BfsSpark.java:44,50): every
 * graph built on a group context is 1-D partitioned over its ranks (as bfsx_dist_graph_*), and bfsx_bfs /
 * bfsx_result / bfsx_validate / bfsx_level_* on such a graph run the partitioned level loop on all ranks and
 * return once, with whole-graph outputs -- the caller sees one call.  The exchange is an RCCL
 * clique over xGMI when the ranks have distinct devices (ncclCommInitAll), else (ranks sharing a device) the
 * in-process group; environment BFSX_GROUP_COMM=local|rccl forces one.  bfsx_set_option applies to every rank.
 * Not available on a group graph: bfsx_validate_result, the bfsx_dist_* calls, bfsx_comm_*. */
int bfsx_init_group(int nranks, bfsx_ctx **out);
/* Ranks of a context: 1 for a bfsx_init context. */
int bfsx_group_size(const bfsx_ctx *ctx);
void bfsx_finalize(bfsx_ctx *ctx);
/* Options (all optional; defaults preserve reference behaviour):
 *   "direction" = auto|topdown|bottomup ; "alpha" = int (default 20) ; "beta" = int (default 24)
 *   "hub_degree" = int (top-down multi-workgroup bin threshold, default 64)
 *   "row_order" = degree|id (adjacency order inside a CSR row for graphs built afterwards; default
 *                 degree = high-degree neighbours first, which shortens bottom-up probes)
 *   "offset_bits" = auto|64 (row offsets the traversal kernels read: auto = uint32 when the graph has
 *                 < 2^32 adjacency entries, int64 otherwise; 64 forces int64; fixed at a graph's first BFS)
 *   "persist" = on|off (narrow top-down levels run back to back inside one launch; default on)
 *   "vis_front" = on|off (one device: the dense pull level after a push, hybrid or K3p level reads the visited
 *                 bitmap itself as its frontier and writes the updated bitmap into a second buffer, instead of
 *                 a copy of it; default on)
 *   "persist_front" = on|off (a BFS's first such launch that stops because the next level pulls hands the pull
 *                 level its frontier bitmap instead of its queue: with vis_front the visited bitmap itself, so the
 *                 launch only skips its queue hand-back; without, a copy of it in the frontier buffer; default on)
 *   "push_log" = on|off (one device: a per-level push level writes its winners as (vertex, parent) pairs at
 *                 their queue positions instead of scattered state stores; the result read scatters them;
 *                 default on)
 *   "hub_lds_skip" = on|off (single device, relabelled graphs: the multi-workgroup push bin reads the visited bits
 *                 of the 2^16 highest-degree ids from an LDS snapshot taken at the level's start and probes no
 *                 target that snapshot marks visited; default on)
 *   "persist_blocks" = auto|int (workgroups of that launch, auto = three per four CUs (192 on MI355X), capped
 *                 by the occupancy API so that every workgroup is resident; fixed at a graph's first BFS)
 *   "pull_min_edges" = int (a push -> pull switch also needs the frontier to hold at least this many edges,
 *                 besides n/512; default 2^16: a pull level's fixed cost is never recovered below it -- the
 *                 largeG stand-in's tail levels stay in the persistent push launch, 9.69 -> 7.30 ms)
 *   "persist_dmax" = int (inside the persistent launch a frontier row longer than this is "heavy": the whole
 *                 grid sweeps it, each workgroup an equal share of its edges; a frontier handed to the launch by
 *                 the host may hold one only if it is the source alone; default 512: 1,481-1,489 against
 *                 1,456-1,470 GTEPS at 2048, interleaved on one box, profiles/r03/r03y_persist_dmax_ab.txt)
 *   "persist_abort_at" = int|off (test hook: that persistent launch aborts at its k-th level as a barrier
 *                 timeout would; the BFS is then re-run without it; default off)
 *   "hub_bits" = auto|off|1..30 (bottom-up probes of the 2^b highest-degree vertices go to a small
 *                 gathered bitmap; auto = n/1024 rounded up to a power of two; fixed at a graph's first BFS)
 *   "hybrid" = auto|off|force (a top-down level whose frontier's edges sit mostly in hub-domain vertices
 *                 runs as pull-from-hubs + push-from-the-rest; force = every eligible level, for tests)
 *   "hybrid_pct" = int (auto: a level goes hybrid when its frontier's hub edges exceed this percentage
 *                 of the unvisited vertex count; default 125)
 *   "bu_unroll" = 4|2 (bottom-up candidates per lane per round)
 *   "bu_pipeline" = on|off (bottom-up: the next round's first-neighbour loads overlap the current round;
 *                 with bu_unroll 4; default on)
 *   "bu_sparse" = int|off (single device: a pull level with at most n/bu_sparse unvisited candidates runs in
 *                 the sparse pull kernel, which also queues the next push frontier; default 64, 1 = every pull
 *                 level, off = never)
 *   "bu_lds_prefix" = on|off (pull kernels read the frontier bits of the 2^16 highest-degree ids of a
 *                 relabelled single-device graph from a per-workgroup LDS copy; default on)
 *   "slot_pairs" = auto|int (partitioned graphs: a push level whose frontier has at most this many edges in
 *                 total exchanges its pairs through fixed per-peer slots, skipping the count all-to-all
 *                 and its host wait; 0 = never; auto (default) = max(16384, 2^20 / (8 (P - 1))) pairs, so a
 *                 rank sends its peers at most 1 MiB of slots, and 2^22 at P = 1, where nothing is sent)
 *   "build_chunk" = int (CSR build: raw adjacency entries per sort/dedup chunk, default 2^30; bounds the
 *                 build's temporary memory, so a scale-30 Kronecker graph builds on one device)
 *   "leaf_skip" = on|off (single device: the degree-1 vertices a pull level discovers stay out of the next
 *                 push level's queue -- their one neighbour is their parent; default on)
 *   "relabel" = on|off (graphs built after the call renumber their vertices by degree, descending, inside every
 *                 rank's id range; results are always in the caller's ids; default on)
 *   Test hooks and diagnostics (not for production): "poison_queues" = on|off (fill the frontier queues and
 *                 the hub list with 0xFF before every BFS), "test_overread" = int|off (that push level reads one
 *                 queue entry past its tail: the id guard must fail the BFS), "bu_force_spill" = on|off (the
 *                 partitioned pull kernel in a build that spills to scratch), "check_retired" = on|off (the
 *                 partitioned loop fails when a launch or exchange would use a replaced (retired) buffer)
 *   "sparse_exchange" = auto|on|off (partitioned graphs: a pull level whose global frontier holds fewer than
 *                 n/128 vertices receives it as every rank's id list instead of the n/8-byte bitmap
 *                 all-gather (auto, the default); on: every pull level at P > 1; off: never)
 *   "big_degree", "big_cap" = int (partitioned graphs: the ids of degree > big_degree, at most big_cap per
 *                 rank, are all-gathered with their degrees at the first BFS, so every rank knows a source's
 *                 degree; defaults 4096 and 2^20; read at a graph's first partitioned BFS)
 *   "comm_timeout_ms" = int (partitioned graphs: a host wait on the other ranks fails with BFSX_E_RCCL after this
 *                 long and aborts the communicator; 0 = no deadline; default 120000.  A rank that FAILS aborts
 *                 the communicator at once: every rank's call then returns BFSX_E_RCCL "peer rank r failed ...")
 *   "check_collectives" = on|off (debug: every collective first checks that all ranks are in the same
 *                 collective of the same level, and fails on every rank with both names otherwise)
 *   "fail_at" = rank:level|rank:setup|off (test hook: that rank of a partitioned BFS fails at the start of that
 *                 level, or before its first collective)
 *   "comm_timing" = on|off (partitioned graphs: hipEvents around every collective of the level loop, read by
 *                 bfsx_comm_times; default off)
 *   "slot_force" = int|off (test hook: the fixed-slot push levels of a partitioned BFS use slots of this many
 *                 pairs, whatever the level's bound; a too-small slot makes the store guard fail the BFS on
 *                 every rank instead of writing past the slot)
 *   "race_probe" = off|delay|nobarrier (test hook: before every partitioned push level the LDS of every CU is
 *                 filled with stale words and k_td's first wave zeroes its queue counts late; nobarrier also
 *                 drops the barrier after that init -- the rounds-3..5 kernel, whose empty workgroups then flush
 *                 stale counts, which the store guard reports) */
int bfsx_set_option(bfsx_ctx *ctx, const char *key, const char *value);

/* ---- host-only parsing (no device work; usable without a GPU) -------------------------------- */
/* GraphFileUtil.convert's parse (GraphFileUtil.java:46-66): line 1 = V (Integer.parseInt, no trim),
 * line 2 ignored, every further line split on single spaces, tokens 0 and 1 parsed, read to EOF.
 * Vertex 0 always exists (GraphFileUtil.java:53), so nv = max(V,1).  Arrays are malloc'd by the
 * library; release with bfsx_free_host. */
int bfsx_parse_algs4(const char *path, int64_t *nv, int64_t *m, uint32_t **u, uint32_t **v);
void bfsx_free_host(void *p);
/* The same parse with the edge lines tokenized on the GPU (what bfsx_graph_load_algs4 uses; the tuples
 * are copied back here only so the result can be compared): identical tuples, codes and line numbers. */
int bfsx_parse_algs4_gpu(bfsx_ctx *ctx, const char *path, int64_t *nv, int64_t *m, uint32_t **u, uint32_t **v);

/* ---- graph construction (device-resident CSR) ------------------------------------------------ */
/* Replaces GraphFileUtil.convert (GraphFileUtil.java:45-69): parse + symmetrise + dedup into
 * neighbour sets, built as CSR on the GPU.  Self-loops are kept once (HashSet semantics).  The header
 * lines are read on the host, the edge lines are tokenized on the GPU (kernels_parse.hip). */
int bfsx_graph_load_algs4(bfsx_ctx *ctx, const char *path, bfsx_graph **out);
/* Same construction from an in-memory tuple list (host arrays of length m, ids < nv). */
int bfsx_graph_from_edges(bfsx_ctx *ctx, int64_t nv, const uint32_t *u, const uint32_t *v, int64_t m,
                          bfsx_graph **out);
/* Graph500 Kronecker graph (A,B,C,D=.57,.19,.19,.05), generated and built on the GPU.
 * n = 2^scale, m = edgefactor * n tuples; deterministic in (scale, edgefactor, seed). */
int bfsx_graph_kronecker(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, bfsx_graph **out);
/* Copy the generator's tuples to host arrays of length edgefactor<<scale (parity testing). */
int bfsx_kronecker_edges(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, uint32_t *u,
                         uint32_t *v);
void bfsx_graph_free(bfsx_graph *g);

int64_t bfsx_graph_nv(const bfsx_graph *g);  /* vertices */
int64_t bfsx_graph_nnz(const bfsx_graph *g); /* directed adjacency entries after dedup */
int64_t bfsx_graph_m(const bfsx_graph *g);   /* input tuples */
/* D2H copy of the CSR: row_off[nv+1], col[nnz] (either may be NULL).  Each row holds one
 * neighbour set; its order follows the "row_order" option the graph was built with. */
int bfsx_graph_csr(const bfsx_graph *g, int64_t *row_off, uint32_t *col);
/* Graph500 root sampling: count distinct vertices with a non-self-loop neighbour, seeded.  On a
 * partitioned graph it is collective over the context's communicator and returns, on every rank,
 * the roots the single-device graph returns. */
int bfsx_sample_roots(bfsx_graph *g, int count, uint64_t seed, int64_t *roots);

/* ---- the hot path ---------------------------------------------------------------------------- */
/* Replaces the level loop BfsSpark.java:57-118: mapper (frontier expansion, :66-87), reducer
 * (min distance / darkest colour, :90-108), collect + termination test (:110-117).
 * dist_out / parent_out may be NULL (results stay on the device, e.g. inside a timed region). */
int bfsx_bfs(bfsx_graph *g, int64_t source, int32_t *dist_out, int64_t *parent_out, bfsx_stats *stats);
/* Copy the most recent bfsx_bfs result of this graph to host (same layout as bfsx_bfs outputs).  Both outputs
 * NULL: the result is materialised on the device only (the unpack kernel, timed by bfsx_last_unpack_ms). */
int bfsx_result(bfsx_graph *g, int32_t *dist_out, int64_t *parent_out);
/* Device time of each level of the most recent bfsx_bfs, cumulative like the reference's
 * Stopwatch (BfsSpark.java:59,63,111-112).  Returns the number of levels written (<= cap). */
int bfsx_level_times(bfsx_graph *g, double *cum_ms, int cap);
/* Device time (ms) of the most recent BFS of g: source init -> last level complete, the stats.t_bfs_ms
 * figure without the m_comp reduction bfsx_bfs performs when stats are requested (benchmark loops). */
int bfsx_last_bfs_ms(const bfsx_graph *g, double *ms);
/* BFS runs of g re-run without the persistent push kernel since g was built (a K3p grid barrier that timed
 * out; each such BFS's t_bfs covers the aborted attempt too).  Per call: bfsx_stats.persist_retries. */
int bfsx_persist_fallbacks(const bfsx_graph *g, int64_t *count);
/* Device time (ms) of the unpack kernel of the most recent bfsx_bfs / bfsx_result copy: the per-vertex state
 * (internal, degree-ordered ids; a pull level's discoveries as 4-B parents + its level record) -> one word per
 * ORIGINAL id (parent, dist) that the outputs are split from.  It runs after t_bfs (outside the timed region),
 * before the D2H copy; -1 if no copy ran yet. */
int bfsx_last_unpack_ms(const bfsx_graph *g, double *ms);
/* Device time (ms) of the first part of that unpack: the push levels' log scattered and the pull levels' records
 * folded into the per-vertex state, so that a distance and a parent exist for every vertex in the graph's
 * internal (degree-ordered) ids -- Graph500 kernel 2's output, before the translation to the caller's ids; -1 if
 * the last copy did not run it (graphs built with "relabel" off unpack in one scatter pass). */
int bfsx_last_resolve_ms(const bfsx_graph *g, double *ms);
/* Per-level direction of the most recent bfsx_bfs: BFSX_DIR_TOPDOWN (1), BFSX_DIR_BOTTOMUP (2), BFSX_DIR_HYBRID (3)
 * or BFSX_DIR_BOTTOMUP_SPARSE (4). */
int bfsx_level_dirs(bfsx_graph *g, int32_t *dirs, int cap);

/* Per-level records of the most recent bfsx_bfs.  Returns the number written (<= cap). */
int bfsx_level_stats(bfsx_graph *g, bfsx_level_stat *out, int cap);

/* Graph500-style validation of the most recent BFS result of g, on the device, at any size (the CPU
 * oracle's orc_validate rules; Graph500 kernel-2 validation; algs4.jar!/BreadthFirstPaths.java:171-212
 * `check`): dist[source] = 0 and parent[source] = source; every reached v has a parent joined to it by
 * an edge with dist[parent] = dist[v] - 1; unreached vertices have no parent and no reached neighbour;
 * every edge joins vertices whose distances differ by at most one.  A result that passes holds exactly
 * the BFS distances of the graph.  errors = violating vertices (0 = valid), first_bad = one violating
 * vertex in original ids (-1 = none): the smallest violating id of a graph built without the relabel, the
 * violating vertex of smallest INTERNAL id (degree order) on a relabelled one, reached / entries = reached vertices / adjacency entries checked (any
 * output may be NULL).  Collective on a partitioned graph (all-gathers the distances).  source < 0 =
 * the source of the most recent BFS. */
int bfsx_validate(bfsx_graph *g, int64_t source, int64_t *errors, int64_t *first_bad, int64_t *reached,
                  int64_t *entries);
/* The same rules on a caller-supplied result (host arrays of length bfsx_graph_nv: this rank's rows on a
 * partitioned graph), e.g. one read back from a reference run or a file written by the host twin. */
int bfsx_validate_result(bfsx_graph *g, int64_t source, const int32_t *dist, const int64_t *parent,
                         int64_t *errors, int64_t *first_bad);

/* ---- multi-GPU: 1-D vertex partition -------------------------------------------
 * Replaces Spark's hash-partitioned reduceByKey shuffle (BfsSpark.java:90) with an owner-routed
 * exchange.  Rank r of P holds the rows of global ids [r*chunk, r*chunk + nv_local), chunk =
 * ceil(nv/P) rounded up to 64; adjacency entries stay global.  Every rank builds its rows from the
 * same tuple list / Kronecker stream (no edge exchange at build).  The whole partitioned level loop,
 * exchanges included, runs inside the library: bfsx_dist_bfs below.  bfsx_bfs rejects a partitioned
 * graph.  (The per-level primitives the test-suite protocol driver, tests/dist_driver.py, steps through
 * are declared in the test-only header include/bfsx_levels.h; they are not part of this ABI.) */
int bfsx_dist_graph_from_edges(bfsx_ctx *ctx, int64_t nv, const uint32_t *u, const uint32_t *v, int64_t m,
                               int rank, int nranks, bfsx_graph **out);
int bfsx_dist_graph_kronecker(bfsx_ctx *ctx, int scale, int edgefactor, uint64_t seed, int rank, int nranks,
                              bfsx_graph **out);
/* GraphFileUtil.convert (GraphFileUtil.java:45-69) for one rank of a partition: the rank tokenizes the whole
 * algs4 file on its own GPU and keeps the rows of the ids it owns (same errors as bfsx_graph_load_algs4). */
int bfsx_dist_graph_load_algs4(bfsx_ctx *ctx, const char *path, int rank, int nranks, bfsx_graph **out);
int bfsx_graph_partition(const bfsx_graph *g, int64_t *nv_global, int64_t *v_lo, int64_t *nv_local,
                         int64_t *chunk, int32_t *rank, int32_t *nranks);
/* Degree of global id v if this rank owns it (else -1). */
int bfsx_graph_degree(const bfsx_graph *g, int64_t v, int64_t *deg);

/* ---- multi-GPU, native exchange: the whole partitioned level loop inside the library ------------
 * (For N ranks inside ONE process, bfsx_init_group does all of the below for the caller.)
 * One rank per GPU.  The exchange runs over RCCL (xGMI) on the BFS stream: top-down levels route
 * (vertex, parent) pairs to their owners (all-to-all of counts + grouped send/recv), bottom-up levels
 * all-gather the frontier bitmap slices, every level all-reduces (n_f, m_f, m_u).
 * bfsx_comm_unique_id: rank 0 creates the RCCL id; the caller distributes the bytes (any channel).
 * bfsx_comm_init: collective over the nranks processes; attaches the communicator to ctx.
 * bfsx_comm_local_group: the same exchange for nranks contexts inside ONE process (one host thread
 * per rank; ranks may share a device) -- the partitioned path testable on a single GPU.
 * bfsx_dist_bfs: collective; every rank passes the same source.  Results: bfsx_result (local rows).
 * stats, if requested, must be requested by every rank (m_comp/reached are all-reduced).
 * Failure: every collective call (bfsx_dist_bfs, bfsx_sample_roots and bfsx_validate on a partition) that fails on
 * one rank aborts the communicator, so it fails on every rank (BFSX_E_RCCL naming the failed rank and its level)
 * instead of leaving the others inside a collective; an aborted communicator fails every later call. */
#define BFSX_COMM_ID_BYTES 128
int bfsx_comm_unique_id(uint8_t *id);
int bfsx_comm_init(bfsx_ctx *ctx, int rank, int nranks, const uint8_t *id);
int bfsx_comm_local_group(bfsx_ctx **ctxs, int nranks);
int bfsx_dist_bfs(bfsx_graph *g, int64_t source, bfsx_stats *stats);
/* Device time of the collectives of the most recent bfsx_dist_bfs on this rank, by kind, with option
 * "comm_timing" on (default off: all zero): ms[0] the level-close all-reduces, ms[1] the pair-count
 * all-to-alls, ms[2] the pair / frontier-id all-to-allvs, ms[3] the frontier all-gathers; count[k] the calls.
 * A collective's span runs from the BFS stream reaching it to its completion, so it includes the wait for the
 * slowest rank.  A group graph reports the largest span over its ranks per kind. */
int bfsx_comm_times(const bfsx_graph *g, double *ms, int64_t *count);

/* ---- device synchronisation helper for benchmarking harnesses ------------------------------- */
int bfsx_device_synchronize(bfsx_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
