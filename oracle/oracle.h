/*
 * oracle.h -- CPU restatement of the reference BFS path.  TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the MI355X BFS engine.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (libbfsx.so) never links or calls it.
 *
 * What it restates (reference = NorthernDemon/BFS-with-MapReduce, Java; it cannot be
 * built here -- no JDK, no Spark jars -- so nothing is compiled from it):
 *   - orc_load_graphfileutil : GraphFileUtil.convert            GraphFileUtil.java:45-69
 *   - orc_build_sets         : Vertex.neighbours HashSet semantics Vertex.java:30,74-76
 *   - orc_mapreduce_bfs      : BfsSpark mapper/reducer loop      BfsSpark.java:57-118
 *   - orc_load_algs4_graph   : algs4 Graph(In)                   algs4.jar!/Graph.java:85-94
 *   - orc_algs4_bfs          : algs4 BreadthFirstPaths.bfs       algs4.jar!/BreadthFirstPaths.java:93-111
 *   - orc_validate           : BreadthFirstPaths.check + Graph500 validation rules
 *                                                                algs4.jar!/BreadthFirstPaths.java:171-212
 *   - orc_kronecker          : Graph500 Kronecker generator (same integer recipe as the GPU one)
 *
 * Pinning: tests/test_oracle.py checks these functions against the golden vectors the
 * reference itself holds -- PDF p.5 Tables 3-6 (tinyCG per-iteration states),
 * BreadthFirstPaths.java:19-25 (tinyCG distances/paths), Graph.java:10-31 (tinyG and
 * mediumG adjacency in Bag order), CC.java:10-18 (components), Cycle.java:10-12
 * (mediumG cycle) -- and the mediumG distance vector of SURVEY.md Appendix A.
 */
#ifndef BFSX_ORACLE_H
#define BFSX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes: same numbering as include/bfsx.h */
#define ORC_OK 0
#define ORC_E_IO (-1)
#define ORC_E_PARSE (-2)
#define ORC_E_RANGE (-3)
#define ORC_E_OOM (-6)
#define ORC_E_ARG (-7)

/* colours, ordinals as Color.java:10-31 (DO NOT RE-ORDER) */
#define ORC_WHITE 0
#define ORC_GRAY 1
#define ORC_BLACK 2

/* GraphFileUtil.convert parse: returns tuples (u[i], v[i]) in file order. */
int orc_load_graphfileutil(const char *path, int64_t *nv, int64_t *m, uint32_t **u, uint32_t **v);
/* algs4 Graph(In) parse: whitespace tokens, exactly E pairs. */
int orc_load_algs4_graph(const char *path, int64_t *nv, int64_t *m, uint32_t **u, uint32_t **v);
void orc_free(void *p);

/* Neighbour sets: CSR with each row sorted ascending and unique; self-loops kept once. */
int orc_build_sets(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t **row_off,
                   uint32_t **col);

/* Level-synchronous restatement of the Spark map/reduceByKey loop.
 * dist: INT32_MAX for WHITE (GraphFileUtil.java:55).  parent: -1 for unreached, source for source.
 * color: final colour.  iter_gray[k] / iter_emits[k]: number of GRAY vertices after iteration k+1 and
 * mapper tuples emitted in iteration k+1 (may be NULL).  *iters = number of map/reduce passes.
 * nthreads <= 0: OpenMP default. */
int orc_mapreduce_bfs(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source,
                      int32_t *dist, int64_t *parent, int8_t *color, int64_t *iter_gray,
                      int64_t *iter_emits, int64_t max_iters, int64_t *iters, int nthreads);

/* Serial queue BFS over algs4 Bag adjacency (LIFO insertion order). edgeTo: -1 for unreached. */
int orc_algs4_bfs(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t source,
                  int32_t *dist, int64_t *edge_to);
/* The Bag adjacency list of vertex x, in iteration order (LIFO).  Returns count written. */
int64_t orc_algs4_adj(int64_t nv, int64_t m, const uint32_t *u, const uint32_t *v, int64_t x,
                      uint32_t *out, int64_t cap);

/* Serial queue BFS directly on a CSR (the scalar CPU baseline). */
int orc_csr_bfs(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source, int32_t *dist,
                int64_t *parent);

/* Graph500-style validation of (dist, parent) on the CSR.
 * Returns 0 if valid, else a negative rule number:
 *  -1 source wrong (dist!=0 or parent!=source)
 *  -2 parent of a reached vertex is not reached, or dist[v] != dist[parent]+1
 *  -3 (parent[v], v) is not an edge of the graph
 *  -4 an edge (a,b) with |dist[a]-dist[b]| > 1 or exactly one endpoint reached
 *  -5 unreached vertex has a parent, or a reached vertex has none */
int orc_validate(int64_t nv, const int64_t *row_off, const uint32_t *col, int64_t source,
                 const int32_t *dist, const int64_t *parent);

/* Kronecker generator: identical integer recipe to the GPU generator. */
void orc_kronecker(int scale, int edgefactor, uint64_t seed, uint32_t *u, uint32_t *v);
/* thresholds (A,B,C) as uint32 fractions of 2^32 */
void orc_kronecker_thresholds(uint32_t *t_ab, uint32_t *t_a_norm, uint32_t *t_c_norm);

/* Number of input tuples whose endpoints are reached (Graph500 m for TEPS). */
int64_t orc_mcomp(int64_t m, const uint32_t *u, const uint32_t *v, const int32_t *dist);

/* sha256 over "v d\n" lines (SURVEY.md Appendix A convention). out: 65 chars incl. NUL */
void orc_dist_sha256(int64_t nv, const int32_t *dist, char *out_hex);

#ifdef __cplusplus
}
#endif
#endif
