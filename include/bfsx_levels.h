/*
 * bfsx_levels.h -- TEST-ONLY level primitives of the partitioned BFS (exported by libbfsx.so, NOT part
 * of the product C-ABI in bfsx.h).
 *
 * The product runs the whole partitioned level loop inside the library (bfsx_dist_bfs, bfsx.h).  These
 * primitives let the test suite's protocol driver (tests/dist_driver.py) step the SAME device kernels
 * one level at a time and perform the exchange itself (gloo on CPU, RCCL on the GPU), so the exchange
 * protocol is checked independently of bfsx_comm.cpp.  All buffer pointers are DEVICE pointers owned by
 * the caller.  Nothing in bfs-with-mapreduce_amd/ or bench.py calls them.
 */
#ifndef BFSX_LEVELS_H
#define BFSX_LEVELS_H

#include "bfsx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Start a BFS from global `source`; deg_local = its degree on the owning rank, 0 elsewhere. */
int bfsx_dist_begin(bfsx_graph *g, int64_t source, int64_t *deg_local);
/* Local frontier size and degree sum (for the caller's all-reduce and buffer sizing). */
int bfsx_dist_frontier_info(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local);
/* Top-down level, local part: expand the local frontier, claim owned targets, and write the
 * (v << 32 | parent) pairs for other ranks' targets into d_send, grouped by destination rank in
 * rank order; send_counts[P] receives the group sizes.  send_cap >= the local m_f is required. */
int bfsx_dist_td_expand(bfsx_graph *g, void *d_send, int64_t send_cap, int64_t *send_counts);
/* Claim the n pairs received from the all-to-all (all target this rank's vertices). */
int bfsx_dist_td_claim(bfsx_graph *g, const void *d_recv, int64_t n);
/* Write the local frontier as a bitmap slice of chunk/64 words (for the all-gather). */
int bfsx_dist_frontier_slice(bfsx_graph *g, void *d_slice);
/* Bottom-up level over the owned unvisited vertices against the all-gathered global frontier
 * bitmap (P * chunk/64 words). */
int bfsx_dist_bu_step(bfsx_graph *g, const void *d_front_global);
/* Close the level: local counts of the new frontier (the caller all-reduces them). */
int bfsx_dist_level_end(bfsx_graph *g, int64_t *nf_local, int64_t *mf_local);
/* After the last level: unreached owned vertices -> INT32_MAX.  Results: bfsx_result (local rows). */
int bfsx_dist_finish(bfsx_graph *g);
/* Local share of m_comp and of the reached count (the caller all-reduces them). */
int bfsx_dist_mcomp(bfsx_graph *g, int64_t *m_local, int64_t *reached_local);

#ifdef __cplusplus
}
#endif
#endif
