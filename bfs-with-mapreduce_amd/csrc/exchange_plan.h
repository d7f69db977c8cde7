// exchange_plan.h -- host arithmetic of the partitioned BFS's pair exchange (multi-GPU).
//
// A top-down level of the 1-D partitioned loop routes (vertex << 32 | parent) pairs to the owner of
// the vertex: the replacement of Spark's hash-partitioned reduceByKey shuffle (BfsSpark.java:90).
// This header holds the pure integer part of that exchange -- who sends how many pairs from which
// offset to whom -- with no HIP or RCCL dependency, so the CPU test suite compiles and checks it
// (tests/cpp/test_exchange_plan.cpp) with the same count tables the in-process group runs on the GPU.
//
//   plan_counted   counts known (all-to-all of the per-destination counts): send/receive blocks packed
//                  in rank order (the device bucketing scatters pairs to destination-ordered blocks)
//   plan_slots     small levels: every peer gets a fixed slot [count, slot pairs] whatever it holds
//   plan_broadcast a sparse frontier exchange: every rank sends its whole id list to every rank (itself
//                  included) and receives every rank's list, packed in rank order
//   alltoallv_ops  the point-to-point operations one rank issues for an all-to-allv (RcclComm: one
//                  ncclSend/ncclRecv pair per peer inside a group, empty blocks skipped)
#pragma once

#include <cstdint>
#include <vector>

namespace bfsx {

struct ExchangePlan {
    std::vector<int64_t> scount, sdispl, rcount, rdispl;
    int64_t send_total = 0, recv_total = 0;
};

// send_counts[p]: pairs this rank routes to rank p; recv_counts[p]: pairs rank p routes to this rank.
template <class U>
inline void plan_counted(int P, const U *send_counts, const U *recv_counts, ExchangePlan &pl) {
    pl.scount.assign(P, 0);
    pl.sdispl.assign(P, 0);
    pl.rcount.assign(P, 0);
    pl.rdispl.assign(P, 0);
    int64_t so = 0, ro = 0;
    for (int p = 0; p < P; p++) {
        pl.scount[p] = (int64_t)send_counts[p];
        pl.rcount[p] = (int64_t)recv_counts[p];
        pl.sdispl[p] = so;
        pl.rdispl[p] = ro;
        so += pl.scount[p];
        ro += pl.rcount[p];
    }
    pl.send_total = so;
    pl.recv_total = ro;
}

// Fixed slots of (slot + 1) words per peer: word 0 = the pair count, then up to `slot` pairs.  The
// receiver's claim kernel reads P * slot candidate entries (entry i -> peer i / slot, pair i % slot).
// self: this rank.  Its own slot is never exchanged -- the push kernels claim their own vertices directly, so
// it is always empty -- and the claim kernel skips it (at P = 1 the level exchanges nothing).  The buffers
// keep the slot's space, so every peer's slot sits at the same offset on both sides.
inline void plan_slots(int P, int64_t slot, ExchangePlan &pl, int self = -1) {
    pl.scount.assign(P, slot + 1);
    pl.rcount.assign(P, slot + 1);
    pl.sdispl.assign(P, 0);
    pl.rdispl.assign(P, 0);
    for (int p = 0; p < P; p++) pl.sdispl[p] = pl.rdispl[p] = (int64_t)p * (slot + 1);
    if (self >= 0 && self < P) pl.scount[self] = pl.rcount[self] = 0;
    pl.send_total = pl.recv_total = (int64_t)P * (slot + 1);
}

// Sparse frontier exchange (a pull level whose global frontier is small): this rank's `mine` ids go to every
// rank from offset 0; counts[p] = rank p's ids (the level close's all-reduced per-rank counts), received in rank
// order -- the receive buffer then holds the whole global frontier as an id list.
template <class U>
inline void plan_broadcast(int P, int64_t mine, const U *counts, ExchangePlan &pl) {
    pl.scount.assign(P, mine);
    pl.sdispl.assign(P, 0);
    pl.rcount.assign(P, 0);
    pl.rdispl.assign(P, 0);
    int64_t ro = 0;
    for (int p = 0; p < P; p++) {
        pl.rcount[p] = (int64_t)counts[p];
        pl.rdispl[p] = ro;
        ro += pl.rcount[p];
    }
    pl.send_total = mine;
    pl.recv_total = ro;
}

// Word offset of candidate entry i of a received slot exchange, or -1 when entry i is past its peer's count
// or in the receiver's own (unexchanged) slot.
template <class U>
inline int64_t slot_entry(const U *recv, int64_t i, int64_t slot, int self = -1) {
    const int64_t p = i / slot, k = i - p * slot;
    const int64_t base = p * (slot + 1);
    if (p == self) return -1;
    return k < (int64_t)recv[base] ? base + 1 + k : -1;
}

struct P2pOp {
    int peer;
    bool send;
    int64_t offset, count; // in 8-byte words of the send / receive buffer
};

// The operations one rank issues for an all-to-allv, in issue order (per peer: send, then receive).
inline void alltoallv_ops(int P, const int64_t *scount, const int64_t *sdispl, const int64_t *rcount,
                          const int64_t *rdispl, std::vector<P2pOp> &ops) {
    ops.clear();
    for (int p = 0; p < P; p++) {
        if (scount[p] > 0) ops.push_back({p, true, sdispl[p], scount[p]});
        if (rcount[p] > 0) ops.push_back({p, false, rdispl[p], rcount[p]});
    }
}

} // namespace bfsx
