// CPU check of the partitioned BFS's exchange arithmetic (bfs-with-mapreduce_amd/csrc/exchange_plan.h):
// P simulated ranks bucket random (vertex << 32 | parent) pairs by owner exactly as k_bucket_count /
// k_bucket_scatter lay them out, plan the all-to-allv, and run it through a simulated point-to-point
// transport that matches ncclSend/ncclRecv per (sender, receiver) pair -- the semantics RcclComm relies
// on.  The result must equal what LocalGroupComm::alltoallv delivers (a copy of rcount[p] words from
// peer p's send buffer at p's sdispl[me], landing at rdispl[p]) and hold exactly the pairs owned by the
// receiver, grouped by sender in rank order.  The fixed-slot plan is checked the same way, including the
// claim kernel's entry mapping.  Exit code 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <random>
#include <vector>

#include "../../bfs-with-mapreduce_amd/csrc/exchange_plan.h"

using namespace bfsx;
using u64 = unsigned long long;

#define CHECK(c)                                                                                   \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c);                   \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

struct Rank {
    std::vector<u64> remote;       // unbucketed pairs (kernel output order)
    std::vector<u64> send, recv;   // bucketed send buffer / receive buffer
    std::vector<u64> counts;       // per destination
    ExchangePlan plan;
};

// Simulated transport: every rank's ops; a recv from p is matched with p's send to this rank.
static void run_p2p(int P, std::vector<Rank> &R) {
    std::vector<std::vector<P2pOp>> ops(P);
    for (int r = 0; r < P; r++)
        alltoallv_ops(P, R[r].plan.scount.data(), R[r].plan.sdispl.data(), R[r].plan.rcount.data(),
                      R[r].plan.rdispl.data(), ops[r]);
    for (int q = 0; q < P; q++) {
        for (const P2pOp &o : ops[q]) {
            if (o.send) continue;
            const P2pOp *match = nullptr;
            int nmatch = 0;
            for (const P2pOp &s : ops[o.peer])
                if (s.send && s.peer == q) {
                    match = &s;
                    nmatch++;
                }
            CHECK(nmatch == 1);
            CHECK(match->count == o.count);
            for (int64_t i = 0; i < o.count; i++) R[q].recv[o.offset + i] = R[o.peer].send[match->offset + i];
        }
        // a peer that sends to q must be received from
        for (int p = 0; p < P; p++)
            for (const P2pOp &s : ops[p])
                if (s.send && s.peer == q) {
                    bool got = false;
                    for (const P2pOp &o : ops[q]) got |= !o.send && o.peer == p;
                    CHECK(got);
                }
    }
}

// LocalGroupComm's pull semantics on the same plans.
static std::vector<std::vector<u64>> local_group(int P, const std::vector<Rank> &R) {
    std::vector<std::vector<u64>> out(P);
    for (int q = 0; q < P; q++) {
        out[q].assign(R[q].recv.size(), ~0ull); // words no block lands on stay as the receive buffer had them
        for (int p = 0; p < P; p++)
            for (int64_t i = 0; i < R[q].plan.rcount[p]; i++)
                out[q][R[q].plan.rdispl[p] + i] = R[p].send[R[p].plan.sdispl[q] + i];
    }
    return out;
}

static void counted_case(int P, uint32_t chunk, int npairs_max, std::mt19937_64 &rng) {
    std::vector<Rank> R(P);
    const uint32_t nglob = chunk * (uint32_t)P;
    for (int r = 0; r < P; r++) {
        const int n = (int)(rng() % (uint64_t)(npairs_max + 1));
        for (int i = 0; i < n; i++) {
            uint32_t v = (uint32_t)(rng() % nglob);
            if (v / chunk == (uint32_t)r) v = (v + chunk) % nglob; // remote pairs only
            if (P == 1) continue;
            R[r].remote.push_back(((u64)v << 32) | (u64)(rng() % nglob));
        }
        // k_bucket_count + k_bucket_scatter: destination blocks in rank order (order inside a block is
        // the kernels' choice; the receiver only needs the set)
        R[r].counts.assign(P, 0);
        for (u64 pr : R[r].remote) R[r].counts[(uint32_t)(pr >> 32) / chunk]++;
        std::vector<u64> cur(P, 0), base(P, 0);
        for (int p = 1; p < P; p++) base[p] = base[p - 1] + R[r].counts[p - 1];
        R[r].send.assign(R[r].remote.size(), 0);
        for (u64 pr : R[r].remote) {
            const uint32_t d = (uint32_t)(pr >> 32) / chunk;
            R[r].send[base[d] + cur[d]++] = pr;
        }
    }
    // all-to-all of the counts (alltoall1), then the plans
    for (int q = 0; q < P; q++) {
        std::vector<u64> rc(P);
        for (int p = 0; p < P; p++) rc[p] = R[p].counts[q];
        plan_counted(P, R[q].counts.data(), rc.data(), R[q].plan);
        CHECK(R[q].plan.send_total == (int64_t)R[q].send.size());
        R[q].recv.assign((size_t)R[q].plan.recv_total, ~0ull);
    }
    for (int q = 0; q < P; q++)
        for (int p = 0; p < P; p++) CHECK(R[p].plan.scount[q] == R[q].plan.rcount[p]);
    run_p2p(P, R);
    const auto lg = local_group(P, R);
    for (int q = 0; q < P; q++) {
        CHECK(lg[q] == R[q].recv);
        // exactly the pairs owned by q, from sender p inside block p
        std::multimap<u64, int> want;
        for (int p = 0; p < P; p++)
            for (u64 pr : R[p].remote)
                if ((uint32_t)(pr >> 32) / chunk == (uint32_t)q) want.insert({pr, p});
        CHECK(want.size() == R[q].recv.size());
        for (int p = 0; p < P; p++)
            for (int64_t i = 0; i < R[q].plan.rcount[p]; i++) {
                const u64 pr = R[q].recv[R[q].plan.rdispl[p] + i];
                CHECK((uint32_t)(pr >> 32) / chunk == (uint32_t)q);
                auto it = want.find(pr);
                bool found = false;
                for (; it != want.end() && it->first == pr; ++it)
                    if (it->second == p) {
                        want.erase(it);
                        found = true;
                        break;
                    }
                CHECK(found);
            }
        CHECK(want.empty());
    }
}

static void slot_case(int P, uint32_t chunk, int64_t slot, std::mt19937_64 &rng) {
    std::vector<Rank> R(P);
    const uint32_t nglob = chunk * (uint32_t)P;
    for (int r = 0; r < P; r++) {
        // a small level: this rank routes at most `slot` pairs in total (the global m_f bound)
        const int n = (int)(rng() % (uint64_t)(slot + 1));
        for (int i = 0; i < n; i++) {
            uint32_t v = (uint32_t)(rng() % nglob);
            if (v / chunk == (uint32_t)r) v = (v + chunk) % nglob;
            if (P == 1) continue;
            R[r].remote.push_back(((u64)v << 32) | (u64)i);
        }
        plan_slots(P, slot, R[r].plan, r);
        CHECK(R[r].plan.scount[r] == 0 && R[r].plan.rcount[r] == 0); // the own slot is not exchanged
        // k_bucket_slots + k_slot_headers
        R[r].send.assign((size_t)R[r].plan.send_total, 0);
        std::vector<u64> cur(P, 0);
        for (u64 pr : R[r].remote) {
            const uint32_t d = (uint32_t)(pr >> 32) / chunk;
            R[r].send[(size_t)d * (slot + 1) + 1 + cur[d]++] = pr;
        }
        for (int p = 0; p < P; p++) R[r].send[(size_t)p * (slot + 1)] = cur[p];
        R[r].recv.assign((size_t)R[r].plan.recv_total, ~0ull);
    }
    run_p2p(P, R);
    const auto lg = local_group(P, R);
    for (int q = 0; q < P; q++) {
        CHECK(lg[q] == R[q].recv);
        // k_claim_remote's entry mapping over P * slot candidates
        std::multiset<u64> got, want;
        for (int64_t i = 0; i < (int64_t)P * slot; i++) {
            const int64_t at = slot_entry(R[q].recv.data(), i, slot, q);
            if (at >= 0) got.insert(R[q].recv[at]);
        }
        for (int p = 0; p < P; p++)
            for (u64 pr : R[p].remote)
                if ((uint32_t)(pr >> 32) / chunk == (uint32_t)q) want.insert(pr);
        CHECK(got == want);
    }
}

// The sparse frontier exchange: every rank's id list reaches every rank, in rank order.
static void broadcast_case(int P, std::mt19937_64 &rng) {
    std::vector<Rank> R(P);
    std::vector<u64> counts(P);
    for (int r = 0; r < P; r++) {
        counts[r] = rng() % 50;
        for (u64 i = 0; i < counts[r]; i++) R[r].send.push_back(((u64)r << 40) | i);
    }
    for (int r = 0; r < P; r++) {
        plan_broadcast(P, (int64_t)counts[r], counts.data(), R[r].plan);
        CHECK(R[r].plan.send_total == (int64_t)counts[r]);
        R[r].recv.assign((size_t)R[r].plan.recv_total, ~0ull);
    }
    run_p2p(P, R);
    const auto lg = local_group(P, R);
    for (int q = 0; q < P; q++) {
        CHECK(lg[q] == R[q].recv);
        std::vector<u64> want;
        for (int p = 0; p < P; p++) want.insert(want.end(), R[p].send.begin(), R[p].send.end());
        CHECK(R[q].recv == want);
    }
}

int main() {
    std::mt19937_64 rng(0x5EED);
    for (int P : {1, 2, 3, 4, 8}) {
        for (int t = 0; t < 20; t++) {
            counted_case(P, 64 * (1 + (uint32_t)(rng() % 8)), 500, rng);
            slot_case(P, 64 * (1 + (uint32_t)(rng() % 8)), 1 + (int64_t)(rng() % 40), rng);
            broadcast_case(P, rng);
        }
        counted_case(P, 64, 0, rng); // every rank sends nothing
    }
    std::printf("exchange plan ok\n");
    return 0;
}
