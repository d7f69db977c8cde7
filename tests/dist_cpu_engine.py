"""numpy model of one rank's libbfsx partition, for CPU (gloo) tests of dist_driver.DistBFS.

TEST INFRASTRUCTURE ONLY.  It implements the same level primitives as the GPU engine
(dist_driver.GpuEngine -> libbfsx bfsx_dist_*), with the same data contracts:
  - partition: chunk = ceil(nv / P) rounded up to 64, rank r owns global ids [r*chunk, +chunk)
  - td_expand: claims owned targets, returns per-destination counts of (v << 32 | parent) pairs
    written to self.send grouped by owner in rank order
  - frontier_slice: chunk/64 int64 words, bit b of word w = local vertex 64w+b
so that the driver's exchange protocol (all-to-all of counts then pairs, all-gather of slices,
all-reduce of counts) is exercised by world_size-2 gloo tests without a GPU.
"""
import numpy as np

import oracle_py as O

INF = 2147483647


def pack_words(bits):
    b = bits.reshape(-1, 64).astype(np.uint64)
    w = np.bitwise_or.reduce(b << np.arange(64, dtype=np.uint64), axis=1)
    return w.view(np.int64)


def unpack_words(words):
    w = np.asarray(words).view(np.uint64)
    return ((w[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool).ravel()


class CpuEngine:
    def __init__(self, torch, nv, u, v, rank, nranks):
        self.torch = torch
        self.nranks, self.rank, self.nv_global = nranks, rank, nv
        self.chunk = ((nv + nranks - 1) // nranks + 63) // 64 * 64
        self.v_lo = min(rank * self.chunk, nv)
        self.nv_local = min(self.chunk, nv - self.v_lo)
        off, col = O.build_sets(nv, u, v)
        lo, n = self.v_lo, self.nv_local
        self.off = off[lo:lo + n + 1] - off[lo]
        self.col = col[off[lo]:off[lo + n]].astype(np.int64)
        self.tcnt = np.bincount(np.asarray(u, np.int64), minlength=nv)[lo:lo + n]
        self.slice_words = self.chunk // 64
        i64 = torch.int64
        self.slice = torch.zeros(self.slice_words, dtype=i64)
        self.front_global = torch.zeros(self.slice_words * nranks, dtype=i64)
        self.send = torch.zeros(1, dtype=i64)
        self.recv = torch.zeros(1, dtype=i64)

    # -- helpers --
    def deg(self, x):
        return int(self.off[x + 1] - self.off[x])

    def _claim(self, vl, parent_g):
        if self.vis[vl]:
            return False
        self.vis[vl] = True
        self.dist[vl] = self.level + 1
        self.parent[vl] = parent_g
        self.new.append(vl)
        return True

    def begin(self, source):
        n = self.nv_local
        self.dist = np.full(n, INF, np.int64)
        self.parent = np.full(n, -1, np.int64)
        self.vis = np.zeros(self.chunk, bool)
        self.vis[n:] = True  # padding
        self.level = 0
        self.queue, self.bitmap = [], None
        self.new = []
        if self.v_lo <= source < self.v_lo + n:
            sl = source - self.v_lo
            self.dist[sl], self.parent[sl], self.vis[sl] = 0, source, True
            self.queue = [sl]
            return self.deg(sl)
        return 0

    def _frontier_local(self):
        if self.queue is not None:
            return list(self.queue)
        return list(np.nonzero(self.bitmap[: self.nv_local])[0])

    def td_expand(self):
        q = self._frontier_local()
        self.queue, self.bitmap, self.new, self.dir = q, None, [], "td"
        remote = []
        for ul in q:
            ug = ul + self.v_lo
            for x in self.col[self.off[ul]:self.off[ul + 1]]:
                x = int(x)
                if x // self.chunk == self.rank:
                    self._claim(x - self.v_lo, ug)
                else:
                    remote.append((x // self.chunk, (x << 32) | ug))
        remote.sort(key=lambda t: t[0])  # grouped by destination, in rank order
        counts = np.zeros(self.nranks, np.int64)
        for d, _ in remote:
            counts[d] += 1
        if len(remote) > self.send.numel():
            self.send = self.torch.zeros(len(remote), dtype=self.torch.int64)
        if remote:
            self.send[: len(remote)] = self.torch.tensor([p for _, p in remote], dtype=self.torch.int64)
        return counts

    def recv_buffer(self, n):
        if n > self.recv.numel():
            self.recv = self.torch.zeros(n, dtype=self.torch.int64)
        return self.recv

    def td_claim(self, n):
        for pr in self.recv[:n].tolist():
            v, p = (pr >> 32) & 0xFFFFFFFF, pr & 0xFFFFFFFF
            assert v // self.chunk == self.rank, "pair routed to the wrong rank"
            self._claim(v - self.v_lo, p)

    def frontier_slice(self):
        bits = np.zeros(self.chunk, bool)
        for x in self._frontier_local():
            bits[x] = True
        self.slice.copy_(self.torch.from_numpy(pack_words(bits)))
        return self.slice

    def bu_step(self):
        front = unpack_words(self.front_global.numpy())
        self.new, self.dir = [], "bu"
        for vl in range(self.nv_local):
            if self.vis[vl]:
                continue
            for x in self.col[self.off[vl]:self.off[vl + 1]]:
                if front[int(x)]:
                    self.vis[vl] = True
                    self.dist[vl] = self.level + 1
                    self.parent[vl] = int(x)
                    self.new.append(vl)
                    break

    def level_end(self):
        nf = len(self.new)
        mf = sum(self.deg(x) for x in self.new)
        if self.dir == "td":
            self.queue, self.bitmap = list(self.new), None
        else:
            bm = np.zeros(self.chunk, bool)
            bm[self.new] = True
            self.queue, self.bitmap = None, bm
        self.level += 1
        return nf, mf

    def finish(self):
        pass

    def mcomp(self):
        reached = self.dist != INF
        return int(self.tcnt[reached].sum()), int(reached.sum())

    def degree(self, v):
        if self.v_lo <= v < self.v_lo + self.nv_local:
            return self.deg(v - self.v_lo)
        return -1

    def nnz_local(self):
        return int(self.off[-1])

    def result(self):
        return self.dist.astype(np.int32), self.parent
