"""Test infrastructure: a Python restatement of the partitioned level loop over libbfsx's level
primitives (bfsx_dist_begin / td_expand / td_claim / frontier_slice / bu_step / level_end / finish),
with the exchange over torch.distributed.  The product loop is the native bfsx_dist_bfs
(csrc/kernels_dist.hip dist_bfs_run over csrc/bfsx_comm.cpp); this driver is the protocol reference the
CPU (gloo, numpy engine) and GPU tests compare it with, and shows how a caller with its own exchange
drives the primitives.  1-D vertex partition, one process per GPU.

Replaces the reference's only collective -- Spark's hash-partitioned reduceByKey shuffle of whole
Vertex objects, every level (BfsSpark.java:90) -- with an owner-routed exchange:

  top-down level   local expand + claim of owned targets (libbfsx k_td<dist>), (v, parent) pairs for
                   other ranks bucketed by owner -> all-to-all of counts -> all-to-all of pairs ->
                   owners claim them (k_claim_remote)
  bottom-up level  each rank's frontier bitmap slice (chunk/64 words) -> all-gather into the global
                   frontier bitmap -> local pull over the owned unvisited vertices (k_bu)
  every level      all-reduce of {n_f, m_f}: termination (BfsSpark.java:117) and Beamer's direction
                   switch, identical on every rank

The compute engine is libbfsx.so on the rank's GPU (GpuEngine); collectives are torch.distributed --
backend "nccl" (= RCCL over xGMI) on device tensors, or "gloo" with host staging (CPU tests and the
one-GPU rehearsal).  tests/dist_cpu_engine.py provides a numpy engine with the same primitive
semantics so the driver and its exchange protocol are exercised by world_size-2 gloo tests on CPU.
"""
import numpy as np


class Comm:
    """Collectives used by the level loop.  `device` = torch device of the exchange buffers;
    staging=True copies device tensors through host memory (gloo)."""

    def __init__(self, torch, dist, device, staging):
        self.torch, self.dist, self.device, self.staging = torch, dist, device, staging
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()

    def _sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    def allreduce_i64(self, vals, op="sum"):
        t = self.torch.tensor(list(vals), dtype=self.torch.int64)
        if not self.staging:
            t = t.to(self.device)
        rop = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX
        self.dist.all_reduce(t, op=rop)
        return [int(x) for x in t.cpu().tolist()]

    def alltoall_counts(self, counts):
        send = self.torch.tensor(counts, dtype=self.torch.int64)
        recv = self.torch.empty(self.world, dtype=self.torch.int64)
        if not self.staging:
            send, recv = send.to(self.device), recv.to(self.device)
        self.dist.all_to_all_single(recv, send)
        return recv.cpu().numpy()

    def alltoall_pairs(self, send, send_counts, recv, recv_counts):
        """send/recv: int64 tensors on self.device holding (v << 32 | parent) pairs."""
        ss, rs = [int(x) for x in send_counts], [int(x) for x in recv_counts]
        if self.staging and self.device.type == "cuda":
            hs, hr = send[: sum(ss)].cpu(), self.torch.empty(sum(rs), dtype=self.torch.int64)
            self.dist.all_to_all_single(hr, hs, rs, ss)
            recv[: sum(rs)].copy_(hr)
            self._sync()
        else:
            self._sync()
            self.dist.all_to_all_single(recv[: sum(rs)], send[: sum(ss)], rs, ss)
            self._sync()

    def allgather(self, out, inp):
        """out: [world * k] int64, inp: [k] int64 (frontier bitmap words)."""
        if self.staging and self.device.type == "cuda":
            ho = self.torch.empty(out.numel(), dtype=self.torch.int64)
            self.dist.all_gather_into_tensor(ho, inp.cpu())
            out.copy_(ho)
            self._sync()
        else:
            self._sync()
            self.dist.all_gather_into_tensor(out, inp)
            self._sync()

    def barrier(self):
        self.dist.barrier()


class GpuEngine:
    """One rank's partition in libbfsx.so; exchange buffers are torch tensors on the rank's GPU."""

    def __init__(self, torch, graph, device):
        self.torch, self.g, self.device = torch, graph, device
        p = graph.partition()
        self.nranks, self.chunk, self.v_lo, self.nv_local = p["nranks"], p["chunk"], p["v_lo"], p["nv_local"]
        self.nv_global = p["nv_global"]
        self.slice_words = self.chunk // 64
        i64 = torch.int64
        self.slice = torch.zeros(self.slice_words, dtype=i64, device=device)
        self.front_global = torch.zeros(self.slice_words * self.nranks, dtype=i64, device=device)
        self.send = torch.empty(1, dtype=i64, device=device)
        self.recv = torch.empty(1, dtype=i64, device=device)

    def _grow(self, name, n):
        t = getattr(self, name)
        if t.numel() < n:
            t = self.torch.empty(max(n, 2 * t.numel()), dtype=self.torch.int64, device=self.device)
            setattr(self, name, t)
        return t

    def begin(self, source):
        return self.g.dist_begin(source)

    def td_expand(self):
        _, mf = self.g.dist_frontier_info()
        send = self._grow("send", max(mf, 1))
        return self.g.dist_td_expand(send.data_ptr(), send.numel(), self.nranks)

    def recv_buffer(self, n):
        return self._grow("recv", max(n, 1))

    def td_claim(self, n):
        self.g.dist_td_claim(self.recv.data_ptr(), n)

    def frontier_slice(self):
        self.g.dist_frontier_slice(self.slice.data_ptr())
        return self.slice

    def bu_step(self):
        self.g.dist_bu_step(self.front_global.data_ptr())

    def level_end(self):
        return self.g.dist_level_end()

    def finish(self):
        self.g.dist_finish()

    def mcomp(self):
        return self.g.dist_mcomp()

    def degree(self, v):
        return self.g.degree(v)

    def nnz_local(self):
        return self.g.nnz

    def result(self):
        return self.g.result()


class DistBFS:
    """Level-synchronous partitioned BFS; every rank runs the same loop in lockstep."""

    def __init__(self, engine, comm, direction="auto", alpha=20, beta=24):
        self.e, self.c = engine, comm
        self.direction, self.alpha, self.beta = direction, alpha, beta
        self.nnz_global = comm.allreduce_i64([engine.nnz_local()])[0]
        self.nv_global = engine.nv_global
        self.level_log = []

    def sample_roots(self, count, seed):
        """Graph500 roots: distinct vertices with degree >= 1 (same sequence on every rank)."""
        def mix64(z):
            m = (1 << 64) - 1
            z = (z + 0x9E3779B97F4A7C15) & m
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
            return z ^ (z >> 31)
        roots, t = [], 0
        while len(roots) < count and t < 1000 + 1000 * count:
            x = mix64(seed + t) % self.nv_global
            t += 1
            if x in roots:
                continue
            if self.c.allreduce_i64([max(self.e.degree(x), 0)], op="max")[0] > 0:
                roots.append(x)
        return roots

    def run(self, source):
        e, c = self.e, self.c
        deg = c.allreduce_i64([e.begin(source)])[0]
        nf, mf, prev_nf = 1, deg, 0
        mu = self.nnz_global - deg
        direction = "bu" if self.direction == "bottomup" else "td"
        self.level_log = []
        levels = 0
        while True:
            if self.direction == "auto" and levels > 0:
                # Beamer's rule plus the exchange cost, as the native loop (kernels_dist.hip
                # dist_bfs_run): pull once a top-down level's pairs would outweigh the bitmap all-gather
                world = self.c.world
                pairs_heavy = world > 1 and mf * 64 * (world - 1) > self.nv_global * world
                if direction == "td" and (mf > mu // self.alpha or pairs_heavy):
                    direction = "bu"
                elif (direction == "bu" and nf < self.nv_global // self.beta and nf < prev_nf
                      and not pairs_heavy):
                    direction = "td"
            if direction == "td":
                counts = e.td_expand()
                rcounts = c.alltoall_counts(counts)
                recv = e.recv_buffer(int(rcounts.sum()))
                c.alltoall_pairs(e.send, counts, recv, rcounts)
                e.td_claim(int(rcounts.sum()))
                sent = int(counts.sum())
            else:
                sl = e.frontier_slice()
                c.allgather(e.front_global, sl)
                e.bu_step()
                sent = 0
            nf_l, mf_l = e.level_end()
            nf_new, mf_new, sent_g = c.allreduce_i64([nf_l, mf_l, sent])
            self.level_log.append(dict(level=levels, direction=direction, frontier_in=nf, frontier_out=nf_new,
                                       mf_in=mf, pairs_exchanged=sent_g))
            levels += 1
            mu -= mf_new
            prev_nf, nf, mf = nf, nf_new, mf_new
            if nf == 0:
                break
        e.finish()
        return levels

    def mcomp(self):
        m, r = self.e.mcomp()
        return self.c.allreduce_i64([m, r])
