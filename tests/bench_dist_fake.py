"""Test infrastructure (CPU): runs bench.py's distributed harness (run_dist: gloo rendezvous, barriers, the
max over ranks of every BFS's device time, one JSON line from rank 0) under torch.distributed.run with a
stand-in for the libbfsx binding, so the N > 1 bench contract is checked without a GPU.  Each fake rank
reports a different device time per BFS; the line's value must use the slowest rank's."""
import importlib.util
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_bfsx():
    m = types.ModuleType("bfsx")

    class BfsxError(Exception):
        pass

    class Graph:
        COMM_KINDS = ("allreduce", "count_alltoall", "alltoallv", "allgather")

        def __init__(self, scale, rank, world, ctx=None):
            self.ctx = ctx
            self.rank, self.world, self.nvg = rank, world, 1 << scale
            self.chunk = self.nvg // world
            self.nnz, self.m = 1000 + rank, 16 << scale

        def partition(self):
            return {"chunk": self.chunk, "nv_global": self.nvg, "v_lo": self.rank * self.chunk,
                    "nv_local": self.chunk}

        def sample_roots(self, n, seed):
            return list(range(1, n + 1))

        def dist_bfs(self, r, want_stats=True):
            if want_stats:  # all-reduced stats: identical on every rank; root 3 sits in a tiny component
                return {"m_comp": 5 if r == 3 else self.m // 2}
            if os.environ.get("BFSX_FAKE_HANG_RANK") == str(self.rank):  # a rank stuck in a collective
                import time
                time.sleep(3600)
            return 1.0 + 0.5 * self.rank + 0.01 * r  # device ms of this rank; rank world-1 is the slowest

        def comm_times(self):
            # per kind (ms, calls) of the last BFS: rank-dependent, so the line must carry the max over ranks;
            # zeros unless the bench turned comm_timing on
            on = self.ctx is not None and self.ctx.opts.get("comm_timing") == "on"
            return {k: ((0.1 * (i + 1) + 0.01 * self.rank) if on else 0.0, (3 + self.rank) if on else 0)
                    for i, k in enumerate(self.COMM_KINDS)}

        def validate(self, source=-1):
            return {"errors": 0}

        def level_stats(self, cap=256):
            return [{"level": 0, "direction": 1, "frontier_in": 1, "frontier_out": 10, "mf_in": 10,
                     "kernel_ms": 0.1, "unvisited_in": 0, "stage2": 0, "claims": 0, "walked": 0, "scanned": 10},
                    {"level": 1, "direction": 2, "frontier_in": 10, "frontier_out": 0, "mf_in": 0,
                     "kernel_ms": 0.2, "unvisited_in": 50, "stage2": 5, "claims": 1, "walked": 3, "scanned": 60}]

        def level_stats_raw(self, cap=256):
            return self.level_stats(cap)

        @staticmethod
        def level_stats_decode(raw):
            return raw

        def free(self):
            pass

    class Context:
        def __init__(self, device=0, **options):
            self.device = device
            self.opts = dict(options)

        def set_option(self, k, v):
            self.opts[k] = v

        def comm_init(self, rank, world, uid):
            assert len(uid) == 128

        def dist_kronecker(self, scale, rank, world, edgefactor=16, seed=0):
            return Graph(scale, rank, world, self)

        def synchronize(self):
            pass

        def close(self):
            pass

    m.BfsxError, m.Context = BfsxError, Context
    m.comm_unique_id = lambda: bytes(128)
    return m


# as a module (bench.py's BFSX_BENCH_BINDING hook): the stand-in binding itself
_fake = fake_bfsx()
Context, BfsxError, comm_unique_id = _fake.Context, _fake.BfsxError, _fake.comm_unique_id


def main():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    bench.load_module = lambda name, file: fake_bfsx()
    sys.argv = ["bench.py", "--gpus", os.environ["WORLD_SIZE"], "--scale", "12", "--roots", "4", "--steps", "2",
                "--warmup", "1"] + os.environ.get("BFSX_FAKE_EXTRA_ARGS", "").split()
    bench.main()


if __name__ == "__main__":
    main()
