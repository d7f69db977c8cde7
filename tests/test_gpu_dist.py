"""Partitioned (multi-GPU) path through libbfsx.so on the GPU.

The GPU box has one MI355X, so the P=2/3 cases run two or three ranks on the same device with a gloo
process group and host-staged exchange buffers: the kernels' partitioned code paths (owner routing,
remote pair bucketing, remote claims, bottom-up against an all-gathered global frontier) are the
ones under test.  P=1 runs the RCCL ("nccl") backend on device tensors.  Distances must be
bit-exact against the oracle; parents are validated."""
import importlib.util
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN, PKG, ROOT

pytestmark = pytest.mark.gpu
INF = 2147483647


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _load(name, file, where=PKG):
    spec = importlib.util.spec_from_file_location(name, os.path.join(where, file))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def _load_test(name, file):
    return _load(name, file, os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, backend, graph, sources, direction, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    bfsx = _load("bfsx", "bfsx.py")
    bd = _load_test("dist_driver", "dist_driver.py")
    dist.init_process_group(backend, rank=rank, world_size=world)
    ctx = bfsx.Context(0)
    try:
        if graph[0] == "edges":
            _, nv, u, v = graph
            g = ctx.dist_from_edges(nv, u, v, rank, world)
        else:
            _, scale, seed = graph
            g = ctx.dist_kronecker(scale, rank, world, seed=seed)
        dev = torch.device("cuda", 0)
        eng = bd.GpuEngine(torch, g, dev)
        comm = bd.Comm(torch, dist, dev, staging=(backend == "gloo"))
        drv = bd.DistBFS(eng, comm, direction=direction)
        out = []
        for s in sources:
            levels = drv.run(s)
            m, r = drv.mcomp()
            d, p = g.result()
            parts = [None] * world
            dist.all_gather_object(parts, (eng.v_lo, d, p))
            out.append((levels, m, r, parts, [x["direction"] for x in drv.level_log]))
        if rank == 0:
            q.put(("ok", out))
        g.free()
    except Exception as e:
        q.put(("err", repr(e)))
        raise
    finally:
        ctx.close()
        dist.destroy_process_group()


def run_dist(world, backend, graph, sources, direction="auto"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, graph, sources, direction, q))
             for r in range(world)]
    for p in procs:
        p.start()
    status, out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", out
    return out


def check(nv, u, v, sources, out, oracle="mapreduce"):
    off, col = O.build_sets(nv, u, v)
    for s, (levels, m, r, parts, dirs) in zip(sources, out):
        dist = np.full(nv, INF, np.int64)
        parent = np.full(nv, -1, np.int64)
        for lo, d, p in parts:
            dist[lo:lo + len(d)] = d
            parent[lo:lo + len(p)] = p
        ref, _ = O.csr_bfs(nv, off, col, s)
        assert np.array_equal(dist.astype(np.int32), ref)
        assert levels == int(ref[ref != INF].max()) + 1
        assert O.validate(nv, off, col, s, dist.astype(np.int32), parent) == 0
        assert m == O.mcomp(u, v, ref) and r == int((ref != INF).sum())


@pytest.mark.parametrize("world,direction", [(2, "auto"), (2, "topdown"), (2, "bottomup"), (3, "auto")])
def test_gpu_dist_random(world, direction):
    rng = np.random.default_rng(world)
    nv = 5000
    u = rng.integers(0, nv, 4 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 4 * nv).astype(np.uint32)
    sources = [0, 2500, 4999]
    out = run_dist(world, "gloo", ("edges", nv, u, v), sources, direction)
    check(nv, u, v, sources, out)


def test_gpu_dist_kronecker_scale16():
    scale, seed = 16, 0xD157
    u, v = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    sources = [int(u[0]), int(u[123])]
    out = run_dist(2, "gloo", ("kron", scale, seed), sources, "auto")
    check(nv, u, v, sources, out)
    assert any("bu" in o[4] for o in out)


def test_gpu_dist_reference_file_and_rccl_single_rank():
    nv, u, v = O.load_graphfileutil(os.path.join(GOLDEN, "mediumG.txt"))
    out = run_dist(1, "nccl", ("edges", nv, u, v), [0, 100], "auto")
    check(nv, u, v, [0, 100], out)
    out = run_dist(2, "gloo", ("edges", nv, u, v), [0], "auto")  # chunk 128: both ranks own rows
    check(nv, u, v, [0], out)
