"""Python level-primitive driver (tests/dist_driver.py DistBFS) on CPU: world_size-2/3 gloo process groups, each rank a
numpy partition engine (tests/dist_cpu_engine.py).  Checks the 1-D partition + owner-routed
exchange protocol end to end: distances bit-exact against the oracle, parent trees valid, level
count = the reference's pass count, m_comp equal to the oracle's."""
import importlib.util
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN, PKG, ROOT

INF = 2147483647


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nv, u, v, sources, direction, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    from dist_cpu_engine import CpuEngine

    spec = importlib.util.spec_from_file_location("dist_driver", os.path.join(ROOT, "tests", "dist_driver.py"))
    bd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bd)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = CpuEngine(torch, nv, u, v, rank, world)
        comm = bd.Comm(torch, dist, torch.device("cpu"), staging=False)
        drv = bd.DistBFS(eng, comm, direction=direction, alpha=4, beta=8)
        out = []
        for s in sources:
            levels = drv.run(s)
            m, r = drv.mcomp()
            d, p = eng.result()
            parts = [None] * world
            dist.all_gather_object(parts, (eng.v_lo, d, p))
            out.append((levels, m, r, parts, [x["direction"] for x in drv.level_log]))
        roots = drv.sample_roots(4, seed=7)
        if rank == 0:
            q.put(("ok", out, roots))
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def run_dist(world, nv, u, v, sources, direction="auto"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nv, u, v, sources, direction, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, out, roots = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", out
    return out, roots


def check(nv, u, v, sources, out):
    off, col = O.build_sets(nv, u, v)
    for s, (levels, m, r, parts, dirs) in zip(sources, out):
        dist = np.full(nv, INF, np.int64)
        parent = np.full(nv, -1, np.int64)
        for lo, d, p in parts:
            dist[lo:lo + len(d)] = d
            parent[lo:lo + len(p)] = p
        ref = O.mapreduce_bfs(nv, off, col, s)
        assert np.array_equal(dist.astype(np.int32), ref["dist"])
        assert levels == ref["iters"]
        assert O.validate(nv, off, col, s, dist.astype(np.int32), parent) == 0
        assert m == O.mcomp(u, v, ref["dist"]) and r == int((ref["dist"] != INF).sum())
    return dirs


def random_graph(seed, nv, deg):
    rng = np.random.default_rng(seed)
    m = nv * deg
    return rng.integers(0, nv, m).astype(np.uint32), rng.integers(0, nv, m).astype(np.uint32)


@pytest.mark.parametrize("direction", ["auto", "topdown", "bottomup"])
def test_dist2_random(direction):
    nv = 700
    u, v = random_graph(1, nv, 3)
    sources = [0, 350, 699]
    out, roots = run_dist(2, nv, u, v, sources, direction)
    check(nv, u, v, sources, out)
    off, _ = O.build_sets(nv, u, v)
    assert len(set(roots)) == 4 and all(off[x + 1] > off[x] for x in roots)


def test_dist2_kronecker_auto_switches():
    scale = 10
    u, v = O.kronecker(scale, 16, 0xC0FFEE)
    nv = 1 << scale
    sources = [int(u[0]), int(v[5])]
    out, _ = run_dist(2, nv, u, v, sources, "auto")
    dirs = check(nv, u, v, sources, out)
    assert "bu" in dirs and "td" in dirs


def test_dist3_path_graph_crosses_partitions():
    nv = 400  # chunk 192: ranks own [0,192), [192,384), [384,400)
    u = np.arange(nv - 1, dtype=np.uint32)
    v = np.arange(1, nv, dtype=np.uint32)
    out, _ = run_dist(3, nv, u, v, [0, 399, 200], "auto")
    check(nv, u, v, [0, 399, 200], out)


def test_dist2_tiny_graph_empty_rank():
    nv, u, v = O.load_graphfileutil(os.path.join(GOLDEN, "tinyCG.txt"))
    out, _ = run_dist(2, nv, u, v, [0, 3], "auto")  # chunk 64: rank 1 owns no vertex
    check(nv, u, v, [0, 3], out)
