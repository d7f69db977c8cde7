"""Full-size parity through a size-independent property: Graph500-style validation on the device.

bfsx_validate (csrc/kernels_validate.hip) checks, in one pass over the CSR, the rules of the oracle's
orc_validate (Graph500 kernel-2 validation + algs4.jar!/BreadthFirstPaths.java:171-212 `check`).  A
result that passes holds exactly the BFS distances of the graph, so at BASELINE.json's full sizes
(scale 26 on one device, partitioned graphs) these tests prove bit-exact distances without a CPU
oracle run.  Small cases first pin the device validator against the oracle's verdict, on correct
results and on deliberately corrupted ones."""
import os
import threading

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN
from test_gpu_parity import random_cases, sort_rows

pytestmark = pytest.mark.gpu
INF = 2147483647


def corruptions(nv, off, col, src, dist, parent, rng):
    """(name, dist, parent) variants that break one validation rule each (when the graph allows it)."""
    out = []
    reached = np.nonzero((dist != INF) & (np.arange(nv) != src))[0]
    if len(reached):
        v = int(rng.choice(reached))
        d = dist.copy()
        d[v] += 1  # distance off by one (parent level rule / edge rule)
        out.append(("dist_plus_one", d, parent))
        p = parent.copy()
        nbrs = set(col[off[v]:off[v + 1]].tolist())
        non = [w for w in range(nv) if w not in nbrs and w != v]
        if non:
            p[v] = non[0]  # parent that is not a neighbour
            out.append(("parent_not_neighbour", dist, p))
        d = dist.copy()
        p = parent.copy()
        d[v] = INF
        p[v] = -1  # a reached vertex dropped from the tree
        out.append(("dropped_vertex", d, p))
    d = dist.copy()
    p = parent.copy()
    p[src] = -1
    out.append(("source_without_self_parent", d, p))
    return out


@pytest.mark.parametrize("case", random_cases()[:14], ids=lambda c: c[0])
def test_device_validator_agrees_with_oracle(ctx, case):
    name, nv, u, v = case
    u = np.asarray(u, np.uint32)
    v = np.asarray(v, np.uint32)
    off, col = O.build_sets(nv, u, v)
    rng = np.random.default_rng(7)
    with ctx.from_edges(nv, u, v) as g:
        for s in sorted({0, nv // 2}):
            dist, parent, st = g.bfs(s)
            res = g.validate()
            assert res["errors"] == 0 and res["first_bad"] == -1, res
            assert res["reached"] == st["reached"] and res["entries"] == g.nnz
            # the oracle's own serial BFS tree (algs4 semantics) is a different valid tree
            refd, refp = O.csr_bfs(nv, off, col, s)
            assert g.validate_result(s, refd, refp) == (0, -1)
            for cname, d, p in corruptions(nv, off, col, s, dist, parent, rng):
                errs, first = g.validate_result(s, d, p)
                assert (errs > 0) == (O.validate(nv, off, col, s, d, p) != 0), cname
                assert errs > 0, cname
                assert first >= 0


@pytest.mark.parametrize("name", ["tinyCG", "mediumG", "tinyG"])
def test_reference_files_validate(ctx, name):
    with ctx.load_algs4(os.path.join(GOLDEN, name + ".txt")) as g:
        for s in range(min(g.nv, 16)):
            g.bfs(s, want_dist=False, want_parent=False)
            res = g.validate()
            assert res["errors"] == 0, (s, res)
        # wrong source: the result of the last BFS checked as if it came from another vertex
        errs, _ = g.validate_result(0, *g.result())
        assert errs > 0


def test_scale26_full_size_validated(ctx):
    """BASELINE.json configs[3] at full size: scale-26 Kronecker (2.1 G adjacency entries).  For 4 roots
    every direction policy validates, and push-only / pull-only / direction-optimising runs return the
    identical distance vector (three different algorithms, one answer)."""
    with ctx.kronecker(26, 16, 0x5EED2026) as g:
        roots = [int(r) for r in g.sample_roots(4, seed=0x5EED)]
        for i, r in enumerate(roots):
            d_auto, _, st = g.bfs(r, want_parent=False)
            res = g.validate()
            assert res["errors"] == 0, (r, res)
            assert res["entries"] == g.nnz and res["reached"] == st["reached"]
            assert st["bottomup_levels"] > 0
            if i < 2:
                for direction in ("topdown", "bottomup"):
                    ctx.set_option("direction", direction)
                    try:
                        d, _, st2 = g.bfs(r, want_parent=False)
                    finally:
                        ctx.set_option("direction", "auto")
                    assert g.validate()["errors"] == 0
                    assert np.array_equal(d, d_auto), direction
                    assert st2["levels"] == st["levels"]


def test_partitioned_validation_collective(bfsx):
    """In-process group of 4 ranks on device 0, scale-20 Kronecker: the collective validator passes on
    every rank and the assembled distances equal the single-device result."""
    world, scale = 4, 20
    ctxs = [bfsx.Context(0) for _ in range(world)]
    graphs = [None] * world
    single = bfsx.Context(0)
    try:
        bfsx.local_group(ctxs)
        for r in range(world):
            graphs[r] = ctxs[r].dist_kronecker(scale, r, world)
        with single.kronecker(scale) as g1:
            for s in [int(x) for x in g1.sample_roots(2, seed=3)]:
                d1, _, _ = g1.bfs(s, want_parent=False)
                res, errs = [None] * world, []

                def work(r):
                    try:
                        graphs[r].dist_bfs(s)
                        v = graphs[r].validate()
                        d, _ = graphs[r].result()
                        res[r] = (v, graphs[r].partition()["v_lo"], d)
                    except Exception as e:  # noqa: BLE001 -- reported below
                        errs.append(repr(e))

                ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
                for t in ths:
                    t.start()
                for t in ths:
                    t.join(timeout=120)
                assert not errs, errs
                assert all(not t.is_alive() for t in ths)
                for v, lo, d in res:
                    assert v["errors"] == 0, v
                    assert v["reached"] == res[0][0]["reached"]  # all-reduced
                    assert np.array_equal(d, d1[lo:lo + len(d)])
                assert res[0][0]["entries"] == g1.nnz
    finally:
        for g in graphs:
            if g is not None:
                g.free()
        for c in ctxs:
            c.close()
        single.close()
