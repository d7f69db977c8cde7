"""BASELINE configs[4] in the GPU suite: Graph500 Kronecker scale 30 (2^30 vertices, 2^34 tuples, 34.0 G
adjacency entries), 1-D partitioned over 8 ranks.

The box has one MI355X, so the 8 ranks run as an in-process exchange group (bfsx_comm_local_group: one host
thread per rank, device copies instead of xGMI) through the SAME native level loop (bfsx_dist_bfs) that
`bench.py --gpus 8` runs over RCCL -- owner-routed pair exchange for push levels (the replacement of
Spark's reduceByKey shuffle, BfsSpark.java:90), all-gathered frontier bitmaps for pull levels, all-reduced
level counters.  The partition holds 149 GB of graph on the one device.

  test_scale30_partition_p8    builds the 8 rank slices, runs a BFS from one sampled root, validates it
                               collectively over all 34.0 G entries (Graph500 rules: a passing result
                               holds exactly the BFS distances) and keeps every rank's distance slice;
  test_scale30_single_device   frees the partition, builds the whole graph on the one device, runs the
                               same root and asserts the distances equal the partition's bit for bit.
"""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCALE, P = 30, 8
_state = {}


def run_ranks(fn):
    res, errs = [None] * P, []

    def work(r):
        try:
            res[r] = fn(r)
        except Exception as e:  # noqa: BLE001 -- re-raised below
            errs.append(f"rank {r}: {e!r}")

    ths = [threading.Thread(target=work, args=(r,)) for r in range(P)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not errs, errs
    assert not any(t.is_alive() for t in ths), "rank thread hung"
    return res


def test_scale30_partition_p8(bfsx):
    # the hub probe domain (a per-device memory decision) stays off: 8 ranks sharing ONE
    # device's HBM cannot each hold one next to 149 GB of graph, as 8 ranks on 8 devices would
    ctxs = [bfsx.Context(0, hub_bits="off") for _ in range(P)]
    graphs = []
    try:
        bfsx.local_group(ctxs)
        t0 = time.perf_counter()
        for r in range(P):  # one rank at a time: the build temporaries never overlap
            graphs.append(ctxs[r].dist_kronecker(SCALE, r, P))
            ctxs[r].synchronize()
        build_s = time.perf_counter() - t0
        parts = [g.partition() for g in graphs]
        assert parts[0]["nv_global"] == 1 << SCALE
        assert all(p["chunk"] == parts[0]["chunk"] for p in parts)
        roots = run_ranks(lambda r: [int(x) for x in graphs[r].sample_roots(1, seed=0x5EED)])
        assert all(x == roots[0] for x in roots)
        root = roots[0][0]

        def one(r):
            st = graphs[r].dist_bfs(root)
            v = graphs[r].validate()
            d, _ = graphs[r].result(want_parent=False)
            return st, v, d

        res = run_ranks(one)
        st, v = res[0][0], res[0][1]
        assert v["errors"] == 0, v
        assert v["entries"] == sum(g.nnz for g in graphs)  # every adjacency entry of the graph checked
        assert v["entries"] > 34_000_000_000
        assert st["reached"] == v["reached"] and st["m_comp"] > 0
        assert st["topdown_levels"] > 0 and st["bottomup_levels"] > 0  # both exchange forms ran
        _state["root"] = root
        _state["levels"] = st["levels"]
        _state["dist"] = [(p["v_lo"], res[r][2]) for r, p in enumerate(parts)]
        print(f"scale-30 P=8 partition: build {build_s:.1f} s, root {root}, {st['levels']} levels, "
              f"{v['entries']} entries validated")
    finally:
        for g in graphs:
            g.free()
        for c in ctxs:
            c.close()


def test_scale30_single_device(bfsx):
    if "root" not in _state:
        pytest.skip("needs test_scale30_partition_p8's distances")
    with bfsx.Context(0) as ctx:
        with ctx.kronecker(SCALE) as g:
            d, _, st = g.bfs(_state["root"], want_parent=False)
            v = g.validate()
    assert v["errors"] == 0
    assert st["levels"] == _state["levels"]
    for lo, dp in _state["dist"]:
        assert np.array_equal(d[lo:lo + len(dp)], dp), f"slice at {lo} differs from the partitioned BFS"
    _state.clear()
