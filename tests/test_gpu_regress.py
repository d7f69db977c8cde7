"""GPU regression tests for the two round-2 wrong-result events ("Wrong-result events").

(a) Garbage distances (round-2 gpurun_out/r02t/parity.log, test_offset_width_paths[auto], root 858): the
    result was staged in the frontier queues qa / qb, so a queue consumer that read past a queue's tail
    met the previous result's distances (INT32_MAX, small ints) as vertex ids.  Now the result has its own
    staging buffers, and every queue consumer checks its ids against the rows it holds (id_ok): a read
    past a tail fails the BFS loudly instead of indexing wild memory.  These tests poison the queues with
    0xFFFFFFFF before every BFS (option poison_queues), so ANY consumer that reads an entry no producer
    wrote trips the guard -- and prove that the guard does trip (option test_overread).
(b) The in-process group corruption with a spilling pull kernel: tests/test_gpu_dist_native.py runs the
    group; here the partitioned loop runs under the same poisoned-queue regime.
"""
import numpy as np
import pytest

import oracle_py as O
from conftest import load_bfsx
from test_gpu_parity import check_against_oracle

pytestmark = [pytest.mark.gpu, pytest.mark.diag]  # test hooks: the diagnostic library
INF = 2147483647


def test_guard_catches_a_read_past_the_queue_tail(ctx):
    """The guard is live: a push level told to read one entry past its queue's tail (test_overread) meets
    the poisoned word and the BFS fails with BFSX_E_HIP naming the id, instead of returning a result."""
    bfsx = load_bfsx()
    u = np.array([0, 1, 2, 3], np.uint32)
    v = np.array([1, 2, 3, 4], np.uint32)
    try:
        ctx.set_option("poison_queues", "on")
        ctx.set_option("persist", "off")
        ctx.set_option("direction", "topdown")
        ctx.set_option("test_overread", "0")
        with ctx.from_edges(5, u, v) as g:
            with pytest.raises(bfsx.BfsxError) as e:
                g.bfs(0)
            assert "4294967295" in str(e.value) and e.value.code == -4
            ctx.set_option("test_overread", "off")
            d, _, _ = g.bfs(0)  # the guard word was cleared: the next BFS is clean
            assert d.tolist() == [0, 1, 2, 3, 4]
    finally:
        for k, val in (("test_overread", "off"), ("persist", "on"), ("direction", "auto"), ("poison_queues", "off")):
            ctx.set_option(k, val)


def test_round2_failing_sequence_poisoned(ctx):
    """The exact sequence of the round-2 failure, once, with poisoned queues: the persist-blocks test's
    graph with persist_blocks changed between runs, then test_offset_width_paths[auto]'s scale-14 graph
    (seed 4242, roots sampled with seed 5 -- 858 among them) in all three direction modes, each result
    bit-exact against the oracle."""
    kids, fan = 1000, 40
    nv = 1 + kids + kids * fan
    child = np.arange(1, kids + 1)
    u = np.r_[np.zeros(kids), np.repeat(child, fan)].astype(np.uint32)
    v = np.r_[child, np.arange(kids + 1, nv)].astype(np.uint32)
    off, col = O.build_sets(nv, u, v)
    try:
        ctx.set_option("poison_queues", "on")
        ctx.set_option("direction", "topdown")
        ctx.set_option("persist_blocks", "2")
        with ctx.from_edges(nv, u, v) as g:
            check_against_oracle(g, nv, off, col, 0, mr=False)
            ctx.set_option("persist_blocks", "auto")
            for src in (0, kids - 2):
                check_against_oracle(g, nv, off, col, src, mr=False)
        ctx.set_option("direction", "auto")
        scale, seed = 14, 4242
        ou, ov = O.kronecker(scale, 16, seed)
        nv = 1 << scale
        off, col = O.build_sets(nv, ou, ov)
        for bits in ("auto", "64"):
            ctx.set_option("offset_bits", bits)
            for direction in ("auto", "topdown", "bottomup"):
                ctx.set_option("direction", direction)
                with ctx.kronecker(scale, 16, seed) as g:
                    roots = [int(r) for r in g.sample_roots(3, seed=5)]
                    for r in roots + [858]:
                        check_against_oracle(g, nv, off, col, r, ou, ov, mr=False)
    finally:
        for k, val in (("persist_blocks", "auto"), ("direction", "auto"), ("offset_bits", "auto"),
                       ("poison_queues", "off")):
            ctx.set_option(k, val)


@pytest.mark.parametrize("floor", ["0", "65536"])
@pytest.mark.parametrize("leaf_skip", ["on", "off"])
@pytest.mark.parametrize("persist,hybrid", [("on", "auto"), ("off", "auto"), ("on", "force")])
def test_poisoned_queues_kronecker(ctx, leaf_skip, persist, hybrid, floor):
    """Every queue hand-off of the single-device loop (push -> push, K3p -> push, pull -> push with the leaf
    skip's shortened queue, hybrid levels) under poisoned queues: bit-exact distances over 12 roots.  floor:
    the push -> pull floor (pull_min_edges); 65,536 is the default the bench runs, under which K3p takes over
    the sparse pull's queue."""
    ou, ov = O.kronecker(16, 16, 0x1EAF)
    nv = 1 << 16
    off, col = O.build_sets(nv, ou, ov)
    try:
        for k, val in (("poison_queues", "on"), ("leaf_skip", leaf_skip), ("persist", persist), ("hybrid", hybrid),
                       ("pull_min_edges", floor)):
            ctx.set_option(k, val)
        with ctx.kronecker(16, 16, 0x1EAF) as g:
            for r in g.sample_roots(12, seed=5):
                check_against_oracle(g, nv, off, col, int(r), ou, ov, mr=False)
    finally:
        for k, val in (("poison_queues", "off"), ("leaf_skip", "on"), ("persist", "on"), ("hybrid", "auto"),
                       ("pull_min_edges", "0")):
            ctx.set_option(k, val)


def test_poisoned_queues_leaf_frontier_and_deep_path(ctx):
    """The leaf-skip edge case (a pull level hands a push level a frontier of leaves only: an empty queue)
    and a 3,000-level path (K3p hand-backs), under poisoned queues."""
    s, h = 0, 1
    c = 2 + np.arange(3000)
    lv = 3002 + np.arange(1000)
    u = np.r_[[s], np.full(3000, h), c[:1000]].astype(np.uint32)
    v = np.r_[[h], c, lv].astype(np.uint32)
    nv = 4002 + 100000
    off, col = O.build_sets(nv, u, v)
    pu = np.arange(2999, dtype=np.uint32)
    pn = 3000
    poff, pcol = O.build_sets(pn, pu, pu + 1)
    try:
        ctx.set_option("poison_queues", "on")
        with ctx.from_edges(nv, u, v) as g:
            _, _, st = check_against_oracle(g, nv, off, col, s, u, v, mr=False)
            assert st["levels"] == 4
        with ctx.from_edges(pn, pu, pu + 1) as g:
            for src in (0, 1500):
                check_against_oracle(g, pn, poff, pcol, src, mr=False)
    finally:
        ctx.set_option("poison_queues", "off")


@pytest.mark.parametrize("world", [2, 4])
def test_poisoned_queues_partitioned_group(bfsx, world):
    """The partitioned loop (in-process group of `world` ranks on one device, ranks running concurrently)
    under poisoned queues: every queue and every received pair is produced before it is read, and the
    distances equal the oracle's."""
    from test_gpu_dist_native import check, run_group
    scale = 14
    ou, ov = O.kronecker(scale, 16, 77)
    nv = 1 << scale
    off, _ = O.build_sets(nv, ou, ov)
    deg = np.diff(off)
    sources = [int(x) for x in np.nonzero(deg > 0)[0][[0, 7, 100]]]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_kronecker(scale, r, w, 16, 77), sources,
                    options={"poison_queues": "on"})
    check(nv, ou, ov, sources, out)


@pytest.mark.parametrize("world", [2, 4])
def test_spilling_pull_kernel_partitioned_group(bfsx, world):
    """Round-2 event (b): the partitioned pull kernel built to spill to scratch (option bu_force_spill,
    k_bu_spill) while the ranks of an in-process group run concurrently.  With replaced buffers retired
    instead of freed mid-loop, the spilling build returns the oracle's distances (pull-only levels, so
    every level runs the spilling kernel)."""
    from test_gpu_dist_native import check, run_group
    scale = 14
    ou, ov = O.kronecker(scale, 16, 91)
    nv = 1 << scale
    off, _ = O.build_sets(nv, ou, ov)
    deg = np.diff(off)
    sources = [int(x) for x in np.nonzero(deg > 0)[0][[0, 11, 300]]]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_kronecker(scale, r, w, 16, 91), sources, "bottomup",
                    options={"bu_force_spill": "on", "poison_queues": "on"})
    check(nv, ou, ov, sources, out)


def test_product_library_refuses_test_hooks(bfsx):
    """The product library compiles no test hook: setting one fails loudly (only "off" is accepted, a no-op);
    the diagnostic library takes it."""
    with bfsx.Context(0) as c:
        assert not c.diag
        for k, val in (("poison_queues", "on"), ("test_overread", "0"), ("bu_force_spill", "on"),
                       ("persist_abort_at", "3"), ("check_retired", "on"), ("fail_at", "0:1")):
            with pytest.raises(bfsx.BfsxError, match="diagnostic library"):
                c.set_option(k, val)
            c.set_option(k, "off")
    with bfsx.Context(0, poison_queues="on") as d:
        assert d.diag
        d.set_option("test_overread", "off")
