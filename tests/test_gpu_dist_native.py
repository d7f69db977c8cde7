"""Partitioned BFS with the level loop AND the exchange inside libbfsx.so (bfsx_dist_bfs).

The exchange layer has two implementations behind one interface (csrc/bfsx_comm.cpp): RCCL (one
process per GPU, what bench.py --gpus N runs) and an in-process group (P ranks = P host threads of one
process, device copies).  The box has one MI355X, so P = 2, 3, 4 run as an in-process group on device 0;
the kernels, the owner routing, the bucketing, the count/pair exchanges, the all-gathered bottom-up
frontier and the all-reduced direction switch are the code under test.  RCCL itself runs at P = 1
(a communicator of one) in a fresh process.  Distances must be bit-exact against the oracle and the
single-device path; parents are validated (Graph500 rules)."""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
INF = 2147483647


# Every group of this suite runs with the collective-sequence guard on (a rank in a different collective or level
# fails every rank, naming both) and a 60 s deadline on every wait for a peer, so a hang becomes an error well
# inside the test's own limit.
GROUP_DEFAULTS = {"check_collectives": "on", "comm_timeout_ms": "60000"}


def join_ranks(ths, errs, limit=90.0):
    """Join the rank threads against one deadline; a thread still alive after it fails the test with every
    rank's error so far (the errors of ranks that did return are the diagnosis of a hang)."""
    import time
    end = time.time() + limit
    for t in ths:
        t.join(timeout=max(0.0, end - time.time()))
    alive = [i for i, t in enumerate(ths) if t.is_alive()]
    assert not alive, f"rank thread(s) {alive} still inside the library after {limit} s; errors so far: {errs}"


def run_group(bfsx, world, make_graph, sources, direction="auto", options=None):
    """One thread per rank; returns per source: (stats, dist, parent, dirs) assembled globally."""
    opts = dict(GROUP_DEFAULTS, **(options or {}))
    ctxs = [bfsx.Context(0, direction=direction, **opts) for _ in range(world)]
    graphs = [None] * world
    try:
        bfsx.local_group(ctxs)
        for r in range(world):
            graphs[r] = make_graph(ctxs[r], r, world)
        out = []
        for s in sources:
            res, errs = [None] * world, []

            def work(r):
                try:
                    st = graphs[r].dist_bfs(s)
                    d, p = graphs[r].result()
                    res[r] = (st, graphs[r].partition()["v_lo"], d, p, list(graphs[r].level_dirs()))
                except Exception as e:  # noqa: BLE001 -- reported below
                    errs.append(repr(e))

            ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
            for t in ths:
                t.start()
            join_ranks(ths, errs)
            assert not errs, errs
            nv = graphs[0].partition()["nv_global"]
            dist = np.full(nv, INF, np.int32)
            parent = np.full(nv, -1, np.int64)
            for st, lo, d, p, _ in res:
                dist[lo:lo + len(d)] = d
                parent[lo:lo + len(p)] = p
            keys = ("levels", "topdown_levels", "bottomup_levels", "m_comp", "reached")
            assert all({k: r[0][k] for k in keys} == {k: res[0][0][k] for k in keys} for r in res), \
                "ranks disagree on the all-reduced stats"
            assert all(r[4] == res[0][4] for r in res), "ranks took different directions"
            out.append((res[0][0], dist, parent, res[0][4]))
        return out
    finally:
        for g in graphs:
            if g is not None:
                g.free()
        for c in ctxs:
            c.close()


def check(nv, u, v, sources, out):
    off, col = O.build_sets(nv, u, v)
    for s, (st, dist, parent, _) in zip(sources, out):
        ref, _ = O.csr_bfs(nv, off, col, s)
        assert np.array_equal(dist, ref)
        assert st["levels"] == int(ref[ref != INF].max()) + 1
        assert O.validate(nv, off, col, s, dist, parent, rows_sorted=True) == 0
        assert st["m_comp"] == O.mcomp(u, v, ref) and st["reached"] == int((ref != INF).sum())


@pytest.mark.parametrize("world,direction", [(2, "auto"), (2, "topdown"), (2, "bottomup"), (3, "auto"),
                                             (4, "auto"), (4, "bottomup")])
def test_native_group_random(bfsx, world, direction):
    rng = np.random.default_rng(100 + world)
    nv = 6000
    u = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    sources = [0, 2999, 5999]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, direction)
    check(nv, u, v, sources, out)


@pytest.mark.parametrize("mode", ["on", "off"])
@pytest.mark.parametrize("world,direction", [(2, "auto"), (3, "bottomup"), (4, "auto")])
def test_native_group_sparse_frontier_exchange(bfsx, world, direction, mode):
    """Option sparse_exchange: a partitioned pull level receives the global frontier as every rank's id list
    (alltoallv of the per-rank lists, the sizes from the last level close's all-reduce) instead of the bitmap
    all-gather.  "on" forces it on every pull level after the first level (pull -> pull included: the record
    is turned into ids), "off" never: bit-exact against the oracle both ways, on random and Kronecker graphs."""
    rng = np.random.default_rng(900 + world)
    nv = 7000
    u = rng.integers(0, nv, 6 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 6 * nv).astype(np.uint32)
    sources = [0, 3500, 6999]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, direction,
                    options={"sparse_exchange": mode, "check_retired": "on"})
    check(nv, u, v, sources, out)
    assert any(2 in o[3] for o in out)  # pull levels ran
    scale, seed = 15, 0x5BA5
    ku, kv = O.kronecker(scale, 16, seed)
    ksrc = [int(ku[1]), int(ku[2024])]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_kronecker(scale, r, w, seed=seed), ksrc, direction,
                    options={"sparse_exchange": mode})
    check(1 << scale, ku, kv, ksrc, out)


@pytest.mark.parametrize("world,direction", [(2, "auto"), (2, "topdown"), (3, "auto"), (4, "bottomup")])
def test_native_group_no_retired_buffer_referenced(bfsx, world, direction):
    """DESIGN.md 4, event (b): with option check_retired, every launch group and exchange of the partitioned
    loop checks its buffer pointers against the buffers retired so far (grown exchange buffers, the degree
    list's temporaries) and fails the BFS on a hit.  Graphs whose frontiers grow level by level and several
    sources per graph make the loop replace its remote / send / receive buffers mid-BFS; the same random
    graphs as test_native_group_random, plus a Kronecker graph (counted exchanges, hub rows)."""
    rng = np.random.default_rng(100 + world)
    nv = 6000
    u = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    sources = [0, 2999, 5999, 17]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, direction,
                    options={"check_retired": "on", "slot_pairs": "64"})
    check(nv, u, v, sources, out)
    scale, seed = 14, 0xC4EC
    ku, kv = O.kronecker(scale, 16, seed)
    ksrc = [int(ku[0]), int(ku[999]), int(ku[4242])]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_kronecker(scale, r, w, seed=seed), ksrc, direction,
                    options={"check_retired": "on"})
    check(1 << scale, ku, kv, ksrc, out)


@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("world", [2, 4])
def test_native_group_kronecker(bfsx, world, relabel):
    """relabel on (the default): every rank's id range renumbered by degree inside the range (ownership
    unchanged); the results come back in original ids either way."""
    scale, seed = 16, 0xD157
    u, v = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    sources = [int(u[0]), int(u[777])]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_kronecker(scale, r, w, seed=seed), sources,
                    options={"relabel": relabel})
    check(nv, u, v, sources, out)
    assert any(2 in o[3] for o in out)  # a bottom-up level ran against the all-gathered frontier
    # the partitioned result equals the single-device result bit for bit
    with bfsx.Context(0) as ctx, ctx.kronecker(scale, 16, seed) as g:
        for s, o in zip(sources, out):
            d, _, _ = g.bfs(s)
            assert np.array_equal(d, o[1])


@pytest.mark.parametrize("world", [2, 3])
def test_native_group_relabel_ranges(bfsx, world):
    """A relabelled partition keeps every id in its owner's range: each rank's CSR (exported in original
    ids) holds exactly its original rows, and the collective validator accepts the result for a source
    given explicitly on every rank (only its owner knows the source's internal id)."""
    rng = np.random.default_rng(7 + world)
    nv = 5000
    u = rng.integers(0, nv, 6 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 6 * nv).astype(np.uint32)
    off, col = O.build_sets(nv, u, v)
    ctxs = [bfsx.Context(0) for _ in range(world)]
    graphs = [None] * world
    try:
        bfsx.local_group(ctxs)
        for r in range(world):
            graphs[r] = ctxs[r].dist_from_edges(nv, u, v, r, world)
        for r in range(world):
            p = graphs[r].partition()
            lo, n = p["v_lo"], p["nv_local"]
            goff, gcol = graphs[r].csr()
            for x in range(0, n, 97):
                assert set(gcol[goff[x]:goff[x + 1]].tolist()) == set(col[off[lo + x]:off[lo + x + 1]].tolist())
            assert goff[n] == off[lo + n] - off[lo]
        res, errs = [None] * world, []

        def work(r):
            try:
                graphs[r].dist_bfs(1234)
                res[r] = graphs[r].validate(1234)
            except Exception as e:  # noqa: BLE001 -- reported below
                errs.append(repr(e))

        ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=120)
        assert not errs, errs
        assert all(x["errors"] == 0 for x in res) and res[0]["reached"] > 0
    finally:
        for g in graphs:
            if g is not None:
                g.free()
        for c in ctxs:
            c.close()


def test_native_group_int64_offsets(bfsx):
    """The int64 row-offset kernels (graphs with >= 2^32 local adjacency entries) on the partitioned path."""
    scale, seed = 14, 0xBEEF
    u, v = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    sources = [int(u[1]), int(v[2])]
    out = run_group(bfsx, 3, lambda c, r, w: c.dist_kronecker(scale, r, w, seed=seed), sources,
                    options={"offset_bits": "64"})
    check(nv, u, v, sources, out)


@pytest.mark.parametrize("name", ["tinyCG", "mediumG", "tinyG"])
def test_native_group_reference_files(bfsx, name):
    nv, u, v = O.load_graphfileutil(os.path.join(GOLDEN, name + ".txt"))
    world = 2
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), [0])
    check(nv, u, v, [0], out)
    ref = np.loadtxt(os.path.join(GOLDEN, name + ".dist"), dtype=np.int64)
    ref = ref[:, 1] if ref.ndim == 2 else ref
    assert np.array_equal(out[0][1].astype(np.int64), ref)


def test_native_rccl_single_rank():
    """RCCL communicator of one: the same loop over ncclAllGather / grouped send-recv / all-reduce."""
    code = f"""
import sys, os, numpy as np
sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
import conftest, oracle_py as O
bfsx = conftest.load_bfsx()
ctx = bfsx.Context(0)
ctx.comm_init(0, 1, bfsx.comm_unique_id())
u, v = O.kronecker(14, 16, 77)
g = ctx.dist_kronecker(14, 0, 1, seed=77)
ref_ctx = bfsx.Context(0)
rg = ref_ctx.kronecker(14, 16, 77)
for s in (int(u[0]), int(u[5])):
    st = g.dist_bfs(s)
    d, p = g.result()
    d1, _, st1 = rg.bfs(s)
    assert np.array_equal(d, d1), "rccl P=1 differs from the single-device path"
    assert st["m_comp"] == st1["m_comp"] and st["levels"] == st1["levels"]
print("rccl-ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "rccl-ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("slot_pairs", ["0", "16384", "100000000", "auto"])
def test_native_group_exchange_modes(bfsx, slot_pairs):
    """Push-level pair exchange in both forms: counts all-to-all then variable sends (slot_pairs=0),
    fixed per-peer slots for every level (huge threshold), and the default mix; all bit-exact."""
    scale, world = 14, 3
    u, v = O.kronecker(scale, 16, 0xABC)
    nv = 1 << scale
    sources = [int(u[0]), int(v[100]), int(u[5000])]
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, "topdown",
                    {"slot_pairs": slot_pairs})
    check(nv, u, v, sources, out)


@pytest.mark.parametrize("world,bits", [(2, "3"), (3, "8"), (4, "30")])
def test_native_group_hub_domain(bfsx, world, bits):
    """The bottom-up hub probe domain on a partition: hubs ranked by GLOBAL degree (all-gathered at the
    first BFS), their bits gathered from the all-gathered frontier; bit-exact in pull-only and auto."""
    rng = np.random.default_rng(7 + world)
    nv = 5000
    hubs = rng.integers(0, nv, 40)
    u = np.r_[rng.integers(0, nv, 4 * nv), np.repeat(hubs, 300)].astype(np.uint32)
    v = np.r_[rng.integers(0, nv, 4 * nv), rng.integers(0, nv, 40 * 300)].astype(np.uint32)
    sources = [0, int(hubs[0]), 4321]
    for direction in ("bottomup", "auto"):
        out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, direction,
                        {"hub_bits": bits})
        check(nv, u, v, sources, out)


@pytest.mark.parametrize("options", [{}, {"big_degree": "8"}, {"big_degree": "8", "big_cap": "16"},
                                     {"big_degree": "0", "slot_pairs": "4"}])
def test_native_group_source_degrees(bfsx, options):
    """The partitioned loop's first level needs the source's global degree, which only its owner holds:
    every rank looks it up in the list of ids with degree > big_degree (all-gathered once per graph, at
    most big_cap per rank); an unlisted source's degree is bounded by big_degree (fixed exchange slots of
    that size), an overflowed list leaves it unknown (counted exchange).  Sources of degree 0, in the last
    rank's partly padded slice, a 5,000-neighbour hub (listed by default) and ordinary ones all give the
    oracle's distances in every mode; an id outside the graph fails on every rank."""
    rng = np.random.default_rng(31)
    nv = 5003  # not a multiple of 64 * world: the last slice is padded
    u = rng.integers(0, nv - 40, 4 * nv).astype(np.uint32)  # the last 40 ids are isolated
    v = rng.integers(0, nv - 40, 4 * nv).astype(np.uint32)
    hub = 4000  # degree > 4096 (the default big_degree): a star over every other non-isolated id
    u = np.r_[u, np.full(nv - 41, hub)].astype(np.uint32)
    v = np.r_[v, np.delete(np.arange(nv - 40), hub)].astype(np.uint32)
    deg = np.bincount(np.concatenate([u, v]), minlength=nv)
    assert deg[hub] > 4096
    sources = [nv - 1, nv - 41, hub, int(np.argmin(np.where(deg > 0, deg, 1 << 30))), 0]
    out = run_group(bfsx, 3, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), sources, options=options)
    check(nv, u, v, sources, out)
    assert out[0][0]["levels"] == 1 and out[0][0]["reached"] == 1
    ctxs = [bfsx.Context(0) for _ in range(2)]
    graphs = []
    try:
        bfsx.local_group(ctxs)
        graphs = [ctxs[r].dist_from_edges(nv, u, v, r, 2) for r in range(2)]
        errs = [None, None]

        def work(r):
            try:
                graphs[r].dist_bfs(nv)
            except Exception as e:  # noqa: BLE001 -- expected
                errs[r] = str(e)

        ths = [threading.Thread(target=work, args=(r,)) for r in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=120)
        assert all(not t.is_alive() for t in ths), "rank thread hung"
        assert all(e is not None and "outside" in e for e in errs), errs
    finally:
        for g in graphs:
            g.free()
        for c in ctxs:
            c.close()


def run_ranks_timed(ths):
    import time
    t0 = time.time()
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
    return time.time() - t0


@pytest.mark.parametrize("world,rank,where", [(2, 1, "2"), (2, 0, "0"), (4, 2, "1"), (4, 3, "3"), (4, 1, "setup"),
                                              (2, 1, "setup")])
def test_native_group_failed_rank_fails_every_rank(bfsx, world, rank, where):
    """a rank that fails (fault injection, option fail_at=rank:level) aborts the group, so
    EVERY rank's bfsx_dist_bfs returns an error within 5 s -- the failing rank its own, its peers BFSX_E_RCCL
    "peer rank r failed at level k: ..." -- instead of waiting for it inside a collective forever (the round-4
    record r04am: one rank left inside bfsx_dist_bfs, its peer gone).  The group stays failed afterwards, as an
    aborted NCCL communicator does; a fresh group on the same contexts' graphs is not needed for that check."""
    scale, seed = 13, 0xFA11
    ctxs = [bfsx.Context(0, **dict(GROUP_DEFAULTS, fail_at=f"{rank}:{where}")) for _ in range(world)]
    graphs = []
    try:
        bfsx.local_group(ctxs)
        graphs = [ctxs[r].dist_kronecker(scale, r, world, seed=seed) for r in range(world)]
        src = int(O.kronecker(scale, 16, seed)[0][0])
        errs = [None] * world

        def work(r):
            try:
                graphs[r].dist_bfs(src)
            except bfsx.BfsxError as e:
                errs[r] = (e.code, str(e))

        ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        took = run_ranks_timed(ths)
        assert all(not t.is_alive() for t in ths), f"rank thread hung after a peer failed: {errs}"
        assert took < 5.0, took
        assert all(e is not None for e in errs), errs
        lvl = "setup" if where == "setup" else f"level {where}"
        assert "fault injection" in errs[rank][1], errs
        for r in range(world):
            if r != rank:
                assert errs[r][0] == bfsx.BFSX_E_RCCL, errs
                assert f"peer rank {rank} failed at {lvl}" in errs[r][1] and "fault injection" in errs[r][1], errs
        # the aborted group fails every later call at once, on every rank
        errs2 = [None] * world

        def again(r):
            try:
                graphs[r].dist_bfs(src)
            except bfsx.BfsxError as e:
                errs2[r] = str(e)

        ths = [threading.Thread(target=again, args=(r,)) for r in range(world)]
        assert run_ranks_timed(ths) < 5.0
        assert all(e is not None and "fault injection" in e for e in errs2), errs2
    finally:
        for g in graphs:
            g.free()
        for c in ctxs:
            c.close()


def test_native_group_collective_mismatch_detected(bfsx):
    """Option check_collectives: ranks in different collectives (here rank 0 validates while rank 1 starts the
    next BFS) fail on every rank with both collectives named, instead of pairing one rank's all-gather with the
    other's exchange."""
    world, scale, seed = 2, 12, 0xC011
    ctxs = [bfsx.Context(0, **GROUP_DEFAULTS) for _ in range(world)]
    graphs = []
    try:
        bfsx.local_group(ctxs)
        graphs = [ctxs[r].dist_kronecker(scale, r, world, seed=seed) for r in range(world)]
        src = int(O.kronecker(scale, 16, seed)[0][0])
        errs = [None] * world

        def first(r):
            graphs[r].dist_bfs(src)

        ths = [threading.Thread(target=first, args=(r,)) for r in range(world)]
        run_ranks_timed(ths)

        def work(r):
            try:
                if r == 0:
                    graphs[r].validate()
                else:
                    graphs[r].dist_bfs(src)
            except bfsx.BfsxError as e:
                errs[r] = str(e)

        ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        assert run_ranks_timed(ths) < 5.0
        assert all(e is not None for e in errs), errs
        assert any("collective mismatch" in e for e in errs), errs
        assert all("all-gather" in e or "all-to-allv" in e or "all-reduce" in e for e in errs), errs
    finally:
        for g in graphs:
            g.free()
        for c in ctxs:
            c.close()


def test_native_group_missing_rank_times_out(bfsx):
    """A rank that never calls (it crashed without aborting, or took another path) is noticed by the deadline
    (comm_timeout_ms): the waiting rank fails with "timed out" instead of hanging."""
    world, scale, seed = 2, 12, 0x71AE
    ctxs = [bfsx.Context(0, comm_timeout_ms="1500") for _ in range(world)]
    graphs = []
    try:
        bfsx.local_group(ctxs)
        graphs = [ctxs[r].dist_kronecker(scale, r, world, seed=seed) for r in range(world)]
        src = int(O.kronecker(scale, 16, seed)[0][0])
        err = []

        def work():
            try:
                graphs[0].dist_bfs(src)
            except bfsx.BfsxError as e:
                err.append(str(e))

        t = threading.Thread(target=work)
        took = run_ranks_timed([t])
        assert not t.is_alive() and err and "timed out" in err[0], err
        assert 1.0 < took < 10.0, took
    finally:
        for g in graphs:
            g.free()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("world", [2, 3])
def test_group_context_one_call(bfsx, world):
    """bfsx_init_group (multi-GPU is internal, the caller sees one call): graphs built on a group
    context are partitioned over its ranks, and bfsx_bfs / bfsx_result / bfsx_validate / bfsx_level_* return the
    whole graph's result from one call.  On this one-GPU box the ranks share device 0 (in-process group); the
    result equals the single-device one bit for bit, from an algs4 file (every rank tokenizes it on its GPU,
    bfsx_dist_graph_load_algs4), a tuple list and the Kronecker generator."""
    with bfsx.Context(group=world, **GROUP_DEFAULTS) as gc, bfsx.Context(0) as one:
        assert gc.group_size == world and one.group_size == 1
        for name in ("mediumG", "tinyCG"):
            path = os.path.join(GOLDEN, name + ".txt")
            with gc.load_algs4(path) as g, one.load_algs4(path) as g1:
                assert g.nv == g1.nv and g.nnz == g1.nnz and g.m == g1.m
                d, p, st = g.bfs(0)
                d1, _, st1 = g1.bfs(0)
                assert np.array_equal(d, d1)
                ref = np.loadtxt(os.path.join(GOLDEN, name + ".dist"), dtype=np.int64)
                assert np.array_equal(d.astype(np.int64), ref[:, 1] if ref.ndim == 2 else ref)
                assert st["levels"] == st1["levels"] and st["m_comp"] == st1["m_comp"]
                assert st["reached"] == st1["reached"]
                assert g.validate()["errors"] == 0
                nv, u, v = O.load_graphfileutil(path)
                off, col = O.build_sets(nv, u, v)
                assert O.validate(nv, off, col, 0, d, p, rows_sorted=False) == 0
                assert len(g.level_times()) == st["levels"] and len(g.level_dirs()) == st["levels"]
                ls = g.level_stats()
                assert sum(x["frontier_out"] for x in ls) == st["reached"] - 1
                # a partition's pull levels store every parent explicitly, summed over the ranks like frontier_out
                pulls = [x for x in ls if x["direction"] == 2]
                assert sum(x["explicit_parents"] for x in pulls) == sum(x["frontier_out"] for x in pulls)
                d2, p2 = g.result()
                assert np.array_equal(d2, d) and np.array_equal(p2, p)
                goff, gcol = g.csr()
                for x in range(0, nv, 7):
                    assert set(gcol[goff[x]:goff[x + 1]].tolist()) == set(col[off[x]:off[x + 1]].tolist())
        scale, seed = 14, 0x6A0B
        u, v = O.kronecker(scale, 16, seed)
        with gc.kronecker(scale, 16, seed) as g, gc.from_edges(1 << scale, u, v) as ge, \
                one.kronecker(scale, 16, seed) as g1:
            roots = g.sample_roots(4)
            assert np.array_equal(roots, g1.sample_roots(4))
            for r in roots.tolist():
                d, p, st = g.bfs(r)
                assert np.array_equal(d, g1.bfs(r)[0])
                assert np.array_equal(ge.bfs(r)[0], d)
                assert g.validate()["errors"] == 0 and st["t_bfs_ms"] > 0
        with pytest.raises(bfsx.BfsxError):
            with gc.kronecker(12, 16, 1) as g:
                g.bfs(1 << 12)  # outside the graph: fails on every rank, and the group stays usable
        with gc.kronecker(12, 16, 1) as g, one.kronecker(12, 16, 1) as g1:
            assert np.array_equal(g.bfs(5)[0], g1.bfs(5)[0])


def run_group_errors(bfsx, world, make_graph, source, options):
    """One partitioned BFS per rank thread; returns every rank's error (None where a rank succeeded)."""
    opts = dict(GROUP_DEFAULTS, **options)
    ctxs = [bfsx.Context(0, **opts) for _ in range(world)]
    graphs = [None] * world
    try:
        bfsx.local_group(ctxs)
        for r in range(world):
            graphs[r] = make_graph(ctxs[r], r, world)
        errs = [None] * world

        def work(r):
            try:
                graphs[r].dist_bfs(source)
            except Exception as e:  # noqa: BLE001 -- returned to the test
                errs[r] = str(e)

        ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ths:
            t.start()
        join_ranks(ths, [e for e in errs if e])
        return errs
    finally:
        for g in graphs:
            if g is not None:
                g.free()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("world", [2, 3])
def test_native_group_store_guard_slot_overflow(bfsx, world):
    """Round 6 (verdict item 1): every computed index of the push / exchange path is checked before its store.
    With fixed exchange slots forced to one pair (test hook slot_force), the level-0 owner routes more pairs
    to a peer than its slot holds: the guard refuses the store, and every rank fails at that level's close
    with the site, index and bound -- an error, not a device fault."""
    rng = np.random.default_rng(61 + world)
    nv = 4000
    u = rng.integers(0, nv, 8 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 8 * nv).astype(np.uint32)
    hub = 5  # degree >> world: some peer receives several of its pairs at level 0
    u = np.r_[u, np.full(nv - 1, hub)].astype(np.uint32)
    v = np.r_[v, np.delete(np.arange(nv), hub)].astype(np.uint32)
    errs = run_group_errors(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), hub,
                            {"slot_force": "1", "direction": "topdown"})
    assert all(e is not None and "device guard" in e and "fired at level 0" in e for e in errs), errs
    assert any("store guard" in e and "fixed exchange slot" in e for e in errs), errs
    # the same graph without the hook: the oracle's distances
    out = run_group(bfsx, world, lambda c, r, w: c.dist_from_edges(nv, u, v, r, w), [hub], "topdown")
    check(nv, u, v, [hub], out)


@pytest.mark.parametrize("world", [2, 3])
def test_native_group_empty_push_workgroup_race(bfsx, world):
    """DESIGN.md 4, event (d), the cause of the rounds-3..5 intermittent "illegal memory access": a k_td workgroup
    with no frontier vertex (every non-owner at level 0) went from the queue init straight to its final flushes,
    and no barrier separated thread 0's zeroing of the LDS queue counts from the other waves' reads.  Test hook
    race_probe fills every CU's LDS with stale words and makes wave 0 zero the counts late:
      delay      the product kernel (barrier after the init): the oracle's distances;
      nobarrier  the rounds-3..5 kernel: the empty workgroup's other waves flush 16,843,009 stale entries to a
                 stale base -- once a wild store, now refused by the store guard on every rank."""
    rng = np.random.default_rng(71 + world)
    nv = 6000
    u = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 5 * nv).astype(np.uint32)
    make = lambda c, r, w: c.dist_from_edges(nv, u, v, r, w)  # noqa: E731
    out = run_group(bfsx, world, make, [0, nv - 1], "auto", {"race_probe": "delay"})
    check(nv, u, v, [0, nv - 1], out)
    errs = run_group_errors(bfsx, world, make, 0, {"race_probe": "nobarrier"})
    assert all(e is not None and "device guard" in e for e in errs), errs
    assert any("store guard" in e for e in errs), errs


def test_group_context_rccl_clique():
    """bfsx_init_group on distinct devices: an RCCL clique (ncclCommInitAll, threaded warm-up, the heap abort board).
    It needs one device per rank, so it skips on a one-GPU box and runs by itself on a multi-GPU one
    (BFSX_GROUP_COMM=rccl makes a group with fewer devices than ranks an error instead of an in-process group)."""
    code = f"""
import ctypes as C, sys, os, numpy as np
n = C.c_int(0)
C.CDLL("libamdhip64.so").hipGetDeviceCount(C.byref(n))
if n.value < 2:
    print("skip: %d device(s)" % n.value); sys.exit(0)
sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
import conftest, oracle_py as O
bfsx = conftest.load_bfsx()
P = min(n.value, 4)
with bfsx.Context(group=P) as gc, bfsx.Context(0) as one:
    with gc.kronecker(16, 16, 0x51) as g, one.kronecker(16, 16, 0x51) as g1:
        for r in g.sample_roots(4).tolist():
            d, p, st = g.bfs(r)
            d1, _, st1 = g1.bfs(r)
            assert np.array_equal(d, d1) and st["m_comp"] == st1["m_comp"]
            assert g.validate()["errors"] == 0
print("clique-ok", P)
"""
    env = dict(os.environ, BFSX_GROUP_COMM="rccl")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    if r.stdout.startswith("skip"):
        pytest.skip(r.stdout.strip())
    assert "clique-ok" in r.stdout, r.stdout + r.stderr


def test_native_group_comm_timing(bfsx):
    """Option comm_timing: hipEvents around every collective of the level loop.  One level-close all-reduce per
    level, one all-gather or id all-to-allv per pull level, one pair all-to-allv per push level that shipped; off
    (the default) reports zeros.  A group graph reports the largest span over its ranks."""
    scale, seed = 14, 0x77
    with bfsx.Context(group=2, **GROUP_DEFAULTS) as gc, gc.kronecker(scale, 16, seed) as g:
        r = int(g.sample_roots(1)[0])
        g.bfs(r)
        assert all(v == (0.0, 0) for v in g.comm_times().values())
        gc.set_option("comm_timing", "on")
        _, _, st = g.bfs(r)
        ct = g.comm_times()
        dirs = list(g.level_dirs())
        assert ct["allreduce"][1] == st["levels"] and ct["allreduce"][0] > 0
        pulls = sum(1 for x in dirs if x == 2)
        assert ct["allgather"][1] + ct["alltoallv"][1] >= pulls
        assert ct["alltoallv"][1] <= len(dirs) and all(ms >= 0 for ms, _ in ct.values())
        gc.set_option("comm_timing", "off")
