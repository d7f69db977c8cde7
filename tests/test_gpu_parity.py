"""GPU parity tests: libbfsx.so on cuda:0 against the CPU oracle and the committed golden vectors.

Distances must be bit-exact (integer work); parent trees are validated (Graph500 rules +
BreadthFirstPaths.check), not compared, because the reference's own tie-break is shuffle-order
dependent (BfsSpark.java:97)."""
import os

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
INF = 2147483647


def read_dist(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return np.array([int(line.split()[1]) for line in f], dtype=np.int32)


def sort_rows(off, col):
    """Rows sorted ascending (device rows may be degree-ordered; the oracle validator bisects)."""
    rows = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
    return col[np.lexsort((col, rows))]


def same_sets(off, col, goff, gcol):
    """CSR equality as neighbour sets."""
    return np.array_equal(goff, off) and np.array_equal(sort_rows(goff, gcol), col)


def check_against_oracle(g, nv, off, col, src, u=None, v=None, mr=True):
    dist, parent, st = g.bfs(src)
    if mr:
        r = O.mapreduce_bfs(nv, off, col, src)
        ref = r["dist"]
        assert st["levels"] == r["iters"]
    else:
        ref, _ = O.csr_bfs(nv, off, col, src)
        assert st["levels"] == int(ref[ref != INF].max()) + 1
    if not np.array_equal(dist, ref):  # gather evidence before failing (a one-off mismatch was seen once)
        bad = np.nonzero(dist != ref)[0]
        d2, _, st2 = g.bfs(src)
        goff, gcol = g.csr()
        raise AssertionError(
            f"distance mismatch from {src}: {bad.size} vertices, first {bad[:8].tolist()} gpu "
            f"{dist[bad[:8]].tolist()} ref {ref[bad[:8]].tolist()}; rerun equal to ref: "
            f"{np.array_equal(d2, ref)}, rerun equal to first run: {np.array_equal(d2, dist)}; CSR equal "
            f"as sets: {same_sets(off, col, goff, gcol)}; stats {st} rerun {st2}")
    assert O.validate(nv, off, col, src, dist, parent) == 0
    assert st["reached"] == int((ref != INF).sum())
    if u is not None:
        assert st["m_comp"] == O.mcomp(u, v, ref)
    return dist, parent, st


@pytest.mark.parametrize("name", ["tinyCG", "mediumG", "tinyG"])
@pytest.mark.parametrize("direction", ["auto", "topdown", "bottomup"])
def test_reference_test_sets_bit_exact(ctx, name, direction):
    ctx.set_option("direction", direction)
    try:
        path = os.path.join(GOLDEN, name + ".txt")
        nv, u, v = O.load_graphfileutil(path)
        off, col = O.build_sets(nv, u, v)
        with ctx.load_algs4(path) as g:
            assert g.nv == nv and g.m == len(u) and g.nnz == off[-1]
            goff, gcol = g.csr()
            assert same_sets(off, col, goff, gcol)
            dist, parent, st = check_against_oracle(g, nv, off, col, 0, u, v)
            assert np.array_equal(dist, read_dist(name + ".dist"))
            assert O.dist_sha256(dist) == O.dist_sha256(read_dist(name + ".dist"))
            assert st["levels"] == {"tinyCG": 3, "mediumG": 14, "tinyG": 3}[name]
            t = g.level_times()
            assert len(t) == st["levels"] and np.all(np.diff(t) >= 0)
    finally:
        ctx.set_option("direction", "auto")


def test_tinycg_every_source(ctx):
    path = os.path.join(GOLDEN, "tinyCG.txt")
    nv, u, v = O.load_graphfileutil(path)
    off, col = O.build_sets(nv, u, v)
    with ctx.load_algs4(path) as g:
        for s in range(nv):
            check_against_oracle(g, nv, off, col, s, u, v)


def random_cases():
    rng = np.random.default_rng(2026)
    cases = []
    # (name, nv, u, v)
    for i in range(12):
        nv = int(rng.integers(1, 3000))
        m = int(rng.integers(0, 6 * nv + 1))
        cases.append((f"rand{i}", nv, rng.integers(0, nv, m), rng.integers(0, nv, m)))
    n = 5000
    cases.append(("path", n, np.arange(n - 1), np.arange(1, n)))             # deep: 5000 levels
    cases.append(("star", 20000, np.zeros(19999, int), np.arange(1, 20000)))  # hub bin
    hubs = np.repeat(np.arange(8), 9000)
    cases.append(("multi_hub", 12000, hubs, rng.integers(0, 12000, hubs.size)))
    cases.append(("isolated", 1000, np.array([3, 5]), np.array([5, 7])))
    cases.append(("self_loops", 100, np.arange(100), np.arange(100)))
    cases.append(("dups", 64, np.tile(np.arange(63), 5), np.tile(np.arange(1, 64), 5)))
    cases.append(("single", 1, np.zeros(0, int), np.zeros(0, int)))
    cases.append(("two_comp", 130, np.r_[np.arange(64), np.arange(65, 129)],
                  np.r_[np.arange(1, 65), np.arange(66, 130)]))
    return cases


@pytest.mark.parametrize("case", random_cases(), ids=lambda c: c[0])
@pytest.mark.parametrize("direction", ["auto", "topdown", "bottomup"])
def test_edge_cases_bit_exact(ctx, case, direction):
    name, nv, u, v = case
    u = np.asarray(u, np.uint32)
    v = np.asarray(v, np.uint32)
    off, col = O.build_sets(nv, u, v)
    ctx.set_option("direction", direction)
    try:
        with ctx.from_edges(nv, u, v) as g:
            goff, gcol = g.csr()
            assert same_sets(off, col, goff, gcol)
            srcs = {0, nv - 1, nv // 2}
            for s in sorted(srcs):
                check_against_oracle(g, nv, off, col, s, u, v, mr=(nv <= 3000))
    finally:
        ctx.set_option("direction", "auto")


def test_hub_threshold_sweep(ctx):
    rng = np.random.default_rng(5)
    nv = 4096
    u = np.r_[np.zeros(3000, int), rng.integers(0, nv, 20000)].astype(np.uint32)
    v = np.r_[rng.integers(0, nv, 3000), rng.integers(0, nv, 20000)].astype(np.uint32)
    off, col = O.build_sets(nv, u, v)
    ref, _ = O.csr_bfs(nv, off, col, 0)
    try:
        for hub in (1, 16, 64, 4096, 1 << 20):
            ctx.set_option("hub_degree", hub)
            ctx.set_option("direction", "topdown")
            with ctx.from_edges(nv, u, v) as g:
                d, p, _ = g.bfs(0)
                assert np.array_equal(d, ref)
                assert O.validate(nv, off, col, 0, d, p) == 0
    finally:
        ctx.set_option("hub_degree", 64)
        ctx.set_option("direction", "auto")


@pytest.mark.parametrize("scale", [8, 12, 16])
def test_kronecker_generator_bit_exact(ctx, scale):
    u, v = ctx.kronecker_edges(scale, 16, 0x5EED2026)
    ou, ov = O.kronecker(scale, 16, 0x5EED2026)
    assert np.array_equal(u, ou) and np.array_equal(v, ov)


@pytest.mark.parametrize("scale", [10, 16])
def test_kronecker_bfs_parity(ctx, scale):
    seed = 0xABCD + scale
    ou, ov = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    off, col = O.build_sets(nv, ou, ov)
    with ctx.kronecker(scale, 16, seed) as g:
        goff, gcol = g.csr()
        assert same_sets(off, col, goff, gcol)
        roots = g.sample_roots(8, seed=3)
        assert len(set(roots.tolist())) == 8
        for r in roots:
            assert off[r + 1] > off[r]
            check_against_oracle(g, nv, off, col, int(r), ou, ov, mr=(scale <= 12))
        dirs = g.level_dirs()
        assert len(dirs) > 0


@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("order", ["id", "degree"])
def test_row_order_option(ctx, order, relabel):
    """Rows in id order are sorted ascending; both orders give identical distances.  Degree order:
    relabel off sorts each row by neighbour degree (after dedup); relabel on (the default) renumbers the
    vertices by tuple-endpoint degree (duplicates counted, ties by id), so a row ascending in internal
    ids is that order -- the exported CSR (original ids) shows it row by row."""
    seed, scale = 77, 12
    ou, ov = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    off, col = O.build_sets(nv, ou, ov)
    ctx.set_option("row_order", order)
    ctx.set_option("relabel", relabel)
    try:
        with ctx.kronecker(scale, 16, seed) as g:
            goff, gcol = g.csr()
            if order == "id":
                assert np.array_equal(gcol, col)
            else:
                assert same_sets(off, col, goff, gcol)
                if relabel == "off":
                    key = np.diff(off).astype(np.int64) * nv  # dedup degree; ties in any order
                    tie = np.zeros(nv, np.int64)
                else:
                    raw = np.bincount(ou, minlength=nv) + np.bincount(ov[ov != ou], minlength=nv)
                    key = raw.astype(np.int64) * nv
                    tie = np.arange(nv, dtype=np.int64)  # equal raw degree: ascending id
                for x in range(0, nv, 97):  # non-increasing (degree, -id) inside a row
                    r = gcol[goff[x]:goff[x + 1]]
                    assert np.all(np.diff(key[r] - tie[r]) <= 0) if relabel == "on" else \
                        np.all(np.diff(key[r]) <= 0)
            r = int(g.sample_roots(1, seed=9)[0])
            check_against_oracle(g, nv, off, col, r, ou, ov)
    finally:
        ctx.set_option("row_order", "degree")
        ctx.set_option("relabel", "on")


@pytest.mark.parametrize("blocks", ["auto", "3"])
@pytest.mark.parametrize("case", ["path", "grid", "kron", "lollipop"])
def test_persistent_topdown_matches_per_level_kernels(ctx, case, blocks):
    """K3p (narrow frontiers, many levels per launch) against the per-level kernels and the oracle:
    identical distances, level counts, per-level frontier sizes, monotone level times; two sources per
    graph (the barrier counters carry over between launches).  blocks: K3p workgroups (auto = three per four CUs;
    3 = uneven slices, several steps per slice).  lollipop: a path into a 20000-leaf star, whose hub
    must hand back to the per-level kernels (a slice could overflow its output segment)."""
    if case == "path":
        nv = 5000
        u, v = np.arange(nv - 1), np.arange(1, nv)          # 5000 levels: five K3p launches
    elif case == "grid":
        side = 120
        idx = np.arange(side * side).reshape(side, side)
        u = np.r_[idx[:, :-1].ravel(), idx[:-1, :].ravel()]
        v = np.r_[idx[:, 1:].ravel(), idx[1:, :].ravel()]
        nv = side * side
    elif case == "lollipop":
        plen, leaves = 300, 20000
        nv = plen + leaves
        u = np.r_[np.arange(plen - 1), np.full(leaves, plen - 1), np.arange(plen, plen + 50)]
        v = np.r_[np.arange(1, plen), np.arange(plen, nv), np.arange(plen + 1, plen + 51)]
    else:
        u, v = O.kronecker(14, 16, 99)
        nv = 1 << 14
    u = np.asarray(u, np.uint32)
    v = np.asarray(v, np.uint32)
    off, col = O.build_sets(nv, u, v)
    srcs = [int(u[0]), int(v[len(v) // 2])]
    refs = [O.csr_bfs(nv, off, col, s)[0] for s in srcs]
    res = {}
    try:
        ctx.set_option("persist_blocks", blocks)
        for mode in ("off", "on"):
            ctx.set_option("persist", mode)
            with ctx.from_edges(nv, u, v) as g:
                for src, ref in zip(srcs, refs):
                    d, p, st = g.bfs(src)
                    assert np.array_equal(d, ref)
                    assert O.validate(nv, off, col, src, d, p) == 0
                    t = g.level_times()
                    assert len(t) == st["levels"] and np.all(np.diff(t) >= 0)
                    res[mode, src] = [(l["direction"], l["frontier_in"], l["frontier_out"])
                                      for l in g.level_stats(1 << 14)]
    finally:
        ctx.set_option("persist", "on")
        ctx.set_option("persist_blocks", "auto")
    for src in srcs:
        assert res["on", src] == res["off", src]


@pytest.mark.parametrize("persist", ["off", "on"])
def test_push_log_matches_state_stores(ctx, persist):
    """push_log (per-level push winners as (vertex, parent) pairs at their queue positions, scattered into the
    state when the result is read) against the packed-state stores: identical distances and a valid parent
    tree, through every reader of the result -- bfsx_bfs's arrays, bfsx_result after another BFS ran, the
    device validator and m_comp -- on a Kronecker graph (hub-bin push levels, pull levels, hybrid levels) and
    a grid (many narrow push levels; persist off puts them all in the per-level kernels)."""
    cases = []
    u, v = O.kronecker(14, 16, 7)
    cases.append((1 << 14, np.asarray(u, np.uint32), np.asarray(v, np.uint32)))
    side = 90
    idx = np.arange(side * side).reshape(side, side)
    cases.append((side * side, np.r_[idx[:, :-1].ravel(), idx[:-1, :].ravel()].astype(np.uint32),
                  np.r_[idx[:, 1:].ravel(), idx[1:, :].ravel()].astype(np.uint32)))
    try:
        ctx.set_option("persist", persist)
        for nv, u, v in cases:
            off, col = O.build_sets(nv, u, v)
            srcs = [int(u[0]), int(v[len(v) // 3]), int(u[-1])]
            refs = [O.csr_bfs(nv, off, col, s)[0] for s in srcs]
            for mode in ("off", "on"):
                ctx.set_option("push_log", mode)
                with ctx.from_edges(nv, u, v) as g:
                    for src, ref in zip(srcs, refs):
                        d, p, st = g.bfs(src)
                        assert np.array_equal(d, ref), (mode, src)
                        assert O.validate(nv, off, col, src, d, p) == 0
                        assert g.validate()["errors"] == 0
                    # the result of the last BFS read again, after the validator resolved it
                    d2, p2 = g.result()
                    assert np.array_equal(d2, refs[-1]) and np.array_equal(p2, p)
    finally:
        ctx.set_option("push_log", "on")
        ctx.set_option("persist", "on")


@pytest.mark.parametrize("hybrid", ["auto", "force"])
def test_vis_front_matches_copy(ctx, hybrid):
    """Round 6, option vis_front: the dense pull level after a push, hybrid or K3p level reads the visited bitmap
    itself as its frontier and writes the updated bitmap into a second buffer (the loop swaps the two); off, it
    reads a copy (K3p's first launch leaves that copy with persist_front, or the loop copies).  Both against the
    oracle, with identical directions and per-level counts, a valid tree, the device validator and a second read of
    the result -- on a Kronecker graph (K3p, hub-bin push, pull and sparse pull levels; forced hybrid levels in the
    second case) and a lollipop (a long path: the K3p launch that stops for a pull comes late)."""
    cases = []
    u, v = O.kronecker(14, 16, 11)
    cases.append((1 << 14, np.asarray(u, np.uint32), np.asarray(v, np.uint32)))
    plen, leaves = 200, 30000
    cases.append((plen + leaves,
                  np.r_[np.arange(plen - 1), np.full(leaves, plen - 1)].astype(np.uint32),
                  np.r_[np.arange(1, plen), np.arange(plen, plen + leaves)].astype(np.uint32)))
    try:
        ctx.set_option("hybrid", hybrid)
        for nv, u, v in cases:
            off, col = O.build_sets(nv, u, v)
            srcs = [int(u[0]), int(v[len(v) // 2]), int(u[-1])]
            refs = [O.csr_bfs(nv, off, col, s)[0] for s in srcs]
            levels = {}
            for mode in ("off", "on"):
                for pf in ("off", "on"):
                    ctx.set_option("vis_front", mode)
                    ctx.set_option("persist_front", pf)
                    with ctx.from_edges(nv, u, v) as g:
                        for src, ref in zip(srcs, refs):
                            d, p, st = g.bfs(src)
                            assert np.array_equal(d, ref), (mode, pf, src)
                            assert O.validate(nv, off, col, src, d, p) == 0
                            assert g.validate()["errors"] == 0
                            levels[mode, pf, src] = [(l["direction"], l["frontier_in"], l["frontier_out"])
                                                     for l in g.level_stats(1 << 14)]
                        d2, _ = g.result()
                        assert np.array_equal(d2, refs[-1])
            for src in srcs:
                assert levels["on", "on", src] == levels["off", "on", src] == levels["off", "off", src] == \
                    levels["on", "off", src], src
    finally:
        ctx.set_option("vis_front", "on")
        ctx.set_option("persist_front", "on")
        ctx.set_option("hybrid", "auto")


@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("direction", ["auto", "bottomup"])
def test_provenance_codes_every_reader(ctx, relabel, direction):
    """Round 5: a pull level stores a 1-B provenance code per discovery (0: top1, 1-3: rest.x/y/z, 4: the
    explicit 4-B parent) instead of the parent itself.  Every reader must decode it to the same tree: the unpack
    read FIRST (k_unpack_live with the original-id copies of top1 / rest, relabel on; k_unpack's scatter form,
    relabel off), then the device validator and m_comp (bfs_resolve folds the records into st lazily), then the
    unpack again from the folded state.  A 160x160 grid pulled from level 0 has more than kMaxRec (32) pull levels,
    so its records are folded mid-BFS (RecLog::take) as well."""
    cases = []
    u, v = O.kronecker(14, 16, 21)
    cases.append((1 << 14, np.asarray(u, np.uint32), np.asarray(v, np.uint32)))
    side = 160
    idx = np.arange(side * side).reshape(side, side)
    cases.append((side * side, np.r_[idx[:, :-1].ravel(), idx[:-1, :].ravel()].astype(np.uint32),
                  np.r_[idx[:, 1:].ravel(), idx[1:, :].ravel()].astype(np.uint32)))
    ctx.set_option("relabel", relabel)
    ctx.set_option("direction", direction)
    try:
        for nv, u, v in cases:
            off, col = O.build_sets(nv, u, v)
            srcs = [int(u[0]), int(v[len(v) // 2]), int(u[-1])]
            with ctx.from_edges(nv, u, v) as g:
                for src in srcs:
                    ref = O.csr_bfs(nv, off, col, src)[0]
                    g.bfs_device_only(src)
                    d, p = g.result()  # first reader: the unpack decodes the codes
                    assert np.array_equal(d, ref), (relabel, direction, src)
                    assert O.validate(nv, off, col, src, d, p) == 0
                    val = g.validate()  # folds the records into st
                    assert val["errors"] == 0 and val["reached"] == int((ref != INF).sum())
                    d2, p2 = g.result()  # again, from the folded state
                    assert np.array_equal(d2, d) and np.array_equal(p2, p)
                _, _, st = g.bfs(srcs[0])
                ref = O.csr_bfs(nv, off, col, srcs[0])[0]
                assert st["m_comp"] == O.mcomp(u, v, ref)
                # the bytes accounting's counter: explicit parents only where a discovery needed one
                ls = g.level_stats()
                assert all(0 <= l["explicit_parents"] <= l["frontier_out"] for l in ls)
                assert all(l["explicit_parents"] == 0 for l in ls if l["direction"] == 1)
                pulled = [l for l in ls if l["direction"] in (2, 4)]
                if nv == side * side and direction == "bottomup":  # rows of <= 4 entries: codes only
                    assert pulled and sum(l["explicit_parents"] for l in pulled) == 0
                if nv == 1 << 14 and direction == "bottomup":  # Kronecker rows walked past their 4th entry
                    assert sum(l["explicit_parents"] for l in pulled) > 0
    finally:
        ctx.set_option("relabel", "on")
        ctx.set_option("direction", "auto")


@pytest.mark.parametrize("skip", ["on", "off"])
@pytest.mark.parametrize("direction", ["auto", "topdown"])
def test_hub_lds_skip_option(ctx, skip, direction):
    """Round 5, option hub_lds_skip: the hub bin (k_td_hubs) of a relabelled graph snapshots the visited bits of
    the 2^16 lowest ids into LDS at the level's start and probes no target the snapshot marks.  Forced push
    levels from hub roots run the hub bin with most of a level's edges pointing at earlier-visited hubs; a
    small hub degree puts many rows into the bin.  Distances against the oracle, trees valid, on and off."""
    ctx.set_option("hub_lds_skip", skip)
    ctx.set_option("direction", direction)
    ctx.set_option("hub_degree", 16)
    try:
        for scale, seed in ((14, 31), (16, 8)):
            ou, ov = O.kronecker(scale, 16, seed)
            nv = 1 << scale
            off, col = O.build_sets(nv, ou, ov)
            deg = np.diff(off)
            with ctx.kronecker(scale, 16, seed) as g:
                roots = [int(np.argmax(deg))] + [int(r) for r in g.sample_roots(3, seed=5)]
                for r in roots:
                    check_against_oracle(g, nv, off, col, r, ou, ov, mr=False)
    finally:
        ctx.set_option("hub_lds_skip", "on")
        ctx.set_option("direction", "auto")
        ctx.set_option("hub_degree", 64)


@pytest.mark.diag
@pytest.mark.parametrize("abort_at", [0, 3])
def test_persistent_abort_falls_back(ctx, abort_at):
    """A K3p launch whose grid barrier gives up (here: the "persist_abort_at" hook, the same exit path a
    barrier timeout takes when another context holds CUs) makes every workgroup exit; the BFS is re-run
    without K3p and still returns the oracle's distances (no random failures from co-residency)."""
    nv = 3000
    u, v = np.arange(nv - 1, dtype=np.uint32), np.arange(1, nv, dtype=np.uint32)  # one long K3p launch
    off, col = O.build_sets(nv, u, v)
    ref, _ = O.csr_bfs(nv, off, col, 0)
    try:
        ctx.set_option("persist_abort_at", str(abort_at))
        with ctx.from_edges(nv, u, v) as g:
            for _ in range(2):  # the barrier counters are reset after an abort
                d, p, st = g.bfs(0)
                assert st["persist_retries"] == 1
                assert np.array_equal(d, ref)
                assert O.validate(nv, off, col, 0, d, p) == 0
                assert st["levels"] == nv
        ctx.set_option("persist_abort_at", "off")
        with ctx.from_edges(nv, u, v) as g:
            d, _, st = g.bfs(0)
            assert st["persist_retries"] == 0 and np.array_equal(d, ref)
    finally:
        ctx.set_option("persist_abort_at", "off")


@pytest.mark.diag
def test_persistent_abort_time_covers_both_attempts(ctx):
    """t_bfs of a BFS whose K3p launch aborted covers the aborted attempt AND the re-run (round-3 verdict: the
    re-run re-recorded the start event, so the aborted attempt's time fell out of t_bfs).  A 1,100-vertex path:
    the launch aborts after 1,000 K3p levels (persist_abort_at), the re-run takes per-level launches; t_bfs must
    exceed the per-level run alone (persist off) by about the 1,000 K3p levels' span.  The graph counts the
    re-run in bfsx_persist_fallbacks (what bench.py reports over its timed loop)."""
    nv = 1100
    u, v = np.arange(nv - 1, dtype=np.uint32), np.arange(1, nv, dtype=np.uint32)
    try:
        with ctx.from_edges(nv, u, v) as g:
            g.bfs_device_only(0)
            k3p = g.level_times()[999]  # the first 1,000 levels inside K3p: the aborted attempt's share
            ctx.set_option("persist", "off")
            t_off = min(g.bfs_device_only(0) for _ in range(3))
            ctx.set_option("persist", "on")
            ctx.set_option("persist_abort_at", "1000")
            f0 = g.persist_fallbacks()
            t_ab = [g.bfs_device_only(0) for _ in range(3)]
            assert g.persist_fallbacks() - f0 == 3
            assert min(t_ab) > t_off + 0.5 * k3p, (t_ab, t_off, k3p)
    finally:
        ctx.set_option("persist_abort_at", "off")
        ctx.set_option("persist", "on")


def test_persist_blocks_changed_between_runs(ctx):
    """persist_blocks raised after a graph's first K3p launch: the launch keeps the grid it was set up
    with, and the entry bound (every slice fits its output segment) is checked against THAT grid."""
    # root 0 -> 1000 children -> 40 leaves each: the second frontier (1000 vertices of degree 41) fits a
    # 192-workgroup (auto) grid's segments (6 x 41 entries) but not a 2-workgroup grid's (500 x 40 discoveries)
    kids, fan = 1000, 40
    nv = 1 + kids + kids * fan
    child = np.arange(1, kids + 1)
    u = np.r_[np.zeros(kids), np.repeat(child, fan)].astype(np.uint32)
    v = np.r_[child, np.arange(kids + 1, nv)].astype(np.uint32)
    plen = kids
    off, col = O.build_sets(nv, u, v)
    ref, _ = O.csr_bfs(nv, off, col, 0)
    try:
        ctx.set_option("direction", "topdown")  # push levels only, so the wide level is a K3p candidate
        ctx.set_option("persist_blocks", "2")
        with ctx.from_edges(nv, u, v) as g:
            d, _, st = g.bfs(0)
            assert np.array_equal(d, ref)
            ctx.set_option("persist_blocks", "auto")
            for src in (0, plen - 2):
                d, p, st = g.bfs(src)
                r2, _ = O.csr_bfs(nv, off, col, src)
                assert np.array_equal(d, r2) and st["persist_retries"] == 0
                assert O.validate(nv, off, col, src, d, p) == 0
    finally:
        ctx.set_option("persist_blocks", "auto")
        ctx.set_option("direction", "auto")


@pytest.mark.parametrize("bits", ["auto", "64"])
def test_offset_width_paths(ctx, bits):
    """uint32 and int64 row-offset instantiations of every traversal kernel agree with the oracle (int64
    is what graphs with >= 2^32 adjacency entries run; forced here on a small graph)."""
    scale, seed = 14, 4242
    ou, ov = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    off, col = O.build_sets(nv, ou, ov)
    ctx.set_option("offset_bits", bits)
    try:
        for direction in ("auto", "topdown", "bottomup"):
            ctx.set_option("direction", direction)
            with ctx.kronecker(scale, 16, seed) as g:
                for r in g.sample_roots(3, seed=5):
                    check_against_oracle(g, nv, off, col, int(r), ou, ov, mr=False)
    finally:
        ctx.set_option("offset_bits", "auto")
        ctx.set_option("direction", "auto")


def test_kronecker_scale20_validated(ctx):
    """Full-size-style property check: Graph500 validation + oracle distances at scale 20."""
    scale = 20
    with ctx.kronecker(scale, 16, 0x5EED2026) as g:
        nv = g.nv
        off, col = g.csr()
        col = sort_rows(off, col)
        for r in g.sample_roots(4, seed=11):
            d, p, st = g.bfs(int(r))
            ref, _ = O.csr_bfs(nv, off, col, int(r))
            assert np.array_equal(d, ref)
            assert O.validate(nv, off, col, int(r), d, p) == 0
            assert st["bottomup_levels"] > 0  # direction optimisation engaged
            assert st["t_bfs_ms"] > 0


def test_errors(ctx, bfsx):
    with pytest.raises(bfsx.BfsxError) as ei:
        ctx.load_algs4("/nonexistent.txt")
    assert ei.value.code == bfsx.BFSX_E_IO
    with ctx.from_edges(10, np.array([1], np.uint32), np.array([2], np.uint32)) as g:
        with pytest.raises(bfsx.BfsxError) as ei:
            g.bfs(10)
        assert ei.value.code == bfsx.BFSX_E_RANGE
    with pytest.raises(bfsx.BfsxError) as ei:
        ctx.from_edges(10, np.array([1], np.uint32), np.array([10], np.uint32))
    assert ei.value.code == bfsx.BFSX_E_RANGE
    with pytest.raises(bfsx.BfsxError):
        ctx.set_option("direction", "sideways")


def test_repeated_bfs_reuses_state(ctx):
    path = os.path.join(GOLDEN, "mediumG.txt")
    with ctx.load_algs4(path) as g:
        d0, _, _ = g.bfs(0)
        for s in (5, 77, 249, 0):
            d, p, _ = g.bfs(s)
        assert np.array_equal(d, d0)
        d2, p2 = g.result()
        assert np.array_equal(d2, d0)


@pytest.mark.diag
@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("bits", ["off", "1", "6", "12", "30"])
@pytest.mark.parametrize("direction", ["auto", "bottomup"])
def test_hub_probe_domain(ctx, bits, direction, relabel):
    """Hub sets of every size (option hub_bits: the 2^b highest-degree vertices; 30 = every vertex is a
    hub, 1 = two hubs): relabel off = k_bu's hub-encoded probe domain (a dense second id per hub); relabel
    on = ids below a limit.  Distances bit-exact and parents valid on edge-case graphs and scale 14."""
    cases = [c for c in random_cases() if c[0] in ("rand3", "star", "multi_hub", "two_comp", "isolated", "dups")]
    ctx.set_option("hub_bits", bits)
    ctx.set_option("direction", direction)
    ctx.set_option("relabel", relabel)
    try:
        for name, nv, u, v in cases:
            u = np.asarray(u, np.uint32)
            v = np.asarray(v, np.uint32)
            off, col = O.build_sets(nv, u, v)
            with ctx.from_edges(nv, u, v) as g:
                for s in sorted({0, nv - 1, nv // 2}):
                    check_against_oracle(g, nv, off, col, s, u, v, mr=False)
                    assert g.validate()["errors"] == 0
        ou, ov = O.kronecker(14, 16, 0x5EED2026)
        off, col = O.build_sets(1 << 14, ou, ov)
        with ctx.kronecker(14, 16, 0x5EED2026) as g:
            for r in g.sample_roots(3, seed=9):
                check_against_oracle(g, 1 << 14, off, col, int(r), ou, ov, mr=False)
    finally:
        ctx.set_option("hub_bits", "auto")
        ctx.set_option("direction", "auto")
        ctx.set_option("relabel", "on")


def raw_degree(nv, u, v):
    """Tuple-endpoint degree (duplicates counted, a self-loop once): the relabel's sort key."""
    u = np.asarray(u, np.int64)
    v = np.asarray(v, np.int64)
    return np.bincount(u, minlength=nv) + np.bincount(v[v != u], minlength=nv)


@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("chunk", ["1", "37", "5000"])
def test_chunked_csr_build(ctx, chunk, relabel):
    """The CSR build sorts/dedups/orders rows in chunks of `build_chunk` raw entries, compacting in place
    (what lets scale 30 build on one device).  Tiny chunks (1 = one row per chunk, rows longer than the
    chunk, chunk edges inside duplicate runs) must give the same neighbour sets and degree order."""
    cases = [c for c in random_cases() if c[0] in ("rand0", "rand5", "star", "dups", "self_loops", "isolated")]
    ctx.set_option("build_chunk", chunk)
    ctx.set_option("relabel", relabel)
    try:
        for name, nv, u, v in cases:
            u = np.asarray(u, np.uint32)
            v = np.asarray(v, np.uint32)
            off, col = O.build_sets(nv, u, v)
            with ctx.from_edges(nv, u, v) as g:
                goff, gcol = g.csr()
                assert same_sets(off, col, goff, gcol), name
                # degree-descending order inside every row (ties by id): the dedup degree, or with the
                # relabel the tuple-endpoint degree it sorts by
                deg = np.diff(goff) if relabel == "off" else raw_degree(nv, u, v)
                rows = np.repeat(np.arange(nv), np.diff(goff))
                key = np.lexsort((gcol, -deg[gcol], rows))
                assert np.array_equal(gcol[key], gcol), name
                check_against_oracle(g, nv, off, col, 0, u, v, mr=False)
        ou, ov = O.kronecker(12, 16, 0x5EED2026)
        off, col = O.build_sets(1 << 12, ou, ov)
        with ctx.kronecker(12, 16, 0x5EED2026) as g:
            goff, gcol = g.csr()
            assert same_sets(off, col, goff, gcol)
    finally:
        ctx.set_option("build_chunk", str(1 << 30))
        ctx.set_option("relabel", "on")


@pytest.mark.diag
@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("unroll", ["2", "4", "4-nopipe", "4-noprefix"])
def test_bottomup_unroll_variants(ctx, unroll, relabel):
    """Every k_bu instantiation (2 or 4 candidates per lane per round; with 4, the next round's top1
    loads pipelined or not; the LDS copy of the hub prefix's frontier bits on or off) is bit-exact,
    pull-only and direction-optimising, with and without hubs."""
    ctx.set_option("bu_unroll", unroll.split("-")[0])
    ctx.set_option("bu_pipeline", "off" if unroll.endswith("nopipe") else "on")
    ctx.set_option("bu_lds_prefix", "off" if unroll.endswith("noprefix") else "on")
    ctx.set_option("relabel", relabel)
    try:
        for hub in ("off", "auto"):
            ctx.set_option("hub_bits", hub)
            for direction in ("bottomup", "auto"):
                ctx.set_option("direction", direction)
                for name, nv, u, v in [c for c in random_cases() if c[0] in ("rand2", "multi_hub", "path")]:
                    u = np.asarray(u, np.uint32)
                    v = np.asarray(v, np.uint32)
                    off, col = O.build_sets(nv, u, v)
                    with ctx.from_edges(nv, u, v) as g:
                        check_against_oracle(g, nv, off, col, 0, u, v, mr=False)
                ou, ov = O.kronecker(16, 16, 0x5EED2026)
                off, col = O.build_sets(1 << 16, ou, ov)
                with ctx.kronecker(16, 16, 0x5EED2026) as g:
                    for r in g.sample_roots(2, seed=4):
                        check_against_oracle(g, 1 << 16, off, col, int(r), ou, ov, mr=False)
    finally:
        for k, val in (("bu_unroll", "4"), ("bu_pipeline", "on"), ("relabel", "on"), ("hub_bits", "auto"),
                       ("direction", "auto"), ("bu_lds_prefix", "on")):
            ctx.set_option(k, val)


@pytest.mark.diag
@pytest.mark.parametrize("relabel", ["on", "off"])
@pytest.mark.parametrize("bits", ["2", "6", "30"])
def test_hybrid_levels(ctx, bits, relabel):
    """Hybrid levels (pull from the frontier's hubs + push from its other vertices; option hybrid=force
    runs every top-down level whose frontier holds a hub that way): bit-exact distances, valid parents
    and the same pass count, whatever the hub count (30 = every vertex is a hub: the push half is empty;
    2 = four hubs: most of the frontier is pushed)."""
    ctx.set_option("hub_bits", bits)
    ctx.set_option("relabel", relabel)
    ctx.set_option("hybrid", "force")
    ctx.set_option("persist", "off")  # every level through the per-level loop (persist=on is covered below)
    try:
        hy = 0
        for name, nv, u, v in [c for c in random_cases() if c[0] in ("rand1", "rand4", "star", "multi_hub",
                                                                      "two_comp", "self_loops")]:
            u = np.asarray(u, np.uint32)
            v = np.asarray(v, np.uint32)
            off, col = O.build_sets(nv, u, v)
            with ctx.from_edges(nv, u, v) as g:
                for s in sorted({0, nv // 2, nv - 1}):
                    check_against_oracle(g, nv, off, col, s, u, v, mr=False)
                    assert g.validate()["errors"] == 0
                    hy += sum(1 for d in g.level_dirs() if d == 3)
        # leaf-heavy: 40 hubs on a ring, each with 300 degree-1 feet and links to 8 other hubs (the
        # frontier after a hub level is almost all leaves, the case round 1's leaf filter faulted on)
        rng = np.random.default_rng(77)
        hubs = np.arange(40)
        feet_u = np.repeat(hubs, 300)
        feet_v = 40 + np.arange(40 * 300)
        hl_u = np.repeat(hubs, 8)
        hl_v = rng.integers(0, 40, hl_u.size)
        u = np.concatenate([feet_u, hl_u, hubs]).astype(np.uint32)
        v = np.concatenate([feet_v, hl_v, (hubs + 1) % 40]).astype(np.uint32)
        nv = 40 + 40 * 300
        off, col = O.build_sets(nv, u, v)
        with ctx.from_edges(nv, u, v) as g:
            for s in (0, 41, nv - 1):
                check_against_oracle(g, nv, off, col, s, u, v, mr=False)
                assert g.validate()["errors"] == 0
                hy += sum(1 for d in g.level_dirs() if d == 3)
        ou, ov = O.kronecker(14, 16, 0x5EED2026)
        off, col = O.build_sets(1 << 14, ou, ov)
        for persist in ("off", "on"):
            ctx.set_option("persist", persist)
            with ctx.kronecker(14, 16, 0x5EED2026) as g:
                for r in g.sample_roots(4, seed=21):
                    check_against_oracle(g, 1 << 14, off, col, int(r), ou, ov, mr=False)
                    hy += sum(1 for d in g.level_dirs() if d == 3)
        assert hy > 0, "no hybrid level ran"
    finally:
        ctx.set_option("hub_bits", "auto")
        ctx.set_option("hybrid", "auto")
        ctx.set_option("persist", "on")
        ctx.set_option("relabel", "on")


@pytest.mark.parametrize("direction", ["topdown", "auto", "bottomup"])
def test_degree_one_vertices(ctx, direction):
    """k_td gives a discovered degree-1 vertex an empty row (its one neighbour is its parent).  The
    source itself is never skipped: BFS from a degree-1 source (a path's end, a star's leaf, a
    caterpillar's foot) reaches everything, with the oracle's distances, valid parents and pass count."""
    ctx.set_option("direction", direction)
    try:
        n = 3000
        path_u = np.arange(n - 1, dtype=np.uint32)
        star_u = np.zeros(n - 1, np.uint32)
        # caterpillar: a spine 0..999, every spine vertex with two feet
        spine = np.arange(999, dtype=np.uint32)
        feet = np.arange(1000, 3000, dtype=np.uint32)
        cat_u = np.concatenate([spine, (feet - 1000) // 2]).astype(np.uint32)
        cat_v = np.concatenate([spine + 1, feet]).astype(np.uint32)
        cases = [("path", path_u, path_u + 1, [0, n - 1]), ("star", star_u, np.arange(1, n, dtype=np.uint32), [7, 0]),
                 ("caterpillar", cat_u, cat_v, [1000, 2999, 0])]
        for name, u, v, sources in cases:
            off, col = O.build_sets(n, u, v)
            with ctx.from_edges(n, u, v) as g:
                for s in sources:
                    assert off[s + 1] - off[s] == 1 or name == "star" or s == 0
                    check_against_oracle(g, n, off, col, s, u, v, mr=False)
    finally:
        ctx.set_option("direction", "auto")


def test_leaf_skip(ctx):
    """Leaf skip (single device): a pull level's discoveries at ids >= leaf_lo (rows of one entry: the
    relabelled graph's degree-1 tail) stay out of the next push level's queue -- their one neighbour is
    their parent.  The pull kernel counts the others, so every later consumer of the queue (k_td, K3p,
    a hybrid level's queue -> bitmap) sees the shortened length; round 1's leaf filter faulted because
    consumers kept the unfiltered count.  Distances, pass counts and parents against the oracle, with the
    option on and off, on (a) a graph whose pull level hands a push level a frontier of leaves only
    (the push level's queue is empty and the pass still counts), (b) Kronecker graphs over many roots,
    with and without K3p and hybrid levels."""
    # (a) s - h - c_i (3,000) ; c_i - leaf_i for i < 1,000 ; 100,000 isolated ids (n/24 above 3,000)
    s, h = 0, 1
    c = 2 + np.arange(3000)
    lv = 3002 + np.arange(1000)
    u = np.r_[[s], np.full(3000, h), c[:1000]].astype(np.uint32)
    v = np.r_[[h], c, lv].astype(np.uint32)
    nv = 4002 + 100000
    off, col = O.build_sets(nv, u, v)
    try:
        for skip in ("on", "off"):
            ctx.set_option("leaf_skip", skip)
            with ctx.from_edges(nv, u, v) as g:
                _, _, st = check_against_oracle(g, nv, off, col, s, u, v, mr=False)
                assert st["levels"] == 4
                ls = g.level_stats()
                # the second pull level (1,000 leaves left) runs in the sparse pull kernel (direction 4)
                assert [x["direction"] for x in ls] == [1, 2, 4, 1], ls
                if skip == "on":
                    assert ls[3]["frontier_in"] == 0  # the leaves stayed out of the queue
                else:
                    assert ls[3]["frontier_in"] == 1000
        # (b) Kronecker: identical results with and without the skip, across K3p / hybrid settings
        ou, ov = O.kronecker(16, 16, 0x1EAF)
        nv = 1 << 16
        off, col = O.build_sets(nv, ou, ov)
        shortened = 0
        for persist, hybrid in (("on", "auto"), ("off", "auto"), ("on", "force")):
            ctx.set_option("persist", persist)
            ctx.set_option("hybrid", hybrid)
            res = {}
            for skip in ("off", "on"):
                ctx.set_option("leaf_skip", skip)
                with ctx.kronecker(16, 16, 0x1EAF) as g:
                    roots = [int(r) for r in g.sample_roots(12, seed=5)]
                    for r in roots:
                        d, p, st = g.bfs(r)
                        res.setdefault(r, []).append((d, st["levels"], g.level_stats()))
                        assert O.validate(nv, off, col, r, d, p) == 0
            for r, ((d0, l0, s0), (d1, l1, s1)) in res.items():
                assert np.array_equal(d0, d1) and l0 == l1
                shortened += sum(1 for a, b in zip(s0, s1) if b["frontier_in"] < a["frontier_in"])
            ref, _ = O.csr_bfs(nv, off, col, roots[0])
            assert np.array_equal(res[roots[0]][0][0], ref)
        assert shortened > 0  # the skip applied somewhere
    finally:
        ctx.set_option("persist", "on")
        ctx.set_option("hybrid", "auto")
        ctx.set_option("leaf_skip", "on")


@pytest.mark.diag
@pytest.mark.parametrize("floor", ["0", "65536"])
@pytest.mark.parametrize("direction", ["auto", "bottomup"])
@pytest.mark.parametrize("sparse", ["1", "64", "off"])
def test_sparse_pull_levels(ctx, direction, sparse, floor):
    """The sparse pull kernel (k_bu_sparse, direction 4 in the level records): bu_sparse=1 runs EVERY pull
    level in it, 64 (the default) the tail levels, off none.  Distances, pass counts and parents against the
    oracle over 10 Kronecker roots, the queues poisoned (the push level after a sparse one reads the queue
    the sparse kernel wrote), with and without the leaf skip."""
    ou, ov = O.kronecker(15, 16, 0x5A5E)
    nv = 1 << 15
    off, col = O.build_sets(nv, ou, ov)
    seen = 0
    try:
        ctx.set_option("direction", direction)
        ctx.set_option("bu_sparse", sparse)
        ctx.set_option("poison_queues", "on")
        ctx.set_option("pull_min_edges", floor)
        for skip in ("on", "off"):
            ctx.set_option("leaf_skip", skip)
            with ctx.kronecker(15, 16, 0x5A5E) as g:
                for r in g.sample_roots(10, seed=11):
                    check_against_oracle(g, nv, off, col, int(r), ou, ov, mr=False)
                    seen += sum(1 for d in g.level_dirs() if d == 4)
        if sparse == "off":
            assert seen == 0
        elif floor == "0" or direction == "bottomup":
            assert seen > 0
    finally:
        for k, val in (("direction", "auto"), ("bu_sparse", "64"), ("poison_queues", "off"), ("leaf_skip", "on"),
                       ("pull_min_edges", "0")):
            ctx.set_option(k, val)


def _star_of_hubs(nhub, fan, tail):
    """Source 0 -> nhub hubs; hub i -> its own `fan` leaves, plus a path of `tail` vertices hanging off
    the last leaf (a few narrow levels after the heavy ones)."""
    hubs = 1 + np.arange(nhub)
    leaves = 1 + nhub + np.arange(nhub * fan)
    u = [np.zeros(nhub), np.repeat(hubs, fan)]
    v = [hubs, leaves]
    last = int(leaves[-1])
    p = last + 1 + np.arange(tail)
    u.append(np.r_[[last], p[:-1]])
    v.append(p)
    nv = int(p[-1]) + 1
    return nv, np.concatenate(u).astype(np.uint32), np.concatenate(v).astype(np.uint32)


@pytest.mark.diag
@pytest.mark.parametrize("floor", ["0", "65536"])
@pytest.mark.parametrize("dmax", ["2048", "64", "8"])
def test_persistent_heavy_rows(ctx, dmax, floor):
    """K3p's heavy rows (round 3): a row longer than persist_dmax is swept by the whole grid at the next
    level (equal edge shares); the source enters as one.  Bit-exact against the oracle and against the
    per-level kernels (persist off): a source of 6,000 hubs (every workgroup's heavy region overflows at
    dmax 8, and the heavy table exceeds its 1,024 rows), a source of 40 hubs of 3,000 leaves (heavy rows at
    level 1, inside the launch), and Kronecker roots."""
    cases = [_star_of_hubs(6000, 12, 30), _star_of_hubs(40, 3000, 30)]
    ou, ov = O.kronecker(15, 16, 0x4EA7)
    try:
        ctx.set_option("persist_dmax", dmax)
        ctx.set_option("direction", "topdown")  # push levels only: every narrow level is a K3p candidate
        ctx.set_option("poison_queues", "on")
        ctx.set_option("pull_min_edges", floor)
        for nv, u, v in cases:
            off, col = O.build_sets(nv, u, v)
            with ctx.from_edges(nv, u, v) as g:
                for s in (0, 1, nv - 1):
                    d, _, st = check_against_oracle(g, nv, off, col, s, u, v, mr=False)
                    assert st["persist_retries"] == 0
        nv = 1 << 15
        off, col = O.build_sets(nv, ou, ov)
        for direction in ("topdown", "auto"):
            ctx.set_option("direction", direction)
            with ctx.kronecker(15, 16, 0x4EA7) as g:
                for r in g.sample_roots(8, seed=21):
                    _, _, st = check_against_oracle(g, nv, off, col, int(r), ou, ov, mr=False)
                    assert st["persist_retries"] == 0
    finally:
        for k, val in (("persist_dmax", "512"), ("direction", "auto"), ("poison_queues", "off"),
                       ("pull_min_edges", "0")):
            ctx.set_option(k, val)


def test_pull_floor_default(ctx):
    """The default push -> pull floor (pull_min_edges = 2^16 frontier edges): a small graph's BFS stays push
    (no pull level at all, K3p runs it), a scale-16 Kronecker BFS still pulls (its frontier passes the floor),
    and both are bit-exact against the oracle; with the floor at 0 the small graph pulls again."""
    rng = np.random.default_rng(61)
    nv = 20000
    u = rng.integers(0, nv, 3 * nv).astype(np.uint32)
    v = rng.integers(0, nv, 3 * nv).astype(np.uint32)
    off, col = O.build_sets(nv, u, v)
    ou, ov = O.kronecker(16, 16, 0x5EED2026)
    koff, kcol = O.build_sets(1 << 16, ou, ov)
    try:
        ctx.set_option("pull_min_edges", "65536")
        with ctx.from_edges(nv, u, v) as g:
            check_against_oracle(g, nv, off, col, 0, u, v, mr=False)
            assert all(d == 1 for d in g.level_dirs())
        with ctx.kronecker(16, 16, 0x5EED2026) as g:
            r = int(g.sample_roots(1, seed=2)[0])
            check_against_oracle(g, 1 << 16, koff, kcol, r, ou, ov, mr=False)
            assert 2 in list(g.level_dirs())
        ctx.set_option("pull_min_edges", "0")
        with ctx.from_edges(nv, u, v) as g:
            check_against_oracle(g, nv, off, col, 0, u, v, mr=False)
            assert any(d in (2, 4) for d in g.level_dirs())
    finally:
        ctx.set_option("pull_min_edges", "0")


def test_level_stats_raw_matches(ctx):
    """bench.py's timed loop copies each BFS's level records raw (level_stats_raw) and decodes them after the
    timed region: the decoded records must equal level_stats()'s, including a cap below the level count."""
    with ctx.kronecker(14, 16, 0xA11) as g:
        for r in [int(x) for x in g.sample_roots(3, seed=5)]:
            g.bfs_device_only(r)
            full = g.level_stats()
            assert len(full) >= 2
            assert g.level_stats_decode(g.level_stats_raw(256)) == full
            assert g.level_stats_decode(g.level_stats_raw(1)) == full[:1]


def test_result_copy_isolated_sources_and_modes(ctx):
    """The result copy fills its staging once per mode and then skips isolated vertices (their entry stays
    unreached); an isolated SOURCE is written and reset by the next copy.  Alternating isolated / connected
    sources and the two copy modes (dist only: int32 staging; dist + parent: packed words) must always match the
    oracle, and a device-only materialisation in between must not disturb the next copy."""
    rng = np.random.default_rng(123)
    nv = 30000
    u = rng.integers(0, nv // 2, 4 * nv).astype(np.uint32)  # ids >= nv/2: isolated (most of them)
    v = rng.integers(0, nv // 2, 4 * nv).astype(np.uint32)
    u = np.r_[u, [nv - 7]].astype(np.uint32)  # a self-loop-only vertex
    v = np.r_[v, [nv - 7]].astype(np.uint32)
    off, col = O.build_sets(nv, u, v)
    with ctx.from_edges(nv, u, v) as g:
        for i, s in enumerate([nv - 1, 0, nv - 7, nv - 2, 5, nv - 1, 17]):
            ref, _ = O.csr_bfs(nv, off, col, s)
            if i % 3 == 2:
                g.bfs_device_only(s)
                g.unpack_device_only()
                d, p = g.result(want_parent=True)
            elif i % 3 == 1:
                d, p, _ = g.bfs(s, want_parent=False)
            else:
                d, p, _ = g.bfs(s)
            assert np.array_equal(d, ref), (i, s)
            if p is not None:
                assert O.validate(nv, off, col, s, d, p) == 0
