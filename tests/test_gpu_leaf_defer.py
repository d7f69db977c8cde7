"""Option leaf_defer (single device): the degree-1 tail of the id space (ids >= leaf_lo; on a relabelled graph
the vertices whose one neighbour is their only adjacency entry) stays out of the level loop and is resolved
from that neighbour after the last level, inside k_finalize.  The result must be the full BFS's: distances
bit-exact against the oracle's restatement of BfsSpark's loop (BfsSpark.java:66-117), the same pass count
(`iters`, ecc(source) + 1, including a last pass that reaches only deferred vertices), one level_times
entry per pass, a valid parent tree -- with the option on and off, in every direction mode, K3p on and off,
under poisoned queues."""
import numpy as np
import pytest

import oracle_py as O
from test_gpu_parity import check_against_oracle

pytestmark = pytest.mark.gpu
INF = 2147483647
DEFAULT = "off"  # the library default (include/bfsx.h)


def run_both(ctx, make, nv, off, col, sources, u=None, v=None, mr=True):
    """BFS every source with leaf_defer on and off; both against the oracle and against each other."""
    out = {}
    try:
        for mode in ("off", "on"):
            ctx.set_option("leaf_defer", mode)
            with make() as g:
                for s in sources:
                    d, p, st = check_against_oracle(g, nv, off, col, s, u, v, mr=mr)
                    t = g.level_times()
                    assert len(t) == st["levels"] and np.all(np.diff(t) >= 0)
                    dirs = list(g.level_dirs())
                    assert len(dirs) == st["levels"]
                    out[mode, s] = (d, st["levels"], dirs)
    finally:
        ctx.set_option("leaf_defer", DEFAULT)
    for s in sources:
        assert np.array_equal(out["on", s][0], out["off", s][0]) and out["on", s][1] == out["off", s][1]
    return out


def test_star_leaf_source_adds_a_leaves_pass(ctx):
    """A star: from a leaf the hub is at 1 and every other leaf at 2.  With the option on the core BFS ends
    after the hub's pass, and the last pass (distance 2, leaves only) is the BFSX_DIR_LEAVES record."""
    k = 50
    u = np.zeros(k, np.uint32)
    v = np.arange(1, k + 1, dtype=np.uint32)
    nv = k + 1
    off, col = O.build_sets(nv, u, v)
    out = run_both(ctx, lambda: ctx.from_edges(nv, u, v), nv, off, col, [0, 7, k], u, v)
    assert out["on", 7][1] == 3
    assert out["on", 7][2][-1] == 5  # BFSX_DIR_LEAVES
    assert 5 not in out["off", 7][2]


def test_two_vertex_components_and_isolated(ctx):
    """Edges whose both ends are leaves (the source's neighbour is itself deferred), a self-loop-only vertex,
    isolated ids, a path and a triangle with a tail."""
    pairs = [(0, 1), (2, 3), (4, 4), (10, 11), (11, 12), (12, 13), (13, 14), (20, 21), (21, 22), (22, 20), (22, 23),
             (23, 24)]
    u = np.array([a for a, _ in pairs], np.uint32)
    v = np.array([b for _, b in pairs], np.uint32)
    nv = 40
    off, col = O.build_sets(nv, u, v)
    run_both(ctx, lambda: ctx.from_edges(nv, u, v), nv, off, col, [0, 1, 2, 4, 10, 12, 14, 20, 24, 30], u, v)


@pytest.mark.parametrize("direction", ["auto", "topdown", "bottomup"])
@pytest.mark.parametrize("persist", ["on", "off"])
def test_kronecker_roots(ctx, direction, persist):
    """Kronecker scale 15: 16 sampled roots (plus a degree-1 root), every direction mode, K3p on and off,
    poisoned queues."""
    scale, seed = 15, 0xD1F
    ou, ov = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    off, col = O.build_sets(nv, ou, ov)
    deg = np.diff(off)
    try:
        ctx.set_option("direction", direction)
        ctx.set_option("persist", persist)
        ctx.set_option("poison_queues", "on")
        with ctx.kronecker(scale, 16, seed) as g:
            roots = [int(r) for r in g.sample_roots(16, seed=9)]
        roots.append(int(np.nonzero(deg == 1)[0][0]))
        run_both(ctx, lambda: ctx.kronecker(scale, 16, seed), nv, off, col, roots, ou, ov, mr=False)
    finally:
        for k, val in (("direction", "auto"), ("persist", "on"), ("poison_queues", "off")):
            ctx.set_option(k, val)


def test_hybrid_levels_forced(ctx):
    """Hybrid levels (hub pull + non-hub push) with the tail deferred."""
    scale, seed = 16, 0x1EAF
    ou, ov = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    off, col = O.build_sets(nv, ou, ov)
    try:
        ctx.set_option("hybrid", "force")
        with ctx.kronecker(scale, 16, seed) as g:
            roots = [int(r) for r in g.sample_roots(8, seed=3)]
        run_both(ctx, lambda: ctx.kronecker(scale, 16, seed), nv, off, col, roots, ou, ov, mr=False)
    finally:
        ctx.set_option("hybrid", "auto")


def test_reference_files_and_source_sequence(ctx, golden):
    """mediumG from every 25th source, then the same graph object re-used across sources with the option
    toggled between BFS runs (the deferred states are rewritten every BFS: no stale state survives)."""
    import os
    path = os.path.join(golden, "mediumG.txt")
    nv, u, v = O.load_graphfileutil(path)
    off, col = O.build_sets(nv, u, v)
    run_both(ctx, lambda: ctx.load_algs4(path), nv, off, col, list(range(0, nv, 25)), u, v)
    scale, seed = 14, 77
    ou, ov = O.kronecker(scale, 16, seed)
    n2 = 1 << scale
    off2, col2 = O.build_sets(n2, ou, ov)
    deg = np.diff(off2)
    leaves = [int(x) for x in np.nonzero(deg == 1)[0][:3]]
    try:
        with ctx.kronecker(scale, 16, seed) as g:
            for i, s in enumerate(leaves + [int(np.argmax(deg))] + leaves):
                ctx.set_option("leaf_defer", "on" if i % 2 else "off")
                check_against_oracle(g, n2, off2, col2, s, ou, ov, mr=False)
    finally:
        ctx.set_option("leaf_defer", DEFAULT)
