"""Pins the CPU oracle against every known answer the reference holds (CPU only).

Known answers used:
  - algs4.jar!/BreadthFirstPaths.java:19-25   tinyCG dist and paths from 0 (serial algs4 BFS)
  - algs4.jar!/BreadthFirstPaths.java:13-18   tinyCG Bag adjacency ("java Graph tinyCG.txt")
  - algs4.jar!/Graph.java:10-31               tinyG and mediumG Bag adjacency
  - algs4.jar!/CC.java:10-18                  tinyG components {0..6},{7,8},{9..12}; mediumG connected
  - algs4.jar!/Cycle.java:10-12               mediumG cycle 15-0-225-15
  - PDF p.5 Table 6                           tinyCG final state of the Spark loop (3 iterations)
  - PDF p.5 1.5                               directed entry counts tiny 16, medium 2,546
  - SURVEY.md Appendix A                      mediumG distance vector sha256, per-iteration counts
"""
import os

import numpy as np
import pytest

import oracle_py as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gpath(name):
    return os.path.join(G, name)


def read_dist(name):
    with open(gpath(name)) as f:
        return np.array([int(line.split()[1]) for line in f], dtype=np.int32)


def parse_vertex_line(line):
    """Vertex(String) (Vertex.java:51-64): split on '|', lists split on ',' trimmed, omit empty."""
    tok = line.strip().split("|")
    lst = lambda s: [int(x.strip()) for x in s.replace("[", "").replace("]", "").split(",") if x.strip()]
    return int(tok[0]), set(lst(tok[1])), lst(tok[2]), int(tok[3]), tok[4]


def path_of(parent, v):
    p = [v]
    while parent[p[-1]] != p[-1]:
        p.append(int(parent[p[-1]]))
    return p[::-1]


def test_tinycg_serial_algs4_known_answer():
    nv, u, v = O.load_algs4_graph(gpath("tinyCG.txt"))
    assert (nv, len(u)) == (6, 8)
    # BreadthFirstPaths.java:13-18 adjacency in Bag order
    assert [O.algs4_adj(nv, u, v, x) for x in range(6)] == [
        [2, 1, 5], [0, 2], [0, 1, 3, 4], [5, 4, 2], [3, 2], [3, 0]]
    dist, edge_to = O.algs4_bfs(nv, u, v, 0)
    assert dist.tolist() == [0, 1, 1, 2, 2, 1]
    # paths printed at BreadthFirstPaths.java:20-25
    assert [path_of(edge_to, x) for x in range(6)] == [
        [0], [0, 1], [0, 2], [0, 2, 3], [0, 2, 4], [0, 5]]


def test_tinycg_mapreduce_matches_pdf_table6():
    nv, u, v = O.load_graphfileutil(gpath("tinyCG.txt"))
    off, col = O.build_sets(nv, u, v)
    assert off[-1] == 16  # PDF p.5: 16 directed entries
    r = O.mapreduce_bfs(nv, off, col, 0)
    assert r["iters"] == 3
    with open(gpath("tinyCG_table6.txt")) as f:
        table = {t[0]: t for t in map(parse_vertex_line, f)}
    for x in range(nv):
        _, nbrs, path, d, colour = table[x]
        assert set(col[off[x]:off[x + 1]].tolist()) == nbrs
        assert r["dist"][x] == d
        assert ["WHITE", "GRAY", "BLACK"][r["color"][x]] == colour
        assert path_of(r["parent"], x) == path  # tie-break restated to reproduce the published run
    assert O.validate(nv, off, col, 0, r["dist"], r["parent"]) == 0


def test_mediumg_known_answers():
    nv, u, v = O.load_graphfileutil(gpath("mediumG.txt"))
    assert (nv, len(u)) == (250, 1273)
    off, col = O.build_sets(nv, u, v)
    assert off[-1] == 2546  # PDF p.5
    # Graph.java:28-30, Bag order (algs4 parse semantics)
    nv2, u2, v2 = O.load_algs4_graph(gpath("mediumG.txt"))
    assert O.algs4_adj(nv2, u2, v2, 0) == [225, 222, 211, 209, 204, 202, 191, 176, 163, 160, 149, 114,
                                           97, 80, 68, 59, 58, 49, 44, 24, 15]
    assert O.algs4_adj(nv2, u2, v2, 1) == [220, 203, 200, 194, 189, 164, 150, 130, 107, 72]
    assert O.algs4_adj(nv2, u2, v2, 2) == [141, 110, 108, 86, 79, 51, 42, 18, 14]
    # Cycle.java:11-12: 15-0-225-15
    for a, b in ((15, 0), (0, 225), (225, 15)):
        assert b in col[off[a]:off[a + 1]]
    r = O.mapreduce_bfs(nv, off, col, 0)
    assert (r["dist"] != O_INF).all()  # CC.java:16-18: one component
    assert O.dist_sha256(r["dist"]) == "0e79715f16d24cb8ccfa662188638202e2b241f5a974915276e751f1f6d6a0b6"
    assert np.array_equal(r["dist"], read_dist("mediumG.dist"))
    assert r["iters"] == 14
    assert list(zip(r["gray"].tolist(), r["emits"].tolist())) == [
        (21, 271), (16, 575), (20, 432), (22, 469), (23, 471), (21, 502), (22, 462), (35, 475),
        (30, 587), (14, 477), (14, 363), (8, 382), (3, 315), (0, 265)]
    d2, e2 = O.algs4_bfs(nv2, u2, v2, 0)
    assert np.array_equal(d2, r["dist"])
    assert O.validate(nv, off, col, 0, d2, e2) == 0
    assert O.validate(nv, off, col, 0, r["dist"], r["parent"]) == 0


O_INF = 2147483647


def test_tiny_g_components_and_bag_order():
    nv, u, v = O.load_graphfileutil(gpath("tinyG.txt"))
    assert (nv, len(u)) == (13, 13)
    # Graph.java:11-24
    expect = [[6, 2, 1, 5], [0], [0], [5, 4], [5, 6, 3], [3, 4, 0], [0, 4], [8], [7], [11, 10, 12],
              [9], [9, 12], [11, 9]]
    assert [O.algs4_adj(nv, u, v, x) for x in range(nv)] == expect
    off, col = O.build_sets(nv, u, v)
    # CC.java:10-14: components {0..6}, {7,8}, {9..12}
    for src, comp in ((0, range(0, 7)), (7, (7, 8)), (9, range(9, 13))):
        r = O.mapreduce_bfs(nv, off, col, src)
        reached = set(np.nonzero(r["dist"] != O_INF)[0].tolist())
        assert reached == set(comp)
        assert O.validate(nv, off, col, src, r["dist"], r["parent"]) == 0
    assert np.array_equal(O.mapreduce_bfs(nv, off, col, 0)["dist"], read_dist("tinyG.dist"))


def test_tinycg_hash():
    nv, u, v = O.load_graphfileutil(gpath("tinyCG.txt"))
    off, col = O.build_sets(nv, u, v)
    r = O.mapreduce_bfs(nv, off, col, 0)
    assert O.dist_sha256(r["dist"]) == "7aaf29ac8c2b7f46ebf2cea4eaa51764dbd5f4e08b5b193607c921fc3f6d2ca5"


def test_validator_rejects_bad_trees():
    nv, u, v = O.load_graphfileutil(gpath("tinyCG.txt"))
    off, col = O.build_sets(nv, u, v)
    d, p = O.csr_bfs(nv, off, col, 0)
    assert O.validate(nv, off, col, 0, d, p) == 0
    bad = d.copy(); bad[3] = 5
    assert O.validate(nv, off, col, 0, bad, p) < 0
    badp = p.copy(); badp[4] = 1  # 1-4 is not an edge
    assert O.validate(nv, off, col, 0, d, badp) == -3
    badp = p.copy(); badp[0] = 2
    assert O.validate(nv, off, col, 0, d, badp) == -1


@pytest.mark.parametrize("threads", [1, 4])
def test_mapreduce_equals_serial_on_random_graphs(threads):
    rng = np.random.default_rng(7)
    for trial in range(20):
        nv = int(rng.integers(1, 400))
        m = int(rng.integers(0, 3 * nv + 1))
        u = rng.integers(0, nv, m).astype(np.uint32)
        v = rng.integers(0, nv, m).astype(np.uint32)
        off, col = O.build_sets(nv, u, v)
        src = int(rng.integers(0, nv))
        r = O.mapreduce_bfs(nv, off, col, src, nthreads=threads)
        d, p = O.csr_bfs(nv, off, col, src)
        assert np.array_equal(r["dist"], d)
        assert O.validate(nv, off, col, src, r["dist"], r["parent"]) == 0
        d2, e2 = O.algs4_bfs(nv, u, v, src)
        assert np.array_equal(d2, d)
        assert r["iters"] == (d[d != O_INF].max() + 1)


def test_kronecker_oracle_shape():
    u, v = O.kronecker(10, 16, 1)
    assert len(u) == 16 << 10 and u.max() < 1024 and v.max() < 1024
    u2, v2 = O.kronecker(10, 16, 1)
    assert np.array_equal(u, u2) and np.array_equal(v, v2)
    u3, _ = O.kronecker(10, 16, 2)
    assert not np.array_equal(u, u3)
    # power-law: a few heavy vertices
    deg = np.bincount(np.concatenate([u, v]), minlength=1024)
    assert deg.max() > 20 * deg.mean()
