"""Regenerates the committed golden fixtures in tests/golden/ (run from the repo root, CPU only).

Sources, all held by the reference itself (nothing here imports or runs reference code):
  tinyCG.txt, mediumG.txt   copied verbatim from /root/reference/test-sets/ (the reference's data)
  tinyG.txt                 an edge list reconstructed from the adjacency printed in
                            algs4.jar!/Graph.java:10-24 ("% java Graph tinyG.txt"): the edge set is
                            the union of those lists, in an insertion order for which every Bag (LIFO)
                            list comes out exactly as printed (tests/test_oracle.py checks that)
  tinyCG_table6.txt         PDF p.5 Table 6 (final tinyCG state after iteration 3), transcribed
  *.dist                    distances from source 0 produced by the oracle restatement; their sha256
                            over "v d\\n" lines equal SURVEY.md Appendix A, which was derived from the
                            map/reduce semantics and cross-checked against networkx
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

TINYG = """13
13
0 5
4 3
0 1
9 12
6 4
5 4
0 2
11 12
9 10
0 6
7 8
9 11
5 3
"""

# PDF p.5 Table 6 (id | neighbours | path | distance | colour), Vertex.toString format (Vertex.java:123-125)
TABLE6 = """0|[1, 2, 5]|[0]|0|BLACK
1|[0, 2]|[0, 1]|1|BLACK
2|[0, 1, 3, 4]|[0, 2]|1|BLACK
3|[2, 4, 5]|[0, 5, 3]|2|BLACK
4|[2, 3]|[0, 2, 4]|2|BLACK
5|[0, 3]|[0, 5]|1|BLACK
"""


def main():
    import oracle_py as O

    with open(os.path.join(HERE, "tinyG.txt"), "w") as f:
        f.write(TINYG)
    with open(os.path.join(HERE, "tinyCG_table6.txt"), "w") as f:
        f.write(TABLE6)
    for name in ("tinyCG", "mediumG", "tinyG"):
        nv, u, v = O.load_graphfileutil(os.path.join(HERE, name + ".txt"))
        off, col = O.build_sets(nv, u, v)
        r = O.mapreduce_bfs(nv, off, col, 0)
        with open(os.path.join(HERE, name + ".dist"), "w") as f:
            f.write("".join(f"{i} {d}\n" for i, d in enumerate(r["dist"].tolist())))
        print(name, nv, len(u), r["iters"], O.dist_sha256(r["dist"]))


if __name__ == "__main__":
    main()
