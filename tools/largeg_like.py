"""largeG stand-in (configs[2]): largeG.txt is not in the reference checkout (.MISSING_LARGE_BLOBS), so this
writes an algs4 edge list of the same size and shape class -- 1,000,000 vertices, 7,586,063 edges, a
high-diameter geometric graph (the reference's known answers put ecc(0) >= 566, BreadthFirstPaths.java:
28-34) -- and times the path end to end:

  host parse (bfsx_parse_algs4) | GPU tokenizer (bfsx_parse_algs4_gpu) | bfsx_graph_load_algs4 (file -> CSR)
  | bfsx_bfs from source 0 (device time, levels, us/level) | the serial algs4 BFS restated in the oracle
  (the reference's SequentialTest path, 1.170 s on the real largeG per PDF p.6) on one host core.

  python tools/largeg_like.py [--out /tmp/largeG_like.txt]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def write_graph(path, side=1000, m=7_586_063, radius=2, seed=2026):
    """Vertices on a side x side grid (id = y*side + x); every edge joins a vertex to a random vertex at
    most `radius` cells away in each axis (a random geometric graph: diameter ~ side)."""
    rng = np.random.default_rng(seed)
    nv = side * side
    a = rng.integers(0, nv, m)
    dx = rng.integers(-radius, radius + 1, m)
    dy = rng.integers(-radius, radius + 1, m)
    x = np.clip(a % side + dx, 0, side - 1)
    y = np.clip(a // side + dy, 0, side - 1)
    b = y * side + x
    import pandas as pd
    with open(path, "w") as f:
        f.write(f"{nv}\n{m}\n")
    pd.DataFrame({"a": a, "b": b}).to_csv(path, sep=" ", header=False, index=False, mode="a")
    return nv, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/tmp/largeG_like.txt")
    ap.add_argument("--option", action="append", default=[], help="libbfsx option key=value")
    a = ap.parse_args()
    t0 = time.perf_counter()
    nv, m = write_graph(a.out)
    res = {"file": a.out, "bytes": os.path.getsize(a.out), "nv": nv, "m": m,
           "write_s": round(time.perf_counter() - t0, 2)}
    t0 = time.perf_counter()
    _, hu, hv = bfsx.parse_algs4(a.out)
    res["host_parse_s"] = round(time.perf_counter() - t0, 3)
    with bfsx.Context(0) as ctx:
        for kv in a.option:
            ctx.set_option(*kv.split("=", 1))
        res["options"] = a.option
        ctx.parse_algs4_gpu(a.out)  # warm-up (code objects, allocator)
        t0 = time.perf_counter()
        _, gu, gv = ctx.parse_algs4_gpu(a.out)
        res["gpu_parse_s_incl_d2h"] = round(time.perf_counter() - t0, 3)
        assert np.array_equal(hu, gu) and np.array_equal(hv, gv)
        t0 = time.perf_counter()
        g = ctx.load_algs4(a.out)
        ctx.synchronize()
        res["load_algs4_s"] = round(time.perf_counter() - t0, 3)
        g.bfs(0)  # warm-up
        d, p, st = g.bfs(0)
        res.update({"levels": st["levels"], "t_bfs_ms": round(st["t_bfs_ms"], 3),
                    "us_per_level": round(st["t_bfs_ms"] * 1e3 / st["levels"], 2),
                    "t_total_ms_incl_d2h": round(st["t_total_ms"], 3), "reached": st["reached"],
                    "mteps": round(st["m_comp"] / (st["t_bfs_ms"] * 1e-3) / 1e6, 1)})
        ls = g.level_stats(4096)
        td = [l for l in ls if l["direction"] == 1]
        res.update({"topdown_levels": len(td), "bottomup_levels": len(ls) - len(td),
                    "kernel_ms_sum": round(sum(l["kernel_ms"] for l in ls), 3),
                    "td_kernel_us_mean": round(1e3 * sum(l["kernel_ms"] for l in td) / max(len(td), 1), 2),
                    "frontier_mean": round(sum(l["frontier_in"] for l in ls) / len(ls), 1),
                    "mf_mean": round(sum(max(l["mf_in"], 0) for l in ls) / len(ls), 1)})
        off, col = g.csr()
        g.free()
    import oracle_py as O
    rows = np.repeat(np.arange(nv, dtype=np.int64), np.diff(off))
    col = col[np.lexsort((col, rows))]
    t0 = time.perf_counter()
    ref, _ = O.csr_bfs(nv, off, col, 0)
    res["cpu_serial_bfs_s"] = round(time.perf_counter() - t0, 3)
    assert np.array_equal(ref, d), "GPU distances differ from the oracle"
    res["dist_equal_oracle"] = True
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
