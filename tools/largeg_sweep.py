"""largeG-class per-level latency (configs[2] stand-in: 1e6-vertex geometric graph, ~560 levels) under option
settings, one line per setting: python tools/largeg_sweep.py key=v1,v2,... [key2=...]   (on a GPU box).
BFSX_PKG=<dir holding bfsx.py + libbfsx.so> runs another build (A/B against an earlier commit)."""
import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.environ.get("BFSX_PKG", os.path.join(ROOT, "bfs-with-mapreduce_amd"))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(PKG, "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)


def standin(side=1000, m=7_586_063, radius=2, seed=2026):  # the generator of tests/test_gpu_largeg.py
    rng = np.random.default_rng(seed)
    nv = side * side
    a = rng.integers(0, nv, m)
    dx = rng.integers(-radius, radius + 1, m)
    dy = rng.integers(-radius, radius + 1, m)
    x = np.clip(a % side + dx, 0, side - 1)
    y = np.clip(a // side + dy, 0, side - 1)
    return nv, a.astype(np.uint32), (y * side + x).astype(np.uint32)


nv, u, v = standin()
ctx = bfsx.Context(0)
# FRESH=1: a new graph per setting (K3p keeps the grid of a graph's first launch, so a persist_blocks sweep
# needs one graph per value)
fresh = os.environ.get("FRESH") == "1"
g = ctx.from_edges(nv, u, v)
with g:
    ref = None
    for arg in sys.argv[1:] or ["persist_blocks=auto"]:
        k, vals = arg.split("=", 1)
        for val in vals.split(","):
            ctx.set_option(k, val)
            if fresh:
                g.free()
                g = ctx.from_edges(nv, u, v)
            ts = []
            for _ in range(4):
                d, _, st = g.bfs(0, want_parent=False)
                ts.append(st["t_bfs_ms"])
            ref = d if ref is None else ref
            if os.environ.get("LEVELS_OUT"):  # per-level records of the last run of this setting
                with open(f"{os.environ['LEVELS_OUT']}_{k}_{val}.json", "w") as f:
                    json.dump(g.level_stats(4096), f)
            print(json.dumps({"pkg": os.path.basename(PKG), k: val, "levels": st["levels"], "t_bfs_ms": round(min(ts), 3),
                              "us_per_level": round(min(ts) * 1e3 / st["levels"], 2), "same": bool(np.array_equal(d, ref)),
                              "persist_retries": st.get("persist_retries")}), flush=True)
        ctx.set_option(k, "auto" if k == "persist_blocks" else vals.split(",")[0])
ctx.close()
