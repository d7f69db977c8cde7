"""Mean device time per BFS (bfsx_last_bfs_ms) over the first N sampled roots of the scale-26 bench graph, for
one library build (BFSX_LIB), interleaved builds A/B'd by calling this once per build:
   BFSX_LIB=ab/x/libbfsx.so python3 tools/r06_tbfs.py [roots] [reps]
Prints one JSON line {lib, roots, reps, t_bfs_ms_mean, hmean_gteps} (m_comp from the bfsx_bfs stats)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bfs-with-mapreduce_amd"))
import bfsx  # noqa: E402

roots_n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ctx = bfsx.Context(0)
g = ctx.kronecker(26, 16)
roots = [int(r) for r in g.sample_roots(roots_n)]
for r in roots:  # warm-up
    g.bfs_device_only(r)
ts = []
for _ in range(reps):
    for r in roots:
        ts.append(g.bfs_device_only(r))
m = g.m
print(json.dumps({"lib": os.environ.get("BFSX_LIB", "in-tree"), "roots": len(roots), "reps": reps,
                  "t_bfs_ms_mean": float(np.mean(ts)), "t_bfs_ms_hmean_basis": float(len(ts) / np.sum(1.0 / np.array(ts)))}))
