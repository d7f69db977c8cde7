"""Round-2 weak #1(b): does a SPILLING pull kernel corrupt a partitioned BFS when the ranks of an
in-process group run concurrently on one device?  One configuration per invocation:

    python tools/spill_experiment.py <pkg dir holding bfsx.py + libbfsx.so> <world> <scale> <roots> [k=v ...]

The group's distances (every rank's slice) are compared with the single-device BFS of the same graph
from the same roots, and every root is validated collectively; prints one line per root."""
import importlib.util
import os
import sys
import threading

import numpy as np

pkg, world, scale, nroots = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
opts = dict(kv.split("=", 1) for kv in sys.argv[5:])
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(pkg, "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)

single = bfsx.Context(0)
g1 = single.kronecker(scale)
roots = [int(x) for x in g1.sample_roots(nroots, seed=3)]
ref = {s: g1.bfs(s, want_parent=False)[0] for s in roots}
g1.free()
single.close()

ctxs = [bfsx.Context(0, **opts) for _ in range(world)]
if world > 1:
    bfsx.local_group(ctxs)
else:
    ctxs[0].comm_init(0, 1, bfsx.comm_unique_id())
graphs = [ctxs[r].dist_kronecker(scale, r, world) for r in range(world)]
total_bad = total_err = 0
for s in roots:
    res = [None] * world

    def work(r):
        graphs[r].dist_bfs(s)
        v = graphs[r].validate()
        d, _ = graphs[r].result(want_parent=False)
        lo = graphs[r].partition()["v_lo"]
        res[r] = (v["errors"], int(np.sum(d != ref[s][lo:lo + len(d)])))

    ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    bad = sum(m for _, m in res)
    err = res[0][0]
    total_bad += bad
    total_err += err
    print(f"root {s}: validation errors {err}, distance mismatches {bad} (per rank {[m for _, m in res]})",
          flush=True)
print(f"SUMMARY pkg={os.path.basename(os.path.dirname(pkg.rstrip('/')))} world={world} scale={scale} "
      f"opts={opts} HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}: mismatches {total_bad}, "
      f"validation errors {total_err}", flush=True)
for g in graphs:
    g.free()
for c in ctxs:
    c.close()
