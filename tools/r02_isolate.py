"""Isolate the partitioned scale-20 validation failure: P=4 in-process group, options toggled."""
import importlib.util, os, sys, threading
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec); spec.loader.exec_module(bfsx)

def run(opts, world=4, scale=20, roots=2):
    ctxs = [bfsx.Context(0, **opts) for _ in range(world)]
    bfsx.local_group(ctxs)
    graphs = [ctxs[r].dist_kronecker(scale, r, world) for r in range(world)]
    single = bfsx.Context(0)
    g1 = single.kronecker(scale)
    out = []
    for s in [int(x) for x in g1.sample_roots(roots, seed=3)]:
        d1, _, _ = g1.bfs(s, want_parent=False)
        res = [None] * world
        def work(r):
            graphs[r].dist_bfs(s)
            v = graphs[r].validate()
            d, _ = graphs[r].result(want_parent=False)
            res[r] = (v["errors"], int(np.sum(d != d1[graphs[r].partition()["v_lo"]:][:len(d)])),
                      [ (l["direction"], l["frontier_out"]) for l in graphs[r].level_stats(64)])
        ths = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        [t.start() for t in ths]; [t.join() for t in ths]
        out.append((s, [(e, m) for e, m, _ in res], res[0][2]))
    for g in graphs: g.free()
    g1.free(); single.close()
    for c in ctxs: c.close()
    return out

import sys
for world in (1, 2, 4):
    for opts in ({}, {"direction": "bottomup"}, {"hub_bits": "off"}):
        r = run(opts, world=world)
        print(world, opts, [(s, e) for s, e, _ in r], flush=True)
