"""Scale-30 single-device diagnosis: one relabelled build, the same root under several runtime options,
each validated on the device (errors, first bad vertex, level directions).  Usage:
    python tools/r02_s30diag.py [root] [relabel on|off]"""
import sys
import time

sys.path.insert(0, "bfs-with-mapreduce_amd")
import bfsx  # noqa: E402

root = int(sys.argv[1]) if len(sys.argv) > 1 else 66103732
relabel = sys.argv[2] if len(sys.argv) > 2 else "on"
variants = [{}, {"hybrid": "off"}, {"persist": "off"}, {"bu_pipeline": "off"}, {"direction": "topdown"},
            {"direction": "bottomup"}]
with bfsx.Context(0) as ctx:
    ctx.set_option("relabel", relabel)
    t0 = time.perf_counter()
    with ctx.kronecker(30) as g:
        print(f"build {time.perf_counter() - t0:.1f} s nnz {g.nnz}", flush=True)
        for var in variants:
            for k, v in var.items():
                ctx.set_option(k, v)
            d, _, st = g.bfs(root, want_parent=False)
            v = g.validate()
            dirs = list(g.level_dirs())
            print(var, "errors", v["errors"], "first_bad", v["first_bad"], "reached", v["reached"], "levels",
                  st["levels"], "dirs", dirs, flush=True)
            if v["first_bad"] >= 0:
                fb = v["first_bad"]
                print("   dist[first_bad]", int(d[fb]), "deg", g.degree(fb), flush=True)
            for k in var:
                ctx.set_option(k, {"hybrid": "auto", "persist": "on", "bu_pipeline": "on",
                                   "direction": "auto"}[k])
