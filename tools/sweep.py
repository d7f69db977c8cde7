"""Direction-policy sweep on one device-resident graph (tuning aid, not part of the product).

  python tools/sweep.py [--scale 26] [--roots 64] alpha=30,60 beta=24 hub_degree=64 ...

Builds the Kronecker graph once, then for every combination of the option values runs the same roots
and prints one JSON line per combination: harmonic-mean GTEPS and mean BFS ms.
"""
import argparse
import importlib.util
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--roots", type=int, default=64)
    ap.add_argument("opts", nargs="*")
    a = ap.parse_args()
    keys, vals = [], []
    for o in a.opts:
        k, v = o.split("=", 1)
        keys.append(k)
        vals.append(v.split(","))
    ctx = bfsx.Context(0)
    g = ctx.kronecker(a.scale, 16, 0x5EED2026)
    roots = [int(r) for r in g.sample_roots(a.roots, seed=0x5EED)]
    mcomp = {r: g.bfs(r, want_dist=False, want_parent=False)[2]["m_comp"] for r in roots}
    for combo in itertools.product(*vals):
        for k, v in zip(keys, combo):
            ctx.set_option(k, v)
        for r in roots[:4]:
            g.bfs_device_only(r)
        ts = [g.bfs_device_only(r) for r in roots]
        gteps = [mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(roots, ts)]
        hm = len(gteps) / sum(1.0 / x for x in gteps)
        print(json.dumps({"opts": dict(zip(keys, combo)), "gteps_hmean": round(hm, 1),
                          "ms_mean": round(sum(ts) / len(ts), 4), "ms_max": round(max(ts), 4)}), flush=True)
    g.free()
    ctx.close()


if __name__ == "__main__":
    sys.exit(main())
