"""Summarise an A/B directory of bench lines (tools/r04_step.sh): GTEPS, t_bfs and per-level-kind times per build.
   usage: python3 tools/ab_summary.py gpurun_out/<tag>"""
import collections
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    if f.endswith(".levels.json"):
        continue
    try:
        r = json.load(open(f))
    except ValueError:
        continue
    rf = r.get("roofline", {})
    print(f"{os.path.basename(f):28s} {r['value']:8.1f} wall {r['value_wall']:8.1f} t_bfs {r['t_bfs_ms_mean']:.4f} "
          f"k_bu {rf.get('avg_launch_ms')} frac {rf.get('frac')} unpack {r.get('t_unpack_ms')} "
          f"vwo {r.get('value_with_output') or 0:.1f} copy {r.get('t_result_copy_ms')}")
    lv = f.replace(".json", ".levels.json")
    if os.path.exists(lv):
        L = json.load(open(lv))
        nb = len({(x["root"], i) for i, x in enumerate(L) if x["level"] == 0})
        by = collections.defaultdict(lambda: [0, 0.0])
        for x in L:
            k = (x["direction"], min(x["level"], 6))
            by[k][0] += 1
            by[k][1] += x["kernel_ms"]
        print("   " + "  ".join(f"d{k[0]}l{k[1]}:{v[1] / v[0] * 1e3:.0f}us/{v[0] / max(nb, 1):.2f}"
                                for k, v in sorted(by.items())))
