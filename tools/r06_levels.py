"""Per-level-kind device time of bench.py --levels-json records, per build (tools/r06_ab.sh directories):
   python3 tools/r06_levels.py gpurun_out/<tag>
Prints, for every (direction, level) kind, the mean kernel_ms (event span: the level's kernels plus its frontier
conversion), its mean gap before it (host round trip) and how often it occurs per BFS."""
import collections
import glob
import json
import os
import sys

import numpy as np

by_build = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.levels.json"))):
    by_build[os.path.basename(f).rsplit("_", 1)[0]].append(f)
for b, files in sorted(by_build.items()):
    kms, gaps, nbfs, tb = collections.defaultdict(list), collections.defaultdict(list), 0, []
    for f in files:
        run, prev = [], None
        for x in json.load(open(f)) + [{"level": 0, "root": None}]:
            if x["level"] == 0 and run:
                nbfs += 1
                last = 0.0
                for y in run:
                    k = (y["direction"], min(y["level"], 7))
                    kms[k].append(y["kernel_ms"])
                    gaps[k].append(y["cum_ms"] - last - y["kernel_ms"])
                    last = y["cum_ms"]
                tb.append(run[-1]["cum_ms"])
                run = []
            if x.get("root") is not None:
                run.append(x)
    print(f"{b}: {nbfs} BFS, mean last-level cum {np.mean(tb) * 1e3:.1f} us")
    print("   " + "  ".join(f"d{k[0]}l{k[1]}:{np.mean(v) * 1e3:.1f}+{np.mean(gaps[k]) * 1e3:.1f}us/{len(v) / nbfs:.2f}"
                            for k, v in sorted(kms.items())))
