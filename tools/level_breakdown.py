"""Where a BFS spends its time, from bench.py --levels-json records (one list of per-level dicts with
`root`; a new BFS starts at level 0).  Groups levels by kind (push before the first pull level, pull k,
hybrid, sparse pull, push after pull) and attributes each level the time since the previous level ended (its own
kernels plus the hand-off before them).   usage: python tools/level_breakdown.py levels.json [...]"""
import collections
import json
import sys


def breakdown(path):
    runs = []
    for l in json.load(open(path)):
        if l["level"] == 0:
            runs.append([])
        runs[-1].append(l)
    agg, cnt, kern = collections.defaultdict(float), collections.Counter(), collections.defaultdict(float)
    for ls in runs:
        prev, npull = 0.0, 0
        for i, l in enumerate(ls):
            d, dt = l["direction"], l["cum_ms"] - prev
            prev = l["cum_ms"]
            if d == 2:
                key = "pull%d" % min(npull, 3)
                npull += 1
            elif d == 4:  # the sparse pull kernel (tail levels)
                key = "pull sparse"
                npull += 1
            elif d == 3:
                key = "hybrid"
            else:
                key = ("push L%d" % min(i, 3)) if npull == 0 else "push after pull"
            agg[key] += dt
            cnt[key] += 1
            kern[key] += l["kernel_ms"]
    tot = sum(agg.values())
    n = len(runs)
    print(f"{path}: {n} BFS runs, {tot / n:.4f} ms per BFS (level ends)")
    for k in sorted(agg):
        print(f"  {k:16s} {cnt[k] / n:5.2f}/BFS  {agg[k] / n * 1e3:7.1f} us/BFS ({100 * agg[k] / tot:4.1f}%)  "
              f"{agg[k] / cnt[k] * 1e3:7.1f} us/level  kernels {kern[k] / cnt[k] * 1e3:7.1f} us/level")


for p in sys.argv[1:]:
    breakdown(p)
