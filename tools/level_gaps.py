"""Host-side gaps between the levels of a bench run (tools/r04_step.sh levels.json): the time between one level's
end and the next level's first kernel, by (direction before, direction after), and before the first level.
   usage: python3 tools/level_gaps.py <levels.json>"""
import collections
import json
import statistics as S
import sys

L = json.load(open(sys.argv[1]))
runs, cur = [], []
for x in L:
    if x["level"] == 0 and cur:
        runs.append(cur)
        cur = []
    cur.append(x)
runs.append(cur)
gap = collections.defaultdict(list)
first = [r[0]["cum_ms"] - r[0]["kernel_ms"] for r in runs]
for r in runs:
    for a, b in zip(r, r[1:]):
        gap[(a["direction"], b["direction"])].append(b["cum_ms"] - b["kernel_ms"] - a["cum_ms"])
print(f"BFS runs {len(runs)}; before the first level {S.mean(first) * 1e3:.1f} us")
tot = 0.0
for k, v in sorted(gap.items()):
    per = len(v) / len(runs)
    tot += per * S.mean(v)
    print(f"  {k[0]} -> {k[1]}: {per:.2f} per BFS, {S.mean(v) * 1e3:.1f} us")
print(f"gaps per BFS {tot * 1e3:.1f} us; t_bfs mean (last level end) {S.mean(r[-1]['cum_ms'] for r in runs) * 1e3:.1f} us")
