"""Per-kernel averages of the SQ counter passes written by tools/sq_passes.sh.
    python tools/sq_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(lambda: collections.Counter())
for f in sorted(glob.glob(f"{root}/pass*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void bfsx::(anonymous namespace)::", "")
        c = r["Counter_Name"]
        acc[k][c] += float(r["Counter_Value"])
        n[k][c] += 1
out = {}
for k in acc:
    out[k] = {c: acc[k][c] / n[k][c] for c in sorted(acc[k])}
    w = out[k]
    if w.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in w:
                w[c + "_frac"] = w[c] / w["SQ_WAVE_CYCLES"]
print(json.dumps(out, indent=1))
