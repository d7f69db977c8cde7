"""Summarise one tools/gpu_round.sh session into profiles/<tag>_*.

  python tools/pmc_summary.py <tag>

Reads gpurun_out/<tag>/{trace,pmc_fetch,pmc_write}/ and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_hbm.json           per-launch HBM bytes of the dominant BFS kernels from the PMC passes,
                                    with the hash of the BFS kernel sources they were measured on (bench.py
                                    BFS_SRCS; bench.py reports `roofline.traffic` only while that hash matches)
  profiles/<tag>_bench.json         the default bench line of the same session (copied)

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950
FETCH_SIZE tallies 128-B requests at 64 B, i.e. it reads 1/2 of a wide streaming read's bytes; the
correction is calibrated per session on k_finalize, whose read is exactly the visited bitmap (8 B/lane,
coalesced).  Random 4-8 B probes are not calibrated by that, so both raw and corrected figures are kept.
"""
import csv
import hashlib
import json
import os
import shutil
import statistics as S
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BFS_SRCS = ("bfs_core.h", "kernels_push.hip", "kernels_pull.hip", "kernels_persist.hip", "kernels_level.hip",
            "kernels_dist.hip")  # as bench.py BFS_SRCS


def src_hash():
    h = hashlib.sha256()
    for f in BFS_SRCS:
        h.update(open(os.path.join(ROOT, "bfs-with-mapreduce_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def short(name):
    n = name.replace("bfsx::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def durations(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(short(r["Kernel_Name"]), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return out


def main():
    tag = sys.argv[1]
    d = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    if os.path.exists(os.path.join(d, "bench.json")):
        shutil.copy(os.path.join(d, "bench.json"), os.path.join(prof, f"{tag}_bench.json"))
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    dur = durations(os.path.join(d, "trace", "run_kernel_trace.csv"))
    nwords = None
    try:
        bl = json.load(open(os.path.join(d, "bench_levels.json")))
        nwords = bl["config"]["nv"] // 64
    except (OSError, KeyError, ValueError):
        pass
    corr = 2.0
    if "k_finalize" in fetch and nwords:
        corr = round((8.0 * nwords) / S.mean(fetch["k_finalize"]), 3)
    # the source the counters were measured on: recorded by the profiling script on the box (src_sha), else
    # the working tree's (summarise right after the run, before editing the kernels)
    try:
        sha = open(os.path.join(d, "src_sha")).read().split()[0][:16]
    except OSError:
        sha = src_hash()
    res = {"tag": tag, "bfs_src_sha": sha, "nwords": nwords, "fetch_correction": corr,
           "fetch_correction_basis": "k_finalize reads exactly 8*nwords B (8 B/lane coalesced)"
           if "k_finalize" in fetch else "guide default (x2 for wide streaming reads)",
           "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        f, w = S.mean(fetch[k]), S.mean(write[k])
        res["kernels"][k] = {
            "launches": len(fetch[k]),
            "fetch_raw_B": f, "write_B": w,
            "traffic_raw_B": f + w, "traffic_B": f * corr + w,
            "avg_ms_trace": S.mean(dur[k]) if k in dur else None,
        }
    # algorithmic bytes of k_bu from the per-level counters of the same session
    try:
        levels = json.load(open(os.path.join(d, "levels.json")))
        bu = [l for l in levels if l["direction"] == 2]
        sys.path.insert(0, ROOT)
        import importlib.util
        spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
        bench = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(bench)
        alg = S.mean([bench.level_bytes(l, nwords) for l in bu])
        res["k_bu_algorithmic_B_per_launch"] = alg
        res["k_bu_avg_ms_levels"] = S.mean([l["kernel_ms"] for l in bu])
        # Per-access-class correction (profiles/r03k_fetch_calibration.json: FETCH_SIZE reads wide coalesced
        # loads at 1/2 -- 128-B requests tallied at 64 B -- and scattered 4/8/16-B loads at 1/1).  k_bu's wide
        # class is the visited-word read (one 512-B load per wave: 8 B per 64 vertices) and the top1 loads of
        # the lane-dense candidate lists (4 B per live candidate); everything else it reads is scattered
        # (rest[], row offsets and entries, frontier probes, the few scattered top1 lines).  So the fabric read
        # bytes = raw + wide/2, with wide taken at its algorithmic size; writes are read as counted.
        wide = S.mean([8 * nwords + 4 * max(l["unvisited_in"], 0) for l in bu])
        res["k_bu_wide_read_B_per_launch"] = wide
        for name, k in res["kernels"].items():
            if name.startswith("k_bu<") and ", false, false, 4, false, true>" in name:
                k["traffic_class_B"] = k["fetch_raw_B"] + wide / 2 + k["write_B"]
                k["traffic_class_basis"] = ("FETCH_SIZE raw + the wide-coalesced class (visited words + top1 of "
                                            "the candidate lists, at algorithmic size) / 2 + WRITE_SIZE")
    except (OSError, KeyError, ValueError, S.StatisticsError):
        pass
    with open(os.path.join(prof, f"{tag}_hbm.json"), "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
