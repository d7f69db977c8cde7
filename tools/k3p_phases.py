"""Where a K3p level's time goes, per workgroup, on the largeG stand-in (a diagnostic build: tools/diag/
k3p_phase_stamps.patch, loaded through BFSX_LIB).  Every workgroup stamps each level three times with the
100 MHz wall clock: level start, sweep done (its record is about to be written), barrier passed (every record
read).  Per level: the sweep of the median and of the slowest workgroup, the arrival skew (slowest record
minus median record), the barrier after the last arrival (median pass minus the last record) and the level
time (median pass to median pass).
    BFSX_LIB=diagbuild/libbfsx_k3pphase.so python tools/k3p_phases.py out.json"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bfs-with-mapreduce_amd"))
import bfsx  # noqa: E402


def standin(side=1000, m=7_586_063, radius=2, seed=2026):  # the generator of tests/test_gpu_largeg.py
    rng = np.random.default_rng(seed)
    nv = side * side
    a = rng.integers(0, nv, m)
    dx = rng.integers(-radius, radius + 1, m)
    dy = rng.integers(-radius, radius + 1, m)
    x = np.clip(a % side + dx, 0, side - 1)
    y = np.clip(a // side + dy, 0, side - 1)
    return nv, a.astype(np.uint32), (y * side + x).astype(np.uint32)


K_LEV, K_G, TICK_US = 640, 256, 0.01  # wall_clock64 runs at 100 MHz

nv, u, v = standin()
lib = C.CDLL(os.environ["BFSX_LIB"])
with bfsx.Context(0) as ctx:
    with ctx.from_edges(nv, u, v) as g:
        for _ in range(3):
            g.bfs_device_only(0)
        levels = g.level_stats(4096)
        buf = (C.c_ulonglong * (K_LEV * K_G * 3))()
        assert lib.bfsx_debug_k3p_phases(buf, C.c_size_t(K_LEV * K_G * 3)) == 0
ph = np.frombuffer(buf, dtype=np.uint64).reshape(K_LEV, K_G, 3).astype(np.int64)
used = [w for w in range(K_G) if ph[1:50, w, 2].max() > 0]  # workgroups of the launch
G = len(used)
ph = ph[:, :G, :]
rows = []
for L in range(1, min(K_LEV, len(levels))):
    s0, s1, s2 = ph[L, :, 0], ph[L, :, 1], ph[L, :, 2]
    if s0.min() <= 0 or s2.min() <= 0 or ph[L - 1, :, 2].min() <= 0:
        continue
    sweep = (s1 - s0) * TICK_US
    rows.append({"level": L, "sweep_med": float(np.median(sweep)), "sweep_max": float(sweep.max()),
                 "arrival_skew": float((s1.max() - np.median(s1)) * TICK_US),
                 "barrier_after_last": float((np.median(s2) - s1.max()) * TICK_US),
                 "level_us": float((np.median(s2) - np.median(ph[L - 1, :, 2])) * TICK_US),
                 "start_after_prev_pass": float((np.median(s0) - np.median(ph[L - 1, :, 2])) * TICK_US),
                 "slowest_wg": int(np.argmax(s1))})
summary = {k: float(np.median([r[k] for r in rows])) for k in
           ("sweep_med", "sweep_max", "arrival_skew", "barrier_after_last", "level_us", "start_after_prev_pass")}
slow = np.bincount([r["slowest_wg"] for r in rows], minlength=G)
out = {"workgroups": G, "levels_stamped": len(rows), "median_over_levels_us": summary,
       "slowest_workgroup_counts_top8": sorted(((int(c), w) for w, c in enumerate(slow)), reverse=True)[:8],
       "levels": rows}
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: out[k] for k in ("workgroups", "levels_stamped", "median_over_levels_us",
                                       "slowest_workgroup_counts_top8")}))
