"""Benchmark: GTEPS (harmonic mean over 64 roots) on Graph500 Kronecker scale-26, edgefactor 16.

BASELINE.json configs[3].  The graph is generated and built on the GPU before the timed region.  A
"step" is one Graph500 BFS pass: one BFS from EACH of the 64 sampled roots (every root validated on the
device beforehand), so every step covers the metric's 64 roots.  TEPS per BFS = m_comp / t with m_comp =
the input tuples inside the root's component (Graph500 convention); value = harmonic mean GTEPS over the
K x 64 timed BFS runs.

  t (both N = 1 and N > 1) = device time from source init to the last level (hipEvents inside
  libbfsx.so); at N > 1 the per-root time is the MAX over ranks (every BFS is collective).  The
  wall-clock aggregate over the barrier-bracketed K steps is reported next to it (value_wall).
  N = 1: single-device level loop.  A partitioned-path rehearsal on the same device (RCCL communicator
         of one, the loop N > 1 runs) is reported as "partitioned_p1".
  N > 1: one process per GPU (torch.distributed.run); the graph is 1-D partitioned over the ranks and
         libbfsx runs the level loop with its own RCCL communicator (all-to-allv of owner-routed pairs,
         all-gather of frontier bitmaps, all-reduce of the level counters).

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline accounting.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu-baseline]

--gpus N > 1 without a launcher (WORLD_SIZE unset) starts the N ranks itself, as one child
`python -m torch.distributed.run --nproc-per-node N` process, and relays its JSON line (launch_ranks).
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "bfs-with-mapreduce_amd")
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def load_module(name, file):
    # test hook: BFSX_BENCH_BINDING names a stand-in for the libbfsx binding (tests/bench_dist_fake.py),
    # so the launcher and the N > 1 harness run on a CPU-only box
    override = os.environ.get("BFSX_BENCH_BINDING")
    path = override if override and name == "bfsx" else os.path.join(PKG, file)
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def found_store_bytes(ls, found_bytes=4, code_bytes=1):
    """Stores of a pull or hybrid level's discoveries.  Round 5 (single device): every discovery stores a 1-B
    provenance code (code_bytes), and the `explicit_parents` among them also a found_bytes parent; the others'
    parent is one of their first four row entries, which the level read anyway.  A partitioned loop stores every
    parent explicitly and no code (code_bytes 0).  Records without the counter (older builds): found_bytes each."""
    f = ls["frontier_out"]
    if "explicit_parents" not in ls:
        return found_bytes * f
    return code_bytes * f + found_bytes * ls["explicit_parents"]


def level_bytes(ls, nwords, off_bytes=4, found_bytes=4, code_bytes=1):
    """Algorithmic bytes of one level: what the level must move at minimum, counted from
    its device counters.  Frontier-bit and visited-bit probes are not counted (the n/8-byte bitmaps are
    cache-resident).  off_bytes: width of the row offsets the traversal kernels read (uint32 when the
    graph has < 2^32 adjacency entries).  found_bytes / code_bytes: the stores of a pull or hybrid level's
    discoveries (found_store_bytes; 4: the 4-B parent, whose distance is the level's record bitmap; 8: a packed
    (parent, dist) state word)."""
    d = ls["direction"]
    if d in (2, 4):  # bottom-up (4: the sparse pull kernel of the tail levels, same accounting): visited word read + next word write, top1 of every live candidate, rest[]
        # (2nd..4th neighbours + degree, 16 B) of every top1 miss, the offset pair of each row walked past
        # its first four entries (`claims`), the adjacency entries walked there, the parent (or packed state)
        # of every vertex found
        return (16 * nwords + 4 * max(ls["unvisited_in"], 0) + 16 * ls["stage2"] + 2 * off_bytes * ls["claims"]
                + 4 * ls["walked"] + found_store_bytes(ls, found_bytes, code_bytes))
    if d == 3:  # hybrid: the pull half's bitmap pass + top1 of the live candidates, the push half's rows, the
        # parent of every vertex found (both halves store the 4-B parent; the distance is the level's record)
        return (16 * nwords + 4 * max(ls["unvisited_in"], 0) + 4 * max(ls["scanned"], 0)
                + found_store_bytes(ls, found_bytes, code_bytes))
    # top-down: queue read + offset pair per frontier vertex, adjacency rows, winners' packed state write,
    # queue append and offset pair (degree) lookup
    return ((4 + 2 * off_bytes) * ls["frontier_in"] + 4 * max(ls["mf_in"], 0)
            + (12 + 2 * off_bytes) * ls["frontier_out"])


def hmean(xs):
    return len(xs) / sum(1.0 / x for x in xs)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10, help="timed steps (one step = one BFS per root)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--roots", type=int, default=64, help="roots per step (the metric's 64)")
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED2026)
    ap.add_argument("--root-seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--serial-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the OpenMP CPU baseline (default: the box's CPU share, OMP_NUM_THREADS, "
                         "else the affinity mask)")
    ap.add_argument("--no-p1", action="store_true", help="skip the partitioned-path P=1 rehearsal at N=1")
    ap.add_argument("--direction", default="auto")
    ap.add_argument("--levels-json", default="")
    ap.add_argument("--option", action="append", default=[], help="libbfsx option key=value")
    ap.add_argument("--dist", action="store_true", help="use the partitioned path even on one rank (rehearsal)")
    ap.add_argument("--scale30-roots", type=int, default=-1,
                    help="N > 1: after the scale-26 metric, BASELINE configs[4] (RMAT scale 30, 1-D partitioned over the "
                         "same ranks) on this many validated roots, reported as the line's 'scale30' object (-1: 4 "
                         "roots when N > 1 and --scale is 26; 0: off)")
    ap.add_argument("--comm-split-roots", type=int, default=8,
                    help="N > 1: roots of the untimed diagnostic pass with hipEvents around every collective "
                         "(per-kind device time per BFS, max over ranks; 0: off)")
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="seconds after which a rank (and the --gpus N launcher) gives up and exits 124 instead of "
                         "waiting on a stuck peer (0: none)")
    return ap.parse_args()


def arm_deadline(seconds, what):
    """End this process with exit code 124 when it still runs after `seconds`.  Every rank arms it: a rank stuck
    behind a failed or diverged peer must not burn the driver's time limit and leave no JSON line (libbfsx also
    fails every rank's call when one rank fails, and gives up a collective after comm_timeout_ms; this is the
    last line).  torch.distributed.run then stops the other ranks."""
    if seconds <= 0:
        return None
    import threading

    def fire():
        print(f"[bench] {what}: deadline of {seconds:.0f} s passed, exiting 124", file=sys.stderr, flush=True)
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def pick_roots(args, g, m_tuples, bfs_mcomp, validate):
    """The first args.roots Graph500 search keys (degree >= 1, in bfsx_sample_roots order) whose component
    holds at least 1/1000 of the input tuples, each validated on the device (untimed).  A key inside a
    component of a few edges (absent at scale 26, seen at scale 30) has a TEPS near 1e-6 that would turn
    the harmonic mean into a statement about that one root; such keys are skipped and listed.  The
    sampling is prefix-stable, so a graph without tiny components keeps exactly the first roots."""
    roots, mcomp, errors, skipped = [], {}, 0, []
    for r in (int(x) for x in g.sample_roots(4 * args.roots, seed=args.root_seed)):
        if len(roots) == args.roots:
            break
        mc = bfs_mcomp(r)
        if mc * 1000 < m_tuples:
            skipped.append({"root": r, "m_comp": mc})
            continue
        mcomp[r] = mc
        errors += validate()
        roots.append(r)
    return roots, mcomp, errors, skipped


def common_fields(args, world, value, wall, nv, m, nnz, nroots, parallelism):
    return {
        "metric": f"GTEPS (harmonic mean, {nroots} roots) on RMAT scale-{args.scale}",
        "value": value,
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / max(args.steps, 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (Graph500 Kronecker A/B/C/D=.57/.19/.19/.05, generated on device)",
        "config": {
            "workload": f"kronecker-s{args.scale}-ef{args.edgefactor}",
            "scale": args.scale,
            "edgefactor": args.edgefactor,
            "seed": hex(args.seed),
            "nv": nv,
            "m_tuples": m,
            "nnz_directed": nnz,
            "roots": nroots,
            "step": f"one BFS from each of the {nroots} roots",
            "direction": args.direction,
            "parallelism": parallelism,
        },
    }


# The BFS kernel sources (one translation unit per kernel family + their shared core): a PMC summary is reported
# only for the source it was measured on, hashed as the concatenation in this order (tools/pmc_summary.py and the
# profiling scripts: cat <these files> | sha256sum)
BFS_SRCS = ("bfs_core.h", "kernels_push.hip", "kernels_pull.hip", "kernels_persist.hip", "kernels_level.hip",
            "kernels_dist.hip")


def bfs_src_sha(pkg=None):
    import hashlib
    h = hashlib.sha256()
    for f in BFS_SRCS:
        h.update(open(os.path.join(pkg or PKG, "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def measured_traffic(kernel="k_bu", nwords=None):
    """Per-launch HBM bytes of `kernel` from the newest committed PMC summary (profiles/<tag>_hbm.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes),
    used only while the BFS kernel sources (BFS_SRCS) still hash to the source they were measured on, and only
    for the graph size it was measured on (nwords: bitmap words of the bench's graph; a scale-26 profile says
    nothing about a scale-30 launch)."""
    import glob
    sha = bfs_src_sha()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        names = [n for n in rec.get("kernels", {}) if n == kernel or n.startswith(kernel + "<")]
        if rec.get("bfs_src_sha") == sha and names and (nwords is None or rec.get("nwords") == nwords):
            # the instantiation with the most launches (the hybrid levels' hub sweep is a second one)
            k = max((rec["kernels"][n] for n in names), key=lambda x: x.get("launches", 0))
            # per-access-class correction when the summary has it (round 3: profiles/r03k_fetch_calibration.json),
            # else the blanket wide-read factor (an upper bound: it doubles the scattered reads too)
            cls = k.get("traffic_class_B")
            tb = cls if cls else k["traffic_B"]
            out = {"traffic": round(tb / 1e6, 1), "traffic_raw": round(k["traffic_raw_B"] / 1e6, 1),
                   "traffic_blanket": round(k["traffic_B"] / 1e6, 1),
                   "traffic_source": os.path.relpath(path, ROOT),
                   "traffic_correction": (k.get("traffic_class_basis") if cls else
                                          f"FETCH_SIZE x {rec.get('fetch_correction')} (blanket) + WRITE_SIZE")}
            if k.get("avg_ms_trace"):  # fabric-side rate of the same launches (rocprof trace durations)
                out["traffic_GBs"] = round(tb / (k["avg_ms_trace"] * 1e-3) / 1e9, 1)
                out["traffic_frac"] = round(out["traffic_GBs"] / PEAK_HBM_GBS, 4)
            return out
    return {"traffic": None, "traffic_source": "no PMC summary for this kernel source and graph size"}


class LevelAccount:
    """Algorithmic bytes of the timed BFS runs: per bottom-up launch (the dominant kernel) and summed
    over every level of every BFS (the whole-BFS figure)."""

    def __init__(self, nwords, off_bytes, found_bytes=4, code_bytes=1):
        self.nwords, self.off_bytes, self.found_bytes, self.code_bytes = nwords, off_bytes, found_bytes, code_bytes
        self.bu_bytes, self.bu_ms, self.bu_launches = 0, 0.0, 0
        self.all_bytes = 0
        self.by_dir = {1: 0, 2: 0, 3: 0}

    def add(self, levels):
        for ls in levels:
            b = level_bytes(ls, self.nwords, self.off_bytes, self.found_bytes, self.code_bytes)
            self.all_bytes += b
            self.by_dir[ls["direction"]] = self.by_dir.get(ls["direction"], 0) + b
            if ls["direction"] == 2:
                self.bu_bytes += b
                self.bu_ms += ls["kernel_ms"]
                self.bu_launches += 1

    def roofline(self, note):
        n = self.bu_launches
        ach = (self.bu_bytes / n) / ((self.bu_ms / n) * 1e-3) / 1e9 if n else 0.0
        tr = measured_traffic(nwords=self.nwords)
        return {
            "bound": "hbm",
            "kernel": "k_bu (bottom-up pull)",
            "achieved": round(ach, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4),
            "traffic": tr.pop("traffic"),
            "traffic_unit": "MB per launch (fabric bytes from FETCH_SIZE / WRITE_SIZE, corrected per access class)",
            "algorithmic": round(self.bu_bytes / max(n, 1) / 1e6, 1),
            **tr,
            "launches": n,
            "avg_launch_ms": round(self.bu_ms / max(n, 1), 4),
            "note": note,
        }

    def whole(self, t_sum_ms, nbfs):
        ach = self.all_bytes / (t_sum_ms * 1e-3) / 1e9 if t_sum_ms > 0 else 0.0
        return {
            "bound": "hbm",
            "achieved": round(ach, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4),
            "algorithmic_MB_per_bfs": round(self.all_bytes / max(nbfs, 1) / 1e6, 2),
            "by_direction_MB_per_bfs": {k: round(v / max(nbfs, 1) / 1e6, 2)
                                        for k, v in (("push", self.by_dir.get(1, 0)), ("pull", self.by_dir.get(2, 0)),
                                                     ("hybrid", self.by_dir.get(3, 0)))},
            "note": "sum of every level's algorithmic bytes (push, pull and hybrid levels, from the device "
                    "counters) over the sum of t_bfs, all timed BFS runs",
        }


def account_levels(acct, g, order, raw, keep):
    """Decode the level records the timed loop copied (one bytes blob per BFS, g.level_stats_raw) into the
    byte account; returns every level tagged with its root when `keep` (--levels-json), else []."""
    kept = []
    for r, blob in zip(order, raw):
        lv = g.level_stats_decode(blob)
        acct.add(lv)
        if keep:
            kept.extend(dict(ls, root=r) for ls in lv)
    return kept


def edge_scan_equivalent(m, nv, t_mean_ms):
    b = 8.0 * m + 12.0 * nv
    ach = b / (t_mean_ms * 1e-3) / 1e9
    return {"model": "B = 4*(2M) + 12*n per BFS (SURVEY 8d edge-scan model)", "achieved_GBs": round(ach, 1),
            "frac_of_peak": round(ach / PEAK_HBM_GBS, 4),
            "note": "NOT a bound: an equivalent rate for the bytes a full edge scan would move. Direction "
                    "optimisation skips most edges, so this can exceed 1.0 of peak; see whole_bfs_roofline for "
                    "the bytes actually counted"}


def cpu_baselines(args, g, roots, mcomp, nv):
    """CPU rows on the host cores (rank 0, N = 1): the OpenMP restatement of the BfsSpark map/reduce
    loop and the serial queue BFS of BreadthFirstPaths (SequentialTest.java:24-27), bounded samples."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O  # cpu_baseline leg only

    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    # The GPU box gives one GPU's job a CPU share of 16 threads (OMP_NUM_THREADS=16 there, which jobs
    # must leave alone) while os.cpu_count() / the affinity mask show the whole host; the row runs on that
    # share and says so.  --cpu-threads overrides it.
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0"))
    nthreads = args.cpu_threads or env_threads or affinity
    off, col = g.csr()
    samples, spent = [], 0.0
    for r in roots:
        c0 = time.perf_counter()
        res = O.mapreduce_bfs(nv, off, col, int(r), nthreads=nthreads, max_iters=1)
        dt = time.perf_counter() - c0
        d_gpu = g.bfs(int(r), want_parent=False)[0]
        assert np.array_equal(res["dist"], d_gpu), "CPU oracle and GPU disagree"
        samples.append(mcomp[int(r)] / dt / 1e9)
        spent += dt
        if spent >= args.cpu_baseline_seconds:
            break
    cpu = {
        "value": hmean(samples),
        "unit": "GTEPS",
        "cores": nthreads,
        "nproc": nproc,
        "affinity_cpus": affinity,
        "threads_from": ("--cpu-threads" if args.cpu_threads else
                         "OMP_NUM_THREADS (the job's CPU share on the GPU box)" if env_threads else "sched_getaffinity"),
        "threads_note": ("the GPU box gives one GPU's job a share of 16 host threads and sets OMP_NUM_THREADS=16, which "
                         "jobs must leave as it is; the affinity mask (affinity_cpus) and nproc show the whole host, whose "
                         "other CPUs serve the other GPUs' jobs.  --cpu-threads N runs the row on N threads instead"
                         if env_threads and not args.cpu_threads else None),
        "kind": "port",
        "sample": f"{len(samples)} root(s) of the same scale-{args.scale} graph, oracle orc_mapreduce_bfs "
                  f"(BfsSpark map/reduce restated, OpenMP), {spent:.1f} s; distances asserted equal to the GPU's",
    }
    ser, spent_s = [], 0.0
    for r in roots:
        if spent_s >= args.serial_baseline_seconds:
            break
        c0 = time.perf_counter()
        d_ser, _ = O.csr_bfs(nv, off, col, int(r))
        dt = time.perf_counter() - c0
        d_gpu = g.bfs(int(r), want_parent=False)[0]
        assert np.array_equal(d_ser, d_gpu), "serial CPU BFS and GPU disagree"
        ser.append(mcomp[int(r)] / dt / 1e9)
        spent_s += dt
    serial = {
        "value": hmean(ser) if ser else None,
        "unit": "GTEPS",
        "cores": 1,
        "kind": "port",
        "sample": f"{len(ser)} root(s), oracle orc_csr_bfs: the FIFO-queue BFS of BreadthFirstPaths "
                  f"(algs4.jar!/BreadthFirstPaths.java:93-111, SequentialTest.java:24-27) on the same CSR, one "
                  f"host core, {spent_s:.1f} s; distances asserted equal to the GPU's",
    }
    del off, col
    return cpu, serial


def p1_rehearsal(args, bfsx, roots):
    """The partitioned level loop (what N > 1 runs) at P = 1 on this device with an RCCL communicator of
    one: the same roots, validated, the same device-time basis."""
    ctx = bfsx.Context(0, direction=args.direction)
    try:
        for kv in args.option:
            k, val = kv.split("=", 1)
            ctx.set_option(k, val)
        ctx.comm_init(0, 1, bfsx.comm_unique_id())
        g = ctx.dist_kronecker(args.scale, 0, 1, args.edgefactor, args.seed)
        mc, errs = {}, 0
        for r in roots:
            mc[r] = g.dist_bfs(r)["m_comp"]
            errs += g.validate()["errors"]
        assert errs == 0, f"partitioned P=1 validation failed: {errs}"
        for r in roots:
            g.dist_bfs(r, want_stats=False)
        ctx.synchronize()
        w0 = time.perf_counter()
        ts = [g.dist_bfs(r, want_stats=False) for _ in range(max(1, min(args.steps, 4))) for r in roots]
        ctx.synchronize()
        wall = time.perf_counter() - w0
        order = [r for _ in range(max(1, min(args.steps, 4))) for r in roots]
        g.free()
        return {"value": hmean([mc[r] / (t * 1e-3) / 1e9 for r, t in zip(order, ts)]), "unit": "GTEPS",
                "value_wall": sum(mc[r] for r in order) / wall / 1e9, "bfs_runs": len(order),
                "validated_roots": len(roots), "t_bfs_ms_mean": float(np.mean(ts)),
                "note": "bfsx_dist_bfs with an RCCL communicator of one on the same device: the N > 1 level loop "
                        "with its per-level collectives"}
    finally:
        ctx.close()


def run_single(args):
    bfsx = load_module("bfsx", "bfsx.py")
    ctx = bfsx.Context(0, direction=args.direction)
    for kv in args.option:
        k, val = kv.split("=", 1)
        ctx.set_option(k, val)
    t0 = time.perf_counter()
    g = ctx.kronecker(args.scale, args.edgefactor, args.seed)
    build_s = time.perf_counter() - t0
    nv, nwords = g.nv, (g.nv + 63) // 64
    off_bytes = 4 if g.nnz < 0xFFFFFFFF and "offset_bits=64" not in args.option else 8
    # untimed pass: m_comp per root (Graph500 counts input tuples inside the root's component)
    # and Graph500-style validation of every root's result on the device (bfsx_validate: a result that
    # passes holds exactly the graph's BFS distances)
    roots, mcomp, val_errors, skipped = pick_roots(
        args, g, g.m, lambda r: g.bfs(r, want_dist=False, want_parent=False)[2]["m_comp"],
        lambda: g.validate()["errors"])
    assert val_errors == 0, f"validation failed: {val_errors} violating vertices"
    for _ in range(args.warmup):
        for r in roots:
            g.bfs_device_only(r)

    acct = LevelAccount(nwords, off_bytes)
    pf0 = g.persist_fallbacks()
    ctx.synchronize()
    w0 = time.perf_counter()
    t_bfs, order, raw = [], [], []
    for _ in range(args.steps):
        for r in roots:
            t_bfs.append(g.bfs_device_only(r))
            order.append(r)
            raw.append(g.level_stats_raw(256))  # decoded after the timed region
    ctx.synchronize()
    wall = time.perf_counter() - w0
    persist_fallbacks = g.persist_fallbacks() - pf0
    all_levels = account_levels(acct, g, order, raw, args.levels_json)

    gteps = [mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(order, t_bfs)]
    # output conversion (outside t_bfs): the unpack kernel that turns the internal-id state (+ the pull levels'
    # records) into one (parent, dist) word per original id, device only, for every root: GTEPS with the
    # promised output materialised on the device (value_with_output)
    unpack_ms, resolve_ms, with_out, complete = [], [], [], []
    for r in roots:
        t = g.bfs_device_only(r)
        u = g.unpack_device_only()
        unpack_ms.append(u)
        with_out.append(mcomp[r] / ((t + u) * 1e-3) / 1e9)
        rs = g.last_resolve_ms()  # its internal-id part: dist + parent of every vertex in internal ids
        if rs >= 0:
            resolve_ms.append(rs)
            complete.append(mcomp[r] / ((t + rs) * 1e-3) / 1e9)
    # then the whole bfsx_result call into caller-owned host arrays (allocated and touched once, as a caller
    # reusing its buffers would): unpack + D2H through pinned chunks + the split into int32 dist / int64 parent
    d2h_ms = []
    hd, hp = np.zeros(nv, np.int32), np.zeros(nv, np.int64)
    for r in roots[:4]:
        g.bfs_device_only(r)
        c0 = time.perf_counter()
        g.result(want_parent=True, dist=hd, parent=hp)
        d2h_ms.append((time.perf_counter() - c0) * 1e3)
    del hd, hp
    cpu = serial = None
    if not args.no_cpu_baseline and args.cpu_baseline_seconds > 0 and g.nnz < (1 << 32):
        cpu, serial = cpu_baselines(args, g, roots, mcomp, nv)
    elif g.nnz >= (1 << 32):  # scale >= 29: the host CSR copy alone would be >= 70 GB
        cpu = serial = {"value": None, "note": "skipped: the CPU restatement needs the whole CSR on the host"}

    out = common_fields(args, 1, hmean(gteps), wall, nv, g.m, g.nnz, len(roots), "single")
    out["value_wall"] = sum(mcomp[r] for r in order) / wall / 1e9
    out["roofline"] = acct.roofline("algorithmic bytes of every bottom-up level / its hipEvent duration")
    out["whole_bfs_roofline"] = acct.whole(float(np.sum(t_bfs)), len(t_bfs))
    out["edge_scan_equivalent"] = edge_scan_equivalent(g.m, nv, float(np.mean(t_bfs)))
    out.update({"t_bfs_ms_mean": float(np.mean(t_bfs)), "t_bfs_ms_min": float(np.min(t_bfs)),
                "t_unpack_ms": round(float(np.mean(unpack_ms)), 4),
                "value_with_output": hmean(with_out),
                "t_resolve_ms": round(float(np.mean(resolve_ms)), 4) if resolve_ms else None,
                "value_complete": hmean(complete) if complete else None,
                "t_result_copy_ms": round(float(np.mean(d2h_ms)), 3),
                "output_note": "t_unpack_ms: device time of the result materialisation outside t_bfs, mean over "
                               "the roots: the push levels' log scattered and the pull levels' records folded into "
                               "the per-vertex state (t_resolve_ms: then a dist and a parent exist for every vertex "
                               "in internal ids, Graph500 kernel 2's output), then one (parent, dist) word per "
                               "original id; value_complete: harmonic-mean GTEPS over t_bfs + t_resolve; "
                               "value_with_output: over t_bfs + t_unpack (the promised output in the caller's ids "
                               "on the device); t_result_copy_ms: host wall time of bfsx_result "
                               "into reused caller arrays (unpack + D2H through pinned chunks + split into int32 dist "
                               "and int64 parent), 4 roots",
                "persist_fallbacks": persist_fallbacks,
                "bfs_runs": len(t_bfs), "m_comp_mean": float(np.mean([mcomp[r] for r in order])),
                "graph_build_s": round(build_s, 3),
                "validation": {"roots": len(roots), "errors": val_errors, "skipped_tiny_component": skipped,
                               "rules": "Graph500 kernel-2 + BreadthFirstPaths.check, on device (bfsx_validate)"},
                "cpu_baseline": cpu, "cpu_baseline_serial": serial})
    if args.levels_json:
        with open(args.levels_json, "w") as f:
            json.dump(all_levels, f)
    g.free()
    if not args.no_p1:
        # RCCL prints its banner on the process's C-level stdout; the contract is ONE JSON line
        sys.stdout.flush()
        real_stdout = os.dup(1)
        os.dup2(2, 1)
        try:
            out["partitioned_p1"] = p1_rehearsal(args, bfsx, roots)
        except (bfsx.BfsxError, AssertionError) as e:
            out["partitioned_p1"] = {"error": str(e)}
        finally:
            sys.stdout.flush()
            os.dup2(real_stdout, 1)
            os.close(real_stdout)
    ctx.close()
    print(json.dumps(out), flush=True)


def rccl_debug_env(rank):
    """Ask RCCL to log its connection setup (NCCL_DEBUG=INFO, INIT/P2P/NET subsystems) into a per-rank file, so
    that rank 0 can report which transport its peers were connected over (its warnings are echoed to stderr
    afterwards); left alone when the caller already directs RCCL's log to a file (NCCL_DEBUG_FILE) or asked for
    more than INFO.  Must run before the first RCCL call."""
    if os.environ.get("NCCL_DEBUG_FILE") or os.environ.get("NCCL_DEBUG", "").upper() in ("INFO", "TRACE"):
        return None
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"bfsx_rccl_{os.getpid()}_rank{rank}.log")
    os.environ.update({"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,P2P,NET,GRAPH", "NCCL_DEBUG_FILE": path})
    return path


def rccl_transports(path):
    """Transport summary of one rank's RCCL log: how many channel connections went over each transport
    ("via P2P/IPC", "via NET/Socket/0", "via SHM/direct/direct", ...) and the communicator sizes RCCL reported."""
    import re
    if not path or not os.path.exists(path):
        return {"note": "RCCL's log directed by the caller (NCCL_DEBUG_FILE / NCCL_DEBUG=INFO|TRACE): no transport summary"}
    via, nranks = {}, set()
    with open(path, errors="replace") as f:
        for ln in f:
            if " WARN " in ln:
                print(ln.rstrip(), file=sys.stderr)
            m = re.search(r" via ([A-Za-z0-9_]+(?:/[A-Za-z0-9_]+)?)", ln)
            if m:
                via[m.group(1)] = via.get(m.group(1), 0) + 1
            m = re.search(r"nRanks (\d+)", ln)
            if m:
                nranks.add(int(m.group(1)))
    try:
        os.unlink(path)
    except OSError:
        pass
    return {"connections_by_transport": via, "comm_sizes_reported": sorted(nranks),
            "note": "rank 0's RCCL INFO log (INIT/P2P/NET): P2P = GPU peer access over xGMI, SHM = host shared "
                    "memory, NET = network (the one-GPU socket rehearsal)"}


def comm_split(args, g, dist, torch, roots, world):
    """Untimed diagnostic pass (option comm_timing): device time of every collective kind per BFS, and of every
    level, each the max over the ranks -- where the time of an N > 1 BFS goes."""
    n = min(args.comm_split_roots, len(roots))
    if n <= 0:
        return None
    g.ctx.set_option("comm_timing", "on")
    kinds = g.COMM_KINDS
    acc, levels = np.zeros(2 * len(kinds)), None
    try:
        for r in roots[:n]:
            g.dist_bfs(r, want_stats=False)
            ct = g.comm_times()
            t = torch.tensor([ct[k][0] for k in kinds] + [float(ct[k][1]) for k in kinds], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            acc += t.numpy()
        ls = g.level_stats(256)
        lt = torch.tensor([x["kernel_ms"] for x in ls], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        levels = [{"level": x["level"], "direction": x["direction"], "ms_max_over_ranks": round(float(v), 4)}
                  for x, v in zip(ls, lt.tolist())]
    finally:
        g.ctx.set_option("comm_timing", "off")
    return {"roots": n,
            "ms_per_bfs": {k: round(acc[i] / n, 4) for i, k in enumerate(kinds)},
            "calls_per_bfs": {k: round(acc[len(kinds) + i] / n, 2) for i, k in enumerate(kinds)},
            "levels_last_bfs": levels,
            "note": "hipEvents around every collective of the level loop on the BFS stream (a span includes the wait "
                    "for the slowest rank), summed per BFS, max over ranks, mean over the roots; levels: device "
                    "time of each level of the last root, max over ranks"}


def scale30_leg(args, bfsx, ctx, dist, torch, rank, world, shared_device):
    """BASELINE configs[4]: RMAT scale 30, edgefactor 16, 1-D partitioned over the same ranks and communicator,
    after the scale-26 metric: the first args.scale30_roots validated roots, one timed BFS each (device time, max
    over ranks).  Every rank takes part; a rank that cannot build its slice makes every rank skip the leg."""
    t0 = time.perf_counter()
    g, err = None, ""
    try:
        if shared_device:
            for r in range(world):
                if r == rank:
                    g = ctx.dist_kronecker(30, rank, world, args.edgefactor, args.seed)
                    ctx.synchronize()
                dist.barrier()
        else:
            g = ctx.dist_kronecker(30, rank, world, args.edgefactor, args.seed)
            ctx.synchronize()
    except bfsx.BfsxError as e:
        err = str(e)
    ok = torch.tensor([0 if err else 1], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok) == 0:
        if g is not None:
            g.free()
        return {"error": f"build failed on some rank (this rank: {err or 'ok'})"}
    build_s = time.perf_counter() - t0
    sub = argparse.Namespace(**dict(vars(args), roots=args.scale30_roots))
    roots, mcomp, val_errors, skipped = pick_roots(sub, g, g.m, lambda r: g.dist_bfs(r)["m_comp"],
                                                   lambda: g.validate()["errors"])
    ctx.synchronize()
    dist.barrier()
    ts = [g.dist_bfs(r, want_stats=False) for r in roots]
    tt = torch.tensor(ts, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    split = comm_split(argparse.Namespace(comm_split_roots=min(2, len(roots))), g, dist, torch, roots, world)
    part, m_tuples = g.partition(), g.m
    g.free()
    return {"metric": f"GTEPS (harmonic mean, {len(roots)} roots) on RMAT scale-30", "workload": "kronecker-s30-ef16",
            "value": hmean([mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(roots, tt.tolist())]), "unit": "GTEPS",
            "n_gpus": world, "nv": part["nv_global"], "m_tuples": m_tuples,
            "t_bfs_ms_mean": float(np.mean(tt.tolist())), "graph_build_s": round(build_s, 3),
            "validation": {"roots": len(roots), "errors": val_errors, "skipped_tiny_component": skipped},
            "comm_split": split,
            "note": "BASELINE configs[4]: one timed BFS per validated root after the scale-26 metric, device time "
                    "(max over ranks), the same partitioned level loop and RCCL communicator"}


def run_dist(args, world, rank, local_rank):
    """One process per GPU: the partitioned level loop and its RCCL exchange run inside libbfsx
    (bfsx_dist_bfs); torch.distributed (gloo, host only) is used for the rendezvous -- the RCCL unique
    id, barriers and the max over ranks of the per-root times -- never on the data path."""
    import torch
    import torch.distributed as dist

    arm_deadline(args.deadline, f"rank {rank} of {world}")
    shared_device = os.environ.get("BFSX_RCCL_SHARED_DEVICE") == "1"
    if shared_device:
        # rehearsal of N > 1 RCCL on a box with fewer GPUs than ranks: RCCL refuses two ranks on one device of
        # one host, so every rank presents a host id of its own and the ranks talk over RCCL's socket transport
        # (loopback). Never set by the driver's runs; see DESIGN §7.
        os.environ["NCCL_HOSTID"] = f"bfsx-rehearsal-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    rccl_log = rccl_debug_env(rank) if world > 1 else None
    # Gloo and RCCL print banners on the process's C-level stdout; the contract is ONE JSON line, so
    # fd 1 points at stderr until the result is printed
    sys.stdout.flush()
    real_stdout = os.dup(1)
    os.dup2(2, 1)
    dist.init_process_group("gloo")
    bfsx = load_module("bfsx", "bfsx.py")
    # one GPU per rank: local_rank indexes the visible devices (a launcher that pins each rank to its
    # own device with HIP_VISIBLE_DEVICES leaves exactly one visible)
    ndev = torch.cuda.device_count()
    device = local_rank if local_rank < ndev else (local_rank % max(ndev, 1))
    ctx = bfsx.Context(device, direction=args.direction)
    for kv in args.option:
        k, val = kv.split("=", 1)
        ctx.set_option(k, val)
    uid = [bfsx.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.comm_init(rank, world, uid[0])
    t0 = time.perf_counter()
    if shared_device:
        # ranks sharing one GPU build one after another: the build's temporaries are several times its slice
        # (four concurrent scale-30 builds do not fit one GPU's 288 GB; on their own GPUs they run at once)
        g = None
        for r in range(world):
            if r == rank:
                g = ctx.dist_kronecker(args.scale, rank, world, args.edgefactor, args.seed)
                ctx.synchronize()
            dist.barrier()
    else:
        g = ctx.dist_kronecker(args.scale, rank, world, args.edgefactor, args.seed)
        ctx.synchronize()
    build_s = time.perf_counter() - t0
    part = g.partition()
    # untimed, collective (m_comp is all-reduced, so every rank keeps the same roots): m_comp and
    # Graph500-style validation of every root
    roots, mcomp, val_errors, skipped = pick_roots(args, g, g.m, lambda r: g.dist_bfs(r)["m_comp"],
                                                   lambda: g.validate()["errors"])
    assert val_errors == 0, f"validation failed: {val_errors} violating vertices"
    for _ in range(args.warmup):
        for r in roots:
            g.dist_bfs(r, want_stats=False)

    off_bytes = 4 if g.nnz < 0xFFFFFFFF and "offset_bits=64" not in args.option else 8
    acct = LevelAccount(part["chunk"] // 64, off_bytes, code_bytes=0)  # a partition's pull parents are explicit
    # The K steps run back to back between two barrier + device-synchronise brackets (the contract's
    # timed region); every BFS is collective, so the ranks stay in step through its RCCL calls.
    ctx.synchronize()
    dist.barrier()
    w0 = time.perf_counter()
    dev_ms, order, raw = [], [], []
    for _ in range(args.steps):
        for r in roots:
            dev_ms.append(g.dist_bfs(r, want_stats=False))
            order.append(r)
            if rank == 0:
                raw.append(g.level_stats_raw(256))  # decoded after the timed region
    ctx.synchronize()
    wall_local = time.perf_counter() - w0
    all_levels = account_levels(acct, g, order, raw, args.levels_json)
    dist.barrier()
    tt = torch.tensor([wall_local] + dev_ms, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)  # max over ranks
    wall = float(tt[0])
    dev_max = tt[1:].tolist()  # per BFS: the slowest rank's device time (source init -> last level)
    m_total = float(sum(mcomp[r] for r in order))
    value = hmean([mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(order, dev_max)])  # same basis as N = 1
    nnz = torch.tensor([g.nnz], dtype=torch.int64)
    dist.all_reduce(nnz)
    if rank == 0:
        out = common_fields(args, world, value, wall, part["nv_global"], g.m, int(nnz), len(roots),
                            f"1d-partition dp{world} (RCCL all-to-allv + all-gather + all-reduce in libbfsx)")
        out["scaling"] = "strong"
        out["value_wall"] = m_total / wall / 1e9
        out["roofline"] = acct.roofline("rank 0; a bottom-up level's time includes its frontier all-gather")
        out["whole_bfs_roofline"] = dict(acct.whole(float(np.sum(dev_max)), len(dev_max)),
                                         note="rank 0's level bytes over the max-over-ranks t_bfs")
        out.update({"t_bfs_ms_mean": float(np.mean(dev_max)), "bfs_runs": len(dev_max),
                    "m_comp_mean": float(np.mean([mcomp[r] for r in order])),
                    "graph_build_s": round(build_s, 3), "cpu_baseline": None,
                    "validation": {"roots": len(roots), "errors": val_errors, "skipped_tiny_component": skipped,
                                   "rules": "Graph500 kernel-2 + BreadthFirstPaths.check, on device, collective"},
                    "levels_last": [{k: ls[k] for k in ("level", "direction", "frontier_in", "frontier_out",
                                                        "kernel_ms")} for ls in g.level_stats(256)]})
    split = comm_split(args, g, dist, torch, roots, world) if world > 1 else None
    if rank == 0:
        out["comm_split"] = split
        out["rccl"] = dict(world_size=world, devices_visible=ndev, device_of_rank0=device,
                           shared_device_rehearsal=shared_device, **rccl_transports(rccl_log))
    elif rccl_log and os.path.exists(rccl_log):
        os.unlink(rccl_log)
    if rank == 0 and args.levels_json:
        with open(args.levels_json, "w") as f:
            json.dump(all_levels, f)
    g.free()
    s30 = args.scale30_roots if args.scale30_roots >= 0 else (4 if world > 1 and args.scale == 26 else 0)
    if s30 > 0:
        args.scale30_roots = s30
        try:
            leg = scale30_leg(args, bfsx, ctx, dist, torch, rank, world, shared_device)
        except (bfsx.BfsxError, AssertionError) as e:
            leg = {"error": str(e)}
        if rank == 0:
            out["scale30"] = leg
    ctx.close()
    dist.destroy_process_group()
    sys.stdout.flush()
    os.dup2(real_stdout, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)


def launch_ranks(args):
    """`--gpus N` (N > 1) run without a launcher -- how the driver calls it: start N ranks as ONE child
    process, `python -m torch.distributed.run --nproc-per-node N ... bench.py <the same arguments>`, before
    this process touches HIP or torch, relay the child's single JSON line to stdout and return its exit
    code.  Everything else the child prints goes to stderr."""
    import subprocess

    # the c10d rendezvous binds port 0 itself (a port probed here and handed over could be taken in between:
    # ADVICE r3); --local-addr keeps MASTER_ADDR at 127.0.0.1 (the container hostname may not resolve)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1",
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] --gpus {args.gpus}: launching {' '.join(cmd)}", file=sys.stderr, flush=True)
    # the ranks arm --deadline themselves; this bound (a minute later) also covers a launcher that hangs, and
    # takes the whole process group (the launcher and every rank) down with it
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=args.deadline + 60 if args.deadline > 0 else None)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        print(f"[bench] ranks still running {args.deadline + 60:.0f} s after the launch: killed", file=sys.stderr,
              flush=True)
        return 124

    class R:
        returncode, stdout = p.returncode, out
    r = R
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    js = [ln for ln in lines if ln.lstrip().startswith("{")]
    for ln in lines:
        if ln not in js:
            print(ln, file=sys.stderr)
    if r.returncode != 0 or len(js) != 1:
        print(f"[bench] ranks exited {r.returncode} with {len(js)} JSON line(s)", file=sys.stderr, flush=True)
        return r.returncode or 1
    print(js[0], flush=True)
    return 0


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus and not (world == 1 and args.dist):
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a different GPU count",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1 or args.dist:
        run_dist(args, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    else:
        run_single(args)


if __name__ == "__main__":
    main()
