"""Benchmark: GTEPS (harmonic mean over roots) on Graph500 Kronecker scale-26, edgefactor 16.

A "step" is one BFS from one root over the device-resident CSR (BASELINE.json configs[3]); the graph
is generated and built on the GPU before the timed region.  TEPS per root = m_comp / t with m_comp =
the input tuples inside the root's component (Graph500 convention); value = harmonic mean GTEPS over
the K timed roots (= K*m / sum t when every root lies in the giant component).

  N = 1: t = device time from source init to the last level (hipEvents inside libbfsx.so).
  N > 1: launched as one process per GPU (torch.distributed.run); the graph is 1-D partitioned over
         the ranks and libbfsx runs the level loop with its own RCCL communicator (all-to-allv of
         owner-routed pairs, all-gather of frontier bitmaps, all-reduce of the level counters);
         t = the max over ranks of the wall time of one BFS, bracketed by barrier + device sync.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline accounting.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu-baseline]
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
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, file))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def level_bytes(ls, nwords):
    """Algorithmic bytes of one level."""
    if ls["direction"] == 2:  # bottom-up: visited word read + next word write, top1 of every live
        # candidate, rest[] (2nd..4th neighbours + degree, 16 B) of every top1 miss, the uint32 offset pair
        # of each row walked past its first four entries (`claims`), the adjacency entries walked there,
        # the packed state word of every vertex found.  Frontier-bit probes are not counted: the 8 MiB
        # bitmap is cache-resident.
        return (16 * nwords + 4 * max(ls["unvisited_in"], 0) + 16 * ls["stage2"] + 8 * ls["claims"]
                + 4 * ls["walked"] + 8 * ls["frontier_out"])
    # top-down: queue read, row offsets (2 x 8 B per frontier vertex), adjacency rows, winners'
    # dist+parent writes, queue append, degree lookups of the winners
    return 20 * ls["frontier_in"] + 4 * max(ls["mf_in"], 0) + 28 * ls["frontier_out"]


def hmean(xs):
    return len(xs) / sum(1.0 / x for x in xs)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED2026)
    ap.add_argument("--root-seed", type=lambda x: int(x, 0), default=0x5EED)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--direction", default="auto")
    ap.add_argument("--levels-json", default="")
    ap.add_argument("--option", action="append", default=[], help="libbfsx option key=value")
    ap.add_argument("--dist", action="store_true", help="use the partitioned path even on one rank (rehearsal)")
    return ap.parse_args()


def common_fields(args, world, value, wall, nv, m, nnz, nroots, parallelism):
    return {
        "metric": f"GTEPS (harmonic mean, {args.steps} roots) on RMAT scale-{args.scale}",
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
            "direction": args.direction,
            "parallelism": parallelism,
        },
    }


def measured_traffic(kernel="k_bu"):
    """Per-launch HBM bytes of `kernel` from the newest committed PMC summary (profiles/<tag>_hbm.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes),
    used only while kernels_bfs.hip still hashes to the source it was measured on."""
    import glob
    import hashlib
    src = os.path.join(PKG, "csrc", "kernels_bfs.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        names = [n for n in rec.get("kernels", {}) if n == kernel or n.startswith(kernel + "<")]
        if rec.get("kernels_bfs_sha") == sha and names:
            # the instantiation with the most launches (the hybrid levels' hub sweep is a second one)
            k = max((rec["kernels"][n] for n in names), key=lambda x: x.get("launches", 0))
            out = {"traffic": round(k["traffic_B"] / 1e6, 1), "traffic_raw": round(k["traffic_raw_B"] / 1e6, 1),
                   "traffic_source": os.path.relpath(path, ROOT), "fetch_correction": rec.get("fetch_correction")}
            if k.get("avg_ms_trace"):  # fabric-side rate of the same launches (rocprof trace durations)
                out["traffic_GBs"] = round(k["traffic_B"] / (k["avg_ms_trace"] * 1e-3) / 1e9, 1)
                out["traffic_frac"] = round(out["traffic_GBs"] / PEAK_HBM_GBS, 4)
            return out
    return {"traffic": None, "traffic_source": "no PMC summary for this kernel source"}


def roofline(bu_bytes, bu_ms, bu_launches, note):
    ach = (bu_bytes / bu_launches) / ((bu_ms / bu_launches) * 1e-3) / 1e9 if bu_launches else 0.0
    tr = measured_traffic()
    return {
        "bound": "hbm",
        "kernel": "k_bu (bottom-up pull)",
        "achieved": round(ach, 1),
        "peak": PEAK_HBM_GBS,
        "unit": "GB/s",
        "frac": round(ach / PEAK_HBM_GBS, 4),
        "traffic": tr.pop("traffic"),
        "traffic_unit": "MB per launch (FETCH_SIZE x correction + WRITE_SIZE)",
        "algorithmic": round(bu_bytes / max(bu_launches, 1) / 1e6, 1),
        **tr,
        "launches": bu_launches,
        "avg_launch_ms": round(bu_ms / max(bu_launches, 1), 4),
        "note": note,
    }


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
    roots = g.sample_roots(min(max(args.steps, 1), 64), seed=args.root_seed)
    # untimed pass: m_comp per root (Graph500 counts input tuples inside the root's component)
    # and Graph500-style validation of every root's result on the device (bfsx_validate: a result that
    # passes holds exactly the graph's BFS distances)
    mcomp, val_errors = {}, 0
    for r in roots:
        _, _, st = g.bfs(int(r), want_dist=False, want_parent=False)
        mcomp[int(r)] = st["m_comp"]
        val_errors += g.validate()["errors"]
    assert val_errors == 0, f"validation failed: {val_errors} violating vertices"
    order = [int(roots[i % len(roots)]) for i in range(args.warmup + args.steps)]
    for r in order[: args.warmup]:
        g.bfs_device_only(r)

    ctx.synchronize()
    w0 = time.perf_counter()
    t_bfs, bu_bytes, bu_ms, bu_launches, all_levels = [], 0, 0.0, 0, []
    for r in order[args.warmup:]:
        t_bfs.append(g.bfs_device_only(r))
        for ls in g.level_stats(256):
            if ls["direction"] == 2:
                bu_bytes += level_bytes(ls, nwords)
                bu_ms += ls["kernel_ms"]
                bu_launches += 1
            if args.levels_json:
                all_levels.append(dict(ls, root=r))
    ctx.synchronize()
    wall = time.perf_counter() - w0

    steps_roots = order[args.warmup:]
    gteps = [mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(steps_roots, t_bfs)]
    bfs_bytes = 8.0 * g.m + 12.0 * nv  # SURVEY 8(d) edge-scan model: B = 4*(2M) + 12*n per BFS
    bfs_ach = bfs_bytes / (np.mean(t_bfs) * 1e-3) / 1e9

    cpu = None
    if not args.no_cpu_baseline and args.cpu_baseline_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py as O  # cpu_baseline leg only

        nthreads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
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
            "kind": "port",
            "sample": f"{len(samples)} root(s) of the same scale-{args.scale} graph, oracle orc_mapreduce_bfs "
                      f"(BfsSpark map/reduce restated, OpenMP), {spent:.1f} s; distances asserted equal to the GPU's",
        }
        del off, col

    out = common_fields(args, 1, hmean(gteps), wall, nv, g.m, g.nnz, len(roots), "single")
    out["roofline"] = roofline(bu_bytes, bu_ms, bu_launches,
                               "algorithmic bytes of every bottom-up level / its hipEvent duration")
    out["bfs_roofline"] = {"model": "B = 4*(2M) + 12*n per BFS (SURVEY 8d)",
                           "achieved_GBs": round(bfs_ach, 1), "frac": round(bfs_ach / PEAK_HBM_GBS, 4)}
    out.update({"t_bfs_ms_mean": float(np.mean(t_bfs)), "t_bfs_ms_min": float(np.min(t_bfs)),
                "m_comp_mean": float(np.mean([mcomp[r] for r in steps_roots])), "graph_build_s": round(build_s, 3),
                "validation": {"roots": len(roots), "errors": val_errors,
                               "rules": "Graph500 kernel-2 + BreadthFirstPaths.check, on device (bfsx_validate)"},
                "cpu_baseline": cpu})
    if args.levels_json:
        with open(args.levels_json, "w") as f:
            json.dump(all_levels, f)
    print(json.dumps(out), flush=True)
    g.free()
    ctx.close()


def run_dist(args, world, rank, local_rank):
    """One process per GPU: the partitioned level loop and its RCCL exchange run inside libbfsx
    (bfsx_dist_bfs); torch.distributed (gloo, host only) is used for the rendezvous -- the RCCL unique
    id, barriers and the max over ranks of the per-root times -- never on the data path."""
    import torch
    import torch.distributed as dist

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
    g = ctx.dist_kronecker(args.scale, rank, world, args.edgefactor, args.seed)
    ctx.synchronize()
    build_s = time.perf_counter() - t0
    part = g.partition()
    roots = [int(r) for r in g.sample_roots(min(max(args.steps, 1), 64), seed=args.root_seed)]
    mcomp, val_errors = {}, 0
    for r in roots:  # untimed, collective: m_comp and Graph500-style validation of every root
        mcomp[r] = g.dist_bfs(r)["m_comp"]
        val_errors += g.validate()["errors"]
    assert val_errors == 0, f"validation failed: {val_errors} violating vertices"
    order = [roots[i % len(roots)] for i in range(args.warmup + args.steps)]
    for r in order[: args.warmup]:
        g.dist_bfs(r, want_stats=False)

    # The K roots run back to back between two barrier + device-synchronise brackets (the contract's
    # timed region); every BFS is collective, so the ranks stay in step through its RCCL calls and a
    # per-root host barrier would only add its own skew to the measurement.
    ctx.synchronize()
    dist.barrier()
    w0 = time.perf_counter()
    dev_ms = [g.dist_bfs(r, want_stats=False) for r in order[args.warmup:]]
    ctx.synchronize()
    wall_local = time.perf_counter() - w0
    dist.barrier()
    tt = torch.tensor([wall_local] + dev_ms, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)  # max over ranks
    wall = float(tt[0])
    dev_max = tt[1:].tolist()  # per root: the slowest rank's device time (source init -> last level)
    steps_roots = order[args.warmup:]
    m_total = float(sum(mcomp[r] for r in steps_roots))
    value = m_total / wall / 1e9  # = harmonic mean of per-root TEPS when the roots share one component
    nnz = torch.tensor([g.nnz], dtype=torch.int64)
    dist.all_reduce(nnz)
    if rank == 0:
        out = common_fields(args, world, value, wall, part["nv_global"], g.m, int(nnz), len(roots),
                            f"1d-partition dp{world} (RCCL all-to-allv + all-gather + all-reduce in libbfsx)")
        out["scaling"] = "strong"
        bu_bytes, bu_ms, bu_launches = 0, 0.0, 0
        for ls in g.level_stats(256):  # rank 0, last timed BFS
            if ls["direction"] == 2:
                bu_bytes += level_bytes(ls, part["chunk"] // 64)
                bu_ms += ls["kernel_ms"]
                bu_launches += 1
        out["roofline"] = roofline(bu_bytes, bu_ms, bu_launches,
                                   "rank 0, last BFS; a bottom-up level's time includes its frontier all-gather")
        out.update({"t_bfs_ms_mean": wall * 1e3 / max(len(steps_roots), 1),
                    "t_bfs_dev_ms_max_mean": float(np.mean(dev_max)),
                    "hmean_gteps_device": hmean([mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(steps_roots, dev_max)]),
                    "m_comp_mean": float(np.mean([mcomp[r] for r in steps_roots])),
                    "graph_build_s": round(build_s, 3), "cpu_baseline": None,
                    "validation": {"roots": len(roots), "errors": val_errors,
                                   "rules": "Graph500 kernel-2 + BreadthFirstPaths.check, on device, collective"},
                    "levels_last": [{k: ls[k] for k in ("level", "direction", "frontier_in", "frontier_out",
                                                        "kernel_ms")} for ls in g.level_stats(256)]})
    g.free()
    ctx.close()
    dist.destroy_process_group()
    sys.stdout.flush()
    os.dup2(real_stdout, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.dist:
        run_dist(args, world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    else:
        run_single(args)


if __name__ == "__main__":
    main()
