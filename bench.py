"""Benchmark: GTEPS (harmonic mean over roots) on Graph500 Kronecker scale-26, edgefactor 16.

A "step" is one BFS from one root over the device-resident CSR (BASELINE.json configs[3]); the graph
is generated and built on the GPU before the timed region.  Per root, t_bfs = device time from
source init to the last level (hipEvents inside libbfsx.so); TEPS = m_comp / t_bfs with m_comp = the
input tuples inside the root's component (Graph500 convention).  value = harmonic mean GTEPS over the
K timed roots (= K*m / sum t when every root lies in the giant component).

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline accounting.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S] [--no-cpu-baseline]
"""
import argparse
import importlib.util
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def load_bfsx():
    spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bfsx"] = mod
    spec.loader.exec_module(mod)
    return mod


def level_bytes(ls, nwords):
    """Algorithmic bytes of one level (DESIGN.md "Roofline accounting")."""
    if ls["direction"] == 2:  # bottom-up: visited word read + next word write, row offsets of the
        # unvisited candidates, adjacency entries actually scanned, dist+parent of the found
        return 16 * nwords + 8 * ls["unvisited_in"] + 4 * ls["scanned"] + 8 * ls["frontier_out"]
    # top-down: queue read, row offsets (2 x 8 B per frontier vertex), adjacency rows, winners'
    # dist+parent writes, queue append, degree lookups of the winners
    return 4 * ls["frontier_in"] + 16 * ls["frontier_in"] + 4 * max(ls["mf_in"], 0) + 28 * ls["frontier_out"]


def main():
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
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    bfsx = load_bfsx()
    dist_mod = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        dist_mod.init_process_group("gloo")

    def barrier():
        if dist_mod is not None:
            dist_mod.barrier()

    ctx = bfsx.Context(local_rank, direction=args.direction)
    for kv in args.option:
        k, val = kv.split("=", 1)
        ctx.set_option(k, val)
    t0 = time.perf_counter()
    g = ctx.kronecker(args.scale, args.edgefactor, args.seed)
    build_s = time.perf_counter() - t0
    nv, nwords = g.nv, (g.nv + 63) // 64
    n_roots = max(args.steps, 1)
    roots = g.sample_roots(min(n_roots, 64), seed=args.root_seed + rank)
    # untimed pass: m_comp per root (Graph500 counts input tuples inside the root's component)
    mcomp = {}
    for r in roots:
        _, _, st = g.bfs(int(r), want_dist=False, want_parent=False)
        mcomp[int(r)] = st["m_comp"]
    order = [int(roots[i % len(roots)]) for i in range(args.warmup + args.steps)]
    for r in order[: args.warmup]:
        g.bfs_device_only(r)

    ctx.synchronize()
    barrier()
    w0 = time.perf_counter()
    t_bfs, bu_bytes, bu_ms, bu_launches, td_ms, all_levels = [], 0, 0.0, 0, 0.0, []
    for r in order[args.warmup:]:
        t_bfs.append(g.bfs_device_only(r))
        for ls in g.level_stats(256):
            if ls["direction"] == 2:
                bu_bytes += level_bytes(ls, nwords)
                bu_ms += ls["kernel_ms"]
                bu_launches += 1
            else:
                td_ms += ls["kernel_ms"]
            if args.levels_json:
                all_levels.append(dict(ls, root=r))
    ctx.synchronize()
    barrier()
    wall = time.perf_counter() - w0
    if dist_mod is not None:
        import torch

        tw = torch.tensor([wall], dtype=torch.float64)
        dist_mod.all_reduce(tw, op=dist_mod.ReduceOp.MAX)
        wall = float(tw[0])

    steps_roots = order[args.warmup:]
    gteps = [mcomp[r] / (t * 1e-3) / 1e9 for r, t in zip(steps_roots, t_bfs)]
    hmean = len(gteps) / sum(1.0 / x for x in gteps)
    total = hmean
    if dist_mod is not None:  # independent replicas: aggregate = sum of per-rank rates
        th = torch.tensor([hmean], dtype=torch.float64)
        dist_mod.all_reduce(th, op=dist_mod.ReduceOp.SUM)
        total = float(th[0])
    m_mean = float(np.mean([mcomp[r] for r in steps_roots]))
    # survey 8(d) edge-scan model: B = 4*(2M) + 12*n per BFS
    bfs_bytes = 8.0 * g.m + 12.0 * nv
    bfs_ach = bfs_bytes / (np.mean(t_bfs) * 1e-3) / 1e9
    bu_ach = (bu_bytes / bu_launches) / ((bu_ms / bu_launches) * 1e-3) / 1e9 if bu_launches else 0.0

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_py as O  # cpu_baseline leg only

        nthreads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        off, col = g.csr()
        samples = []
        spent = 0.0
        for r in roots:
            c0 = time.perf_counter()
            res = O.mapreduce_bfs(nv, off, col, int(r), nthreads=nthreads, max_iters=1)
            dt = time.perf_counter() - c0
            d_gpu, _ = g.bfs(int(r), want_parent=False)[:2]
            assert np.array_equal(res["dist"], d_gpu), "CPU oracle and GPU disagree"
            samples.append(mcomp[int(r)] / dt / 1e9)
            spent += dt
            if spent >= args.cpu_baseline_seconds:
                break
        cpu = {
            "value": len(samples) / sum(1.0 / x for x in samples),
            "unit": "GTEPS",
            "cores": nthreads,
            "kind": "port",
            "sample": f"{len(samples)} root(s) of the same scale-{args.scale} graph, oracle "
                      f"orc_mapreduce_bfs (BfsSpark map/reduce restated, OpenMP), {spent:.1f} s",
        }
        del off, col

    out = {
        "metric": f"GTEPS (harmonic mean, {len(t_bfs)} roots) on RMAT scale-{args.scale}",
        "value": total,
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall * 1e3 / max(args.steps, 1),
        "higher_is_better": True,
        "scaling": "weak" if world > 1 else "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (Graph500 Kronecker A/B/C/D=.57/.19/.19/.05, generated on device)",
        "config": {
            "workload": f"kronecker-s{args.scale}-ef{args.edgefactor}",
            "scale": args.scale,
            "edgefactor": args.edgefactor,
            "seed": hex(args.seed),
            "nv": nv,
            "m_tuples": g.m,
            "nnz_directed": g.nnz,
            "roots": len(roots),
            "direction": args.direction,
            "parallelism": "replica" if world > 1 else "single",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_bu (bottom-up pull)",
            "achieved": round(bu_ach, 1),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(bu_ach / PEAK_HBM_GBS, 4),
            "traffic": None,
            "launches": bu_launches,
            "avg_launch_ms": round(bu_ms / max(bu_launches, 1), 4),
        },
        "bfs_roofline": {
            "model": "B = 4*(2M) + 12*n per BFS (SURVEY 8d)",
            "achieved_GBs": round(bfs_ach, 1),
            "frac": round(bfs_ach / PEAK_HBM_GBS, 4),
        },
        "t_bfs_ms_mean": float(np.mean(t_bfs)),
        "t_bfs_ms_min": float(np.min(t_bfs)),
        "m_comp_mean": m_mean,
        "graph_build_s": round(build_s, 3),
        "cpu_baseline": cpu,
    }
    if args.levels_json and rank == 0:
        with open(args.levels_json, "w") as f:
            json.dump(all_levels, f)
    if rank == 0:
        print(json.dumps(out), flush=True)
    g.free()
    ctx.close()
    if dist_mod is not None:
        dist_mod.destroy_process_group()


if __name__ == "__main__":
    main()
