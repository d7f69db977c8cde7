"""Partitioned-BFS rehearsal on ONE device: P ranks as an in-process exchange group (one host thread per
rank, device copies for the exchange) running the same native level loop (bfsx_dist_bfs) that
bench.py --gpus P runs over RCCL.  Purpose: show that BASELINE.json configs[4] (scale 30, 1-D
partition over 8 ranks) builds, traverses and VALIDATES (bfsx_validate, collective), and record its
level structure and exchange volumes.  The times are NOT multi-GPU numbers: all P ranks share one
MI355X's CUs and HBM, and the exchange is device-to-device copies instead of xGMI.

  python tools/dist_rehearsal.py --scale 30 --nranks 8 --roots 2 [--single]

--single also builds the whole graph on the one device (the single-GPU path at that scale) after the
partition is freed and checks that its distances equal the partitioned result.
"""
import argparse
import ctypes as C
import importlib.util
import json
import os
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)


def mem_free_gb():
    hip = C.CDLL("libamdhip64.so")
    free, total = C.c_size_t(), C.c_size_t()
    hip.hipMemGetInfo(C.byref(free), C.byref(total))
    return free.value / 1e9


def run_ranks(P, fn):
    res, errs = [None] * P, []

    def work(r):
        try:
            res[r] = fn(r)
        except Exception as e:  # noqa: BLE001 -- reported by the caller
            errs.append(f"rank {r}: {e!r}")

    ths = [threading.Thread(target=work, args=(r,)) for r in range(P)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    if errs or any(t.is_alive() for t in ths):
        raise RuntimeError(errs or "rank thread hung")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=30)
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--roots", type=int, default=2)
    ap.add_argument("--single", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    P = a.nranks
    out = {"scale": a.scale, "nranks": P, "device_free_GB_start": round(mem_free_gb(), 1),
           "note": "in-process group on ONE MI355X: ranks share the device, exchange = device copies; "
                   "times are not multi-GPU numbers"}
    ctxs = [bfsx.Context(0) for _ in range(P)]
    bfsx.local_group(ctxs)
    graphs = []
    t0 = time.perf_counter()
    for r in range(P):  # one rank at a time: the build's temporaries never overlap
        graphs.append(ctxs[r].dist_kronecker(a.scale, r, P))
        ctxs[r].synchronize()
        print(json.dumps({"built_rank": r, "nnz_local": graphs[r].nnz, "t_s": round(time.perf_counter() - t0, 1),
                          "free_GB": round(mem_free_gb(), 1)}), flush=True)
    out["build_s"] = round(time.perf_counter() - t0, 1)
    out["nnz_global"] = int(sum(g.nnz for g in graphs))
    out["device_free_GB_after_build"] = round(mem_free_gb(), 1)
    roots = run_ranks(P, lambda r: [int(x) for x in graphs[r].sample_roots(a.roots, seed=0x5EED)])
    assert all(x == roots[0] for x in roots), "ranks sampled different roots"
    out["roots"] = roots[0]
    out["bfs"] = []
    dist_parts = {}
    for s in roots[0]:
        def one(r):
            w0 = time.perf_counter()
            st = graphs[r].dist_bfs(s)
            wall = time.perf_counter() - w0
            v = graphs[r].validate()
            lv = [{k: ls[k] for k in ("level", "direction", "frontier_in", "frontier_out", "mf_in", "scanned",
                                      "claims", "walked", "kernel_ms", "cum_ms")}
                  for ls in graphs[r].level_stats(256)]
            d = graphs[r].result()[0] if a.single else None
            return st, wall, v, lv, d
        res = run_ranks(P, one)
        st = res[0][0]
        rec = {"root": s, "levels": st["levels"], "topdown_levels": st["topdown_levels"],
               "bottomup_levels": st["bottomup_levels"], "m_comp": st["m_comp"], "reached": st["reached"],
               "wall_ms_max_over_ranks": round(max(x[1] for x in res) * 1e3, 2),
               "validation_errors": res[0][2]["errors"], "validated_entries": res[0][2]["entries"],
               "levels_rank0": res[0][3], "levels_all_ranks": [x[3] for x in res]}
        # exchange volumes from the level records (all ranks), per level, bytes received summed over the ranks:
        #   push level: the (vertex, parent) pairs the ranks shipped (8 B each; `walked` of a push record);
        #   pull level: the global frontier -- as id lists (8 B per id to every rank) when it holds fewer than
        #   n/128 vertices (option sparse_exchange=auto, the default), else the n/8-byte bitmap all-gathered
        #   (each rank receives the P - 1 slices it does not own)
        n = 1 << a.scale
        ex = []
        for li, lv in enumerate(res[0][3]):
            per = [x[3][li] for x in res]
            if lv["direction"] == 2:
                nf = sum(x["frontier_in"] for x in per)
                sparse = P > 1 and li > 0 and nf * 128 < n
                b = nf * 8 * (P - 1) if sparse else (n // 8) * (P - 1)
                ex.append({"level": lv["level"], "kind": "pull", "frontier_in": nf,
                           "exchange": "id lists" if sparse else "bitmap all-gather", "bytes": b})
            else:
                pairs = sum(x["walked"] for x in per)
                ex.append({"level": lv["level"], "kind": "push", "frontier_in": sum(x["frontier_in"] for x in per),
                           "exchange": "pairs", "bytes": pairs * 8})
        rec["exchange"] = ex
        rec["exchange_bytes_total"] = sum(x["bytes"] for x in ex)
        out["bfs"].append(rec)
        print(json.dumps({k: rec[k] for k in rec if not k.startswith("levels_")}), flush=True)
        assert rec["validation_errors"] == 0
        if a.single:
            dist_parts[s] = [(graphs[r].partition()["v_lo"], res[r][4]) for r in range(P)]
    for g in graphs:
        g.free()
    for c in ctxs:
        c.close()
    if a.single:
        ctx = bfsx.Context(0)
        ctx.set_option("hub_bits", "off")
        t1 = time.perf_counter()
        g = ctx.kronecker(a.scale)
        ctx.synchronize()
        out["single_build_s"] = round(time.perf_counter() - t1, 1)
        out["single"] = []
        for s in roots[0]:
            d, _, st = g.bfs(s, want_parent=False)
            v = g.validate()
            same = all(np.array_equal(d[lo:lo + len(dp)], dp) for lo, dp in dist_parts[s])
            rec = {"root": s, "t_bfs_ms": round(st["t_bfs_ms"], 3),
                   "gteps": round(st["m_comp"] / (st["t_bfs_ms"] * 1e-3) / 1e9, 1),
                   "validation_errors": v["errors"], "equals_partitioned": bool(same)}
            out["single"].append(rec)
            print(json.dumps(rec), flush=True)
            assert same and v["errors"] == 0
        g.free()
        ctx.close()
    js = json.dumps(out)
    print(js, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
