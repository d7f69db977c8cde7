"""Graph-build capacity probe (tuning aid): build one Kronecker partition and report its size, build
time and the device memory left, e.g. the rank-0 slice of scale 30 over 8 GPUs on a single device.

  python tools/build_probe.py --scale 30 --rank 0 --nranks 8 [--bfs]
"""
import argparse
import ctypes as C
import importlib.util
import json
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bfsx)


def mem_info():
    hip = C.CDLL("libamdhip64.so")
    free, total = C.c_size_t(), C.c_size_t()
    hip.hipMemGetInfo(C.byref(free), C.byref(total))
    return free.value, total.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--bfs", action="store_true", help="single-device graphs: also run 4 BFS")
    a = ap.parse_args()
    ctx = bfsx.Context(0)
    f0, total = mem_info()
    t0 = time.perf_counter()
    if a.nranks > 1:
        g = ctx.dist_kronecker(a.scale, a.rank, a.nranks)
    else:
        g = ctx.kronecker(a.scale)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    f1, _ = mem_info()
    out = {"scale": a.scale, "rank": a.rank, "nranks": a.nranks, "nv_local": g.nv, "nnz_local": g.nnz,
           "build_s": round(dt, 2), "graph_GB": round((f0 - f1) / 1e9, 2), "device_total_GB": round(total / 1e9, 1)}
    if a.bfs and a.nranks == 1:
        roots = g.sample_roots(4, seed=0x5EED)
        ts, ms = [], []
        for r in roots:
            _, _, st = g.bfs(int(r), want_dist=False, want_parent=False)
            ts.append(st["t_bfs_ms"])
            ms.append(st["m_comp"])
        out["gteps"] = [round(m / (t * 1e-3) / 1e9, 1) for m, t in zip(ms, ts)]
        out["t_bfs_ms"] = [round(t, 3) for t in ts]
    print(json.dumps(out), flush=True)
    g.free()
    ctx.close()


if __name__ == "__main__":
    main()
