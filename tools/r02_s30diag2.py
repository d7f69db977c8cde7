"""Relabelled vs plain CSR build at scales 28..30: nnz, and (largest scale) which original vertices' degrees differ.
    python tools/r02_s30diag2.py [max_scale]"""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, "bfs-with-mapreduce_amd")
import bfsx  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 30


def degrees(g):
    off = np.empty(g.nv + 1, np.int64)
    bfsx._check(bfsx.lib().bfsx_graph_csr(g._h, off.ctypes.data_as(C.c_void_p), None))
    return np.diff(off)


with bfsx.Context(0) as ctx:
    for scale in range(28, top + 1):
        res = {}
        for rl in ("off", "on"):
            ctx.set_option("relabel", rl)
            t0 = time.perf_counter()
            with ctx.kronecker(scale) as g:
                res[rl] = (g.nnz, degrees(g) if scale == top else None)
                print(f"scale {scale} relabel {rl}: nnz {g.nnz} build+export {time.perf_counter() - t0:.1f} s",
                      flush=True)
        if scale == top:
            d0, d1 = res["off"][1], res["on"][1]
            bad = np.nonzero(d0 != d1)[0]
            print(f"vertices whose degree differs: {len(bad)}; sum off-on {int((d0 - d1).sum())}", flush=True)
            for v in bad[:20]:
                print(f"  v {v} deg off {d0[v]} on {d1[v]}", flush=True)
            if len(bad):
                print("  deg(off) of differing vertices: min", int(d0[bad].min()), "max", int(d0[bad].max()),
                      flush=True)
