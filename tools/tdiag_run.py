"""DIAG (not part of the product): per-section cycle split of the push sweep for roots with a large top-down L2."""
import ctypes as C
import json
import sys

sys.path.insert(0, "bfs-with-mapreduce_amd")
import bfsx  # noqa: E402

lib = bfsx.lib()
out = (C.c_ulonglong * 8)()
res = []
with bfsx.Context(0) as ctx:
    with ctx.kronecker(26) as g:
        roots = [int(r) for r in g.sample_roots(64, seed=0x5EED)]
        for r in roots:
            g.bfs_device_only(r)
            ls = g.level_stats(256)
            if len(ls) > 2 and ls[2]["direction"] == 1 and ls[2]["scanned"] > 5_000_000:
                lib.bfsx_diag_tdiag_reset()
                t = g.bfs_device_only(r)
                lib.bfsx_diag_tdiag(out)
                v = list(out)
                tot = sum(v[:7])
                res.append({"root": r, "ms": t, "edges": ls[2]["scanned"], "steps": v[7],
                            "split": [round(x / tot, 3) for x in v[:7]], "cyc_per_step": tot / max(v[7], 1)})
print(json.dumps(res, indent=0))
