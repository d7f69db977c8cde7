"""Per-level times of the bench workload WITHOUT validation, for knockout builds (BFSX_LIB=<a build with a
part of a kernel removed>: results are wrong by construction, only the times matter).
    BFSX_LIB=... python tools/knockout_levels.py out.json [steps]"""
import json
import sys

sys.path.insert(0, "bfs-with-mapreduce_amd")
import bfsx  # noqa: E402

out, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
with bfsx.Context(0) as ctx:
    with ctx.kronecker(26) as g:
        roots = [int(r) for r in g.sample_roots(64, seed=0x5EED)]
        for r in roots:
            g.bfs_device_only(r)
        levels, t = [], []
        for _ in range(steps):
            for r in roots:
                t.append(g.bfs_device_only(r))
                levels.extend(dict(ls, root=r) for ls in g.level_stats(256))
json.dump(levels, open(out, "w"))
print(json.dumps({"t_bfs_ms_mean": sum(t) / len(t)}))
