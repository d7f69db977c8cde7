"""Single-device: validation errors per option set over many roots (bu_pipeline isolation)."""
import importlib.util, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bfsx", os.path.join(ROOT, "bfs-with-mapreduce_amd", "bfsx.py"))
bfsx = importlib.util.module_from_spec(spec); spec.loader.exec_module(bfsx)
for scale in (20, 23):
    for opts in ({}, {"relabel": "off"}, {"direction": "bottomup"}, {"relabel": "off", "direction": "bottomup"},
                 {"bu_pipeline": "off", "direction": "bottomup"}):
        with bfsx.Context(0, **opts) as ctx:
            with ctx.kronecker(scale) as g:
                errs = 0
                for r in g.sample_roots(24, seed=5):
                    g.bfs(int(r), want_dist=False, want_parent=False)
                    errs += g.validate()["errors"]
                print(scale, opts, "errors", errs, flush=True)
