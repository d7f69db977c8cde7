"""bench.py's N > 1 harness at world_size 2 over gloo on the CPU (tests/bench_dist_fake.py stands in for
the GPU library): one JSON line from rank 0, n_gpus = 2, strong scaling, and `value` = the harmonic mean
of m_comp over the SLOWEST rank's device time of each BFS, with a tiny-component root skipped."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def test_bench_dist_harness_two_ranks_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "tests", "bench_dist_fake.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["steps"] == 2
    assert d["metric"] == "GTEPS (harmonic mean, 4 roots) on RMAT scale-12"
    roots = [1, 2, 4, 5]  # root 3 skipped: its component holds 5 of 65,536 tuples
    assert d["validation"]["skipped_tiny_component"] == [{"root": 3, "m_comp": 5}]
    m_comp = (16 << 12) // 2
    slowest = [1.0 + 0.5 * 1 + 0.01 * r for r in roots] * 2  # rank 1's times, 2 steps
    want = len(slowest) / sum(t * 1e-3 * 1e9 / m_comp for t in slowest)
    assert abs(d["value"] - want) < 1e-9 * want
    assert d["bfs_runs"] == 8 and d["config"]["parallelism"].startswith("1d-partition dp2")


def test_bench_gpus_flag_launches_its_own_ranks():
    """`python bench.py --gpus 2` exactly as the driver runs it (no launcher, WORLD_SIZE unset): bench.py
    starts the two ranks itself as one torch.distributed.run child and relays the single JSON line, which
    reports n_gpus = 2 (round 2 silently measured one GPU here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               BFSX_BENCH_BINDING=os.path.join(ROOT, "tests", "bench_dist_fake.py"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--scale", "12", "--roots",
                        "4", "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["bfs_runs"] == 8 and d["config"]["parallelism"].startswith("1d-partition dp2")


def test_bench_refuses_mismatched_world_size():
    """Inside a launcher, --gpus must equal WORLD_SIZE (exit code 2, no JSON line)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="", BFSX_BENCH_BINDING=os.path.join(ROOT, "tests", "bench_dist_fake.py"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--scale", "12"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and not r.stdout.strip(), (r.returncode, r.stdout, r.stderr[-2000:])


def test_bench_deadline_ends_a_stuck_run():
    """A rank stuck in the timed loop (here the stand-in's rank 1 never returns from its BFS, as a rank left inside
    a collective by a failed peer would) must not hold the run past --deadline: every rank arms it, the stuck one
    exits 124, torch.distributed.run stops the other, and `bench.py --gpus 2` exits non-zero with no JSON line,
    long before the test's own limit."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", BFSX_FAKE_HANG_RANK="1",
               BFSX_BENCH_BINDING=os.path.join(ROOT, "tests", "bench_dist_fake.py"))
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--scale", "12", "--roots",
                        "4", "--steps", "2", "--warmup", "1", "--deadline", "20"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    took = time.time() - t0
    assert r.returncode != 0 and not r.stdout.strip(), (r.returncode, r.stdout, r.stderr[-3000:])
    assert "deadline of 20 s passed" in r.stderr, r.stderr[-3000:]
    assert took < 150, took


def test_bench_shared_device_rehearsal_mode():
    """BFSX_RCCL_SHARED_DEVICE=1 (the one-GPU RCCL rehearsal): every rank gets its own NCCL_HOSTID and
    the ranks build their slices one after another; the line is the same as without it."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", BFSX_RCCL_SHARED_DEVICE="1",
               BFSX_BENCH_BINDING=os.path.join(ROOT, "tests", "bench_dist_fake.py"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--scale", "12", "--roots",
                        "4", "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["bfs_runs"] == 8


def test_bench_dist_line_diagnostics_and_scale30_leg():
    """Round 6 (verdict item 5): the N > 1 line says where the time goes and covers configs[4].
      comm_split  per collective kind, the device time per BFS (each BFS's max over ranks, mean over the roots) and
                  the calls; the last root's per-level time, max over ranks
      rccl        the world size and the transport summary of rank 0's RCCL log (no log here: a stand-in binding)
      scale30     the scale-30 leg on the same ranks (--scale30-roots; on by default at N > 1 with --scale 26)"""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", BFSX_FAKE_EXTRA_ARGS="--scale30-roots 2",
               NCCL_DEBUG="WARN")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "tests", "bench_dist_fake.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    cs = d["comm_split"]
    assert cs["roots"] == 4  # min(--comm-split-roots 8, the 4 roots)
    for i, k in enumerate(("allreduce", "count_alltoall", "alltoallv", "allgather")):
        assert abs(cs["ms_per_bfs"][k] - (0.1 * (i + 1) + 0.01)) < 1e-9  # rank 1's, the slower
        assert cs["calls_per_bfs"][k] == 4
    assert [x["direction"] for x in cs["levels_last_bfs"]] == [1, 2]
    assert d["rccl"]["world_size"] == 2 and "note" in d["rccl"]
    s30 = d["scale30"]
    assert s30["workload"] == "kronecker-s30-ef16" and s30["n_gpus"] == 2
    assert s30["metric"] == "GTEPS (harmonic mean, 2 roots) on RMAT scale-30"
    assert s30["validation"]["errors"] == 0 and s30["value"] > 0 and s30["comm_split"]["roots"] == 2
