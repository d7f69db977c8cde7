"""bench.py end to end on a small graph: the single-GPU line (with its CPU baseline and P = 1 rehearsal legs)
and the distributed harness that `bench.py --gpus N` runs under torch.distributed.run (one process per GPU,
RCCL inside libbfsx, gloo for the rendezvous), here with one rank.  Checks the contract of the one JSON line
(metric, value, n_gpus, steps, roots, validation) rather than any number."""
import json
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run(cmd, timeout=300):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # the contract: ONE JSON line on stdout
    return json.loads(lines[0])


def check_line(d, n_gpus, roots):
    assert d["metric"] == f"GTEPS (harmonic mean, {roots} roots) on RMAT scale-16"
    assert d["unit"] == "GTEPS" and d["higher_is_better"] is True and d["n_gpus"] == n_gpus
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["steps"] == 1
    assert d["config"]["workload"] == "kronecker-s16-ef16" and d["config"]["roots"] == roots
    assert d["validation"]["roots"] == roots and d["validation"]["errors"] == 0
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["peak"] == 8000.0


def test_bench_single_gpu_line():
    d = run([sys.executable, "bench.py", "--scale", "16", "--roots", "8", "--steps", "1", "--warmup", "0",
             "--cpu-baseline-seconds", "1", "--serial-baseline-seconds", "1"])
    check_line(d, 1, 8)
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["value"] > 0
    assert d["partitioned_p1"]["value"] > 0 and d["partitioned_p1"]["validated_roots"] == 8


def test_bench_distributed_harness_one_rank():
    d = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
             "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "1",
             "--dist", "--scale", "16", "--roots", "8", "--steps", "1", "--warmup", "0"])
    check_line(d, 1, 8)
    assert d["scaling"] == "strong" and d["config"]["parallelism"].startswith("1d-partition dp1")
    assert d["bfs_runs"] == 8 and d["value_wall"] > 0
