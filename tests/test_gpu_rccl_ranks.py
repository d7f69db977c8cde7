"""The partitioned level loop over a real multi-rank RCCL communicator: P processes, one rank each.

The box has one MI355X and RCCL refuses two ranks on one device of one host, so every rank process gets its
own NCCL_HOSTID: RCCL then takes them for P hosts and moves the exchange over its socket transport on the
loopback interface. What runs is RcclComm (csrc/bfsx_comm.cpp) at P > 1 -- ncclCommInitRank over P
processes, the grouped send/recv all-to-allv of the push levels, the frontier all-gather of the pull levels,
the level-close all-reduce, ncclCommAbort with the shared abort board -- which the in-process groups of
test_gpu_dist_native.py do not reach. Only xGMI itself (the driver's 8-GPU run) is left out.

Distances are bit-exact against the oracle and the parents satisfy Graph500's rules (checked on the host and
by the collective device validator); a failed rank fails every rank within 5 s."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import oracle_py as O
from conftest import ROOT

pytestmark = pytest.mark.gpu
INF = 2147483647
WORKER = os.path.join(ROOT, "tests", "rccl_rank_worker.py")


def launch(tmp_path, world, mode, scale, seed, sources, limit=150, options=None):
    """Start the P rank processes (each its own NCCL_HOSTID), wait for all of them against one deadline."""
    uid = str(tmp_path / "rccl.uid")
    procs = []
    for r in range(world):
        env = dict(os.environ, NCCL_HOSTID=f"bfsx-test-rank{r}", NCCL_SOCKET_IFNAME="lo",
                   BFSX_WORKER_STACK_AFTER=str(limit - 20),
                   BFSX_WORKER_OPTIONS=",".join(f"{k}={v}" for k, v in (options or {}).items()))
        env.pop("BFSX_RCCL_SHARED_DEVICE", None)
        cmd = [sys.executable, WORKER, str(r), str(world), uid, str(tmp_path / f"rank{r}"), mode, str(scale),
               hex(seed), ",".join(str(s) for s in sources)]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      start_new_session=True))
    outs, end = [], time.time() + limit
    for p in procs:
        try:
            outs.append(p.communicate(timeout=max(1.0, end - time.time()))[0])
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            outs.append(p.communicate()[0] + "\n[test] killed at the deadline")
    tails = "\n".join(f"--- rank {r} rc {p.returncode}\n" + o[-3000:] for r, (p, o) in enumerate(zip(procs, outs)))
    assert all(p.returncode == 0 for p in procs), tails
    return tails


@pytest.mark.parametrize("world,options", [
    (2, {}), (4, {}),
    # every push level through the counted exchange (count all-to-all, then the pair all-to-allv)
    (2, {"slot_pairs": "0"}), (4, {"slot_pairs": "0"}),
    # every pull level after the first receives the frontier as id lists (all-to-allv) instead of the all-gather
    (2, {"sparse_exchange": "on"}), (4, {"sparse_exchange": "on", "direction": "bottomup"}),
])
def test_rccl_ranks_parity(tmp_path, world, options):
    scale, seed = 15, 0x2CC1
    u, v = O.kronecker(scale, 16, seed)
    nv = 1 << scale
    sources = [int(u[0]), int(u[4321]), int(v[99])]
    launch(tmp_path, world, "parity", scale, seed, sources, options=options)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    off, col = O.build_sets(nv, u, v)
    for i, s in enumerate(sources):
        dist = np.full(nv, INF, np.int32)
        parent = np.full(nv, -1, np.int64)
        for x in res:
            lo = int(x["v_lo"])
            dist[lo:lo + len(x[f"dist{i}"])] = x[f"dist{i}"]
            parent[lo:lo + len(x[f"parent{i}"])] = x[f"parent{i}"]
        ref, _ = O.csr_bfs(nv, off, col, s)
        assert np.array_equal(dist, ref), f"source {s}: RCCL P={world} distances differ from the oracle"
        assert O.validate(nv, off, col, s, dist, parent, rows_sorted=True) == 0
        levels, m_comp, reached = (int(t) for t in res[0][f"stats{i}"])
        assert all(np.array_equal(x[f"stats{i}"], res[0][f"stats{i}"]) for x in res), "ranks disagree on stats"
        assert levels == int(ref[ref != INF].max()) + 1
        assert m_comp == O.mcomp(u, v, ref) and reached == int((ref != INF).sum())
        assert all(int(x[f"errors{i}"][0]) == 0 for x in res)


@pytest.mark.parametrize("world,rank,where,checks", [(2, 1, "2", "on"), (4, 2, "1", "on"), (2, 0, "setup", "on"),
                                                     (2, 1, "2", "off"), (4, 3, "3", "off")])
def test_rccl_failed_rank_fails_every_rank(tmp_path, world, rank, where, checks):
    """VERDICT r4 item 1 on the RCCL communicator: the failing rank returns its own error, every peer
    BFSX_E_RCCL naming it (the shared abort board, then ncclCommAbort), all within 5 s, and the aborted
    communicator fails every later call at once.  This test found the one hang the in-process groups could not
    show: a device -> host copy into pageable memory right after a collective blocks the host inside HIP, out of
    reach of the abort polling, while the collective waits for the failed peer (event (e))."""
    scale, seed = 13, 0xFA11
    src = int(O.kronecker(scale, 16, seed)[0][0])
    tails = launch(tmp_path, world, f"fail:{rank}:{where}:{checks}", scale, seed, [src])
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    lvl = "setup" if where == "setup" else f"level {where}"
    assert all("error" in x for x in recs), (recs, tails)
    assert all(x["seconds"] < 5.0 for x in recs), recs
    assert "fault injection" in recs[rank]["error"], recs
    for r in range(world):
        if r != rank:
            assert recs[r]["code"] == -5, recs  # BFSX_E_RCCL
            assert f"peer rank {rank} failed at {lvl}" in recs[r]["error"], recs
        assert "again" in recs[r], recs


def test_rccl_vanished_rank_times_out(tmp_path):
    """A rank that leaves without aborting (a crash, a kill) writes nothing on the board: its peers' waits end at
    comm_timeout_ms (4 s here) at the latest with BFSX_E_RCCL, and the communicator is aborted instead of hanging."""
    scale, seed = 13, 0xFA11
    src = int(O.kronecker(scale, 16, seed)[0][0])
    launch(tmp_path, 2, "exit:1", scale, seed, [src])
    rec = json.load(open(tmp_path / "rank0.json"))
    assert rec.get("code") == -5, rec
    # whichever notices first: RCCL's own asynchronous error (the socket transport sees the peer's connection
    # close), the board's pid check, or the deadline
    assert any(w in rec["error"] for w in ("timed out", "exited without finishing", "RCCL asynchronous error")), rec
    assert rec["seconds"] < 15.0, rec
    assert "again" in rec, rec
