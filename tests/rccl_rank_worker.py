"""One rank of a multi-process RCCL group on a box with fewer GPUs than ranks (test infrastructure, started by
tests/test_gpu_rccl_ranks.py, one process per rank).

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"). The parent gives every rank its
own NCCL_HOSTID, so RCCL sees P hosts and its ranks talk over the socket transport (loopback) instead of xGMI.
Everything above the transport is what `bench.py --gpus N` runs on N GPUs: RcclComm (bfsx_comm.cpp), the
grouped send/recv all-to-allv, the frontier all-gather, the level-close all-reduce and the abort path
(ncclCommAbort + the shared abort board).

usage: rccl_rank_worker.py RANK WORLD UID_FILE OUT_PREFIX MODE SCALE SEED SOURCES
  MODE  parity           run every source, write OUT_PREFIX.npz (v_lo, per-source dist/parent/stats)
        fail:R:LEVEL[:off]  option fail_at=R:LEVEL (off: check_collectives off), one source; write OUT_PREFIX.json
                         (error code, text, seconds)
        exit:R           rank R exits after the graph build; the others' first BFS fails at comm_timeout_ms
"""
import faulthandler
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conftest  # noqa: E402


def rendezvous(rank, uid_file, bfsx):
    """Rank 0 writes the RCCL unique id; the others poll for it (atomic rename, so no partial read)."""
    if rank == 0:
        uid = bfsx.comm_unique_id()
        with open(uid_file + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uid_file + ".tmp", uid_file)
        return uid
    end = time.time() + 60
    while not os.path.exists(uid_file):
        if time.time() > end:
            raise TimeoutError("no RCCL unique id from rank 0 within 60 s")
        time.sleep(0.05)
    with open(uid_file, "rb") as f:
        return f.read()


def main():
    rank, world, uid_file, out, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    scale, seed = int(sys.argv[6]), int(sys.argv[7], 0)
    sources = [int(x) for x in sys.argv[8].split(",")]
    # a rank still running after the parent's limit prints every thread's Python stack (the call it is stuck in)
    faulthandler.dump_traceback_later(float(os.environ.get("BFSX_WORKER_STACK_AFTER", "100")), exit=True)

    def say(what):
        print(f"[rank {rank} {time.time() - t00:7.2f}s] {what}", file=sys.stderr, flush=True)

    t00 = time.time()
    bfsx = conftest.load_bfsx()
    opts = {"check_collectives": "on", "comm_timeout_ms": "60000"}
    for kv in filter(None, os.environ.get("BFSX_WORKER_OPTIONS", "").split(",")):  # extra options, k=v,k=v
        k, v = kv.split("=", 1)
        opts[k] = v
    if mode.startswith("fail:"):  # fail:R:LEVEL[:off] -- off: without the collective-sequence check
        f = mode.split(":")
        opts["fail_at"] = f"{f[1]}:{f[2]}"
        if len(f) > 3:
            opts["check_collectives"] = f[3]
    if mode.startswith("exit:"):  # exit:R -- rank R leaves after the graph build; its peers' deadline ends the wait
        opts["comm_timeout_ms"] = "4000"
    ctx = bfsx.Context(0, **opts)
    ctx.comm_init(rank, world, rendezvous(rank, uid_file, bfsx))
    say("communicator up")
    g = ctx.dist_kronecker(scale, rank, world, seed=seed)
    say("graph built")
    if mode.startswith("exit:") and rank == int(mode.split(":")[1]):
        say("leaving without a word")
        os._exit(0)
    if mode == "parity":
        res = {"v_lo": g.partition()["v_lo"]}
        for i, s in enumerate(sources):
            st = g.dist_bfs(s)
            d, p = g.result()
            res[f"dist{i}"], res[f"parent{i}"] = d, p
            res[f"stats{i}"] = np.array([st["levels"], st["m_comp"], st["reached"]], np.int64)
            res[f"errors{i}"] = np.array([g.validate()["errors"]], np.int64)  # collective, Graph500 rules
        np.savez(out + ".npz", **res)
    else:
        rec = {}
        t0 = time.time()
        try:
            g.dist_bfs(sources[0])
        except bfsx.BfsxError as e:
            rec["code"], rec["error"] = e.code, str(e)
        rec["seconds"] = time.time() - t0
        say(f"first call returned: {rec}")
        try:  # the aborted communicator fails every later call at once
            g.dist_bfs(sources[0])
        except bfsx.BfsxError as e:
            rec["again"] = str(e)
        say("second call returned")
        with open(out + ".json", "w") as f:
            json.dump(rec, f)
    g.free()
    say("graph freed")
    ctx.close()
    say("context closed")


if __name__ == "__main__":
    main()
