#!/bin/bash
# Round 5: the partitioned loop over a real P-process RCCL communicator on one GPU (per-rank NCCL_HOSTID, socket
# transport over loopback): the RCCL rank tests, the in-process group suite, then bench.py --gpus 2 / 4 at scale 26
# (16 roots, one step: the socket transport, not xGMI, so the numbers say nothing about N-GPU speed).
set -e -o pipefail
O=gpurun_out/r05rccl; mkdir -p $O
export NCCL_DEBUG=WARN
timeout -k 10 500 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_rccl_ranks.py > $O/tests3.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dist_native.py tests/test_gpu_dist.py > $O/dist_suite.log 2>&1
for n in 2 4; do
  BFSX_RCCL_SHARED_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus $n --steps 1 --warmup 1 --roots 16 --deadline 350 \
    > $O/bench_s26_p$n.json 2> $O/bench_s26_p$n.err
  python3 -c "import json; d=json.load(open('$O/bench_s26_p$n.json')); print($n, round(d['value'],1), d['t_bfs_ms_mean'], d['validation'])"
done
