#!/bin/bash
# Round 5: configs[4] (scale 30) through bench.py --gpus P with real multi-process RCCL on one GPU (a NCCL_HOSTID per
# rank, socket transport over loopback; BFSX_RCCL_SHARED_DEVICE=1). 4 roots, 1 step: a path check, not a speed.
set -e -o pipefail
O=gpurun_out/r05rccl30; mkdir -p $O
export NCCL_DEBUG=WARN
for n in ${@:-2}; do
  BFSX_RCCL_SHARED_DEVICE=1 timeout -k 10 1000 python3 bench.py --gpus $n --scale 30 --steps 1 --warmup 0 --roots 4 \
    --deadline 900 > $O/bench_s30_p$n.json 2> $O/bench_s30_p$n.err
  python3 -c "import json; d=json.load(open('$O/bench_s30_p$n.json')); print($n, round(d['value'],1), d['t_bfs_ms_mean'], d['graph_build_s'], d['validation'])"
done
