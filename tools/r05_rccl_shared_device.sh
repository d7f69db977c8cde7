set -o pipefail
mkdir -p gpurun_out/r05rccl2
export BFSX_RCCL_SHARED_DEVICE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,NET
timeout -k 10 300 python3 bench.py --gpus 2 --scale 20 --steps 1 --warmup 0 --roots 8 --deadline 200 > gpurun_out/r05rccl2/s20.json 2> gpurun_out/r05rccl2/s20.err
echo rc=$?
cat gpurun_out/r05rccl2/s20.json
