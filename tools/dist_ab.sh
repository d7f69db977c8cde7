set -e -o pipefail
O=gpurun_out/dab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_native.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1
for i in 1 2; do for L in libbfsx_base libbfsx; do
BFSX_LIB=$PWD/bfs-with-mapreduce_amd/$L.so timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --dist --steps 64 --warmup 4 > $O/${L}_$i.json 2> $O/${L}_$i.err
done; done
