set -e -o pipefail
O=gpurun_out/r05x; mkdir -p $O
for L in B D; do
  BFSX_LIB=$PWD/ab/$L/libbfsx.so timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-p1 --levels-json $O/$L.levels.json > $O/$L.json 2> $O/$L.err
done
