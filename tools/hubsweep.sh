# bottom-up hub probe domain sweep: bench at several hub_bits (usage: bash tools/hubsweep.sh <tag> <bits...>)
set -e -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for hb in "$@"; do
  timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline --option hub_bits=$hb > gpurun_out/$TAG/bench_$hb.json 2> gpurun_out/$TAG/bench_$hb.err
done
