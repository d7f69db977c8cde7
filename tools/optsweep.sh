# bench sweep over libbfsx options (tuning aid): bash tools/optsweep.sh <tag> "<k=v[,k=v]>" ...
set -e -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for combo in "$@"; do
  i=$((i+1))
  opts=""
  for kv in ${combo//,/ }; do opts="$opts --option $kv"; done
  echo "$i $combo" >> gpurun_out/$TAG/index.txt
  timeout -k 10 300 python bench.py --steps 64 --warmup 4 --no-cpu-baseline $opts > gpurun_out/$TAG/bench_$i.json 2> gpurun_out/$TAG/bench_$i.err
done
