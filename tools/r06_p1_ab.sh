set -e -o pipefail
O=gpurun_out/r06dw; mkdir -p $O
for i in 1 2 3; do for L in base dv; do
  BFSX_LIB=$PWD/ab/$L/libbfsx.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/${L}_$i.json 2> $O/${L}_$i.err
  python3 -c "import json; d=json.load(open('$O/${L}_$i.json')); p=d['partitioned_p1']; print('$L run $i:', round(d['value'],1), 'p1', round(p['value'],1), 't_bfs', round(p['t_bfs_ms_mean'],4))" | tee -a $O/summary.txt
done; done
