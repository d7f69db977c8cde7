set -e -o pipefail
O=gpurun_out/sw; mkdir -p $O
B="python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline"
run(){ n=$1; shift; timeout -k 10 120 $B "$@" > $O/$n.json 2> $O/$n.err; }
run base
run beta12 --option beta=12
run beta48 --option beta=48
run beta96 --option beta=96
run hd32 --option hub_degree=32
run hd128 --option hub_degree=128
run base2
run alpha25 --option alpha=25
run beta18 --option beta=18
run beta36 --option beta=36
run base3
echo done > $O/DONE
