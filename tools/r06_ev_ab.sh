set -e -o pipefail
mkdir -p gpurun_out/r06ev
for i in 1 2; do for L in base noev; do
  BFSX_LIB=$PWD/ab/$L/libbfsx.so timeout -k 10 300 python3 tools/r06_tbfs.py 64 4 | tee -a gpurun_out/r06ev/summary.txt
done; done
