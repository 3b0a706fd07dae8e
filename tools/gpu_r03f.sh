set -o pipefail
mkdir -p gpurun_out
for spec in "0,0 3" "0,0,0,0 2" "0 6"; do
  set -- $spec
  timeout -k 10 200 python3 tools/multi_bench.py --devices $1 --inflight $2 > gpurun_out/r03f_multi_bench.log 2>&1 || { tail -5 gpurun_out/r03f_multi_bench.log; exit 1; }
  grep '^{' gpurun_out/r03f_multi_bench.log
done
bash tools/gpu_r03d.sh
