set -o pipefail
mkdir -p gpurun_out
for spec in "0 6" "0,0 4" "0,0,0,0 2"; do
  set -- $spec
  timeout -k 10 200 python3 tools/multi_bench.py --devices $1 --inflight $2 > gpurun_out/r03h_multi.log 2>&1 || { tail -5 gpurun_out/r03h_multi.log; exit 1; }
  grep '^{' gpurun_out/r03h_multi.log | tee -a gpurun_out/r03h_multi_all.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03h_tests.log; exit $rc
