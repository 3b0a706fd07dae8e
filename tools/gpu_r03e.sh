set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/multi_bench.py > gpurun_out/r03e_multi_bench.log 2>&1 || { tail -5 gpurun_out/r03e_multi_bench.log; exit 1; }
grep '^{' gpurun_out/r03e_multi_bench.log
bash tools/gpu_r03d.sh
