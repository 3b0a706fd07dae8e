set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/row_probe > gpurun_out/r03b_row_probe.txt 2>&1; rc=$?; cat gpurun_out/r03b_row_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/submit_probe.py > gpurun_out/r03b_submit_probe.log 2>&1; rc=$?; cat gpurun_out/r03b_submit_probe.log | grep -v amdgpu.ids; exit $rc
