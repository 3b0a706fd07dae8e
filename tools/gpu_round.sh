#!/bin/bash
# GPU-box helper: every GPU test, then the bench and the configs[3] fallback bench; each step
# under its own time limit, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/fallback_bench.py > gpurun_out/fb.log 2>&1
rc=$?; echo "fb_rc=$rc"; tail -1 gpurun_out/fb.log
exit $rc
