#!/bin/bash
# GPU-box helper: parity tests then a short bench; every GPU step under its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/bench.log
exit $rc
