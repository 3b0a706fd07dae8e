#!/bin/bash
# GPU-box iteration helper: GPU parity tests, alternating A/B bench of the variant builds named in
# $AB (default "head base"), then optional steps: PMC=1 (WRITE_SIZE and FETCH_SIZE passes of the
# product build), TRACE=1 (pipelined kernel trace + tools/timeline.py). Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  AB_STEPS=${AB_STEPS:-40} bash tools/ab_variants.sh ${AB:-head base} || exit 1
done
if [ "${PMC:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_it_$c -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 > gpurun_out/pmc_it_$c.log 2>&1
    rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
if [ "${TRACE:-0}" = 1 ]; then
  TAG=${TAG:-it} bash tools/trace_bench.sh || exit 1
fi
exit 0
