#!/bin/bash
# GPU-box: configs[2] bench with and without the validator-key cache, then the key-cache tests.
mkdir -p gpurun_out
for kc in "" "--keycache"; do
  for r in 1 2; do
    timeout -k 10 120 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --profile-steps 1 $kc > gpurun_out/kcb.log 2>&1 || exit $?
    echo "kc='$kc' $(tail -1 gpurun_out/kcb.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["phases_ms"])')"
  done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -1 gpurun_out/gpu_tests.log; exit $rc
