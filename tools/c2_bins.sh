#!/bin/bash
# configs[1] and the headline by MSM bin target (edc_set_msm_bin_entries) and window width
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-c2}; do for wb in ${BITS:-0}; do for be in ${ENTRIES:-0 2048 4096 8192}; do
  timeout -k 10 120 python -u bench.py --config $cfg --steps ${STEPS:-30} --warmup 4 --inflight ${INFLIGHT:-8} --no-cpu-baseline --window-bits $wb --bin-entries $be > gpurun_out/c2b.log 2>&1 || { echo fail; tail -5 gpurun_out/c2b.log; exit 1; }
  echo "$cfg wb=$wb entries=$be $(tail -1 gpurun_out/c2b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); ph=d["phases_ms"]; print(d["ms_per_step"], "%.3e" % d["value"], ph["msm_bin"], ph["msm_bucket"], ph["msm_window_final"])')"
done; done; done
