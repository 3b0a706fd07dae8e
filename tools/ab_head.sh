#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    (cd $d && timeout -k 10 120 python -u bench.py --steps 40 --warmup 4 --no-cpu-baseline ${ARGS}) > gpurun_out/abh_$v.log 2>&1 || { echo fail $v; tail -5 gpurun_out/abh_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/abh_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); ph=d["phases_ms"]; print(d["ms_per_step"], "%.3e" % d["value"], ph["msm_bucket"], ph["msm_window_final"])')"
  done
done
