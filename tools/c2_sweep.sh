#!/bin/bash
# configs[1] (2^16 distinct keys): step time by (window bits, MSM parts), one batch at a time
# (INFLIGHT=1, with the per-phase times) or pipelined (INFLIGHT=8)
set -o pipefail
mkdir -p gpurun_out
inf=${INFLIGHT:-1}
for wb in ${BITS:-11 12 13}; do for p in ${PARTS:-1 2 4 8}; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 30 --warmup 4 --inflight $inf --no-cpu-baseline --window-bits $wb --msm-parts $p > gpurun_out/c2s.log 2>&1 || { echo fail; tail -5 gpurun_out/c2s.log; exit 1; }
  echo "wb=$wb parts=$p inflight=$inf $(tail -1 gpurun_out/c2s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); ph=d["phases_ms"]; print(d["ms_per_step"], ph["msm_bin"], ph["msm_bucket"], ph["msm_window_final"])')"
done; done
