#!/bin/bash
# GPU-box: first timed run after a spin-up of S ms (bench.py --spinup-ms), S swept, alternating.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-spinsweep}
for rep in 1 2; do
  for sp in 0 50 100 200 400 800; do
    for shape in "c3x20:--steps 20" "n17x20:--n 131072 --steps 20"; do
      name=${shape%%:*}; args=${shape#*:}
      log=gpurun_out/${tag}_${name}_sp${sp}_$rep.log
      timeout -k 10 200 python3 -u bench.py $args --warmup 5 --spinup-ms $sp --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); print('$name spinup $sp rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_ab.log
    done
  done
done
