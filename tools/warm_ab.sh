#!/bin/bash
# GPU-box: does a timed run starting on never-used in-flight slots pay for it? 2^17 x 20 steps with
# 16 in flight after 5 warmup steps (11 slots first used inside the timed region) against 16 warmup
# steps (every slot used once before timing), alternating; extra bench.py args in $1.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${TAG:-warm}
for rep in 1 2 3; do
  for w in 5 16; do
    log=gpurun_out/${tag}_w${w}_$rep.log
    timeout -k 10 200 python3 -u bench.py --n 131072 --steps 20 --warmup $w --no-cpu-baseline --no-host-api --profile-steps 1 $1 > $log 2>&1 || { tail -5 $log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); print('warmup $w rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_ab.log
  done
done
