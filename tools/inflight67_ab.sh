#!/bin/bash
# GPU-box: 6 against 7 batches in flight (bench.py --inflight), alternating: configs[2] over the
# driver's 20 steps and over 40, and the 2^19 shard (2-rank strong shape) over 20.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-if67}
for rep in 1 2 3 4; do
  for f in 6 7; do
    for shape in "c3x20:--steps 20" "c3x40:--steps 40" "n19x20:--n 524288 --steps 20"; do
      name=${shape%%:*}; args=${shape#*:}
      log=gpurun_out/${tag}_${name}_if${f}_$rep.log
      timeout -k 10 200 python3 -u bench.py $args --warmup 5 --inflight $f --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); print('$name inflight $f rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_ab.log
    done
  done
done
