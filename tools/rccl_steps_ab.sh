#!/bin/bash
# GPU-box: forced single-rank RCCL loop against one rank without a process group at 2^17 for
# 20 and 160 timed steps: a fixed cost per timed region (exchange drain, closing barrier) shrinks
# with the region, a per-batch cost does not.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-rst}
for rep in 1 2; do
  for st in 20 160; do
    for b in nccl plain; do
      log=gpurun_out/${tag}_${b}_s${st}_$rep.log
      if [ $b = plain ]; then
        timeout -k 10 300 python3 -u bench.py --n 131072 --steps $st --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      else
        EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port $((29650 + rep * 10 + st / 20)) bench.py --batch 131072 --steps $st \
          --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      fi
      python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); c=d['comm'] or {}; print('$b steps $st rep $rep', d['value'], d['ms_per_step'], 'tail_us', c.get('timed_tail_us'))" | tee -a gpurun_out/${tag}_ab.log
    done
  done
done
