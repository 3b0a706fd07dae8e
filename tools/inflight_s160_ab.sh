#!/bin/bash
# GPU-box: in-flight depth 12 against 16 at 2^17 over 160 steps, for one rank without a process
# group and for the forced single-rank RCCL loop, alternating.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-if160}
for rep in 1 2; do
  for f in 12 16; do
    for b in plain nccl; do
      log=gpurun_out/${tag}_${b}_f${f}_$rep.log
      if [ $b = plain ]; then
        timeout -k 10 300 python3 -u bench.py --n 131072 --steps 160 --warmup 5 --inflight $f --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      else
        EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port $((29450 + rep * 10 + f / 4)) bench.py --batch 131072 --steps 160 \
          --inflight $f --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
      fi
      python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); print('$b inflight $f rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_ab.log
    done
  done
done
