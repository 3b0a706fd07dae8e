#!/bin/bash
# GPU-box: the forced single-rank RCCL loop (process group, all-gather ring, device combine) at the
# 8-rank strong shard size (2^17, the driver's 20 steps), 12 against 16 batches in flight,
# alternating. Logs: gpurun_out/<tag>_rccl_if<F>_<rep>.log, summary gpurun_out/<tag>_rccl_ab.log
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-rccl}
for rep in 1 2 3; do
  for f in 12 16; do
    log=gpurun_out/${tag}_rccl_if${f}_$rep.log
    EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29600 + rep * 10 + f)) bench.py --batch 131072 --steps 20 \
      --warmup 5 --inflight $f --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); o=d['scaling_other_shape']; print('inflight $f rep $rep', d['value'], d['ms_per_step'], 'repeat', o['value'], o['ms_per_step'])" | tee -a gpurun_out/${tag}_rccl_ab.log
  done
done
