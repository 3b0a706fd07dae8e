#!/bin/bash
# GPU-box: forced single-rank loop at 2^17 x 20 with the record exchange over RCCL (device
# all-gather + device combine) or over gloo (host all-gather, no GPU stream work), alternating,
# plus one rank without a process group. Splits the multi-rank loop cost into the host-side
# loop and the RCCL stream work.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-xbe}
for rep in 1 2 3; do
  for b in nccl gloo plain; do
    log=gpurun_out/${tag}_${b}_$rep.log
    case $b in nccl) port=1;; gloo) port=2;; *) port=3;; esac
    if [ $b = plain ]; then
      timeout -k 10 300 python3 -u bench.py --n 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    else
      EDC_DIST_BACKEND=$b EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $((29750 + rep * 10 + port)) bench.py --batch 131072 --steps 20 \
        --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    fi
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); o=d['scaling_other_shape'] or {}; print('backend $b rep $rep', d['value'], d['ms_per_step'], 'repeat', o.get('value'))" | tee -a gpurun_out/${tag}_ab.log
  done
done
