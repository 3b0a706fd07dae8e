#!/bin/bash
# GPU-box: forced single-rank RCCL loop at 2^17 x 20 with 1 / 4 / 16 records per all-gather
# (--exchange-group), alternating, against one rank without a process group.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-grp}
for rep in 1 2 3; do
  for g in 1 4 16 plain; do
    log=gpurun_out/${tag}_g${g}_$rep.log
    if [ $g = plain ]; then
      timeout -k 10 300 python3 -u bench.py --n 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    else
      EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $((29950 + rep * 10 + g % 10)) bench.py --batch 131072 --steps 20 \
        --warmup 5 --exchange-group $g --exchange-lag 16 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    fi
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); o=d['scaling_other_shape'] or {}; print('group $g rep $rep', d['value'], d['ms_per_step'], 'repeat', o.get('value'), (d['comm'] or {}).get('exchange_us'))" | tee -a gpurun_out/${tag}_ab.log
  done
done
