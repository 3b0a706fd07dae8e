#!/bin/bash
# GPU-box: forced single-rank RCCL loop at the 8-rank strong shard (2^17 x 20): exchanges in flight
# before the host completes the oldest (--exchange-lag 8 / 16 / 32), alternating, and the same shard
# on one rank without a process group beside them.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-lag}
for rep in 1 2 3; do
  for lag in ${LAGS:-8 16 32 plain}; do
    log=gpurun_out/${tag}_lag${lag}_$rep.log
    if [ $lag = plain ]; then
      timeout -k 10 300 python3 -u bench.py --n 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    else
      EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $((29900 + rep * 10 + lag % 10)) bench.py --batch 131072 --steps 20 \
        --warmup 5 --exchange-lag ${LAGARG:-$lag} ${EXTRA:-} --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    fi
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); o=d['scaling_other_shape'] or {}; print('lag $lag rep $rep', d['value'], d['ms_per_step'], 'repeat', o.get('value'), (d['comm'] or {}).get('exchange_us'))" | tee -a gpurun_out/${tag}_ab.log
  done
done
