#!/bin/bash
# GPU-box: 2^17 x 20 on one rank without a process group at 12 / 16 in flight, and under the
# forced single-rank RCCL loop at 10 / 12 in flight (the loop adds the exchange ring's and RCCL's
# streams, i.e. hardware queues, beside the slots), alternating.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-queues}
for rep in 1 2 3; do
  for c in plain:12 plain:16 rccl:10 rccl:12; do
    kind=${c%%:*}; f=${c#*:}
    log=gpurun_out/${tag}_${kind}${f}_$rep.log
    if [ $kind = plain ]; then
      timeout -k 10 300 python3 -u bench.py --n 131072 --steps 20 --warmup 5 --inflight $f --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    else
      EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $((29750 + rep * 10 + f % 10)) bench.py --batch 131072 --steps 20 \
        --warmup 5 --inflight $f --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    fi
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); print('$kind inflight $f rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${tag}_ab.log
  done
done
