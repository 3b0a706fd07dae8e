#!/bin/bash
# GPU-box: is the forced single-rank loop's per-batch share at 2^17 (160 steps) the ring's torch
# work or the process group's presence? Group 4 / lag 8 (the default) against group 64 / lag 64
# (one collective per 64 batches) and one rank without a process group, alternating.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-rrw}
for rep in 1 2; do
  for v in g4 g64 plain; do
    log=gpurun_out/${tag}_${v}_$rep.log
    case $v in
      plain) timeout -k 10 300 python3 -u bench.py --n 131072 --steps 160 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; } ;;
      *) if [ $v = g4 ]; then x="--exchange-group 4 --exchange-lag 8"; p=1; else x="--exchange-group 64 --exchange-lag 64"; p=2; fi
         EDC_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
           --master-addr 127.0.0.1 --master-port $((29550 + rep * 10 + p)) bench.py --batch 131072 --steps 160 $x \
           --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > $log 2>&1 || { tail -5 $log; exit 1; } ;;
    esac
    python3 -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); c=d['comm'] or {}; print('$v rep $rep', d['value'], d['ms_per_step'], 'xus', c.get('exchange_us'), 'tail', c.get('timed_tail_us'))" | tee -a gpurun_out/${tag}_ab.log
  done
done
