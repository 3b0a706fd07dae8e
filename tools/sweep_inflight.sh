#!/bin/bash
# GPU-box: batches in flight x batch size (bench.py configs[2] shape / configs[1]).
mkdir -p gpurun_out
for cfg in ${CFGS:-c3}; do
  for n in ${NS:-1048576}; do
    for f in ${FS:-4 6 8}; do
      timeout -k 10 120 python -u bench.py --config $cfg --n $n --inflight $f --steps ${STEPS:-40} --warmup 4 --no-cpu-baseline --profile-steps 1 > gpurun_out/infl_${cfg}_${n}_${f}.log 2>&1 || exit $?
      echo "$cfg n=$n inflight=$f $(tail -1 gpurun_out/infl_${cfg}_${n}_${f}.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
