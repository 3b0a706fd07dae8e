#!/bin/bash
# GPU-box: Pippenger window width sweep per batch size (bench.py), one JSON summary line per run.
mkdir -p gpurun_out
for cfg in ${CFGS:-c2}; do
  for n in ${NS:-65536}; do
    for b in ${BITS:-0 10 11 12 13 14 16}; do
      timeout -k 10 120 python -u bench.py --config $cfg --n $n --window-bits $b --msm-parts ${PARTS:-0} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --profile-steps 1 > gpurun_out/bits_${cfg}_${n}_${b}.log 2>&1 || exit $?
      echo "$cfg n=$n bits=$b $(tail -1 gpurun_out/bits_${cfg}_${n}_${b}.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["phases_ms"])')"
    done
  done
done
