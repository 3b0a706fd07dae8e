#!/bin/bash
# GPU-box sweep: hardware queues per process x batches in flight (bench.py, configs[2]).
mkdir -p gpurun_out
for q in ${QS:-4 8}; do
  for f in ${FS:-3 4}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u bench.py --steps 30 --warmup 3 --inflight $f --no-cpu-baseline --profile-steps 1 > gpurun_out/hwq_${q}_${f}.log 2>&1 || exit $?
    echo "q=$q inflight=$f $(tail -1 gpurun_out/hwq_${q}_${f}.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
