#!/bin/bash
# GPU-box: multi-batch launches (bench --multi) against single batches on one box, alternating
# (2^17 vote shards and configs[1] 2^16 distinct-key batches); summary in gpurun_out/<tag>_summary.log
set -o pipefail
tag=${1:-r04j}
one() {  # label args
  local label=$1; shift
  bash tools/gpu_session.sh $tag "bench=$*" || exit 1
  sed -i "s/^ *bench /$label /" gpurun_out/${tag}_summary.log
}
for rep in 1 2; do
  one n17 --n,131072,--steps,40,--no-cpu-baseline
  one m17x4 --n,131072,--multi,4,--inflight,4,--steps,20,--no-cpu-baseline
  one m17x8 --n,131072,--multi,8,--inflight,3,--steps,20,--no-cpu-baseline
  one m17x8i4 --n,131072,--multi,8,--inflight,4,--steps,20,--no-cpu-baseline
  one c2 --config,c2,--steps,40,--no-cpu-baseline
  one m16x4 --config,c2,--multi,4,--inflight,4,--steps,20,--no-cpu-baseline
  one m16x8 --config,c2,--multi,8,--inflight,3,--steps,20,--no-cpu-baseline
  one m16x16 --config,c2,--multi,16,--inflight,2,--steps,10,--no-cpu-baseline
done
