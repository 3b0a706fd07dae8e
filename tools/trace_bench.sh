#!/bin/bash
# GPU-box: kernel trace of the pipelined default bench (4 in flight) and of one batch at a time,
# then tools/timeline.py over the pipelined trace. Output under gpurun_out/trace_*.
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$tag -o run --output-format csv -- \
  python3 bench.py --steps 25 --warmup 3 --no-cpu-baseline --profile-steps 1 ${BENCH_ARGS} > gpurun_out/trace_${tag}_bench.log 2>&1 \
  || { echo trace_fail; tail -20 gpurun_out/trace_${tag}_bench.log; exit 1; }
f=$(find gpurun_out/trace_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$f" --batches 20 > gpurun_out/trace_${tag}_timeline.txt 2>&1 || { echo timeline_fail; cat gpurun_out/trace_${tag}_timeline.txt; exit 1; }
cat gpurun_out/trace_${tag}_timeline.txt
tail -1 gpurun_out/trace_${tag}_bench.log | cut -c1-400
