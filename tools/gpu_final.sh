#!/bin/bash
# GPU-box: the measurement set of a round: smoke, default bench (with the CPU baseline),
# rocprofv3 kernel stats one batch at a time and pipelined, PMC passes + summary.
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-r02}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1_$tag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline > gpurun_out/bench_prof1_$tag.log 2>&1 || { echo prof_fail; tail -20 gpurun_out/bench_prof1_$tag.log; exit 1; }
tail -1 gpurun_out/bench_prof1_$tag.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profp_$tag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_profp_$tag.log 2>&1 || { echo profp_fail; tail -20 gpurun_out/bench_profp_$tag.log; exit 1; }
tail -1 gpurun_out/bench_profp_$tag.log | cut -c1-200
bash tools/pmc_passes.sh || exit 1
# then, in the repo (profiles/ is not merged back from the box): python tools/pmc_summary.py gpurun_out
