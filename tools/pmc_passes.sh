#!/bin/bash
# GPU-box: PMC passes over the bench (one batch at a time), each pass in its own rocprofv3 run
# (counter limits per pass: MI355X_MICROARCH.md), for tools/pmc_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export EDC_SINGLE_STREAM=1    # one batch at a time, no decode beside SHA-512 (per-kernel issue fractions)
mkdir -p gpurun_out
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-host-api --profile-steps 1 $BENCH_ARGS > gpurun_out/pmc_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run int SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS &&
[ -n "$VALU_ONLY" ] || { run fetch FETCH_SIZE && run write WRITE_SIZE; }
