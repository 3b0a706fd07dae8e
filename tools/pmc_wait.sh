#!/bin/bash
# GPU-box: one PMC pass of wave-state counters over the bench (one batch at a time): where each
# kernel's wave-cycles go (issuing / parked on s_waitcnt or barrier / issue-stalled) and the
# effective clock (GRBM_GUI_ACTIVE / 8 / wall). Summarised by tools/pmc_wait_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
  -d gpurun_out/pmc_wait${TAG} -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 ${BENCH_ARGS} > gpurun_out/pmc_wait${TAG}.log 2>&1
rc=$?; echo "pmc wait rc=$rc"; exit $rc
