# GPU-box: wave-state and HBM-fetch PMC passes of the configs[4] and configs[2] batches (one batch
# at a time) to see what bounds k_challenge on variable-length messages.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c5 c3; do
  TAG=_r03q_$cfg BENCH_ARGS="--config $cfg" bash tools/pmc_wait.sh || exit 1
  python3 tools/pmc_batch_table.py $(find gpurun_out/pmc_wait_r03q_$cfg -name '*counter_collection.csv' | head -1) > gpurun_out/r03q_wait_$cfg.txt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_r03q_$cfg -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 --config $cfg > gpurun_out/pmc_fetch_r03q_$cfg.log 2>&1 || { echo fetch_fail; exit 1; }
  python3 tools/pmc_batch_table.py $(find gpurun_out/pmc_fetch_r03q_$cfg -name '*counter_collection.csv' | head -1) > gpurun_out/r03q_fetch_$cfg.txt
  head -12 gpurun_out/r03q_wait_$cfg.txt; head -12 gpurun_out/r03q_fetch_$cfg.txt
done
