# GPU-box: per-batch VALU tables of configs[1] and configs[4] (one batch at a time).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in c2 c5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/r03z_pmc_$cfg -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 > gpurun_out/r03z_pmc_$cfg.log 2>&1 || { echo pmc_fail; tail -5 gpurun_out/r03z_pmc_$cfg.log; exit 1; }
  python3 tools/pmc_batch_table.py $(find gpurun_out/r03z_pmc_$cfg -name '*counter_collection.csv' | head -1) > gpurun_out/r03z_pmc_table_$cfg.txt
  cat gpurun_out/r03z_pmc_table_$cfg.txt
done
