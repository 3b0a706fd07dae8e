set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/multi_bench.py --devices 0 --inflight 6 > gpurun_out/r03g_multi1.log 2>&1 || { tail -5 gpurun_out/r03g_multi1.log; exit 1; }
grep '^{' gpurun_out/r03g_multi1.log
timeout -k 10 200 python3 tools/multi_bench.py --devices 0,0 --inflight 3 > gpurun_out/r03g_multi2.log 2>&1 || { tail -5 gpurun_out/r03g_multi2.log; exit 1; }
grep '^{' gpurun_out/r03g_multi2.log
for n in 131072 1048576; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES -d gpurun_out/r03g_pmc_$n -o run --output-format csv -- \
    python3 bench.py --n $n --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 > gpurun_out/r03g_pmc_$n.log 2>&1 || { echo pmc_fail; tail -5 gpurun_out/r03g_pmc_$n.log; exit 1; }
  python3 tools/pmc_batch_table.py $(find gpurun_out/r03g_pmc_$n -name '*counter_collection.csv' | head -1) > gpurun_out/r03g_pmc_table_$n.txt
  cat gpurun_out/r03g_pmc_table_$n.txt
done
