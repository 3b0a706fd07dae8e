# GPU-box baseline of the session: GPU tests + smoke, the driver's bench command and the 40-step
# default, 2^17 / configs[1] / configs[4] shapes, the multi-device pipelined entry, small calls,
# and the per-batch VALU table at 2^17 and 2^20. Output under gpurun_out/r03i_*.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03i
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/${t}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${t}_smoke.log 2>&1 || { tail -5 gpurun_out/${t}_smoke.log; exit 1; }
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${t}_bench_driver.log 2>&1 || exit 1
echo "driver $(tail -1 gpurun_out/${t}_bench_driver.log | cut -c1-160)"
timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_bench_40.log 2>&1 || exit 1
echo "c3-40 $(tail -1 gpurun_out/${t}_bench_40.log | cut -c1-160)"
for spec in "n17:--n 131072 --inflight 8" "c2:--config c2 --inflight 8" "c5:--config c5"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 180 python3 bench.py $args --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_bench_$name.log 2>&1 || exit 1
  echo "$name $(tail -1 gpurun_out/${t}_bench_$name.log | cut -c1-160)"; grep -o '"phases_ms.*batch_latency_ms": [0-9.]*' gpurun_out/${t}_bench_$name.log
done
for spec in "0 6" "0,0 4" "0,0,0,0 2"; do
  set -- $spec
  timeout -k 10 200 python3 tools/multi_bench.py --devices $1 --inflight $2 > gpurun_out/${t}_multi.log 2>&1 || { tail -5 gpurun_out/${t}_multi.log; exit 1; }
  grep '^{' gpurun_out/${t}_multi.log | tee -a gpurun_out/${t}_multi_all.log
done
timeout -k 10 200 python3 tools/smallbatch_bench.py --sizes 64,150,1024 > gpurun_out/${t}_smallbatch.log 2>&1 || { tail -5 gpurun_out/${t}_smallbatch.log; exit 1; }
grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*, "gpu_batch_dev_ms": [0-9.]*' gpurun_out/${t}_smallbatch.log
for n in 131072 1048576; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES -d gpurun_out/${t}_pmc_$n -o run --output-format csv -- \
    python3 bench.py --n $n --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 > gpurun_out/${t}_pmc_$n.log 2>&1 || { echo pmc_fail; tail -5 gpurun_out/${t}_pmc_$n.log; exit 1; }
  python3 tools/pmc_batch_table.py $(find gpurun_out/${t}_pmc_$n -name '*counter_collection.csv' | head -1) > gpurun_out/${t}_pmc_table_$n.txt
  cat gpurun_out/${t}_pmc_table_$n.txt
done
echo done
