# GPU-box: full GPU suite + smoke + the driver's bench command and the other configs on the current tree.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-r03ac}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${t}_smoke.log 2>&1 || { tail -5 gpurun_out/${t}_smoke.log; exit 1; }
tail -1 gpurun_out/${t}_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${t}_bench_driver.log 2>&1 || { tail -5 gpurun_out/${t}_bench_driver.log; exit 1; }
echo "driver $(tail -1 gpurun_out/${t}_bench_driver.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
for spec in "c5:--config c5 --steps 12 --warmup 3" "c2:--config c2 --steps 40 --warmup 6" "n17:--n 131072 --steps 40 --warmup 6" "c3:--steps 40 --warmup 5"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python3 bench.py $args --no-cpu-baseline > gpurun_out/${t}_bench_$name.log 2>&1 || { tail -5 gpurun_out/${t}_bench_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/${t}_bench_$name.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')"
done
