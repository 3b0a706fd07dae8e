# GPU-box: GPU tests, then the headline / 2^17 / configs[1] benches and the small-call latencies
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-r03c}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/${tag}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit 1
echo "c3 $(tail -1 gpurun_out/${tag}_bench.log | cut -c1-150)"; grep -o '"phases_ms.*batch_latency_ms": [0-9.]*' gpurun_out/${tag}_bench.log
timeout -k 10 120 python3 bench.py --n 131072 --inflight 8 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_n17.log 2>&1 || exit 1
echo "n17 $(tail -1 gpurun_out/${tag}_bench_n17.log | cut -c1-150)"; grep -o '"phases_ms.*batch_latency_ms": [0-9.]*' gpurun_out/${tag}_bench_n17.log
timeout -k 10 120 python3 bench.py --config c2 --inflight 8 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_c2.log 2>&1 || exit 1
echo "c2 $(tail -1 gpurun_out/${tag}_bench_c2.log | cut -c1-150)"; grep -o '"phases_ms.*batch_latency_ms": [0-9.]*' gpurun_out/${tag}_bench_c2.log
timeout -k 10 200 python3 tools/smallbatch_bench.py ${SB_ARGS:---sizes 64,150,1024} > gpurun_out/${tag}_smallbatch.log 2>&1 || { tail -5 gpurun_out/${tag}_smallbatch.log; exit 1; }
grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*, "gpu_batch_dev_ms": [0-9.]*' gpurun_out/${tag}_smallbatch.log
exit 0
