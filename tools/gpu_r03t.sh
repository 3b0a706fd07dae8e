# GPU-box: fused batch tail (k_msm_tail): full GPU suite, then A/B against the previous tree
# (libedc_cur.so) at 2^17 / configs[1] / configs[2], and the small-call latencies.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-r03t}
D=ed25519-consensus_amd/csrc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 8 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_window_final": [0-9.]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur tail; do
    ab "--n 131072 --inflight 16" $lib n17
    ab "--config c2 --inflight 16" $lib c2
    ab "--config c3" $lib c3
  done
done
for lib in cur tail cur tail; do
  timeout -k 10 200 python3 tools/smallbatch_bench.py --sizes 64,150,1024 --lib $D/libedc_$lib.so > gpurun_out/${t}_smallbatch.log 2>&1 || { tail -5 gpurun_out/${t}_smallbatch.log; exit 1; }
  echo "smallbatch $lib"; grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*, "gpu_batch_dev_ms": [0-9.]*' gpurun_out/${t}_smallbatch.log | tee -a gpurun_out/${t}_smallbatch_all.log
done
