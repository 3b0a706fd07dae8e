# GPU-box: (1) parity of the split per-item failure bits (product build); (2) the decode on a
# second stream per slot beside SHA-512 / coefficients / binning (dual8: 8 slots x 2 queues,
# dual12: 12 x 2) against the single-stream 16-slot product, throughput and one-batch latency.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03af
D=ed25519-consensus_amd/csrc
timeout -k 10 400 python -u -m pytest tests/test_gpu_maxsize.py tests/test_gpu_plans.py tests/test_gpu_config3.py tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  ab "--config c3 --steps 20" cur c3-20
  ab "--config c3 --steps 20" dual8 c3-20
  ab "--config c3 --steps 20" dual12 c3-20
  ab "--n 131072 --steps 40" cur n17
  ab "--n 131072 --steps 40 --inflight 8" dual8 n17
  ab "--n 131072 --steps 40 --inflight 12" dual12 n17
  ab "--config c2 --steps 40" cur c2
  ab "--config c2 --steps 40 --inflight 12" dual12 c2
done
for lib in cur dual8; do
  timeout -k 10 200 python3 tools/smallbatch_bench.py --sizes 150,1024 --reps 30 --lib $D/libedc_$lib.so > gpurun_out/${t}_sb.log 2>&1 || { tail -5 gpurun_out/${t}_sb.log; exit 1; }
  echo "smallbatch $lib"; grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*' gpurun_out/${t}_sb.log | tee -a gpurun_out/${t}_all.log
done
for lib in cur dual8; do
  timeout -k 10 200 python3 tools/burst_probe.py --n 1048576 --ks 1 --lib $D/libedc_$lib.so > gpurun_out/${t}_lat.log 2>&1 || { echo nolib-arg; break; }
  echo "latency $lib $(grep '^{' gpurun_out/${t}_lat.log)" | tee -a gpurun_out/${t}_all.log
done
