# GPU-box: 15-bit windows from 2^17 to 2^19 signatures (auto) against 14 (libedc_cur.so).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03y
D=ed25519-consensus_amd/csrc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur c15; do ab "--n 131072" $lib n17; ab "--n 262144" $lib n18; ab "--n 262144 --keys 0" $lib n18d; done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_plans.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; exit $rc
