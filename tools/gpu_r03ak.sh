# GPU-box: SHA-512 + decode in one launch on the pipelined slots (fused) against separate launches.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03ak
D=ed25519-consensus_amd/csrc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plans.py tests/test_gpu_multiblock.py tests/test_gpu_config3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 5 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur fused; do
    ab "--steps 20" $lib c3-20
    ab "--steps 40" $lib c3-40
    ab "--n 131072 --steps 40" $lib n17
    ab "--config c2 --steps 40" $lib c2
    ab "--config c5 --steps 12" $lib c5
  done
done
for lib in cur fused; do
  timeout -k 10 200 python3 tools/burst_probe.py --n 1048576 --ks 1,2 --lib $D/libedc_$lib.so > gpurun_out/${t}_lat.log 2>&1 || exit 1
  echo "latency $lib $(grep '^{' gpurun_out/${t}_lat.log | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
  timeout -k 10 200 python3 tools/burst_probe.py --n 131072 --ks 1,2 --lib $D/libedc_$lib.so > gpurun_out/${t}_lat.log 2>&1 || exit 1
  echo "latency17 $lib $(grep '^{' gpurun_out/${t}_lat.log | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
done
