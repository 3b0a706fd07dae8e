# GPU-box: bin reduction with 16 lanes per bin (fewer additions, longer chains) against 32.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03aa
D=ed25519-consensus_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_plans.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc (product)"; tail -1 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_bucket": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur r16; do ab "--config c3 --steps 40" $lib c3; ab "--config c2 --steps 40" $lib c2; ab "--n 131072 --steps 40" $lib n17; ab "--config c5 --steps 12" $lib c5; done
done
