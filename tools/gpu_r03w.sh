# GPU-box: column chains alternating asm / compiler v_mad_u64_u32 (fewer hazard s_nops) against
# the all-asm chains (libedc_cur.so): parity, then alternating A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03w
D=ed25519-consensus_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plans.py tests/test_gpu_edges.py tests/test_gpu_keysplit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"decompress_R": [0-9.]*\|"msm_bucket": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2 3; do
  for lib in cur nop; do ab "--config c3" $lib c3; ab "--n 131072" $lib n17; done
done
for lib in cur nop; do ab "--config c2" $lib c2; done
