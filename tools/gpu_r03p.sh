# GPU-box: parity of the branch-free SHA-512 message words (0..1024-byte messages vs hashlib and
# the oracle, every golden fixture), then A/B against the previous tree (hw) on configs[4]/[2]/[1].
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-r03p}
D=ed25519-consensus_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiblock.py tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"challenge_sha512": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in sha sort; do ab "--config c5 --steps 20" $lib c5; ab "--config c3 --steps 40" $lib c3; ab "--config c2 --inflight 16 --steps 40" $lib c2; done
done
