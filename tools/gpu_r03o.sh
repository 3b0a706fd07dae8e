# GPU-box: (1) parity of the current tree; (2) price of a kernel boundary inside the pipeline:
# 10 extra empty (e10) or 1 MB-writing (w10) dependent launches per batch against the 16-slot
# build (s16); (3) hw = s16 + result block stored straight to pinned host memory (no copy
# packet); sha = hw + SHA-512 regrouped over up to 1024 items per workgroup.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03o
D=ed25519-consensus_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plans.py tests/test_gpu_multi.py tests/test_gpu_keysplit.py tests/test_gpu_multiblock.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"challenge_sha512": [0-9.]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in s16 e10 w10 hw; do ab "--n 131072 --inflight 16" $lib n17; done
done
for rep in 1 2; do
  for lib in s16 hw sha; do ab "--config c2 --inflight 16" $lib c2; ab "--config c5 --steps 20" $lib c5; ab "--config c3 --inflight 8" $lib c3; done
done
