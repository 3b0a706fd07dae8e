# GPU-box: the 1024-lane scatter build (libedc.so) against the session-start build on every
# config, then 12 / 16 batches in flight (16-slot build) at 2^17 and configs[1].
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03l
timeout -k 10 300 python -u -m pytest tests/test_gpu_plans.py tests/test_gpu_config4.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
B=ed25519-consensus_amd/csrc/libedc_base.so; N=ed25519-consensus_amd/csrc/libedc.so; S=ed25519-consensus_amd/csrc/libedc_s16.so
ab() {  # cfg-args lib tag
  timeout -k 10 180 python3 bench.py $1 --steps 30 --warmup 5 --no-cpu-baseline --lib $2 > gpurun_out/${t}_ab.log 2>&1 || { tail -3 gpurun_out/${t}_ab.log; exit 1; }
  echo "$3 $(basename $2) $(tail -1 gpurun_out/${t}_ab.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_bin": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_ab_all.log
}
for rep in 1 2; do
  for lib in $B $N; do
    ab "--config c3" $lib c3
    ab "--config c2 --inflight 8" $lib c2
    ab "--n 131072 --inflight 8" $lib n17
  done
done
for inf in 8 12 16; do
  ab "--n 131072 --inflight $inf" $S n17-if$inf
  ab "--config c2 --inflight $inf" $S c2-if$inf
done
ab "--config c3 --inflight 10" $S c3-if10
R=ed25519-consensus_amd/csrc/libedc_r256.so
for lib in $N $R $N $R; do
  ab "--n 131072 --inflight 8" $lib n17
  ab "--config c2 --inflight 8" $lib c2
done
echo done
