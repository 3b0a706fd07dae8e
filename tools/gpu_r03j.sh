# GPU-box: plan / scatter-path parity, then alternating A/B of the two-region scatter (configs[4],
# configs[1], configs[2]) against the session-start build (libedc_base.so), then a 2^17 trace
# with the per-queue view (tools/queue_gaps.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_plans.py tests/test_gpu_config4.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_tests.log; [ $rc -eq 0 ] || exit $rc
B=ed25519-consensus_amd/csrc/libedc_base.so; N=ed25519-consensus_amd/csrc/libedc.so
for cfg in c5 c2 c5 c3 c2 c3; do
  for lib in $B $N; do
    timeout -k 10 180 python3 bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --lib $lib > gpurun_out/${t}_ab.log 2>&1 || { tail -3 gpurun_out/${t}_ab.log; exit 1; }
    echo "$cfg $(basename $lib) $(tail -1 gpurun_out/${t}_ab.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_bin": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_ab_all.log
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_trace -o run --output-format csv -- \
  python3 bench.py --n 131072 --inflight 8 --steps 25 --warmup 3 --no-cpu-baseline --profile-steps 1 > gpurun_out/${t}_trace_bench.log 2>&1 || { echo trace_fail; tail -5 gpurun_out/${t}_trace_bench.log; exit 1; }
f=$(find gpurun_out/${t}_trace -name '*kernel_trace.csv' | head -1)
head -1 $f
python3 tools/queue_gaps.py $f > gpurun_out/${t}_queue_gaps.txt 2>&1; cat gpurun_out/${t}_queue_gaps.txt
python3 tools/timeline.py $f --batches 20 > gpurun_out/${t}_timeline.txt 2>&1; head -8 gpurun_out/${t}_timeline.txt
echo done
