# GPU-box: decode on a second stream for slot 0 only (dual0: 16 slots + 1 queue; dual0s15: 15 + 1)
# against the single-stream product: pipelined throughput, driver command, small calls, latency.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03ag
D=ed25519-consensus_amd/csrc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur dual0 dual0s15; do
    ab "--config c3 --steps 20" $lib c3-20
    ab "--n 131072 --steps 40 --inflight 15" $lib n17
    ab "--config c2 --steps 40 --inflight 15" $lib c2
  done
done
for lib in cur dual0 dual0s15; do
  timeout -k 10 200 python3 tools/smallbatch_bench.py --sizes 64,150,1024 --reps 30 --lib $D/libedc_$lib.so > gpurun_out/${t}_sb.log 2>&1 || { tail -5 gpurun_out/${t}_sb.log; exit 1; }
  echo "smallbatch $lib"; grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*' gpurun_out/${t}_sb.log | tee -a gpurun_out/${t}_all.log
  timeout -k 10 200 python3 tools/burst_probe.py --n 1048576 --ks 1 --lib $D/libedc_$lib.so > gpurun_out/${t}_lat.log 2>&1 || exit 1
  echo "latency $lib $(grep '^{' gpurun_out/${t}_lat.log)" | tee -a gpurun_out/${t}_all.log
done
