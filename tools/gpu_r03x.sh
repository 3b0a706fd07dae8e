# GPU-box: window-width sweep at the small-shard sizes with 16 in flight (the auto choice was
# swept in round 2 at 8 in flight).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03x
run() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for b in 0 13 15 16; do run "--n 131072 --window-bits $b" "n17-c$b"; done
  for b in 0 12 14 15; do run "--config c2 --window-bits $b" "c2-c$b"; done
done
