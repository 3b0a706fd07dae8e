# GPU-box: in-flight depth under the driver's command (20 timed steps after 5 warmup steps).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03ad
for rep in 1 2 3; do
  for inf in 4 6 8 12; do
    timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --inflight $inf --no-cpu-baseline --profile-steps 1 > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
    echo "if$inf $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
  done
done
