# GPU-box: bench rotating over exactly `inflight` slots: default config, driver command, 2^17,
# and the multi-rank rehearsals (forced single-rank RCCL, 2 gloo ranks on this GPU).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03ai
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_c3.log 2>&1 || exit 1
  echo "c3-40 $(tail -1 gpurun_out/${t}_c3.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"inflight": [0-9]*' | tr '\n' ' ')"
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_drv.log 2>&1 || exit 1
  echo "driver $(tail -1 gpurun_out/${t}_drv.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
  timeout -k 10 200 python3 bench.py --n 131072 --steps 40 --warmup 6 --no-cpu-baseline > gpurun_out/${t}_n17.log 2>&1 || exit 1
  echo "n17 $(tail -1 gpurun_out/${t}_n17.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"inflight": [0-9]*' | tr '\n' ' ')"
done
EDC_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_rccl_forced1.log 2>&1 || { echo rccl_fail; tail -20 gpurun_out/${t}_rccl_forced1.log; exit 1; }
echo "rccl1 $(grep '^{' gpurun_out/${t}_rccl_forced1.log | tail -1 | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/${t}_weak2_gloo.log 2>&1 || { echo weak_fail; tail -20 gpurun_out/${t}_weak2_gloo.log; exit 1; }
echo "weak2 $(grep '^{' gpurun_out/${t}_weak2_gloo.log | tail -1 | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scaling strong --steps 20 --warmup 3 > gpurun_out/${t}_strong2_gloo.log 2>&1 || { echo strong_fail; tail -20 gpurun_out/${t}_strong2_gloo.log; exit 1; }
echo "strong2 $(grep '^{' gpurun_out/${t}_strong2_gloo.log | tail -1 | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
