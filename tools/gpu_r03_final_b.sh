# GPU-box, round-3 measurement set (part B): the other BASELINE configs, shard sizes, the
# multi-rank rehearsals (2 gloo ranks on this GPU, forced single-rank RCCL), the in-process
# multi-device pipeline, small calls, configs[3]'s fallback and the PCIe-inclusive rates.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-r03f}
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline > gpurun_out/${t}_bench_$name.log 2>&1 || { echo ${name}_fail; tail -5 gpurun_out/${t}_bench_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/${t}_bench_$name.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"inflight": [0-9]*\|"batch_latency_ms": [0-9.]*' | tr '\n' ' ')"
}
run c2 --config c2 --steps 40 --warmup 6
run c5 --config c5 --steps 12 --warmup 3
run n17 --n 131072 --steps 60 --warmup 8
run n18 --n 262144 --steps 60 --warmup 8
run n19 --n 524288 --steps 40 --warmup 6
run n17kc --n 131072 --steps 60 --warmup 8 --keycache
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scaling strong --steps 20 --warmup 3 > gpurun_out/${t}_strong2_gloo.log 2>&1 || { echo strong_fail; tail -20 gpurun_out/${t}_strong2_gloo.log; exit 1; }
echo "strong2 $(grep '^{' gpurun_out/${t}_strong2_gloo.log | tail -1 | cut -c1-200)"
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/${t}_weak2_gloo.log 2>&1 || { echo weak_fail; tail -20 gpurun_out/${t}_weak2_gloo.log; exit 1; }
echo "weak2 $(grep '^{' gpurun_out/${t}_weak2_gloo.log | tail -1 | cut -c1-200)"
EDC_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 1 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_rccl_forced1.log 2>&1 || { echo rccl_fail; tail -20 gpurun_out/${t}_rccl_forced1.log; exit 1; }
echo "rccl1 $(grep '^{' gpurun_out/${t}_rccl_forced1.log | tail -1 | cut -c1-200)"
for spec in "0 6" "0,0 4" "0,0,0,0 2"; do
  set -- $spec
  timeout -k 10 200 python3 tools/multi_bench.py --devices $1 --inflight $2 > gpurun_out/${t}_multi.log 2>&1 || { tail -5 gpurun_out/${t}_multi.log; exit 1; }
  grep '^{' gpurun_out/${t}_multi.log | tee -a gpurun_out/${t}_multi_all.log
done
timeout -k 10 200 python3 tools/smallbatch_bench.py --sizes 8,64,150,1024 > gpurun_out/${t}_smallbatch.log 2>&1 || { tail -5 gpurun_out/${t}_smallbatch.log; exit 1; }
grep -o '"n": [0-9]*, "keys": "[a-z]*", "keycache": [a-z]*, "gpu_batch_ms": [0-9.]*, "gpu_batch_dev_ms": [0-9.]*' gpurun_out/${t}_smallbatch.log
timeout -k 10 300 python3 tools/fallback_bench.py > gpurun_out/${t}_fallback_c4.log 2>&1 || { echo fb_fail; tail -5 gpurun_out/${t}_fallback_c4.log; exit 1; }
tail -3 gpurun_out/${t}_fallback_c4.log | cut -c1-300
timeout -k 10 200 python3 tools/host_bench.py > gpurun_out/${t}_host_bench.log 2>&1 || { echo host_fail; tail -5 gpurun_out/${t}_host_bench.log; exit 1; }
tail -3 gpurun_out/${t}_host_bench.log | cut -c1-300
echo done
