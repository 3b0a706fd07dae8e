#!/bin/bash
# GPU-box: the non-headline BASELINE configs and the strong-scaling rehearsal.
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-r02}
timeout -k 10 200 python -u bench.py --config c2 --steps 40 --warmup 4 --inflight 8 > gpurun_out/${tag}_bench_c2.log 2>&1 || { echo c2_fail; tail -5 gpurun_out/${tag}_bench_c2.log; exit 1; }
echo "c2 $(tail -1 gpurun_out/${tag}_bench_c2.log | cut -c1-220)"
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 > gpurun_out/${tag}_bench_c5.log 2>&1 || { echo c5_fail; tail -5 gpurun_out/${tag}_bench_c5.log; exit 1; }
echo "c5 $(tail -1 gpurun_out/${tag}_bench_c5.log | cut -c1-220)"
for n in 131072 262144 524288; do
  timeout -k 10 200 python -u bench.py --n $n --steps 40 --warmup 4 --inflight 8 --no-cpu-baseline > gpurun_out/${tag}_bench_n$n.log 2>&1 || { echo n${n}_fail; exit 1; }
  echo "n=$n $(tail -1 gpurun_out/${tag}_bench_n$n.log | cut -c1-200)"
done
# strong-scaling rehearsal of the multi-rank path: 2 ranks split ONE 2^20 batch, both on this GPU (gloo all-gather)
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scaling strong --steps 20 --warmup 3 > gpurun_out/${tag}_strong2_gloo.log 2>&1 || { echo strong_fail; tail -20 gpurun_out/${tag}_strong2_gloo.log; exit 1; }
echo "strong2 $(grep '^{' gpurun_out/${tag}_strong2_gloo.log | tail -1 | cut -c1-300)"
# weak-scaling rehearsal (the driver's default multi-GPU shape): 2 ranks, 2^20 each, both on this GPU
EDC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/${tag}_weak2_gloo.log 2>&1 || { echo weak_fail; tail -20 gpurun_out/${tag}_weak2_gloo.log; exit 1; }
echo "weak2 $(grep '^{' gpurun_out/${tag}_weak2_gloo.log | tail -1 | cut -c1-300)"
# the shard size of a 2^20 batch over 8 GPUs, with the validator keys in the key cache (split coefficients)
timeout -k 10 200 python -u bench.py --n 131072 --steps 40 --warmup 4 --inflight 8 --keycache --no-cpu-baseline > gpurun_out/${tag}_bench_n131072_keycache.log 2>&1 || { echo kc_fail; exit 1; }
echo "n=131072 keycache $(tail -1 gpurun_out/${tag}_bench_n131072_keycache.log | cut -c1-200)"
timeout -k 10 200 python -u tools/host_bench.py > gpurun_out/${tag}_host_bench.log 2>&1 || { echo host_fail; tail -5 gpurun_out/${tag}_host_bench.log; exit 1; }
tail -3 gpurun_out/${tag}_host_bench.log
