set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03a_bench_driver.log 2>&1 || exit 1
tail -1 gpurun_out/r03a_bench_driver.log | cut -c1-300
timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r03a_bench_40.log 2>&1 || exit 1
tail -1 gpurun_out/r03a_bench_40.log | cut -c1-300
TAG=r03a_n17 BENCH_ARGS="--n 131072 --inflight 8" bash tools/trace_bench.sh > /dev/null || exit 1
TAG=r03a_c2 BENCH_ARGS="--config c2 --inflight 8" bash tools/trace_bench.sh > /dev/null || exit 1
echo done
