set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo bench_fail; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline > gpurun_out/bench_prof1.log 2>&1 || { echo prof_fail; tail -20 gpurun_out/bench_prof1.log; exit 1; }
tail -1 gpurun_out/bench_prof1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof4.log 2>&1 || { echo prof4_fail; tail -20 gpurun_out/bench_prof4.log; exit 1; }
tail -1 gpurun_out/bench_prof4.log
