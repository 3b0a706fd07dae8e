# GPU-box, round-3 measurement set (part A): GPU suite, smoke, the driver's bench command (with
# the CPU baseline and the openssl anchor), the 40-step default, rocprofv3 kernel stats of one
# batch at a time (the roofline's cross-check) and of the pipelined default.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-r03f}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${t}_gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/${t}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${t}_smoke.log 2>&1 || { tail -5 gpurun_out/${t}_smoke.log; exit 1; }
tail -1 gpurun_out/${t}_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${t}_bench_driver.log 2>&1 || { tail -5 gpurun_out/${t}_bench_driver.log; exit 1; }
echo "driver $(tail -1 gpurun_out/${t}_bench_driver.log | cut -c1-200)"
timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${t}_bench_40.log 2>&1 || exit 1
echo "40 $(tail -1 gpurun_out/${t}_bench_40.log | cut -c1-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_prof1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline > gpurun_out/${t}_bench_prof1.log 2>&1 || { echo prof_fail; tail -5 gpurun_out/${t}_bench_prof1.log; exit 1; }
echo "prof1 $(tail -1 gpurun_out/${t}_bench_prof1.log | grep -o '"avg_launch_ms": [0-9.]*')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${t}_profp -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${t}_bench_profp.log 2>&1 || { echo profp_fail; tail -5 gpurun_out/${t}_bench_profp.log; exit 1; }
head -6 $(find gpurun_out/${t}_prof1 -name '*kernel_stats.csv' | head -1) | cut -c1-160
echo done
