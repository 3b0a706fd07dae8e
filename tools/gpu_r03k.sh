# GPU-box: burst probe (how many in-flight batches run at once) at 2^17 and configs[1], a kernel
# trace of 8-batch bursts (queues running at once), then A/B of the scatter block size on configs[4].
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03k
timeout -k 10 120 python3 tools/burst_probe.py --n 131072 --keys 150 > gpurun_out/${t}_burst_n17.log 2>&1 || { tail -3 gpurun_out/${t}_burst_n17.log; exit 1; }
grep '^{' gpurun_out/${t}_burst_n17.log
timeout -k 10 120 python3 tools/burst_probe.py --n 65536 --keys 0 > gpurun_out/${t}_burst_c2.log 2>&1 || { tail -3 gpurun_out/${t}_burst_c2.log; exit 1; }
grep '^{' gpurun_out/${t}_burst_c2.log
timeout -k 10 120 python3 tools/burst_probe.py --n 1048576 --keys 150 --ks 1,2,4,8 > gpurun_out/${t}_burst_n20.log 2>&1 || { tail -3 gpurun_out/${t}_burst_n20.log; exit 1; }
grep '^{' gpurun_out/${t}_burst_n20.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${t}_trace -o run --output-format csv -- \
  python3 tools/burst_probe.py --n 131072 --keys 150 --ks 8 --reps 3 > gpurun_out/${t}_trace_probe.log 2>&1 || { echo trace_fail; tail -5 gpurun_out/${t}_trace_probe.log; exit 1; }
B=ed25519-consensus_amd/csrc/libedc_base.so; N=ed25519-consensus_amd/csrc/libedc.so; S=ed25519-consensus_amd/csrc/libedc_s1024.so
for cfg in c5 c5; do
  for lib in $B $N $S; do
    timeout -k 10 180 python3 bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --lib $lib > gpurun_out/${t}_ab.log 2>&1 || { tail -3 gpurun_out/${t}_ab.log; exit 1; }
    echo "$cfg $(basename $lib) $(tail -1 gpurun_out/${t}_ab.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_bin": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_ab_all.log
  done
done
echo done
