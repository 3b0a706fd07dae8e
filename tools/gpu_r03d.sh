set -o pipefail
mkdir -p gpurun_out
for cfg in "--n 131072" "--config c2"; do
 for inf in 8 12 16; do
  timeout -k 10 120 python3 bench.py $cfg --inflight $inf --steps 60 --warmup 8 --no-cpu-baseline --profile-steps 1 --lib ed25519-consensus_amd/csrc/libedc_s16.so > gpurun_out/r03d.log 2>&1 || { tail -3 gpurun_out/r03d.log; exit 1; }
  echo "$cfg inflight $inf: $(tail -1 gpurun_out/r03d.log | grep -o '"value": [0-9.]*, [^,]*, [^,]*, [^,]*, [^,]*, "ms_per_step": [0-9.]*')"
 done
done
