# GPU-box: marginal pipeline cost of each batch phase. Probe builds skip one phase's launches
# (EDC_PROBE_SKIP bit: 2 SHA-512, 4 coefficients, 8 binning, 16 decompression, 32 sort +
# accumulation, 64 bin reduction, 128 window combine + Horner, 256 bucket sort; after each slot's first batch, whose outputs the repeated batches reuse), all with
# 16 slots; throughput at 16 in flight against the full 16-slot build, for the given config.
# Usage: CFG="--n 131072" bash tools/phase_cost.sh
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=${TAG:-phase_cost}
D=ed25519-consensus_amd/csrc
# p256 (sort skipped) reuses a slot's first sorted array; when a later batch's plan grows the
# workspace the array is stale and the accumulation gathers out of bounds (round 5: a GPU fault),
# so it is not in the default list
for lib in ${LIBS:-s16 p2 p4 p8 p16 p32 p64 p128 s16}; do
  timeout -k 10 180 python3 bench.py $CFG --inflight ${INF:-16} --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$lib.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
done
