# GPU-box: deeper pipelines (32-slot build) at 2^17 and configs[1] against the 16-slot product.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03s
D=ed25519-consensus_amd/csrc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 60 --warmup 8 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  ab "--n 131072 --inflight 16" cur n17-if16
  ab "--n 131072 --inflight 24" s32 n17-if24
  ab "--n 131072 --inflight 32" s32 n17-if32
  ab "--config c2 --inflight 16" cur c2-if16
  ab "--config c2 --inflight 24" s32 c2-if24
  ab "--config c2 --inflight 32" s32 c2-if32
done
