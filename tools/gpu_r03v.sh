# GPU-box: accumulation at 5 waves per SIMD (96 VGPRs, 124 B/lane spilled) against 4 (128 VGPRs).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03v
D=ed25519-consensus_amd/csrc
ab() {
  timeout -k 10 180 python3 bench.py $1 --steps 40 --warmup 6 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"msm_bucket": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2 3; do
  for lib in cur acc5; do ab "--config c3" $lib c3; ab "--config c2" $lib c2; done
done
