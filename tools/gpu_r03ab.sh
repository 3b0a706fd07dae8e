# GPU-box: SHA-512 next-block message prefetch (pf: occupancy 4; pf5: forced 5 waves/SIMD, 20 B
# spilled) against the current tree, on configs[4] and configs[2].
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
t=r03ab
D=ed25519-consensus_amd/csrc
ab() {
  timeout -k 10 180 python3 bench.py $1 --warmup 4 --no-cpu-baseline --profile-steps 1 --lib $D/libedc_$2.so > gpurun_out/${t}.log 2>&1 || { tail -3 gpurun_out/${t}.log; exit 1; }
  echo "$3 $2 $(tail -1 gpurun_out/${t}.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"challenge_sha512": [0-9.]*\|"verdict_ok": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/${t}_all.log
}
for rep in 1 2; do
  for lib in cur pf pf5; do ab "--config c5 --steps 12" $lib c5; ab "--config c3 --steps 40" $lib c3; done
done
