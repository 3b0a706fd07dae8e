set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06x_inflight_sweep.log
: > $out
for rep in 1 2; do
  for cfg in "131072 4" "131072 6" "131072 8" "131072 12" "131072 16" "262144 4" "262144 6" "262144 8" "262144 12" "524288 4" "524288 6" "524288 8"; do
    set -- $cfg
    timeout -k 10 200 python3 -u bench.py --n $1 --steps 20 --warmup 5 --inflight $2 --no-cpu-baseline --no-host-api > gpurun_out/r06x_one.log 2>&1 || { tail -5 gpurun_out/r06x_one.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06x_one.log').read().strip().splitlines()[-1]); print('n=$1 inflight=$2 rep=$rep', '%.4e'%d['value'], d['ms_per_step'])" | tee -a $out
  done
done
