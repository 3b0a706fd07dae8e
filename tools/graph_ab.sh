#!/bin/bash
# GPU-box: graph-replay tests, device timelines (EDC_BATCH_STAMPS build) and an alternating A/B of
# graphs off / on for 20-step 2^17 and configs[2] runs (EDC_GRAPHS=0/1). Logs: gpurun_out/s3_*
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=ed25519-consensus_amd/csrc/libedc_bstamps.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 || { tail -30 gpurun_out/s3_tests.log; exit 1; }
tail -2 gpurun_out/s3_tests.log
timeout -k 10 200 python3 -u tools/batch_timeline.py --lib $L --n 131072 --steps 20 > gpurun_out/s3_tl17_off.log 2>&1 || exit 1
EDC_GRAPHS=1 timeout -k 10 200 python3 -u tools/batch_timeline.py --lib $L --n 131072 --steps 20 > gpurun_out/s3_tl17_on.log 2>&1 || exit 1
grep "^{" gpurun_out/s3_tl17_off.log gpurun_out/s3_tl17_on.log
for r in 1 2; do
 for g in 0 1; do
  EDC_GRAPHS=$g timeout -k 10 200 python3 -u bench.py --n 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > gpurun_out/s3_n17_g$g.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/s3_n17_g$g.log').read().strip().splitlines()[-1]);print('n17x20 graphs=$g',d['value'],d['ms_per_step'])"
  EDC_GRAPHS=$g timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-api --profile-steps 1 > gpurun_out/s3_c3_g$g.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/s3_c3_g$g.log').read().strip().splitlines()[-1]);print('c3x20 graphs=$g',d['value'],d['ms_per_step'])"
 done
done
