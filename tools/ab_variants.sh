#!/bin/bash
# A/B measurement of variant builds (ed25519-consensus_amd/csrc/libedc_<name>.so) on the GPU box:
# one short bench per variant, phase timings only. Usage: tools/ab_variants.sh name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=ed25519-consensus_amd/csrc/libedc_$v.so
  [ "$v" = "base" ] && lib=ed25519-consensus_amd/csrc/libedc.so
  timeout -k 10 120 python -u bench.py --lib $PWD/$lib --steps ${AB_STEPS:-20} --warmup 2 --no-cpu-baseline --profile-steps 3 ${AB_ARGS} > gpurun_out/ab_$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v FAILED rc=$rc"; tail -5 gpurun_out/ab_$v.log; [ $rc -ge 124 ] && exit $rc; continue; fi
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1])
print('%-12s %8.3f ms/step  %.3e sigs/s ' % ('$v', d['ms_per_step'], d['value']), ' '.join('%s=%.3f'%(k[:10],v) for k,v in d['phases_ms'].items()))
"
done
