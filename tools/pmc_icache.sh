#!/bin/bash
# GPU-box: instruction-fetch counters of each kernel, one batch at a time, for the builds named in
# $LIBS ("base" = libedc.so, else csrc/libedc_<v>.so), on the configs in $CONFIGS (bench --config).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export EDC_SINGLE_STREAM=1
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_list_avail.txt 2>&1
grep -oE "SQC?_(ICACHE|IFETCH|WAIT_INST|INST_LEVEL|WAVE_CYCLES|BUSY_CYCLES|INSTS_VALU)[A-Z_]*" gpurun_out/pmc_list_avail.txt | sort -u > gpurun_out/pmc_icache_names.txt
cat gpurun_out/pmc_icache_names.txt
for lib in ${LIBS:-base}; do
  for cfg in ${CONFIGS:-c3}; do
    libarg=""
    [ "$lib" != base ] && libarg="--lib ed25519-consensus_amd/csrc/libedc_$lib.so"
    timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES} \
      -d gpurun_out/pmc_ic_${lib}_$cfg -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --profile-steps 1 --config $cfg $libarg \
      > gpurun_out/pmc_ic_${lib}_$cfg.log 2>&1 || { echo "pass $lib $cfg failed"; exit 1; }
    echo "pass $lib $cfg ok"
  done
done
