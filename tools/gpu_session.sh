#!/bin/bash
# GPU-box session runner (replaces the per-session gpu_r03*.sh scripts). Runs the named steps in
# order, each under its own time limit, logs to gpurun_out/<tag>_<step>.log, and stops at the first
# failure (a GPU fault, abort or time limit ends the call: nothing else touches the GPU after it).
#
#   tools/gpu_session.sh <tag> <step> [<step> ...]
#
# steps:
#   tests            every -m gpu test            tests=<pytest args>  a subset, e.g. tests=tests/test_gpu_prehashed.py
#   smoke            __graft_entry__.smoke()
#   driver           the driver's bench command (--gpus 1 --steps 20 --warmup 5, with the CPU baseline)
#   c3 | c2 | c5     40-step benches of configs[2] / configs[1] / configs[4] (no CPU baseline)
#   n17 | n18 | n19  2^17 / 2^18 / 2^19 shards of the vote batch (strong-scaling per-GPU rates)
#   n17s | c2s       2^17 shards / configs[1] over 1600 steps: the steady state (40 steps of a
#                    0.25 ms batch are mostly the fill and drain of 16 batches in flight)
#   fallback         tools/fallback_bench.py (configs[3])    host  tools/host_bench.py
#   small            tools/smallbatch_bench.py               multi tools/multi_bench.py
#   prof             rocprofv3 kernel-trace stats of the bench, one batch at a time and pipelined
#   pmc              tools/pmc_passes.sh (VALU / INT / FETCH / WRITE passes; then tools/pmc_summary.py here)
#   rccl1            forced single-rank RCCL loop (process group + per-batch all-gather)
#   gloo2            two ranks sharing the GPU over gloo, weak and strong
#   lat | lat=<v>    tools/latency_probe.py (one synchronous batch at a time) on the product / a variant build
#   gloo4            four ranks sharing the GPU over gloo (weak, with the strong shape beside it)
#   ab=<v1,v2,..>    alternating A/B of variant builds csrc/libedc_<v>.so ("base" = libedc.so) on
#                    AB_CONFIGS (default "c3 n17 c2 c5"), AB_REPS rounds (default 2)
#   bench=<args>     one bench.py run with these arguments (commas for spaces)
#   pre              configs[2] with prehashed items (edc_batch_submit_prehashed_device)
#   m17 | m16        8 consecutive 2^17 vote shards / configs[1] batches per launch (--multi 8, union first)
#   m17x | m16x      the same batch by batch (--multi-exact)
#   hapi | hapi0     the host_api leg: chunked (default) / one piece
#   htrace           rocprofv3 copy + kernel trace of synchronous host-buffer calls, last call's timeline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
D=ed25519-consensus_amd/csrc
log() { echo "gpurun_out/${tag}_$1.log"; }

run() {   # run <name> <timeout> <cmd...>: stop the session on failure
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$(log "$name")" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 "$(log "$name")" | cut -c1-400)"
  if [ $rc -ne 0 ]; then tail -15 "$(log "$name")"; exit $rc; fi
}

summ() {  # one line per bench log: value, ms/step, decode roofline fraction
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(f"{sys.argv[2]:>14} {d['value']:.4e} sigs/s {d['ms_per_step']:.3f} ms/step frac {r.get('frac')} "
      f"pipe {r.get('pipeline', {}).get('frac')} lat {d.get('batch_latency_ms')} "
      + " ".join(f"{k[:8]}={v:.3f}" for k, v in d.get("phases_ms", {}).items()))
EOF
}

bench_step() {   # bench_step <name> <args...>
  local name=$1; shift
  run "$name" 400 python3 -u bench.py "$@"
  summ "$(log "$name")" "$name" | tee -a "gpurun_out/${tag}_summary.log"
}

for step in "$@"; do
  case "$step" in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s ;;
    tests=*) run tests 900 python -u -m pytest ${step#tests=} -m gpu -x -v --timeout 300 --timeout-method thread -s ;;
    smoke) run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) bench_step driver --gpus 1 --steps 20 --warmup 5 ;;
    c3) bench_step c3 --steps 40 --warmup 5 --no-cpu-baseline ;;
    c2) bench_step c2 --config c2 --steps 40 --warmup 5 --no-cpu-baseline ;;
    c5) bench_step c5 --config c5 --steps 12 --warmup 3 --no-cpu-baseline ;;
    n17) bench_step n17 --n 131072 --steps 40 --warmup 5 --no-cpu-baseline ;;
    n17s) bench_step n17s --n 131072 --steps 1600 --warmup 5 --no-cpu-baseline ;;
    c2s) bench_step c2s --config c2 --steps 1600 --warmup 5 --no-cpu-baseline ;;
    n18) bench_step n18 --n 262144 --steps 40 --warmup 5 --no-cpu-baseline ;;
    n19) bench_step n19 --n 524288 --steps 40 --warmup 5 --no-cpu-baseline ;;
    bench=*) a=${step#bench=}; bench_step bench ${a//,/ } ;;
    pre) bench_step pre --prehashed --steps 40 --warmup 5 --no-cpu-baseline ;;
    m17) bench_step m17 --n 131072 --multi 8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    m16) bench_step m16 --config c2 --multi 8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    m17x) bench_step m17x --n 131072 --multi 8 --multi-exact --steps 20 --warmup 5 --no-cpu-baseline ;;
    m16x) bench_step m16x --config c2 --multi 8 --multi-exact --steps 20 --warmup 5 --no-cpu-baseline ;;
    fallback) run fallback 300 python3 -u tools/fallback_bench.py ;;
    host) run host 300 python3 -u tools/host_bench.py ;;
    small) run small 300 python3 -u tools/smallbatch_bench.py ;;
    multi) run multi 300 python3 -u tools/multi_bench.py ;;
    prof)
      run prof1 300 env EDC_SINGLE_STREAM=1 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof1 -o k -- python3 -u bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-host-api
      run profp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_profp -o k -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-api
      # --stats layout from the trace database (this image's rocprofv3 writes rocpd databases)
      for p in prof1 profp; do
        python3 tools/rocpd_stats.py "gpurun_out/${tag}_$p/k_results.db" > "gpurun_out/${tag}_${p}_kernel_stats.csv" || exit 1
      done ;;
    pmc) run pmc 600 bash tools/pmc_passes.sh ;;
    # FETCH_SIZE / WRITE_SIZE passes of one build (base = libedc.so), one batch at a time:
    # gpurun_out/<tag>_pmcf_<v>_{fetch,write}/ for tools/pmc_batch_table.py-style summaries
    pmcf=*)
      v=${step#pmcf=}; lib=$PWD/$D/libedc_$v.so; [ "$v" = base ] && lib=$PWD/$D/libedc.so
      for c in FETCH_SIZE WRITE_SIZE; do
        run pmcf_${v}_$c 150 env EDC_SINGLE_STREAM=1 timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/${tag}_pmcf_${v}_$c -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-host-api --profile-steps 1 --lib "$lib"
      done ;;
    rccl1) run rccl1 300 env EDC_FORCE_DIST=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 40 --warmup 5 --no-cpu-baseline ;;
    gloo2)
      run gloo2_weak 300 env EDC_DIST_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --scaling weak --steps 20 --warmup 3 --no-cpu-baseline
      run gloo2_strong 300 env EDC_DIST_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --scaling strong --steps 20 --warmup 3 --no-cpu-baseline ;;
    lat) run lat 300 python3 -u tools/latency_probe.py --sizes c3,n17,c2,n150 ;;
    lat=*) v=${step#lat=}; run lat_$v 300 python3 -u tools/latency_probe.py --sizes c3,n17,c2,n150 --lib "$PWD/$D/libedc_$v.so" ;;
    gloo4) run gloo4 300 env EDC_DIST_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 20 --warmup 3 --no-cpu-baseline ;;
    # bench.py's own launcher (no outer torch.distributed.run): two gloo ranks sharing the GPU
    # must run and report n_gpus 2 / comm.world_size 2; two RCCL ranks on a one-GPU box must
    # refuse within seconds (non-zero exit, expected)
    launch2g) run launch2g 300 env EDC_DIST_BACKEND=gloo python3 -u bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline ;;
    launch2r)
      t0=$(date +%s.%N)
      timeout -k 10 120 python3 -u bench.py --gpus 2 --steps 4 > "$(log launch2r)" 2>&1
      rc=$?; t1=$(date +%s.%N)
      echo "[launch2r] rc=$rc (expected non-zero) in $(python3 -c "print(round($t1-$t0,1))") s: $(grep -m1 'GPU(s) visible' "$(log launch2r)")" | tee -a "$(log launch2r)"
      if [ $rc -eq 0 ] || [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit 1; fi ;;
    # the strong shape's per-rank shard at the driver's run length: 20 steps of 2^20 split over
    # 8 ranks = 160 batches of 2^17 per GPU (over 4 ranks: 80 of 2^18)
    n17x160) bench_step n17x160 --n 131072 --steps 160 --warmup 5 --no-cpu-baseline --no-host-api ;;
    n18x80) bench_step n18x80 --n 262144 --steps 80 --warmup 5 --no-cpu-baseline --no-host-api ;;
    n17x20) bench_step n17x20 --n 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-host-api ;;
    # host-buffer synchronous calls (bench.py's host_api leg): chunked (default) and one piece
    hapi) run hapi 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline
          python3 -c "import json,sys; d=json.loads(open('$(log hapi)').read().strip().splitlines()[-1]); print('hapi', json.dumps(d['host_api']))" | tee -a "gpurun_out/${tag}_summary.log" ;;
    hapi=*) v=${step#hapi=}; run hapi_$v 300 env EDC_HOST_BODY_CHUNKS=$v python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline
          python3 -c "import json,sys; d=json.loads(open('$(log hapi_$v)').read().strip().splitlines()[-1]); print('hapi=$v', json.dumps(d['host_api']))" | tee -a "gpurun_out/${tag}_summary.log" ;;
    hapi0) run hapi0 300 env EDC_HOST_CHUNKS=0 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline
          python3 -c "import json,sys; d=json.loads(open('$(log hapi0)').read().strip().splitlines()[-1]); print('hapi0', json.dumps(d['host_api']))" | tee -a "gpurun_out/${tag}_summary.log" ;;
    # copies and kernels of one synchronous host-buffer call on one time axis (tools/host_timeline.py)
    htrace)
      run htrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${tag}_htrace -o ht -- python3 -u tools/host_trace.py
      python3 tools/host_timeline.py gpurun_out/${tag}_htrace > "gpurun_out/${tag}_htrace_timeline.txt" || exit 1
      head -1 "gpurun_out/${tag}_htrace_timeline.txt" ;;
    ab=*)
      IFS=, read -ra libs <<< "${step#ab=}"
      for rep in $(seq 1 "${AB_REPS:-2}"); do
        for v in "${libs[@]}"; do
          lib=$D/libedc_$v.so; [ "$v" = base ] && lib=$D/libedc.so
          for c in ${AB_CONFIGS:-c3 n17 c2 c5}; do
            case $c in
              c3) a="--steps 40";; c2) a="--config c2 --steps 40";; c5) a="--config c5 --steps 12";;
              n17) a="--n 131072 --steps 40";; n17x20) a="--n 131072 --steps 20";; driver) a="--steps 20";; *) a="$c";;
            esac
            run ab 300 python3 -u bench.py $a --warmup 5 --no-cpu-baseline --profile-steps 1 --lib "$PWD/$lib"
            summ "$(log ab)" "$c-$v" | tee -a "gpurun_out/${tag}_ab_summary.log"
          done
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
