#!/bin/bash
# GPU-box: kernel trace of tools/fallback_bench.py (configs[3]); per-kernel stats under gpurun_out/trace_fb_*.
set -o pipefail
mkdir -p gpurun_out
tag=${TAG:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_fb_$tag -o run --output-format csv -- \
  python3 tools/fallback_bench.py --reps 1 ${FB_ARGS} > gpurun_out/trace_fb_${tag}.log 2>&1 \
  || { echo trace_fail; tail -20 gpurun_out/trace_fb_${tag}.log; exit 1; }
tail -1 gpurun_out/trace_fb_${tag}.log | cut -c1-600
f=$(find gpurun_out/trace_fb_$tag -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{r["Name"].split("(")[0][:40]:40s} calls {r["Calls"]:>5s} total {float(r["TotalDurationNs"])/1e6:8.3f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
