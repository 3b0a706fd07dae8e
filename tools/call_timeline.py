"""Per-call kernel chain of a synchronous small-batch run, from a rocprofv3 --kernel-trace CSV
(tools/smallbatch_bench.py): the kernels of one edc_batch_verify call are the launches between
two k_init_batch launches. Prints, averaged over the last --calls calls, each kernel's duration
and the idle gap before it, and the call's span (first start -> last end).
Usage: python tools/call_timeline.py <kernel_trace.csv> [--calls 30] [--first k_init_batch]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--first", default="k_init_batch")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0].split("::")[-1]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.first in r[2]]
    calls = [rows[s:e] for s, e in zip(starts, starts[1:] + [len(rows)])]
    calls = calls[-a.calls - 1:-1] if len(calls) > a.calls else calls[:-1]
    if not calls:
        raise SystemExit("no complete calls in trace")
    dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
    order = []
    spans, busy = [], []
    for c in calls:
        prev_end = c[0][0]
        seen = defaultdict(int)
        for s, e, n in c:
            seen[n] += 1
            key = n if seen[n] == 1 else f"{n}#{seen[n]}"
            if key not in dur:
                order.append(key)
            dur[key] += e - s
            gap[key] += max(0, s - prev_end)
            cnt[key] += 1
            prev_end = max(prev_end, e)
        spans.append(max(e for s, e, n in c) - c[0][0])
        busy.append(sum(e - s for s, e, n in c))
    nc = len(calls)
    print(f"{nc} calls: span {sum(spans)/nc/1e3:.1f} us, kernel time {sum(busy)/nc/1e3:.1f} us, "
          f"{len(calls[0])} kernels per call")
    for k in order:
        print(f"  {k:28s} {dur[k]/cnt[k]/1e3:8.1f} us   gap before {gap[k]/cnt[k]/1e3:6.1f} us   ({cnt[k]} launches)")


if __name__ == "__main__":
    main()
