"""Kernel-timeline summary of a pipelined bench run from a rocprofv3 --kernel-trace CSV:
GPU busy (union of kernel intervals) vs wall span, time at each concurrency level, and per-kernel
busy share over the last `--window` k_challenge launches (the steady state).
Usage: python tools/timeline.py <kernel_trace.csv> [--batches 20] [--skip-last 1]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--skip-last", type=int, default=1,
                    help="trailing batches to drop (bench.py's instrumented --profile-steps batches run alone)")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
    rows.sort()
    ch = [r for r in rows if "k_challenge" in r[2]]
    if len(ch) < a.batches + a.skip_last + 1:
        raise SystemExit("not enough batches in trace")
    t0 = ch[-a.batches - a.skip_last - 1][0]
    t1 = ch[-a.skip_last - 1][0] if a.skip_last else max(e for s, e, n in rows)
    sel = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
    ev = []
    for s, e, n in sel:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    level = defaultdict(int)
    cur, last = 0, t0
    for t, d in ev:
        level[cur] += t - last
        cur += d
        last = t
    span = t1 - t0
    busy = span - level[0]
    per = defaultdict(int)
    for s, e, n in sel:
        per[n] += e - s
    print(f"span {span/1e6:.3f} ms over {a.batches} batches = {span/1e6/a.batches:.3f} ms/batch; "
          f"GPU busy {busy/span*100:.1f} %")
    for k in sorted(level):
        print(f"  concurrency {k}: {level[k]/span*100:.1f} %")
    # what runs alone: time at concurrency 1 per kernel, and time when only latency-tail kernels
    # (single-workgroup Horner / window combine) or runtime fills occupy the GPU
    tail = ("k_msm_final", "k_msm_window", "k_msm_range_final", "__amd_rocclr")
    ev2 = sorted([(s, 1, n) for s, e, n in sel] + [(e, -1, n) for s, e, n in sel], key=lambda x: (x[0], x[1]))
    running = defaultdict(int)
    solo = defaultdict(int)
    tail_only = 0
    last = t0
    for t, d, n in ev2:
        live = [k for k, c in running.items() if c > 0]
        if len(live) == 1 and sum(running.values()) == 1:
            solo[live[0]] += t - last
        if live and all(any(x in k for x in tail) for k in live):
            tail_only += t - last
        running[n] += d
        last = t
    print(f"  only tail kernels / fills running: {tail_only/span*100:.1f} % of the span")
    for n, v in sorted(solo.items(), key=lambda x: -x[1]):
        print(f"  alone: {n:40s} {v/span*100:.1f} %")
    tot = sum(per.values())
    for n, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {n:40s} {v/1e6/a.batches:.3f} ms/batch (kernel-time {v/tot*100:.1f} %)")


if __name__ == "__main__":
    main()
