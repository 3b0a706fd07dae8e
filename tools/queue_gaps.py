"""Per-queue view of a pipelined bench trace (rocprofv3 --kernel-trace CSV): each in-flight slot is
one stream with its own hardware queue, so a queue's idle gap between two of its kernels is time in
which that batch had work enqueued (the host enqueues a whole batch at once) but nothing running.
Prints the distribution of running queues, the waves in flight (grid / 64) over time, and the gap
before each kernel name, over the steady state (the same window tools/timeline.py uses).
Usage: python tools/queue_gaps.py <kernel_trace.csv> [--batches 20] [--skip-last 1]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--skip-last", type=int, default=1)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = (r.get("Kernel_Name") or r.get("KernelName") or "").split("(")[0].replace("edc::", "").replace("void ", "")
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            gx = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q, gx))
    rows.sort()
    ch = [r for r in rows if r[2] == "k_challenge"]
    t0 = ch[-a.batches - a.skip_last - 1][0]
    t1 = ch[-a.skip_last - 1][0]
    span = t1 - t0
    sel = [r for r in rows if r[1] > t0 and r[0] < t1]
    # running queues and waves over time
    ev = []
    for s, e, n, q, g in sel:
        ev.append((max(s, t0), 1, q, (g + 63) // 64))
        ev.append((min(e, t1), -1, q, (g + 63) // 64))
    ev.sort()
    run_q = defaultdict(int)
    waves = 0
    lvl = defaultdict(int)
    wbin = defaultdict(int)
    last = t0
    for t, d, q, w in ev:
        nq = sum(1 for v in run_q.values() if v > 0)
        lvl[nq] += t - last
        wb = 0 if waves == 0 else (1 if waves < 1024 else (2 if waves < 4096 else (3 if waves < 16384 else 4)))
        wbin[wb] += t - last
        last = t
        run_q[q] += d
        waves += d * w
    print(f"span {span / 1e6:.3f} ms, {len({r[3] for r in sel})} queues")
    for k in sorted(lvl):
        print(f"  queues running {k}: {lvl[k] / span * 100:5.1f} %")
    names = ["0", "<1024 (<1 wave/SIMD)", "1024-4095", "4096-16383", ">=16384"]
    for k in sorted(wbin):
        print(f"  waves in flight {names[k]:22s}: {wbin[k] / span * 100:5.1f} %")
    # gaps inside each queue
    byq = defaultdict(list)
    for r in rows:
        byq[r[3]].append(r)
    gap = defaultdict(float)
    cnt = defaultdict(int)
    for q, ks in byq.items():
        ks.sort()
        for i in range(1, len(ks)):
            s, e, n = ks[i][0], ks[i][1], ks[i][2]
            if s < t0 or s > t1:
                continue
            g = s - ks[i - 1][1]
            if 0 < g < 200000:               # < 0.2 ms: the same batch's chain (larger = waiting for the host)
                gap[n] += g
                cnt[n] += 1
    print("queue-idle gap before each kernel (same batch chain), ms per batch / mean us:")
    for n in sorted(gap, key=lambda k: -gap[k]):
        print(f"  {n:32s} {gap[n] / 1e6 / a.batches:7.4f} {gap[n] / 1e3 / cnt[n]:8.1f}")


if __name__ == "__main__":
    main()
