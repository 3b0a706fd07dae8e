"""Copies and kernels of the LAST synchronous host-buffer call in a rocprofv3 trace
(tools/host_trace.py) on one time axis: start / end in us from the call's first H2D copy.

  python tools/host_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>
"""
import csv
import glob
import os
import sys


def rows(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Direction") or r.get("Operation") or kind
            nbytes = r.get("Size") or r.get("Bytes") or ""
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name.split("(")[0], nbytes))
    return out


def main(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = rows(kt[0], "kernel") + (rows(mt[0], "copy") if mt else [])
    ev.sort()
    # the last call: from the last k_init_batch back to the copies that precede it within 5 ms
    inits = [e for e in ev if "k_init_batch" in e[3]]
    t_init = inits[-1][0]
    start = min(e[0] for e in ev if e[2] == "copy" and t_init - 5_000_000 < e[0] <= t_init + 1) \
        if any(e[2] == "copy" for e in ev) else t_init
    last = [e for e in ev if e[0] >= start]
    end = max(e[1] for e in last)
    print(f"call span {(end - start) / 1e3:.1f} us, {len(last)} events")
    for s, e, kind, name, nb in last:
        print(f"{(s - start) / 1e3:9.1f} {(e - start) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {kind:6s} {name} {nb}")


if __name__ == "__main__":
    main(sys.argv[1])
