"""Per-batch PMC table of every kernel of the batch pipeline from one rocprofv3 --pmc run of
bench.py: each counter summed over all dispatches of a kernel, divided by the number of batches
(k_challenge dispatches). Shows where a batch's VALU work goes at a given batch size and the
issue-bound time it implies (INT64 ops at 4.46 cycles, other VALU at 2.5, 1024 SIMDs).
Usage: python tools/pmc_batch_table.py <run_counter_collection.csv> [--clock-ghz 2.1]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--clock-ghz", type=float, default=2.1)
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("edc::", "").replace("void ", "")
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    nb = max(1, len(disp.get("k_challenge", ())))
    cols = sorted({c for k in tot.values() for c in k})
    print(f"batches: {nb}")
    print(f"{'kernel':32s} {'disp/b':>6s} " + " ".join(f"{c:>16s}" for c in cols))
    rows = sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0))
    sums = defaultdict(float)
    for name, cs in rows:
        print(f"{name:32s} {len(disp[name]) / nb:6.2f} " + " ".join(f"{cs.get(c, 0) / nb:16.0f}" for c in cols))
        for c in cols:
            sums[c] += cs.get(c, 0) / nb
    print(f"{'TOTAL per batch':32s} {'':6s} " + " ".join(f"{sums[c]:16.0f}" for c in cols))
    if "SQ_INSTS_VALU" in sums:
        v = sums["SQ_INSTS_VALU"]
        i64 = sums.get("SQ_INSTS_VALU_INT64", 0.0)
        cyc = (i64 * 4.46 + (v - i64) * 2.5) / 1024 if i64 else v * 3.5 / 1024
        print(f"VALU issue-bound time per batch: {cyc / (a.clock_ghz * 1e9) * 1e3:.4f} ms at {a.clock_ghz} GHz "
              f"({'INT64 4.46 / other 2.5 cycles' if i64 else 'flat 3.5 cycles'} per wave-instruction per SIMD)")


if __name__ == "__main__":
    main()
