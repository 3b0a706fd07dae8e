"""Summarise tools/pmc_wait.sh: per kernel (largest-grid dispatches), the share of wave-cycles
spent issuing, parked on s_waitcnt / barriers (SQ_WAIT_ANY) and issue-stalled (SQ_WAIT_INST_ANY),
VALU instructions per wave, and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time).
  python tools/pmc_wait_summary.py gpurun_out/pmc_wait/run_counter_collection.csv"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = defaultdict(lambda: defaultdict(list))
    grid = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("edc::", "")
        g = int(r["Grid_Size"])
        key = (name, g, r.get("Dispatch_Id") or r.get("Correlation_Id"))
        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        grid[name] = max(grid.get(name, 0), g)
    per = defaultdict(lambda: defaultdict(list))
    for (name, g, _), cs in rows.items():
        if g == grid[name]:
            for c, v in cs.items():
                per[name][c].append(sum(v))
    print(f"{'kernel':24s} {'issue%':>7s} {'parked%':>8s} {'stall%':>7s} {'valu/wave':>10s} {'waves':>8s} {'GHz':>6s}")
    for name, cs in sorted(per.items(), key=lambda x: -statistics.median(x[1].get("SQ_WAVE_CYCLES", [0]))):
        m = {c: statistics.median(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0)
        if not wc:
            continue
        print(f"{name:24s} {100*m.get('SQ_ACTIVE_INST_ANY',0)/wc:7.1f} {100*m.get('SQ_WAIT_ANY',0)/wc:8.1f} "
              f"{100*m.get('SQ_WAIT_INST_ANY',0)/wc:7.1f} {m.get('SQ_INSTS_VALU',0)/max(m.get('SQ_WAVES',1),1):10.0f} "
              f"{m.get('SQ_WAVES',0):8.0f} {m.get('GRBM_GUI_ACTIVE',0)/8/max(m.get('GRBM_COUNT',1),1):6.3f}")


if __name__ == "__main__":
    main()
