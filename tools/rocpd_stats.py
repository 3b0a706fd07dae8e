"""Per-kernel duration summary (like rocprofv3 --stats) from a rocprofv3 rocpd SQLite database.
Usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    for n, k, s, a, lo, hi in rows:
        out.append([n.split("(")[0], k, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in out:
        print(",".join(str(x) for x in r))


if __name__ == "__main__":
    main()
