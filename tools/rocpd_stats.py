"""Kernel statistics (rocprofv3 --stats layout: Name,Calls,TotalDurationNs,AverageNs,Percentage,
MinNs,MaxNs) from a rocprofv3 kernel-trace database (<dir>/<name>_results.db, the default output
format of this image's rocprofv3), for profiles/.

  python tools/rocpd_stats.py gpurun_out/<tag>_prof1/k_results.db > profiles/.../kernel_stats.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print("Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs")
    for n, calls, tot, avg, mn, mx in rows:
        short = n.split("(")[0].replace("void ", "")
        print(f"{short},{calls},{tot},{avg:.1f},{100.0 * tot / total:.2f},{mn},{mx}")


if __name__ == "__main__":
    main(sys.argv[1])
