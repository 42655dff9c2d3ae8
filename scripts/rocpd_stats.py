"""Kernel statistics (rocprofv3 --stats form) from a rocprofv3 rocpd
database (ROCm 7.2's default output, `-d DIR -o run` -> run_results.db):
Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, one CSV
row per kernel, sorted by total time.

    python scripts/rocpd_stats.py DB [OUT.csv]
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), min(duration), max(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    table = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    for name, n, tot, mn, mx in rows:
        table.append([name, n, tot, round(tot / n, 1), round(100.0 * tot / total, 3), mn, mx])
    f = open(out, "w", newline="") if out else sys.stdout
    csv.writer(f).writerows(table)


if __name__ == "__main__":
    main()
