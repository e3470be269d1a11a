"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite
database, for runs whose output format was the default database.

usage: python tools/rocpd_stats.py RESULTS.db [OUT.csv]
Columns: Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs,StdDevNs
"""
import csv
import math
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    by = {}
    for name, d in rows:
        by.setdefault(name, []).append(float(d))
    total = sum(sum(v) for v in by.values()) or 1.0
    out = []
    for name, v in by.items():
        n = len(v)
        avg = sum(v) / n
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
        out.append((name, n, sum(v), avg, 100.0 * sum(v) / total, min(v), max(v), sd))
    out.sort(key=lambda r: -r[2])
    return out


def main():
    rows = stats(sys.argv[1])
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDevNs"])
    for r in rows:
        w.writerow([r[0], r[1], int(r[2]), f"{r[3]:.1f}", f"{r[4]:.4f}", int(r[5]), int(r[6]),
                    f"{r[7]:.1f}"])


if __name__ == "__main__":
    main()
