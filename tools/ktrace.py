"""Per-kernel average durations from a rocprofv3 kernel_trace.csv, split into
call windows (e.g. the warm-handle and cold-handle halves of a bench leg).

usage: python tools/ktrace.py TRACE.csv [TRACE2.csv ...] [--windows a:b,c:d]
Windows index the calls of each kernel (python slice bounds).
"""
import csv
import sys

from kstats import short


def main(argv):
    wins = [(1, 21), (22, 42)]
    paths = []
    for a in argv:
        if a.startswith("--windows="):
            wins = [tuple(int(v) for v in w.split(":")) for w in a.split("=", 1)[1].split(",")]
        else:
            paths.append(a)
    cols = []
    names = []
    for p in paths:
        per = {}
        for r in csv.DictReader(open(p)):
            per.setdefault(short(r["Kernel_Name"]), []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k in sorted(per, key=lambda k: -sum(per[k])):
            if k not in names:
                names.append(k)
        for a, b in wins:
            cols.append((f"{p.split('/')[-2][:7]}[{a}:{b}]", {k: v[a:b] for k, v in per.items()}))
    print(f"{'kernel':44s}" + "".join(f" {c[0]:>13s}" for c in cols))
    tot = [0.0] * len(cols)
    for k in names:
        line = f"{k:44s}"
        for i, (_, d) in enumerate(cols):
            v = d.get(k) or []
            if v:
                m = sum(v) / len(v)
                tot[i] += m
                line += f" {m:13.2f}"
            else:
                line += f" {'-':>13s}"
        print(line)
    print(f"{'sum':44s}" + "".join(f" {t:13.2f}" for t in tot))


if __name__ == "__main__":
    main(sys.argv[1:])
