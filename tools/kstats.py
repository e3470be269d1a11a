"""Print rocprofv3 kernel_stats.csv files side by side (average µs per call).

usage: python tools/kstats.py A/run_kernel_stats.csv [B/run_kernel_stats.csv ...]

Kernel names are shortened to their function name (template arguments kept);
a column per file, plus the per-file sum of averages weighted by calls per
step (calls / the most frequent kernel's calls).
"""
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)\(", name)
    s = m.group(1) if m else name
    return s.replace("pbx::prof::", "").replace("pbx::prim::(anonymous namespace)::", "")[:48]


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    return out


def main(paths):
    tabs = [load(p) for p in paths]
    names = []
    for t in tabs:
        for k in sorted(t, key=lambda k: -t[k][1]):
            if k not in names:
                names.append(k)
    print(f"{'kernel':48s}" + "".join(f" {p.split('/')[-2][:10]:>10s}" for p in paths))
    for k in names:
        print(f"{k:48s}" + "".join(f" {t[k][1]:10.2f}" if k in t else f" {'-':>10s}" for t in tabs))
    sums = []
    for t in tabs:
        top = max(c for c, _ in t.values())
        sums.append(sum(a * c / top for c, a in t.values() if c >= top // 2))
    print(f"{'sum per step (kernels with >= top/2 calls)':48s}" + "".join(f" {s:10.2f}" for s in sums))


if __name__ == "__main__":
    main(sys.argv[1:])
