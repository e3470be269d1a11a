"""Print one step's kernel timeline from a rocprofv3 kernel trace CSV.
usage: trace_step.py TRACE.csv FIRST_KERNEL_SUBSTRING [count]"""
import csv
import sys

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(tr) if sys.argv[2] in r['Kernel_Name']]
s = idx[-1]
t0 = prev = int(tr[s]['Start_Timestamp'])
for r in tr[s:s + int(sys.argv[3]) if len(sys.argv) > 3 else s + 40]:
    st, en = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(st - t0) / 1e3:9.1f} +gap {(st - prev) / 1e3:7.1f}  dur {(en - st) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
    prev = en
