"""Per-kernel timeline of the last profile step (selection kernel on the
largest grid) in a rocprofv3 kernel trace.
usage: python tools/trace_last_step.py <run_kernel_trace.csv> [kernel-substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
key = sys.argv[2] if len(sys.argv) > 2 else 'select_onepass'
idx = [i for i, r in enumerate(rows) if key in r['Kernel_Name']]
gmax = max(int(rows[i]['Grid_Size_X']) for i in idx)
idx = [i for i in idx if int(rows[i]['Grid_Size_X']) == gmax]
i0, i1 = idx[-2], idx[-1]
t0 = int(rows[i0]['Start_Timestamp'])
prev = t0
for r in rows[i0:i1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f}  "
          f"{r['Kernel_Name'][:64]} grid {r['Grid_Size_X']}")
    prev = e
