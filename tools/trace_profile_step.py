"""Per-kernel timeline of profile-leg steps from a rocprofv3 kernel trace.
usage: python tools/trace_profile_step.py <run_kernel_trace.csv> [step index ...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'select_onepass' in r['Kernel_Name']]
print("selects (grid):", [rows[i]['Grid_Size_X'] for i in idx])
which = [int(a) for a in sys.argv[2:]] or [1]
for w in which:
    i0 = idx[w]
    i1 = idx[w + 1] if w + 1 < len(idx) else len(rows)
    t0 = int(rows[i0]['Start_Timestamp'])
    prev = t0
    print("=== step", w)
    for r in rows[i0:i1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if (s - t0) / 1e3 > 5000:
            break
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f}  "
              f"{r['Kernel_Name'][:60]} grid {r['Grid_Size_X']}")
        prev = e
