#!/usr/bin/env python3
"""HBM bytes of one profile step at any size from two rocprofv3 --pmc runs of
tools/run_leg.py profile N STEPS (FETCH_SIZE and WRITE_SIZE passes, csv):
reads = 2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half the bytes of wide
streaming reads, MI355X_MICROARCH.md), writes = WRITE_SIZE, both KiB per
dispatch, summed over the profile kernels.  A run_leg profile run makes
2 warm-up + STEPS hinted calls and then max(20, STEPS // 10) cold-handle
calls (level-0 hint off): dispatch 0 of each kernel is the first (unhinted)
call, 1 .. 1 + STEPS the warm ones, the rest cold.

usage: python tools/pmc_profile.py FETCH_DIR WRITE_DIR N STEPS COMMIT OUT_JSON
Writes OUT_JSON and, for bench.py's roofline "traffic", a copy at
profiles/pmc_profile_<N/1e6>M.json."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def load(d):
    per = defaultdict(list)
    for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
        per[r["Kernel_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]),
                                      int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k in per:
        per[k].sort()
    return per


def main():
    fd, wd, n, steps, commit, out = sys.argv[1:7]
    n, steps = int(n), int(steps)
    pf, pw = load(fd), load(wd)
    rows, warm, cold = [], 0.0, 0.0
    for k, f in pf.items():
        if not ("pbx::prof::" in k or "scan_onepass" in k):
            continue
        w = pw.get(k, [])
        a, b = 1, 1 + steps

        def avg(v, lo, hi):
            s = v[lo:hi]
            return sum(x for _, x, _ in s) / max(len(s), 1)

        rd_w, wr_w = 2048.0 * avg(f, a, b), 1024.0 * avg(w, a, b)
        rd_c, wr_c = 2048.0 * avg(f, b, len(f)), 1024.0 * avg(w, b, len(w))
        dur = sum(d for _, _, d in f[a:b]) / max(len(f[a:b]), 1)
        rows.append({"kernel": k.split("(")[0].replace("void ", ""), "warm_read_bytes": rd_w,
                     "warm_write_bytes": wr_w, "cold_read_bytes": rd_c, "cold_write_bytes": wr_c,
                     "warm_pmc_duration_us": dur / 1e3})
        warm += rd_w + wr_w
        cold += rd_c + wr_c
    rows.sort(key=lambda r: -(r["warm_read_bytes"] + r["warm_write_bytes"]))
    res = {"n": n, "commit": commit,
           "workload": f"{n // 1_000_000}M Plummer, Sphere(10) & dm family, equaln 128, "
                       f"sum m + mean r, CSR (tools/run_leg.py profile {n} {steps})",
           "hbm_bytes_per_step": warm, "hbm_bytes_per_step_cold": cold,
           "note": "per step: sum over the profile kernels of 2 x FETCH_SIZE + WRITE_SIZE of the "
                   "warm (hinted) dispatches; _cold: level-0 hint off",
           "per_kernel": rows, "source": str(Path(out))}
    Path(out).parent.mkdir(parents=True, exist_ok=True)
    Path(out).write_text(json.dumps(res, indent=1))
    (ROOT / "profiles" / f"pmc_profile_{n // 1_000_000}M.json").write_text(json.dumps(res, indent=1))
    print(f"profile {n}: {warm / 1e9:.3f} GB warm, {cold / 1e9:.3f} GB cold per step")


if __name__ == "__main__":
    main()
