#!/usr/bin/env python3
"""HBM bytes per call of one kind of radial-profile call, from two
rocprofv3 --pmc runs of tools/profile_calls.py N MODE CALLS (a FETCH_SIZE
pass and a WRITE_SIZE pass, csv): per call = the sum over the profile
kernels' dispatches of 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE
counts half the bytes of wide streaming reads, MI355X_MICROARCH.md; both in
KiB per dispatch), divided by the number of calls (select_tiles dispatches).
The warm-up calls profile_calls makes before its timed ones are counted
too: every call of a mode is the same kind of call.

usage: python tools/pmc_calls.py FETCH_DIR WRITE_DIR N MODE COMMIT [OUT_JSON]
With MODE "changing" the figure is also written into
profiles/pmc_profile_<N/1e6>M.json as hbm_bytes_per_step_changing (what
bench.py's profile roofline "traffic" reads for changing inputs)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def load(d):
    out = {}
    for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
    return out


def main():
    fd, wd, n, mode, commit = sys.argv[1:6]
    out_json = sys.argv[6] if len(sys.argv) > 6 else None
    n = int(n)
    pf, pw = load(fd), load(wd)
    per = defaultdict(lambda: [0.0, 0.0, 0])
    calls = 0
    for did, (k, v) in pf.items():
        if not ("pbx::prof::" in k or "scan_onepass" in k):
            continue
        name = k.split("(")[0].replace("void ", "").replace("pbx::prof::", "")
        if name.startswith("select_tiles"):
            calls += 1
        e = per[name]
        e[0] += 2048.0 * v
        e[2] += 1
    for did, (k, v) in pw.items():
        if not ("pbx::prof::" in k or "scan_onepass" in k):
            continue
        name = k.split("(")[0].replace("void ", "").replace("pbx::prof::", "")
        per[name][1] += 1024.0 * v
    calls = max(calls, 1)
    rows = [{"kernel": k, "read_bytes": v[0] / calls, "write_bytes": v[1] / calls,
             "dispatches_per_call": v[2] / calls} for k, v in per.items()]
    rows.sort(key=lambda r: -(r["read_bytes"] + r["write_bytes"]))
    tot = sum(r["read_bytes"] + r["write_bytes"] for r in rows)
    res = {"n": n, "mode": mode, "commit": commit, "calls": calls, "hbm_bytes_per_call": tot,
           "per_kernel": rows,
           "workload": f"tools/profile_calls.py {n} {mode}: {n // 1_000_000}M Plummer, Sphere(10) & "
                       "dm family, equaln 128, sum m + mean r, CSR",
           "note": "per call: sum over the profile kernels of 2 x FETCH_SIZE + WRITE_SIZE"}
    print(json.dumps({"n": n, "mode": mode, "calls": calls, "hbm_gb_per_call": tot / 1e9}))
    if out_json:
        Path(out_json).parent.mkdir(parents=True, exist_ok=True)
        Path(out_json).write_text(json.dumps(res, indent=1))
    if mode == "changing":
        f = ROOT / "profiles" / f"pmc_profile_{n // 1_000_000}M.json"
        d = json.loads(f.read_text()) if f.exists() else {"n": n}
        d["hbm_bytes_per_step_changing"] = tot
        d["changing"] = res
        f.write_text(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
