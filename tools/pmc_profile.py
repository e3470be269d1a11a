#!/usr/bin/env python3
"""HBM bytes of one profile step at any size from two rocprofv3 --pmc runs of
tools/run_leg.py profile N STEPS (FETCH_SIZE and WRITE_SIZE passes, csv):
reads = 2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half the bytes of wide
streaming reads, MI355X_MICROARCH.md), writes = WRITE_SIZE, both KiB per
dispatch, summed over the profile kernels.  A run_leg profile run makes
2 warm-up + STEPS hinted calls and then max(20, STEPS // 10) first calls
(forget_history); the calls are told apart by their selection kernel (see
main).

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
    wmap = {}
    for k, v in pw.items():
        for did, val, _ in v:
            wmap[did] = val
    # every dispatch of the profile kernels in order, split into calls at each
    # select_tiles launch; a call is "spec" (select_tiles<.., true>: the
    # speculative assignment, the steady state of a repeated call), "cold"
    # (the level-0 hint off: after the 2 warm-up + STEPS calls) or "warm"
    disp = []
    for k, f in pf.items():
        if not ("pbx::prof::" in k or "scan_onepass" in k):
            continue
        for did, val, dur in f:
            disp.append((did, k, 2048.0 * val, 1024.0 * wmap.get(did, 0.0), dur))
    disp.sort()
    calls = []
    for d in disp:
        # a call starts at its selection, or at the sampled level-0 geometry
        # launched just before a first call's selection
        sampled_before = calls and calls[-1] and "sample_hint" in calls[-1][-1][1]
        if "sample_hint" in d[1] or ("select_tiles" in d[1] and not sampled_before) or not calls:
            calls.append([])
        calls[-1].append(d)
    kinds = {"spec": [], "warm": [], "cold": []}
    for i, c in enumerate(calls):
        sel = next((k for _, k, *_ in c if "select_tiles" in k), c[0][1])
        kind = "cold" if i >= 2 + steps else ("spec" if "true>" in sel.split("(")[0] else "warm")
        kinds[kind].append(c)

    def summary(cs):
        if not cs:
            return None
        per = {}
        for c in cs:
            for _, k, rd, wr, dur in c:
                e = per.setdefault(k.split("(")[0].replace("void ", ""), [0.0, 0.0, 0.0, 0])
                e[0] += rd
                e[1] += wr
                e[2] += dur
                e[3] += 1
        rows = [{"kernel": k, "read_bytes": v[0] / len(cs), "write_bytes": v[1] / len(cs),
                 "pmc_duration_us": v[2] / max(v[3], 1) / 1e3} for k, v in per.items()]
        rows.sort(key=lambda r: -(r["read_bytes"] + r["write_bytes"]))
        tot = sum(r["read_bytes"] + r["write_bytes"] for r in rows)
        return {"calls": len(cs), "hbm_bytes_per_step": tot, "per_kernel": rows}

    res = {"n": n, "commit": commit,
           "workload": f"{n // 1_000_000}M Plummer, Sphere(10) & dm family, equaln 128, "
                       f"sum m + mean r, CSR (tools/run_leg.py profile {n} {steps})",
           "note": "per call: sum over the profile kernels of 2 x FETCH_SIZE + WRITE_SIZE; "
                   "spec = the steady state of a repeated call (the selection bins with the "
                   "stored table), warm = hinted calls before that, cold = a handle's first call "
                   "(forget_history: its level-0 geometry sampled, the full assignment)",
           "spec": summary(kinds["spec"]), "warm": summary(kinds["warm"]),
           "cold": summary(kinds["cold"]), "source": str(Path(out))}
    steady = res["spec"] or res["warm"]
    res["hbm_bytes_per_step"] = steady["hbm_bytes_per_step"]
    res["hbm_bytes_per_step_cold"] = res["cold"]["hbm_bytes_per_step"] if res["cold"] else None
    Path(out).parent.mkdir(parents=True, exist_ok=True)
    Path(out).write_text(json.dumps(res, indent=1))
    (ROOT / "profiles" / f"pmc_profile_{n // 1_000_000}M.json").write_text(json.dumps(res, indent=1))
    for k in ("spec", "warm", "cold"):
        if res[k]:
            print(f"profile {n} {k}: {res[k]['calls']} calls, "
                  f"{res[k]['hbm_bytes_per_step'] / 1e9:.3f} GB per step")


if __name__ == "__main__":
    main()
