#!/usr/bin/env python3
"""PMC summaries of a tools/gpu_session.sh run (rocprofv3 --pmc, csv output):
the walk kernel and the 64M profile step, written as the JSON files bench.py
reads for its roofline "traffic" (profiles/pmc_{tree,profile}_latest.json)
plus per-kernel tables under OUT_DIR.

usage: python tools/pmc_r4.py SESSION_DIR OUT_DIR COMMIT

SESSION_DIR holds pmc_walk_{fetch,write,sq}/ and pmc_p64_{fetch,write,sq,sq2}/
(run_counter_collection.csv each).  FETCH_SIZE / WRITE_SIZE are KiB per
dispatch; on gfx950 FETCH_SIZE counts half the bytes of wide streaming
vector reads (MI355X_MICROARCH.md, HBM), so reads = 2 x FETCH_SIZE for the
profile kernels.  The walk reads its node records with SCALAR loads, for
which that factor is uncalibrated: both the raw and the doubled figure are
recorded.  The 64M run is tools/run_leg.py profile 64000000 5: dispatches
1-6 of each kernel are the warm steps (the previous call's level-0 geometry
reused, the bench's case), dispatches 7.. the cold-handle steps (hint off).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def load(path):
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(
            (int(r["Dispatch_Id"]), float(r["Counter_Value"]),
             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k in per:
        for c in per[k]:
            per[k][c].sort()
    return per


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    sess, out, commit = Path(sys.argv[1]).resolve(), Path(sys.argv[2]).resolve(), sys.argv[3]
    out.mkdir(parents=True, exist_ok=True)
    prof = ROOT / "profiles"
    # ---- walk
    wf = load(sess / "pmc_walk_fetch" / "run_counter_collection.csv")
    ww = load(sess / "pmc_walk_write" / "run_counter_collection.csv")
    wq = load(sess / "pmc_walk_sq" / "run_counter_collection.csv")
    wk = [k for k in wf if "walk_kernel<3, 3" in k][0]
    fetch = [v for _, v, _ in wf[wk]["FETCH_SIZE"]]
    write = [v for _, v, _ in ww[wk]["WRITE_SIZE"]]
    raw = 1024.0 * sum(fetch) / len(fetch)
    wr = 1024.0 * sum(write) / len(write)
    sq = {c: sum(v for _, v, _ in vals) / len(vals) for c, vals in wq[wk].items()}
    walk = {
        "kernel": wk, "commit": commit,
        "workload": "4M Plummer (seed 1003), theta 0.5, leaf 8, order 3, force+potential, fast "
                    "mode (tools/run_leg.py tree 4000000 2; 3 walks)",
        "hbm_bytes_per_launch": 2 * raw + wr,
        "read_bytes_per_launch": 2 * raw, "read_bytes_raw_fetch_size": raw,
        "write_bytes_per_launch": wr,
        "sq_per_walk": sq,
        "note": "2 x FETCH_SIZE + WRITE_SIZE; the walk reads node records and leaf particles "
                "with scalar (s_load) requests, for which the gfx950 x2 correction is "
                "uncalibrated: the raw FETCH_SIZE bytes are the lower figure. Memory-side "
                "requests incl. Infinity-Cache hits.",
        "source": str((out / "walk_pmc.json").relative_to(ROOT)),
    }
    (out / "walk_pmc.json").write_text(json.dumps(walk, indent=1))
    (prof / "pmc_tree_latest.json").write_text(json.dumps(walk, indent=1))
    # ---- 64M profile step
    pf = load(sess / "pmc_p64_fetch" / "run_counter_collection.csv")
    pw = load(sess / "pmc_p64_write" / "run_counter_collection.csv")
    sq1 = load(sess / "pmc_p64_sq" / "run_counter_collection.csv")
    sq2 = load(sess / "pmc_p64_sq2" / "run_counter_collection.csv")
    rows, warm_total, cold_total = [], 0.0, 0.0
    for k in pf:
        if not ("pbx::prof::" in k or "scan_onepass" in k):
            continue
        f = pf[k]["FETCH_SIZE"]
        w = pw.get(k, {}).get("WRITE_SIZE", [])
        if len(f) < 7:
            continue

        def avg(vals, lo, hi):
            s = vals[lo:hi]
            return sum(v for _, v, _ in s) / max(len(s), 1)

        rd_w, rd_c = 2048.0 * avg(f, 1, 7), 2048.0 * avg(f, 7, len(f))
        wr_w, wr_c = 1024.0 * avg(w, 1, 7), 1024.0 * avg(w, 7, len(w))
        dur = sum(d for _, _, d in f[1:7]) / 6.0
        sqv = {}
        for src in (sq1, sq2):
            for c, vals in src.get(k, {}).items():
                sqv[c] = sum(v for _, v, _ in vals[1:7]) / 6.0
        rows.append({"kernel": short(k), "warm_read_bytes": rd_w, "warm_write_bytes": wr_w,
                     "cold_read_bytes": rd_c, "cold_write_bytes": wr_c,
                     "warm_pmc_duration_us": dur / 1e3, "sq_warm": sqv})
        warm_total += rd_w + wr_w
        cold_total += rd_c + wr_c
    rows.sort(key=lambda r: -(r["warm_read_bytes"] + r["warm_write_bytes"]))
    profj = {
        "n": 64_000_000, "commit": commit,
        "workload": "64M Plummer (seed 1002 + 0), Sphere(10) & dm family, equaln 128, Σm + mean r, "
                    "CSR (tools/run_leg.py profile 64000000 5)",
        "hbm_bytes_per_step": warm_total,
        "hbm_bytes_per_step_cold": cold_total,
        "note": "per step: sum over the profile kernels of 2 x FETCH_SIZE + WRITE_SIZE, warm "
                "dispatches (the bench's repeated-snapshot case); _cold: level-0 hint off "
                "(fused_hist0 re-reads x)",
        "per_kernel": rows,
        "source": str((out / "profile64_pmc.json").relative_to(ROOT)),
    }
    (out / "profile64_pmc.json").write_text(json.dumps(profj, indent=1))
    (prof / "pmc_profile_latest.json").write_text(json.dumps(profj, indent=1))
    print(f"walk: {2 * raw / 1e9:.2f} GB read (x2), {raw / 1e9:.2f} raw, {wr / 1e9:.3f} GB written")
    print(f"profile 64M: {warm_total / 1e9:.3f} GB warm, {cold_total / 1e9:.3f} GB cold per step")


if __name__ == "__main__":
    main()
