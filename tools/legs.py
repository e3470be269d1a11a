"""Print the result lines of a tools/gpu_session.sh run (gpurun_out/<step>.out):
the last JSON line of each step, selected keys.  usage: python tools/legs.py step [step...]"""
import json
import sys
from pathlib import Path

for name in sys.argv[1:]:
    f = Path("gpurun_out") / f"{name}.out"
    if not f.exists():
        print(name, "missing")
        continue
    js = [ln for ln in f.read_text().splitlines() if ln.startswith("{")]
    if not js:
        print(name, "no json")
        continue
    d = json.loads(js[-1])
    if "phases_ms" in d:
        print(name, {k: round(v, 3) for k, v in d["phases_ms"].items()})
    elif "cost_balanced" in d:
        c = d["cost_balanced"]
        print(name, "full", round(d["full_walk_ms"], 2), "ranges", [round(x, 2) for x in c["walk_ms"]],
              "max/mean", round(c["max_over_mean"], 3), "bound", round(c["bound_speedup_vs_full"], 2))
    else:
        print(name, js[-1][:300])
