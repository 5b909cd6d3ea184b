"""Dev tool: the cfg3 training line (bench.py --mode train) under P3D_LIB, one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--mode", "train", "--steps", "400", "--warmup", "64",
       "--no-cpu"] + sys.argv[1:]
r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
ro = d["roofline"]
print(json.dumps({"value": d["value"], "ms_per_step": d["ms_per_step"], "wgrad_us": ro.get("avg_us"),
                  "frac": ro.get("frac"), "kernels_us": ro.get("event_pair_avg_us")}))
sys.exit(r.returncode)
