"""Dev tool: the cfg5 stress line (bench.py --mode stress) under P3D_LIB, one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--mode", "stress", "--steps", "32", "--warmup", "8",
       "--no-cpu"] + sys.argv[1:]
r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
print(json.dumps({"value": d["value"], "ms_per_step": d["ms_per_step"], "kernel": d["roofline"].get("kernel"),
                  "kernel_us": d["roofline"].get("avg_us"), "frac": d["roofline"].get("frac")}))
sys.exit(r.returncode)
