"""Dev tool: the serve-only bench line under the library P3D_LIB names (tools/lib_ab.py runs it
alternately for two builds): bench.py --steps 20 with every sub-measurement but the serve launch
and the lone batch-64 request switched off."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20", "--warmup", "5", "--no-streams",
       "--no-eval", "--no-data", "--no-api", "--no-stress", "--train-steps", "0", "--no-cpu", "--no-dp1"] + sys.argv[1:]
r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
import json  # noqa: E402
line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
d = json.loads(line)
ro = d["roofline"]
print(json.dumps({"value": d["value"], "ms_per_step": d["ms_per_step"], "kernel_us": ro["avg_us"], "frac": ro["frac"],
                  "repeats_us": ro["host_us"]["timed_region_repeats_us"],
                  "b64_device_us": d.get("latency_b64", {}).get("serve", {}).get("device_us")}))
sys.exit(r.returncode)
