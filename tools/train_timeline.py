"""Timeline of the cfg3 training step from a rocprofv3 --kernel-trace CSV of
`bench.py --gpus 1 --mode train` (tools/profile_driver.sh, step 3): the dispatches of graph-replayed
steps, one step = the launches from one k_fwd input layer (the step's first launch) to the next.
Prints per launch of the median step: kernel, start offset from the step's start, duration, and the
gap before it (the dependent boundary), plus per-step totals.

    python tools/train_timeline.py <train_trace dir> > profiles/rNN_train_timeline.json
"""
import csv
import glob
import json
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if not r["Kernel_Name"].startswith("__amd")]
    first = "k_fwd<1, 2, 1, 2, false, true, 0>"   # the BN-train input layer: every step's first launch
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        ent, prev_end = [], t0
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ent.append({"kernel": r["Kernel_Name"].split("(")[0], "start_us": round((s - t0) / 1e3, 2),
                        "dur_us": round((e - s) / 1e3, 2), "gap_us": round((s - prev_end) / 1e3, 2)})
            prev_end = e
        steps.append({"step_us": round((int(rows[b]["Start_Timestamp"]) - t0) / 1e3, 2), "launches": ent})
    steps = [s for s in steps if len(s["launches"]) == len(steps[-1]["launches"])]
    steps.sort(key=lambda s: s["step_us"])
    med = steps[len(steps) // 2]
    out = {"source": f, "steps": len(steps), "median_step_us": med["step_us"],
           "launches_per_step": len(med["launches"]),
           "kernel_time_us": round(sum(x["dur_us"] for x in med["launches"]), 2),
           "gap_time_us": round(sum(x["gap_us"] for x in med["launches"][1:]), 2),
           "median_step": med["launches"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
