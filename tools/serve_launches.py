"""Durations of every persistent serve launch in a rocprofv3 --kernel-trace CSV of
`bench.py --gpus 1 --steps 20 --warmup 5` (tools/profile_driver.sh), with bench_serve's launch
order, next to what the bench measured in the same run.

    python tools/serve_launches.py <trace dir> <bench_under_rocprof.json> > profiles/rNN_serve_launches.json
"""
import csv
import glob
import json
import os
import sys


def main():
    tdir, bench = sys.argv[1], sys.argv[2]
    f = glob.glob(os.path.join(tdir, "*kernel_trace.csv"))[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_serve" in r["Kernel_Name"] and "prep" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = sorted({r["Kernel_Name"] for r in rows})
    dur = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0, 3) for r in rows]
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    wl = line["roofline"]["warmup_launches"]
    timed = wl + 100 + 3                       # bench_serve: warm-up, pre-warm, 3 rehearsals, then the timed launch
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5",
           "kernel": names, "launches": len(dur),
           "order": "bench_serve: %d warm-up + 100 pre-warm + 3 untimed rehearsal launches, #%d the timed one, "
                    "then 8 repeats of the timed region, 30 + 30 host-overhead samples, the last the "
                    "event-timed (roofline) launch" % (wl, timed + 1),
           "timed_launch_us": dur[timed] if timed < len(dur) else None,
           "event_timed_launch_us": dur[-1],
           "median_after_prewarm_us": sorted(dur[wl + 100:])[len(dur[wl + 100:]) // 2],
           "bench_value_same_run": line["value"], "bench_event_avg_us_same_run": line["roofline"]["avg_us"],
           "durations_us": dur}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
