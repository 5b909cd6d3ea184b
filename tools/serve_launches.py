"""Durations of the headline's persistent serve launches in a rocprofv3 --kernel-trace CSV of
`bench.py --gpus 1 --steps 20 --warmup 5` (tools/profile_driver.sh), in bench_serve's launch order,
next to what the bench measured with its own dispatch-attached events in the same run:

    python tools/serve_launches.py <trace dir> <bench_under_rocprof.json> > profiles/rNN_serve_launches.json

bench_serve's launches of the headline kernel, in order: W warm-up, P pre-warm (prewarm_launches), 3 untimed
rehearsals of the timed region, the 9 timed repeats, 30 enqueue samples, 30 launch + synchronize
samples, 3 settling launches, the 9 paired repeats of the region accounting (each with its event
pair: the line's roofline avg_us is their median), 1 more event-timed launch."""
import csv
import glob
import json
import os
import sys


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    tdir, bench = sys.argv[1], sys.argv[2]
    line = json.loads([ln for ln in open(bench) if ln.startswith("{")][-1])
    roof = line["roofline"]
    kname = roof["kernel"].split(" (")[0]
    f = glob.glob(os.path.join(tdir, "*kernel_trace.csv"))[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("void " + kname[:-1])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0, 3) for r in rows]
    wl = roof["warmup_launches"]
    i_timed = wl + roof.get("prewarm_launches", 100) + 3
    i_paired = i_timed + 9 + 30 + 30 + 3
    acc = roof["host_us"].get("accounting", {}).get("serve_paired", {})
    timed, paired = dur[i_timed:i_timed + 9], dur[i_paired:i_paired + 9]
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-dp1",
           "kernel": sorted({r["Kernel_Name"] for r in rows}), "launches": len(dur),
           "timed_repeats_us": timed, "timed_repeats_median_us": med(timed),
           "paired_repeats_us": paired, "paired_repeats_median_us": med(paired),
           "bench_paired_event_us_same_run": acc.get("devices_us"),
           "bench_paired_event_median_us_same_run": acc.get("device_us"),
           "bench_roofline_avg_us_same_run": roof["avg_us"],
           "last_launch_us": dur[-1] if dur else None,
           "all_launches_avg_us": round(sum(dur) / len(dur), 3) if dur else None,
           "median_after_prewarm_us": med(dur[wl + roof.get("prewarm_launches", 100):]),
           "bench_value_same_run": line["value"],
           "durations_us": dur}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
