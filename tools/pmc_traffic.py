"""Average rocprofv3 PMC counters per kernel (HBM-side traffic per launch).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [kernel-substring] [--config key=value ...]

--config entries are stored under "__config__": bench.py takes a committed figure as the
`roofline.traffic` of its run only when every one of them equals its own configuration
(e.g. steps_per_launch=20 for the persistent serve kernel).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) counts exactly half
the bytes of a wide coalesced read -> doubled; WRITE_SIZE (KB) is exact for 16-B/lane
stores.  Each counter comes from its own --pmc pass (they do not fit one TCC pass).
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    acc = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):   # rocpd format
        q = ("select kernel_name, dispatch_id, sum(value) from counters_collection "
             "where counter_name = ? group by dispatch_id order by dispatch_id")
        for name, _, v in sqlite3.connect(db).execute(q, (counter,)):
            acc[name].append(float(v))
    return acc


def main():
    argv, config = [], {}
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--config":
            k, v = next(it).split("=", 1)
            config[k] = int(v) if v.lstrip("-").isdigit() else v
        else:
            argv.append(a)
    fd, wd = argv[0], argv[1]
    sub = argv[2] if len(argv) > 2 else ""
    fe, wr = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    out = {"__config__": config} if config else {}
    for k in sorted(set(fe) | set(wr)):
        if sub and sub not in k:
            continue
        f = fe.get(k, [])
        w = wr.get(k, [])
        fkb = sum(f) / len(f) if f else 0.0
        wkb = sum(w) / len(w) if w else 0.0
        out[k] = {"launches": max(len(f), len(w)), "fetch_kb_raw": round(fkb, 2), "write_kb": round(wkb, 2),
                  "hbm_bytes_per_launch": int((2 * fkb + wkb) * 1024)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
