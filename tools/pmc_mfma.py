"""MFMA utilisation per kernel from rocprofv3 PMC counters.

    python tools/pmc_mfma.py <mfma_dir> <grbm_dir> [kernel-substring ...]

util = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE / 8):
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every SIMD's SQ
(MI355X_MICROARCH.md, 'SQ PMC units'); GRBM_GUI_ACTIVE is summed over the 8 XCDs, so /8 is
the dispatch's GPU-busy cycles.  Each counter comes from its own --pmc pass; values are
averaged over the launches of each kernel.  Short dispatches (< ~0.3 ms) read the clock
high (guide, 'DVFS give-back'), so util is a lower bound there.
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys

SIMDS = 4 * 256


def load(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
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
    md, gd = sys.argv[1], sys.argv[2]
    subs = sys.argv[3:]
    mf, gr = load(md, "SQ_VALU_MFMA_BUSY_CYCLES"), load(gd, "GRBM_GUI_ACTIVE")
    out = {}
    for k in sorted(set(mf) & set(gr)):
        if subs and not any(s in k for s in subs):
            continue
        m = sum(mf[k]) / len(mf[k])
        g = sum(gr[k]) / len(gr[k])
        if g <= 0:
            continue
        out[k] = {"launches": len(mf[k]), "mfma_busy_cycles": round(m, 1), "gpu_busy_cycles": round(g / 8, 1),
                  "mfma_util": round(m / (SIMDS * g / 8), 4)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
