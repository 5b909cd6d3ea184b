"""Per-launch averages of the cfg5 unit counters (tools/profile_driver.sh step 7) for one kernel.

    python tools/pmc_units.py <prof_dir> <kernel-substring>

Reads every <prof_dir>/stress_*/ pass except the MFMA/GRBM ones, sums each counter over its
instances per dispatch, averages over the kernel's dispatches.  Derived (MI355X_MICROARCH.md:
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; SQ_LDS_BANK_CONFLICT and
SQ_LDS_IDX_ACTIVE are LDS-array cycles; TA_TA_BUSY is summed over the 256 CUs' TAs, SQ_BUSY_CYCLES
over the 32 shader engines): the share of wave cycles parked in waits, stalled on LDS issue, the
LDS conflict cycles per LDS-array cycle, and per-CU TA busy cycles against the SE busy cycles.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "stress_*", "**", "*counter_collection*.csv"), recursive=True):
        if "stress_mfma" in f or "stress_grbm" in f:
            continue
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
    out = {c: round(sum(v.values()) / len(v), 1) for c, v in acc.items() if v}
    g = lambda k: out.get(k)   # noqa: E731
    der = {}
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY"):
            if g(k) is not None:
                der[k + "/SQ_WAVE_CYCLES"] = round(g(k) / g("SQ_WAVE_CYCLES"), 4)
    if g("SQ_LDS_IDX_ACTIVE"):
        der["SQ_LDS_BANK_CONFLICT/SQ_LDS_IDX_ACTIVE"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 4)
    if g("TA_TA_BUSY_sum") and g("SQ_BUSY_CYCLES"):
        der["TA busy per CU / SE busy cycles"] = round((g("TA_TA_BUSY_sum") / 256) / (g("SQ_BUSY_CYCLES") / 32), 4)
    json.dump({"kernel_substring": sub, "per_launch": out, "derived": der}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
