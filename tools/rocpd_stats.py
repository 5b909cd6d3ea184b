"""Per-kernel duration summary from a rocprofv3 rocpd database (run_results.db), in the
column layout of rocprofv3 --stats (kernel_stats.csv).  Dev tool: used when a profile was
written in the default rocpd format instead of --output-format csv.

    python tools/rocpd_stats.py gpurun_out/prof18/run_results.db > profiles/xxx_kernel_stats.csv
    python tools/rocpd_stats.py DB --phase 'k_fwd<1, 8, 8, 2, true, true, 1>' 200
        (also prints the stats of the LAST 200 dispatches of that symbol: the bench's
         roofline launches, which run after the timed region)
"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    rows = sqlite3.connect(db).execute("select name, duration from kernels order by start").fetchall()
    agg = {}
    for name, d in rows:
        agg.setdefault(name, []).append(d)
    total = sum(sum(v) for v in agg.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    if "--phase" in sys.argv:
        i = sys.argv.index("--phase")
        sym, n = sys.argv[i + 1], int(sys.argv[i + 2])
        v = [d for name, d in rows if sym in name][-n:]
        print("# last %d dispatches of %s: avg %.1f ns min %d max %d" % (len(v), sym, sum(v) / len(v), min(v), max(v)),
              file=sys.stderr)


if __name__ == "__main__":
    main()


def roofline_phase_csv(trace_csv, symbol, graph_streams_min=2):
    """From a --kernel-trace CSV of bench.py's default run: durations (ns) of the launches of
    `symbol` on the model's own stream that follow the last graph replay (the roofline phase:
    20 warm-up + 200 back-to-back + 200 event-timed launches), in order."""
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if symbol in r["Kernel_Name"]]
    from collections import Counter
    cnt = Counter(r["Stream_Id"] for r in ks)
    own = [s for s, _ in cnt.most_common() if s == "0"] or [cnt.most_common()[-1][0]]
    graph_streams = {s for s in cnt if s not in own}
    last_graph = max(int(r["Start_Timestamp"]) for r in ks if r["Stream_Id"] in graph_streams)
    return [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks
            if r["Stream_Id"] in own and int(r["Start_Timestamp"]) > last_graph]
