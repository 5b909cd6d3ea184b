"""Dev tool: timeline of one k_serve6 launch from a -DP3D_TRACE build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -DP3D_TRACE \\
        -o 3d-pose-baseline_amd/libp3d_trace.so 3d-pose-baseline_amd/csrc/p3d.hip
    P3D_LIB=$PWD/3d-pose-baseline_amd/libp3d_trace.so python tools/trace_serve6.py [steps] [reps]

For every XCD group of the last launch (its first step): rank-0 member and the first member
holding the most column tiles; times in us from the earliest workgroup start (wall_clock64,
100 MHz).  Columns per hidden phase: contraction, K-combine, epilogue, hand-off wait, then inside the
epilogue: the K-slice sums (LDS), the epilogue math + stores.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _p3d  # noqa: E402
import linear_model  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=3, max_batch=64)
    x = torch.randn((64 * nb, 32), device="cuda")
    for _ in range(reps):
        m.serve_device(x)
    torch.cuda.synchronize()
    m.serve_check()
    lib = _p3d.lib()
    lib.p3d_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.p3d_debug_trace(buf.ctypes.data, buf.size) == 0
    t = buf[:64 * 2 * 128].astype(np.int64).reshape(64, 2, 128)
    NH = 4
    live = [(g, r) for g in range(64) for r in range(2) if t[g, r, 0] and t[g, r, 8 * (NH + 1)]]
    t0 = min(t[g, r, 0] for g, r in live)
    us = lambda v: round((v - t0) / 100.0, 2)   # noqa: E731
    out = []
    pair = os.environ.get("P3D_SERVE6_PAIR", "0") == "1"
    for g, r in live:
        row = t[g, r]
        if row[8 * (NH + 1)] < row[0]:          # stale (a group idle in the last launch)
            continue
        if pair:
            # the pair form's blocks (unit s & 1, phase s // 2 + 1) at 8 + 4 s: contraction start,
            # contraction end, K-combine barrier passed, epilogue stores issued
            blk = [[round((row[8 + 4 * s + 1] - row[8 + 4 * s]) / 100, 2),
                    round((row[8 + 4 * s + 2] - row[8 + 4 * s + 1]) / 100, 2),
                    round((row[8 + 4 * s + 3] - row[8 + 4 * s + 2]) / 100, 2),
                    round((row[8 + 4 * (s + 1)] - row[8 + 4 * s + 3]) / 100, 2) if s + 1 < 2 * NH else None]
                   for s in range(2 * NH)]
            cyc = sum(row[64 + 8 + 4 * s + 1] - row[64 + 8 + 4 * s] for s in range(2 * NH))
            wall = sum(row[8 + 4 * s + 1] - row[8 + 4 * s] for s in range(2 * NH))
            out.append({"group": g, "row": r, "clock_ghz": round(cyc / max(wall, 1) / 10.0, 3), "start": us(row[0]),
                        "in_a": us(row[5]), "in_b": us(row[2]), "handoff0": us(row[3]), "first_block": us(row[8]),
                        "last_stores": us(row[8 + 4 * (2 * NH - 1) + 3]), "reduce_end": us(row[8 * (NH + 1)]),
                        "blocks_us": blk})
            continue
        ph = []
        for p in range(1, NH + 1):
            b, c, k, e, h, r5, r6 = (row[8 * p + i] for i in (0, 1, 2, 3, 4, 5, 6))
            ph.append([round((c - b) / 100, 2), round((k - c) / 100, 2), round((e - k) / 100, 2),
                       round((h - e) / 100, 2), round((r5 - k) / 100, 2), round((r6 - r5) / 100, 2)])
        # core clock over the contractions: s_memtime cycles / wall_clock64 (100 MHz) ticks
        cyc = sum(row[64 + 8 * p + 1] - row[64 + 8 * p] for p in range(1, NH + 1))
        wall = sum(row[8 * p + 1] - row[8 * p] for p in range(1, NH + 1))
        out.append({"group": g, "row": r, "clock_ghz": round(cyc / max(wall, 1) / 10.0, 3), "start": us(row[0]), "census": us(row[1]), "input": us(row[2]),
                    "consts": us(row[4]), "in_mfma": us(row[5]), "handoff0": us(row[3]), "end_phase": [us(row[8 * p + 4]) for p in range(1, NH + 1)],
                    "reduce_end": us(row[8 * (NH + 1)]), "phases_us": ph,
                    # (trace builds: phase start to the ring's first operands in hand)
                    "ring_fill_us": [round((row[8 * p + 7] - row[8 * p]) / 100, 2) for p in range(1, NH + 1)]})
    out.sort(key=lambda d: d["reduce_end"])
    for d in out:
        print(json.dumps(d))
    print("launch end (latest reduce): %.2f us" % max(d["reduce_end"] for d in out))
    # every workgroup's start / arrival / census end (the dispatch ramp)
    wg = buf[16384:16384 + 4 * 1024].astype(np.int64).reshape(1024, 4)
    wg = wg[(wg[:, 0] >= t0) & (wg[:, 2] >= wg[:, 0])]
    if len(wg):
        st = np.sort((wg[:, 0] - t0) / 100.0)
        ar = np.sort((wg[:, 1] - t0) / 100.0)
        ce = (wg[:, 2] - t0) / 100.0
        q = lambda a: [round(float(np.quantile(a, f)), 2) for f in (0, 0.25, 0.5, 0.75, 0.9, 1.0)]  # noqa: E731
        print(json.dumps({"workgroups": len(wg), "start_q": q(st), "arrive_q": q(ar), "census_end_q": q(ce),
                          "arrive_minus_start_q": q((wg[:, 1] - wg[:, 0]) / 100.0),
                          "per_xcd_last_start": [round(float(((wg[(wg[:, 3] & 255) == x, 0] - t0) / 100.0).max()), 2)
                                                 if ((wg[:, 3] & 255) == x).any() else None for x in range(8)],
                          "start_xcd_offsets": sorted(set(int(v) for v in ((wg[:, 3] >> 16) & 255)))}))
    # output phase per workgroup (round 5): 3 last phase's stores issued, 0 its hand-off done,
    # 1 first tile contracted, 2 first tile stored
    o = buf[21504:21504 + 256 * 4].astype(np.int64).reshape(256, 4)
    ok = (o[:, 0] >= t0) & (o[:, 3] >= t0)
    if ok.any():
        o = o[ok]
        qq = lambda a: [round(float(np.quantile(a, f)), 2) for f in (0, 0.1, 0.5, 0.9, 1.0)]   # noqa: E731
        has = o[:, 2] > o[:, 0]   # workgroups with an output tile
        print(json.dumps({"out_last_handoff_us_q": qq((o[:, 0] - o[:, 3]) / 100.0),
                          "out_contract_us_q": qq((o[has, 1] - o[has, 0]) / 100.0) if has.any() else None,
                          "out_store_us_q": qq((o[has, 2] - o[has, 1]) / 100.0) if has.any() else None,
                          "out_entry_q": qq((o[:, 0] - t0) / 100.0), "tiles": int(has.sum())}))
    # every workgroup's end (round 5 builds: after the output phase)
    ends = buf[20480:20480 + 1024].astype(np.int64)
    ends = ends[ends >= t0]
    if len(ends):
        e = np.sort((ends - t0) / 100.0)
        print(json.dumps({"workgroup_end_q": [round(float(np.quantile(e, f)), 2) for f in (0, 0.25, 0.5, 0.75, 0.9, 1.0)],
                          "launch_end_us": round(float(e[-1]), 2)}))


if __name__ == "__main__":
    main()
