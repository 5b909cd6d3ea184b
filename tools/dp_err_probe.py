"""Diagnostic: data-parallel training (2 gloo ranks on one GPU) vs the oracle's DP step, per
step and per tensor, over a few shapes / forms -- which of (L, B, exchange form, buckets)
moves the HIP result away from the fp64 oracle, and how far the fp32 oracle itself moves.

    python tools/dp_err_probe.py OUT.json
"""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out, L, B, mb, xchg, steps):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["P3D_TRAIN_XCHG"] = str(xchg)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    m = linear_model.LinearModel(L, 2, True, True, False, B, 1e-3, "/tmp/p3d_dpe", seed=5, data_parallel=True)
    m.dp_buckets(mb, gloo=True)
    res = {"init": m.get_weights(include_moving=True)}
    rng = np.random.default_rng(60 + rank)
    xs = rng.standard_normal((steps, B, 32))
    ts = rng.standard_normal((steps, B, 48))
    for s in range(steps):
        m.step(None, xs[s], ts[s], 0.5, isTraining=True)
        res["s%d" % s] = m.get_weights(include_moving=False)
    m.check_errors()
    gx = [torch.zeros(steps, B, 32, dtype=torch.float64) for _ in range(world)]
    gt = [torch.zeros(steps, B, 48, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(gx, torch.from_numpy(xs))
    dist.all_gather(gt, torch.from_numpy(ts))
    if rank == 0:
        flat = {"seed": np.int64(m.seed), "xs": torch.stack(gx).numpy(), "ts": torch.stack(gt).numpy()}
        for k, d in res.items():
            for n, v in d.items():
                flat[k + "/" + n] = v
        np.savez(out, **flat)
    m.close()
    dist.destroy_process_group()


def main(out_json):
    from oracle import ref_mlp
    report = []
    steps = 3
    for L, B, mb, xchg in ((1024, 64, 8.0, 1), (1024, 64, 0.0, 1), (1024, 64, 0.0, 0), (1024, 32, 0.0, 1),
                           (256, 64, 0.0, 1), (256, 32, 0.0, 1)):
        out = "/tmp/dpe.npz"
        mp.spawn(worker, args=(2, free_port(), out, L, B, mb, xchg, steps), nprocs=2, join=True)
        r = np.load(out)
        cfg = ref_mlp.Cfg(linear_size=L, num_layers=2, residual=True, batch_norm=True)
        init = {k[5:]: r[k] for k in r.files if k.startswith("init/")}
        params = {k: v.astype(np.float32) for k, v in init.items() if "moving" not in k}
        moving = {k: v.astype(np.float32) for k, v in init.items() if "moving" in k}
        row = {"L": L, "B": B, "bucket_mb": mb, "xchg": xchg, "steps": []}
        reps = {dt: [ref_mlp.State(cfg=cfg, params={k: v.copy() for k, v in params.items()},
                                   moving={k: v.copy() for k, v in moving.items()}) for _ in range(2)]
                for dt in (np.float64, np.float32)}
        for s in range(steps):
            for dt, rp in reps.items():
                ref_mlp.dp_train_step(rp, [r["xs"][0, s], r["xs"][1, s]], [r["ts"][0, s], r["ts"][1, s]], 0.5, 1e-3,
                                      seed=int(r["seed"]), ctr=s, dt=dt)
            errs = {}
            for n in params:
                if "/b1" in n or "/b2_" in n or "/b3_" in n:
                    continue
                ref = reps[np.float64][0].params[n]
                errs[n] = {"hip": float(np.abs(r["s%d/%s" % (s, n)] - ref).max()),
                           "np32": float(np.abs(reps[np.float32][0].params[n] - ref).max())}
            row["steps"].append(errs)
        report.append(row)
        print(json.dumps({"L": L, "B": B, "mb": mb, "xchg": xchg,
                          "worst": max((v["hip"], k) for k, v in row["steps"][-1].items())}), flush=True)
    json.dump(report, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
