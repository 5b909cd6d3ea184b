"""Diagnostic: per-replica gradients of the second data-parallel step (2 gloo ranks on one
GPU, L = 1024, B = 64 per rank) vs the oracle's per-replica backward at the same state.

    python tools/dp_grad_probe.py OUT.json
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)


def free_port():
    import dist_utils   # the shared helper (3d-pose-baseline_amd/dist_utils.py)
    return dist_utils.free_port()


def worker(rank, world, port, out, L, B, keep):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    m = linear_model.LinearModel(L, 2, True, True, False, B, 1e-3, "/tmp/p3d_dpg", seed=5, data_parallel=True)
    m.dp_buckets(0)
    init = m.get_weights(include_moving=True)
    rng = np.random.default_rng(60 + rank)
    xs = rng.standard_normal((2, B, 32))
    ts = rng.standard_normal((2, B, 48))
    m.step(None, xs[0], ts[0], keep, isTraining=True)
    after0 = m.get_weights(include_moving=True)
    am0, av0 = m.flat["adam_m"].cpu().numpy().copy(), m.flat["adam_v"].cpu().numpy().copy()
    x1 = torch.from_numpy(xs[1].astype(np.float32)).cuda()
    t1 = torch.from_numpy(ts[1].astype(np.float32)).cuda()
    loss, y = m.compute_gradients(x1, t1, keep, ctr=1)
    torch.cuda.synchronize()
    g = {n: m.grad(n).cpu().numpy().copy() for n in m.trainable_names()}
    # and the real second DP step: averaged gradient (left in the grads buffer) and the update
    m.set_weights({k: v for k, v in after0.items()})   # compute_gradients moved the moving stats
    m.step(None, xs[1], ts[1], keep, isTraining=True)
    torch.cuda.synchronize()
    flat = {"am0": am0, "av0": av0, "gavg": m.flat["grads"].cpu().numpy().copy(),
            "p1": m.flat["params"].cpu().numpy().copy(), "p0flat": None}
    flat.pop("p0flat")
    offs = {n: (o, k) for n, k, kind, o in [(a, b, c, d) for a, b, c, d in m.param_table] if kind == 0}
    flat["w2off"] = np.int64(offs["linear_model/two_linear_0/w2_0"][0])
    for tag, d in (("init", init), ("after0", after0), ("grad", g)):
        for n, v in d.items():
            flat[tag + "/" + n] = v
    flat["xs"], flat["ts"], flat["seed"], flat["y"] = xs, ts, np.int64(m.seed), y.cpu().numpy()
    np.savez(out % rank, **flat)
    m.close()
    dist.destroy_process_group()


def main(out_json, L=1024, B=64, keep=0.5):
    from oracle import ref_mlp
    out = "/tmp/dpg_%d.npz"
    mp.spawn(worker, args=(2, free_port(), out, L, B, keep), nprocs=2, join=True)
    rs = [np.load(out % r) for r in range(2)]
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=2, residual=True, batch_norm=True)
    r0 = rs[0]
    init = {k[5:]: r0[k] for k in r0.files if k.startswith("init/")}
    params = {k: v.astype(np.float32) for k, v in init.items() if "moving" not in k}
    moving = {k: v.astype(np.float32) for k, v in init.items() if "moving" in k}
    reps = [ref_mlp.State(cfg=cfg, params={k: v.copy() for k, v in params.items()},
                          moving={k: v.copy() for k, v in moving.items()}) for _ in range(2)]
    seed = int(r0["seed"])
    ref_mlp.dp_train_step(reps, [rs[0]["xs"][0], rs[1]["xs"][0]], [rs[0]["ts"][0], rs[1]["ts"][0]], keep, 1e-3,
                          seed=seed, ctr=0)
    report = {"after0": {}, "grad": {}, "out": {}}
    for n in params:
        report["after0"][n] = float(np.abs(r0["after0/" + n] - reps[0].params[n]).max())
    for r in range(2):
        st = reps[r]
        # the oracle's state after step 0 replaced by the GPU's (isolates this step's gradient)
        for n in params:
            st.params[n] = rs[r]["after0/" + n].astype(np.float64)
        for n in moving:
            st.moving[n] = rs[r]["after0/" + n].astype(np.float64)
        outp, cache = ref_mlp.forward(st, rs[r]["xs"][1], True, keep, seed, 1, r * B)
        loss, dy = ref_mlp.mse(outp, rs[r]["ts"][1])
        gr = ref_mlp.backward(st, cache, dy)
        report["out"]["rank%d" % r] = float(np.abs(rs[r]["y"] - outp).max())
        for n in gr:
            scale = float(np.abs(gr[n]).max()) or 1.0
            report["grad"].setdefault(n, {})["rank%d" % r] = float(np.abs(rs[r]["grad/" + n] - gr[n]).max()) / scale
    # the second step's update of w2_0 on the GPU vs TF1 Adam (fp64) from the GPU's own state
    # and averaged gradient, and vs the oracle's averaged gradient
    off = int(r0["w2off"])
    n2 = "linear_model/two_linear_0/w2_0"
    sz = params[n2].size
    p0 = r0["after0/" + n2].reshape(-1).astype(np.float64)
    m0, v0 = r0["am0"][off:off + sz].astype(np.float64), r0["av0"][off:off + sz].astype(np.float64)
    ggpu = r0["gavg"][off:off + sz].astype(np.float64)
    p1 = r0["p1"][off:off + sz].astype(np.float64)
    b1p, b2p = 0.9 ** 2, 0.999 ** 2
    alpha = 1e-3 * np.sqrt(1 - b2p) / (1 - b1p)
    def adam(g):
        mm = m0 + (g - m0) * 0.1
        vv = v0 + (g * g - v0) * 0.001
        return p0 - mm * alpha / (np.sqrt(vv) + 1e-8)
    gref = (rs[0]["grad/" + n2].reshape(-1) + rs[1]["grad/" + n2].reshape(-1)).astype(np.float64) / 2
    e_gpu_adam = np.abs(adam(ggpu) - p1)
    i = int(np.argmax(e_gpu_adam))
    report["w2_0_step1"] = {"adam_from_gpu_grad_max": float(e_gpu_adam.max()), "at": i,
                            "g_gpu": float(ggpu[i]), "g_avg_of_rank_grads": float(gref[i]),
                            "m0": float(m0[i]), "v0": float(v0[i]), "p0": float(p0[i]), "p1": float(p1[i]),
                            "grad_avg_vs_rank_grads_max": float(np.abs(ggpu - gref).max())}
    json.dump(report, open(out_json, "w"), indent=1)
    print(json.dumps(report["w2_0_step1"]))
    print(json.dumps(report["out"]))
    print(json.dumps(sorted(((max(v.values()), k) for k, v in report["grad"].items()), reverse=True)[:6]))


if __name__ == "__main__":
    main(sys.argv[1])
