"""Data-parallel training and sharded evaluation through the real HIP path, two ranks
on the box's one GPU (gloo backend, device tensors staged through the host).  The
8-GPU RCCL run is the driver's; this checks the DP logic of LinearModel end to end."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    import dist_utils   # the shared helper (3d-pose-baseline_amd/dist_utils.py)
    return dist_utils.free_port()


def _worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    import predict_3dpose
    from oracle import ref_eval
    m = linear_model.LinearModel(256, 2, True, True, False, 32, 1e-3, "/tmp/p3d_dp", seed=5 + rank,
                                 data_parallel=True)
    assert m.data_parallel and m.world == 2
    rng = np.random.default_rng(50 + rank)
    xs, ts = [], []
    for step in range(3):
        x, t = rng.standard_normal((32, 32)), rng.standard_normal((32, 48))
        xs.append(x)
        ts.append(t)
        m.step(None, x, t, 0.5, isTraining=True)
    flat = m.flat["params"].double().cpu()
    g = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(g, flat)
    # BN moving statistics: per replica while training, averaged by sync_moving_stats
    mv = m.flat["moving"].double().cpu()
    gm = [torch.zeros_like(mv) for _ in range(world)]
    dist.all_gather(gm, mv)
    m.sync_moving_stats()
    mv2 = m.flat["moving"].double().cpu()
    gm2 = [torch.zeros_like(mv2) for _ in range(world)]
    dist.all_gather(gm2, mv2)
    # sharded action-wise eval == one process over everything (tables summed over ranks)
    stats = ref_eval.synthetic_stats()
    s2, s3 = ref_eval.synthetic_test_set(scale=0.01)
    acts = ref_eval.define_actions("All")
    errs, avg = predict_3dpose.evaluate_action_wise(m, s2, s3, stats["mean3"], stats["std3"], stats["use3"], acts)
    if rank == 0:
        np.savez(out, params=torch.stack(g).numpy(), avg=avg, xs=np.stack(xs), ts=np.stack(ts),
                 moving=torch.stack(gm).numpy(), moving_synced=torch.stack(gm2).numpy())
    dist.destroy_process_group()


def test_dp_two_ranks_one_gpu(tmp_path):
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["params"][0], r["params"][1])
    assert np.isfinite(r["avg"])
    assert not np.array_equal(r["moving"][0], r["moving"][1])          # different local batches
    np.testing.assert_array_equal(r["moving_synced"][0], r["moving_synced"][1])
    np.testing.assert_allclose(r["moving_synced"][0], r["moving"].mean(axis=0), rtol=1e-6, atol=1e-7)


def _worker_buckets(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    import linear_model
    res = {}
    for max_norm in (False, True):
        ms = {}
        for tag, mb in (("bucketed", 1.0), ("single", 0.0), ("local", None)):
            m = linear_model.LinearModel(1024, 2, True, True, max_norm, 64, 1e-3, "/tmp/p3d_dpb", seed=9,
                                         data_parallel=(mb is not None))
            m.initialize(seed=4)
            if mb is not None:
                plan = m.dp_buckets(mb)
                if mb > 0:
                    assert plan and len(plan) >= 3, plan
                    cov = sorted((lo, hi) for lo, hi, _ in plan)
                    assert cov[0][0] == 0 and all(a[1] == b[0] for a, b in zip(cov, cov[1:]))
                    assert cov[-1][1] == m.flat["grads"].numel()
                else:
                    assert not plan
            rng = np.random.default_rng(3)
            for _ in range(3):
                m.train_step_device(torch.from_numpy(rng.standard_normal((64, 32)).astype(np.float32)).cuda(),
                                    torch.from_numpy(rng.standard_normal((64, 48)).astype(np.float32)).cuda(), 0.5)
            torch.cuda.synchronize()
            ms[tag] = m.flat["params"].cpu().numpy().copy()
            m.close()
        res["mn%d" % max_norm] = np.stack([ms["bucketed"], ms["single"], ms["local"]])
    np.savez(out, **res)
    import dist_utils
    dist_utils.close_native_comms()
    dist.destroy_process_group()


def test_dp_bucketed_allreduce_rccl(tmp_path):
    """The bucketed all-reduce (per-layer gradient-ready events, one RCCL all-reduce per
    bucket from a side stream) gives the same bits as the single all-reduce and as the
    local single-GPU step (world 1: the average of one replica), with and without max-norm."""
    out = str(tmp_path / "b.npz")
    mp.spawn(_worker_buckets, args=(1, free_port(), out), nprocs=1, join=True)
    r = np.load(out)
    for k in r.files:
        np.testing.assert_array_equal(r[k][0], r[k][1])
        np.testing.assert_array_equal(r[k][0], r[k][2])


def _worker_dp_oracle(rank, world, port, out, L=256, B=32, bucket_mbs=(0.25, 0.0), steps=3):
    """Both forms (bucketed, single all-reduce) of `steps` DP steps; rank 0 keeps the full state
    (tf.global_variables + the averaged gradient) before and after every step, every rank's
    moving statistics are gathered (they stay per replica)."""
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    res = {}

    def gather_moving(m):
        mv = m.flat["moving"].double().cpu()
        gm = [torch.zeros_like(mv) for _ in range(world)]
        dist.all_gather(gm, mv)
        return torch.stack(gm).numpy()

    for tag, mb in zip(("bucketed", "single"), bucket_mbs):
        m = linear_model.LinearModel(L, 2, True, True, False, B, 1e-3, "/tmp/p3d_dpo", seed=5 + rank,
                                     data_parallel=True)
        plan = m.dp_buckets(mb, gloo=True)
        assert (len(plan) >= 2) if mb > 0 else not plan, plan
        rng = np.random.default_rng(60 + rank)
        xs = rng.standard_normal((steps, B, 32))
        ts = rng.standard_normal((steps, B, 48))
        for step in range(steps + 1):
            st = m.get_state()
            mvr = gather_moving(m)
            if rank == 0:
                for k, v in st.items():
                    res["%s/s%d/%s" % (tag, step, k)] = np.asarray(v)
                res["%s/s%d/moving_ranks" % (tag, step)] = mvr
                if step > 0:
                    res["%s/s%d/grads" % (tag, step)] = m.flat["grads"].cpu().numpy().copy()
            if step < steps:
                m.step(None, xs[step], ts[step], 0.5, isTraining=True)
        m.check_errors()
        gx = [torch.zeros(steps, B, 32, dtype=torch.float64) for _ in range(world)]
        gt = [torch.zeros(steps, B, 48, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gx, torch.from_numpy(xs))
        dist.all_gather(gt, torch.from_numpy(ts))
        if rank == 0:
            res[tag + "/xs"] = torch.stack(gx).numpy()
            res[tag + "/ts"] = torch.stack(gt).numpy()
            res[tag + "/seed"] = np.int64(m.seed)
            res[tag + "/offsets"] = np.array([[o, n] for _, n, k, o in m.param_table if k == 0], np.int64)
            res[tag + "/names"] = np.array([nm for nm, _, k, _ in m.param_table if k == 0])
            res[tag + "/moving_names"] = np.array([nm for nm, _, k, _ in m.param_table if k == 1])
            res[tag + "/moving_offsets"] = np.array([[o, n] for _, n, k, o in m.param_table if k == 1], np.int64)
        m.close()
    if rank == 0:
        np.savez(out, **res)
    dist.destroy_process_group()


PRE_BN = ("/b1", "/b2_", "/b3_")


def _check_dp_vs_oracle(r, L, steps=3, wtol=5e-5):
    """Every DP step of the HIP path vs the oracle's DP step (oracle/ref_mlp.dp_train_step, fp64
    arithmetic, fp32 variables as TF1) taken from the HIP path's own state before that step
    (weights, Adam slots, step state, each replica's moving statistics) on the same two batches.
    Per-step forcing measures each step's arithmetic: after a few free-running steps TF1 Adam
    (eps 1e-8) turns a noise-level difference of one weight's gradient into an update that differs
    by a sizeable fraction of the learning rate -- measured at L = 1024: |dw| 2.9e-4 after three
    free-running steps while every step, forced, agrees to a few 1e-6 (tools/dp_grad_probe.py).
    Pre-BN biases (their gradient is analytically zero under BN): their averaged
    gradient must be at noise level and their update TF1 Adam of it.  Both forms must also agree
    bit for bit (the bucketed all-reduce changes no value)."""
    from oracle import ref_mlp
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=2, residual=True, batch_norm=True)
    worst = 0.0
    for tag in ("bucketed", "single"):
        names = [str(n) for n in r[tag + "/names"]]
        offs = {n: tuple(o) for n, o in zip(names, r[tag + "/offsets"])}
        mnames = [str(n) for n in r[tag + "/moving_names"]]
        moffs = {n: tuple(o) for n, o in zip(mnames, r[tag + "/moving_offsets"])}
        xs, ts, seed = r[tag + "/xs"], r[tag + "/ts"], int(r[tag + "/seed"])
        for s in range(steps):
            pre = lambda k: r["%s/s%d/%s" % (tag, s, k)]            # noqa: E731
            post = lambda k: r["%s/s%d/%s" % (tag, s + 1, k)]       # noqa: E731
            reps = []
            for rr in range(2):
                mv = pre("moving_ranks")[rr]
                reps.append(ref_mlp.State(
                    cfg=cfg, params={n: pre(n).astype(np.float32) for n in names},
                    moving={n: mv[o:o + c].astype(np.float32) for n, (o, c) in moffs.items()},
                    m={n: pre(n + "/Adam").astype(np.float32) for n in names},
                    v={n: pre(n + "/Adam_1").astype(np.float32) for n in names},
                    global_step=int(pre("global_step")), beta1_power=np.float32(pre("beta1_power")),
                    beta2_power=np.float32(pre("beta2_power"))))
            ref_mlp.dp_train_step(reps, [xs[0, s], xs[1, s]], [ts[0, s], ts[1, s]], 0.5, 1e-3, seed=seed, ctr=s)
            g = post("grads")
            lr = ref_mlp.decayed_lr(1e-3, s)
            b1p, b2p = float(pre("beta1_power")), float(pre("beta2_power"))
            alpha = lr * np.sqrt(1.0 - b2p) / (1.0 - b1p)
            for n in names:
                got = post(n)
                if any(t in n for t in PRE_BN):
                    o, c = offs[n]
                    gb = g[o:o + c].astype(np.float64)
                    gw = np.abs(g[offs[n.replace("/b", "/w")][0]:][:offs[n.replace("/b", "/w")][1]]).max()
                    assert np.abs(gb).max() <= 1e-4 * gw, (tag, s, n, np.abs(gb).max(), gw)
                    mm = pre(n + "/Adam").astype(np.float64) + (gb - pre(n + "/Adam")) * 0.1
                    vv = pre(n + "/Adam_1").astype(np.float64) + (gb * gb - pre(n + "/Adam_1")) * 0.001
                    want = pre(n).astype(np.float64) - mm * alpha / (np.sqrt(vv) + 1e-8)
                    assert np.abs(got - want).max() <= 1e-6, (tag, s, n, np.abs(got - want).max())
                    continue
                err = float(np.abs(got - reps[0].params[n]).max())
                worst = max(worst, err)
                assert err < wtol, (tag, s, n, err)
            for rr in range(2):
                mv = post("moving_ranks")[rr]
                for n, (o, c) in moffs.items():
                    np.testing.assert_allclose(mv[o:o + c], reps[rr].moving[n], rtol=2e-5, atol=2e-5,
                                               err_msg="%s step %d rank %d %s" % (tag, s, rr, n))
    for k in r.files:
        if k.startswith("single/s"):
            np.testing.assert_array_equal(r[k], r["bucketed/" + k[len("single/"):]], err_msg=k)
    return worst


def _check_dp_free_running(r, L, steps, tag="bucketed"):
    """The same DP run free-running: the oracle's DP step from the run's INITIAL state (weights,
    Adam slots, step state, each replica's moving statistics) for every step, in float64 and in
    float32, against the HIP run's final state.  As in tests/test_gpu_train_epoch.py, two correct
    arithmetics part ways (TF1 Adam's eps = 1e-8 turns a noise-level gradient difference into a
    sizeable update difference), so the yardstick is the oracle's own float32 restatement: per
    tensor the HIP path's deviation from float64 (L2, relative to how far training moved the
    tensor; moving statistics relative to their norm) must stay within twice float32's + 1e-5.
    Pre-BN biases are excluded (their gradient is analytically zero under BN).
    Returns {tensor: (hip, f32)}."""
    from oracle import ref_mlp
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=2, residual=True, batch_norm=True)
    names = [str(n) for n in r[tag + "/names"]]
    mnames = [str(n) for n in r[tag + "/moving_names"]]
    moffs = {n: tuple(o) for n, o in zip(mnames, r[tag + "/moving_offsets"])}
    xs, ts, seed = r[tag + "/xs"], r[tag + "/ts"], int(r[tag + "/seed"])
    pre = lambda k: r["%s/s0/%s" % (tag, k)]              # noqa: E731
    fin = lambda k: r["%s/s%d/%s" % (tag, steps, k)]      # noqa: E731

    def replicas():
        out = []
        for rr in range(2):
            mv = pre("moving_ranks")[rr]
            out.append(ref_mlp.State(
                cfg=cfg, params={n: pre(n).astype(np.float32) for n in names},
                moving={n: mv[o:o + c].astype(np.float32) for n, (o, c) in moffs.items()},
                m={n: pre(n + "/Adam").astype(np.float32) for n in names},
                v={n: pre(n + "/Adam_1").astype(np.float32) for n in names},
                global_step=int(pre("global_step")), beta1_power=np.float32(pre("beta1_power")),
                beta2_power=np.float32(pre("beta2_power"))))
        return out
    r64, r32 = replicas(), replicas()
    for s in range(steps):
        ref_mlp.dp_train_step(r64, [xs[0, s], xs[1, s]], [ts[0, s], ts[1, s]], 0.5, 1e-3, seed=seed, ctr=s)
        ref_mlp.dp_train_step(r32, [xs[0, s], xs[1, s]], [ts[0, s], ts[1, s]], 0.5, 1e-3, seed=seed, ctr=s,
                              dt=np.float32)
    assert int(fin("global_step")) == r64[0].global_step == steps
    stats = {}
    for n in names:
        if any(t in n for t in PRE_BN):
            continue
        ref, p0 = r64[0].params[n].astype(np.float64), pre(n).astype(np.float64)
        moved = np.linalg.norm(ref - p0)
        stats[n] = (float(np.linalg.norm(fin(n) - ref) / moved), float(np.linalg.norm(r32[0].params[n] - ref) / moved))
    for rr in range(2):
        mv = fin("moving_ranks")[rr]
        for n, (o, c) in moffs.items():
            ref = r64[rr].moving[n].astype(np.float64)
            stats["%s[rank %d]" % (n, rr)] = (float(np.linalg.norm(mv[o:o + c] - ref) / np.linalg.norm(ref)),
                                             float(np.linalg.norm(r32[rr].moving[n] - ref) / np.linalg.norm(ref)))
    worst = max(stats, key=lambda k: stats[k][0])
    print("free-running DP, %d steps: worst %s hip %.3g (float32 oracle %.3g)" % (steps, worst, *stats[worst]))
    for n, (hip, f32) in stats.items():
        # a floor scaled to the measured drift (worst tensor 3.1e-5 vs the float32
        # oracle's 3.8e-5), so a DP-path error of 1e-4 relative fails
        assert hip <= 2 * f32 + 1e-5, (n, hip, f32)
    return stats


def test_dp_two_ranks_match_oracle(tmp_path):
    """Two data-parallel replicas x 32 rows (gloo, one GPU; bucketed all-reduce driven by the
    per-layer gradient-ready events, and the single all-reduce) == the oracle's DP step
    (oracle/ref_mlp.dp_train_step: per-replica forward/backward with global dropout rows,
    averaged gradients, one TF1 Adam update, per-replica BN statistics) over 3 steps."""
    out = str(tmp_path / "o.npz")
    mp.spawn(_worker_dp_oracle, args=(2, free_port(), out), nprocs=2, join=True)
    _check_dp_vs_oracle(np.load(out), 256)


def test_dp_cfg3_two_ranks_match_oracle(tmp_path):
    """BASELINE configs[2] at its own size: L = 1024, 2 residual blocks, BN, keep 0.5, batch 64
    PER RANK, two data-parallel ranks (gloo on the box's one GPU; RCCL refuses two ranks on one
    device), the bucketed event-driven all-reduce (4 MB buckets) and the single all-reduce, 3
    steps vs the oracle's DP step (src/linear_model.py:137-145: one optimizer step per global
    batch, gradients averaged over the replicas): teacher-forced per step, and
    free-running against the oracle's float64 / float32 runs from the same initial state."""
    out = str(tmp_path / "c.npz")
    mp.spawn(_worker_dp_oracle, args=(2, free_port(), out, 1024, 64, (4.0, 0.0), 4), nprocs=2, join=True)
    r = np.load(out)
    _check_dp_vs_oracle(r, 1024, steps=4)
    # and free-running over the same 4 steps: the HIP run's final state vs the oracle started once
    # from the run's initial state (the per-step forcing hides accumulated divergence)
    _check_dp_free_running(r, 1024, 4)


def _worker_graph_vs_eager(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    rng = np.random.default_rng(80 + rank)
    xs = torch.from_numpy(rng.standard_normal((4, 64, 32)).astype(np.float32)).cuda()
    ts = torch.from_numpy(rng.standard_normal((4, 64, 48)).astype(np.float32)).cuda()
    res = {}
    for tag in ("eager", "graph"):
        m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_dpg", seed=3,
                                     data_parallel=True)
        m.initialize(seed=12)
        if tag == "eager":
            m.dp_buckets(8, gloo=True)
            for i in range(4):
                m.train_step_device(xs[i], ts[i], 0.5)
        else:
            xb, tb = torch.empty_like(xs[0]), torch.empty_like(ts[0])
            step = m.train_step_graph(xb, tb, 0.5)
            for i in range(4):
                xb.copy_(xs[i])
                tb.copy_(ts[i])
                step()
        torch.cuda.synchronize()
        m.check_errors()
        for k in ("params", "moving", "adam_m", "adam_v"):
            res[tag + "/" + k] = m.flat[k].cpu().numpy().copy()
        res[tag + "/step"] = np.array(m.get_step(), np.float64)
        m.close()
    g = [torch.zeros(res["graph/params"].size, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(g, torch.from_numpy(res["graph/params"]))
    if rank == 0:
        res["graph/params_ranks"] = torch.stack(g).numpy()
        np.savez(out, **res)
    dist.destroy_process_group()


def test_dp_graph_step_bit_identical_to_eager(tmp_path):
    """The data-parallel step captured in HIP graphs (LinearModel.train_step_graph; under gloo:
    a forward + backward graph, the host all-reduce, an optimizer graph) == the eager bucketed
    DP step, bit for bit over 4 steps at cfg3's size (L = 1024, B = 64 per rank, keep 0.5):
    weights, Adam slots, moving statistics, step state; replicas identical."""
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker_graph_vs_eager, args=(2, free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    for k in ("params", "moving", "adam_m", "adam_v", "step"):
        np.testing.assert_array_equal(r["graph/" + k], r["eager/" + k], err_msg=k)
    np.testing.assert_array_equal(r["graph/params_ranks"][0], r["graph/params_ranks"][1])
    assert r["graph/step"][0] == 4


def _worker_rccl_graph(rank, world, port, out, bucket_mb=8):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    import linear_model
    rng = np.random.default_rng(90)
    xs = torch.from_numpy(rng.standard_normal((3, 64, 32)).astype(np.float32)).cuda()
    ts = torch.from_numpy(rng.standard_normal((3, 64, 48)).astype(np.float32)).cuda()
    res = {}
    for tag in ("eager", "graph", "local"):
        m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_dpr", seed=4,
                                     data_parallel=(tag != "local"))
        m.initialize(seed=13)
        if tag == "local":
            for i in range(3):
                m.train_step_device(xs[i], ts[i], 0.5)
        else:
            m.dp_buckets(bucket_mb)
            m.train_step_device(xs[0], ts[0], 0.5)       # eager first step (communicator set up)
            if tag == "eager":
                for i in (1, 2):
                    m.train_step_device(xs[i], ts[i], 0.5)
            else:
                xb, tb = xs[1].clone(), ts[1].clone()
                step = m.train_step_graph(xb, tb, 0.5)
                step()
                xb.copy_(xs[2])
                tb.copy_(ts[2])
                step()
        torch.cuda.synchronize()
        m.check_errors()
        res[tag] = m.flat["params"].cpu().numpy().copy()
        res[tag + "_step"] = np.array(m.get_step()[0])
        m.close()
    np.savez(out, **res)
    import dist_utils
    dist_utils.close_native_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize("force_multi,bucket_mb", [("0", 8), ("1", 8), ("1", 0)])
def test_dp_rccl_step_graph_capture(tmp_path, monkeypatch, force_multi, bucket_mb):
    """The RCCL data-parallel step captured in ONE HIP graph: a 1-rank RCCL group (the box has one
    GPU) at cfg3's size; the captured step == the eager DP step, and (average of one replica) ==
    the fused single-GPU step, bit for bit.
    bucket_mb = 8: 2 buckets, the bucket all-reduces captured on the comm stream, forked from the
    step by the bucket events and joined before Adam.
    force_multi = 1 (P3D_DP_FORCE_MULTI): the 1-rank group takes p3d_train_step_dp's
    N > 1 branch, the code every rank of an 8-GPU run executes, captured and eager, still
    bit-identical to the fused step -- with buckets (the comm-stream fork, one
    ncclAllReduce(ncclAvg) per bucket behind its gradient-ready event, the rev joins, per-bucket
    Adam on the compute stream) and without (round 6's default: one ncclAllReduce(ncclAvg) of the
    flat gradient on the compute stream after the backward, then one optimizer pass)."""
    monkeypatch.setenv("P3D_DP_FORCE_MULTI", force_multi)
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker_rccl_graph, args=(1, free_port(), out, bucket_mb), nprocs=1, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["graph"], r["eager"])
    np.testing.assert_array_equal(r["graph"], r["local"])
    assert int(r["graph_step"]) == int(r["eager_step"]) == 3


def _worker_rccl_capture_linger(rank, world, port, out):
    """BENCH_r03's abort, reproduced deterministically: eager DP steps, a torch collective still in
    flight, then -- with no synchronisation in between -- the capture of the DP step, and replays
    spread over ~3 s (many ProcessGroupNCCL watchdog polls) before the bits are compared."""
    import time
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    import dist_utils
    import linear_model
    rng = np.random.default_rng(91)
    x0 = torch.from_numpy(rng.standard_normal((64, 32)).astype(np.float32)).cuda()
    t0 = torch.from_numpy(rng.standard_normal((64, 48)).astype(np.float32)).cuda()
    reps, per = 12, 2
    res = {}
    for tag in ("graph", "eager", "local"):
        m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_dpl", seed=6,
                                     data_parallel=(tag != "local"))
        m.initialize(seed=14)
        if tag != "local":
            m.dp_buckets(8)
        xb, tb = x0.clone(), t0.clone()
        for _ in range(3):
            m.train_step_device(xb, tb, 0.5)
        if tag == "graph":
            w = torch.ones(1 << 16, device="cuda")
            work = dist.all_reduce(w, async_op=True)        # a torch Work the watchdog still holds
            s0 = torch.cuda.Stream()
            s0.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s0, capture_error_mode="thread_local"):
                for _ in range(per):
                    m.train_step_device(xb, tb, 0.5)
            m._step_host -= per
            torch.cuda.current_stream().wait_stream(s0)
            for _ in range(reps):
                g.replay()
                torch.cuda.synchronize()
                time.sleep(0.25)
            work.wait()
        else:
            for _ in range(reps * per):
                m.train_step_device(xb, tb, 0.5)
        torch.cuda.synchronize()
        m.check_errors()
        res[tag] = m.flat["params"].cpu().numpy().copy()
        res[tag + "_step"] = np.array(m.get_step()[0])
        m.close()
    dist_utils.close_native_comms()
    np.savez(out, **res)
    dist.destroy_process_group()


def test_dp_rccl_capture_after_eager_lingers(tmp_path):
    """The RCCL DP step (libp3d's own communicator, p3d_train_step_dp) captured right after eager DP
    steps with a torch collective in flight, then replayed over ~3 s: the process survives the
    watchdog's polls, and graph == eager == the fused single-GPU step bit for bit (1-rank group)."""
    out = str(tmp_path / "l.npz")
    mp.spawn(_worker_rccl_capture_linger, args=(1, free_port(), out), nprocs=1, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["graph"], r["eager"])
    np.testing.assert_array_equal(r["graph"], r["local"])
    assert int(r["graph_step"]) == int(r["eager_step"]) == 3 + 24
