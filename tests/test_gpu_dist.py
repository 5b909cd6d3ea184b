"""Data-parallel training and sharded evaluation through the real HIP path, two ranks
on the box's one GPU (gloo backend, device tensors staged through the host).  The
8-GPU RCCL run is the driver's; this checks the DP logic of LinearModel end to end."""
import os
import socket
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
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


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


def _worker_dp_oracle(rank, world, port, out, L=256, B=32, bucket_mbs=(0.25, 0.0)):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import linear_model
    res = {}
    for tag, mb in zip(("bucketed", "single"), bucket_mbs):
        m = linear_model.LinearModel(L, 2, True, True, False, B, 1e-3, "/tmp/p3d_dpo", seed=5 + rank,
                                     data_parallel=True)
        plan = m.dp_buckets(mb, gloo=True)
        assert (len(plan) >= 3) if mb > 0 else not plan, plan
        init = m.get_weights(include_moving=True)
        rng = np.random.default_rng(60 + rank)
        xs = rng.standard_normal((3, B, 32))
        ts = rng.standard_normal((3, B, 48))
        for step in range(3):
            m.step(None, xs[step], ts[step], 0.5, isTraining=True)
        m.check_errors()
        fin = m.get_weights(include_moving=True)
        gx = [torch.zeros(3, B, 32, dtype=torch.float64) for _ in range(world)]
        gt = [torch.zeros(3, B, 48, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gx, torch.from_numpy(xs))
        dist.all_gather(gt, torch.from_numpy(ts))
        mv = torch.from_numpy(np.concatenate([fin[k].ravel() for k in sorted(fin) if "moving" in k]))
        gm = [torch.zeros_like(mv) for _ in range(world)]
        dist.all_gather(gm, mv)
        if rank == 0:
            res.update({tag + "/init/" + k: v for k, v in init.items()})
            res.update({tag + "/final/" + k: v for k, v in fin.items()})
            res[tag + "/xs"] = torch.stack(gx).numpy()
            res[tag + "/ts"] = torch.stack(gt).numpy()
            res[tag + "/moving_ranks"] = torch.stack(gm).numpy()
            res[tag + "/seed"] = np.int64(m.seed)
        m.close()
    if rank == 0:
        np.savez(out, **res)
    dist.destroy_process_group()


def _check_dp_vs_oracle(r, L, wtol=5e-5):
    from oracle import ref_mlp
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=2, residual=True, batch_norm=True)
    finals = {}
    for tag in ("bucketed", "single"):
        init = {k.split("/init/", 1)[1]: r[k] for k in r.files if k.startswith(tag + "/init/")}
        params = {k: v.astype(np.float32) for k, v in init.items() if "moving" not in k}
        moving = {k: v.astype(np.float32) for k, v in init.items() if "moving" in k}
        reps = [ref_mlp.State(cfg=cfg, params={k: v.copy() for k, v in params.items()},
                              moving={k: v.copy() for k, v in moving.items()}) for _ in range(2)]
        xs, ts, seed = r[tag + "/xs"], r[tag + "/ts"], int(r[tag + "/seed"])
        for step in range(3):
            ref_mlp.dp_train_step(reps, [xs[0, step], xs[1, step]], [ts[0, step], ts[1, step]], 0.5, 1e-3,
                                  seed=seed, ctr=step)
        fin = {k.split("/final/", 1)[1]: r[k] for k in r.files if k.startswith(tag + "/final/")}
        finals[tag] = fin
        for name, ref in reps[0].params.items():
            if "/b1" in name or "/b2_" in name or "/b3_" in name:
                continue        # pre-BN biases: noise-driven under BN
            err = np.abs(fin[name] - ref).max()
            assert err < wtol, (tag, name, err)
        # per-replica moving statistics (rank 0's in `fin`, both ranks' gathered)
        mk = sorted(k for k in reps[0].moving)
        for rr in range(2):
            got = r[tag + "/moving_ranks"][rr]
            ref = np.concatenate([reps[rr].moving[k].ravel() for k in mk])
            np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-5)
    for k in finals["single"]:
        np.testing.assert_array_equal(finals["bucketed"][k], finals["single"][k], err_msg=k)


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
    batch, gradients averaged over the replicas)."""
    out = str(tmp_path / "c.npz")
    mp.spawn(_worker_dp_oracle, args=(2, free_port(), out, 1024, 64, (4.0, 0.0)), nprocs=2, join=True)
    _check_dp_vs_oracle(np.load(out), 1024)


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


def _worker_rccl_graph(rank, world, port, out):
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
            m.dp_buckets(8)
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
    dist.destroy_process_group()


def test_dp_rccl_step_graph_capture(tmp_path):
    """The RCCL data-parallel step captured in ONE HIP graph (the bucket all-reduces captured on
    the comm stream, forked from the step by the bucket events and joined before Adam): a 1-rank
    RCCL group (the box has one GPU), 2 buckets at cfg3's size; the captured step == the eager DP
    step, and (average of one replica) == the fused single-GPU step, bit for bit."""
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker_rccl_graph, args=(1, free_port(), out), nprocs=1, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["graph"], r["eager"])
    np.testing.assert_array_equal(r["graph"], r["local"])
    assert int(r["graph_step"]) == int(r["eager_step"]) == 3
