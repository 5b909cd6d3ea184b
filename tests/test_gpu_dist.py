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
