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
