"""Multi-process tests of the data-parallel / sharded paths with the gloo backend on CPU
(world_size 2).  The per-rank arithmetic is the CPU oracle standing in for the GPU
kernels; what is under test is the collective logic of dist_utils.py that the GPU path
runs over RCCL: batch sharding, gradient averaging, parameter broadcast, per-action
all-reduce."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)


def free_port():
    import dist_utils   # the shared helper (3d-pose-baseline_amd/dist_utils.py)
    return dist_utils.free_port()


def _init(rank, world, port):
    sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_train(rank, world, port, out):
    _init(rank, world, port)
    import dist_utils
    from oracle import ref_mlp
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=2)
    st = ref_mlp.init_state(cfg, seed=10 + rank)          # ranks start different ...
    names = [n for n, _ in ref_mlp.param_names(cfg)]
    flat = torch.from_numpy(np.concatenate([st.params[n].ravel() for n in names]).astype(np.float32))
    dist_utils.broadcast_([flat], src=0)                  # ... until rank 0's values are broadcast
    off = 0
    for n in names:
        k = st.params[n].size
        st.params[n] = flat[off:off + k].numpy().reshape(st.params[n].shape).copy()
        off += k
    rng = np.random.default_rng(100 + rank)
    for step in range(3):
        x, t = rng.standard_normal((16, 32)), rng.standard_normal((16, 48))
        o, cache = ref_mlp.forward(st, x, True, 0.5, 7, step, row0=16 * rank)
        _, dy = ref_mlp.mse(o, t)
        grads = ref_mlp.backward(st, cache, dy)
        g = torch.from_numpy(np.concatenate([grads[n].ravel() for n in names]))
        local = g.clone()
        dist_utils.allreduce_mean_(g)
        gathered = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        assert torch.allclose(g, sum(gathered) / world, rtol=1e-12, atol=1e-15)
        off = 0
        avg = {}
        for n in names:
            k = grads[n].size
            avg[n] = g[off:off + k].numpy().reshape(grads[n].shape)
            off += k
        ref_mlp.bn_update(st, cache)
        ref_mlp.adam_apply(st, avg, 1e-3)
    flat = torch.from_numpy(np.concatenate([st.params[n].ravel() for n in names]).astype(np.float64))
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        np.save(out, torch.stack(gathered).numpy())
    dist.destroy_process_group()


def test_dp_ranks_stay_identical(tmp_path):
    out = str(tmp_path / "p.npy")
    mp.spawn(_worker_train, args=(2, free_port(), out), nprocs=2, join=True)
    p = np.load(out)
    np.testing.assert_array_equal(p[0], p[1])


def _worker_eval(rank, world, port, out):
    _init(rank, world, port)
    import dist_utils
    import linear_model
    from oracle import ref_eval, ref_mlp
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=1)
    st = ref_mlp.init_state(cfg, seed=3, bn_seed=4)
    stats = ref_eval.synthetic_stats()
    s2, s3 = ref_eval.synthetic_test_set(scale=0.005)
    actions = ref_eval.define_actions("All")
    table = torch.zeros((len(actions), 18), dtype=torch.float64)
    for ai, a in enumerate(actions):
        enc, dec = linear_model.get_all_batches(ref_eval.get_action_subset(s2, a),
                                                ref_eval.get_action_subset(s3, a), True, 64, training=False)
        lo, hi = dist_utils.shard_range(len(enc), rank, world)
        for e, d in zip(enc[lo:hi], dec[lo:hi]):
            _, o = ref_mlp.eval_step(st, e, d)
            dd = ref_eval.batch_dists(o.astype(np.float32), d, stats["mean3"], stats["std3"], stats["ign3"],
                                      stats["use3"])
            table[ai, :17] += torch.from_numpy(dd.sum(0))
            table[ai, 17] += dd.shape[0]
    dist_utils.allreduce_sum_(table)
    if rank == 0:
        np.save(out, table.numpy())
    dist.destroy_process_group()


def test_sharded_eval_equals_single_process(tmp_path):
    from oracle import ref_eval, ref_mlp
    import linear_model
    out = str(tmp_path / "t.npy")
    mp.spawn(_worker_eval, args=(2, free_port(), out), nprocs=2, join=True)
    t = np.load(out)
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=1)
    st = ref_mlp.init_state(cfg, seed=3, bn_seed=4)
    stats = ref_eval.synthetic_stats()
    s2, s3 = ref_eval.synthetic_test_set(scale=0.005)
    for ai, a in enumerate(ref_eval.define_actions("All")):
        enc, dec = linear_model.get_all_batches(ref_eval.get_action_subset(s2, a),
                                                ref_eval.get_action_subset(s3, a), True, 64, training=False)
        err, _, _ = ref_eval.evaluate_batches(lambda e, d: ref_mlp.eval_step(st, e, d), enc, dec, stats["mean3"],
                                              stats["std3"], stats["use3"], stats["ign3"])
        assert t[ai, 17] == 64 * len(enc)
        assert abs(t[ai, :17].sum() / (t[ai, 17] * 17) - err) < 1e-9


def test_shard_range_partition():
    import dist_utils
    for n in (0, 1, 7, 64, 313):
        for w in (1, 2, 3, 8):
            parts = [dist_utils.shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def test_plan_buckets_cover_backward_order():
    """DP gradient buckets (dist_utils.plan_buckets): every layer range exactly once,
    formed from the output layer down, each ready with its lowest layer."""
    import dist_utils
    # cfg2-like flat layout: input 32x1024 (+b, gamma, beta), 4 hidden 1024^2 (+3x1024), output 1024x48 (+48)
    sizes = [32 * 1024 + 3 * 1024] + [1024 * 1024 + 3 * 1024] * 4 + [1024 * 48 + 64]
    ranges, off = [], 0
    for s in sizes:
        ranges.append((off, off + s))
        off += s
    plan = dist_utils.plan_buckets(ranges, (4 << 20) // 4)
    assert [b[2] for b in plan] == sorted((b[2] for b in plan), reverse=True)
    cov = sorted((lo, hi) for lo, hi, _ in plan)
    assert cov[0][0] == 0 and cov[-1][1] == off and all(a[1] == b[0] for a, b in zip(cov, cov[1:]))
    for lo, hi, layer in plan:       # ready layer = the lowest layer the bucket touches
        assert ranges[layer][0] == lo
    assert len(plan) == 4 and plan[-1][2] == 0      # the short input-layer remainder joined
    assert dist_utils.plan_buckets(ranges, 1) == [(r[0], r[1], l) for l, r in reversed(list(enumerate(ranges)))]
    assert dist_utils.plan_buckets(ranges, off * 2) == [(0, off, 0)]
