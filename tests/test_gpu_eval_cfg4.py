"""cfg4 (BASELINE.json configs[3]): the evaluateActionWise sweep over the FULL synthetic
H3.6M-shaped test set -- 15 actions, frames per action ~ U[20000, 40000] drawn as bench.py's
eval_sweep draws them, the reference's per-action n % 64 tail drop: 494,784 frames
(tests/golden/cfg4_data.py) -- through the HIP path (predict_3dpose.evaluate_action_wise:
large-M GEMM launches + the fused MPJPE kernel, fp64 per-action sums, one all-reduce), on one
rank and on two gloo ranks sharing the GPU, against the oracle's per-action MPJPE
(src/predict_3dpose.py:274-298 calling evaluate_batches :352-444 on get_action_subset
:337-349; oracle/ref_eval.py with the fp64 forward of oracle/ref_mlp.py), committed as
tests/golden/cfg4_oracle.npz by tests/golden/make_cfg4_oracle.py (75 s of CPU: too long to
recompute inside a GPU test).  Tolerance: north_star's 1e-4 mm on every action and on the
unweighted Average.
"""
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
GOLD = os.path.join(ROOT, "tests", "golden")
TOL_MM = 1e-4


def _setup():
    for p in (os.path.join(ROOT, "3d-pose-baseline_amd"), ROOT, GOLD):
        if p not in sys.path:
            sys.path.insert(0, p)
    from cfg4_data import ACTIONS, make_cfg4_set
    from oracle import ref_eval, ref_mlp
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    s2, s3 = make_cfg4_set()
    return st, ref_eval.synthetic_stats(), s2, s3, list(ACTIONS)


def _hip_sweep(st, stats, s2, s3, acts):
    import linear_model
    import predict_3dpose
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_cfg4", seed=3, max_batch=8192)
    m.set_weights({**st.params, **st.moving})
    errs, avg = predict_3dpose.evaluate_action_wise(m, s2, s3, stats["mean3"], stats["std3"], stats["use3"], acts)
    m.close()
    return errs, avg


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "cfg4_oracle.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_cfg4_action_wise_one_rank_vs_oracle(gold):
    st, stats, s2, s3, acts = _setup()
    assert list(gold["actions"]) == acts
    assert int(gold["frames"].sum()) == 494784       # BASELINE configs[3] as bench.py draws it
    errs, avg = _hip_sweep(st, stats, s2, s3, acts)
    for a, ref in zip(acts, gold["mpjpe_mm"]):
        assert abs(errs[a] - float(ref)) <= TOL_MM, (a, errs[a], float(ref))
    assert abs(avg - float(gold["average_mm"])) <= TOL_MM, (avg, float(gold["average_mm"]))


def _free_port():
    import dist_utils   # the shared helper (3d-pose-baseline_amd/dist_utils.py)
    return dist_utils.free_port()


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st, stats, s2, s3, acts = _setup()
    errs, avg = _hip_sweep(st, stats, s2, s3, acts)
    if rank == 0:
        np.savez(out, errs=np.array([errs[a] for a in acts]), avg=avg)
    dist.destroy_process_group()


def test_cfg4_action_wise_two_ranks_vs_oracle(gold, tmp_path):
    """Frames sharded over two ranks (contiguous slices of each action's batch list after
    the tail drop), one all-reduce of the [15, 19] fp64 table: the same per-action MPJPE."""
    out = str(tmp_path / "cfg4.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    for i, a in enumerate(gold["actions"]):
        assert abs(float(r["errs"][i]) - float(gold["mpjpe_mm"][i])) <= TOL_MM, (a, float(r["errs"][i]))
    assert abs(float(r["avg"]) - float(gold["average_mm"])) <= TOL_MM
