"""OpenPose front-end lifting: FrameLifter's one-graph-per-frame path
(H2D, p3d_normalize, the six layer kernels, p3d_unnormalize, D2H) against the oracle's
per-frame restatement of src/openpose_3dpose_sandbox.py:317-356."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import data_utils  # noqa: E402
import linear_model  # noqa: E402
import openpose_frontend as of  # noqa: E402
from oracle import ref_frontend, ref_mlp  # noqa: E402


def setup(seed=3):
    rng = np.random.default_rng(seed)
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st = ref_mlp.init_state(cfg, seed=seed, bn_seed=seed + 1)
    m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_fe", seed=11)
    m.set_weights({**st.params, **st.moving})
    use2, _ = data_utils.dimension_sets(2)
    use3, ign3 = data_utils.dimension_sets(3)
    stats = dict(mean2=rng.uniform(200, 600, 64), std2=rng.uniform(50, 150, 64),
                 mean3=rng.uniform(-400, 400, 96), std3=rng.uniform(30, 300, 96))
    frames = rng.uniform(100, 900, (23, 36))      # 23 OpenPose frames, 18 joints x (x, y)
    return st, m, stats, use2, use3, ign3, frames


def test_frame_lifter_matches_oracle_and_batches_agree():
    st, m, s, use2, use3, ign3, frames = setup()
    fl1 = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=1)
    got = fl1.lift(frames)
    ref_mm, ref_norm = ref_frontend.lift_frames(st, frames, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3)
    # network outputs vs the fp64 oracle (the tolerance of the MLP parity tests), then x std
    norm = (got[:, use3] - s["mean3"][use3]) / s["std3"][use3]
    err = np.abs(norm - ref_norm)
    assert np.all(err <= 2e-5 + 2e-5 * np.abs(ref_norm)), err.max()
    np.testing.assert_array_equal(got[:, ign3], np.tile(s["mean3"][ign3], (len(frames), 1)))
    assert np.abs(got - ref_mm).max() <= 1e-4 * s["std3"].max()
    # batch 4 runs the same k_gemv layers (rows independent): bit-identical, ragged last call
    fl4 = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=4)
    np.testing.assert_array_equal(fl4.lift(frames), got)
    # batch 8 runs the 16-row MFMA kernels (another summation order): the MLP tolerance
    fl8 = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=8)
    got8 = fl8.lift(frames)                                   # 3 calls, ragged last one
    norm8 = (got8[:, use3] - s["mean3"][use3]) / s["std3"][use3]
    assert np.all(np.abs(norm8 - ref_norm) <= 2e-5 + 2e-5 * np.abs(ref_norm))
    m.close()


def test_frame_lifter_rejects_bad_input():
    st, m, s, use2, use3, ign3, frames = setup(4)
    fl = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=2)
    with pytest.raises(ValueError):
        fl.lift_mapped(np.zeros((3, 64)))
    with pytest.raises(ValueError):
        of.map_frames(np.zeros((2, 10)))
    with pytest.raises(ValueError):
        of.FrameLifter(m, s["mean2"], s["std2"], use2[:10], s["mean3"], s["std3"], ign3)
    m.close()


@pytest.mark.parametrize("B", [1, 3, 4, 8])
def test_lift_bit_identical_to_three_steps(B, monkeypatch):
    """p3d_lift (normalise + forward + unNormalizeData; one persistent launch at B <= 4) == the
    three calls p3d_normalize (float32) -> forward -> p3d_unnormalize, bit for bit; and with the
    chain off (P3D_GEMV_CHAIN=0: p3d_lift takes the three steps itself)."""
    import data_pipeline as dp
    outs = []
    for chain in ("1", "0"):
        monkeypatch.setenv("P3D_GEMV_CHAIN", chain)
        st, m, s, use2, use3, ign3, frames = setup()
        e = torch.from_numpy(of.map_frames(frames[:B])).cuda()
        m2, s2, m3, s3 = (dp.as_device(s[k]) for k in ("mean2", "std2", "mean3", "std3"))
        u2, u3 = dp._dims(use2, 64, "t"), dp._dims(use3, 96, "t")
        out = torch.empty((B, 96), dtype=torch.float64, device="cuda")
        of.lift(m, e, m2, s2, u2, m3, s3, u3, out=out)
        x = dp.normalize(e, m2, s2, u2, out_dtype=torch.float32)
        y = m.forward_device(x, False, 1.0, ctr=0)
        ref = dp.unnormalize(y, m3, s3, u3, 96)
        assert torch.equal(out, ref), (chain, (out - ref).abs().max().item())
        m.check_errors()
        outs.append(out.cpu())
        m.close()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("env", [("P3D_GEMV_FOLD", "0"), ("P3D_GEMV_MAXB", "0")])
def test_frame_lifter_without_batch4_forms(env, monkeypatch):
    """Advisor r4 (medium): FrameLifter must work where the batch <= 4 fold / chain is not
    configured (p3d_lift then runs its three steps itself): without the fold the six k_gemv
    launches give the chain's bits; without the batch <= 4 forms (P3D_GEMV_MAXB=0) the 16-row
    MFMA kernels run (another summation order): the MLP tolerance."""
    st, m, s, use2, use3, ign3, frames = setup()
    ref = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=1).lift(frames[:5])
    m.close()
    monkeypatch.setenv(*env)
    st, m, s, use2, use3, ign3, frames = setup()
    got = of.FrameLifter(m, s["mean2"], s["std2"], use2, s["mean3"], s["std3"], ign3, batch=1).lift(frames[:5])
    if env[0] == "P3D_GEMV_FOLD":
        np.testing.assert_array_equal(got, ref)
    else:
        assert np.abs(got - ref).max() <= 1e-4 * s["std3"].max()
    m.check_errors()
    m.close()


def test_frame_lifter_eager_equals_graph(monkeypatch):
    """FrameLifter's one-launch path (round 6: p3d_lift_sync on the pinned frame and output rows,
    arguments bound once, returning once the launch's completion word says the rows are in host
    memory) == the same launch + a stream synchronize (P3D_HOST_WAIT=0) == its HIP-graph path
    (P3D_LIFT_EAGER=0: H2D, p3d_lift, D2H), bit for bit, at batch 1 and 4 (the chain) and 8 (the
    three calls, where the sync call waits on the stream) -- 6 calls on different frames each, so a
    call returning the previous call's rows would show."""
    for B in (1, 4, 8):
        rng = np.random.default_rng(700 + B)
        use2, _ = data_utils.dimension_sets(2)
        _, ign3 = data_utils.dimension_sets(3)
        stats = (rng.uniform(200, 600, 64), rng.uniform(50, 150, 64), use2, rng.uniform(-400, 400, 96),
                 rng.uniform(30, 300, 96), ign3)
        frames = [of.map_frames(rng.uniform(100, 900, (B, 36))) for _ in range(6)]
        res = {}
        for eager, hw in (("1", "1"), ("1", "0"), ("0", "1")):
            monkeypatch.setenv("P3D_LIFT_EAGER", eager)
            monkeypatch.setenv("P3D_HOST_WAIT", hw)
            cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
            st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
            m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_fl", seed=3, max_batch=64)
            m.set_weights({**st.params, **st.moving})
            fl = of.FrameLifter(m, *stats, batch=B)
            assert (fl._launch is not None) == (eager == "1")
            assert fl._host_wait == (eager == "1" and hw == "1")
            res[eager + hw] = [fl.lift_mapped(e) for e in frames]
            del fl
            m.close()
        for k in ("10", "01"):
            for a, b in zip(res["11"], res[k]):
                np.testing.assert_array_equal(a, b)
        assert not np.array_equal(res["11"][0], res["11"][1])
