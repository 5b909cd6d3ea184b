"""A whole training epoch of predict_3dpose.train() (src/predict_3dpose.py:231-259) against
the oracle: the same initial variables, the same shuffled batch list (get_all_batches draws
its permutation from the global numpy RNG, src/linear_model.py:247-300), and one oracle
TF1 train step (oracle/ref_mlp.py train_step) per batch with the dropout stream keyed by the
global step, as the HIP path keys it.

Tolerances.  After hundreds of steps two correct arithmetics no longer agree element by
element: a trainable whose gradient sits at rounding-noise level gets Adam's full normalised
step in whichever direction each arithmetic's noise points (m / (sqrt(v) + eps)), and the
differences feed forward through BN.  The yardstick is therefore the oracle's own float32
restatement (ref_mlp train_step(dt=float32)) run beside the float64 one on the same batches:
the HIP path's deviation from float64 must stay within twice float32's, per tensor (L2,
relative to how far training moved the tensor) and for the trained network's evaluation
outputs on 256 fresh inputs (max |d| / spread); the global step and Adam beta powers match
exactly.  Measured on MI355X (synthetic H3.6M-shaped data, L = 256, 2 residual BN blocks,
keep 0.5, lr 1e-3 -- the reference's flag default of 1.0 makes any two arithmetics part ways
within a few steps -- 328 steps): worst tensor 6.0 % vs float32's 5.9 %, outputs 7.9 % vs
float32's 10.0 %.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import predict_3dpose  # noqa: E402
from oracle import ref_mlp  # noqa: E402


@pytest.mark.parametrize("device_loop", [1])
def test_epoch_tracks_oracle(device_loop, monkeypatch, tmp_path):
    cfg = ref_mlp.Cfg(linear_size=256, num_layers=2, residual=True, batch_norm=True)
    st = ref_mlp.init_state(cfg, seed=3, bn_seed=4)
    st0_params = {k: v.astype(np.float64) for k, v in st.params.items()}
    s32 = st.copy()
    seen = {}
    real_create = predict_3dpose.create_model

    def create(sess, actions, batch_size, flags=None):
        m = real_create(sess, actions, batch_size, flags)
        m.set_weights({**st.params, **st.moving})
        real_gab = m.get_all_batches

        def gab(data_x, data_y, camera_frame, training=True):
            enc, dec = real_gab(data_x, data_y, camera_frame, training=training)
            if training:
                seen["train"] = ([np.array(e) for e in enc], [np.array(d) for d in dec])
            return enc, dec

        m.get_all_batches = gab
        seen["model"] = m
        return m

    monkeypatch.setattr(predict_3dpose, "create_model", create)
    np.random.seed(7)
    flags = predict_3dpose.build_parser().parse_args(
        ["--synthetic", "--epochs", "1", "--linear_size", "256", "--num_layers", "2", "--residual",
         "--batch_norm", "--dropout", "0.5", "--learning_rate", "1e-3", "--train_dir", str(tmp_path), "--device_loop", str(device_loop)])
    model = predict_3dpose.train(flags)
    enc, dec = seen["train"]
    nb = len(enc)
    assert nb > 100
    for i in range(nb):
        ref_mlp.train_step(st, enc[i], dec[i], 0.5, flags.learning_rate, seed=model.seed, ctr=i)
        ref_mlp.train_step(s32, enc[i], dec[i], 0.5, flags.learning_rate, seed=model.seed, ctr=i,
                           dt=np.float32)
    gs, b1, b2 = model.get_step()
    assert gs == nb
    # both sides form the powers as float32 products, one rounding per step
    assert abs(b1 - float(st.beta1_power)) <= 1e-6 * float(st.beta1_power), (b1, st.beta1_power)
    assert abs(b2 - float(st.beta2_power)) <= 1e-6 * float(st.beta2_power), (b2, st.beta2_power)
    w = model.get_weights()
    w32 = {**s32.params, **s32.moving}
    stats = {}
    for name in model.trainable_names():
        if "/b1" in name or "/b2_" in name or "/b3_" in name:   # pre-BN biases: DESIGN.md section 3
            continue
        ref = st.params[name].astype(np.float64)
        moved = np.linalg.norm(ref - st0_params[name])
        stats[name] = (float(np.linalg.norm(w[name] - ref) / moved),
                       float(np.linalg.norm(w32[name] - ref) / moved))
    for name, ref in st.moving.items():
        ref = ref.astype(np.float64)
        stats[name] = (float(np.linalg.norm(w[name] - ref) / np.linalg.norm(ref)),
                       float(np.linalg.norm(w32[name] - ref) / np.linalg.norm(ref)))
    rng = np.random.default_rng(5)
    xe = rng.standard_normal((256, 32))
    ye = model.forward_device(torch.from_numpy(xe.astype(np.float32)).cuda(), False, 1.0).cpu().numpy()
    yr, _ = ref_mlp.forward(st, xe, False, 1.0, 0, 0, 0)
    y32, _ = ref_mlp.forward(s32, xe, False, 1.0, 0, 0, 0)
    out_hip = float(np.abs(ye - yr).max() / np.abs(yr).std())
    out_f32 = float(np.abs(y32 - yr).max() / np.abs(yr).std())
    worst = max(stats, key=lambda k: stats[k][0])
    print("epoch of %d steps: worst tensor deviation %.3g (%s; float32 oracle %.3g, its worst %.3g); "
          "eval outputs %.3g (float32 oracle %.3g)" % (nb, stats[worst][0], worst, stats[worst][1],
                                                        max(v[1] for v in stats.values()), out_hip, out_f32))
    for name, (hip, f32) in stats.items():
        assert hip <= 2 * f32 + 1e-3, (name, hip, f32)
    assert out_hip <= 2 * out_f32 + 1e-3, (out_hip, out_f32)
    model.close()
