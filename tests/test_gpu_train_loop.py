"""predict_3dpose.train(): the device-resident epoch loop (--device_loop 1) and the
reference's per-batch step() loop (--device_loop 0) train bit-identically (synthetic
H3.6M-shaped data, 1 epoch, L = 256, then the evaluation pass and a checkpoint)."""
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import predict_3dpose  # noqa: E402


def _run(device_loop, tdir):
    np.random.seed(123)   # get_all_batches shuffles with the global numpy RNG, as the reference
    flags = predict_3dpose.build_parser().parse_args(
        ["--synthetic", "--epochs", "1", "--linear_size", "256", "--num_layers", "2", "--residual",
         "--batch_norm", "--dropout", "0.5", "--train_dir", tdir, "--device_loop", str(device_loop)])
    model = predict_3dpose.train(flags)
    w = model.get_weights()
    gs = model.get_step()
    model.close()
    return w, gs


def test_device_loop_matches_step_loop():
    with tempfile.TemporaryDirectory() as tdir:
        wa, ga = _run(1, os.path.join(tdir, "a"))
        wb, gb = _run(0, os.path.join(tdir, "b"))
    assert ga == gb and ga[0] > 0
    for k in wa:
        np.testing.assert_array_equal(wa[k], wb[k], err_msg=k)


def test_create_model_load_restores_latest(tmp_path):
    """create_model(--load N) after a real train() run (src/predict_3dpose.py:163-181): two
    epochs write checkpoint-S1 and checkpoint-S2; --load S1 checks that checkpoint-S1.index
    exists and then restores the checkpoint the directory's `checkpoint` file names as the
    latest (S2) -- the reference's own behaviour (:180 restores ckpt.model_checkpoint_path);
    load_exact=True (this build's keyword) restores S1 itself; a missing N raises ValueError."""
    import checkpoint_io
    import tf_bundle
    tdir = str(tmp_path)
    args = ["--synthetic", "--epochs", "2", "--linear_size", "256", "--num_layers", "1", "--residual",
            "--batch_norm", "--dropout", "0.5", "--learning_rate", "1e-3", "--train_dir", tdir]
    np.random.seed(7)
    flags = predict_3dpose.build_parser().parse_args(args)
    model = predict_3dpose.train(flags)
    final = model.get_state()
    model.close()
    ck_dir = predict_3dpose.train_dir_for(flags)
    latest = tf_bundle.read_checkpoint_state(ck_dir)
    s2 = int(latest.rsplit("-", 1)[1])
    s1 = s2 // 2
    assert s1 > 0 and os.path.isfile(os.path.join(ck_dir, "checkpoint-%d.index" % s1))
    assert int(final["global_step"]) == s2
    first = tf_bundle.read_bundle(os.path.join(ck_dir, "checkpoint-%d" % s1))
    lflags = predict_3dpose.build_parser().parse_args(args + ["--load", str(s1)])
    for exact, want in ((False, final), (True, first)):
        m = predict_3dpose.create_model(None, ["All"], lflags.batch_size, lflags, load_exact=exact)
        got = m.get_state()
        for k in checkpoint_io.global_order(m.param_table):
            np.testing.assert_array_equal(np.asarray(got[k], np.float64), np.asarray(want[k], np.float64),
                                          err_msg="%s (load_exact=%s)" % (k, exact))
        assert m.get_step()[0] == (s1 if exact else s2)
        m.close()
    with pytest.raises(ValueError, match="does not seem to exist"):
        bad = predict_3dpose.build_parser().parse_args(args + ["--load", str(s1 + 1)])
        predict_3dpose.create_model(None, ["All"], bad.batch_size, bad)


def test_create_model_load_npz_only_directory(tmp_path):
    """Advisor r3 (low): a directory holding only an earlier build's checkpoint-N.npz (no
    `checkpoint` state file) restores N itself; a missing N still raises ValueError."""
    import checkpoint_io
    args = ["--linear_size", "256", "--num_layers", "1", "--residual", "--batch_norm",
            "--learning_rate", "1e-3", "--train_dir", str(tmp_path)]
    flags = predict_3dpose.build_parser().parse_args(args)
    m = predict_3dpose.create_model(None, ["All"], flags.batch_size, flags)
    rng = np.random.default_rng(3)
    for _ in range(3):
        m.step(None, rng.standard_normal((64, 32)), rng.standard_normal((64, 48)), 0.5, isTraining=True)
    want = m.get_state()
    m.close()
    d = predict_3dpose.train_dir_for(flags)
    os.makedirs(d, exist_ok=True)
    np.savez(os.path.join(d, "checkpoint-3.npz"), **want)
    lflags = predict_3dpose.build_parser().parse_args(args + ["--load", "3"])
    m2 = predict_3dpose.create_model(None, ["All"], lflags.batch_size, lflags)
    got = m2.get_state()
    for k in checkpoint_io.global_order(m2.param_table):
        np.testing.assert_array_equal(np.asarray(got[k], np.float64), np.asarray(want[k], np.float64), err_msg=k)
    assert m2.get_step()[0] == 3
    m2.close()
    with pytest.raises(ValueError, match="does not seem to"):
        bad = predict_3dpose.build_parser().parse_args(args + ["--load", "4"])
        predict_3dpose.create_model(None, ["All"], bad.batch_size, bad)


@pytest.mark.parametrize("use_sh", [False, True])
def test_train_from_archives(tmp_path, use_sh):
    """train() on files (src/predict_3dpose.py:194-208): cameras, 3D poses and 2D inputs read
    from the .npz archive forms of cameras.h5 and the H3.6M tree through data_utils'
    read_3d_data / create_2d_data (or read_2d_predictions), one epoch, evaluation, checkpoint."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from synth_cameras import write_h36m_archives
    rng = np.random.default_rng(31)
    tree, camsp = str(tmp_path / "h36m.npz"), str(tmp_path / "cameras.npz")
    write_h36m_archives(tree, camsp, rng, ["Walking", "Directions"], frames=400, sh=use_sh)
    np.random.seed(5)
    args = ["--epochs", "1", "--linear_size", "128", "--num_layers", "1", "--residual", "--batch_norm",
            "--dropout", "0.5", "--learning_rate", "1e-3", "--camera_frame", "--action", "Walking",
            "--data_dir", tree, "--cameras_path", camsp, "--train_dir", str(tmp_path / "exp")]
    flags = predict_3dpose.build_parser().parse_args(args + (["--use_sh"] if use_sh else []))
    d = predict_3dpose.load_data(flags)
    n2 = sum(len(v) for v in d["train_set_2d"].values())
    assert n2 == sum(len(v) for v in d["train_set_3d"].values())   # camera frame: one 3D row per 2D row
    assert all(v.shape[1] == 32 for v in d["train_set_2d"].values())
    assert all(v.shape[1] == 48 for v in d["train_set_3d"].values())
    model = predict_3dpose.train(flags)
    step = model.get_step()[0]
    w = model.get_weights()
    model.close()
    assert step == n2 // 64                          # get_all_batches drops the n % 64 tail
    assert all(np.isfinite(v).all() for v in w.values())
    ck = predict_3dpose.train_dir_for(flags)
    assert os.path.isfile(os.path.join(ck, "checkpoint-%d.index" % step))
