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
