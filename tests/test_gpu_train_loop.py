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
