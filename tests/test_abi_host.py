"""CPU tests: the C-ABI library loads and exports every entry point of include/p3d.h,
its argument validation answers without a GPU, and the host-side mirror of the
reference interface (data_utils, get_all_batches, lr decay, flags, train_dir)
matches the reference's behaviour (goldens / oracle)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import _p3d
import data_utils
import linear_model
import predict_3dpose
from oracle import ref_eval, ref_mlp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "p3d.h")
GOLD = os.path.join(ROOT, "tests", "golden", "reference_goldens.npz")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(p3d_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = _p3d.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s
    bound = {n for n, _, _ in _p3d.SIGNATURES}
    assert set(syms) == bound, set(syms) ^ bound


def test_library_is_gfx950():
    blob = open(_p3d.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_argument_validation_without_gpu():
    lib = _p3d.lib()
    cfg = _p3d.P3DCfg(100, 1, 1, 1, 0, 32, 48, 0, 64, 1e-3, 0.99)
    h = ctypes.c_void_p()
    assert lib.p3d_create(ctypes.byref(cfg), ctypes.byref(h)) == 1
    assert b"multiple of 64" in lib.p3d_last_error()
    assert lib.p3d_forward(None, None, 0, None, 0, 1.0, 0, 0, 0, None) == 1
    with pytest.raises(ValueError):
        _p3d.check(lib.p3d_mse(None, None, 1, 48, None, None, None), "p3d_mse")
    assert lib.p3d_destroy(None) == 0


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_p3d.P3DError):
        _p3d.load(str(tmp_path / "libp3d.so"))


@pytest.fixture(scope="module")
def g():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_data_utils_match_reference(g):
    use3, ign3 = data_utils.dimension_sets(3)
    np.testing.assert_array_equal(use3, g["ns_use3"])
    np.testing.assert_array_equal(ign3, g["ns_ign3"])
    use2, ign2 = data_utils.dimension_sets(2)
    np.testing.assert_array_equal(use2, g["ns_use2"])
    np.testing.assert_array_equal(ign2, g["ns_ign2"])
    u14, i14 = data_utils.dimension_sets(3, predict_14=True)
    np.testing.assert_array_equal(u14, g["ns_use3_14"])
    # the numeric functions run on the GPU only (tests/test_gpu_data.py pins them to these
    # goldens); without one they fail loudly instead of computing on the host
    if not torch.cuda.is_available():
        with pytest.raises(_p3d.P3DError):
            data_utils.normalization_stats(g["ns_in3"], 3)
        with pytest.raises(_p3d.P3DError):
            data_utils.unNormalizeData(g["un_in"], g["nd_mean"], g["nd_std"], g["ns_ign3"])
        with pytest.raises(_p3d.P3DError):
            data_utils.normalize_data({1: g["nd_in0"]}, g["nd_mean"], g["nd_std"], g["ns_use3"])
    assert data_utils.define_actions("All") == list(g["actions"])
    assert data_utils.define_actions("Walking") == ["Walking"]
    with pytest.raises(ValueError):
        data_utils.define_actions("Dancing")
    assert data_utils.H36M_NAMES == list(g["h36m_names"])
    assert data_utils.SH_NAMES == list(g["sh_names"])


def test_get_all_batches_matches_oracle():
    s2, s3 = ref_eval.synthetic_test_set(scale=0.01)
    for cam in (True,):
        a_enc, a_dec = linear_model.get_all_batches(s2, s3, cam, 64, training=False)
        b_enc, b_dec = ref_eval.get_all_batches(s2, s3, 64, camera_frame=cam, training=False)
        assert len(a_enc) == len(b_enc) > 0
        for x, y in zip(a_enc, b_enc):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a_dec, b_dec):
            np.testing.assert_array_equal(x, y)
    np.random.seed(0)
    enc, dec = linear_model.get_all_batches(s2, s3, True, 64, training=True)
    n = sum(v.shape[0] for v in s2.values())
    assert len(enc) == n // 64 and all(e.shape == (64, 32) and e.dtype == np.float64 for e in enc)
    assert linear_model.get_all_batches({(1, "a", "x.h5"): np.zeros((10, 32))},
                                        {(1, "a", "x.h5"): np.zeros((10, 48))}, True, 64) == ([], [])


def test_lr_decay_and_kaiming_match_oracle():
    for gs in (0, 1, 777, 100000, 4874200):
        assert linear_model.exponential_decay(1.0, gs) == float(ref_mlp.decayed_lr(1.0, gs))
    w = linear_model.kaiming((1024, 1024), np.random.default_rng(0))
    r = ref_mlp.kaiming(np.random.default_rng(0), (1024, 1024))
    np.testing.assert_array_equal(w, r)


def test_flags_defaults_follow_reference():
    """Defaults of src/predict_3dpose.py:31-104 (lr 1.0, keep 1, batch 64, 200 epochs,
    linear 1024, 2 blocks, booleans off)."""
    f = predict_3dpose.build_parser().parse_args([])
    assert (f.learning_rate, f.dropout, f.batch_size, f.epochs) == (1.0, 1, 64, 200)
    assert (f.linear_size, f.num_layers, f.action, f.load) == (1024, 2, "All", 0)
    assert not any([f.camera_frame, f.max_norm, f.batch_norm, f.predict_14, f.use_sh, f.residual,
                    f.procrustes, f.evaluateActionWise, f.sample, f.use_cpu, f.use_fp16])
    f = predict_3dpose.build_parser().parse_args(["--residual", "--batch_norm", "--dropout", "0.5", "--max_norm",
                                                  "--camera_frame", "--evaluateActionWise"])
    d = predict_3dpose.train_dir_for(f)
    assert d == os.path.join("experiments", "All", "dropout_0.5", "epochs_200", "lr_1.0", "residual", "depth_2",
                             "linear_size1024", "batch_size_64", "no_procrustes", "maxnorm",
                             "batch_normalization", "not_stacked_hourglass", "predict_17")


def test_flags_include_openpose_frontend_flags():
    """src/openpose_3dpose_sandbox.py:240-446 reads these through `from predict_3dpose import
    FLAGS`; names and defaults of src/predict_3dpose.py:76-91."""
    f = predict_3dpose.FLAGS
    assert (f.pose_estimation_json, f.interpolation, f.multiplier) == ("/tmp/", False, 0.1)
    assert (f.write_gif, f.gif_fps, f.verbose, f.cache_on_fail) == (False, 30, 2, True)
    g = predict_3dpose.build_parser().parse_args(["--interpolation", "--multiplier", "0.5", "--write_gif",
                                                  "--gif_fps", "10", "--verbose", "3",
                                                  "--pose_estimation_json", "/data/json/"])
    assert (g.interpolation, g.multiplier, g.write_gif, g.gif_fps, g.verbose) == (True, 0.5, True, 10, 3)
    assert g.pose_estimation_json == "/data/json/"


def test_model_requires_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_p3d.P3DError):
        linear_model.LinearModel(256, 1, True, True, False, 64, 1e-3, "/tmp/x")


def test_session_shim_summary():
    s = predict_3dpose.Session()
    ph = linear_model.Placeholder("error_mm")
    out = s.run(("summary", "loss/error_mm"), {ph: 12.5})
    assert out.tag == "loss/error_mm" and out.value == 12.5


def test_checkpoint_io_names_and_order():
    """TF1 global-variable order and the reference's npy-dump file names
    (src/predict_3dpose.py:548-568) -- host logic only."""
    import checkpoint_io as cio
    table = [("linear_model/w1", 32 * 256, 0, 0), ("linear_model/b1", 256, 0, 8192),
             ("linear_model/batch_normalization/gamma", 256, 0, 8448),
             ("linear_model/batch_normalization/beta", 256, 0, 8704),
             ("linear_model/batch_normalization/moving_mean", 256, 1, 0),
             ("linear_model/batch_normalization/moving_variance", 256, 1, 256),
             ("linear_model/w4", 256 * 48, 0, 8960), ("linear_model/b4", 48, 0, 21248)]
    g = cio.global_order(table)
    assert g[:4] == ["learning_rate", "global_step", "linear_model/w1", "linear_model/b1"]
    assert g.index("linear_model/batch_normalization/moving_mean") == 6
    assert g[g.index("beta1_power") + 1] == "beta2_power"
    assert g[-2:] == ["linear_model/b4/Adam", "linear_model/b4/Adam_1"]
    assert cio.trainable_order(table) == [n for n, _, k, _ in table if k == 0]
    f = cio.dump_filename(7, "linear_model/batch_normalization/gamma")
    assert f == "0007 - linear_model-batch_normalization-gamma:0.npy"
    assert cio.parse_dump_filename(f) == (7, "linear_model/batch_normalization/gamma")
    assert cio.parse_dump_filename("notes.txt") is None


def test_checkpoint_global_order_library_table():
    """The table as p3d_create lays it out (every trainable, then every moving statistic):
    tf.global_variables() still puts each BN scope's moving_mean / moving_variance right
    after its beta (src/linear_model.py:112,181,193; the dump of src/predict_3dpose.py:559-568)."""
    import checkpoint_io as cio
    bn = ["linear_model/batch_normalization", "linear_model/two_linear_0/batch_normalization10",
          "linear_model/two_linear_0/batch_normalization20"]
    table = [("linear_model/w1", 8192, 0, 0), ("linear_model/b1", 256, 0, 0),
             (bn[0] + "/gamma", 256, 0, 0), (bn[0] + "/beta", 256, 0, 0),
             ("linear_model/two_linear_0/w2_0", 65536, 0, 0), ("linear_model/two_linear_0/b2_0", 256, 0, 0),
             (bn[1] + "/gamma", 256, 0, 0), (bn[1] + "/beta", 256, 0, 0),
             ("linear_model/two_linear_0/w3_0", 65536, 0, 0), ("linear_model/two_linear_0/b3_0", 256, 0, 0),
             (bn[2] + "/gamma", 256, 0, 0), (bn[2] + "/beta", 256, 0, 0),
             ("linear_model/w4", 12288, 0, 0), ("linear_model/b4", 48, 0, 0)]
    for s in bn:
        table += [(s + "/moving_mean", 256, 1, 0), (s + "/moving_variance", 256, 1, 0)]
    g = cio.global_order(table)
    for s in bn:
        i = g.index(s + "/beta")
        assert g[i - 1] == s + "/gamma"
        assert g[i + 1:i + 3] == [s + "/moving_mean", s + "/moving_variance"]
    assert g.index("linear_model/w4") == g.index(bn[2] + "/moving_variance") + 1
    assert len(g) == 2 + len(table) + 2 + 2 * 14
    assert g.index("beta1_power") == 2 + len(table)


def test_openpose_mapping_matches_oracle():
    """Host joint mapping of the OpenPose front end (src/openpose_3dpose_sandbox.py:25,326-342)."""
    import openpose_frontend
    from oracle import ref_frontend
    rng = np.random.default_rng(9)
    frames = rng.uniform(0, 1000, (7, 36))
    got = openpose_frontend.map_frames(frames)
    for i in range(7):
        np.testing.assert_array_equal(got[i], ref_frontend.map_frame(frames[i]))
    assert openpose_frontend.ORDER == ref_frontend.ORDER


def test_dp_epoch_share_equal_disjoint():
    """Data-parallel epoch: equal contiguous shares of one shared batch list (every replica
    runs the same number of steps; < world leftover batches dropped)."""
    enc = [np.full((2, 32), i) for i in range(11)]
    dec = [np.full((2, 48), i) for i in range(11)]
    seen = []
    for r in range(3):
        e, d = predict_3dpose.dp_epoch_share(enc, dec, r, 3)
        assert len(e) == len(d) == 3
        assert [int(a[0, 0]) for a in e] == [int(a[0, 0]) for a in d]
        seen += [int(a[0, 0]) for a in e]
    assert seen == list(range(9))
