"""CPU tests of the oracle: pinned against the reference's own outputs where the reference
can run in this image (tests/golden/reference_goldens.npz, made by importing the
reference's data_utils/procrustes -- tests/golden/make_golden.py), against published
Philox4x32-10 known-answer vectors, and cross-checked against torch-CPU autograd for the
MLP arithmetic that TensorFlow (absent) would compute ("parity unpinned")."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import ref_eval, ref_mlp

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.npz")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def g():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# ------------------------------------------------------------------ reference goldens
def test_index_sets_match_reference(g):
    use3, ign3 = ref_eval.dims_to_use(3)
    use2, ign2 = ref_eval.dims_to_use(2)
    use14, ign14 = ref_eval.dims_to_use(3, predict_14=True)
    np.testing.assert_array_equal(use3, g["ns_use3"])
    np.testing.assert_array_equal(ign3, g["ns_ign3"])
    np.testing.assert_array_equal(use2, g["ns_use2"])
    np.testing.assert_array_equal(ign2, g["ns_ign2"])
    np.testing.assert_array_equal(use14, g["ns_use3_14"])
    np.testing.assert_array_equal(ign14, g["ns_ign3_14"])
    assert len(use3) == 48 and len(use2) == 32


def test_normalization_stats_match_reference(g):
    m3, s3, ign3, use3 = ref_eval.normalization_stats(g["ns_in3"], 3)
    m2, s2, _, _ = ref_eval.normalization_stats(g["ns_in2"], 2)
    np.testing.assert_array_equal(m3, g["ns_mean3"])
    np.testing.assert_array_equal(s3, g["ns_std3"])
    np.testing.assert_array_equal(m2, g["ns_mean2"])
    np.testing.assert_array_equal(s2, g["ns_std2"])


def test_normalize_unnormalize_match_reference(g):
    use3 = g["ns_use3"]
    d = {("a",): g["nd_in0"], ("b",): g["nd_in1"]}
    out = ref_eval.normalize_data(d, g["nd_mean"], g["nd_std"], use3)
    np.testing.assert_array_equal(out[("a",)], g["nd_out0"])
    np.testing.assert_array_equal(out[("b",)], g["nd_out1"])
    np.testing.assert_array_equal(ref_eval.unNormalizeData(g["un_in"], g["nd_mean"], g["nd_std"], g["ns_ign3"]),
                                  g["un_out"])
    np.testing.assert_array_equal(ref_eval.unNormalizeData(g["un_in32"], g["nd_mean"], g["nd_std"], g["ns_ign3"]),
                                  g["un_out32"])


def test_mpjpe_dists_match_reference(g):
    d = ref_eval.batch_dists(g["mp_pred_n"], g["mp_gt_n"], g["nd_mean"], g["nd_std"], g["ns_ign3"], g["ns_use3"])
    np.testing.assert_array_equal(d, g["mp_dists"])
    dp = ref_eval.batch_dists(g["mp_pred_n"], g["mp_gt_n"], g["nd_mean"], g["nd_std"], g["ns_ign3"],
                              g["ns_use3"], procrustes=True)
    np.testing.assert_allclose(dp, g["mp_dists_procrustes"], rtol=1e-12, atol=1e-10)


def test_mpjpe_predict14_and_mirrored_match_reference(g):
    ign14 = g["ns_ign3_14"]
    for proc, key in ((False, "mp14_dists"), (True, "mp14_dists_procrustes")):
        d = ref_eval.batch_dists(g["mp14_pred_n"], g["mp14_gt_n"], g["mp14_mean"], g["mp14_std"], ign14,
                                 g["ns_use3_14"], predict_14=True, procrustes=proc)
        np.testing.assert_allclose(d, g[key], rtol=1e-12, atol=1e-10)
    # mirrored predictions: the det < 0 branch of compute_similarity_transform
    d = ref_eval.batch_dists(g["mpr_pred_n"], g["mpr_gt_n"], g["nd_mean"], g["nd_std"], g["ns_ign3"],
                             g["ns_use3"], procrustes=True)
    np.testing.assert_allclose(d, g["mpr_dists_procrustes"], rtol=1e-12, atol=1e-10)


def test_procrustes_matches_reference(g):
    for tag, scale in (("s", True), ("n", False)):
        d, Z, T, b, c = ref_eval.compute_similarity_transform(g["pr_X"], g["pr_Y"], compute_optimal_scale=scale)
        np.testing.assert_allclose(d, g["pr_%s_d" % tag], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(Z, g["pr_%s_Z" % tag], rtol=1e-12, atol=1e-10)
        np.testing.assert_allclose(T, g["pr_%s_T" % tag], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(b, g["pr_%s_b" % tag], rtol=1e-12)
        np.testing.assert_allclose(c, g["pr_%s_c" % tag], rtol=1e-12, atol=1e-10)


def test_actions_and_names_match_reference(g):
    assert ref_eval.define_actions("All") == list(g["actions"])
    assert ref_eval.H36M_NAMES == list(g["h36m_names"])
    with pytest.raises(ValueError):
        ref_eval.define_actions("Dancing")


def test_sh_permutation_known_answer(g):
    """SH_TO_GT_PERM known answer asserted by the reference (src/data_utils.py:136)."""
    sh = list(g["sh_names"])
    perm = np.array([sh.index(n) for n in ref_eval.H36M_NAMES if n != '' and n != 'Neck/Nose'])
    np.testing.assert_array_equal(perm, [6, 2, 1, 0, 3, 4, 5, 7, 8, 9, 13, 14, 15, 12, 11, 10])


# ------------------------------------------------------------------ Philox known answers
@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_known_answers(ctr, key, expect):
    """Random123 philox4x32-10 KAT vectors (the same stream the HIP kernels use)."""
    out = ref_mlp.philox4x32_10(*ctr, *key)
    assert tuple(int(np.asarray(o)) for o in out) == expect


def test_dropout_uniform_properties():
    u = ref_mlp.dropout_uniform(7, 3, 1, 0, 256, 1024)
    assert u.dtype == np.float32 and u.min() >= 0 and u.max() < 1
    assert abs(float(u.mean()) - 0.5) < 0.01
    # keyed by global row: a row-shifted window reproduces the same values
    np.testing.assert_array_equal(ref_mlp.dropout_uniform(7, 3, 1, 64, 64, 1024), u[64:128])
    m = ref_mlp.dropout_mask(0.5, u)
    assert set(np.unique(m)) <= {0.0, 1.0} and abs(m.mean() - 0.5) < 0.01
    assert np.all(ref_mlp.dropout_mask(1.0, u) == 1.0)


# ------------------------------------------------------------------ MLP vs torch autograd
def torch_loss(cfg, st, x, t, keep, seed, ctr):
    """Independent restatement of the TF1 graph in torch (float64), for autograd."""
    P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in st.params.items()}
    bns = ref_mlp.bn_names(cfg)

    def eff(name):
        w = P[name]
        if cfg.max_norm:
            n = torch.sqrt(torch.sum(w * w))
            return w / torch.maximum(n, torch.tensor(1.0, dtype=torch.float64))
        return w

    def layer(xx, w, b, bn, site):
        z = xx @ eff(w) + P[b]
        if bn is not None:
            mean = z.mean(0)
            var = ((z - mean.detach()) ** 2).mean(0)
            inv = torch.rsqrt(var + cfg.bn_eps) * P[bn + "/gamma"]
            z = z * inv + (P[bn + "/beta"] - mean * inv)
        r = torch.relu(z)
        if keep < 1:
            u = ref_mlp.dropout_uniform(seed, ctr, site, 0, xx.shape[0], r.shape[1])
            r = r / keep * torch.tensor(ref_mlp.dropout_mask(keep, u), dtype=torch.float64)
        return r

    xx = torch.tensor(np.asarray(x, np.float32), dtype=torch.float64)
    y = layer(xx, "linear_model/w1", "linear_model/b1", bns[0] if bns else None, 0)
    for i in range(cfg.num_layers):
        s = "linear_model/two_linear_%d/" % i
        h = layer(y, s + "w2_%d" % i, s + "b2_%d" % i, bns[1 + 2 * i] if bns else None, 1 + 2 * i)
        y2 = layer(h, s + "w3_%d" % i, s + "b3_%d" % i, bns[2 + 2 * i] if bns else None, 2 + 2 * i)
        y = y + y2 if cfg.residual else y2
    out = y @ eff("linear_model/w4") + P["linear_model/b4"]
    tt = torch.tensor(np.asarray(t, np.float32), dtype=torch.float64)
    loss = ((out - tt) ** 2).mean()
    loss.backward()
    return loss.item(), out.detach().numpy(), {k: v.grad.numpy() for k, v in P.items()}


@pytest.mark.parametrize("residual,batch_norm,max_norm,keep", [
    (True, True, False, 1.0), (True, True, False, 0.5), (False, False, False, 0.7),
    (True, False, True, 1.0), (True, True, True, 0.5), (False, True, False, 1.0)])
def test_oracle_backward_matches_autograd(residual, batch_norm, max_norm, keep):
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=2, residual=residual, batch_norm=batch_norm, max_norm=max_norm)
    st = ref_mlp.init_state(cfg, seed=3, bn_seed=4)
    rng = np.random.default_rng(1)
    x, t = rng.standard_normal((16, 32)), rng.standard_normal((16, 48))
    out, cache = ref_mlp.forward(st, x, True, keep, 5, 2, 0)
    loss, dy = ref_mlp.mse(out, t)
    grads = ref_mlp.backward(st, cache, dy)
    tl, to, tg = torch_loss(cfg, st, x, t, keep, 5, 2)
    assert abs(loss - tl) < 1e-12 * max(1, tl)
    np.testing.assert_allclose(out, to, rtol=1e-10, atol=1e-12)
    for k in grads:
        np.testing.assert_allclose(grads[k], tg[k], rtol=1e-7, atol=1e-12, err_msg=k)


def test_eval_mode_uses_moving_stats():
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=1)
    st = ref_mlp.init_state(cfg, seed=3, bn_seed=4)
    x = np.random.default_rng(2).standard_normal((8, 32))
    o1, _ = ref_mlp.forward(st, x, False)
    o2, _ = ref_mlp.forward(st, x[:3], False)
    np.testing.assert_allclose(o1[:3], o2, rtol=1e-12)   # rows independent in eval


def test_adam_tf1_form_and_bn_updates():
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=1)
    st = ref_mlp.init_state(cfg, seed=3)
    rng = np.random.default_rng(4)
    x, t = rng.standard_normal((16, 32)), rng.standard_normal((16, 48))
    w0 = st.params["linear_model/w4"].astype(np.float64).copy()
    out, cache = ref_mlp.forward(st, x, True)
    _, dy = ref_mlp.mse(out, t)
    grads = ref_mlp.backward(st, cache, dy)
    ref_mlp.bn_update(st, cache)
    ref_mlp.adam_apply(st, grads, 0.01)
    g = grads["linear_model/w4"]
    m = 0.1 * g
    v = 0.001 * g * g
    alpha = 0.01 * np.sqrt(1 - 0.999) / (1 - 0.9)
    np.testing.assert_allclose(st.params["linear_model/w4"], w0 - m * alpha / (np.sqrt(v) + 1e-8), rtol=1e-6,
                               atol=1e-7)
    assert st.global_step == 1 and abs(st.beta1_power - 0.81) < 1e-7
    mm = st.moving["linear_model/batch_normalization/moving_mean"]
    np.testing.assert_allclose(mm, cache["in"]["mean"] * (1 - np.float32(0.99)), rtol=1e-5, atol=1e-9)


def test_decayed_lr():
    assert ref_mlp.decayed_lr(1.0, 0) == np.float32(1.0)
    np.testing.assert_allclose(ref_mlp.decayed_lr(1.0, 100000), 0.96, rtol=1e-6)
    np.testing.assert_allclose(ref_mlp.decayed_lr(0.5, 50000), 0.5 * 0.96 ** 0.5, rtol=1e-6)


def test_kaiming_truncation():
    w = ref_mlp.kaiming(np.random.default_rng(0), (1024, 1024))
    s = np.sqrt(2 / 1024)
    assert np.abs(w).max() <= 2 * s + 1e-7
    assert abs(w.std() / s - 0.8796) < 0.01      # std of N(0,1) truncated at 2 sigma


def test_get_all_batches_tail_drop_and_order():
    d2 = {(9, "Walking", "a.1.h5"): np.arange(70 * 32).reshape(70, 32).astype(float),
          (11, "Walking", "b.2.h5"): np.ones((30, 32))}
    d3 = {k: np.zeros((v.shape[0], 48)) for k, v in d2.items()}
    enc, dec = ref_eval.get_all_batches(d2, d3, 64, camera_frame=True, training=False)
    assert len(enc) == 1 and enc[0].shape == (64, 32)
    np.testing.assert_array_equal(enc[0], d2[(9, "Walking", "a.1.h5")][:64])
    enc, dec = ref_eval.get_all_batches(d2, d3, 64, training=True, rng=np.random.default_rng(0))
    assert len(enc) == 1


def test_dp_train_step_oracle_consistent():
    """oracle dp_train_step: one replica == train_step; two replicas on identical batches
    (keep 1: identical gradients) == train_step on that batch; replicas stay identical."""
    from oracle import ref_mlp
    cfg = ref_mlp.Cfg(linear_size=64, num_layers=1, residual=True, batch_norm=True)
    rng = np.random.default_rng(0)
    x, t = rng.standard_normal((16, 32)), rng.standard_normal((16, 48))
    a = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    b = a.copy()
    reps = [a.copy(), a.copy()]
    ref_mlp.train_step(a, x, t, 0.5, 1e-3, seed=3, ctr=0)
    ref_mlp.dp_train_step([b], [x], [t], 0.5, 1e-3, seed=3, ctr=0)
    for k in a.params:
        np.testing.assert_array_equal(a.params[k], b.params[k])
    c = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    ref_mlp.train_step(c, x, t, 1.0, 1e-3, seed=3, ctr=0)
    ref_mlp.dp_train_step(reps, [x, x], [t, t], 1.0, 1e-3, seed=3, ctr=0)
    for k in c.params:
        np.testing.assert_allclose(reps[0].params[k], c.params[k], rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(reps[0].params[k], reps[1].params[k])


def test_cfg4_fixture_matches_its_generator():
    """tests/golden/cfg4_oracle.npz (the oracle's per-action MPJPE of the cfg4 sweep, used by
    tests/test_gpu_eval_cfg4.py) was made from cfg4_data.make_cfg4_set: same actions, same
    tail-dropped frame counts (494,784 in all, bench.py's eval_sweep draw)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from cfg4_data import ACTIONS, make_cfg4_set
    from oracle import ref_eval
    g = np.load(os.path.join(ROOT, "tests", "golden", "cfg4_oracle.npz"), allow_pickle=False)
    assert list(g["actions"]) == ACTIONS == ref_eval.define_actions("All")
    s2, s3 = make_cfg4_set()
    for a, n in zip(ACTIONS, g["frames"]):
        enc, _ = ref_eval.get_all_batches(ref_eval.get_action_subset(s2, a), ref_eval.get_action_subset(s3, a), 64,
                                          camera_frame=True, training=False)
        assert 64 * len(enc) == int(n), a
    assert int(g["frames"].sum()) == 494784
    counts = np.random.default_rng(4).integers(20000, 40001, 15)   # bench.py bench_eval's draw
    assert int(sum(int(c) // 64 for c in counts)) * 64 == 494784


@pytest.mark.parametrize("L,N,nnz,B", [(1024, 2, 8, 1280), (4096, 4, 4, 1024), (512, 1, 8, 200)])
def test_integer_models_are_exact(L, N, nnz, B):
    """tests/exact_models.py: the integer-valued models the bit-exact GPU tests use really are
    exact -- every float32 oracle value an integer below 2^23 (exact_forward asserts it), the
    float64 and float32 accumulations of the bf16 emulation identical -- so 'bit for bit' there is
    a property of the arithmetic, not of one summation order."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import exact_models
    cfg, st = exact_models.integer_state(L, N, nnz=nnz)
    x = exact_models.integer_inputs(B, seed=L + B)
    out = exact_models.exact_forward(st, x)
    assert float((out != 0).mean()) > 0.5            # not a degenerate all-zero network
    assert np.array_equal(ref_mlp.forward_bf16(st, x, acc=np.float64), ref_mlp.forward_bf16(st, x, acc=np.float32))
