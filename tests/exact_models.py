"""Integer-valued models: parity checks that need no tolerance (round 6).

Every weight is 0 or +-1 (a few non-zeros per column), every bias, BN shift and moving mean a small
integer, BN gamma 1 or 2, the moving variance 0.999f -- so that in float32 var + eps == 1.0
exactly and the eval-BN scale gamma / sqrt(var + eps) is gamma itself -- and the inputs integers in
[-4, 4].  Then every product, partial sum, BN affine, ReLU and residual add of the forward is an
integer below 2^24, which float32 represents exactly whatever the summation order: the GPU paths
(any tiling, K split, wave association, launch shape) and the oracle's float32 forward
(oracle/ref_mlp.forward, dt=float32) must agree BIT FOR BIT, at the BASELINE configurations' full
sizes.  A wrong k-slice, a skipped or doubled tile, a stale hand-off or a misplaced row changes an
integer and fails.  bf16 paths: +-1 weights and small integers are exact in bf16, every activation
is rounded to bf16 (round-to-nearest-even of an exactly accumulated integer) by the kernels and by
the oracle's bf16 emulation alike, so they too must agree bit for bit.

(The test data is synthetic; the arithmetic it checks is that of src/linear_model.py:92-128 with
BN in inference mode -- the reference's own outputs for it are not available here)"""
import numpy as np

from oracle import ref_mlp


def integer_state(L, N, nnz=8, seed=5, residual=True, batch_norm=True, predict_14=False):
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=N, residual=residual, batch_norm=batch_norm,
                      predict_14=predict_14)
    st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    rng = np.random.default_rng(seed)
    for name, v in list(st.params.items()):
        leaf = name.split("/")[-1]
        if leaf.startswith("w"):
            K, Nn = v.shape
            w = np.zeros((K, Nn), np.float32)
            for j in range(Nn):
                rows = rng.choice(K, size=min(nnz, K), replace=False)
                w[rows, j] = rng.choice([-1.0, 1.0], size=len(rows))
            st.params[name] = w
        elif leaf == "gamma":
            st.params[name] = rng.choice([1.0, 2.0], size=v.shape).astype(np.float32)
        else:
            st.params[name] = rng.integers(-3, 4, size=v.shape).astype(np.float32)
    for name, v in list(st.moving.items()):
        st.moving[name] = (np.full(v.shape, 0.999, np.float32) if name.endswith("moving_variance")
                           else rng.integers(-3, 4, size=v.shape).astype(np.float32))
    return cfg, st


def integer_inputs(B, seed=1, dim=32):
    return np.random.default_rng(seed).integers(-4, 5, size=(B, dim)).astype(np.float32)


def exact_forward(st, x):
    """The oracle's float32 forward, with the check that it IS exact: every pre-activation,
    activation and output an integer of magnitude < 2^23."""
    out, cache = ref_mlp.forward(st, x, False, dt=np.float32)
    vals = [cache[k][f] for k in cache if k not in ("order", "out") for f in ("z", "a")] + [out]
    for v in vals:
        assert np.array_equal(v, np.round(v)), "not an integer model"
        assert float(np.abs(v).max()) < 2.0 ** 23, "integer model leaves float32's exact range"
    return out
