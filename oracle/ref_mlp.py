"""CPU oracle for the 2D->3D lifting MLP hot path.  TEST INFRASTRUCTURE ONLY.

This module is the *checker*, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``3d-pose-baseline_amd/``) runs hand-written HIP kernels and
fails loudly when they are missing.

It restates, op for op, the TF1 graph the reference builds in
``src/linear_model.py`` (reference at EsauPR/3d-pose-baseline):

* ``kaiming``                      -- src/linear_model.py:17-29
* input layer  (w1/b1/BN/relu/dropout)   -- src/linear_model.py:103-114
* ``two_linear`` residual block    -- src/linear_model.py:154-201
* output layer (w4/b4)             -- src/linear_model.py:120-124
* MSE loss                         -- src/linear_model.py:129
* Adam + exponential decay + BN UPDATE_OPS -- src/linear_model.py:84-90,136-145
* ``step`` return tuples           -- src/linear_model.py:203-245

TensorFlow itself is NOT installed anywhere in this image, so the MLP arithmetic
is "parity unpinned" against the reference: this
restatement follows TF1 op semantics (non-fused batch_normalization with biased
variance and eps=1e-3, ``x/keep*floor(keep+U)`` dropout, ApplyAdam's
``alpha = lr*sqrt(1-b2^t)/(1-b1^t)`` form, ``clip_by_norm``), and is
cross-checked against torch-CPU autograd in ``tests/test_oracle.py``.

Two numeric modes: ``np.float64`` ("truth") and ``np.float32`` ("TF-like": every
tensor op rounded to fp32 the way TF1 CPU would).

Dropout randomness cannot match TF's (its Philox stream is keyed by op seeds
we cannot reproduce), so the oracle and the HIP kernels share one counter-based
Philox4x32-10 stream (``dropout_uniform``) and dropout parity is exact.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------------------
# configuration
# --------------------------------------------------------------------------------------


@dataclass
class Cfg:
    """Constructor arguments of ``LinearModel`` (src/linear_model.py:34-44)."""

    linear_size: int = 1024
    num_layers: int = 2
    residual: bool = True
    batch_norm: bool = True
    max_norm: bool = False
    predict_14: bool = False
    input_size: int = 32           # HUMAN_2D_SIZE, src/linear_model.py:62
    bn_eps: float = 1e-3           # tf.layers.batch_normalization default
    bn_momentum: float = 0.99      # tf.layers.batch_normalization default

    @property
    def output_size(self) -> int:  # HUMAN_3D_SIZE, src/linear_model.py:72
        return 14 * 3 if self.predict_14 else 16 * 3


def param_names(cfg: Cfg):
    """Trainable variables in TF creation order (= ``tf.trainable_variables()``).

    Names follow src/linear_model.py:103-124,171-193 under scope ``linear_model``.
    Yields (name, shape).
    """
    L = cfg.linear_size
    out = [("linear_model/w1", (cfg.input_size, L)), ("linear_model/b1", (L,))]
    if cfg.batch_norm:
        out += [("linear_model/batch_normalization/gamma", (L,)),
                ("linear_model/batch_normalization/beta", (L,))]
    for i in range(cfg.num_layers):
        s = "linear_model/two_linear_%d/" % i
        out += [(s + "w2_%d" % i, (L, L)), (s + "b2_%d" % i, (L,))]
        if cfg.batch_norm:
            out += [(s + "batch_normalization1%d/gamma" % i, (L,)),
                    (s + "batch_normalization1%d/beta" % i, (L,))]
        out += [(s + "w3_%d" % i, (L, L)), (s + "b3_%d" % i, (L,))]
        if cfg.batch_norm:
            out += [(s + "batch_normalization2%d/gamma" % i, (L,)),
                    (s + "batch_normalization2%d/beta" % i, (L,))]
    out += [("linear_model/w4", (L, cfg.output_size)), ("linear_model/b4", (cfg.output_size,))]
    return out


def bn_names(cfg: Cfg):
    """Batch-norm scopes in layer order (input layer, then 1i/2i per block)."""
    if not cfg.batch_norm:
        return []
    out = ["linear_model/batch_normalization"]
    for i in range(cfg.num_layers):
        s = "linear_model/two_linear_%d/" % i
        out += [s + "batch_normalization1%d" % i, s + "batch_normalization2%d" % i]
    return out


# --------------------------------------------------------------------------------------
# initialisation
# --------------------------------------------------------------------------------------


def truncated_normal(rng: np.random.Generator, shape):
    """tf.truncated_normal: N(0,1) re-drawn outside 2 standard deviations."""
    x = rng.standard_normal(shape)
    bad = np.abs(x) > 2.0
    while bad.any():
        x[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(x) > 2.0
    return x


def kaiming(rng: np.random.Generator, shape):
    """src/linear_model.py:17-29 -- truncated_normal(shape)*sqrt(2/shape[0]).

    Used for weights AND biases (a bias's fan is its own length).
    """
    return (truncated_normal(rng, shape) * math.sqrt(2.0 / float(shape[0]))).astype(np.float32)


def init_state(cfg: Cfg, seed: int = 1, bn_seed: int | None = None):
    """Fresh model state: trainables (kaiming), BN moving stats, Adam slots.

    With ``bn_seed`` the BN affine params and moving stats are randomised
    (gamma~U(.5,1.5), beta~N(0,.1), mean~N(0,.1), var~U(.5,2)) so eval-mode
    BN is non-trivial; otherwise TF defaults (1,0,0,1).
    """
    rng = np.random.default_rng(seed)
    params = {}
    for name, shape in param_names(cfg):
        if name.endswith("/gamma"):
            params[name] = np.ones(shape, np.float32)
        elif name.endswith("/beta"):
            params[name] = np.zeros(shape, np.float32)
        else:
            params[name] = kaiming(rng, shape)
    moving = {}
    for s in bn_names(cfg):
        moving[s + "/moving_mean"] = np.zeros(cfg.linear_size, np.float32)
        moving[s + "/moving_variance"] = np.ones(cfg.linear_size, np.float32)
    if bn_seed is not None:
        r2 = np.random.default_rng(bn_seed)
        L = cfg.linear_size
        for s in bn_names(cfg):
            params[s + "/gamma"] = r2.uniform(0.5, 1.5, L).astype(np.float32)
            params[s + "/beta"] = r2.normal(0.0, 0.1, L).astype(np.float32)
            moving[s + "/moving_mean"] = r2.normal(0.0, 0.1, L).astype(np.float32)
            moving[s + "/moving_variance"] = r2.uniform(0.5, 2.0, L).astype(np.float32)
    return State(cfg=cfg, params=params, moving=moving)


@dataclass
class State:
    cfg: Cfg
    params: dict
    moving: dict
    m: dict = field(default_factory=dict)      # Adam slot "m"
    v: dict = field(default_factory=dict)      # Adam slot "v"
    global_step: int = 0
    beta1_power: np.float32 = np.float32(0.9)  # AdamOptimizer._create_slots: starts at beta1
    beta2_power: np.float32 = np.float32(0.999)

    def copy(self):
        return State(cfg=self.cfg,
                     params={k: v.copy() for k, v in self.params.items()},
                     moving={k: v.copy() for k, v in self.moving.items()},
                     m={k: v.copy() for k, v in self.m.items()},
                     v={k: v.copy() for k, v in self.v.items()},
                     global_step=self.global_step,
                     beta1_power=self.beta1_power, beta2_power=self.beta2_power)


# --------------------------------------------------------------------------------------
# Philox4x32-10 dropout stream (shared bit-for-bit with the HIP kernels)
# --------------------------------------------------------------------------------------

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds; all args uint32 arrays/scalars.

    Round: (c0,c1,c2,c3) <- (hi(M1*c2)^c1^k0, lo(M1*c2), hi(M0*c0)^c3^k1, lo(M0*c0));
    the key is bumped by (W0,W1) between rounds.
    """
    c0 = np.asarray(c0, np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, np.uint32).astype(np.uint64)
    k0 = np.uint64(np.uint32(k0))
    k1 = np.uint64(np.uint32(k1))
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(_W0)) & _MASK32
            k1 = (k1 + np.uint64(_W1)) & _MASK32
        p0 = _M0 * c0
        p1 = _M1 * c2
        n0 = ((p1 >> np.uint64(32)) ^ c1 ^ k0) & _MASK32
        n1 = p1 & _MASK32
        n2 = ((p0 >> np.uint64(32)) ^ c3 ^ k1) & _MASK32
        n3 = p0 & _MASK32
        c0, c1, c2, c3 = n0, n1, n2, n3
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32), c3.astype(np.uint32))


def dropout_uniform(seed: int, ctr: int, site: int, row0: int, rows: int, cols: int):
    """U[0,1) fp32 for dropout site ``site`` at call counter ``ctr``.

    Element (global row g, column c) takes word (c & 3) of
    Philox(counter=(g, c>>2, site, ctr), key=(seed_lo, seed_hi)); the fp32 is
    ``float((w & 0x7fffff) | 0x3f800000) - 1`` (TF's uint32->float conversion).
    Keyed by the *global* row so the mask does not depend on how rows are sharded.
    """
    g = (np.arange(rows, dtype=np.uint64) + np.uint64(row0)).astype(np.uint32)[:, None]
    c = np.arange(cols, dtype=np.uint32)[None, :]
    G, C = np.broadcast_arrays(g, c)
    words = philox4x32_10(G, C >> np.uint32(2), np.uint32(site), np.uint32(ctr & 0xFFFFFFFF),
                          np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF))
    sel = (C & np.uint32(3)).astype(np.int64)
    w = np.choose(sel, words)
    bits = (w & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)
    return bits.view(np.float32) - np.float32(1.0)


def dropout_mask(keep: float, u: np.ndarray) -> np.ndarray:
    """tf.nn.dropout (TF1): binary = floor(keep + U), evaluated in fp32."""
    return np.floor(np.float32(keep) + u.astype(np.float32)).astype(np.float32)


# --------------------------------------------------------------------------------------
# forward / backward
# --------------------------------------------------------------------------------------


def _maxnorm_scale(w, dt):
    """clip_by_norm(w, 1): w * 1 / max(||w||_F, 1) (src/linear_model.py:108,123,178,189)."""
    n = np.sqrt(np.sum(w.astype(dt) * w.astype(dt), dtype=dt), dtype=dt)
    return dt(1.0) / max(n, dt(1.0)), n


def _eff_w(state: State, name: str, dt):
    w = state.params[name].astype(dt)
    if state.cfg.max_norm:
        s, _ = _maxnorm_scale(w, dt)
        return (w * dt(1.0)) / max(np.sqrt(np.sum(w * w, dtype=dt), dtype=dt), dt(1.0))
    return w


def _layer_fwd(state, x, wname, bname, bn, training, keep, seed, ctr, site, row0, dt, cache, key):
    """Linear -> (BN) -> relu -> dropout, recording what backward needs."""
    cfg = state.cfg
    w = _eff_w(state, wname, dt)
    z = (x @ w + state.params[bname].astype(dt)).astype(dt)
    rec = {"x": x, "z": z, "wname": wname, "bname": bname, "bn": bn, "site": site}
    if bn is not None:
        gamma = state.params[bn + "/gamma"].astype(dt)
        beta = state.params[bn + "/beta"].astype(dt)
        eps = dt(cfg.bn_eps)
        if training:
            mean = np.mean(z, axis=0, dtype=dt)
            var = np.mean((z - mean) ** 2, axis=0, dtype=dt)   # biased (nn.moments)
        else:
            mean = state.moving[bn + "/moving_mean"].astype(dt)
            var = state.moving[bn + "/moving_variance"].astype(dt)
        rstd = dt(1.0) / np.sqrt(var + eps)
        inv = rstd * gamma
        a = z * inv + (beta - mean * inv)                     # nn.batch_normalization form
        rec.update(mean=mean, var=var, rstd=rstd, inv=inv, gamma=gamma)
    else:
        a = z
    r = np.maximum(a, dt(0.0))
    rec["a"] = a
    if keep < 1.0:
        u = dropout_uniform(seed, ctr, site, row0, x.shape[0], r.shape[1])
        mask = dropout_mask(keep, u).astype(dt)
        y = (r / dt(keep)) * mask
        rec["mask"] = mask
    else:
        y = r
    rec["keep"] = keep
    cache[key] = rec
    return y


def forward(state: State, x, training: bool, keep: float = 1.0, seed: int = 0, ctr: int = 0,
            row0: int = 0, dt=np.float64):
    """Graph of src/linear_model.py:92-128. Returns (outputs, cache).

    ``training`` selects batch statistics in BN (the fed ``isTraining``); ``keep``
    is the fed ``dropout_keep_prob``.  Dropout sites: 0 = input layer,
    1+2i / 2+2i = the two layers of block i.
    """
    cfg = state.cfg
    x = np.asarray(x).astype(np.float32).astype(dt)   # placeholder is float32
    cache = {"order": []}
    bns = bn_names(cfg)
    y = _layer_fwd(state, x, "linear_model/w1", "linear_model/b1", bns[0] if bns else None,
                   training, keep, seed, ctr, 0, row0, dt, cache, "in")
    cache["order"].append("in")
    for i in range(cfg.num_layers):
        s = "linear_model/two_linear_%d/" % i
        xin = y
        h = _layer_fwd(state, xin, s + "w2_%d" % i, s + "b2_%d" % i, bns[1 + 2 * i] if bns else None,
                       training, keep, seed, ctr, 1 + 2 * i, row0, dt, cache, "A%d" % i)
        y2 = _layer_fwd(state, h, s + "w3_%d" % i, s + "b3_%d" % i, bns[2 + 2 * i] if bns else None,
                        training, keep, seed, ctr, 2 + 2 * i, row0, dt, cache, "B%d" % i)
        y = (xin + y2) if cfg.residual else y2
        cache["order"] += ["A%d" % i, "B%d" % i]
    w4 = _eff_w(state, "linear_model/w4", dt)
    out = (y @ w4 + state.params["linear_model/b4"].astype(dt)).astype(dt)
    cache["out"] = {"x": y}
    return out, cache


def mse(out, target, dt=np.float64):
    """src/linear_model.py:129 -- reduce_mean(square(y - t)) and its gradient."""
    t = np.asarray(target).astype(np.float32).astype(dt)
    d = out - t
    n = d.size
    loss = np.mean(d * d, dtype=dt)
    dy = (dt(1.0) / dt(n)) * (d * dt(2.0))
    return loss, dy


def _maxnorm_backward(w, g_eff, dt):
    """d/dw of w/max(||w||,1): g/m - [n>=1] sum(g*w) w / (m^2 n)."""
    n = np.sqrt(np.sum(w * w, dtype=dt), dtype=dt)
    m = max(n, dt(1.0))
    g = g_eff / m
    if n >= 1.0:
        g = g - (np.sum(g_eff * w, dtype=dt) / (m * m * n)) * w
    return g


def backward(state: State, cache, dy, dt=np.float64):
    """Hand-derived gradients of the graph (== tf.gradients of the loss)."""
    cfg = state.cfg
    grads = {}
    P = state.params

    def lin_grads(wname, bname, x, dz):
        w = P[wname].astype(dt)
        weff = _eff_w(state, wname, dt)
        g_eff = x.T @ dz
        grads[wname] = _maxnorm_backward(w, g_eff, dt) if cfg.max_norm else g_eff
        grads[bname] = np.sum(dz, axis=0, dtype=dt)
        return dz @ weff.T

    def layer_bwd(rec, dout):
        g = dout
        if rec["keep"] < 1.0:
            g = (g * rec["mask"]) / dt(rec["keep"])
        g = g * (rec["a"] > 0)
        if rec["bn"] is not None:
            bn = rec["bn"]
            z, mean, rstd = rec["z"], rec["mean"], rec["rstd"]
            xhat = (z - mean) * rstd
            grads[bn + "/gamma"] = np.sum(g * xhat, axis=0, dtype=dt)
            grads[bn + "/beta"] = np.sum(g, axis=0, dtype=dt)
            if rec.get("training", True):
                B = z.shape[0]
                dz = (rec["inv"] / dt(B)) * (dt(B) * g - np.sum(g, axis=0, dtype=dt)
                                             - xhat * np.sum(g * xhat, axis=0, dtype=dt))
            else:
                dz = g * rec["inv"]
        else:
            dz = g
        return lin_grads(rec["wname"], rec["bname"], rec["x"], dz)

    dh = lin_grads("linear_model/w4", "linear_model/b4", cache["out"]["x"], dy)
    for i in reversed(range(cfg.num_layers)):
        dout = dh
        dh_a = layer_bwd(cache["B%d" % i], dout)
        dxin = layer_bwd(cache["A%d" % i], dh_a)
        dh = dxin + dout if cfg.residual else dxin
    layer_bwd(cache["in"], dh)
    return grads


# --------------------------------------------------------------------------------------
# optimizer (TF1 AdamOptimizer + exponential_decay) and BN UPDATE_OPS
# --------------------------------------------------------------------------------------

ADAM_B1, ADAM_B2, ADAM_EPS = 0.9, 0.999, 1e-8
DECAY_STEPS, DECAY_RATE = 100000, 0.96   # src/linear_model.py:88-89


def decayed_lr(lr0: float, global_step: int) -> np.float32:
    """tf.train.exponential_decay(lr, gs, 1e5, 0.96), continuous (src/linear_model.py:90)."""
    p = np.float32(global_step) / np.float32(DECAY_STEPS)
    return np.float32(np.float32(lr0) * np.power(np.float32(DECAY_RATE), p, dtype=np.float32))


def adam_apply(state: State, grads, lr0: float, dt=np.float64):
    """TF1 ApplyAdam on every trainable, then global_step += 1 (src/linear_model.py:137,145).

    alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
    w -= (m*alpha)/(sqrt(v)+eps).
    """
    lr = decayed_lr(lr0, state.global_step)
    b1p, b2p = state.beta1_power, state.beta2_power
    alpha = dt(lr) * np.sqrt(dt(1.0) - dt(b2p)) / (dt(1.0) - dt(b1p))
    for name, _ in param_names(state.cfg):
        g = grads[name].astype(dt)
        m = state.m.get(name, np.zeros_like(g)).astype(dt)
        v = state.v.get(name, np.zeros_like(g)).astype(dt)
        m = m + (g - m) * (dt(1.0) - dt(ADAM_B1))
        v = v + (g * g - v) * (dt(1.0) - dt(ADAM_B2))
        w = state.params[name].astype(dt) - (m * alpha) / (np.sqrt(v) + dt(ADAM_EPS))
        state.m[name], state.v[name] = m.astype(np.float32), v.astype(np.float32)
        state.params[name] = w.astype(np.float32)
    state.beta1_power = np.float32(b1p * np.float32(ADAM_B1))
    state.beta2_power = np.float32(b2p * np.float32(ADAM_B2))
    state.global_step += 1


def bn_update(state: State, cache, dt=np.float64):
    """UPDATE_OPS: moving -= (moving - batch_stat) * (1 - momentum), biased variance."""
    decay = dt(1.0) - dt(np.float32(state.cfg.bn_momentum))
    for key in cache["order"]:
        rec = cache[key]
        bn = rec["bn"]
        if bn is None:
            continue
        mm = state.moving[bn + "/moving_mean"].astype(dt)
        mv = state.moving[bn + "/moving_variance"].astype(dt)
        state.moving[bn + "/moving_mean"] = (mm - (mm - rec["mean"]) * decay).astype(np.float32)
        state.moving[bn + "/moving_variance"] = (mv - (mv - rec["var"]) * decay).astype(np.float32)


def train_step(state: State, x, t, keep: float, lr0: float, seed: int = 0, ctr: int | None = None,
               row0: int = 0, dt=np.float64):
    """``LinearModel.step(isTraining=True)`` (src/linear_model.py:225-237).

    Returns (loss, outputs); mutates ``state``.  ``ctr`` defaults to the global step,
    which is how the HIP path keys its dropout stream.
    """
    if ctr is None:
        ctr = state.global_step
    out, cache = forward(state, x, True, keep, seed, ctr, row0, dt)
    loss, dy = mse(out, t, dt)
    grads = backward(state, cache, dy, dt)
    bn_update(state, cache, dt)
    adam_apply(state, grads, lr0, dt)
    return loss, out


def dp_train_step(replicas, xs, ts, keep: float, lr0: float, seed: int = 0, ctr: int | None = None,
                  dt=np.float64):
    """One data-parallel step of R replicas: replica r
    runs forward + MSE + backward on its own batch xs[r] (dropout rows keyed globally, row0 =
    r * B), the gradients are averaged over the replicas, every replica applies the same TF1
    Adam update; BN statistics and the moving-average UPDATE_OPS stay per replica (no
    SyncBN).  ``replicas`` share trainables and Adam slots on entry; returns the losses."""
    if ctr is None:
        ctr = replicas[0].global_step
    R = len(replicas)
    grads, losses = None, []
    for r, st in enumerate(replicas):
        out, cache = forward(st, xs[r], True, keep, seed, ctr, r * xs[r].shape[0], dt)
        loss, dy = mse(out, ts[r], dt)
        g = backward(st, cache, dy, dt)
        grads = g if grads is None else {k: grads[k] + g[k] for k in grads}
        bn_update(st, cache, dt)
        losses.append(loss)
    grads = {k: v / dt(R) for k, v in grads.items()}
    adam_apply(replicas[0], grads, lr0, dt)
    for st in replicas[1:]:
        st.params.update({k: v.copy() for k, v in replicas[0].params.items()})
        st.m = {k: v.copy() for k, v in replicas[0].m.items()}
        st.v = {k: v.copy() for k, v in replicas[0].v.items()}
        st.global_step = replicas[0].global_step
        st.beta1_power, st.beta2_power = replicas[0].beta1_power, replicas[0].beta2_power
    return losses


def eval_step(state: State, x, t, dt=np.float64):
    """``LinearModel.step(isTraining=False)`` with keep=1 (src/linear_model.py:239-245)."""
    out, _ = forward(state, x, False, 1.0, 0, 0, 0, dt)
    loss, _ = mse(out, t, dt)
    return loss, out


# --------------------------------------------------------------------------------------
# bf16 inference emulation (cfg5: bf16 weights/activations, fp32 accumulate + BN)
# --------------------------------------------------------------------------------------


def bf16_round(a):
    """Round to the nearest bf16 (ties to even), returned as float32."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return r.astype(np.uint32).view(np.float32)


def forward_bf16(state: State, x, acc=np.float64):
    """Inference forward of the bf16 path: x and every weight rounded to bf16, products
    accumulated in ``acc``, epilogue (bias, BN eval, ReLU, residual) in fp32, each hidden
    activation rounded to bf16 when stored; output layer stays fp32."""
    cfg = state.cfg
    P = state.params
    f32 = np.float32

    def layer(a, wname, bname, bn, res=None):
        z = (a.astype(acc) @ bf16_round(P[wname]).astype(acc)).astype(f32) + P[bname]
        if bn is not None:
            inv = (f32(1.0) / np.sqrt(state.moving[bn + "/moving_variance"] + f32(cfg.bn_eps))) * P[bn + "/gamma"]
            z = z * inv + (P[bn + "/beta"] - state.moving[bn + "/moving_mean"] * inv)
        y = np.maximum(z, f32(0.0))
        if res is not None:
            y = y + res
        return bf16_round(y)

    bns = bn_names(cfg)
    h = layer(bf16_round(np.asarray(x, np.float32)), "linear_model/w1", "linear_model/b1", bns[0] if bns else None)
    for i in range(cfg.num_layers):
        s = "linear_model/two_linear_%d/" % i
        xin = h
        a = layer(xin, s + "w2_%d" % i, s + "b2_%d" % i, bns[1 + 2 * i] if bns else None)
        h = layer(a, s + "w3_%d" % i, s + "b3_%d" % i, bns[2 + 2 * i] if bns else None,
                  res=xin if cfg.residual else None)
    out = (h.astype(acc) @ bf16_round(P["linear_model/w4"]).astype(acc)).astype(np.float32) + P["linear_model/b4"]
    return out
