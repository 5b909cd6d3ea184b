"""p3d_serve (k_serve: persistent XCD-local evaluation of batch-64 steps) vs the oracle.

Reference behaviour: predict_3dpose.py:evaluate_batches (:352-444) runs LinearModel.step
(linear_model.py:203-245, isTraining=False, keep_prob 1) once per batch of 64; the rows
of a batch are independent in eval mode, so every output row must equal the oracle's
eval forward of that row.  Tolerance as tests/test_gpu_parity.py: |d| <= 2e-5 + 2e-5|ref|
(fp32 MFMA chain vs the fp64 oracle); vs the batch-64 HIP kernels 5e-5 (the output layer
sums 32-column partials in a different, fixed order).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import linear_model  # noqa: E402
from oracle import ref_mlp  # noqa: E402


def make(cfg, max_batch=64, seed=1, bn_seed=2):
    st = ref_mlp.init_state(cfg, seed=seed, bn_seed=bn_seed)
    m = linear_model.LinearModel(cfg.linear_size, cfg.num_layers, cfg.residual, cfg.batch_norm, cfg.max_norm,
                                 64, 1e-3, "/tmp/p3d_test", cfg.predict_14, seed=11, max_batch=max_batch)
    m.set_weights({**st.params, **st.moving})
    return st, m


def close(a, b, atol=2e-5, rtol=2e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b)
    assert np.all(err <= tol), "max err %.3g (at ref %.3g)" % (err.max(), b.flat[np.argmax(err - tol)])


def test_serve_cfg2_ragged_vs_oracle():
    """cfg2 network, 37 full steps + a 13-row tail: oracle, batch-64 kernels, determinism."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg)
    B = 64 * 37 + 13
    x = np.random.default_rng(3).standard_normal((B, 32)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    y = m.serve_device(xd)
    y2 = m.serve_device(xd)
    torch.cuda.synchronize()
    m.serve_check()
    assert torch.equal(y, y2), "k_serve is not deterministic"
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    close(y.cpu().numpy(), ro)
    y64 = torch.cat([m.forward_device(xd[i:i + 64]) for i in range(0, B, 64)])
    close(y.cpu().numpy(), y64.cpu().numpy(), atol=5e-5, rtol=5e-5)
    m.close()


@pytest.mark.parametrize("L,N,residual,batch_norm,max_norm,p14", [
    (256, 1, True, True, False, False),      # cfg1
    (256, 0, False, True, False, False),     # no blocks: the input layer feeds the output partials
    (256, 3, True, True, True, False),       # max-norm on every weight
    (512, 2, False, False, False, False),    # no BN, no residual
    (1024, 2, True, True, False, True),      # --predict_14: 42 outputs
    (2048, 1, True, True, False, False),     # 64 units per layer: two per workgroup
])
def test_serve_variants_vs_oracle(L, N, residual, batch_norm, max_norm, p14):
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=N, residual=residual, batch_norm=batch_norm, max_norm=max_norm,
                      predict_14=p14)
    st, m = make(cfg)
    B = 64 * 19 + 5
    x = np.random.default_rng(L + N).standard_normal((B, 32)).astype(np.float32)
    y = m.serve_device(torch.from_numpy(x).cuda()).cpu().numpy()
    m.serve_check()
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    assert y.shape == ro.shape
    close(y, ro, atol=5e-5, rtol=5e-5)
    m.close()


def test_serve_small_batches():
    """Fewer steps than XCD groups (most groups idle), single rows."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg)
    for B in (1, 7, 64, 65, 300):
        x = np.random.default_rng(B).standard_normal((B, 32)).astype(np.float32)
        y = m.serve_device(torch.from_numpy(x).cuda()).cpu().numpy()
        ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
        close(y, ro)
    m.serve_check()
    m.close()


def test_serve_many_steps_every_row():
    """2,000 steps (~250 per XCD group, ten thousand group barriers) with distinct rows:
    every output row vs the large-M HIP path.  A stale hand-off (a layer reading an L1
    line or a partial from an earlier step) would show up as a wrong row."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg, max_batch=8192)
    B = 64 * 2000
    xd = torch.randn((B, 32), device="cuda", generator=torch.Generator("cuda").manual_seed(5))
    y = m.serve_device(xd)
    ref = torch.cat([m.forward_device(xd[i:i + 8192]) for i in range(0, B, 8192)])
    torch.cuda.synchronize()
    m.serve_check()
    d = (y - ref).abs()
    tol = 5e-5 + 5e-5 * ref.abs()
    assert bool((d <= tol).all()), "max err %.3g" % float(d.max())
    # and a sample of rows vs the fp64 oracle
    idx = np.random.default_rng(0).choice(B, 512, replace=False)
    ro, _ = ref_mlp.forward(st, xd[idx].cpu().numpy(), False, 1.0, 0, 0, 0)
    close(y[idx].cpu().numpy(), ro)
    m.close()


def test_serve_rejects_bad_shapes():
    cfg = ref_mlp.Cfg(linear_size=256, num_layers=1, residual=True, batch_norm=True)
    st, m = make(cfg)
    with pytest.raises(ValueError):
        m.serve_device(torch.zeros((64, 31), device="cuda"))
    m.close()


@pytest.mark.parametrize("L,N", [(1024, 2), (256, 1), (2048, 1), (384, 1)])
def test_serve5_vs_oracle(L, N):
    """k_serve5 (launches of more than 32 steps) gives the oracle's outputs: groups with fewer
    members than units per contraction (L = 256), several contractions per phase (L = 2048), the
    2-deep ring (L = 384: six k-groups per wave).  (Round 6 removed the group-count, pairing and
    ring-depth knob forms that measured slower)"""
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=N, residual=True, batch_norm=True)
    st, m = make(cfg)
    B = 64 * 300 + 13
    x = np.random.default_rng(L + N).standard_normal((B, 32)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    y = m.serve_device(xd)
    torch.cuda.synchronize()
    m.serve_check()
    idx = np.r_[0:64, np.random.default_rng(1).choice(B, 448, replace=False), B - 13:B]
    ro, _ = ref_mlp.forward(st, x[idx], False, 1.0, 0, 0, 0)
    close(y.cpu().numpy()[idx], ro)
    m.close()


def _serve6_model(monkeypatch, cfg, split=None, mode=None, seed=1, rt=None, pair=None):
    if split is not None:
        monkeypatch.setenv("P3D_SERVE6_SPLIT", str(split))
    if mode is not None:
        monkeypatch.setenv("P3D_SERVE6", str(mode))
    if rt is not None:
        monkeypatch.setenv("P3D_SERVE6_RT", str(rt))
    if pair is not None:
        monkeypatch.setenv("P3D_SERVE6_PAIR", str(pair))
    st, m = make(cfg, seed=seed)
    for k in ("P3D_SERVE6_SPLIT", "P3D_SERVE6", "P3D_SERVE6_RT", "P3D_SERVE6_PAIR"):
        monkeypatch.delenv(k, raising=False)
    return st, m


def test_serve6_every_split_same_bits_and_oracle(monkeypatch):
    """k_serve6 (launches of <= 32 steps; the driver's 20-step headline): 1-4 groups per XCD of
    batch-64 units (16-column tiles dealt contiguously, 7 tiles per CU at 3 groups) and 32-row
    half-step units at 5 (and 3) groups per XCD, and XCD-wide units of 6 / 8 / 16 row tiles give
    the same bits -- the association of every sum is fixed by the tile, not by the group or unit
    shape -- and the oracle's outputs; the auto choice for 20 steps is 160 rows per XCD on all 32
    of its CUs, 2 column tiles each: one unit, or (the pair form, P3D_SERVE6_PAIR) two 80-row units
    with alternating phases -- both forms run here, the same bits."""
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    B = 64 * 20
    x = np.random.default_rng(620).standard_normal((B, 32)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    outs = {}
    for split, rt in ((None, None), (1, 4), (2, 4), (3, 4), (4, 4), (5, 2), (3, 2), (1, 6), (1, 8), (1, 16),
                      ("pair0", None), ("pair1", None)):
        if isinstance(split, str):
            st, m = _serve6_model(monkeypatch, cfg, pair=int(split[-1]))
        else:
            st, m = _serve6_model(monkeypatch, cfg, split, rt=rt)
        y = m.serve_device(xd)
        torch.cuda.synchronize()
        m.serve_check()
        name = _p3d.ctypes.create_string_buffer(128)
        _p3d.check(_p3d.lib().p3d_kernel_name(m._h, 3, name, 128), "p3d_kernel_name")
        assert name.value.decode().startswith("k_serve6<"), name.value
        outs[(split, rt)] = (y, name.value.decode())
        m.close()
    auto = outs[(None, None)]
    # 20 steps -> 160 rows per XCD: one unit, or two of 80 side by side (the pair form)
    assert outs[("pair0", None)][1] == "k_serve6<4, 3, 2, 10>", outs[("pair0", None)][1]
    assert outs[("pair1", None)][1] == "k_serve6<4, 3, 2, 5, true>", outs[("pair1", None)][1]
    assert auto[1] in ("k_serve6<4, 3, 2, 10>", "k_serve6<4, 3, 2, 5, true>"), auto[1]
    assert outs[(3, 4)][1] == "k_serve6<2, 3, 7, 4>", outs[(3, 4)][1]
    for key, (y, _) in outs.items():
        assert torch.equal(y, auto[0]), key
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    close(auto[0].cpu().numpy(), ro)


@pytest.mark.parametrize("B", [1, 13, 64, 64 * 5 + 7, 64 * 8, 64 * 16, 64 * 24 + 1, 64 * 32])
def test_serve6_launch_sizes_vs_oracle(B):
    """Every launch size k_serve6 takes (<= 32 steps; the split chosen per launch), ragged
    tails, against the oracle; and equal bits whatever the launch size (same rows)."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg)
    x = np.random.default_rng(B).standard_normal((B, 32)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    y = m.serve_device(xd)
    m.serve_check()
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    close(y.cpu().numpy(), ro)
    if B >= 64:   # the first step alone as its own launch: same bits
        assert torch.equal(m.serve_device(xd[:64]), y[:64])
    m.close()


@pytest.mark.parametrize("L,N,residual,batch_norm,max_norm,p14", [
    (256, 1, True, True, False, False),      # cfg1: 16 tiles, idle members at 1-2 groups per XCD
    (512, 3, True, True, True, False),       # max-norm, three blocks
    (1024, 2, False, False, False, False),   # no BN, no residual
    (1024, 2, True, True, False, True),      # --predict_14
    (2048, 1, True, True, False, False),     # 128 tiles: 13 per CU at 3 groups -> two contractions
])
@pytest.mark.parametrize("split,rt,pair", [(None, None, None), (3, 4, None), (5, 2, None), (1, 10, 0), (1, 10, 1)])
def test_serve6_variants_vs_oracle(monkeypatch, L, N, residual, batch_norm, max_norm, p14, split, rt, pair):
    """(rt 10 with pair 1: the pair form where the width allows it (L >= 768), 17 units of 80 rows --
    a group runs two pairs, the last unit's partner past the last row)"""
    cfg = ref_mlp.Cfg(linear_size=L, num_layers=N, residual=residual, batch_norm=batch_norm, max_norm=max_norm,
                      predict_14=p14)
    st, m = _serve6_model(monkeypatch, cfg, split, rt=rt, pair=pair)
    B = 64 * 20 + 5
    x = np.random.default_rng(L + N).standard_normal((B, 32)).astype(np.float32)
    y = m.serve_device(torch.from_numpy(x).cuda()).cpu().numpy()
    m.serve_check()
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    close(y, ro, atol=5e-5, rtol=5e-5)
    m.close()


@pytest.mark.parametrize("split,rt,pair", [(1, 4, None), (2, 4, None), (3, 4, None), (5, 2, None), (1, 10, 0),
                                           (1, 10, 1)])
def test_serve6_many_steps_per_group(monkeypatch, split, rt, pair):
    """k_serve6 forced on a long launch (P3D_SERVE6=2): every group runs many steps, so the
    next step's input layer rides in the last phase and each step's output layer runs as its own
    phase after that hand-off (tiles dealt over the members); every row vs the oracle / k_serve5."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    B = 64 * 300 + 9
    x = np.random.default_rng(77 + split).standard_normal((B, 32)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    st, m6 = _serve6_model(monkeypatch, cfg, split, mode=2, rt=rt, pair=pair)
    y6 = m6.serve_device(xd)
    torch.cuda.synchronize()
    m6.serve_check()
    _, m5 = _serve6_model(monkeypatch, cfg, mode=0)
    y5 = m5.serve_device(xd)
    torch.cuda.synchronize()
    m5.serve_check()
    close(y6.cpu().numpy(), y5.cpu().numpy(), atol=5e-5, rtol=5e-5)
    idx = np.r_[0:64, np.random.default_rng(2).choice(B, 448, replace=False), B - 9:B]
    ro, _ = ref_mlp.forward(st, x[idx], False, 1.0, 0, 0, 0)
    close(y6.cpu().numpy()[idx], ro)
    # the same rows as a 20-step launch: same bits
    assert torch.equal(m6.serve_device(xd[:64 * 20]), y6[:64 * 20])
    m6.close()
    m5.close()


def test_serve6_constants_follow_parameter_updates():
    """k_serve6 reads its epilogue constants (bias, BN inv / shift, max-norm divisors) from a
    table formed once per parameter version: after a training step (new weights, new moving
    statistics) and after set_weights, the next serve launch agrees with the eval forward of
    the updated model, not with the stale table."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True, max_norm=True)
    st, m = make(cfg, max_batch=64 * 20)
    rng = np.random.default_rng(31)
    xd = torch.from_numpy(rng.standard_normal((64 * 20, 32)).astype(np.float32)).cuda()
    y0 = m.serve_device(xd).clone()
    m.step(None, rng.standard_normal((64, 32)), rng.standard_normal((64, 48)), 0.5, isTraining=True)
    y1 = m.serve_device(xd).clone()
    m.serve_check()
    assert not torch.equal(y0, y1)
    close(y1.cpu().numpy(), m.forward_device(xd, False, 1.0).cpu().numpy(), atol=5e-5, rtol=5e-5)
    # a second step() replays the cached training graph (no host code of the library runs
    # for it; p3d_params_changed marks the table stale)
    m.step(None, rng.standard_normal((64, 32)), rng.standard_normal((64, 48)), 0.5, isTraining=True)
    y1b = m.serve_device(xd).clone()
    m.serve_check()
    assert not torch.equal(y1, y1b)
    close(y1b.cpu().numpy(), m.forward_device(xd, False, 1.0).cpu().numpy(), atol=5e-5, rtol=5e-5)
    st2 = ref_mlp.init_state(cfg, seed=9, bn_seed=10)
    m.set_weights({**st2.params, **st2.moving})
    y2 = m.serve_device(xd)
    m.serve_check()
    ro, _ = ref_mlp.forward(st2, xd.cpu().numpy(), False, 1.0, 0, 0, 0)
    close(y2.cpu().numpy(), ro)
    m.close()


def test_serve_census_failure_reports_and_fills_nan(monkeypatch):
    """A launch whose census cannot complete (test hook P3D_SERVE_TEST_FAULT: the census waits
    for one workgroup more than the grid) ends within its bounded spin, fills its rows with
    NaN (never unwritten or stale rows), sets the pinned error word (read without a device
    round trip, LinearModel.check_errors), and p3d_serve refuses further launches until the
    error is collected; serve_check reports it once (P3D_ERR_HIP)."""
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=256, num_layers=1, residual=True, batch_norm=True)
    monkeypatch.setenv("P3D_SERVE_TEST_FAULT", "1")
    st, m = make(cfg)
    monkeypatch.delenv("P3D_SERVE_TEST_FAULT")
    x = torch.randn((64 * 5 + 3, 32), device="cuda")
    y = torch.zeros((x.shape[0], 48), device="cuda")
    m.serve_device(x, out=y)
    torch.cuda.synchronize()
    assert bool(torch.isnan(y).all()), "failed launch left non-NaN rows"
    with pytest.raises(_p3d.P3DError, match="earlier launch failed"):
        m.serve_device(x, out=y)                      # refused: nobody collected the error
    with pytest.raises(_p3d.P3DError, match="synchronisation timed out"):
        m.serve_check()
    m.serve_check()                                   # reported once
    # the pinned-word path (no device round trip): the next failure surfaces in check_errors
    m.serve_device(x, out=y)
    torch.cuda.synchronize()
    with pytest.raises(_p3d.P3DError, match="p3d_serve launch failed"):
        m.check_errors()
    m.check_errors()                                  # cleared
    m.close()
    # a healthy model on the same device is unaffected
    st2, m2 = make(cfg)
    x2 = np.random.default_rng(9).standard_normal((64 * 3, 32)).astype(np.float32)
    y2 = m2.serve_device(torch.from_numpy(x2).cuda()).cpu().numpy()
    m2.serve_check()
    ro, _ = ref_mlp.forward(st2, x2, False, 1.0, 0, 0, 0)
    close(y2, ro)
    m2.close()


def test_serve_graph_replay_follows_inputs_and_parameters():
    """p3d_serve captured in a HIP graph (advisor r2: the sync-word bank was picked on the host
    and the epilogue constants formed at capture time): every replay alternates the banks on
    the device and re-forms the constants, so replays with new inputs and new parameters equal
    the eager batch-64 kernels."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg)
    B = 64 * 20
    x = torch.zeros((B, 32), device="cuda")
    y = torch.zeros((B, 48), device="cuda")
    m.serve_device(x, out=y)                          # warm-up (tables, buffers)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        m.serve_device(x, out=y)
    rng = np.random.default_rng(21)
    for rep in range(6):
        x.copy_(torch.from_numpy(rng.standard_normal((B, 32)).astype(np.float32)))
        if rep == 3:      # new parameters between replays (as a training graph would change them)
            st2 = ref_mlp.init_state(cfg, seed=31, bn_seed=32)
            m.set_weights({**st2.params, **st2.moving})
            st = st2
        g.replay()
        torch.cuda.synchronize()
        ref = torch.cat([m.forward_device(x[i:i + 64]) for i in range(0, B, 64)])
        torch.cuda.synchronize()
        d = (y - ref).abs()
        assert bool((d <= 5e-5 + 5e-5 * ref.abs()).all()), (rep, float(d.max()))
    m.serve_check()
    ro, _ = ref_mlp.forward(st, x.cpu().numpy(), False, 1.0, 0, 0, 0)
    close(y.cpu().numpy(), ro)
    del g
    m.close()


@pytest.mark.parametrize("xcc", [0, 3, 7])
def test_serve6_late_xcd_group_keeps_launch_epochs(monkeypatch, xcc):
    """Advisor r3 (high): k_serve6 picks its sync-word bank from a device epoch word.  Round 3
    advanced the epoch at the end of workgroup 0's work, so a whole XCD group that started after
    workgroup 0 had finished (possible with max_groups = 1: workgroup 0 often idles) read the next
    epoch, ran on the other bank and left its flags there -- the NEXT launch's hand-offs then passed
    on stale flags.  Now every group slot has its own epoch word, read by each member at its start
    and advanced by the group's rank-0 member at the end of its work (by then every member has read
    it: rank 0's waves waited for a flag of every member, posted after that read).  Test hook
    P3D_SERVE_TEST_DELAY=n,xcc: on every other call all workgroups of XCD xcc start ~n x 3.4 us
    late; the launches alternate delayed / on time and every output must equal an undelayed
    model's bits."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    monkeypatch.setenv("P3D_SERVE_TEST_DELAY", "300,%d" % xcc)
    monkeypatch.setenv("P3D_SERVE_GROUPS", "1")
    st, m = make(cfg)
    monkeypatch.delenv("P3D_SERVE_TEST_DELAY")
    monkeypatch.delenv("P3D_SERVE_GROUPS")
    _, ref = make(cfg)
    rng = np.random.default_rng(40 + xcc)
    B = 64 * 20
    for call in range(6):
        x = torch.from_numpy(rng.standard_normal((B, 32)).astype(np.float32)).cuda()
        y = m.serve_device(x)
        y0 = ref.serve_device(x)
        torch.cuda.synchronize()
        m.serve_check()
        assert torch.equal(y, y0), "launch %d (delayed=%s) differs" % (call, call % 2 == 0)
    ro, _ = ref_mlp.forward(st, x.cpu().numpy(), False, 1.0, 0, 0, 0)
    close(y.cpu().numpy(), ro)
    m.close()
    ref.close()


@pytest.mark.parametrize("B,max_norm,p14", [(64, False, False), (37, False, False), (1280, False, False),
                                            (200, True, False), (64, False, True)])
def test_serve_mse_fused_loss_and_pinned_io(B, max_norm, p14):
    """p3d_serve_mse (round 6): the eval loss fused into k_serve6's output phase, x / t / y / loss
    in pinned host memory read and written by the kernel itself.  y equals p3d_serve's on device
    buffers bit for bit; the loss equals mean((y - t)^2) of the oracle within 1e-5 relative (the
    reference's eval loss, src/linear_model.py:129); repeated launches give the same bits (the
    arrival counter resets itself)."""
    import ctypes
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True, max_norm=max_norm,
                      predict_14=p14)
    st, m = make(cfg)
    D = cfg.output_size
    rng = np.random.default_rng(B + 3)
    x = rng.standard_normal((B, 32)).astype(np.float32)
    t = rng.standard_normal((B, D)).astype(np.float32)
    hx = torch.from_numpy(x).pin_memory()
    ht = torch.from_numpy(t).pin_memory()
    hy = torch.empty((B, D), dtype=torch.float32).pin_memory()
    hl = torch.zeros(4, dtype=torch.float32).pin_memory()
    c = ctypes.c_void_p
    outs, losses = [], []
    for _ in range(3):
        hy.zero_()
        _p3d.check(_p3d.lib().p3d_serve_mse(m._h, c(hx.data_ptr()), B, c(hy.data_ptr()), c(ht.data_ptr()),
                                             c(hl.data_ptr()), c(_p3d.stream_handle())), "p3d_serve_mse")
        torch.cuda.synchronize()
        outs.append(hy.numpy().copy())
        losses.append(float(hl[0]))
    m.serve_check()
    ydev = m.serve_device(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_array_equal(outs[0], ydev)
    assert all(np.array_equal(o, outs[0]) for o in outs) and len(set(losses)) == 1
    ro, _ = ref_mlp.forward(st, x, False, 1.0, 0, 0, 0)
    close(outs[0], ro)
    rl = float(np.mean((ro - t.astype(np.float64)) ** 2))
    assert abs(losses[0] - rl) <= 1e-5 * max(1.0, rl), (losses[0], rl)
    m.close()


def test_step_eval_one_launch_path_and_fallback():
    """LinearModel.step(isTraining=False) from numpy: B <= 2048 runs ONE p3d_serve_mse launch on
    pinned buffers (B = 3: the batch <= 4 chain with its fused loss); B = 2100 (> 32 batch-64 steps:
    no k_serve6 form, the library answers P3D_ERR_ARG once) takes the cached-graph path.  Every path
    equals the oracle's eval step (outputs 2e-5, loss 1e-5 relative)."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg, max_batch=4096)
    for B, one_launch in ((64, True), (300, True), (3, True), (2100, False)):
        rng = np.random.default_rng(B)
        x, t = rng.standard_normal((B, 32)), rng.standard_normal((B, 48))
        for _ in range(2):
            loss, _, out = m.step(None, x, t, 1.0, isTraining=False)
        assert (m._serve_steps.get(B) is not None) == one_launch, B
        rl, ro = ref_mlp.eval_step(st, x, t)
        close(out, ro)
        assert abs(loss - rl) <= 1e-5 * max(1.0, abs(rl)), (B, loss, rl)
    m.close()


@pytest.mark.parametrize("B", [64, 37, 300, 1280, 1, 4])
def test_serve_mse_sync_returns_with_results_in_host_memory(B):
    """p3d_serve_mse_sync (round 6): returns once y and the loss are in the pinned buffers -- the
    launch's last output tile stores a completion word the host waits on (B = 1280: the pair form,
    which carries no word, waits on the stream instead; B = 1, 4: the batch <= 4 chain, whose last
    output workgroup reduces the loss before it stores the word).  Read straight after the call, with no
    synchronize, 12 calls on fresh inputs each equal p3d_serve_mse's results on the same inputs
    (stream-synchronised) bit for bit -- a result of the previous call would show as a mismatch."""
    import ctypes
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg, max_batch=max(B, 64))
    c = ctypes.c_void_p
    hx = torch.empty((B, 32), dtype=torch.float32).pin_memory()
    ht = torch.empty((B, 48), dtype=torch.float32).pin_memory()
    hy = torch.empty((B, 48), dtype=torch.float32).pin_memory()
    hl = torch.zeros(4, dtype=torch.float32).pin_memory()
    ry = torch.empty((B, 48), dtype=torch.float32).pin_memory()
    rl = torch.zeros(4, dtype=torch.float32).pin_memory()
    rng = np.random.default_rng(B + 17)
    lib = _p3d.lib()
    for it in range(12):
        hx.copy_(torch.from_numpy(rng.standard_normal((B, 32)).astype(np.float32)))
        ht.copy_(torch.from_numpy(rng.standard_normal((B, 48)).astype(np.float32)))
        _p3d.check(lib.p3d_serve_mse_sync(m._h, c(hx.data_ptr()), B, c(hy.data_ptr()), c(ht.data_ptr()),
                                          c(hl.data_ptr()), c(_p3d.stream_handle())), "p3d_serve_mse_sync")
        got_y, got_l = hy.numpy().copy(), float(hl[0])
        _p3d.check(lib.p3d_serve_mse(m._h, c(hx.data_ptr()), B, c(ry.data_ptr()), c(ht.data_ptr()),
                                     c(rl.data_ptr()), c(_p3d.stream_handle())), "p3d_serve_mse")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got_y, ry.numpy(), err_msg="call %d" % it)
        assert got_l == float(rl[0]), (it, got_l, float(rl[0]))
    m.serve_check()
    m.check_errors()
    ro, _ = ref_mlp.forward(st, hx.numpy().astype(np.float64), False, 1.0, 0, 0, 0)
    close(hy.numpy(), ro)
    m.close()


@pytest.mark.parametrize("knob", ["P3D_GEMV_CHAIN", "P3D_GEMV_MAXB"])
def test_serve_mse_small_batch_without_the_chain(knob, monkeypatch):
    """p3d_serve_mse(_sync) at B = 3 on a model without the batch <= 4 chain (P3D_GEMV_CHAIN=0: the
    forward's fold form, which carries no fused loss; P3D_GEMV_MAXB=0: no small-batch forms) falls
    through to k_serve6: one launch still, y equals p3d_serve's bit for bit, y and the loss match the
    oracle's eval step, and the sync call's results are in host memory when it returns."""
    import ctypes
    import _p3d
    monkeypatch.setenv(knob, "0")
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st, m = make(cfg)
    B, c, lib = 3, ctypes.c_void_p, _p3d.lib()
    rng = np.random.default_rng(29)
    hx = torch.from_numpy(rng.standard_normal((B, 32)).astype(np.float32)).pin_memory()
    ht = torch.from_numpy(rng.standard_normal((B, 48)).astype(np.float32)).pin_memory()
    hy = torch.empty((B, 48), dtype=torch.float32).pin_memory()
    hl = torch.zeros(4, dtype=torch.float32).pin_memory()
    _p3d.check(lib.p3d_serve_mse_sync(m._h, c(hx.data_ptr()), B, c(hy.data_ptr()), c(ht.data_ptr()),
                                      c(hl.data_ptr()), c(_p3d.stream_handle())), "p3d_serve_mse_sync")
    got_y, got_l = hy.numpy().copy(), float(hl[0])
    torch.cuda.synchronize()
    m.serve_check()
    np.testing.assert_array_equal(got_y, m.serve_device(hx.cuda()).cpu().numpy())
    rl, ro = ref_mlp.eval_step(st, hx.numpy().astype(np.float64), ht.numpy().astype(np.float64))
    close(got_y, ro)
    assert abs(got_l - rl) <= 1e-5 * max(1.0, abs(rl)), (got_l, rl)
    m.close()


@pytest.mark.parametrize("B,p14,max_norm", [(1, False, False), (3, False, False), (4, True, False),
                                            (2, False, True)])
def test_serve_mse_small_batch_is_forward_and_mse(B, p14, max_norm):
    """p3d_serve_mse at B <= 4 (round 6): the persistent small-batch forward with the loss reduced by
    its last output workgroup in k_mse's order.  y equals p3d_forward's at that batch and the loss
    equals p3d_mse's on that y, bit for bit, over 6 calls on fresh pinned inputs, and both match the
    oracle's eval step (src/linear_model.py:129)."""
    import ctypes
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True, max_norm=max_norm,
                      predict_14=p14)
    st, m = make(cfg)
    D = cfg.output_size
    c = ctypes.c_void_p
    lib = _p3d.lib()
    hx = torch.empty((B, 32), dtype=torch.float32).pin_memory()
    ht = torch.empty((B, D), dtype=torch.float32).pin_memory()
    hy = torch.empty((B, D), dtype=torch.float32).pin_memory()
    hl = torch.zeros(4, dtype=torch.float32).pin_memory()
    dl = torch.zeros(4, dtype=torch.float32, device="cuda")
    rng = np.random.default_rng(B + 91)
    for it in range(6):
        hx.copy_(torch.from_numpy(rng.standard_normal((B, 32)).astype(np.float32)))
        ht.copy_(torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)))
        _p3d.check(lib.p3d_serve_mse(m._h, c(hx.data_ptr()), B, c(hy.data_ptr()), c(ht.data_ptr()),
                                     c(hl.data_ptr()), c(_p3d.stream_handle())), "p3d_serve_mse")
        torch.cuda.synchronize()
        yd = m.forward_device(hx.cuda())
        td = ht.cuda()
        _p3d.check(lib.p3d_mse(c(yd.data_ptr()), c(td.data_ptr()), B, D, c(dl.data_ptr()), None,
                               c(_p3d.stream_handle())), "p3d_mse")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(hy.numpy(), yd.cpu().numpy(), err_msg="call %d" % it)
        assert float(hl[0]) == float(dl[0].cpu()), (it, float(hl[0]), float(dl[0].cpu()))
    m.check_errors()
    rl, ro = ref_mlp.eval_step(st, hx.numpy().astype(np.float64), ht.numpy().astype(np.float64))
    close(hy.numpy(), ro)
    assert abs(float(hl[0]) - rl) <= 1e-5 * max(1.0, abs(rl)), (float(hl[0]), rl)
    m.close()


@pytest.mark.parametrize("B", [64, 3, 2100])
def test_step_eval_host_wait_equals_stream_sync(monkeypatch, B):
    """LinearModel.step(isTraining=False) through the host-wait forms (default) and through the
    stream-synchronised ones (P3D_HOST_WAIT=0): B = 64 and B = 3 (the batch <= 4 chain with its
    fused loss) are one p3d_serve_mse_sync call vs p3d_serve_mse + a synchronize; B = 2100 (no
    one-launch form) is the captured forward + MSE whose last node is p3d_host_signal, reading x / t
    from pinned memory and writing y / the loss into coherent host memory, vs the copy-node graph +
    a synchronize.  10 steps on fresh inputs, the same outputs and loss bit for bit, step by step,
    and the oracle's eval step."""
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    res = {}
    for hw in ("1", "0"):
        monkeypatch.setenv("P3D_HOST_WAIT", hw)
        st, m = make(cfg, max_batch=max(B, 64))
        rng = np.random.default_rng(77)
        xs = [(rng.standard_normal((B, 32)), rng.standard_normal((B, 48))) for _ in range(10)]
        res[hw] = [m.step(None, x, t, 1.0, isTraining=False) for x, t in xs]
        if B <= 2048:
            assert m._serve_steps[B]["sync"] == (hw == "0")
        else:
            assert bool(m._host_steps[(False, B, 1.0, m.lr0, m.seed)].get("signal")) == (hw == "1")
        m.close()
    for (la, _, ya), (lb, _, yb) in zip(res["1"], res["0"]):
        assert la == lb
        np.testing.assert_array_equal(ya, yb)
    rl, ro = ref_mlp.eval_step(st, xs[-1][0], xs[-1][1])
    close(res["1"][-1][2], ro)
    assert abs(res["1"][-1][0] - rl) <= 1e-5 * max(1.0, abs(rl))


def test_step_eval_reports_a_failed_launch(monkeypatch):
    """The eval step's one launch (p3d_serve_mse_sync) on a model whose serve launches fail their
    placement (test hook P3D_SERVE_TEST_FAULT): step() raises -- the sync call reads the kernels'
    error words after its wait and fails, and the host names the failure -- instead of returning
    the launch's NaN rows as a result."""
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=256, num_layers=1, residual=True, batch_norm=True)
    monkeypatch.setenv("P3D_SERVE_TEST_FAULT", "1")
    st, m = make(cfg)
    monkeypatch.delenv("P3D_SERVE_TEST_FAULT")
    rng = np.random.default_rng(4)
    x, t = rng.standard_normal((64, 32)), rng.standard_normal((64, 48))
    with pytest.raises(_p3d.P3DError):
        m.step(None, x, t, 1.0, isTraining=False)
    torch.cuda.synchronize()
    m.close()


def test_host_wait_reports_instead_of_spinning():
    """p3d_host_wait / the *_sync calls never spin on a word nothing will store: waiting for a
    signal count no launch was issued for returns P3D_ERR_HIP once the stream reports idle; a
    signal then a wait for its count returns at once; p3d_serve_mse_sync on a capturing stream is
    refused (P3D_ERR_STATE) before anything is launched."""
    import ctypes
    import _p3d
    cfg = ref_mlp.Cfg(linear_size=256, num_layers=1, residual=True, batch_norm=True)
    st, m = make(cfg)
    lib = _p3d.lib()
    sh = ctypes.c_void_p(_p3d.stream_handle())
    torch.cuda.synchronize()
    rc = lib.p3d_host_wait(m._h, (m._hsig + 5) & 0xffffffff, sh)
    assert rc == 2 and b"without storing" in lib.p3d_last_error()
    _p3d.check(lib.p3d_host_signal(m._h, sh), "p3d_host_signal")
    m._hsig = (m._hsig + 1) & 0xffffffff
    _p3d.check(lib.p3d_host_wait(m._h, m._hsig, sh), "p3d_host_wait")
    # refused inside a capture, nothing launched (the capture then ends empty)
    hx = torch.zeros((64, 32)).pin_memory()
    ht = torch.zeros((64, 48)).pin_memory()
    hy = torch.empty((64, 48)).pin_memory()
    hl = torch.zeros(4).pin_memory()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rc = lib.p3d_serve_mse_sync(m._h, ctypes.c_void_p(hx.data_ptr()), 64, ctypes.c_void_p(hy.data_ptr()),
                                    ctypes.c_void_p(ht.data_ptr()), ctypes.c_void_p(hl.data_ptr()),
                                    ctypes.c_void_p(_p3d.stream_handle()))
    assert rc == 3, rc
    torch.cuda.synchronize()
    m.check_errors()
    m.close()
