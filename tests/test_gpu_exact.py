"""Bit-exact parity of the inference paths against the oracle at full size (tests/exact_models.py:
integer-valued models, for which float32 and the bf16 emulation are exact whatever the summation
order).  Every launch form the library picks for a batch size is covered: the persistent forms of
p3d_serve (k_serve6: the 20-request headline's pair form, a lone batch-64 request, ragged row
counts; k_serve5: long launches), the per-layer kernel chain (k_fwd), the batch <= 4 persistent
GEMV chain (k_gemv_chain), the large-M GEMM (k_gemm_f32) and the cfg5 bf16 GEMMs (k_gemm_bf16p)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import exact_models  # noqa: E402
import linear_model  # noqa: E402
from oracle import ref_mlp  # noqa: E402


def _model(cfg, st, max_batch, dtype=None):
    kw = {"dtype": dtype} if dtype else {}
    m = linear_model.LinearModel(cfg.linear_size, cfg.num_layers, cfg.residual, cfg.batch_norm, False, 64, 1e-3,
                                 "/tmp/p3d_exact", cfg.predict_14, seed=3, max_batch=max_batch, **kw)
    m.set_weights({**st.params, **st.moving})
    return m


@pytest.fixture(scope="module")
def cfg2():
    cfg, st = exact_models.integer_state(1024, 2, nnz=8)
    return cfg, st


@pytest.mark.parametrize("B", [1280, 1217, 64, 37, 64 * 300 + 13])
def test_serve_bit_exact(cfg2, B):
    """p3d_serve (1280 rows = the driver's 20-request launch: k_serve6's pair form; 1217 ragged;
    64 = one request; 37; 19,213 rows = k_serve5) == the oracle, bit for bit."""
    cfg, st = cfg2
    x = exact_models.integer_inputs(B, seed=B)
    ref = exact_models.exact_forward(st, x)
    m = _model(cfg, st, max_batch=64)
    y = m.serve_device(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    m.serve_check()
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    m.close()


@pytest.mark.parametrize("B", [1, 3, 4, 37, 64, 300, 4096])
def test_forward_bit_exact(cfg2, B):
    """forward_device (B <= 4: k_gemv_chain; B <= 64: the per-layer k_fwd chain; B >= 256: the
    large-M k_gemm_f32) == the oracle, bit for bit."""
    cfg, st = cfg2
    x = exact_models.integer_inputs(B, seed=100 + B)
    ref = exact_models.exact_forward(st, x)
    m = _model(cfg, st, max_batch=max(B, 64))
    y = m.forward_device(torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    m.close()


@pytest.mark.parametrize("residual,batch_norm,p14", [(False, True, False), (True, False, False), (True, True, True)])
def test_flag_variants_bit_exact(residual, batch_norm, p14):
    """Flag combinations (no residual, no BN, --predict_14's 42 outputs) through p3d_serve and the
    kernel chain, bit for bit."""
    cfg, st = exact_models.integer_state(1024, 2, nnz=8, residual=residual, batch_norm=batch_norm, predict_14=p14)
    x = exact_models.integer_inputs(1280, seed=9)
    ref = exact_models.exact_forward(st, x)
    m = _model(cfg, st, max_batch=64)
    if cfg.output_size == 48:   # (p3d_serve's persistent forms are built for 48 outputs)
        y = m.serve_device(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
        m.serve_check()
        np.testing.assert_array_equal(y.cpu().numpy(), ref)
    y = torch.cat([m.forward_device(torch.from_numpy(x[i:i + 64]).cuda()) for i in range(0, 1280, 64)])
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    m.close()


@pytest.mark.parametrize("L,N,B,nnz", [(4096, 4, 1024, 4), (1024, 2, 256, 8), (512, 1, 200, 8)])
def test_bf16_bit_exact(L, N, B, nnz):
    """cfg5's bf16 path (BASELINE configs[4] at full size: L = 4096, 4 blocks, B = 1024) == the
    oracle's bf16 emulation, bit for bit (replaces a 1 %-of-range bound)."""
    cfg, st = exact_models.integer_state(L, N, nnz=nnz)
    x = exact_models.integer_inputs(B, seed=L + B)
    exact_models.exact_forward(st, x)                       # (the model is exact in float32)
    ref = ref_mlp.forward_bf16(st, x, acc=np.float64)
    assert np.array_equal(ref, ref_mlp.forward_bf16(st, x, acc=np.float32))   # order-independent
    m = _model(cfg, st, max_batch=B, dtype="bfloat16")
    y = m.forward_device(torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    m.close()
