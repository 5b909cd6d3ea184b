"""Process teardown with live models, cached HIP graphs and queued work: the process must
end with its own exit status -- 0, or 1 after an uncaught exception's traceback -- never a
signal.  Round 1 worked around a SIGSEGV at teardown (os._exit in bench.py, a Python atexit
close); p3d_destroy now synchronises before freeing and the library releases the models
still alive from an exit handler that runs before the HIP runtime's teardown (p3d.hip,
release_live_models_at_exit).  Each case runs in a fresh interpreter."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = """
import sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import numpy as np, torch
import linear_model
m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_td", seed=1, max_batch=8192)
rng = np.random.default_rng(0)
x, t = rng.standard_normal((64, 32)), rng.standard_normal((64, 48))
m.step(None, x, t, 1.0, isTraining=False)            # cached eval graph (H2D + 6 layers + D2H)
m.step(None, x, t, 0.5, isTraining=True)
xd = torch.randn((64 * 20, 32), device="cuda")
m.serve_device(xd)                                    # persistent serve launch
g = torch.cuda.CUDAGraph()                            # a torch graph over the model's buffers
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m.forward_device(xd[:64])
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    y = m.forward_device(xd[:64])
g.replay()
m2 = linear_model.LinearModel(256, 1, True, True, False, 64, 1e-3, "/tmp/p3d_td", seed=2)
for _ in range(50):
    m.serve_device(xd)                                # work still queued at the end
""" % (os.path.join(ROOT, "3d-pose-baseline_amd"), ROOT)


def run(body):
    return subprocess.run([sys.executable, "-c", PRELUDE + body], capture_output=True, text=True, timeout=150)


def test_exit_with_live_models_and_graphs():
    r = run("print('done', flush=True)\n")
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "done" in r.stdout


def test_uncaught_exception_with_live_models_and_graphs():
    r = run("raise RuntimeError('boom')\n")
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert "RuntimeError: boom" in r.stderr


def test_explicit_close_then_exit():
    r = run("m.close(); m2.close(); m.close(); print('done', flush=True)\n")
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
