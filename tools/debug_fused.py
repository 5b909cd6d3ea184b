"""Dev: where do fused (p3d_train_step) and unfused train steps first differ?"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd")); sys.path.insert(0, ROOT)
import linear_model, _p3d
from oracle import ref_mlp
cfg = ref_mlp.Cfg(linear_size=256, num_layers=2, residual=True, batch_norm=True)
st = ref_mlp.init_state(cfg, seed=4, bn_seed=5)
ms = []
for _ in range(2):
    m = linear_model.LinearModel(256, 2, True, True, False, 64, 1e-3, "/tmp/p3d_test", seed=9)
    m.set_weights({**st.params, **st.moving}); ms.append(m)
fused, plain = ms
MODE = sys.argv[1] if len(sys.argv) > 1 else "fused-plain"
rng = np.random.default_rng(3)

def plain_step(m, x, t, y):
    _p3d.check(_p3d.lib().p3d_train_fwd_bwd(m._h, x.data_ptr(), t.data_ptr(), 64, y.data_ptr(), 0.5,
                                             m.seed, 0, m._loss_dev.data_ptr(), m.stream()), "fb")
    _p3d.check(_p3d.lib().p3d_adam_step_decay(m._h, m.lr0, 100000.0, 0.96, m.stream()), "adam")

for step in range(4):
    x = torch.from_numpy(rng.standard_normal((64, 32)).astype(np.float32)).cuda()
    t = torch.from_numpy(rng.standard_normal((64, 48)).astype(np.float32)).cuda()
    yf = torch.empty((64, 48), device="cuda"); yp = torch.empty((64, 48), device="cuda")
    if MODE == "plain-plain":
        plain_step(fused, x, t, yf); plain_step(plain, x, t, yp)
    elif MODE == "fused-fused":
        fused.train_step_device(x, t, 0.5, out=yf); plain.train_step_device(x, t, 0.5, out=yp)
    else:
        fused.train_step_device(x, t, 0.5, out=yf); plain_step(plain, x, t, yp)
    torch.cuda.synchronize()
    print(MODE, "step", step, "y equal", torch.equal(yf, yp), "max", (yf - yp).abs().max().item())
    for name, numel, kind, off in fused.param_table:
        key = "params" if kind == 0 else "moving"
        a = fused.flat[key][off:off + numel]; b = plain.flat[key][off:off + numel]
        if not torch.equal(a, b):
            d = (a - b).abs()
            print("  ", key, name, "ndiff", int((d > 0).sum()), "max", d.max().item())
        if kind == 0 and name.split("/")[-1].startswith("b"):
            a = fused.flat["grads"][off:off + numel]; b = plain.flat["grads"][off:off + numel]
            if not torch.equal(a, b):
                print("  grad", name, "ndiff", int(((a - b).abs() > 0).sum()), "max", (a - b).abs().max().item(),
                      "scale", b.abs().max().item())
        if kind == 0:
            for slot in ("adam_m", "adam_v"):
                a = fused.flat[slot][off:off + numel]; b = plain.flat[slot][off:off + numel]
                if not torch.equal(a, b):
                    print("  ", slot, name, "ndiff", int(((a - b).abs() > 0).sum()))
