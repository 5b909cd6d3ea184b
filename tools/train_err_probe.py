"""Dev probe: how far the fp32 HIP training step's outputs and weights are from the fp64
oracle over 5 TF1 steps (cfg2, keep 0.5) -- the data behind the tolerances of
tests/test_gpu_parity.py::test_train_steps_track_oracle."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import linear_model  # noqa: E402
from oracle import ref_mlp  # noqa: E402


def main():
    out = {}
    for split in ("1", "0"):
        os.environ["P3D_TRAIN_SPLIT"] = split
        cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
        st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
        m = linear_model.LinearModel(1024, 2, True, True, False, 64, 1e-3, "/tmp/p3d_probe", seed=11, max_batch=64)
        m.set_weights({**st.params, **st.moving})
        rng = np.random.default_rng(21)
        rows = []
        for step in range(5):
            x = rng.standard_normal((64, 32))
            t = rng.standard_normal((64, 48))
            loss, _, _, o = m.step(None, x, t, 0.5, isTraining=True)
            rl, ro = ref_mlp.train_step(st, x, t, 0.5, 1e-3, seed=m.seed, ctr=step)
            d = np.abs(o - ro)
            rows.append({"abs_max": float(d.max()), "rel_max": float((d / (np.abs(ro) + 1e-30)).max()),
                         "excess_over_2e5": float((d - 2e-5 - 2e-5 * np.abs(ro)).max()),
                         "loss_rel": float(abs(loss - rl) / max(1.0, rl))})
        w = m.get_weights()
        werr = max(float(np.abs(w[k] - st.params[k]).max()) for k in m.trainable_names()
                   if not ("/b1" in k or "/b2_" in k or "/b3_" in k))
        out["split" + split] = {"steps": rows, "weights_abs_max": werr}
        m.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
