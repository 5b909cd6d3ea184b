"""Writes tests/golden/cfg4_oracle.npz: the oracle's evaluateActionWise result on the cfg4
set of cfg4_data.py -- per-action MPJPE (mm) of src/predict_3dpose.py:274-298 / evaluate_batches
(:352-444) restated in oracle/ref_eval.py, fp64 forward of oracle/ref_mlp.py.  Run on the CPU:
    python tests/golden/make_cfg4_oracle.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from cfg4_data import ACTIONS, make_cfg4_set  # noqa: E402
from oracle import ref_eval, ref_mlp  # noqa: E402


def main():
    cfg = ref_mlp.Cfg(linear_size=1024, num_layers=2, residual=True, batch_norm=True)
    st = ref_mlp.init_state(cfg, seed=1, bn_seed=2)
    stats = ref_eval.synthetic_stats()
    s2, s3 = make_cfg4_set()
    errs, frames = [], []
    for a in ACTIONS:
        enc, dec = ref_eval.get_all_batches(ref_eval.get_action_subset(s2, a), ref_eval.get_action_subset(s3, a),
                                            64, camera_frame=True, training=False)
        X, Y = np.vstack(enc), np.vstack(dec)
        d = []
        for i in range(0, len(X), 8192):
            out, _ = ref_mlp.forward(st, X[i:i + 8192], False, 1.0, 0, 0, 0)
            d.append(ref_eval.batch_dists(out, Y[i:i + 8192], stats["mean3"], stats["std3"], stats["ign3"],
                                          stats["use3"]))
        errs.append(float(np.mean(np.vstack(d))))
        frames.append(len(X))
        print(a, frames[-1], errs[-1], flush=True)
    np.savez(os.path.join(HERE, "cfg4_oracle.npz"), actions=np.array(ACTIONS), mpjpe_mm=np.array(errs),
             frames=np.array(frames), average_mm=np.float64(np.mean(errs)))
    print("frames", sum(frames), "average", np.mean(errs))


if __name__ == "__main__":
    main()
