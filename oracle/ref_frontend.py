"""CPU oracle for the OpenPose front end's per-frame lifting.
TEST INFRASTRUCTURE ONLY.

Restates src/openpose_3dpose_sandbox.py:317-356 (reference EsauPR/3d-pose-baseline):

* the joint mapping of an OpenPose frame (18 joints, x/y interleaved; the first 14 are used,
  ``order`` of :25) into the 64-wide H3.6M 2D vector, then the derived joints (:336-342):
  Hip = mean(RHip, LHip), Neck/Nose = mean(Head, Spine), Thorax = 2*Spine - Neck/Nose
  (in that order; the Thorax line reads the Neck/Nose just written);
* normalisation with the training-set 2D statistics over ``dim_to_use_2d`` (:347-350),
  float64, then the float32 cast of the ``enc_in`` placeholder;
* the MLP (oracle/ref_mlp.py) and ``unNormalizeData`` of the 3D output (:356).

No reference fixture exercises this script (it needs TensorFlow, the H3.6M data and OpenPose
JSON): the mapping is pinned by the reference's tables only (``order``, ``H36M_NAMES``),
"parity unpinned" beyond the pieces pinned elsewhere (normalisation, unNormalizeData, MLP).
"""
from __future__ import annotations

import numpy as np

from oracle import ref_eval, ref_mlp

ORDER = [15, 12, 25, 26, 27, 17, 18, 19, 1, 2, 3, 6, 7, 8]   # src/openpose_3dpose_sandbox.py:25


def map_frame(xy, enc_in=None):
    """One OpenPose frame (>= 28 values) -> the [64] H3.6M 2D vector (float64)."""
    e = np.zeros(64) if enc_in is None else np.array(enc_in, np.float64)
    for i, h in enumerate(ORDER):
        for j in range(2):
            e[h * 2 + j] = float(xy[i * 2 + j])
    for j in range(2):
        e[0 * 2 + j] = (e[1 * 2 + j] + e[6 * 2 + j]) / 2
        e[14 * 2 + j] = (e[15 * 2 + j] + e[12 * 2 + j]) / 2
        e[13 * 2 + j] = 2 * e[12 * 2 + j] - e[14 * 2 + j]
    return e


def lift_frames(state, frames_xy, mean2, std2, use2, mean3, std3, ign3, dt=np.float64):
    """Lift a sequence of frames one at a time as the sandbox does: ([N, 96] mm poses,
    [N, 48] normalized network outputs)."""
    out, norm = [], []
    for xy in frames_xy:
        e = map_frame(xy)[None, :]
        x = ((e[:, use2] - mean2[use2]) / std2[use2]).astype(np.float32)
        y = ref_mlp.forward(state, x.astype(dt), training=False, dt=dt)
        y = y[0] if isinstance(y, tuple) else y
        norm.append(np.asarray(y)[0])
        out.append(ref_eval.unNormalizeData(np.asarray(y, np.float32), mean3, std3, ign3)[0])
    return np.stack(out), np.stack(norm)
