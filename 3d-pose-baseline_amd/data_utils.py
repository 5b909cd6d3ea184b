"""Host-side helpers of src/data_utils.py that the hot path's callers use.

Only what the evaluation sweep and the front ends need to feed / read the MLP:
the H3.6M joint tables (src/data_utils.py:18-53), the used/ignored dimension
sets of ``normalization_stats`` (:195-230), ``normalize_data`` (:260-280),
``unNormalizeData`` (:283-311) and ``define_actions`` (:314-336).  The H3.6M
loaders / camera projection are one-time preprocessing and out of scope for
this round.  The per-frame MPJPE itself runs
on the GPU (libp3d: p3d_mpjpe_accum), not here.
"""
from __future__ import annotations

import numpy as np

TRAIN_SUBJECTS = [1, 5, 6, 7, 8]
TEST_SUBJECTS = [9, 11]

_JOINTS = {0: 'Hip', 1: 'RHip', 2: 'RKnee', 3: 'RFoot', 6: 'LHip', 7: 'LKnee', 8: 'LFoot',
           12: 'Spine', 13: 'Thorax', 14: 'Neck/Nose', 15: 'Head', 17: 'LShoulder',
           18: 'LElbow', 19: 'LWrist', 25: 'RShoulder', 26: 'RElbow', 27: 'RWrist'}
H36M_NAMES = [_JOINTS.get(i, '') for i in range(32)]

SH_NAMES = ['RFoot', 'RKnee', 'RHip', 'LHip', 'LKnee', 'LFoot', 'Hip', 'Spine', 'Thorax', 'Head',
            'RWrist', 'RElbow', 'RShoulder', 'LShoulder', 'LElbow', 'LWrist']

_ACTIONS = ("Directions", "Discussion", "Eating", "Greeting", "Phoning", "Photo", "Posing",
            "Purchases", "Sitting", "SittingDown", "Smoking", "Waiting", "WalkDog", "Walking",
            "WalkTogether")


def define_actions(action):
    """'All'/'all' -> the 15 H3.6M actions; otherwise the single named action."""
    if action in ("All", "all"):
        return list(_ACTIONS)
    if action not in _ACTIONS:
        raise ValueError("Unrecognized action: %s" % action)
    return [action]


def dimension_sets(dim, predict_14=False):
    """(dimensions_to_use, dimensions_to_ignore) of normalization_stats for dim 2 or 3."""
    if dim not in (2, 3):
        raise ValueError('dim must be 2 or 3')
    named = np.array([n != '' for n in H36M_NAMES])
    if dim == 2:
        joints = np.flatnonzero(named & (np.array(H36M_NAMES) != 'Neck/Nose'))
    else:
        joints = np.flatnonzero(named)
        drop = [0, 7, 9] if predict_14 else [0]
        joints = np.delete(joints, drop)
    use = np.sort((joints[:, None] * dim + np.arange(dim)[None, :]).ravel())
    ignore = np.setdiff1d(np.arange(len(H36M_NAMES) * dim), use)
    return use, ignore


def normalization_stats(complete_data, dim, predict_14=False):
    """mean, std (population), dims_to_ignore, dims_to_use."""
    use, ignore = dimension_sets(dim, predict_14)
    return np.mean(complete_data, axis=0), np.std(complete_data, axis=0), ignore, use


def normalize_data(data, data_mean, data_std, dim_to_use):
    """(x[:, use] - mean[use]) / std[use] for every entry of a dict of pose arrays."""
    mu, sd = data_mean[dim_to_use], data_std[dim_to_use]
    return {k: np.divide(v[:, dim_to_use] - mu, sd) for k, v in data.items()}


def unNormalizeData(normalized_data, data_mean, data_std, dimensions_to_ignore):
    """Inverse of normalize_data: scatter used dims into a float32 [T, D] zero matrix
    (so float64 inputs are rounded to float32, as in the reference), then *std + mean
    in float64."""
    T, D = normalized_data.shape[0], data_mean.shape[0]
    used = np.setdiff1d(np.arange(D), np.asarray(dimensions_to_ignore, dtype=np.int64))
    full = np.zeros((T, D), dtype=np.float32)
    full[:, used] = normalized_data
    return full * data_std.reshape(1, D) + data_mean.reshape(1, D)
