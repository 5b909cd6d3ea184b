"""src/data_utils.py for the hot path's callers, with its numeric work on the GPU.

* H3.6M tables (src/data_utils.py:18-53), ``define_actions`` (:314-336) and the used/ignored
  dimension sets of ``normalization_stats`` (:195-230): host tables.
* On the GPU (libp3d, float64, bit-identical to the reference's numpy; data_pipeline.py):
  ``normalization_stats`` mean/std (:210-211), ``normalize_data`` (:260-280),
  ``unNormalizeData`` (:283-311), ``transform_world_to_camera`` (:233-257),
  ``project_to_cameras`` (:339-364) and ``postprocess_3d`` (:474-494).  Each batches all the
  sequences of a subject into one launch.
* The HDF5 loaders (``load_data``, ``load_stacked_hourglass``, ``read_*``) read the H3.6M
  files, which are not in the image: out of scope.
"""
from __future__ import annotations

import numpy as np

import data_pipeline as dp

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
    """mean, std (population, over axis 0; computed on the GPU), dims_to_ignore, dims_to_use."""
    if dim not in (2, 3):
        raise ValueError('dim must be 2 or 3')
    use, ignore = dimension_sets(dim, predict_14)
    mean, std = dp.moments(complete_data)
    return mean.cpu().numpy(), std.cpu().numpy(), ignore, use


def _stack(data, keys):
    rows = [np.asarray(data[k]) for k in keys]
    return np.concatenate(rows) if len(rows) > 1 else rows[0], [r.shape[0] for r in rows]


def normalize_data(data, data_mean, data_std, dim_to_use):
    """(x[:, use] - mean[use]) / std[use] for every entry of a dict of pose arrays.  Like the
    reference, ``data``'s entries are replaced by their used columns as a side effect."""
    keys = list(data.keys())
    if not keys:
        return {}
    x, sizes = _stack(data, keys)
    y = dp.normalize(x, data_mean, data_std, dim_to_use).cpu().numpy()
    out, off = {}, 0
    use = np.asarray(dim_to_use)
    for k, n in zip(keys, sizes):
        data[k] = data[k][:, use]
        out[k] = y[off:off + n]
        off += n
    return out


def unNormalizeData(normalized_data, data_mean, data_std, dimensions_to_ignore):
    """Inverse of normalize_data: the used columns rounded to float32 (the reference scatters
    them into a float32 zero matrix), then * std + mean in float64."""
    D = data_mean.shape[0]
    used = np.setdiff1d(np.arange(D), np.asarray(dimensions_to_ignore, dtype=np.int64))
    return dp.unnormalize(normalized_data, data_mean, data_std, used, D).cpu().numpy()


def _by_subject(poses_set):
    groups = {}
    for key in sorted(poses_set.keys()):
        groups.setdefault(key[0], []).append(key)
    return groups


def _camera_key(key, cam):
    subj, action, seqname = key
    return (subj, action, seqname[:-3] + "." + cam[6] + ".h5")   # e.g. "Waiting 1.58860488.h5"


def _per_camera(poses_set, cams, ncams, width, run):
    out = {}
    for subj, keys in _by_subject(poses_set).items():
        pts = [np.reshape(np.asarray(poses_set[k], np.float64), (-1, 3)) for k in keys]
        camlist = [cams[(subj, c + 1)] for c in range(ncams)]
        res = run(np.concatenate(pts), dp.pack_cameras(camlist)).cpu().numpy()
        off = 0
        for k, p in zip(keys, pts):
            for c, cam in enumerate(camlist):
                out[_camera_key(k, cam)] = np.reshape(res[c, off:off + p.shape[0]], (-1, width))
            off += p.shape[0]
    return out


def transform_world_to_camera(poses_set, cams, ncams=4):
    """3D poses of every sequence in the frame of each of the subject's ncams cameras."""
    return _per_camera(poses_set, cams, ncams, len(H36M_NAMES) * 3, dp.world_to_camera)


def project_to_cameras(poses_set, cams, ncams=4):
    """2D projections (radial + tangential distortion) of every sequence into each camera."""
    return _per_camera(poses_set, cams, ncams, len(H36M_NAMES) * 2, dp.project)


def postprocess_3d(poses_set):
    """Centre every pose on its root joint, in place like the reference; returns
    (poses_set, root_positions)."""
    keys = list(poses_set.keys())
    if not keys:
        return poses_set, {}
    x, sizes = _stack(poses_set, keys)
    centred, root = dp.root_center(np.asarray(x, np.float64))
    centred, root = centred.cpu().numpy(), root.cpu().numpy()
    roots, off = {}, 0
    for k, n in zip(keys, sizes):
        roots[k] = root[off:off + n]
        poses_set[k] = centred[off:off + n]
        off += n
    return poses_set, roots
