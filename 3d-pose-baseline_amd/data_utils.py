"""src/data_utils.py for the hot path's callers, with its numeric work on the GPU.

* H3.6M tables (src/data_utils.py:18-53), ``define_actions`` (:314-336) and the used/ignored
  dimension sets of ``normalization_stats`` (:195-230): host tables.
* On the GPU (libp3d, float64, bit-identical to the reference's numpy; data_pipeline.py):
  ``normalization_stats`` mean/std (:210-211), ``normalize_data`` (:260-280),
  ``unNormalizeData`` (:283-311), ``transform_world_to_camera`` (:233-257),
  ``project_to_cameras`` (:339-364) and ``postprocess_3d`` (:474-494).  Each batches all the
  sequences of a subject into one launch.
* The loaders ``load_data`` (:61-117), ``load_stacked_hourglass`` (:120-192) and the
  pipelines ``read_3d_data`` (:431-471), ``create_2d_data`` (:395-428) and
  ``read_2d_predictions`` (:367-392) read the H3.6M tree either as the reference's directory of
  HDF5 files (needs h5py, which this image lacks) or as ONE ``.npz`` archive whose member names
  are the tree's relative paths (``S1/MyPoses/3D_positions/Walking 1.h5`` holding the file's
  dataset as stored, e.g. [96, n]) -- the same files, sequence names, selection rules and
  counts; the numeric stages above run on the GPU.
"""
from __future__ import annotations

import copy
import fnmatch
import glob
import os

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


# ---- the H3.6M tree: an npz archive of its files, or the directory itself ----------------
class _Tree:
    """Files of the H3.6M tree under ``bpath`` by relative path: an ``.npz`` archive (member
    name = relative path of the file, value = the file's dataset) or a directory of the
    reference's HDF5 files (h5py)."""

    def __init__(self, bpath):
        self.bpath = bpath
        self.npz = None
        if os.path.isfile(bpath):
            self.npz = np.load(bpath, allow_pickle=False)
            self.names = list(self.npz.files)

    def close(self):
        if self.npz is not None:
            self.npz.close()
            self.npz = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def glob(self, pattern):
        """Relative paths matching ``pattern`` (glob semantics on the archive's names; the
        reference's glob.glob on a directory), sorted: the reference's order is whatever its
        directory listing gave (src/data_utils.py:87,145), and it feeds the normalisation
        statistics' vstack and the training-set order, so this build fixes it instead of
        inheriting the archive's member order or the file system's (parity unpinned)."""
        if self.npz is None:
            base = os.path.join(self.bpath, "")
            return sorted(f[len(base):] if f.startswith(base) else f
                          for f in glob.glob(os.path.join(self.bpath, pattern)))
        d, leaf = os.path.split(pattern)
        return sorted(n for n in self.names
                      if os.path.dirname(n) == d and fnmatch.fnmatchcase(os.path.basename(n), leaf))

    def read(self, rel, dataset):
        if self.npz is not None:
            return np.asarray(self.npz[rel])
        try:
            import h5py
        except ImportError as e:   # the image has no h5py: the archive form is the supported one
            raise ImportError("reading the H3.6M HDF5 files needs h5py; pass the tree as an .npz archive "
                              "(data_utils module docstring)") from e
        with h5py.File(os.path.join(self.bpath, rel), "r") as h5f:
            return h5f[dataset][:]


def load_data(bpath, subjects, actions, dim=3):
    """{(subject, action, seqname): [n, 32 * dim]} from ``S<subj>/MyPoses/<dim>D_positions/<action>*.h5``
    (src/data_utils.py:61-117): the same Sitting / SittingDown and prefix rules, 2 sequences per
    subject and action for 3D, 8 for 2D."""
    if dim not in (2, 3):
        raise ValueError('dim must be 2 or 3')
    with _Tree(bpath) as tree:
        return _load_data(tree, subjects, actions, dim)


def _load_data(tree, subjects, actions, dim):
    data = {}
    for subj in subjects:
        for action in actions:
            names = tree.glob(os.path.join('S{0}'.format(subj), 'MyPoses/{0}D_positions'.format(dim),
                                           '{0}*.h5'.format(action)))
            loaded = 0
            for rel in names:
                seqname = os.path.basename(rel)
                if action == "Sitting" and seqname.startswith("SittingDown"):
                    continue
                if seqname.startswith(action):
                    loaded += 1
                    data[(subj, action, seqname)] = tree.read(rel, '{0}D_positions'.format(dim)).T
            want = 8 if dim == 2 else 2
            assert loaded == want, "Expecting {0} sequences, found {1} instead".format(want, loaded)
    return data


# Stacked Hourglass joint order -> H3.6M (src/data_utils.py:134-135)
SH_TO_GT_PERM = np.array([SH_NAMES.index(h) for h in H36M_NAMES if h != '' and h in SH_NAMES])


def load_stacked_hourglass(data_dir, subjects, actions):
    """{(subject, action, seqname + '-sh'): [n, 64]} from ``S<subj>/StackedHourglass/<action>*.h5``
    (src/data_utils.py:120-192): detections permuted to H3.6M order and scattered into the 64
    2D columns; 8 sequences per subject and action (7 for S11 Directions)."""
    with _Tree(data_dir) as tree:
        return _load_stacked_hourglass(tree, subjects, actions)


def _load_stacked_hourglass(tree, subjects, actions):
    xs = np.flatnonzero(np.array([x != '' and x != 'Neck/Nose' for x in H36M_NAMES])) * 2
    cols = np.zeros(len(SH_NAMES) * 2, dtype=np.int32)
    cols[0::2], cols[1::2] = xs, xs + 1
    data = {}
    for subj in subjects:
        for action in actions:
            names = tree.glob(os.path.join('S{0}'.format(subj), 'StackedHourglass/{0}*.h5'.format(action)))
            loaded = 0
            for rel in names:
                seqname = os.path.basename(rel).replace('_', ' ')
                if action == "Sitting" and seqname.startswith("SittingDown"):
                    continue
                if seqname.startswith(action):
                    loaded += 1
                    poses = tree.read(rel, 'poses')[:, SH_TO_GT_PERM, :]
                    poses = np.reshape(poses, [poses.shape[0], -1])
                    final = np.zeros([poses.shape[0], len(H36M_NAMES) * 2])
                    final[:, cols] = poses
                    data[(subj, action, seqname + '-sh')] = final
            want = 7 if (subj == 11 and action == 'Directions') else 8
            assert loaded == want, "Expecting {0} sequences, found {1} instead. S:{2} {3}".format(
                want, loaded, subj, action)
    return data


def read_3d_data(actions, data_dir, camera_frame, rcams, predict_14=False):
    """3D poses: (optionally) into every camera's frame, root-centred, normalised with the
    training set's statistics (src/data_utils.py:431-471).  Returns train_set, test_set,
    data_mean, data_std, dim_to_ignore, dim_to_use, train_root_positions, test_root_positions."""
    train_set = load_data(data_dir, TRAIN_SUBJECTS, actions, dim=3)
    test_set = load_data(data_dir, TEST_SUBJECTS, actions, dim=3)
    if camera_frame:
        train_set = transform_world_to_camera(train_set, rcams)
        test_set = transform_world_to_camera(test_set, rcams)
    train_set, train_root_positions = postprocess_3d(train_set)
    test_set, test_root_positions = postprocess_3d(test_set)
    complete_train = copy.deepcopy(np.vstack(list(train_set.values())))
    data_mean, data_std, dim_to_ignore, dim_to_use = normalization_stats(complete_train, dim=3,
                                                                         predict_14=predict_14)
    train_set = normalize_data(train_set, data_mean, data_std, dim_to_use)
    test_set = normalize_data(test_set, data_mean, data_std, dim_to_use)
    return (train_set, test_set, data_mean, data_std, dim_to_ignore, dim_to_use, train_root_positions,
            test_root_positions)


def _normalized_2d(train_set, test_set):
    complete_train = copy.deepcopy(np.vstack(list(train_set.values())))
    data_mean, data_std, dim_to_ignore, dim_to_use = normalization_stats(complete_train, dim=2)
    train_set = normalize_data(train_set, data_mean, data_std, dim_to_use)
    test_set = normalize_data(test_set, data_mean, data_std, dim_to_use)
    return train_set, test_set, data_mean, data_std, dim_to_ignore, dim_to_use


def create_2d_data(actions, data_dir, rcams):
    """2D inputs: the 3D poses projected into every camera, normalised with the training set's
    statistics (src/data_utils.py:395-428)."""
    train_set = project_to_cameras(load_data(data_dir, TRAIN_SUBJECTS, actions, dim=3), rcams)
    test_set = project_to_cameras(load_data(data_dir, TEST_SUBJECTS, actions, dim=3), rcams)
    return _normalized_2d(train_set, test_set)


def read_2d_predictions(actions, data_dir):
    """2D inputs from the Stacked Hourglass detections (src/data_utils.py:367-392)."""
    return _normalized_2d(load_stacked_hourglass(data_dir, TRAIN_SUBJECTS, actions),
                          load_stacked_hourglass(data_dir, TEST_SUBJECTS, actions))
