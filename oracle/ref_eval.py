"""CPU oracle for the evaluation half of the hot path.  TEST INFRASTRUCTURE ONLY.

Restates (reference EsauPR/3d-pose-baseline):

* ``unNormalizeData``          -- src/data_utils.py:283-311
* ``normalize_data``           -- src/data_utils.py:260-280
* ``normalization_stats`` index sets -- src/data_utils.py:195-230 (H36M_NAMES :18-35)
* ``define_actions``           -- src/data_utils.py:314-336
* ``get_all_batches``          -- src/linear_model.py:247-300
* ``get_action_subset``        -- src/predict_3dpose.py:337-349
* ``evaluate_batches`` MPJPE   -- src/predict_3dpose.py:352-444 (procrustes branch :413-421)
* ``compute_similarity_transform`` -- src/procrustes.py:2-63

These are pinned against fixtures produced by importing the reference's own
``data_utils``/``procrustes`` modules (tests/golden/make_golden.py, run under the
image's python3.9 which has h5py) -- see tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np

H36M_NAMES = [''] * 32
for _i, _n in {0: 'Hip', 1: 'RHip', 2: 'RKnee', 3: 'RFoot', 6: 'LHip', 7: 'LKnee', 8: 'LFoot',
               12: 'Spine', 13: 'Thorax', 14: 'Neck/Nose', 15: 'Head', 17: 'LShoulder',
               18: 'LElbow', 19: 'LWrist', 25: 'RShoulder', 26: 'RElbow', 27: 'RWrist'}.items():
    H36M_NAMES[_i] = _n

ACTIONS = ["Directions", "Discussion", "Eating", "Greeting", "Phoning", "Photo", "Posing",
           "Purchases", "Sitting", "SittingDown", "Smoking", "Waiting", "WalkDog", "Walking",
           "WalkTogether"]


def define_actions(action):
    if action in ("All", "all"):
        return list(ACTIONS)
    if action not in ACTIONS:
        raise ValueError("Unrecognized action: %s" % action)
    return [action]


def dims_to_use(dim: int, predict_14: bool = False):
    """Index sets of normalization_stats (data_mean/std are not recomputed here)."""
    names = np.array(H36M_NAMES)
    if dim == 2:
        use = np.where((names != '') & (names != 'Neck/Nose'))[0]
        use = np.sort(np.hstack((use * 2, use * 2 + 1)))
        ignore = np.delete(np.arange(len(H36M_NAMES) * 2), use)
    else:
        use = np.where(names != '')[0]
        use = np.delete(use, [0, 7, 9] if predict_14 else 0)
        use = np.sort(np.hstack((use * 3, use * 3 + 1, use * 3 + 2)))
        ignore = np.delete(np.arange(len(H36M_NAMES) * 3), use)
    return use, ignore


def normalization_stats(complete_data, dim, predict_14=False):
    mean = np.mean(complete_data, axis=0)
    std = np.std(complete_data, axis=0)
    use, ignore = dims_to_use(dim, predict_14)
    return mean, std, ignore, use


def normalize_data(data, data_mean, data_std, dim_to_use):
    out = {}
    for key in data.keys():
        sub = data[key][:, dim_to_use]
        out[key] = np.divide(sub - data_mean[dim_to_use], data_std[dim_to_use])
    return out


def unNormalizeData(normalized_data, data_mean, data_std, dimensions_to_ignore):
    """Scatter the used dims into a float32 zero matrix, then *std + mean in float64."""
    T = normalized_data.shape[0]
    D = data_mean.shape[0]
    orig = np.zeros((T, D), dtype=np.float32)
    use = np.array([d for d in range(D) if d not in set(np.asarray(dimensions_to_ignore).tolist())])
    orig[:, use] = normalized_data
    return np.multiply(orig, np.repeat(data_std.reshape((1, D)), T, axis=0)) + \
        np.repeat(data_mean.reshape((1, D)), T, axis=0)


def get_all_batches(data_x, data_y, batch_size, camera_frame=True, training=True, rng=None):
    """Concatenate in dict order, permute if training, drop the n % B tail, split."""
    n = sum(v.shape[0] for v in data_x.values())
    d_in = next(iter(data_x.values())).shape[1]
    d_out = next(iter(data_y.values())).shape[1]
    enc = np.zeros((n, d_in), dtype=float)
    dec = np.zeros((n, d_out), dtype=float)
    idx = 0
    for key2d in data_x.keys():
        subj, b, fname = key2d
        key3d = key2d if camera_frame else (subj, b, '{0}.h5'.format(fname.split('.')[0]))
        key3d = (subj, b, fname[:-3]) if fname.endswith('-sh') and camera_frame else key3d
        n2d = data_x[key2d].shape[0]
        enc[idx:idx + n2d] = data_x[key2d]
        dec[idx:idx + n2d] = data_y[key3d]
        idx += n2d
    if training:
        perm = (rng or np.random).permutation(n)
        enc, dec = enc[perm], dec[perm]
    extra = n % batch_size
    if extra > 0:
        enc, dec = enc[:-extra], dec[:-extra]
    nb = n // batch_size
    if nb == 0:
        return [], []
    return np.split(enc, nb), np.split(dec, nb)


def get_action_subset(poses_set, action):
    return {k: v for k, v in poses_set.items() if k[1] == action}


def compute_similarity_transform(X, Y, compute_optimal_scale=False):
    """src/procrustes.py:2-63 (orthogonal Procrustes with optional scale)."""
    muX, muY = X.mean(0), Y.mean(0)
    X0, Y0 = X - muX, Y - muY
    ssX, ssY = (X0 ** 2.).sum(), (Y0 ** 2.).sum()
    normX, normY = np.sqrt(ssX), np.sqrt(ssY)
    X0, Y0 = X0 / normX, Y0 / normY
    A = np.dot(X0.T, Y0)
    U, s, Vt = np.linalg.svd(A, full_matrices=False)
    V = Vt.T
    T = np.dot(V, U.T)
    detT = np.linalg.det(T)
    V[:, -1] *= np.sign(detT)
    s[-1] *= np.sign(detT)
    T = np.dot(V, U.T)
    traceTA = s.sum()
    if compute_optimal_scale:
        b = traceTA * normX / normY
        d = 1 - traceTA ** 2
        Z = normX * traceTA * np.dot(Y0, T) + muX
    else:
        b = 1
        d = 1 + ssY / ssX - 2 * traceTA * normY / normX
        Z = normY * np.dot(Y0, T) + muX
    c = muX - b * np.dot(muY, T)
    return d, Z, T, b, c


def batch_dists(poses3d_n, dec_out_n, data_mean_3d, data_std_3d, dim_to_ignore_3d, dim_to_use_3d,
                predict_14=False, procrustes=False):
    """Per-frame per-joint L2 errors (mm) of one batch: src/predict_3dpose.py:399-430."""
    n_joints = 14 if predict_14 else 17
    dec = unNormalizeData(dec_out_n, data_mean_3d, data_std_3d, dim_to_ignore_3d)
    pred = unNormalizeData(poses3d_n, data_mean_3d, data_std_3d, dim_to_ignore_3d)
    dtu3d = np.hstack((np.arange(3), dim_to_use_3d)) if not predict_14 else dim_to_use_3d
    dec, pred = dec[:, dtu3d], pred[:, dtu3d]
    if procrustes:
        for j in range(pred.shape[0]):
            gt = np.reshape(dec[j, :], [-1, 3])
            out = np.reshape(pred[j, :], [-1, 3])
            _, Z, T, b, c = compute_similarity_transform(gt, out, compute_optimal_scale=True)
            out = (b * out.dot(T)) + c
            pred[j, :] = np.reshape(out, [-1, n_joints * 3])
    sqerr = (pred - dec) ** 2
    dists = np.zeros((sqerr.shape[0], n_joints))
    for j, k in enumerate(np.arange(0, n_joints * 3, 3)):
        dists[:, j] = np.sqrt(np.sum(sqerr[:, k:k + 3], axis=1))
    return dists


def evaluate_batches(predict_fn, encoder_inputs, decoder_outputs, data_mean_3d, data_std_3d,
                     dim_to_use_3d, dim_to_ignore_3d, predict_14=False, procrustes=False):
    """MPJPE of a list of batches: returns (total_err, joint_err, loss)."""
    all_dists, loss = [], 0.0
    for enc, dec in zip(encoder_inputs, decoder_outputs):
        step_loss, poses3d = predict_fn(enc, dec)
        loss += step_loss
        all_dists.append(batch_dists(poses3d, dec, data_mean_3d, data_std_3d, dim_to_ignore_3d,
                                     dim_to_use_3d, predict_14, procrustes))
    all_dists = np.vstack(all_dists)
    return np.mean(all_dists), np.mean(all_dists, axis=0), loss / max(len(encoder_inputs), 1)


# --------------------------------------------------------------------------------------
# synthetic H3.6M-shaped data: the dataset itself is not in the image
# --------------------------------------------------------------------------------------


def synthetic_stats(seed: int = 3, predict_14: bool = False):
    """mean96 ~ U(-500,500) mm, std96 ~ U(50,300) mm on used dims; root dims 0."""
    rng = np.random.default_rng(seed)
    use3, ign3 = dims_to_use(3, predict_14)
    mean = np.zeros(96)
    std = np.zeros(96)
    mean[use3] = rng.uniform(-500, 500, len(use3))
    std[use3] = rng.uniform(50, 300, len(use3))
    use2, ign2 = dims_to_use(2)
    mean2 = np.zeros(64)
    std2 = np.ones(64)
    mean2[use2] = rng.uniform(200, 800, len(use2))
    std2[use2] = rng.uniform(20, 120, len(use2))
    return dict(mean3=mean, std3=std, use3=use3, ign3=ign3, mean2=mean2, std2=std2, use2=use2, ign2=ign2)


def synthetic_test_set(seed: int = 4, lo: int = 20000, hi: int = 40000, out_dim: int = 48,
                       subjects=(9, 11), scale: float = 1.0):
    """Per-action normalized 2D/3D test dicts keyed (subject, action, seqname).

    Frames per action ~ U[lo, hi] (not multiples of 64, to exercise tail drop),
    split across subjects/cameras so get_action_subset's concatenation order matters.
    """
    rng = np.random.default_rng(seed)
    set2d, set3d = {}, {}
    for a in ACTIONS:
        n = int(rng.integers(int(lo * scale), int(hi * scale) + 1))
        cuts = np.sort(rng.choice(np.arange(1, n), size=3, replace=False))
        parts = np.split(np.arange(n), cuts)
        for j, p in enumerate(parts):
            subj = subjects[j % len(subjects)]
            key = (subj, a, "%s %d.5486%04d.h5" % (a, j, j))
            set2d[key] = rng.standard_normal((len(p), 32))
            set3d[key] = rng.standard_normal((len(p), out_dim))
    return set2d, set3d
