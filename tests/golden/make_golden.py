"""Generate golden vectors by importing the REFERENCE's own modules.

Run in the build container only (the reference is not on the GPU box):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

python3.9 is the image interpreter that has h5py, which the reference's
``src/data_utils.py`` imports at module load.  ``src/linear_model.py`` and
``src/predict_3dpose.py`` import TensorFlow, which is absent from the image, so
the MLP itself cannot be run here ("parity unpinned" for the MLP arithmetic,
SURVEY.md section 8c); what CAN be pinned is everything around it:

* ``data_utils.unNormalizeData``   (src/data_utils.py:283)
* ``data_utils.normalize_data``    (src/data_utils.py:260)
* ``data_utils.normalization_stats`` index sets + mean/std (src/data_utils.py:195)
* ``data_utils.define_actions``    (src/data_utils.py:314)
* ``procrustes.compute_similarity_transform`` (src/procrustes.py:2)
* the MPJPE arithmetic of ``evaluate_batches`` (src/predict_3dpose.py:399-430),
  driven through the reference's own ``unNormalizeData``.

Outputs: tests/golden/reference_goldens.npz (inputs and expected outputs only).
"""
import os
import sys

import numpy as np

REF = "/root/reference/src"
sys.path.insert(0, REF)
import matplotlib  # noqa: E402

matplotlib.use("Agg")
import data_utils  # noqa: E402  (reference module)
import procrustes  # noqa: E402  (reference module)

out = {}
rng = np.random.default_rng(20240601)

# --- normalization_stats: index sets and stats -------------------------------------
d3 = rng.normal(0, 300, (257, 96))
d2 = rng.normal(400, 100, (257, 64))
m3, s3, ign3, use3 = data_utils.normalization_stats(d3, 3)
m2, s2, ign2, use2 = data_utils.normalization_stats(d2, 2)
m3_14, s3_14, ign3_14, use3_14 = data_utils.normalization_stats(d3, 3, predict_14=True)
out.update(ns_in3=d3, ns_in2=d2, ns_mean3=m3, ns_std3=s3, ns_ign3=ign3, ns_use3=use3,
           ns_mean2=m2, ns_std2=s2, ns_ign2=ign2, ns_use2=use2, ns_ign3_14=ign3_14,
           ns_use3_14=use3_14)

# --- normalize_data / unNormalizeData ----------------------------------------------
mean3 = np.zeros(96)
std3 = np.zeros(96)
mean3[use3] = rng.uniform(-500, 500, len(use3))
std3[use3] = rng.uniform(50, 300, len(use3))
raw = {(9, "Walking", "Walking 1.54138969.h5"): rng.normal(0, 300, (70, 96)),
       (11, "Walking", "Walking 2.55011271.h5"): rng.normal(0, 300, (33, 96))}
normd = data_utils.normalize_data(dict(raw), mean3, std3, use3)
keys = list(raw.keys())
out.update(nd_in0=raw[keys[0]], nd_in1=raw[keys[1]], nd_mean=mean3, nd_std=std3,
           nd_out0=normd[keys[0]], nd_out1=normd[keys[1]])

un_in = rng.standard_normal((64, 48))
un_in32 = rng.standard_normal((64, 48)).astype(np.float32)
out.update(un_in=un_in, un_in32=un_in32,
           un_out=data_utils.unNormalizeData(un_in, mean3, std3, ign3),
           un_out32=data_utils.unNormalizeData(un_in32, mean3, std3, ign3))

# --- MPJPE arithmetic of evaluate_batches, through the reference's unNormalizeData ----
pred_n = rng.standard_normal((64, 48)).astype(np.float32)      # network outputs (fp32)
gt_n = rng.standard_normal((64, 48))                           # normalized GT (fp64)
dec = data_utils.unNormalizeData(gt_n, mean3, std3, ign3)
poses = data_utils.unNormalizeData(pred_n, mean3, std3, ign3)
dtu3d = np.hstack((np.arange(3), use3))
dec, poses = dec[:, dtu3d], poses[:, dtu3d]
sqerr = (poses - dec) ** 2
dists = np.zeros((64, 17))
for j, k in enumerate(np.arange(0, 51, 3)):
    dists[:, j] = np.sqrt(np.sum(sqerr[:, k:k + 3], axis=1))
# procrustes branch (src/predict_3dpose.py:413-421) on the same batch
poses_p = poses.copy()
for j in range(64):
    g = np.reshape(dec[j, :], [-1, 3])
    o = np.reshape(poses_p[j, :], [-1, 3])
    _, Z, T, b, c = procrustes.compute_similarity_transform(g, o, compute_optimal_scale=True)
    poses_p[j, :] = np.reshape((b * o.dot(T)) + c, [-1, 51])
sq_p = (poses_p - dec) ** 2
dists_p = np.zeros((64, 17))
for j, k in enumerate(np.arange(0, 51, 3)):
    dists_p[:, j] = np.sqrt(np.sum(sq_p[:, k:k + 3], axis=1))
out.update(mp_pred_n=pred_n, mp_gt_n=gt_n, mp_dists=dists, mp_dists_procrustes=dists_p)

# --- procrustes alone ---------------------------------------------------------------
X = rng.normal(0, 100, (17, 3))
Y = 1.7 * X @ np.linalg.qr(rng.normal(size=(3, 3)))[0] + rng.normal(0, 5, (17, 3)) + 20
for scale in (True, False):
    d, Z, T, b, c = procrustes.compute_similarity_transform(X, Y, compute_optimal_scale=scale)
    tag = "s" if scale else "n"
    out.update({"pr_%s_d" % tag: np.array(d), "pr_%s_Z" % tag: Z, "pr_%s_T" % tag: T,
                "pr_%s_b" % tag: np.array(b), "pr_%s_c" % tag: c})
out.update(pr_X=X, pr_Y=Y)

# --- predict_14 protocol (14 joints, no root prefix) + procrustes, and reflected poses ---
def mpjpe_dists(pred_n_, gt_n_, mean_, std_, ign_, use_, n_joints, proc):
    dec_ = data_utils.unNormalizeData(gt_n_, mean_, std_, ign_)
    pose_ = data_utils.unNormalizeData(pred_n_, mean_, std_, ign_)
    dtu = np.hstack((np.arange(3), use_)) if n_joints == 17 else use_
    dec_, pose_ = dec_[:, dtu], pose_[:, dtu]
    if proc:
        for j in range(pose_.shape[0]):
            g_ = np.reshape(dec_[j, :], [-1, 3])
            o_ = np.reshape(pose_[j, :], [-1, 3])
            _, Z_, T_, b_, c_ = procrustes.compute_similarity_transform(g_, o_, compute_optimal_scale=True)
            pose_[j, :] = np.reshape((b_ * o_.dot(T_)) + c_, [-1, n_joints * 3])
    sq_ = (pose_ - dec_) ** 2
    dd = np.zeros((pose_.shape[0], n_joints))
    for j, k in enumerate(np.arange(0, n_joints * 3, 3)):
        dd[:, j] = np.sqrt(np.sum(sq_[:, k:k + 3], axis=1))
    return dd


mean14 = np.zeros(96)
std14 = np.zeros(96)
mean14[use3_14] = rng.uniform(-500, 500, len(use3_14))
std14[use3_14] = rng.uniform(50, 300, len(use3_14))
pred14 = rng.standard_normal((64, 42)).astype(np.float32)
gt14 = rng.standard_normal((64, 42))
out.update(mp14_mean=mean14, mp14_std=std14, mp14_pred_n=pred14, mp14_gt_n=gt14,
           mp14_dists=mpjpe_dists(pred14, gt14, mean14, std14, ign3_14, use3_14, 14, False),
           mp14_dists_procrustes=mpjpe_dists(pred14, gt14, mean14, std14, ign3_14, use3_14, 14, True))
# mirrored predictions (det < 0 branch of compute_similarity_transform) + small noise
gtr = rng.standard_normal((32, 48))
decr = data_utils.unNormalizeData(gtr, mean3, std3, ign3)
mir = decr.copy()
mir[:, 0::3] = -mir[:, 0::3]
predr = ((mir[:, use3] - mean3[use3]) / std3[use3] + rng.normal(0, 0.01, (32, 48))).astype(np.float32)
out.update(mpr_pred_n=predr, mpr_gt_n=gtr,
           mpr_dists_procrustes=mpjpe_dists(predr, gtr, mean3, std3, ign3, use3, 17, True))

# --- define_actions -----------------------------------------------------------------
out["actions"] = np.array(data_utils.define_actions("All"))

# --- known answer held by the reference (src/data_utils.py:136 SH_TO_GT_PERM) --------
out["sh_names"] = np.array(data_utils.SH_NAMES)
out["h36m_names"] = np.array(data_utils.H36M_NAMES)

dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_goldens.npz")
np.savez_compressed(dst, **out)
print("wrote", dst, len(out), "arrays")
