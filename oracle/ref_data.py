"""CPU oracle for the H3.6M data pipeline.  TEST INFRASTRUCTURE ONLY.

Restates, in float64 numpy (reference EsauPR/3d-pose-baseline):

* ``project_point_radial``      -- src/cameras.py:13-53 (radial k1..k3 + tangential p1, p2)
* ``world_to_camera_frame``     -- src/cameras.py:55-72   X_cam = R (P - T)
* ``camera_to_world_frame``     -- src/cameras.py:74-90   P = R^T X_cam + T
* ``transform_world_to_camera`` -- src/data_utils.py:233-257 (4 cameras per subject, key rename)
* ``project_to_cameras``        -- src/data_utils.py:339-364
* ``postprocess_3d``            -- src/data_utils.py:474-494 (root-centring, root positions kept)
* ``moments``                   -- the mean / population std of normalization_stats (:210-211)

A camera is the reference's tuple ``(R, T, f, c, k, p, name)`` with ``R`` 3x3 (already
transposed by ``load_camera_params``, src/cameras.py:112-113), ``T`` 3x1, ``f`` and ``c`` 2x1,
``k`` 3x1, ``p`` 2x1.  Pinned against tests/golden/reference_goldens_data.npz, produced by
importing the reference's own ``cameras``/``data_utils`` (tests/golden/make_golden_data.py).
"""
from __future__ import annotations

import numpy as np


def _mat3(M, V):
    """M [3, 3] times the columns of V [3, N] as the reference's numpy evaluates R.dot(..)
    for these shapes: (m0*v0 + m1*v1) + m2*v2, every product and sum rounded (no FMA;
    pinned bit-exact by the goldens -- a BLAS dot with FMA differs in the last bit)."""
    M = np.asarray(M, np.float64)
    return np.stack([(M[r, 0] * V[0] + M[r, 1] * V[1]) + M[r, 2] * V[2] for r in range(3)])


def world_to_camera_frame(P, R, T):
    """[N, 3] world points -> [N, 3] camera-frame points."""
    P = np.asarray(P, np.float64)
    assert P.ndim == 2 and P.shape[1] == 3
    return _mat3(R, P.T - np.asarray(T).reshape(3, 1)).T


def camera_to_world_frame(P, R, T):
    P = np.asarray(P, np.float64)
    assert P.ndim == 2 and P.shape[1] == 3
    return (_mat3(np.asarray(R).T, P.T) + np.asarray(T).reshape(3, 1)).T


def project_point_radial(P, R, T, f, c, k, p):
    """(proj [N, 2], depth [N], radial [N], tan [N], r2 [N]) as src/cameras.py:13-53."""
    P = np.asarray(P, np.float64)
    assert P.ndim == 2 and P.shape[1] == 3
    X = _mat3(R, P.T - np.asarray(T).reshape(3, 1))
    uv = X[:2] / X[2]
    r2 = uv[0] ** 2 + uv[1] ** 2
    k = np.asarray(k).reshape(3)
    p = np.asarray(p).reshape(2)
    radial = 1 + (k[0] * r2 + k[1] * r2 ** 2 + k[2] * r2 ** 3)
    tan = p[0] * uv[1] + p[1] * uv[0]
    dist = uv * (radial + tan) + np.array([p[1], p[0]]).reshape(2, 1) * r2
    proj = (np.asarray(f).reshape(2, 1) * dist + np.asarray(c).reshape(2, 1)).T
    return proj, X[2], radial, tan, r2


def _renamed(seqname, cam_name):
    # "Walking 1.h5" + camera "54138969" -> "Walking 1.54138969.h5"
    return seqname[:-3] + "." + cam_name + ".h5"


def transform_world_to_camera(poses_set, cams, ncams=4):
    out = {}
    for key in sorted(poses_set):
        subj, action, seq = key
        pts = np.reshape(poses_set[key], (-1, 3))
        for ci in range(ncams):
            R, T, f, c, k, p, name = cams[(subj, ci + 1)]
            out[(subj, action, _renamed(seq, name))] = np.reshape(world_to_camera_frame(pts, R, T), (-1, 96))
    return out


def project_to_cameras(poses_set, cams, ncams=4):
    out = {}
    for key in sorted(poses_set):
        subj, action, seq = key
        pts = np.reshape(poses_set[key], (-1, 3))
        for ci in range(ncams):
            R, T, f, c, k, p, name = cams[(subj, ci + 1)]
            proj = project_point_radial(pts, R, T, f, c, k, p)[0]
            out[(subj, action, _renamed(seq, name))] = np.reshape(proj, (-1, 64))
    return out


def postprocess_3d(poses_set):
    """Root-centre every pose; returns (centred set, root positions [N, 3])."""
    roots, centred = {}, {}
    for key, poses in poses_set.items():
        roots[key] = poses[:, :3].copy()
        centred[key] = poses - np.tile(poses[:, :3], (1, poses.shape[1] // 3))
    return centred, roots


def moments(data):
    """np.mean / np.std (population) over axis 0."""
    return np.mean(data, axis=0), np.std(data, axis=0)
