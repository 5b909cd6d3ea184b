"""src/cameras.py's point functions on the GPU (libp3d, float64), same signatures and returns.

* ``project_point_radial(P, R, T, f, c, k, p)`` -> ``(Proj [N, 2], D [N], radial [N], tan [N],
  r2 [N])`` (src/cameras.py:13-53)
* ``world_to_camera_frame(P, R, T)`` -> ``[N, 3]`` (src/cameras.py:55-72)
* ``camera_to_world_frame(P, R, T)`` -> ``[N, 3]`` (src/cameras.py:74-90)

Arguments are numpy arrays as in the reference (R 3x3 already transposed by
``load_camera_params``, T 3x1, f/c 2x1, k 3x1, p 2x1); results come back as numpy float64,
bit-identical to the reference's.  The HDF5 camera loaders (``load_camera_params``,
``load_cameras``) need h5py and the H3.6M ``cameras.h5``, neither of which is in scope here;
any dict ``{(subject, cam): (R, T, f, c, k, p, name)}`` in that shape drives the data_utils
functions.
"""
from __future__ import annotations

import numpy as np

import data_pipeline as dp

_NO_DISTORTION = (np.zeros((2, 1)), np.zeros((2, 1)), np.zeros((3, 1)), np.zeros((2, 1)))


def _check_points(P):
    # the reference asserts these (src/cameras.py:34-35, :67-68, :85-86)
    P = np.asarray(P)
    if len(P.shape) != 2:
        raise AssertionError("points must be a 2-d array")
    if P.shape[1] != 3:
        raise AssertionError("points must have 3 columns")
    return P


def project_point_radial(P, R, T, f, c, k, p):
    P = _check_points(P)
    cam = dp.pack_camera(R, T, f, c, k, p)
    proj, depth, radial, tan, r2 = dp.project(P, cam, aux=True)
    return (proj[0].cpu().numpy(), depth[0].cpu().numpy(), radial[0].cpu().numpy(), tan[0].cpu().numpy(),
            r2[0].cpu().numpy())


def world_to_camera_frame(P, R, T):
    P = _check_points(P)
    return dp.world_to_camera(P, dp.pack_camera(R, T, *_NO_DISTORTION))[0].cpu().numpy()


def camera_to_world_frame(P, R, T):
    P = _check_points(P)
    return dp.camera_to_world(P, dp.pack_camera(R, T, *_NO_DISTORTION))[0].cpu().numpy()
