"""src/cameras.py's point functions on the GPU (libp3d, float64), same signatures and returns.

* ``project_point_radial(P, R, T, f, c, k, p)`` -> ``(Proj [N, 2], D [N], radial [N], tan [N],
  r2 [N])`` (src/cameras.py:13-53)
* ``world_to_camera_frame(P, R, T)`` -> ``[N, 3]`` (src/cameras.py:55-72)
* ``camera_to_world_frame(P, R, T)`` -> ``[N, 3]`` (src/cameras.py:74-90)

Arguments are numpy arrays as in the reference (R 3x3 already transposed by
``load_camera_params``, T 3x1, f/c 2x1, k 3x1, p 2x1); results come back as numpy float64,
bit-identical to the reference's.  ``load_camera_params`` / ``load_cameras``
(src/cameras.py:92-140) read ``cameras.h5`` (h5py, absent from this image) or an ``.npz``
archive of the same datasets under the same paths (``subject1/camera1/R`` ...; ``Name`` as its
character codes); any dict ``{(subject, cam): (R, T, f, c, k, p, name)}`` in that shape drives
the data_utils functions.
"""
from __future__ import annotations

import os

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


def load_camera_params(hf, path):
    """(R, T, f, c, k, p, name) of one camera; R transposed as stored, name from its character
    codes (src/cameras.py:92-120).  ``hf``: an open h5py file or an npz archive."""
    R = np.asarray(hf[path.format('R')][:]).T
    T = np.asarray(hf[path.format('T')][:])
    f = np.asarray(hf[path.format('f')][:])
    c = np.asarray(hf[path.format('c')][:])
    k = np.asarray(hf[path.format('k')][:])
    p = np.asarray(hf[path.format('p')][:])
    name = "".join([chr(int(item)) for item in np.asarray(hf[path.format('Name')][:]).reshape(-1)])
    return R, T, f, c, k, p, name


def load_cameras(bpath='cameras.h5', subjects=(1, 5, 6, 7, 8, 9, 11)):
    """{(subject, 1..4): camera tuple} for the four H3.6M cameras of each subject
    (src/cameras.py:122-140)."""
    rcams = {}
    if os.path.isfile(bpath) and bpath.endswith(".npz"):
        with np.load(bpath, allow_pickle=False) as hf:
            for s in subjects:
                for c in range(4):
                    rcams[(s, c + 1)] = load_camera_params(hf, 'subject%d/camera%d/{0}' % (s, c + 1))
        return rcams
    try:
        import h5py
    except ImportError as e:
        raise ImportError("reading cameras.h5 needs h5py; pass the cameras as an .npz archive "
                          "(cameras module docstring)") from e
    with h5py.File(bpath, 'r') as hf:
        for s in subjects:
            for c in range(4):
                rcams[(s, c + 1)] = load_camera_params(hf, 'subject%d/camera%d/{0}' % (s, c + 1))
    return rcams
