"""Synthetic H3.6M-like cameras and world-frame poses (numpy only; the real cameras.h5 and
pose files are not in the image).  Used by make_golden_data.py (python3.9, reference side),
the tests and bench.py's data-pipeline measurement.

Camera tuple as the reference's ``load_cameras`` returns it (src/cameras.py:92-140):
``(R, T, f, c, k, p, name)`` with R 3x3 such that X_cam = R (P - T), T 3x1 the camera centre
in world mm, f/c 2x1, k 3x1, p 2x1.  The packed form is 21 float64 per camera:
R (row-major, 9), T (3), f (2), c (2), k (3), p (2).
"""
import numpy as np

CAM_NAMES = ["54138969", "55011271", "58860488", "60457274"]


def _look_at(centre, rng):
    z = -centre / np.linalg.norm(centre)
    up = np.array([0.0, 0.0, 1.0]) + rng.normal(0, 0.05, 3)
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])


def synth_cameras(rng, subjects=(1, 5, 6, 7, 8, 9, 11)):
    """(rcams dict {(subject, 1..4): tuple}, packed [S, 4, 21] array, names [S][4])."""
    cams, packed, names = {}, [], []
    for s in subjects:
        row, nrow = [], []
        for ci in range(4):
            ang = 2 * np.pi * ci / 4 + rng.uniform(-0.3, 0.3)
            centre = np.array([4500 * np.cos(ang), 4500 * np.sin(ang), rng.uniform(1200, 1800)])
            R = _look_at(centre, rng)
            T = centre.reshape(3, 1)
            f = rng.uniform(1140, 1150, (2, 1))
            c = rng.uniform(500, 520, (2, 1))
            k = np.array([[rng.uniform(-0.21, -0.19)], [rng.uniform(0.2, 0.25)], [rng.uniform(-0.01, 0.01)]])
            p = rng.uniform(-0.002, 0.002, (2, 1))
            name = CAM_NAMES[ci]
            cams[(s, ci + 1)] = (R, T, f, c, k, p, name)
            row.append(pack_camera(R, T, f, c, k, p))
            nrow.append(name)
        packed.append(row)
        names.append(nrow)
    return cams, np.array(packed), names


def pack_camera(R, T, f, c, k, p):
    return np.concatenate([np.asarray(R, np.float64).reshape(9), np.asarray(T, np.float64).reshape(3),
                           np.asarray(f, np.float64).reshape(2), np.asarray(c, np.float64).reshape(2),
                           np.asarray(k, np.float64).reshape(3), np.asarray(p, np.float64).reshape(2)])


def synth_world_poses(rng, n, joints=32):
    """[n, joints*3] world-frame poses (mm): a walking root plus joint offsets."""
    root = np.cumsum(rng.normal(0, 10, (n, 3)), axis=0) + np.array([0.0, 0.0, 900.0])
    off = rng.normal(0, 250, (1, joints, 3)) + rng.normal(0, 20, (n, joints, 3))
    off[:, 0] = 0.0
    return (root[:, None, :] + off).reshape(n, joints * 3)
