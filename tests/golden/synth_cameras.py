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


def write_h36m_archives(tree_path, cams_path, rng, actions, frames=120, subjects=(1, 5, 6, 7, 8, 9, 11),
                        sh=False, decoys=True):
    """Synthetic H3.6M tree and cameras as .npz archives (member name = the file's relative path
    in the reference's tree / the dataset path in cameras.h5, value = the dataset as stored:
    3D_positions [96, n], StackedHourglass poses [n, 16, 2], R transposed, Name as character
    codes).  Two 3D sequences per subject and action ("<action> 1.h5", "<action>.h5"); with
    ``sh`` the 8 Stacked Hourglass files (7 for S11 Directions); ``decoys`` adds files the
    reference's selection rules must skip (SittingDown under Sitting, other actions).
    Returns (rcams, {(subject, action, seqname): world poses [n, 96]})."""
    cams, _, _ = synth_cameras(rng, subjects)
    cz = {}
    for (s, ci), (R, T, f, c, k, p, name) in cams.items():
        pre = "subject%d/camera%d/" % (s, ci)
        cz[pre + "R"] = R.T
        cz[pre + "T"], cz[pre + "f"], cz[pre + "c"], cz[pre + "k"], cz[pre + "p"] = T, f, c, k, p
        cz[pre + "Name"] = np.array([ord(ch) for ch in name], np.int64)
    np.savez(cams_path, **cz)
    tree, world = {}, {}
    for s in subjects:
        for a in actions:
            for seq in ("%s 1.h5" % a, "%s.h5" % a):
                P = synth_world_poses(rng, frames + int(rng.integers(0, 17)))
                tree["S%d/MyPoses/3D_positions/%s" % (s, seq)] = P.T
                world[(s, a, seq)] = P
                if sh:
                    for ci, cname in enumerate(CAM_NAMES):
                        if s == 11 and a == "Directions" and seq == "%s.h5" % a and ci == 3:
                            continue   # the reference's damaged video
                        fn = (seq[:-3] + "." + cname + ".h5").replace(" ", "_")
                        tree["S%d/StackedHourglass/%s" % (s, fn)] = rng.normal(500, 100, (len(P), 16, 2))
            if decoys and a == "Sitting" and "SittingDown" not in actions:
                tree["S%d/MyPoses/3D_positions/SittingDown 1.h5" % s] = synth_world_poses(rng, 5).T
                if sh:
                    tree["S%d/StackedHourglass/SittingDown_1.%s.h5" % (s, CAM_NAMES[0])] = rng.normal(0, 1, (5, 16, 2))
        if decoys:
            tree["S%d/MyPoses/2D_positions/%s" % (s, "Walking 1.h5")] = synth_world_poses(rng, 3)[:, :64].T
    np.savez(tree_path, **tree)
    return cams, world
