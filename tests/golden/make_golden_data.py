"""Golden vectors for the H3.6M data pipeline, made by importing the REFERENCE's modules.

Run in the build container only (the reference is not on the GPU box):

    /opt/conda/bin/python3.9 tests/golden/make_golden_data.py

Drives the reference's own functions on synthetic cameras and poses (the H3.6M
``cameras.h5`` and pose files are not in the image):

* ``cameras.project_point_radial``   (src/cameras.py:13-53)
* ``cameras.world_to_camera_frame``  (src/cameras.py:55-72)
* ``cameras.camera_to_world_frame``  (src/cameras.py:74-90)
* ``data_utils.transform_world_to_camera`` (src/data_utils.py:233-257)
* ``data_utils.project_to_cameras``  (src/data_utils.py:339-364)
* ``data_utils.postprocess_3d``      (src/data_utils.py:474-494)
* ``data_utils.normalization_stats`` mean / std on a larger matrix (src/data_utils.py:195-230)

Output: tests/golden/reference_goldens_data.npz (inputs and expected outputs only).
"""
import os
import sys

import numpy as np

REF = "/root/reference/src"
sys.path.insert(0, REF)
import matplotlib  # noqa: E402

matplotlib.use("Agg")
import cameras  # noqa: E402  (reference module)
import data_utils  # noqa: E402  (reference module)

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from synth_cameras import synth_cameras, synth_world_poses  # noqa: E402

out = {}
rng = np.random.default_rng(20240907)
cams, cam_arr, names = synth_cameras(rng, subjects=(9, 11))
out["cams"] = cam_arr                       # [2 subjects, 4 cameras, 21]: R9 T3 f2 c2 k3 p2
out["cam_names"] = np.array(names)          # [2, 4] camera names

# --- per-point camera functions (one camera, including points near the optical axis) ----
P = rng.normal(0, 400, (300, 3))
P[:5] = 0.0                                 # the world origin: the camera looks at it
R, T, f, c, k, p, name = cams[(9, 1)]
proj, D, radial, tan, r2 = cameras.project_point_radial(P, R, T, f, c, k, p)
out.update(pp_in=P, pp_proj=proj, pp_depth=D, pp_radial=radial, pp_tan=tan, pp_r2=r2)
Xc = cameras.world_to_camera_frame(P, R, T)
out.update(w2c_out=Xc, c2w_out=cameras.camera_to_world_frame(Xc, R, T))

# --- dictionary-level pipeline: 2 subjects x 2 sequences of world-frame 32-joint poses ---
world = {}
for subj, seq, n in [(9, "Walking 1.h5", 37), (9, "Walking.h5", 20), (11, "Eating 2.h5", 64), (11, "Eating.h5", 5)]:
    world[(subj, seq.split(" ")[0].split(".")[0], seq)] = synth_world_poses(rng, n)
keys = sorted(world)
for i, key in enumerate(keys):
    out["world_%d" % i] = world[key]
out["world_keys"] = np.array(["%d|%s|%s" % key for key in keys])

cam3d = data_utils.transform_world_to_camera(dict(world), cams)
proj2d = data_utils.project_to_cameras(dict(world), cams)
ckeys = sorted(cam3d)
out["cam_keys"] = np.array(["%d|%s|%s" % key for key in ckeys])
for i, key in enumerate(ckeys):
    out["cam3d_%d" % i] = cam3d[key]
    out["proj2d_%d" % i] = proj2d[key]
centred, roots = data_utils.postprocess_3d({key: cam3d[key].copy() for key in ckeys})
for i, key in enumerate(ckeys):
    out["centred_%d" % i] = centred[key]
    out["root_%d" % i] = roots[key]

# --- normalization_stats mean / std on a stacked matrix -----------------------------------
stacked = np.vstack([proj2d[key] for key in ckeys])
m2, s2, _, _ = data_utils.normalization_stats(stacked, dim=2)
out.update(ms_mean=m2, ms_std=s2)   # input: the proj2d_* arrays stacked in cam_keys order

np.savez_compressed(os.path.join(HERE, "reference_goldens_data.npz"), **out)
print("wrote", len(out), "arrays")
