"""The data-pipeline oracle (oracle/ref_data.py) against the reference's own outputs
(tests/golden/reference_goldens_data.npz, made by tests/golden/make_golden_data.py)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from oracle import ref_data  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "reference_goldens_data.npz"), allow_pickle=False)


def golden_cams():
    cams = {}
    for si, subj in enumerate((9, 11)):
        for ci in range(4):
            v = G["cams"][si, ci]
            cams[(subj, ci + 1)] = (v[:9].reshape(3, 3), v[9:12].reshape(3, 1), v[12:14].reshape(2, 1),
                                    v[14:16].reshape(2, 1), v[16:19].reshape(3, 1), v[19:21].reshape(2, 1),
                                    str(G["cam_names"][si, ci]))
    return cams


def keyed(prefix, keyname):
    out = {}
    for i, k in enumerate(G[keyname]):
        s, a, q = str(k).split("|")
        out[(int(s), a, q)] = G["%s_%d" % (prefix, i)]
    return out


def test_project_point_radial_matches_reference():
    R, T, f, c, k, p, _ = golden_cams()[(9, 1)]
    proj, D, radial, tan, r2 = ref_data.project_point_radial(G["pp_in"], R, T, f, c, k, p)
    # bit-exact except where numpy's BLAS dot / libm pow round differently: 1e-12 relative
    np.testing.assert_allclose(proj, G["pp_proj"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(D, G["pp_depth"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(radial, G["pp_radial"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(tan, G["pp_tan"], rtol=1e-12, atol=1e-18)
    np.testing.assert_allclose(r2, G["pp_r2"], rtol=1e-12, atol=0)


def test_camera_frames_match_reference():
    R, T, *_ = golden_cams()[(9, 1)]
    Xc = ref_data.world_to_camera_frame(G["pp_in"], R, T)
    np.testing.assert_allclose(Xc, G["w2c_out"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(ref_data.camera_to_world_frame(G["w2c_out"], R, T), G["c2w_out"], rtol=1e-12, atol=1e-9)


def test_dict_pipeline_matches_reference():
    cams = golden_cams()
    world = keyed("world", "world_keys")
    cam3d = ref_data.transform_world_to_camera(world, cams)
    proj2d = ref_data.project_to_cameras(world, cams)
    g3, g2 = keyed("cam3d", "cam_keys"), keyed("proj2d", "cam_keys")
    assert sorted(cam3d) == sorted(g3) and sorted(proj2d) == sorted(g2)
    for key in g3:
        np.testing.assert_allclose(cam3d[key], g3[key], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(proj2d[key], g2[key], rtol=1e-12, atol=0)
    centred, roots = ref_data.postprocess_3d(g3)
    gc, gr = keyed("centred", "cam_keys"), keyed("root", "cam_keys")
    for key in g3:
        np.testing.assert_array_equal(centred[key], gc[key])   # pure subtraction: bit-exact
        np.testing.assert_array_equal(roots[key], gr[key])


def test_moments_match_reference():
    stacked = np.vstack([G["proj2d_%d" % i] for i in range(len(G["cam_keys"]))])
    mean, std = ref_data.moments(stacked)
    np.testing.assert_array_equal(mean, G["ms_mean"])
    np.testing.assert_array_equal(std, G["ms_std"])


@pytest.mark.parametrize("name", ["pp_proj", "w2c_out"])
def test_golden_shapes(name):
    assert G[name].shape[0] == G["pp_in"].shape[0]
