"""The H3.6M loaders over the .npz archive form of the tree and of cameras.h5 (host logic, no
GPU): the reference's file selection rules and counts (src/data_utils.py:61-117, :120-192),
the camera parameter layout (src/cameras.py:92-140)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import cameras  # noqa: E402
import data_utils  # noqa: E402
from synth_cameras import write_h36m_archives  # noqa: E402


@pytest.fixture
def archives(tmp_path):
    rng = np.random.default_rng(11)
    tree, cams = str(tmp_path / "h36m.npz"), str(tmp_path / "cameras.npz")
    rcams, world = write_h36m_archives(tree, cams, rng, ["Sitting", "Walking", "Directions"], frames=20, sh=True)
    return tree, cams, rcams, world


def test_load_data_selection_rules(archives):
    tree, _, _, world = archives
    got = data_utils.load_data(tree, data_utils.TRAIN_SUBJECTS, ["Sitting", "Walking"], dim=3)
    want = {k: v for k, v in world.items() if k[0] in data_utils.TRAIN_SUBJECTS and k[1] in ("Sitting", "Walking")}
    assert sorted(got) == sorted(want)                       # SittingDown skipped under Sitting
    for k in want:
        np.testing.assert_array_equal(got[k], want[k])      # [96, n] as stored -> [n, 96]
    with pytest.raises(AssertionError, match="Expecting 8 sequences"):
        data_utils.load_data(tree, [1], ["Walking"], dim=2)  # one 2D file: the reference's count check
    with pytest.raises(ValueError):
        data_utils.load_data(tree, [1], ["Walking"], dim=4)


def test_load_cameras_layout(archives):
    _, cams, rcams, _ = archives
    got = cameras.load_cameras(cams, [1, 9])
    assert sorted(got) == [(1, 1), (1, 2), (1, 3), (1, 4), (9, 1), (9, 2), (9, 3), (9, 4)]
    for key, tup in got.items():
        for a, b in zip(tup[:6], rcams[key][:6]):
            np.testing.assert_array_equal(a, b)
        assert tup[6] == rcams[key][6]


def test_load_stacked_hourglass(archives):
    tree, _, _, _ = archives
    got = data_utils.load_stacked_hourglass(tree, [9, 11], ["Directions", "Sitting"])
    counts = {}
    for (s, a, q) in got:
        counts[(s, a)] = counts.get((s, a), 0) + 1
        assert q.endswith(".h5-sh") and "_" not in q
    assert counts == {(9, "Directions"): 8, (11, "Directions"): 7, (9, "Sitting"): 8, (11, "Sitting"): 8}
    # the permutation and scatter, restated: SH joint j of H3.6M joint i lands in columns 2i, 2i+1
    raw = np.load(tree)["S9/StackedHourglass/Sitting_1.54138969.h5"]
    out = got[(9, "Sitting", "Sitting 1.54138969.h5-sh")]
    names = data_utils.H36M_NAMES
    for i, n in enumerate(names):
        if n in data_utils.SH_NAMES:
            np.testing.assert_array_equal(out[:, 2 * i:2 * i + 2], raw[:, data_utils.SH_NAMES.index(n), :])
        else:
            assert not out[:, 2 * i:2 * i + 2].any()
    with pytest.raises(AssertionError, match="Expecting 8 sequences"):
        data_utils.load_stacked_hourglass(tree, [1], ["Eating"])


def test_hdf5_tree_needs_h5py(tmp_path):
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py present")
    except ImportError:
        pass
    d = tmp_path / "S1" / "MyPoses" / "3D_positions"
    d.mkdir(parents=True)
    (d / "Walking 1.h5").write_bytes(b"")
    with pytest.raises(ImportError, match="npz archive"):
        data_utils.load_data(str(tmp_path), [1], ["Walking"], dim=3)
    with pytest.raises(ImportError, match="npz archive"):
        cameras.load_cameras(str(tmp_path / "cameras.h5"), [1])
