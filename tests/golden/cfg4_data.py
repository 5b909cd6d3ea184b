"""The cfg4 evaluation set (BASELINE.json configs[3]) as bench.py's eval_sweep draws it:
15 actions, frames per action ~ U[20000, 40000] from default_rng(4) (494,784 frames after the
reference's per-action n % 64 tail drop), here as H3.6M-keyed dicts (subject, action,
"<seq>.<camera>.h5") split over both test subjects and four sequences, normalized N(0, 1)
2D inputs / 3D targets; weights of the cfg2 network: oracle init_state(seed=1, bn_seed=2);
3D statistics: oracle synthetic_stats() (mean U(-500, 500) mm, std U(50, 300) mm).
Deterministic (numpy PCG64 streams): the oracle's per-action MPJPE is a committed fixture
(cfg4_oracle.npz, make_cfg4_oracle.py) that the GPU test compares against."""
import numpy as np

ACTIONS = ["Directions", "Discussion", "Eating", "Greeting", "Phoning", "Photo", "Posing", "Purchases", "Sitting",
           "SittingDown", "Smoking", "Waiting", "WalkDog", "Walking", "WalkTogether"]


def make_cfg4_set(seed=4, data_seed=40):
    counts = np.random.default_rng(seed).integers(20000, 40001, 15)
    rng = np.random.default_rng(data_seed)
    s2, s3 = {}, {}
    for a, n in zip(ACTIONS, counts):
        n = int(n)
        cuts = np.sort(rng.choice(np.arange(1, n), size=3, replace=False))
        for j, p in enumerate(np.split(np.arange(n), cuts)):
            key = ((9, 11)[j % 2], a, "%s %d.5486%04d.h5" % (a, j, j))
            s2[key] = rng.standard_normal((len(p), 32))
            s3[key] = rng.standard_normal((len(p), 48))
    return s2, s3
