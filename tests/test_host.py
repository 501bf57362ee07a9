"""CPU: host-side logic (synthetic batches, parameter packing, work model, sharding)."""
import numpy as np
import pytest

from mpcqp import params as P
from mpcqp.roofline import algorithmic_flops, input_bytes
from mpcqp.synthetic import gait_table, make_batch


def test_synthetic_batch_shapes_and_ranges():
    bt = make_batch(32, 10, seed=3, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                    tilt_deg=15.0)
    assert bt["x0"].shape == (32, 13) and bt["x0"].dtype == np.float32
    assert bt["xref"].shape == (32, 10, 13)
    assert bt["contact"].shape == (32, 10, 4)
    assert bt["feet"].shape == (32, 4, 3)
    assert bt["robot"].shape == (32, P.ROBOT_STRIDE)
    assert np.all(bt["x0"][:, 12] == np.float32(-9.81))
    assert np.all(np.abs(bt["x0"][:, :2]) <= 0.1)
    # every benchmark gait has exactly two stance legs per step -> n = 6N
    assert np.all(bt["contact"].sum(axis=2) == 2)
    n = np.linalg.norm(bt["robot"][:, 9:12], axis=1)
    np.testing.assert_allclose(n, 1.0, rtol=1e-6)
    tilt = np.degrees(np.arccos(bt["robot"][:, 11]))
    assert tilt.max() <= 15.0 + 1e-3
    again = make_batch(32, 10, seed=3, gaits=("trot10", "pace10", "bound8"), robots=("a1", "aliengo"),
                       tilt_deg=15.0)
    for k in bt:
        np.testing.assert_array_equal(bt[k], again[k])


def test_bound_gait_synthesised_from_commented_definition():
    """gait.py:20 (commented): offsets [4,4,0,0], durations 4, period 8."""
    t = gait_table("bound8", 0, 8)
    assert t.shape == (8, 4)
    np.testing.assert_array_equal(t[:, 0], t[:, 1])
    np.testing.assert_array_equal(t[:, 2], t[:, 3])
    np.testing.assert_array_equal(t[:, 0], 1 - t[:, 2])


def test_pack_robot_layout():
    rec = P.pack_robot(P.ROBOT_PRESETS["a1"])
    assert rec.dtype == np.float32 and rec.shape == (16,)
    assert rec[P.R_MASS] == np.float32(4.713)
    assert rec[P.R_IXX] == np.float32(np.float32(0.01683993) * np.float32(10))
    assert rec[P.R_MU] == np.float32(0.7) and rec[P.R_FZMAX] == 500.0
    assert tuple(rec[P.R_NX:P.R_NZ + 1]) == (0.0, 0.0, 1.0)


def test_robot_from_config_class():
    class FakeAliengo:   # duck-typed RobotConfig (robot_configs.py:44-60)
        mass_base = 9.042
        fz_max = 500.0
        base_inertia_base = np.array([[1, 2, 3], [2, 4, 5], [3, 5, 6]], dtype=np.float32)
    rec = P.robot_from_config(FakeAliengo)
    assert rec[P.R_MASS] == np.float32(9.042)
    assert list(rec[P.R_IXX:P.R_IZZ + 1]) == [1, 2, 3, 4, 5, 6]


def test_work_model_matches_survey_figures():
    """at n = 12N, K = 50 the algorithmic work is 6.37 / 22.6 / 42.0 MFLOP."""
    for N, mf in ((10, 6.37), (16, 22.6), (20, 42.0)):
        assert abs(algorithmic_flops(N, 12 * N, 50) / 1e6 - mf) / mf < 0.01
    assert input_bytes(10) == 4 * (13 + 130 + 40 + 12 + 16) + 56


@pytest.mark.parametrize("total,world", [(10, 3), (1024, 8), (7, 8), (0, 2)])
def test_shard_partition(total, world):
    from mpcqp.dist import shard
    ranges = [shard(total, r, world) for r in range(world)]
    assert sum(c for _, c in ranges) == total
    pos = 0
    for s, c in ranges:
        assert s == pos
        pos += c
