"""CPU: the C-ABI library loads, exports every symbol include/mpcqp.h declares,
and its host-side contract holds without a GPU (no compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpcqp.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[a-zA-Z_][\w\s\*]*?)\b(mpcqp_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    from mpcqp import _lib
    assert _declared() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    from mpcqp import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.mpcqp_abi_version() == _lib.ABI_VERSION == 6


def test_params_struct_layout():
    from mpcqp import _lib
    assert ctypes.sizeof(_lib.MpcqpParams) == 4 + 4 + 8 + 13 * 8 + 12 * 8


def test_default_params_are_the_reference_config():
    """mpcqp_default_params == LinearMpcConfig (linear_mpc_configs.py:4-24) + dt (mpc.py:38)."""
    from mpcqp import _lib
    p = _lib.default_params(16)
    assert p.horizon == 16 and p.dt == 0.05 and p.max_iter == 0
    assert list(p.q_diag) == [5., 5., 10., 10., 10., 50., 0.01, 0.01, 0.2, 0.2, 0.2, 0.2, 0.]
    assert list(p.r_diag) == [1e-5] * 12


def test_create_rejects_bad_arguments_without_crashing():
    from mpcqp import _lib
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    p = _lib.default_params(0)   # horizon 0 is invalid
    assert lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)) == -1
    p = _lib.default_params(10)
    # device -1 never exists: an error code, never an exception or a crash
    assert lib.mpcqp_create(ctypes.byref(p), -1, ctypes.byref(ctx)) != 0
    assert lib.mpcqp_solve(None, 1, None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.mpcqp_set_stance_hint(None, 3) == -1
    assert lib.mpcqp_set_stance_range(None, 1, 3) == -1
    assert lib.mpcqp_set_order(None, 1) == -1
    assert lib.mpcqp_plan(None, 1, 1, *([None] * 15)) == -1
    assert lib.mpcqp_plan_root_states(None, 1, 1, *([None] * 11)) == -1
    assert lib.mpcqp_stance_torques(None, 1, None, None, 4, None, None, None) == -1
    assert lib.mpcqp_set_planner(None, 0.001, 9.81, 0.1) == -1
    assert lib.mpcqp_set_warm_start(None, None, 0) == -1
    assert lib.mpcqp_destroy(None) == 0


def test_header_constants_match_binding():
    """MPCQP_PLAN_STRIDE / GAIT_STRIDE / plan flags are what the Python side uses."""
    from mpcqp import _lib
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define (MPCQP_\w+) (\d+)", src))
    assert int(consts["MPCQP_PLAN_STRIDE"]) == _lib.PLAN_STRIDE
    assert int(consts["MPCQP_GAIT_STRIDE"]) == _lib.GAIT_STRIDE
    assert int(consts["MPCQP_PLAN_REFERENCE"]) == _lib.PLAN_REFERENCE
    assert int(consts["MPCQP_PLAN_NO_INTEGRATE"]) == _lib.PLAN_NO_INTEGRATE
    assert int(consts["MPCQP_ROBOT_STRIDE"]) == _lib.ROBOT_STRIDE
    assert int(consts["MPCQP_WARM_BYTES"]) == _lib.WARM_BYTES == 4 * _lib.MAX_HORIZON


def test_horizon_limit_is_the_create_limit():
    """MPCQP_MAX_HORIZON (include/mpcqp.h) is exactly what mpcqp_create accepts (the
    horizon check runs before any HIP call), and the Python surfaces raise on a longer
    horizon with the limit in the message (linear_mpc_configs.py:11 is a free value)."""
    from mpcqp import _lib, LinearMpc
    src = open(HEADER).read()
    limit = int(re.search(r"#define MPCQP_MAX_HORIZON (\d+)", src).group(1))
    assert limit == _lib.MAX_HORIZON == 32
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    p = _lib.default_params(limit + 1)
    assert lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx)) == -1   # MPCQP_ERR_ARG
    p = _lib.default_params(limit)
    rc = lib.mpcqp_create(ctypes.byref(p), 0, ctypes.byref(ctx))
    assert rc != -1   # accepted (no GPU here: MPCQP_ERR_HIP from the device query)
    if rc == 0:
        lib.mpcqp_destroy(ctx)
    with pytest.raises(ValueError, match="1..32"):
        LinearMpc(horizon=limit + 1, device="cuda:0")


def test_gait_records_are_the_reference_gaits():
    """gait.py:16-22 member names -> [period, offsets, durations]."""
    from mpcqp.params import gait_record
    assert gait_record("TROTTING10").tolist() == [10, 0, 5, 5, 0, 5, 5, 5, 5]
    assert gait_record("PACING16").tolist() == [16, 8, 0, 8, 0, 8, 8, 8, 8]
    assert gait_record("bound8").tolist() == [8, 4, 4, 0, 0, 4, 4, 4, 4]
    with pytest.raises(ValueError):
        gait_record((0, (0, 0, 0, 0), (1, 1, 1, 1)))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: a missing .so is an error, never a silent substitute."""
    from mpcqp import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "absent.so"))
    with pytest.raises(_lib.MpcqpError):
        _lib.load()


def test_engine_refuses_cpu_device():
    torch = pytest.importorskip("torch")
    from mpcqp import LinearMpc
    with pytest.raises(ValueError):
        LinearMpc(horizon=10, device="cpu")
