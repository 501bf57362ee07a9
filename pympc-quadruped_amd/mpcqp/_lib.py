"""ctypes binding of libmpcqp.so (include/mpcqp.h).

The shared library is built in-tree (``__graft_entry__.build()`` or
``python -m mpcqp.build``) next to this file.  There is deliberately no
fallback: if the library is missing or fails to load, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPCQP_LIB: diagnostic override (A/B builds); the default is the in-tree build
LIB_PATH = os.environ.get("MPCQP_LIB") or os.path.join(_HERE, "libmpcqp.so")

MPCQP_OK = 0
ERR_ARG = -1
ERR_HIP = -2
ERR_ALLOC = -3
STATUS_OK = 0
STATUS_MAX_ITER = 1
STATUS_INFEASIBLE = 2
STATUS_TOO_LARGE = 3
STATUS_NONFINITE = 4
STATUS_UNSUPPORTED = 5
ROBOT_STRIDE = 16
MAX_HORIZON = 32    # MPCQP_MAX_HORIZON: mpcqp_create rejects a longer horizon

# every symbol declared in include/mpcqp.h
EXPORTED_SYMBOLS = (
    "mpcqp_abi_version",
    "mpcqp_default_params",
    "mpcqp_create",
    "mpcqp_solve",
    "mpcqp_set_stance_hint",
    "mpcqp_set_stance_range",
    "mpcqp_set_order",
    "mpcqp_set_weights",
    "mpcqp_set_warm_start",
    "mpcqp_destroy",
    "mpcqp_last_error",
    "mpcqp_plan",
    "mpcqp_plan_root_states",
    "mpcqp_set_planner",
    "mpcqp_stance_torques",
)
ABI_VERSION = 6
WARM_BYTES = 128     # MPCQP_WARM_BYTES: warm-start memory per robot
PLAN_STRIDE = 8     # MPCQP_PLAN_STRIDE: float64 planner state per robot
GAIT_STRIDE = 9     # MPCQP_GAIT_STRIDE: period, offsets[4], durations[4]
PLAN_REFERENCE = 1      # MPCQP_PLAN_REFERENCE: build X_ref (+ gait table) this tick
PLAN_NO_INTEGRATE = 2   # MPCQP_PLAN_NO_INTEGRATE: skip the desired-pose integrators


class MpcqpParams(ctypes.Structure):
    """struct mpcqp_params (include/mpcqp.h)."""
    _fields_ = [
        ("horizon", ctypes.c_int32),
        ("max_iter", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("q_diag", ctypes.c_double * 13),
        ("r_diag", ctypes.c_double * 12),
    ]


class MpcqpError(RuntimeError):
    pass


_lib = None


def load():
    """Load libmpcqp.so once; raise MpcqpError if it is absent (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcqpError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                         "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i32, f32p, i32p = ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p
    lib.mpcqp_abi_version.restype = i32
    lib.mpcqp_abi_version.argtypes = []
    lib.mpcqp_default_params.restype = None
    lib.mpcqp_default_params.argtypes = [ctypes.POINTER(MpcqpParams), i32]
    lib.mpcqp_create.restype = ctypes.c_int
    lib.mpcqp_create.argtypes = [ctypes.POINTER(MpcqpParams), i32, ctypes.POINTER(vp)]
    lib.mpcqp_solve.restype = ctypes.c_int
    lib.mpcqp_solve.argtypes = [vp, i32, f32p, f32p, f32p, f32p, f32p, f32p, f32p, i32p, i32p, vp]
    lib.mpcqp_set_stance_hint.restype = ctypes.c_int
    lib.mpcqp_set_stance_hint.argtypes = [vp, i32]
    lib.mpcqp_set_stance_range.restype = ctypes.c_int
    lib.mpcqp_set_stance_range.argtypes = [vp, i32, i32]
    lib.mpcqp_set_order.restype = ctypes.c_int
    lib.mpcqp_set_order.argtypes = [vp, i32]
    lib.mpcqp_set_weights.restype = ctypes.c_int
    lib.mpcqp_set_weights.argtypes = [vp, vp, vp]
    lib.mpcqp_set_warm_start.restype = ctypes.c_int
    lib.mpcqp_set_warm_start.argtypes = [vp, vp, i32]
    lib.mpcqp_destroy.restype = ctypes.c_int
    lib.mpcqp_destroy.argtypes = [vp]
    lib.mpcqp_last_error.restype = ctypes.c_char_p
    lib.mpcqp_last_error.argtypes = [vp]
    lib.mpcqp_plan.restype = ctypes.c_int
    lib.mpcqp_plan.argtypes = [vp, i32, i32] + [vp] * 14 + [vp]
    lib.mpcqp_plan_root_states.restype = ctypes.c_int
    lib.mpcqp_plan_root_states.argtypes = [vp, i32, i32] + [vp] * 10 + [vp]
    lib.mpcqp_set_planner.restype = ctypes.c_int
    lib.mpcqp_set_planner.argtypes = [vp, ctypes.c_double, ctypes.c_double, ctypes.c_double]
    lib.mpcqp_stance_torques.restype = ctypes.c_int
    lib.mpcqp_stance_torques.argtypes = [vp, i32, vp, vp, i32, vp, vp, vp]
    if lib.mpcqp_abi_version() != ABI_VERSION:
        raise MpcqpError("libmpcqp ABI version mismatch")
    _lib = lib
    return lib


def default_params(horizon):
    p = MpcqpParams()
    load().mpcqp_default_params(ctypes.byref(p), int(horizon))
    return p


def lib_sha256(path=None):
    """SHA-256 of the engine library file (ties a profile's counters to the build that made them)."""
    import hashlib
    with open(path or LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def check(ctx, code, what):
    if code != MPCQP_OK:
        msg = load().mpcqp_last_error(ctx) if ctx else b""
        raise MpcqpError(f"{what} failed ({code}): {msg.decode() if msg else ''}")
