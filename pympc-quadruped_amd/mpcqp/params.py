"""Problem constants and per-robot parameter packing.

Constants restate the reference's configuration classes:
  LinearMpcConfig  -- config/linear_mpc_configs.py:4-24 (Q, R, mu, g, horizon)
  AliengoConfig    -- config/robot_configs.py:44-60
  A1Config         -- config/robot_configs.py:63-79 (inertia x10 at :73)
  dt = 0.05        -- hard-coded in ModelPredictiveController (mpc.py:38)
Gaits restate linear_mpc/gait.py:16-22 (+ the commented BOUNDING8 at :20).
"""
import numpy as np

# state weights: r, p, y, x, y, z, wx, wy, wz, vx, vy, vz, g   (linear_mpc_configs.py:19)
Q_DIAG = (5., 5., 10., 10., 10., 50., 0.01, 0.01, 0.2, 0.2, 0.2, 0.2, 0.)
R_DIAG = (1e-5,) * 12                                          # linear_mpc_configs.py:20
DT_MPC = 0.05                                                  # mpc.py:38
GRAVITY = 9.81                                                 # linear_mpc_configs.py:13
MU = 0.7                                                       # linear_mpc_configs.py:15

# per-robot parameter record (float32 x ROBOT_STRIDE), consumed by the kernel
ROBOT_STRIDE = 16
R_MASS, R_IXX, R_IXY, R_IXZ, R_IYY, R_IYZ, R_IZZ, R_MU, R_FZMAX, R_NX, R_NY, R_NZ = range(12)


def _inertia(ixx, ixy, ixz, iyy, iyz, izz, scale=1.0):
    # make_com_inertial_matrix (utils/dynamics.py:3-18) stores float32; A1 scales
    # the float32 matrix by 10 in float32 (robot_configs.py:73)
    m = np.array([ixx, ixy, ixz, iyy, iyz, izz], dtype=np.float32)
    return m * np.float32(scale) if scale != 1.0 else m


ROBOT_PRESETS = {
    "aliengo": dict(mass=9.042, height=0.38, fz_max=500.0, mu=MU,
                    inertia=_inertia(0.033260231, -0.000451628, 0.000487603,
                                     0.16117211, 4.8356e-05, 0.17460442)),
    "a1": dict(mass=4.713, height=0.42, fz_max=500.0, mu=MU,
               inertia=_inertia(0.01683993, 8.3902e-05, 0.000597679,
                                0.056579028, 2.5134e-05, 0.064713601, scale=10)),
}

# hip x offset, hip y + thigh y offset (a1.urdf:90,212,254; aliengo.urdf:99,254,297)
HIP_OFFSETS = {"a1": (0.183, 0.047 + 0.08505), "aliengo": (0.2399, 0.051 + 0.083)}

# name: (period, stance offsets, stance durations)    linear_mpc/gait.py:16-22
GAITS = {
    "standing": (16, (0, 0, 0, 0), (16, 16, 16, 16)),
    "trot16": (16, (0, 8, 8, 0), (8, 8, 8, 8)),
    "trot10": (10, (0, 5, 5, 0), (5, 5, 5, 5)),
    "jump16": (16, (0, 0, 0, 0), (4, 4, 4, 4)),
    "bound8": (8, (4, 4, 0, 0), (4, 4, 4, 4)),      # commented out at gait.py:20
    "pace16": (16, (8, 0, 8, 0), (8, 8, 8, 8)),
    "pace10": (10, (5, 0, 5, 0), (5, 5, 5, 5)),
}


# Gait enum member names (gait.py:16-22) -> GAITS keys
GAIT_MEMBERS = {"STANDING": "standing", "TROTTING16": "trot16", "TROTTING10": "trot10",
                "JUMPING16": "jump16", "PACING16": "pace16", "PACING10": "pace10", "BOUNDING8": "bound8"}


def gait_record(gait):
    """One MPCQP_GAIT_STRIDE record: [period, offsets[4], durations[4]] int32.

    ``gait`` is a GAITS key, a Gait enum member name, or a (period, offsets,
    durations) triple."""
    if isinstance(gait, str):
        period, offsets, durations = GAITS[GAIT_MEMBERS.get(gait, gait)]
    else:
        period, offsets, durations = gait
    rec = np.array([period, *offsets, *durations], dtype=np.int32)
    if rec.shape != (9,) or rec[0] <= 0:
        raise ValueError(f"bad gait {gait!r}")
    return rec


def pack_robot(preset, normal=(0.0, 0.0, 1.0), mu=None, fz_max=None):
    """One robot record: [mass, ixx, ixy, ixz, iyy, iyz, izz, mu, fz_max, nx, ny, nz, 0...]."""
    rec = np.zeros(ROBOT_STRIDE, dtype=np.float32)
    rec[R_MASS] = preset["mass"]
    rec[R_IXX:R_IZZ + 1] = preset["inertia"]
    rec[R_MU] = preset["mu"] if mu is None else mu
    rec[R_FZMAX] = preset["fz_max"] if fz_max is None else fz_max
    rec[R_NX:R_NZ + 1] = normal
    return rec


def robot_from_config(robot_config, mu=MU, normal=(0.0, 0.0, 1.0)):
    """Pack a reference RobotConfig class (robot_configs.py:32-79) into a record."""
    I = np.asarray(robot_config.base_inertia_base, dtype=np.float32)
    preset = dict(mass=float(robot_config.mass_base), fz_max=float(robot_config.fz_max), mu=mu,
                  inertia=np.array([I[0, 0], I[0, 1], I[0, 2], I[1, 1], I[1, 2], I[2, 2]],
                                   dtype=np.float32))
    return pack_robot(preset, normal=normal)
