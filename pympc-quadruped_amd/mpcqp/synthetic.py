"""Seeded synthetic robot batches, host-side NumPy.

Produces exactly the inputs the reference's ``_solve_mpc`` consumes, batched:
  x0[B,13] f32, xref[B,N,13] f32, contact[B,N,4] f32, feet[B,4,3] f32,
  robot[B, ROBOT_STRIDE] f32 (mass, inertia(6), mu, fz_max, normal(3)).

The contact rule follows ``Gait.get_gait_table`` (linear_mpc/gait.py:81-100);
the bounding gait is synthesised from the commented definition at gait.py:20.
The reference trajectory follows ``generate_reference_trajectory``
(linear_mpc/mpc.py:110-170) on a controller's first MPC tick.
"""
import math

import numpy as np

from .params import GAITS, ROBOT_PRESETS, pack_robot, HIP_OFFSETS

STATE_DIM = 13


def gait_table(gait, iteration, horizon):
    """gait.py:81-100 for one robot: (horizon, 4) float32, 1 = stance."""
    period, offsets, durations = GAITS[gait]
    table = np.zeros((horizon, 4), dtype=np.float32)
    for i in range(horizon):
        i_h = (i + 1 + iteration) % period
        for leg in range(4):
            seg = i_h - offsets[leg]
            if seg < 0:
                seg += period
            table[i, leg] = 1.0 if seg < durations[leg] else 0.0
    return table


def reference_trajectory(x0, v_des_world, yaw_rate, xy_des, yaw_des, roll_init, pitch_init,
                         height, horizon, dt=0.05, gravity=9.81):
    """mpc.py:110-170 for one robot, first-tick semantics; returns (horizon*13,) f32."""
    cx, cy = xy_des
    max_err = 0.1
    if cx - x0[3] > max_err:
        cx = x0[3] + max_err
    if x0[3] - cx > max_err:
        cx = x0[3] - max_err
    if cy - x0[4] > max_err:
        cy = x0[4] + max_err
    if x0[4] - cy > max_err:
        cy = x0[4] - max_err
    if abs(x0[9]) > 0.2:
        pitch_init += dt * (0.0 - x0[1]) / x0[9]
    if abs(x0[10]) > 0.1:
        roll_init += dt * (0.0 - x0[0]) / x0[10]
    roll_init = min(max(roll_init, -0.25), 0.25)
    pitch_init = min(max(pitch_init, -0.25), 0.25)
    roll_comp = x0[10] * roll_init
    pitch_comp = x0[9] * pitch_init
    X = np.zeros(STATE_DIM * horizon, dtype=np.float32)
    X[0::13] = roll_comp
    X[1::13] = pitch_comp
    X[2] = yaw_des
    X[3] = cx
    X[4] = cy
    X[5::13] = height
    X[8::13] = yaw_rate
    X[9::13] = v_des_world[0]
    X[10::13] = v_des_world[1]
    X[12::13] = -gravity
    for i in range(1, horizon):
        X[2 + 13 * i] = X[2 + 13 * (i - 1)] + dt * yaw_rate
        X[3 + 13 * i] = X[3 + 13 * (i - 1)] + dt * v_des_world[0]
        X[4 + 13 * i] = X[4 + 13 * (i - 1)] + dt * v_des_world[1]
    return X


def make_batch(batch, horizon, seed=0, gaits=("trot10",), robots=("a1",), tilt_deg=0.0,
               gravity=9.81, dt=0.05):
    """Seeded batch of B robots (SURVEY §8(d) distributions).

    gaits / robots are sampled uniformly per robot from the given tuples.
    tilt_deg > 0 draws a per-robot friction-cone normal tilted by U(0, tilt).
    """
    rng = np.random.default_rng(seed)
    B, N = batch, horizon
    x0 = np.zeros((B, 13), dtype=np.float32)
    xref = np.zeros((B, N, 13), dtype=np.float32)
    contact = np.zeros((B, N, 4), dtype=np.float32)
    feet = np.zeros((B, 4, 3), dtype=np.float32)
    robot = np.zeros((B, len(pack_robot(ROBOT_PRESETS["a1"]))), dtype=np.float32)
    gait_ids = rng.integers(0, len(gaits), size=B)
    robot_ids = rng.integers(0, len(robots), size=B)
    for b in range(B):
        rp = ROBOT_PRESETS[robots[robot_ids[b]]]
        h = rp["height"]
        roll, pitch = rng.uniform(-0.1, 0.1, size=2)
        yaw = rng.uniform(-math.pi, math.pi)
        px, py = rng.uniform(-1, 1, size=2)
        pz = h + rng.uniform(-0.03, 0.03)
        w = rng.normal(0, 0.3, size=3)
        v = np.array([rng.uniform(-0.5, 1.5), rng.uniform(-0.3, 0.3), rng.normal(0, 0.05)])
        x0[b] = [roll, pitch, yaw, px, py, pz, *w, *v, -gravity]
        # desired command: body-frame velocity rotated by yaw (mpc.py:83)
        vb = np.array([rng.uniform(0, 1.5), 0.0])
        c, s = math.cos(yaw), math.sin(yaw)
        v_world = (c * vb[0] - s * vb[1], s * vb[0] + c * vb[1])
        yaw_rate = rng.uniform(-0.5, 0.5)
        xy_des = (float(x0[b, 3]) + rng.uniform(-0.15, 0.15),
                  float(x0[b, 4]) + rng.uniform(-0.15, 0.15))
        xref[b] = reference_trajectory(x0[b], v_world, yaw_rate, xy_des, float(x0[b, 2]),
                                       0.0, 0.0, h, N, dt, gravity).reshape(N, 13)
        g = gaits[gait_ids[b]]
        period = GAITS[g][0]
        contact[b] = gait_table(g, int(rng.integers(0, period)), N)
        hx, hy = HIP_OFFSETS[robots[robot_ids[b]]]
        for leg, (sx, sy) in enumerate(((1, 1), (1, -1), (-1, 1), (-1, -1))):
            body = np.array([sx * hx, sy * hy, -h]) + rng.uniform(-0.05, 0.05, size=3)
            feet[b, leg] = [c * body[0] - s * body[1], s * body[0] + c * body[1], body[2]]
        normal = (0.0, 0.0, 1.0)
        if tilt_deg > 0:
            th = math.radians(rng.uniform(0, tilt_deg))
            az = rng.uniform(0, 2 * math.pi)
            normal = (math.sin(th) * math.cos(az), math.sin(th) * math.sin(az), math.cos(th))
        robot[b] = pack_robot(rp, normal=normal)
    return dict(x0=x0, xref=xref, contact=contact, feet=feet, robot=robot)
