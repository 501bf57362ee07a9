// mpcqp_plan.h -- the hot path's callers on the device:
// state packing, the desired-pose integrators, the reference trajectory and the gait
// table of every robot in one launch, so a batched MPC tick runs without per-robot
// host work (included by mpcqp.hip inside its anonymous namespace).
//
//   pack           ModelPredictiveController.update_robot_state   mpc.py:55-79
//                  quat2ZYXangle                                   kinematics.py:40-49
//   integrate      update_mpc_if_needed (pose integrators)        mpc.py:81-92
//   reference      generate_reference_trajectory                   mpc.py:110-170
//   gait table     Gait.set_iteration / get_gait_table             gait.py:76-100
//   stance torque  LegController stance branch, tau = Jv^T (-f)    leg_controller.py:86-89
//
// Arithmetic follows the reference's types under its pinned NumPy 1.24 promotion
// rules (requirements.txt:50): the pose integrators and compensation gains are
// float64 (Python floats), the state and X_ref are float32 arrays, so each horizon
// step of X_ref is a float64 add rounded to float32 (mpc.py:165-168).  FP contraction
// is off in both kernels so every product and sum rounds exactly where NumPy's does.

// per-robot planner state (doubles): x / y desired (mpc.py:86-90), yaw desired
// (:88,91), roll / pitch compensation integrators (:143-150), first-run flag
constexpr int PL_X = 0, PL_Y = 1, PL_YAW = 2, PL_ROLL = 3, PL_PITCH = 4, PL_STARTED = 5;

struct PlanParams {
  int N;
  int mpc_tick;          // 1: also build X_ref and the gait table (iter % iterations_between_mpc == 0)
  int root_layout;       // 1: `quat` points at Isaac Gym actor root states [B][13]
  int integrate;         // 1: run the desired-pose integrators (mpc.py:84-92) first
  double dt;             // 0.05 (mpc.py:38)
  double dt_control;     // 0.001 (linear_mpc_configs.py:6)
  double gravity;        // 9.81 (linear_mpc_configs.py:13)
  double max_pos_error;  // 0.1 (mpc.py:121)
};

// A workgroup owns kPlanRobots consecutive robots.  Phase 1: one thread per robot
// does the sequential, stateful part (pack, integrate, clamp, compensate) and leaves
// the per-robot row seeds in LDS.  Phase 2: the whole workgroup writes the robots'
// X_ref and gait-table slabs as one contiguous range each, so the stores coalesce.
constexpr int kPlanRobots = 64;
constexpr int kPlanThreads = 256;

struct PlanSeed {
  double rate, vx, vy, yawd, xd, yd;
  float roll_comp, pitch_comp, height;
  int period, ih0, off[4], dur[4];
};

__global__ __launch_bounds__(kPlanThreads) void mpcqp_plan_kernel(
    PlanParams pp, int B, const float* __restrict__ quat, const float* __restrict__ pos,
    const float* __restrict__ omega, const float* __restrict__ vel, const float* __restrict__ rot,
    const double* __restrict__ vbody, const double* __restrict__ yaw_rate, const int* __restrict__ gait,
    const int* __restrict__ iteration, const float* __restrict__ height, double* __restrict__ state,
    float* __restrict__ x0, float* __restrict__ xref, float* __restrict__ contact) {
#pragma clang fp contract(off)   // every product and sum rounds, as in NumPy
  __shared__ PlanSeed seed[kPlanRobots];
  __shared__ float seq[kPlanRobots][3][kMaxN];   // yaw / x / y along the horizon
  const int N = pp.N;
  const int b0 = blockIdx.x * kPlanRobots;
  const int nrob = min(kPlanRobots, B - b0);
  const int t = threadIdx.x;

  if (t < nrob) {
    const int b = b0 + t;
    // ---- inputs: separate arrays, or one Isaac Gym actor-root-state row
    // [pos(3), quat(x, y, z, w), lin_vel(3), ang_vel(3)] (isaacgym_a1.py:119-128)
    float qw, qx, qy, qz, p3[3], w3[3], v3[3];
    if (pp.root_layout) {
      const float* rs = quat + (size_t)b * 13;
      qx = rs[3], qy = rs[4], qz = rs[5], qw = rs[6];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        p3[k] = rs[k];
        v3[k] = rs[7 + k];
        w3[k] = rs[10 + k];
      }
    } else {
      qw = quat[4 * b], qx = quat[4 * b + 1], qy = quat[4 * b + 2], qz = quat[4 * b + 3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        p3[k] = pos[3 * b + k];
        w3[k] = omega[3 * b + k];
        v3[k] = vel[3 * b + k];
      }
    }
    // ---- pack the state (mpc.py:64-76).  quat2ZYXangle (kinematics.py:40-49) on a
    // float32 quaternion: NumPy float32 scalar products and sums, each rounded (the
    // contract(off) pragma above keeps them unfused), then math.atan2 / asin in float64
    const float a_r = 2.f * ((qw * qx) + (qy * qz));
    const float b_r = (1.f - 2.f * ((qx * qx) + (qy * qy)));
    const float a_p = 2.f * ((qw * qy) - (qz * qx));
    const float a_y = 2.f * ((qw * qz) + (qx * qy));
    const float b_y = (1.f - 2.f * ((qy * qy) + (qz * qz)));
    const double roll = atan2((double)a_r, (double)b_r);
    const double pitch = asin(fmin(fmax((double)a_p, -1.0), 1.0));   // math.asin raises instead
    const double yaw = atan2((double)a_y, (double)b_y);
    float xs[NX];
    xs[0] = (float)roll;
    xs[1] = (float)pitch;
    xs[2] = (float)yaw;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      xs[3 + k] = p3[k];
      xs[6 + k] = w3[k];
      xs[9 + k] = v3[k];
    }
    xs[12] = (float)(-pp.gravity);
#pragma unroll
    for (int k = 0; k < NX; ++k) x0[(size_t)b * NX + k] = xs[k];

    // ---- desired velocity in the world frame: R_base @ v_body (mpc.py:83).  Without
    // a caller-supplied R_base it is quat2matrix(quat) (robot_data.py:75,
    // kinematics.py:51-71) in the same float32 scalar arithmetic
    float R[9];
    if (rot != nullptr) {
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = rot[9 * b + k];
    } else {
      const float ww = (qw * qw), xx = (qx * qx), yy = (qy * qy),
                  zz = (qz * qz);
      R[0] = (((ww + xx) - yy) - zz);
      R[1] = 2.f * ((qx * qy) - (qw * qz));
      R[2] = 2.f * ((qw * qy) + (qx * qz));
      R[3] = 2.f * ((qw * qz) + (qx * qy));
      R[4] = (((ww - xx) + yy) - zz);
      R[5] = 2.f * ((qy * qz) - (qw * qx));
      R[6] = 2.f * ((qx * qz) - (qw * qy));
      R[7] = 2.f * ((qw * qx) + (qy * qz));
      R[8] = (((ww - xx) - yy) + zz);
    }
    // the body-frame command is float64 (a Python list / float64 array in the scripts)
    double vdes[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      vdes[r] = (double)R[3 * r] * vbody[3 * b] + (double)R[3 * r + 1] * vbody[3 * b + 1] +
                (double)R[3 * r + 2] * vbody[3 * b + 2];
    const double rate = yaw_rate[b];

    // ---- pose integrators (mpc.py:84-92); the yaw is self.yaw = rpy[2] in float64
    double* st = state + (size_t)b * 8;
    const bool started = st[PL_STARTED] != 0.0;
    double xd, yd, yawd;
    if (pp.integrate) {
      xd = started ? st[PL_X] + pp.dt_control * vdes[0] : 0.0;
      yd = started ? st[PL_Y] + pp.dt_control * vdes[1] : 0.0;
      yawd = started ? yaw + pp.dt_control * rate : yaw;
    } else {   // generate_reference_trajectory alone (mpc.py:110) reads the last integration
      xd = st[PL_X];
      yd = st[PL_Y];
      yawd = started ? st[PL_YAW] : yaw;
    }
    double roll_init = started ? st[PL_ROLL] : 0.0;
    double pitch_init = started ? st[PL_PITCH] : 0.0;

    if (pp.mpc_tick) {
      // ---- position clamp (mpc.py:121-140)
      const double px = xs[3], py = xs[4], e = pp.max_pos_error;
      if (xd - px > e) xd = px + e;
      if (px - xd > e) xd = px - e;
      if (yd - py > e) yd = py + e;
      if (py - yd > e) yd = py - e;
      // ---- roll / pitch compensation (mpc.py:143-152), NumPy 1.x promotion: float64
      const double vx = xs[9], vy = xs[10];
      if (fabs(vx) > 0.2) pitch_init += pp.dt * (0.0 - (double)xs[1]) / vx;
      if (fabs(vy) > 0.1) roll_init += pp.dt * (0.0 - (double)xs[0]) / vy;
      roll_init = fmin(fmax(roll_init, -0.25), 0.25);
      pitch_init = fmin(fmax(pitch_init, -0.25), 0.25);
      PlanSeed& sd = seed[t];
      sd.rate = rate;
      sd.vx = vdes[0];
      sd.vy = vdes[1];
      sd.yawd = yawd;
      sd.xd = xd;
      sd.yd = yd;
      sd.roll_comp = (float)(vy * roll_init);
      sd.pitch_comp = (float)(vx * pitch_init);
      sd.height = height[b];
      if (gait != nullptr) {
        const int* gs = gait + 9 * b;   // period, offsets[4], durations[4] (gait.py:16-22)
        sd.period = gs[0];
        sd.ih0 = iteration[b];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          sd.off[l] = gs[1 + l];
          sd.dur[l] = gs[5 + l];
        }
      }
    }
    st[PL_X] = xd;
    st[PL_Y] = yd;
    st[PL_YAW] = yawd;
    st[PL_ROLL] = roll_init;
    st[PL_PITCH] = pitch_init;
    if (pp.integrate) st[PL_STARTED] = 1.0;
  }
  if (!pp.mpc_tick) return;   // uniform over the workgroup
  __syncthreads();

  // ---- yaw / x / y along the horizon (mpc.py:165-168) accumulate in float32
  // storage, each step a float64 add rounded: a serial recursion, one thread per
  // (robot, component), into LDS
  if (t < 3 * nrob) {
    const int r = t / 3, c = t - 3 * (t / 3);
    const PlanSeed& sd = seed[r];
    const double step = pp.dt * (c == 0 ? sd.rate : (c == 1 ? sd.vx : sd.vy));
    float a = (float)(c == 0 ? sd.yawd : (c == 1 ? sd.xd : sd.yd));
    float* q = seq[r][c];
    q[0] = a;
    for (int i = 1; i < N; ++i) {
      a = (float)((double)a + step);
      q[i] = a;
    }
  }
  __syncthreads();

  // ---- X_ref rows (mpc.py:154-168) and gait-table rows (gait.py:81-100): one
  // thread per (robot, horizon step); a wave's 64 rows are one contiguous range,
  // so its 13 row stores merge in L2 and the gait row is one 16-byte store
  const int rows = nrob * N;
  for (int row = t; row < rows; row += kPlanThreads) {
    const int r = row / N, i = row - r * N;
    const PlanSeed& sd = seed[r];
    float* xr = xref + ((size_t)b0 * N + row) * NX;
    xr[0] = sd.roll_comp;
    xr[1] = sd.pitch_comp;
    xr[2] = seq[r][0][i];
    xr[3] = seq[r][1][i];
    xr[4] = seq[r][2][i];
    xr[5] = sd.height;
    xr[6] = 0.f;
    xr[7] = 0.f;
    xr[8] = (float)sd.rate;
    xr[9] = (float)sd.vx;
    xr[10] = (float)sd.vy;
    xr[11] = 0.f;
    xr[12] = (float)(-pp.gravity);
    if (gait == nullptr) continue;   // the caller supplies its own gait table
    // stance when the leg's segment, offset-shifted into [0, period), is inside its
    // stance duration; a malformed gait (period <= 0) schedules no stance
    const int p = sd.period;
    float c[4] = {0.f, 0.f, 0.f, 0.f};
    if (p > 0) {
      int ih = (i + 1 + sd.ih0) % p;
      if (ih < 0) ih += p;
#pragma unroll
      for (int leg = 0; leg < 4; ++leg) {
        int seg = ih - sd.off[leg];
        if (seg < 0) seg += p;
        c[leg] = seg < sd.dur[leg] ? 1.f : 0.f;
      }
    }
    *reinterpret_cast<float4*>(contact + ((size_t)b0 * N + row) * 4) = make_float4(c[0], c[1], c[2], c[3]);
  }
}

// tau_leg = Jv_leg^T (-f_leg) for legs in stance at the first horizon step
// (leg_controller.py:86-89, the leg's 3x3 block of the 3x18 foot Jacobian);
// swing legs are left to the swing controller (their entries are not written).
__global__ __launch_bounds__(256) void mpcqp_stance_torque_kernel(int B, const float* __restrict__ jac,
                                                                  const float* __restrict__ contact0,
                                                                  int contact_stride, const float* __restrict__ u0,
                                                                  float* __restrict__ tau) {
#pragma clang fp contract(off)
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;   // (robot, leg, joint)
  if (gid >= B * 12) return;
  const int b = gid / 12, leg = (gid % 12) / 3, j = gid % 3;
  if (!(contact0[(size_t)b * contact_stride + leg] > 0.f)) return;
  const float* J = jac + ((size_t)b * 4 + leg) * 9;   // row-major 3x3: J[r][c] = d p_r / d q_c
  const float* f = u0 + (size_t)b * 12 + 3 * leg;
  tau[(size_t)b * 12 + 3 * leg + j] = -(J[j] * f[0] + J[3 + j] * f[1] + J[6 + j] * f[2]);
}
