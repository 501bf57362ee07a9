/*
 * mpcqp.h -- C ABI of the MI355X batched convex-MPC QP engine (libmpcqp.so).
 *
 * Replaces, for a batch of B independent robots, the per-tick
 * formulate-and-solve of the reference's ModelPredictiveController:
 *
 *   _generate_state_space_model   /root/reference/linear_mpc/mpc.py:173-192
 *   _discretize_continuous_model  /root/reference/linear_mpc/mpc.py:194-208
 *   _generate_QP_cost             /root/reference/linear_mpc/mpc.py:211-235
 *   _generate_QP_constraints      /root/reference/linear_mpc/mpc.py:237-260
 *   _solve_mpc (Drake branch)     /root/reference/linear_mpc/mpc.py:262-286
 *
 * i.e.  min_U 1/2 U^T H U + g^T U  s.t.  lb <= C U <= ub  (Drake
 * AddQuadraticCost semantics, mpc.py:281-282), returning the first-step
 * ground-reaction forces U[0:12] (mpc.py:99).  The reference binds that path
 * through pydrake (mpc.py:13, :278-286); the ctypes binding that replaces it
 * is shown in INTEGRATION.md.
 *
 * All array arguments are DEVICE pointers owned by the caller (e.g. torch
 * tensors on the context's device).  Calls are asynchronous on `stream`.
 * No exception crosses the ABI: every entry point returns MPCQP_OK (0) or a
 * negative error code; mpcqp_last_error() describes the last failure.
 * Per-robot solver outcome is reported in status[] (MPCQP_STATUS_*).
 * A context keeps per-stream device queues for up to 8 streams; a solve on a 9th
 * distinct stream takes over the least recently used stream's queues once that stream's
 * last solve on this context has finished (the host waits on an event recorded after
 * it -- not on the device or the other streams).  Round-robin over at most 8 streams per
 * context to stay fully asynchronous.
 *
 * Layouts (float32, row-major, robot-major):
 *   x0      [B][13]   [roll, pitch, yaw, px, py, pz, wx, wy, wz, vx, vy, vz, -g]
 *                     (mpc.py:65-77; x0[2] is also the model yaw, mpc.py:77)
 *   xref    [B][N][13] reference of x_{1..N} (mpc.py:154-168)
 *   contact [B][N][4]  legs FL, FR, RL, RR; > 0 = stance (gait.py:87-98);
 *                      ub of the normal-force row is contact * fz_max (mpc.py:257)
 *   feet    [B][4][3]  foot position relative to the CoM, world frame
 *                      (RobotData.pos_base_feet, robot_data.py:101,144-149)
 *   robot   [B][16]    per-robot record: mass, ixx, ixy, ixz, iyy, iyz, izz,
 *                      mu, fz_max, nx, ny, nz, 0, 0, 0, 0
 *                      (robot_configs.py:44-79; normal (0,0,1) = reference cone)
 *   u0      [B][12]    out: first-step GRFs, world frame (mpc.py:99)
 *   U       [B][N][12] out (nullable): the whole optimal input sequence
 *   status  [B]        out (nullable): MPCQP_STATUS_*
 *   iters   [B]        out (nullable): active-set steps executed (a pair step counts 2);
 *                      for a robot with more than 128 stance variables (the interior-point
 *                      class: standing schedules at N >= 11) the Newton factorisations
 *
 * Input reads: a robot's x0 / xref / contact / feet / robot slices are staged with
 * 16-byte loads of the 16-byte-aligned chunks that cover them, so up to 12 bytes
 * before and after each slice (never across a 4 KiB page) are read and ignored.
 * The buffers must be device allocations (hipMalloc / torch: page-granular, no
 * guard pages); the values read outside a slice never reach any result.
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCQP_ABI_VERSION 6
#define MPCQP_ROBOT_STRIDE 16
#define MPCQP_MAX_HORIZON 32   /* mpcqp_create rejects horizon > 32 (MPCQP_ERR_ARG).  Horizons
                                  up to 20 use every capacity class; longer ones are solved by
                                  the interior-point class alone (its per-robot LDS scratch is
                                  sized for 32 stages, the dense classes' for 20) */

/* error codes (return values) */
#define MPCQP_OK 0
#define MPCQP_ERR_ARG -1
#define MPCQP_ERR_HIP -2
#define MPCQP_ERR_ALLOC -3

/* per-robot status */
#define MPCQP_STATUS_OK 0          /* the optimum: every cone row feasible, every active
                                      multiplier >= 0 (checked); stationarity holds by
                                      construction of the dual active-set updates (dense
                                      classes) or is checked on the active set's null
                                      space (interior-point class, n > 128) */
#define MPCQP_STATUS_MAX_ITER 1    /* iteration cap hit: best iterate returned */
#define MPCQP_STATUS_INFEASIBLE 2  /* cannot happen for this QP (U = 0 is feasible) */
#define MPCQP_STATUS_TOO_LARGE 3   /* stance variables exceed the engine's capacity */
#define MPCQP_STATUS_NONFINITE 4   /* non-finite input or result */
#define MPCQP_STATUS_UNSUPPORTED 5 /* weights the robot's capacity class cannot apply; no
                                      weights reach it since ABI 6's cross-leg stage weights
                                      (kept as a guard); u0 / U are 0 */

typedef struct mpcqp_params {
  int32_t horizon;       /* N (LinearMpcConfig.horizon, linear_mpc_configs.py:11) */
  int32_t max_iter;      /* active-set iteration cap per robot of the dense classes (n <= 126),
                            0 = default; the interior-point class (n > 128) stops after its own
                            60 Newton iterations and does not read it */
  double dt;             /* model step, 0.05 in the reference (mpc.py:38) */
  double q_diag[13];     /* state weights (linear_mpc_configs.py:19) */
  double r_diag[12];     /* input weights (linear_mpc_configs.py:20) */
} mpcqp_params;

typedef struct mpcqp_ctx mpcqp_ctx;

/* Fill `p` with the reference's LinearMpcConfig values for horizon N. */
void mpcqp_default_params(mpcqp_params* p, int32_t horizon);

/* Create a context on HIP device `device`; the context owns scratch memory. */
int mpcqp_create(const mpcqp_params* p, int32_t device, mpcqp_ctx** out);

/* Formulate and solve B QPs (see header comment for layouts). */
int mpcqp_solve(mpcqp_ctx* ctx, int32_t batch, const float* x0, const float* xref,
                const float* contact, const float* feet, const float* robot, float* u0,
                float* U, int32_t* status, int32_t* iters, void* stream /* hipStream_t */);

/* Full state / input weights (mpc.py:49-52 builds kron(I_N, Q), kron(I_N, R) from any
 * LinearMpcConfig.Q / R): Q [13][13] and R [12][12] row-major HOST arrays, symmetric and
 * finite (else MPCQP_ERR_ARG); NULL keeps the current matrix (as last set, off-diagonal
 * entries included).  Diagonal matrices select the diagonal fast path (equivalent to
 * setting q_diag / r_diag).  The weights are copied before the call returns; solves issued
 * before it are unaffected.  A failed call (error code) leaves the previous weights in
 * force.  The previous full-weight buffer is kept until mpcqp_destroy (solves in flight
 * may still read it); only every 64th change synchronises the whole device
 * (hipDeviceSynchronize) to release the kept buffers -- not while a stream of this
 * device is being captured into a graph.
 * Every capacity class takes any symmetric Q and R; an R coupling different legs
 * (R[i][j] != 0 for i / 3 != j / 3) runs the interior-point class (robots with more than 128
 * stance variables) with whole 12 x 12 stage weights instead of per-leg blocks. */
int mpcqp_set_weights(mpcqp_ctx* ctx, const double* Q, const double* R);

/* Largest number of stance foot-steps the caller promises per robot
 * (0 = unknown: the engine dispatches every capacity class). */
int mpcqp_set_stance_hint(mpcqp_ctx* ctx, int32_t max_stance);

/* Both bounds on the stance foot-steps per robot (min 0 and max 0 = no promise):
 * classes no robot can need are not launched, and when the range rules out the
 * smaller classes the first possible one takes the batch directly (the drop-in
 * controller passes its gait table's exact count).  A robot outside the range is
 * still solved if a launched class covers it, else reports MPCQP_STATUS_TOO_LARGE.
 * MPCQP_ERR_ARG when min_stance > 4 * horizon (no schedule has that many) or
 * min_stance > max_stance > 0. */
int mpcqp_set_stance_range(mpcqp_ctx* ctx, int32_t min_stance, int32_t max_stance);

/* Dispatch order (ABI 6; the reference solves one robot at a time and has no batch order).
 * mode 1 (the default): when a batch queues on the CUs (more robots than its first capacity
 * class holds on the device at once: 4 per CU for class 64, 1 for classes 96 / 128), its
 * robots are dealt to workgroups largest predicted solve time first -- the key is the robot's
 * horizontal velocity error |v0 - vref_0|, which tracks its active-set size -- so the longest
 * robots start first and the launch ends near its mean load.  Costs one small sort launch per
 * such solve; the results are bitwise those of mode 0 (batch order: robot b on workgroup b).
 * The order needs the stream's queue set even for a batch class 64 solves alone: the first
 * such call on a stream allocates it (hipMalloc + an asynchronous clear), and a later, larger
 * batch reallocates it after a synchronisation of that stream.  To capture solves into a HIP
 * graph, make one call of at least the captured batch size on the capture stream first, or
 * set mode 0 (a class-64-only solve in batch order allocates nothing).
 * MPCQP_ERR_ARG for any other mode. */
int mpcqp_set_order(mpcqp_ctx* ctx, int32_t mode);

/* Warm start (ABI 5; no counterpart in the reference, whose Drake solve starts cold every
 * MPC tick, mpc.py:277-286): per-robot memory of the last verified active set, for
 * callers that solve the same robots tick after tick (the drop-in controller, a fleet in
 * a simulation loop).  The interior-point class (robots with more than 128 stance
 * variables, e.g. Gait.STANDING at N >= 11) then first tries the remembered rows -- one
 * equality-constrained solve and the KKT check its polish always runs, corrected up to 8
 * times -- and runs the interior point only when that fails.  The result does not depend
 * on the memory: a status-OK solution is the checked optimum either way.
 *   memory    DEVICE buffer of capacity * MPCQP_WARM_BYTES bytes, zero-filled by the
 *             caller before first use (zero = nothing remembered).  Robot b of every later
 *             mpcqp_solve on this context reads and rewrites memory + b * MPCQP_WARM_BYTES
 *             (byte 4 k + leg: 0x80 | the foot-step's active cone rows; b >= capacity: no
 *             memory).  Solves running concurrently on different streams must not share it.
 *   NULL / capacity 0 disables (the default).  The dense classes (n <= 128) do not use it.
 * MPCQP_ERR_ARG for capacity < 0, or memory NULL with capacity > 0. */
#define MPCQP_WARM_BYTES 128   /* 4 * MPCQP_MAX_HORIZON */
int mpcqp_set_warm_start(mpcqp_ctx* ctx, void* memory, int32_t capacity);

/* ---- the hot path's callers on the device -------------
 *
 * mpcqp_plan replaces, per control iteration and batched over robots:
 *   ModelPredictiveController.update_robot_state  (state packing)  mpc.py:55-79
 *     quat2ZYXangle                                                kinematics.py:40-49
 *   update_mpc_if_needed (desired-pose integrators)                mpc.py:81-92
 *   generate_reference_trajectory          (MPCQP_PLAN_REFERENCE)  mpc.py:110-170
 *   Gait.set_iteration / get_gait_table    (MPCQP_PLAN_REFERENCE)  gait.py:76-100
 * Its x0 / xref / contact outputs feed mpcqp_solve directly (no host round trip).
 * Call it every control iteration (the integrators run at 1/dt_control) with
 * flags = MPCQP_PLAN_REFERENCE when iter % iterations_between_mpc == 0 (mpc.py:95),
 * else 0.  MPCQP_PLAN_NO_INTEGRATE skips the integrators: REFERENCE | NO_INTEGRATE
 * is generate_reference_trajectory alone (mpc.py:110-170).
 *
 *   quat         [B][4]  base orientation (w, x, y, z)            robot_data.quat_base
 *   pos, omega, vel [B][3]  base position, angular / linear velocity (world)
 *   rot          [B][3][3]  R_base, row-major (mpc.py:83); NULL = quat2matrix(quat)
 *                        computed on the device (robot_data.py:75)
 *   vel_body_des [B][3]  float64 desired base velocity, body frame (mpc.py:83)
 *   yaw_rate_des [B]     float64 desired yaw rate
 *   gait         [B][9]  int32: period, stance offsets[4], stance durations[4]
 *                        (gait.py:16-22; e.g. TROTTING10 = 10, 0 5 5 0, 5 5 5 5);
 *                        NULL = the caller supplies its own contact schedule
 *   iteration    [B]     int32 gait segment: floor(iter / iterations_between_mpc) % period
 *                        (gait.py:76-78)
 *   height_des   [B]     desired CoM height (robot_configs.py:50,69)
 *   plan_state   [B][MPCQP_PLAN_STRIDE] float64 in/out: x_des, y_des, yaw_des,
 *                        roll_init, pitch_init, started, 0, 0; all-zero = first run
 *   x0 [B][13], xref [B][N][13], contact [B][N][4]: out (xref / contact only written
 *                        with MPCQP_PLAN_REFERENCE; contact only with a gait)
 */
#define MPCQP_PLAN_STRIDE 8
#define MPCQP_GAIT_STRIDE 9
#define MPCQP_PLAN_REFERENCE 1
#define MPCQP_PLAN_NO_INTEGRATE 2
int mpcqp_plan(mpcqp_ctx* ctx, int32_t batch, int32_t flags, const float* quat, const float* pos,
               const float* omega, const float* vel, const float* rot, const double* vel_body_des,
               const double* yaw_rate_des, const int32_t* gait, const int32_t* iteration,
               const float* height_des, double* plan_state, float* x0, float* xref, float* contact,
               void* stream);

/* The same, reading Isaac Gym's actor root-state tensor in place:
 * root_states [B][13] = pos(3), quat(x, y, z, w), lin_vel(3), ang_vel(3) -- the
 * layout isaacgym_a1.py:119-128 slices and reorders per robot on the host.  R_base
 * is quat2matrix of that quaternion. */
int mpcqp_plan_root_states(mpcqp_ctx* ctx, int32_t batch, int32_t flags, const float* root_states,
                           const double* vel_body_des, const double* yaw_rate_des, const int32_t* gait,
                           const int32_t* iteration, const float* height_des, double* plan_state, float* x0,
                           float* xref, float* contact, void* stream);

/* Planner constants: dt_control (linear_mpc_configs.py:6, default 0.001), gravity
 * (:13, 9.81) and the reference-position clamp (mpc.py:121, 0.1). */
int mpcqp_set_planner(mpcqp_ctx* ctx, double dt_control, double gravity, double max_pos_error);

/* Stance-leg joint torques tau = Jv_leg^T (-f_leg) (leg_controller.py:86-89,
 * SURVEY §8 f4) for the legs with stance[b * stance_stride + leg] > 0 -- the
 * controller's `not swing_states[leg]` (leg_controller.py:77); swing-leg entries of
 * tau are not written.  jac [B][4][3][3]: each leg's 3x3 block of its foot Jacobian (rows = world
 * x, y, z; columns = the leg's 3 joints), row-major.  u0 [B][12], tau [B][12]. */
int mpcqp_stance_torques(mpcqp_ctx* ctx, int32_t batch, const float* jac, const float* stance,
                         int32_t stance_stride, const float* u0, float* tau, void* stream);

int mpcqp_destroy(mpcqp_ctx* ctx);

const char* mpcqp_last_error(const mpcqp_ctx* ctx);

int32_t mpcqp_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MPCQP_H */
