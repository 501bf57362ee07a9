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
 *   iters   [B]        out (nullable): active-set iterations executed
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCQP_ABI_VERSION 1
#define MPCQP_ROBOT_STRIDE 16
#define MPCQP_MAX_HORIZON 32

/* error codes (return values) */
#define MPCQP_OK 0
#define MPCQP_ERR_ARG -1
#define MPCQP_ERR_HIP -2
#define MPCQP_ERR_ALLOC -3

/* per-robot status */
#define MPCQP_STATUS_OK 0          /* KKT verified */
#define MPCQP_STATUS_MAX_ITER 1    /* iteration cap hit: best iterate returned */
#define MPCQP_STATUS_INFEASIBLE 2  /* cannot happen for this QP (U = 0 is feasible) */
#define MPCQP_STATUS_TOO_LARGE 3   /* stance variables exceed the engine's capacity */
#define MPCQP_STATUS_NONFINITE 4   /* non-finite input or result */

typedef struct mpcqp_params {
  int32_t horizon;       /* N (LinearMpcConfig.horizon, linear_mpc_configs.py:11) */
  int32_t max_iter;      /* active-set iteration cap per robot, 0 = default */
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

/* Largest number of stance foot-steps the caller promises per robot
 * (0 = unknown: the engine dispatches every capacity class). */
int mpcqp_set_stance_hint(mpcqp_ctx* ctx, int32_t max_stance);

int mpcqp_destroy(mpcqp_ctx* ctx);

const char* mpcqp_last_error(const mpcqp_ctx* ctx);

int32_t mpcqp_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MPCQP_H */
