/*
 * vcmpc.h -- C ABI of the MI355X-native batched MPC solve path (libvcmpc.so).
 *
 * Drop-in boundary for the per-step predict -> linearize -> QP-solve loop of
 * neverorfrog/vehicle-control (reference @ 2024-12-20).  Each entry point names
 * the reference interface it replaces (paths relative to the reference checkout):
 *
 *   vc_create        KinematicMPC.__init__            vehicle_control/controllers/mpc/kinematic_mpc.py:15-30
 *                    (the once-only NLP transcription + IPOPT setup, :39-52)
 *   vc_solve         KinematicMPC.command             kinematic_mpc.py:160-168 (opti.solve at :162)
 *                    CascadedMPC.command (single-track, horizon_pm = 0)
 *                                                     controllers/mpc/cascaded_mpc.py:306-314 (opti.solve
 *                                                     at :308; NLP built at :17-39,91-179,279-304)
 *   vc_solve_from    the same, with the warm start and u* in separate buffers (the reference passes
 *                    its warm start in by opti.set_initial, kinematic_mpc.py:175-176, and reads u* back
 *                    by sol.value, :163)
 *   vc_rollout       KinematicCar.spatial_transition  vehicle_control/models/kinematic_car.py:61-64,70-72,
 *                    applied along the horizon        (the dynamics rows of kinematic_mpc.py:95-99)
 *   vc_linearize     CasADi AD of the dynamics inside IPOPT ("expand": True, kinematic_mpc.py:51)
 *   vc_condense      the condensed-QP Hessian/gradient of the build's LTV-QP contract
 *                    (restates the NLP cost kinematic_mpc.py:101-158 linearised)
 *   vc_plant_step    RacingCar.drive / Robot.transition  vehicle_control/models/racing_car.py:34-46,
 *                    kinematic_car.py:34-45,66-68 (Euler), dynamic_car.py:144-167,193-195 (RK4)
 *   vc_spatial_step  <Model>.spatial_transition       kinematic_car.py:70-72, dynamic_car.py:169-199
 *   vc_ode           the vector field f(x, u, curvature) the integrators wrap (utils/integrators.py:18,29):
 *                    temporal kinematic_car.py:34-40, dynamic_car.py:153-167; spatial :47-60, :169-191
 *   vc_set_obstacles Track._construct_obstacles       environment/track.py:131-138 (the obstacle list the
 *                                                     barrier terms kinematic_mpc.py:130-133 read)
 *   vc_track_set     Track._precompute_curvatures     environment/track.py:156-167 (the bspline k(s) table)
 *   vc_track_k       Track.k                          track.py:162-166
 *   vc_horizon       KinematicMPC._init_horizon       kinematic_mpc.py:170-187
 *                    CascadedMPC._init_horizon        cascaded_mpc.py:316-330 (horizon_pm = 0)
 *   vc_drive         RacingCar.drive                  models/racing_car.py:34-46 (k = track.k(s), fp64 plant)
 *   vc_simulate      RacingSimulator.update / step    simulation/racing.py:217-242,416-423 (command ->
 *                                                     drive -> log, every vehicle, `steps` times)
 *
 * Conventions
 *   - All arrays are C-contiguous, batch-outermost ("AoS"):
 *       x0[B][nx], kappa[B][N], ds[B][N], ubar[B][N][nu], xbar[B][N+1][nx], u0[B][nu].
 *     The reference stores state_prediction as (nx, N+1) and action_prediction as
 *     (nu, N) (kinematic_mpc.py:59-67); the Python mirror transposes.
 *   - State / action orderings are the reference FancyVector keys:
 *       kinematic x = [v, delta, s, ey, epsi, t],  u = [a, w]   (kinematic_car.py:81,117)
 *       dynamic   x = [Ux, Uy, r, delta, s, ey, epsi, t], u = [Fx, w] (dynamic_car.py:209,247)
 *   - flags = VC_HOST_PTRS: pointers are host memory; the call copies in, runs and
 *     copies out, and returns when the results are in the caller's buffers.
 *     flags = VC_DEVICE_PTRS: pointers are device memory on the context's device;
 *     the call only enqueues work on the context stream (vc_set_stream) and
 *     returns immediately; call vc_synchronize() before reading results.
 *   - Return value: 0 on success, a negative VC_E* code on an API or HIP error
 *     (message via vc_last_error).  Per-problem outcomes are reported in status[b]
 *     (VC_SOLVED, VC_MAX_ITER, VC_NONFINITE, VC_OUT_OF_DOMAIN); no exception-style failure, unlike the
 *     reference simulator's catch-all (simulation/racing.py:416-423).
 *   - Threading: one context per device per host thread; calls on one context
 *     are serialised on its stream.
 */
#ifndef VCMPC_H
#define VCMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VCMPC_ABI_VERSION 13
#define VC_MAX_OBSTACLES 16

typedef struct vc_ctx vc_ctx;

enum vc_model { VC_MODEL_KINEMATIC = 0, VC_MODEL_DYNAMIC = 1, VC_MODEL_CASCADED = 2 };
enum vc_dtype { VC_F64 = 0, VC_F32 = 1 };
enum vc_flags { VC_HOST_PTRS = 0, VC_DEVICE_PTRS = 1 };
enum vc_tyre { VC_TYRE_FIALA = 0, VC_TYRE_LINEAR = 1 };
/* VC_OUT_OF_DOMAIN (ABI 12, SQP contexts): the returned x* = rollout(u*) leaves the spatial
 * model's domain (Ux > 0 and s' = (Ux cos epsi - Uy sin epsi) / (1 - kappa ey) > 0 at every
 * stage, dynamic_car.py:169-191 divides by s') although every QP converged: the SQP started
 * from a warm start outside the domain and never got back in.  Not a solution of the NLP. */
enum vc_status { VC_SOLVED = 0, VC_MAX_ITER = 1, VC_NONFINITE = 2, VC_OUT_OF_DOMAIN = 3 };
enum vc_error {
  VC_OK = 0,
  VC_E_ARG = -1,      /* bad argument / dimension */
  VC_E_HIP = -2,      /* HIP runtime error (launch, copy, OOM) */
  VC_E_UNSUPPORTED = -3 /* model/dtype/horizon combination not built */
};

/* Kinematic bicycle (config/models/kinematic_car.yaml). */
typedef struct vc_kin_car {
  double l; /* wheelbase car.l [m] (kinematic_car.py:39,53 via racing_car.py:27) */
} vc_kin_car;

/* Dynamic bicycle (config/models/dynamic_car.yaml, dynamic_car.py:62-151). */
typedef struct vc_dyn_car {
  double l, m, Izz, a, b, h, eps, Peng;
  double Xdf, Xdr, Xbf, Xbr; /* drive / brake force distribution */
  double Caf, Car;           /* cornering stiffness front / rear */
  double Cd, muf, mur, theta, phi, Av2, Frr;
  int32_t tyre;              /* enum vc_tyre */
  int32_t pad_;
} vc_dyn_car;

/* Kinematic MPC weights and bounds (config/controllers/kinematic.yaml). */
typedef struct vc_kin_mpc {
  double w_time, w_ey, w_epsi, w_v, w_w, w_a, w_dev, w_b; /* cost_weights */
  double a_min, a_max, w_min, w_max;                      /* input_constraints */
  double v_min, v_max, delta_min, delta_max, ey_min, ey_max; /* state_constraints */
  double w_obs;     /* cost_weights.obstacles (kinematic_mpc.py:130-133; used when obs.n > 0) */
} vc_kin_mpc;

/* Dynamic single-track MPC weights and bounds (config/controllers/singletrack.yaml,
 * read by cascaded_mpc.py:91-179,279-304) and the build's SQP knobs. */
typedef struct vc_dyn_mpc {
  double w_time, w_speed, w_ey, w_epsi, w_w, w_Fx, w_dev, w_b, w_slip; /* cost_weights */
  double w_min, w_max;                                                /* input_constraints */
  double Ux_min, max_speed, delta_min, delta_max, ey_min, ey_max;     /* state_constraints */
  double fx_scale;   /* Fx unit of the scaled decision variable [N] (no reference counterpart) */
  double trust_Fx;   /* SQP trust region |Fx - Fxbar| <= trust_Fx [N] (0 = off) */
  int32_t sqp_iters; /* SQP iterations per solve (BASELINE config 3: 3) */
  int32_t pad_;
  double w_obs;      /* cost_weights.obstacles (cascaded_mpc.py:173-176; used when obs.n > 0) */
} vc_dyn_mpc;

/* The build's LTV-QP contract knobs (no reference counterpart). */
typedef struct vc_qp {
  double prox;      /* proximal weight: + prox * ||u - ubar||^2 */
  double tol;       /* interior-point stopping tolerance (scaled) */
  double trust_a;   /* trust region |u_a - ubar_a| <= trust_a (0 = off) */
  double trust_w;   /* trust region |u_w - ubar_w| <= trust_w (0 = off) */
  int32_t max_iter; /* interior-point iteration cap */
  int32_t polish;   /* active-set polish rounds after the interior point (0 = off) */
  int32_t solver;   /* solve-kernel choice (ABI 5).  Kinematic: 0 = condensed (kin_ltv.hip) where
                       built (N = 20) and kin_sqp == 0, else stagewise Riccati (kin_ric.hip);
                       1 = stagewise Riccati always.  Cascaded: 0 / 1 = stagewise Riccati (casc_ric.hip),
                       2 = condensed (casc_sqp.hip, M = 40 only).  Single-track: the dtype
                       picks the kernel (VC_F32: dyn_sqp.hip, VC_F64: st_sqp.hip). */
  int32_t kin_sqp;  /* kinematic (ABI 6): 0 = one LTV-QP step (the C2 contract); k > 0 = k SQP
                       steps, each QP step followed by an Armijo line search on the exact NLP cost
                       + an L1 state-row penalty (kin_merit.hip, oracle/kin_sqp.py) -- the
                       globalised step for the obstacle barrier (kinematic_mpc.py:130-133) */
  int32_t shift;    /* ABI 7: vc_simulate shifts a solved vehicle's warm start one stage ahead
                       (stage k <- k + 1, the last stage kept) before the next step; 0 keeps the
                       reference's unshifted warm start (kinematic_mpc.py:170-187).  Kinematic and
                       single-track contexts (ignored for cascaded ones) */
  int32_t ms;       /* ABI 8, kinematic stagewise kernel: 1 = multiple shooting -- linearise at the
                       warm-start states xbar (read from vc_solve's xbar, x0 replacing its first
                       column) instead of the rollout of ubar; the defects enter as a linear
                       offset (oracle/ltv_qp.py kin_qp(..., x_ws=)) */
  double elastic;   /* ABI 9, kinematic stagewise kernel: rho > 0 makes the v / delta state rows
                       elastic -- row i gets a slack t_i >= 0 at cost rho t_i + 1e-8 t_i^2 (the QP
                       model of kin_merit's L1 penalty), so every QP has a solution; the plain
                       step whenever that is feasible with multipliers below rho
                       (oracle/ltv_qp.py elastic_qp).  -rho < 0 (kin_sqp > 0): elastic on failure
                       -- every QP is solved with hard rows and only the ones that solve leaves
                       non-solved are solved again with elastic rows at rho (SNOPT's elastic mode).
                       0 = hard rows.  rho > 0 on a one-step context routes to the stagewise kernel;
                       rho < 0 needs kin_sqp > 0 (vc_solve returns VC_E_ARG otherwise) */
} vc_qp;

/* Cascaded controller: single-track stages followed by a point-mass tail
 * (config/controllers/cascaded.yaml, cascaded_mpc.py:181-277).  The single-track part
 * and the SQP knobs come from vc_dyn_mpc; these are the tail's own settings. */
typedef struct vc_casc_mpc {
  int32_t horizon_pm;  /* M point-mass stages (cascaded.yaml horizon_pm) */
  int32_t pad_;
  double ds_pm;        /* point-mass stage length [m] (cascaded.yaml ds_pm) */
  double w_dev_pm, w_Fy, w_switch;       /* cost_weights deviation_pm, Fy, switch_F */
  double V_min, ey_min_pm, ey_max_pm;    /* state_pm_constraints */
} vc_casc_mpc;

/* Circular obstacles in track coordinates (Track._construct_obstacles, environment/
 * track.py:131-138, data `obstacle_data: [s, ey, r]` of config/environment/<track>.yaml).
 * n = 0 switches the barrier terms off (the controller's `obstacles: False`).
 * The reference's stage cost w_obs ds / (dist - (r + 0.1)), dist = |(s, ey) - (s_j, ey_j)|
 * (kinematic_mpc.py:130-133, cascaded_mpc.py:173-176) enters each QP as the convexified
 * second-order model of its sum over obstacles in ey at the prediction; the margin
 * dist - (r + 0.1) is floored at margin_min. */
typedef struct vc_obstacles {
  int32_t n;          /* number of obstacles, 0..VC_MAX_OBSTACLES */
  int32_t inside;     /* 0: the margin is floored at margin_min everywhere below it (default);
                         1: inside an obstacle beyond the floor band (dist - (r + 0.1) < -margin_min)
                         the QP model takes the reference's own barrier w ds / (dist - r - 0.1),
                         negative there; the floor then acts only in |dist - (r + 0.1)| <= margin_min
                         (ABI 11).  Dynamic / cascaded contexts only: vc_create rejects 1 for
                         the kinematic model (its merit keeps the C1 extension) and any value
                         other than 0 and 1 (ABI 12) */
  double margin_min;  /* floor of dist - (r + 0.1) in the barrier's derivatives [m] */
  double s[VC_MAX_OBSTACLES], ey[VC_MAX_OBSTACLES], radius[VC_MAX_OBSTACLES];
} vc_obstacles;

typedef struct vc_params {
  vc_kin_car kin_car;
  vc_dyn_car dyn_car;
  vc_kin_mpc kin_mpc;
  vc_qp qp;         /* trust_a is the kinematic acceleration trust region; trust_w serves both */
  vc_dyn_mpc dyn_mpc;
  vc_obstacles obs;
  vc_casc_mpc casc;
} vc_params;

int vc_abi_version(void);
/* sizeof(vc_params): lets an FFI binding check its struct mirror. */
int vc_params_sizeof(void);

/* Create a solve context on `device` for `model` with horizon N and workspace for
 * up to max_batch problems.  Returns NULL on failure (reason: vc_last_error(NULL)).
 * Built combinations for vc_solve (and vc_horizon / vc_simulate):
 *   (VC_MODEL_KINEMATIC, VC_F64, N = 20) condensed (kin_ltv.hip; also vc_condense) and
 *     N = 10, 20, 30, 40, 50, 60 stagewise Riccati (kin_ric.hip; kinematic.yaml N = 50);
 *   (VC_MODEL_DYNAMIC, VC_F64, N = 20, 30, 40, 50, 60) single-track SQP, stagewise Riccati
 *     (st_sqp.hip; singletrack.yaml N = 60, recorded N = 50); (VC_MODEL_DYNAMIC, VC_F32,
 *     N = 40) the condensed fp32 SQP (dyn_sqp.hip, BASELINE config 3);
 *   (VC_MODEL_CASCADED, VC_F64, N = 20 single-track stages, casc.horizon_pm = 15, 25, 35,
 *     40) stagewise Riccati (casc_ric.hip), horizon_pm = 40 also condensed (casc_sqp.hip,
 *     vc_condense); the arrays span H = N + horizon_pm stages.
 * Other combinations create a context whose vc_solve returns VC_E_UNSUPPORTED.
 * vc_rollout / vc_linearize / vc_plant_step / vc_spatial_step: every N >= 1. */
vc_ctx* vc_create(int device, int model, int N, int max_batch, int dtype, const vc_params* params);
void vc_destroy(vc_ctx* ctx);
const char* vc_last_error(const vc_ctx* ctx);

/* Use an external HIP stream (hipStream_t passed as void*; NULL = the context's
 * own stream).  Lets a caller time the work with events on that stream. */
int vc_set_stream(vc_ctx* ctx, void* stream);

/* Replace the context's obstacle set (vc_params.obs) for later solves: n <= VC_MAX_OBSTACLES
 * obstacles at host arrays s[n], ey[n], radius[n] (track.py:131-138); n = 0 turns the
 * barrier terms off.  margin_min <= 0 keeps the current floor. */
int vc_set_obstacles(vc_ctx* ctx, int n, const double* s, const double* ey, const double* radius,
                     double margin_min);
int vc_synchronize(vc_ctx* ctx);

/* One MPC step for B problems (B <= max_batch):
 *   in:     x0[B][nx], kappa[B][N], ds[B][N], ubar[B][N][nu] (warm start)
 *   out:    ubar <- u*[B][N][nu], xbar <- x*[B][NS][nx], u0[B][nu] = u*[:,0],
 *           status[B] (enum vc_status), iters[B] (interior-point iterations, summed
 *           over the SQP iterations for the dynamic model).
 * Kinematic: one LTV-QP step, NS = N + 1 state columns (kinematic_mpc.py:59-64).
 * Dynamic:   dyn_mpc.sqp_iters QP steps, NS = N columns with dynamics for k < N-1
 *            (cascaded_mpc.py:70,116-122); x* is the rollout of u*.
 * Cascaded:  dyn_mpc.sqp_iters QP steps over H = N + casc.horizon_pm stages: kappa, ds
 *            [B][H], ubar [B][H][2] (Fx, w for k < N; Fx, Fy for the point mass), xbar
 *            [B][H][8] (point-mass states V, s, ey, epsi, t in slots 0..4, 5..7 = 0). 
 * xbar is output only: the prediction is re-rolled from (x0, ubar). */
int vc_solve(vc_ctx* ctx, int B, const void* x0, const void* kappa, const void* ds,
             void* xbar, void* ubar, void* u0, int32_t* status, int32_t* iters, int flags);

/* vc_solve with the warm start read from ubar_in, which is left unchanged, and u* written to
 * u_out (same shape; u_out == ubar_in is vc_solve).  The kinematic kernels read and write through
 * the two pointers (no copy); the SQP contexts, which iterate in place, copy ubar_in to u_out
 * first.  For callers that keep their warm start, e.g. a batch re-solved from the same guess. */
int vc_solve_from(vc_ctx* ctx, int B, const void* x0, const void* kappa, const void* ds, const void* ubar_in,
                  void* xbar, void* u_out, void* u0, int32_t* status, int32_t* iters, int flags);

/* vc_solve plus per-problem solver diagnostics diag[B][4]:
 *   [0] final scaled KKT residual, [1] final scaled complementarity mu,
 *   [2] flags: 1 = interior-point factorisation failed, 2 = interior point
 *       converged, 4 = active-set polish certified, 8 = polish factorisation failed,
 *   [3] polish rounds used.  diag follows the pointer convention of `flags`.
 * Kinematic (kin_ltv) [0] is the true residual of the interior point's last iterate.
 * Single-track / cascaded SQP contexts: [2] = 1 any QP failed, 2 every QP converged,
 * 4 every converged QP's answer certified by the active-set polish, 16 the SQP stopped early (a QP after the first had no solution: its step was refused and
 * the earlier iterate returned, so `status` reflects the QPs before it only); [3] the largest
 * interior-point iteration count of one QP. */
int vc_solve_diag(vc_ctx* ctx, int B, const void* x0, const void* kappa, const void* ds,
                  void* xbar, void* ubar, void* u0, int32_t* status, int32_t* iters, void* diag,
                  int flags);

/* Test diagnostics (dynamic fp32 contexts): vc_solve plus a dump of the first QP
 * of the first SQP iteration into dbg[B][vc_debug_stride()] floats:
 * [0,80) gradient g, [80,6480) interior-point normal matrix M at the start point
 * (row-major, lower tiles + diagonal blocks valid), [6480,12880) the factor storage
 * after the blocked Cholesky (Y = L^-T in the upper triangle), [12880,12960) the
 * predictor right-hand side, [12960,13040) the predictor step.  No reference
 * counterpart: used by tests/test_gpu_parity.py to check each stage of the kernel. */
int vc_solve_debug(vc_ctx* ctx, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar,
                   void* u0, int32_t* status, int32_t* iters, void* dbg, int flags);
int vc_debug_stride(void);

/* Test hook (kinematic SQP contexts, vc_qp.kin_sqp > 0): after the QP of SQP iteration
 * `sqp_iter` (0-based), problem `problem`'s QP output is replaced by NaN with status
 * VC_NONFINITE -- a QP that failed with non-finite output -- so tests can check that the
 * merit line search refuses the step and keeps the previous iterate.  sqp_iter < 0 turns
 * it off (the default).  No reference counterpart. */
int vc_debug_qp_fault(vc_ctx* ctx, int sqp_iter, int problem);

/* Test diagnostics: the reciprocal forms of the solve kernels evaluated on the device for n
 * (<= max_batch) inputs x[n] fp64, out[n][4] fp64: IEEE 1/x, rcp_nr(x) (kin_ltv), the
 * Riccati kernels' v_rcp_f64 + two Newton steps, the raw v_rcp_f64 (csrc/numerics.hip).
 * No reference counterpart. */
int vc_debug_rcp(vc_ctx* ctx, int n, const void* x, void* out, int flags);

/* Predict: xbar[B][N+1][nx] from x0[B][nx] and ubar[B][N][nu] (spatial step). */
int vc_rollout(vc_ctx* ctx, int B, const void* x0, const void* ubar, const void* kappa,
               const void* ds, void* xbar, int flags);

/* Linearize: A[B][N][nx][nx], Bm[B][N][nx][nu] of the spatial step at (xbar_k, ubar_k). */
int vc_linearize(vc_ctx* ctx, int B, const void* xbar, const void* ubar, const void* kappa,
                 const void* ds, void* A, void* Bm, int flags);

/* Condense: the LTV-QP Hessian H[B][nu*N][nu*N] and gradient g[B][nu*N] (kinematic);
 * on a cascaded context the first SQP iteration's QP Hessian H[B][2H][2H] and gradient
 * g[B][2H] in the scaled variable (oracle/casc_sqp.py casc_qp), ubar[B][H][2]. */
int vc_condense(vc_ctx* ctx, int B, const void* x0, const void* ubar, const void* kappa,
                const void* ds, void* H, void* g, int flags);

/* Plant step x_next = transition(x, u, kappa, dt) (temporal ODE), one per problem:
 * x[B][nx], u[B][nu], kappa[B], x_next[B][nx]. */
int vc_plant_step(vc_ctx* ctx, int B, const void* x, const void* u, const void* kappa,
                  double dt, void* x_next, int flags);

/* Spatial step x_next = spatial_transition(x, u, kappa, ds): ds[B]. */
int vc_spatial_step(vc_ctx* ctx, int B, const void* x, const void* u, const void* kappa,
                    const void* ds, void* x_next, int flags);

/* The continuous model f[b] = f(x[b], u[b], kappa[b]): space = 0 the temporal ODE (dx/dt, the
 * `f` of the plant's integrator), space = 1 the spatial ODE (dx/ds of the MPC's integrator).
 * x[B][nx], u[B][nu], kappa[B], f[B][nx] in the context dtype. */
int vc_ode(vc_ctx* ctx, int B, const void* x, const void* u, const void* kappa, int space, void* f, int flags);

/* ---- Track curvature and the batched closed loop ---------------
 *
 * The curvature k(s) is a piecewise cubic on a uniform grid, uploaded once per context:
 *   k(s) = c0 + c1 t + c2 t^2 + c3 t^3,  i = clamp(floor(s' / h), 0, n_pieces - 1),
 *   t = s' - i h,  coef[i] = (c0, c1, c2, c3),  s' = fmod(s, length)
 * i.e. the not-a-knot cubic through the curvature samples every h = 0.05 m of
 * track.py:156-167 (the CasADi bspline), extrapolating its last piece up to `length`.
 * Evaluated in fp64 on the device whatever the context dtype.  Deviation: the
 * reference's k does not wrap s (its simulator stops after one lap, racing.py:219);
 * the table is lap-periodic like get_curvature (track.py:111).
 * coef is host memory [n_pieces][4]; the call copies it and synchronises. */
int vc_track_set(vc_ctx* ctx, int n_pieces, double h, double length, const double* coef);

/* k[b] = k(s[b]) for B points (context dtype). */
int vc_track_k(vc_ctx* ctx, int B, const void* s, void* k, int flags);

/* Horizon parameters from the unshifted warm start (context dtype):
 *   kinematic (kinematic_mpc.py:178-187), xbar[B][N+1][6]:
 *     d_j = mpc_dt * v_j + 0.5 (j = 0..N), ds = d[0:N],
 *     kappa_k = k(s0 + (d_1 + ... + d_k)),  k = 0..N-1
 *   dynamic (cascaded_mpc.py:323-330), xbar[B][N][8]:
 *     ds_k = mpc_dt * Ux_k,  kappa_k = k(((ds_0 + ... + ds_k) - ds_0) + s0)
 * computed in fp64 in numpy's operation order, rounded to the context dtype on store. */
int vc_horizon(vc_ctx* ctx, int B, const void* x0, const void* xbar, double mpc_dt, void* kappa, void* ds,
               int flags);

/* Plant step of RacingCar.drive: x64 <- transition(x64, u0, k(s), dt) in fp64 (the
 * reference's plant is an fp64 CasADi function; kinematic Euler, dynamic RK4), with
 * k from the track table.  x64[B][nx] fp64 in/out, u0[B][nu] context dtype;
 * x_ctx[B][nx] (context dtype, may be NULL) receives the new state for the next solve. */
int vc_drive(vc_ctx* ctx, int B, double* x64, const void* u0, double dt, void* x_ctx, int flags);

/* `steps` closed-loop steps for B vehicles, all on the device (one HIP stream):
 *   vc_horizon(x, xbar) -> vc_solve(x, kappa, ds, xbar, ubar) -> vc_drive(x, u0)
 * x64[B][nx] fp64 in/out (plant state), xbar/ubar the warm starts in/out (context
 * dtype, shapes of vc_solve).  A problem whose status is not VC_SOLVED applies the
 * neutral input u = 0, increments nfail[b] (int32, may be NULL; not cleared), and restarts
 * from the neutral warm start (ubar = 0, xbar = the new state).  This is the build's own
 * policy: in the reference a failed IPOPT solve raises, step()'s catch-all prints it and
 * returns None (racing.py:416-423), and the caller's unpacking `action, state = self.step(...)`
 * (racing.py:232) raises TypeError, which ends the run.
 * Optional logs (may be NULL): log_x[steps+1][B][nx] fp64 (the state before each step
 * and after the last), log_u[steps][B][nu] context dtype (the applied u0).
 * Requires vc_track_set and a built vc_solve combination. */
int vc_simulate(vc_ctx* ctx, int B, int steps, double mpc_dt, double dt, double* x64, void* xbar, void* ubar,
                double* log_x, void* log_u, int32_t* nfail, int flags);

#ifdef __cplusplus
}
#endif
#endif /* VCMPC_H */
