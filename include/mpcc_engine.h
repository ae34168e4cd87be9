/*
 * mpcc_engine.h — C ABI of the MI355X batched MPCC solve engine (libmpcc_engine.so).
 *
 * Drop-in boundary for the reference's per-control-step solve (JunHeonYoon/MPCC_manipulator):
 *   - the solver plugin interface  SolverInterface            cpp/include/Interfaces/solver_interface.h:44-54
 *       setTrack(ArcLengthSpline)           -> mpcc_set_track
 *       setParam(const ParamValue&)         -> mpcc_set_params (+ mpcc_params_load_json)
 *       setEnvData(obs_position, radius)    -> per-instance obs[] argument of mpcc_solve
 *       setInitialGuess(vector<OptVariables>) + setCurrentInput(Input)
 *                                           -> device-resident warm start (mpcc_set_warmstart) and u0[]
 *       solveOCP(opt_sol, Status*, ComputeTime*) -> mpcc_solve (status[], horizon[], mpcc_timing)
 *   - the controller entry point MPC::runMPC_                cpp/src/MPC/mpc.cpp:104-190
 *       (projection, vs estimate, warm-start shift/regeneration, solve, status bookkeeping)
 *       -> mpcc_solve / mpcc_solve_device for B independent controllers at once.
 *   - MPC::setTrack(X, Y, Z, R)                              cpp/src/MPC/mpc.cpp:192-197
 *   - Params JSON loaders + ParamValue overrides           cpp/src/Params/params.cpp:24-448
 *
 * Conventions: plain pointers and sizes, row-major doubles, no C++ types and no exceptions across
 * the ABI.  Every entry point returns 0 on success or a negative MPCC_E_* code; the message of
 * the last error of the calling thread is available from mpcc_last_error().  Calls on one engine
 * handle must be serialized by the caller (as the reference's RobotModel is not reentrant);
 * engines on different devices are independent.
 *
 * Robot dimensions are compile-time, as the reference's NX/NU (config.h:29-38): MPCC_DOF = 7 is the
 * Franka Panda (libmpcc_engine.so), MPCC_DOF = 10 the Husky+Panda mobile manipulator of BASELINE
 * configs[3] (libmpcc_engine_mobile.so: planar base joints xb, yb, thb before q1..q7).  A client of
 * the mobile library compiles with -DMPCC_DOF=10; mpcc_robot_dof() reports the library's value.
 * NX = DOF + 2, NU = DOF + 1 below (9 / 8 for the Panda).
 *
 * Layouts (per instance b):
 *   x0     [NX]           q1..q7, s, vs         (types.h:33-57)       in/out: s, vs are overwritten
 *   u0     [NU]           dq1..dq7, dVs         (types.h:59-76)       current input (setCurrentInput)
 *   obs    [4]            obstacle x, y, z [m], radius [cm]  (runMPC_ obs_position, obs_radius)
 *   guess  [(N+1)*NXU]    per stage [x_k(NX), u_k(NU)] (OptVariables, osqp_interface.h:48-62)
 *   status                Status enum values (solver_interface.h:28-42)
 *   ok                    runMPC_ return value (mpc.cpp:188-189)
 */
#ifndef MPCC_ENGINE_H
#define MPCC_ENGINE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MPCC_ABI_VERSION 1

#ifndef MPCC_DOF
#define MPCC_DOF 7                       /* joints: 7 = Panda, 10 = Husky base (x, y, theta) + Panda */
#endif
/* Husky+Panda: panda_link0 sits at (0, 0, MPCC_MOBILE_MOUNT_Z) m in the base frame, a compile-time part of the
 * robot definition like the joint frames; mpcc_params_load_json refuses a parameter file whose
 * robot.mount differs, so editing it cannot silently have no effect */
#ifndef MPCC_MOBILE_MOUNT_Z
#define MPCC_MOBILE_MOUNT_Z 0.35
#endif
#define MPCC_NX (MPCC_DOF + 2)           /* state  [q, s, vs]   (config.h:29 NX = 9)  */
#define MPCC_NU (MPCC_DOF + 1)           /* input  [dq, dVs]    (config.h:30 NU = 8)  */
#define MPCC_NXU (MPCC_NX + MPCC_NU)     /* one horizon stage of OptVariables         */

enum {
    MPCC_OK = 0,
    MPCC_E_INVALID = -1,     /* bad argument / size / state */
    MPCC_E_HIP = -2,         /* HIP runtime error */
    MPCC_E_OOM = -3,         /* device allocation failed */
    MPCC_E_IO = -4,          /* file / JSON error */
    MPCC_E_NOTRACK = -5      /* solve before set_track */
};

/* Status — solver_interface.h:28-42 (same numeric values) */
enum {
    MPCC_SOLVED = 0, MPCC_MAX_ITER_EXCEEDED, MPCC_QP_DualInfeasibleInaccurate,
    MPCC_QP_PrimalInfeasibleInaccurate, MPCC_QP_SolvedInaccurate, MPCC_QP_MaxIterReached,
    MPCC_QP_PrimalInfeasible, MPCC_QP_DualInfeasible, MPCC_Sigint, MPCC_INVALID_SETTINGS,
    MPCC_NAN_HESSIAN, MPCC_NON_PD_HESSIAN
};

/* constraint_mask bits (polytopic rows, constraints.cpp:192-243) */
#define MPCC_CON_SELFCOL 1
#define MPCC_CON_SING 2
#define MPCC_CON_ENVCOL 4

/* Effective parameter values per consumer.  The reference keeps one copy per class and applies
 * ParamValue overrides inconsistently; mpcc_params_load_json resolves them exactly
 * as the reference's constructors and setParam do. */
typedef struct {
    int32_t N;                 /* horizon length (runtime; reference: compile-time, config.h:36) */
    double  Ts;                /* sample time (config.json) */
    int32_t constraint_mask;   /* MPCC_CON_* bits; reference behaviour = 7 */

    double proj_max_dist;      /* ArcLengthSpline::param_.max_dist_proj (projection)   */
    double guess_max_dist;     /* MPC::param_.max_dist_proj (warm-start invalidation)  */
    double desired_ee_velocity, deacc_ratio, cost_tol_selcol, cost_tol_sing;   /* Cost::param_ */
    double q_c, q_c_N_mult, q_l, q_vs, q_ori, q_sing, r_dq, r_dVs;              /* Cost::cost_param_ */
    double q_c_red_ratio, q_l_inc_ratio, q_ori_red_ratio;
    double qp_r_ddq;           /* OsqpInterface::cost_param_.r_ddq (file value only, Q8) */
    double con_tol_selcol, con_tol_sing, con_tol_envcol;                        /* Constraints::param_ */
    double s_trust_region;                                                      /* Bounds::param_ */
    double lx[MPCC_NX], ux[MPCC_NX], lu[MPCC_NU], uu[MPCC_NU];                  /* BoundsParam (file) */
    double lddq[MPCC_DOF], uddq[MPCC_DOF];
    double Tx[MPCC_NX], Tu[MPCC_NU];                                            /* NormalizationParam */
    double eps_prim, eps_dual, line_search_tau, line_search_eta, line_search_rho; /* SQPParam */
    int32_t max_iter, line_search_max_iter, do_SOC, use_BFGS;
    /* Parity policy P1: per-row constraint violations <= vio_floor count as zero in
     * the filter line search's constraint_norm (osqp_interface.cpp:824-833).  An exactly solved QP step
     * leaves violations at rounding-noise level (~1e-16..1e-12) where the reference's OSQP steps carry
     * ~eps_abs = 1e-4; without the floor the filter decision compares noise.  Default 1e-9. */
    double vio_floor;
} mpcc_params;

/* PathToJson (types.h:63-70).  Any of the six may be NULL when 'merged' is given: a single JSON
 * object with sections "model","cost","bounds","normalization","sqp","config". */
typedef struct {
    const char* param_path;
    const char* cost_path;
    const char* bounds_path;
    const char* normalization_path;
    const char* sqp_path;
    const char* merged_path;
} mpcc_json_paths;

/* One ParamValue entry (types.h:72-79): section in {"param","cost","bounds","normalization","sqp"} */
typedef struct {
    const char* section;
    const char* key;
    double value;
} mpcc_override;

typedef struct {
    int32_t N;                 /* horizon */
    double  Ts;
    int32_t max_batch;         /* instances the engine can hold (warm-start state is allocated for this many) */
    int32_t device;            /* HIP device ordinal */
    int32_t constraint_mask;   /* overrides params.constraint_mask when >= 0 */
    int32_t faithful_dead_trials; /* 1: also evaluate the line-search trials whose result the reference discards */
} mpcc_config;

/* ComputeTime (osqp_interface.h:71-79) for one batch call, seconds of device time (HIP events) */
typedef struct {
    double set_env;     /* stage linearization: kinematics, manipulability, NN distances */
    double set_qp;      /* QP assembly (cost/constraint/bound records) */
    double solve_qp;    /* interior-point QP solves */
    double get_alpha;   /* line search / step */
    double total;       /* whole runMPC_ batch incl. projection and warm start */
} mpcc_timing;

typedef struct mpcc_engine mpcc_engine;

int         mpcc_abi_version(void);
int         mpcc_robot_dof(void);   /* MPCC_DOF this library was built with (7 or 10) */
const char* mpcc_last_error(void);

/* Params JSON files + ParamValue -> effective values.  ctor_semantics=1 resolves as the
 * MPC(Ts, path, param_value) constructor (normalization/sqp overrides applied); 0 as
 * MPC::setParam (normalization/sqp keep their file values, osqp_interface.cpp:95-100). */
int mpcc_params_load_json(const mpcc_json_paths* paths, const mpcc_override* overrides, int n_overrides,
                          int ctor_semantics, int N, mpcc_params* out);

int  mpcc_create(const mpcc_config* cfg, const mpcc_params* params, const char* nn_dir, mpcc_engine** out);
void mpcc_destroy(mpcc_engine* e);
int  mpcc_set_params(mpcc_engine* e, const mpcc_params* params);
int  mpcc_get_params(mpcc_engine* e, mpcc_params* out);

/* MPC::setTrack(X, Y, Z, R): n way-points, R9 = n row-major 3x3.  Builds the arc-length spline on
 * the host (gen6DSpline, arc_length_spline.cpp:213-265) and uploads its tables.  Invalidates
 * every instance's warm start (mpc.cpp:196). */
int    mpcc_set_track(mpcc_engine* e, int n, const double* X, const double* Y, const double* Z, const double* R9);
/* SolverInterface::setTrack(const ArcLengthSpline) (solver_interface.h:46): the spline's regular path
 * data (ArcLengthSpline::getPathData(), arc_length_spline.h:108) — n = 100 points — refit exactly as
 * the reference's final fit (arc_length_spline.cpp:245-252).  Invalidates every warm start. */
int    mpcc_set_track_path(mpcc_engine* e, int n, const double* s, const double* X, const double* Y, const double* Z,
                           const double* R9);
/* Batched extension: one track per instance, instance b following way-points
 * [b*n, (b+1)*n) of X, Y, Z (R9: 9 per point) — each built as MPC::setTrack would.  Later calls may use
 * at most B instances; mpcc_set_track returns to one shared track.  mpcc_track_length / get_track_path
 * report instance 0's track.  Invalidates every warm start. */
int    mpcc_set_tracks(mpcc_engine* e, int B, int n, const double* X, const double* Y, const double* Z, const double* R9);
double mpcc_track_length(mpcc_engine* e);
/* final regular path data (getPathData): s, X, Y, Z [100], R9 [100*9] */
/* host-only: build the arc-length spline from way-points without an engine (no GPU needed) and
 * return its path data and total length (ArcLengthSpline::gen6DSpline + getPathData). */
int    mpcc_track_build_host(int n, const double* X, const double* Y, const double* Z, const double* R9,
                             double* s, double* Xo, double* Yo, double* Zo, double* Ro9, double* length);
/* host-only ArcLengthSpline queries on the spline of n way-points (built as mpcc_track_build_host):
 * getPosition / getDerivative / getSecondDerivative / getOrientation / getOrientationDerivative at M
 * arc lengths s (pos, d1, d2 [M*3], R [M*9], dR [M*3]; any may be NULL) and projectOnSpline(s_guess, ee)
 * for M points (arc_length_spline.cpp:267-379) */
int    mpcc_track_eval_host(int n, const double* X, const double* Y, const double* Z, const double* R9, int M,
                            const double* s, double* pos, double* d1, double* d2, double* R, double* dR);
int    mpcc_track_project_host(int n, const double* X, const double* Y, const double* Z, const double* R9, int M,
                               double proj_max_dist, const double* s_guess, const double* ee, double* s_out);
int    mpcc_get_track_path(mpcc_engine* e, double* s, double* X, double* Y, double* Z, double* R9);

/* Per-instance controller state (mpc.h:119-127), device resident.  guess [B*(N+1)*NXU]. */
int mpcc_set_warmstart(mpcc_engine* e, int B, const double* guess, const int32_t* valid, const int32_t* fails);
int mpcc_get_warmstart(mpcc_engine* e, int B, double* guess, int32_t* valid, int32_t* fails);
int mpcc_reset_warmstart(mpcc_engine* e, int B, const uint8_t* mask /* NULL = all */);

/* Device-to-device variant of mpcc_set_warmstart (asynchronous on 'stream', NULL = engine stream). */
int mpcc_set_warmstart_device(mpcc_engine* e, int B, const double* d_guess, const int32_t* d_valid,
                              const int32_t* d_fails, void* stream);

/* Live per-phase device timing of mpcc_solve_device calls: between begin and end every call records
 * HIP events on its stream (no synchronization); end synchronizes and returns the summed phase times
 * and the number of calls and of IPM (k_ipm) launches timed. */
int mpcc_timing_begin(mpcc_engine* e);
int mpcc_timing_end(mpcc_engine* e, mpcc_timing* sum, int32_t* n_calls, int32_t* n_ipm_launches);
/* the collision-MLP launches of the last timing window (after mpcc_timing_end): total seconds and launch count of
 * k_mlp_self and of k_mlp_env, from HIP events around those launches alone on the engine stream */
int mpcc_timing_mlp(mpcc_engine* e, double* self_s, int32_t* self_n, double* env_s, int32_t* env_n);
/* the fused SQP kernel (k_sqp, with k_sqp_solo beside it) of the last timing window: the summed launch spans in
 * seconds, the launch count, and the fractions of its waves' cycles in the phases of solveOCP's ComputeTime
 * (osqp_interface.cpp:435-564): frac[0] set_qp (QP assembly and Hessian update of SQP iterations >= 1), frac[1]
 * solve_qp (the QP solves and the correction), frac[2] get_alpha (line-search trials and the filter), frac[3] the
 * step update.  mpcc_timing_end splits the k_sqp span into set_qp / solve_qp / get_alpha by these fractions (the
 * step's share stays in total only, as in the reference).  n = 0 in the staged path (every phase has its own
 * launches and events there). */
int mpcc_timing_sqp(mpcc_engine* e, double* span_s, int32_t* n, double* frac4);
/* the launches of one kernel of e's last timing window (kind: MPCC_TIMING_QP = the QP solve, k_sqp or k_ipm in
 * the staged path; MPCC_TIMING_MLP_SELF / _MLP_ENV = the collision networks) as [start, end] in ms after the
 * first event of `anchor`'s window (anchor = e, or another engine on the same device): several engines stepping
 * on their own streams measure the union of their kernels' busy time.  *n = the number of intervals recorded,
 * of which the first min(*n, max) are written (*n > max: the buffers were too small) */
#define MPCC_TIMING_QP 0
#define MPCC_TIMING_MLP_SELF 1
#define MPCC_TIMING_MLP_ENV 2
int mpcc_timing_intervals(mpcc_engine* e, mpcc_engine* anchor, int kind, int max, double* start_ms, double* end_ms,
                          int32_t* n);

/* Per-instance iteration counts of the last solve: SQP iteration index at exit and IPM iterations of
 * the last QP (host arrays, may be NULL). */
int mpcc_get_solve_stats(mpcc_engine* e, int B, int32_t* sqp_iter, int32_t* ipm_iters, int32_t* qp_status);

/* Batched MPC::runMPC_ on host arrays (H2D, solve, D2H).  Any output pointer may be NULL. */
int mpcc_solve(mpcc_engine* e, int B, double* x0, const double* u0, const double* obs,
               double* u0_out, double* horizon_out, int32_t* status, int32_t* ok, mpcc_timing* timing);

/* Same on device-resident arrays; asynchronous on 'stream' (hipStream_t, NULL = engine stream).
 * Instances [0, B) of the engine's warm-start state are used. */
int mpcc_solve_device(mpcc_engine* e, int B, double* d_x0, const double* d_u0, const double* d_obs,
                      double* d_u0_out, double* d_horizon, int32_t* d_status, int32_t* d_ok, void* stream);

/* SolverInterface granularity (solver_interface.h:44-54): for B instances, setInitialGuess(guess) +
 * setCurrentInput(u_cur) + setEnvData(obs) + solveOCP(opt_sol, status, time)
 * (osqp_interface.cpp:102-127, 398-590).  No projection, warm-start shift or valid/fail bookkeeping:
 * that stays with the caller's MPC (mpc.cpp:104-189), as in the reference.  guess, opt_sol
 * [B*(N+1)*NXU]; u_cur [B*NU]; obs [B*4]; status [B]; solved [B] = solveOCP's bool (may be NULL).
 * Uses the engine's warm-start slots [0, B) as the iterate (they are overwritten). */
int mpcc_solve_ocp(mpcc_engine* e, int B, const double* guess, const double* u_cur, const double* obs,
                   double* opt_sol, int32_t* status, int32_t* solved, mpcc_timing* timing);

/* The reference's closed-loop driver (main.cpp:100-114) for B instances, device resident: each step runs
 * runMPC_ (the engine's warm-start state carries over; x's s and vs are updated as mpc.cpp:107-115), takes
 * u0 and integrates the updated state with simTimeStep (integrator.cpp:55-68).  An instance whose runMPC_
 * returns false stops (main.cpp:108-112): its state stays the one that entered that step and later steps
 * report status -1.  x0 [B*NX] / u0 [B*NU] in, out: final state / input; obs [B*4] constant;
 * x_traj [(steps+1)*B*NX], u_traj [steps*B*NU], status_traj [steps*B] (any may be NULL).
 * use_graph = 1 captures one control step in a hipGraph and replays it (same results, fewer launches). */
int mpcc_closed_loop(mpcc_engine* e, int B, int steps, double* x0, double* u0, const double* obs, double* x_traj,
                     double* u_traj, int32_t* status_traj, int use_graph);

/* Integrator::simTimeStep (integrator.cpp:55-68) for B states, host arrays (closed-loop driver). */
int mpcc_sim_time_step(mpcc_engine* e, int B, const double* x, const double* u, double ts, double* x_next);

/* ---- stand-alone objects of the reference's Python surface (MPCC_wrapper.cpp:254-347) ---- */
/* SelCollNNmodel / EnvCollNNmodel (SelfCollisionModel.cpp / EnvCollisionModel.cpp:75-250): setNeuralNetwork(
 * n_input, n_output, n_hidden, is_nerf) with the weights of dir (weight_l / bias_l as this repo's .f64 or the
 * reference's .txt), and calculateMlpOutput for M inputs on the GPU: out [M*n_output] and the full Jacobian
 * jac [M*n_output*n_input] (row-major; may be NULL).  At most 16 inputs and 7 hidden layers. */
typedef struct mpcc_mlp mpcc_mlp;
int  mpcc_mlp_create(int device, const char* dir, int n_input, int n_output, const int32_t* n_hidden, int n_layers_hidden,
                     int is_nerf, mpcc_mlp** out);
int  mpcc_mlp_eval(mpcc_mlp* m, int M, const double* in, double* out, double* jac);
int  mpcc_mlp_dims(mpcc_mlp* m, int32_t* n_input, int32_t* n_output);
void mpcc_mlp_destroy(mpcc_mlp* m);
/* RobotModel::getPosition / getOrientation / getJacobian / getManipulability / getDManipulability with a frame_id
 * (robot_model.cpp:354-450; frame 1 = panda_link0, 2..8 = panda_link1..7, 9 = panda_hand_tcp) for M joint vectors
 * q [M*7] (Panda library only) on GPU 'device': pos [M*3], R [M*9], J [M*42] (rows Jv; Jw), mani [M], dmani [M*7]; any may be NULL. */
int  mpcc_robot_frames(int device, int M, const double* q, int frame_id, double* pos, double* R, double* J, double* mani,
                       double* dmani);
/* CubicSpline::genSpline + getPoint/getDerivative/getSecondDerivative (cubic_spline.cpp:65-246) of n points at m
 * abscissas, host only: out3 [m*3] = value, d1, d2.  regular = 1: regular grid (index by floor(x/dx)). */
int  mpcc_cubic_spline_host(int n, const double* x, const double* y, int regular, int m, const double* xq, double* out3);
/* CubicSplineRot::genSpline + getPoint/getDerivative (cubic_spline_rot.cpp:142-259), host only: R9 [n*9] in,
 * Rq [m*9], dRq [m*3] out (either may be NULL). */
int  mpcc_rot_spline_host(int n, const double* x, const double* R9, int regular, int m, const double* xq, double* Rq,
                          double* dRq);
/* LogMatrix / ExpMatrix (cubic_spline_rot.cpp:44-95, quirks Q10/Q11), host only: 3x3 row-major */
int  mpcc_so3_log(const double* R9, double* S9);
int  mpcc_so3_exp(const double* S9, double* R9);

/* ---- stage-level entry points for parity tests (host arrays) ---- */
#define MPCC_REC_SIZE (24 + 17 * MPCC_DOF)   /* 143 for the Panda: robot_data.h:13-31 */
/* RobotData::update + updateEnv (robot_data.h:55-88) for M joint vectors q[M*DOF], obs[M*4] */
int mpcc_debug_robot_records(mpcc_engine* e, int M, const double* q, const double* obs, double* rec);
/* ArcLengthSpline evals at M arc lengths: pos,d,dd [M*3], R [M*9], dR [M*3] */
int mpcc_debug_spline(mpcc_engine* e, int M, const double* s, double* pos, double* d, double* dd, double* R, double* dR);
/* Cost::getCost for M (x,u,rec,k) tuples: obj [M], fx [M*NX], fu [M*NU], fxx [M*NX*NX], fuu [M*NU*NU] */
int mpcc_debug_stage_cost(mpcc_engine* e, int M, const double* x, const double* u, const double* rec, const int32_t* k,
                          double* obj, double* fx, double* fu, double* fxx, double* fuu);
/* ArcLengthSpline::projectOnSpline (arc_length_spline.cpp:318-379) for M (s_guess, ee[3]) pairs */
int mpcc_debug_project(mpcc_engine* e, int M, const double* s_guess, const double* ee, double* s_out);

/* one QP of the SQP for B instances: guess [B*(N+1)*NXU], rec [B*(N+1)*MPCC_REC_SIZE], u_cur [B*NU]
 * -> step [B*(NXU*N+NX)] in the reference's stacked layout, qp_status [B], ipm_iters [B] */
int mpcc_debug_solve_qp(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur,
                        double* step, int32_t* qp_status, int32_t* ipm_iters);

/* the same QP with low-rank Hessian terms sum_j lrc_j u_j u_j^T (the damped-BFGS QP form): lr [nlr*(N+1)*NXU]
 * (per stage [x | u], u_N = 0), lrc [nlr], nlr <= 28, solved by the 32-lane interior point with the Woodbury
 * correction (nlr > 4: the extended path, Woodbury columns and capacitance matrix in memory) */
int mpcc_debug_solve_qp_lr(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur, int nlr,
                           const double* lr, const double* lrc, double* step, int32_t* qp_status, int32_t* ipm_iters);

/* SQP trace of the next solves (test instrumentation, off by default): per instance and SQP iteration
 * (at most 4) 8 doubles: qp status, ipm iterations, trial objective and violation at alpha = 1,
 * accepted, |step|_inf, alpha, alpha*|step|_inf (osqp_interface.cpp:540-574, 759-808). */
int mpcc_debug_trace_enable(mpcc_engine* e, int enable);
/* raw interior-point workspace of the last solve [B*(N+1)*MPCC_IPM_WS] (layout: csrc/ipm.hip WF_*,
 * csrc/ipm_wide.hip for the mobile library) */
#if MPCC_DOF == 7
#define MPCC_IPM_WS 816
#else
#define MPCC_IPM_WS 2048
#endif
int mpcc_debug_workspace(mpcc_engine* e, int B, double* out);
int mpcc_debug_trace_get(mpcc_engine* e, int B, double* out /* [B*4*8] */);
/* bounds-checked build only (mpcc_build_flags() & MPCC_BUILD_BOUNDS_CHECK): OR of the violation bits every kernel
 * recorded since the last clear (0 = every computed workspace / record / ring / LDS / spline index in range;
 * bits: csrc/dev_common.h BC_*); MPCC_E_INVALID on a normal build */
int mpcc_debug_bounds(mpcc_engine* e, uint32_t* flags, int clear);
/* QP solves the fused kernels finished in tail mode (the wave's last running instance on all four 16-lane groups,
 * csrc/ipm_tail.h) since the last reset, over all engines of the process; Panda library, <= 2 polytopic rows */
int mpcc_debug_tail_solves(long long* out, int reset);
/* k_sqp's group slots of the last fused solve (csrc/kernels.hip k_order): out[i] = instance of 16-lane group slot i
 * (wave i / 4), -1 empty, for 4 * (ceil(B / 4) + 64) slots, then k_prepare's cold-start flag of each instance [B];
 * returns the number copied.  Cold-started instances get a wave of their own (solo waves); with solo waves off
 * (MPCC_SOLO=0) k_order does not run and the slots are stale. */
int mpcc_debug_order(mpcc_engine* e, int32_t* out, int n);

/* Build provenance (no reference counterpart): a hash of the sources the library was compiled from
 * (csrc/ and include/, mpcc_manipulator_amd/_build.py source_hash) and the build's variant bits. */
const char* mpcc_build_id(void);
#define MPCC_BUILD_BOUNDS_CHECK 1
#define MPCC_BUILD_PROF 2
int mpcc_build_flags(void);

#ifdef __cplusplus
}
#endif
#endif /* MPCC_ENGINE_H */
