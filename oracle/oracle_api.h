/*
 * oracle_api.h — C interface of the CPU parity ORACLE.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is a line-by-line CPU restatement of the reference
 * MPCC hot path (JunHeonYoon/MPCC_manipulator, cpp/src/...).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / CPU baseline — the
 * product (mpcc_manipulator_amd, libmpcc_engine.so) never links or calls it.
 *
 * Parity pinning: the reference itself cannot be built here (Eigen, RBDL,
 * OSQP, osqp-eigen are absent and fetched at unpinned HEAD by cpp/install.sh:39-44), so this
 * restatement is pinned by the reference's known-answer values (python/main_utils.py:50,52;
 * cpp/include/Tests/robot_model_test.h:28-29,80-82) and by its property tests (cpp/include/Tests/ headers),
 * ported in tests/test_oracle_*.py.  OSQP (time-limited ADMM, osqp_interface.cpp:620-651) is replaced
 * by an exact interior-point solve of the same QP; "dense" mode solves the reference's dense
 * QP layout verbatim, "riccati" mode the equivalent stage-structured QP.
 */
#ifndef MPCC_ORACLE_API_H
#define MPCC_ORACLE_API_H
/* Robot: ORC_DOF 7 = Franka Panda (liboracle.so), 10 = Husky+Panda mobile manipulator
 * (liboracle_mobile.so, BASELINE configs[3]); arrays below are sized by it. */
#ifndef ORC_DOF
#define ORC_DOF 7
#endif
#define ORC_NX (ORC_DOF + 2)
#define ORC_NU (ORC_DOF + 1)
#ifdef __cplusplus
extern "C" {
#endif

/* Effective parameter values per consumer (the reference keeps separate copies per class and
 * applies overrides inconsistently — SURVEY §9 Q8; the caller resolves them). */
typedef struct {
    int    N;                 /* horizon (reference: compile-time N, config.h:36) */
    double Ts;                /* sample time */
    int    constraint_mask;   /* bit0 self-collision rows, bit1 singularity row, bit2 env rows */

    /* ArcLengthSpline::param_ (projection) and MPC::param_ (guess invalidation) */
    double proj_max_dist, guess_max_dist;
    /* Cost::param_ + Cost::cost_param_ (cost.cpp) */
    double desired_ee_velocity, deacc_ratio, cost_tol_selcol, cost_tol_sing;
    double q_c, q_c_N_mult, q_l, q_vs, q_ori, q_sing, r_dq, r_dVs;
    double q_c_red_ratio, q_l_inc_ratio, q_ori_red_ratio;
    /* OsqpInterface::cost_param_.r_ddq (osqp_interface.cpp:28; never overridden — Q8) */
    double qp_r_ddq;
    /* Constraints::param_ */
    double con_tol_selcol, con_tol_sing, con_tol_envcol;
    /* Bounds (bounds.cpp) */
    double s_trust_region;
    double lx[ORC_NX], ux[ORC_NX], lu[ORC_NU], uu[ORC_NU], lddq[ORC_DOF], uddq[ORC_DOF];
    /* NormalizationParam diag(T_x), diag(T_u) */
    double Tx[ORC_NX], Tu[ORC_NU];
    /* SQPParam */
    double eps_prim, eps_dual, line_search_tau, line_search_eta, line_search_rho;
    int    max_iter, line_search_max_iter, do_SOC, use_BFGS;
    /* Parity policy P1: per-row constraint violations <= vio_floor count as zero in the
     * filter line search (constraint_norm), removing the rounding noise an exact QP leaves behind. */
    double vio_floor;
} OracleParams;

typedef struct {
    int    qp_mode;        /* 0 = riccati (stage-structured IPM), 1 = dense reference layout IPM, 2 = dense with the
                              reference's in-place BFGSUpdate verbatim (no low-rank cap / restart: deviation 7) */
    int    nthreads;       /* OpenMP threads for batch calls */
} OracleOptions;

void*  oracle_create(const OracleParams* p, const char* nn_dir, OracleOptions opt);
int    oracle_dof(void);  /* ORC_DOF of this build */
void   oracle_destroy(void* h);
void   oracle_set_params(void* h, const OracleParams* p);
/* MPC::setTrack(X,Y,Z,R) -> ArcLengthSpline::gen6DSpline (arc_length_spline.cpp:213-265) */
void   oracle_set_track(void* h, int n, const double* X, const double* Y, const double* Z, const double* R9);
double oracle_track_length(void* h);
/* final regular spline tables: s[100], x,y,z [100] */
void   oracle_track_path(void* h, double* s, double* X, double* Y, double* Z, double* R9);

/* RobotModel (robot_model.cpp:366-450) */
void   oracle_fk(const double* q, double* pos3, double* R9, double* J42);
double oracle_manipulability(const double* q);
/* RobotModel frame 1..9 (panda_link0..7, panda_hand_tcp): robot_model.cpp:354-398 */
void   oracle_fk_frame(const double* q, int frame, double* pos3, double* R9, double* J42);
double oracle_manip_from_J(const double* J42);
void   oracle_dmanipulability(const double* q, double* d7);
/* NN models (SelfCollisionModel.cpp:140-250, EnvCollisionModel.cpp:137-247) */
void   oracle_self_mlp(void* h, const double* q7, double* d, double* grad7);
void   oracle_env_mlp(void* h, const double* in10, double* d9, double* jac90);
/* Spline eval (arc_length_spline.cpp:267-316) */
void   oracle_spline_eval(void* h, double s, double* pos, double* d, double* dd, double* R9, double* dR);
double oracle_project(void* h, double s, const double* ee3);
/* RobotData::update + updateEnv (robot_data.h:55-88); record layout = ORACLE_REC_* */
void   oracle_robot_record(void* h, const double* q7, const double* obs3, double obs_r, double* rec);
/* Cost::getCost (cost.cpp:290-357): obj, f_x[9], f_u[8], f_xx[81], f_uu[64], f_xu[72] */
void   oracle_stage_cost(void* h, const double* x9, const double* u8, const double* rec, int k,
                         double* obj, double* fx, double* fu, double* fxx, double* fuu, double* fxu);
/* Constraints::getConstraints (constraints.cpp:192-243): c[11], l[11], u[11], cx[99], cu[88] */
void   oracle_stage_constraints(void* h, const double* x9, const double* u8, const double* rec, int k,
                                double* c, double* l, double* u, double* cx, double* cu);
/* OsqpInterface::setQP in the reference's dense layout (osqp_interface.cpp:129-396).
 * guess = (N+1)*17 [x_k(9), u_k(8)], recs = (N+1)*ORACLE_REC_SIZE.
 * P [nv*nv], g [nv], A [nc*nv], l,u,c [nc]; nv = 17N+9, nc = 45N+29. obj returned. */
double oracle_dense_qp(void* h, const double* guess, const double* recs, const double* u_current,
                       double* P, double* g, double* A, double* c, double* l, double* u);
/* Solve one SQP QP (given guess/recs/u_current) with the selected solver; step [nv]; returns status
 * (0 ok, else Status code).  iters = IPM iterations used. */
int    oracle_solve_qp(void* h, int mode, const double* guess, const double* recs, const double* u_current,
                       double* step, int* iters);
/* one QP with low-rank Hessian terms sum_j lrc_j u_j u_j^T (u_j [(N+1)*NXU] horizon layout; damped-BFGS form) */
int    oracle_solve_qp_lr(void* h, int mode, const double* guess, const double* recs, const double* u_current, int nlr,
                          const double* lr, const double* lrc, double* step, int* iters);
/* SecondOrderCorrection QP (osqp_interface.cpp:658-681) after the first step step_in [nv]: same P, q, A,
 * bounds at guess + step_in shifted by A step_in; step_out [nv]; returns status. */
int    oracle_solve_soc(void* h, int mode, const double* guess, const double* recs, const double* u_current,
                        const double* step_in, double* step_out, int* iters);
/* Integrator (integrator.cpp:29-68) */
void   oracle_rk4(const double* x9, const double* u8, double ts, double* out9);
void   oracle_sim_time_step(const double* x9, const double* u8, double ts, double* out9);

/* Batched MPC::runMPC_ (mpc.cpp:104-190).  Per-instance controller state (mpc.h:119-127) is
 * owned by the caller: guess [B*(N+1)*17], valid [B], fails [B] (in/out).
 * x0 [B*9] in/out (s and vs are overwritten as the reference does), u0 [B*8], obs [B*4] (xyz, r).
 * Outputs: u0_out [B*8], horizon [B*(N+1)*17], status [B], ok [B] (runMPC_ return value),
 * sqp_iters [B] (may be NULL).  Returns 0. */
int    oracle_run_mpc(void* h, int B, double* x0, const double* u0, const double* obs,
                      double* guess, int* valid, int* fails,
                      double* u0_out, double* horizon, int* status, int* ok, int* sqp_iters);
/* runMPC_ up to the SQP (projection, warm start, robot records at the warm start) -> recs [B*(N+1)*REC] */
int    oracle_prepare(void* h, int B, double* x0, const double* u0, const double* obs, double* guess, int* valid,
                      int* fails, double* recs);
/* same, plus a per-instance SQP trace [B*4*8] (see mpcc_debug_trace_get) */
int    oracle_run_mpc_trace(void* h, int B, double* x0, const double* u0, const double* obs, double* guess, int* valid,
                            int* fails, double* u0_out, double* horizon, int* status, int* ok, int* sqp_iters,
                            double* trace);

int    oracle_rec_size(void);
/* CubicSpline (cubic_spline.cpp) fit to (x, y) [n], evaluated at xq [m] -> out [m*3]: y, y', y'' */
void   oracle_cubic_spline(int n, const double* x, const double* y, int regular, int m, const double* xq, double* out3);

#ifdef __cplusplus
}
#endif
#endif
