// mpcc_mpc.hpp — C++ host surface of the MI355X engine, mirroring the reference's controller API.
//
// Reference: cpp/include/MPC/mpc.h:58-128 (class MPC, struct MPCReturn), cpp/include/types.h (State,
// Input, OptVariables, ParamValue, PathToJson), cpp/include/Interfaces/solver_interface.h:28-54
// (Status).  Same names, argument meaning and return rule; differences:
//   * no Eigen in the interface: vectors are std::array / std::vector<double>;
//   * the horizon N is a constructor argument (reference: compile-time config.h:36);
//   * the solver behind runMPC_ is the engine (libmpcc_engine.so, include/mpcc_engine.h) instead of
//     OsqpInterface (mpc.cpp:31,45) — the OSQP QP is replaced by an exact interior-point solve;
//   * BatchMPC adds the batched entry (B independent controllers per call), SURVEY.md §8(b);
//   * engine/HIP failures throw mpcc_amd::Error (the reference has no failure path there).
#pragma once
#include <array>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mpcc_engine.h"

namespace mpcc_amd {

constexpr int NX = 9, NU = 8;

struct State {   // types.h: q1..q7, s, vs
    double q1 = 0, q2 = 0, q3 = 0, q4 = 0, q5 = 0, q6 = 0, q7 = 0, s = 0, vs = 0;
};
struct Input {   // types.h: dq1..dq7, dVs
    double dq1 = 0, dq2 = 0, dq3 = 0, dq4 = 0, dq5 = 0, dq6 = 0, dq7 = 0, dVs = 0;
};
struct OptVariables {
    State xk;
    Input uk;
};
struct ComputeTime {  // types.h ComputeTime (seconds)
    double set_env = 0, set_qp = 0, solve_qp = 0, get_alpha = 0, total = 0;
};
enum Status {  // solver_interface.h:28-42
    SOLVED, MAX_ITER_EXCEEDED, QP_DualInfeasibleInaccurate, QP_PrimalInfeasibleInaccurate, QP_SolvedInaccurate,
    QP_MaxIterReached, QP_PrimalInfeasible, QP_DualInfeasible, Sigint, INVALID_SETTINGS, NAN_HESSIAN, NON_PD_HESSIAN
};
struct MPCReturn {  // mpc.h:35-48
    Input u0;
    std::vector<OptVariables> mpc_horizon;
    ComputeTime compute_time;
};
struct PathToJson {  // types.h PathToJson (+ nn_dir: the reference reads the weights from pkg_path)
    std::string param_path, cost_path, bounds_path, track_path, normalization_path, sqp_path;
    std::string nn_dir;
    std::string merged_path;  // alternative to the five files: one JSON with a section per file
};
// the package's shipped data (mpcc_manipulator_amd/data): merged params, default track, MLP weights
PathToJson defaultPaths(const std::string& data_dir);
// types.h:143-150 ParamValue (same members; 'track' is carried but, as in the reference, not read)
struct ParamValue {
    std::map<std::string, double> param, cost, bounds, track, normalization, sqp;
};
using Rot = std::array<double, 9>;  // row-major 3x3

class Error : public std::runtime_error {
   public:
    using std::runtime_error::runtime_error;
};

struct TrackPoints {  // Track::getTrack result (track.cpp:56-66)
    std::vector<double> X, Y, Z;
    std::vector<Rot> R;
};
// Track(file).getTrack(init_position): Params/track.json (X, Y, Z, quat_X..quat_W) offset so that the
// path starts at init_position (track.cpp:19-66).  Also reads the package's {"points": [[x,y,z,qx,qy,qz,qw]..]}.
TrackPoints loadTrack(const std::string& track_json, const std::array<double, 3>& init_position);

// B independent controllers on one GPU; per-instance warm start (mpc.h:119-127) stays in HBM.
class BatchMPC {
   public:
    BatchMPC(int N, double Ts, int max_batch, const PathToJson& path, const ParamValue& param_value = ParamValue{},
             int device = 0, int constraint_mask = MPCC_CON_SELFCOL | MPCC_CON_SING | MPCC_CON_ENVCOL);
    ~BatchMPC();
    BatchMPC(const BatchMPC&) = delete;
    BatchMPC& operator=(const BatchMPC&) = delete;

    void setTrack(const std::vector<double>& X, const std::vector<double>& Y, const std::vector<double>& Z,
                  const std::vector<Rot>& R);
    double getTrackLength();
    void setParam(const ParamValue& param_value);  // MPC::setParam semantics (mpc.cpp:204-209)
    // runMPC_ for instances 0..B-1: x0 [B*9] in/out (s, vs replaced as mpc.cpp:107-115), u0 [B*8],
    // obs [B*4] (xyz in m, radius in cm) -> u0_out [B*8], horizon [B*(N+1)*17], status [B], ok [B]
    void runMPCBatch(int B, double* x0, const double* u0, const double* obs, double* u0_out, double* horizon,
                     int32_t* status, int32_t* ok, ComputeTime* time = nullptr);
    void resetWarmStart(int B);
    // RobotModel::getEEPosition (robot_model.cpp:366-398), evaluated on the GPU
    std::array<double, 3> eePosition(const std::array<double, 7>& q);
    int horizon() const { return N_; }
    mpcc_engine* engine() { return e_; }

   private:
    int N_;
    double Ts_;
    PathToJson path_;
    int mask_;
    mpcc_engine* e_ = nullptr;
};

// The reference's solver plugin interface without Eigen (SolverInterface, solver_interface.h:44-54),
// one controller.  A reference-side `HipSolverInterface : SolverInterface` forwards
// its six virtuals here, and MPC keeps its own projection / warm-start code (mpc.cpp:104-189).
class OcpSolver {
   public:
    OcpSolver(int N, double Ts, const PathToJson& path, const ParamValue& param_value = ParamValue{},
              int device = 0, int constraint_mask = MPCC_CON_SELFCOL | MPCC_CON_SING | MPCC_CON_ENVCOL);
    // ArcLengthSpline::getPathData() of the caller's spline: s, X, Y, Z, R (100 points)
    void setTrack(const std::vector<double>& s, const std::vector<double>& X, const std::vector<double>& Y,
                  const std::vector<double>& Z, const std::vector<Rot>& R);
    void setParam(const ParamValue& param_value);
    void setEnvData(const std::array<double, 3>& obs_position, const double& obs_radius);
    void setInitialGuess(const std::vector<OptVariables>& initial_guess);
    void setCurrentInput(const Input& current_input);
    bool solveOCP(std::vector<OptVariables>& opt_sol, Status* status, ComputeTime* mpc_time);

   private:
    BatchMPC impl_;
    double obs_[4] = {3.0, 3.0, 3.0, 0.0};
    double ucur_[NU] = {};
    std::vector<double> guess_;
};

// One controller, the reference's MPC (mpc.h:58-128).
class MPC {
   public:
    MPC(int N, double Ts, const PathToJson& path, int device = 0);
    MPC(int N, double Ts, const PathToJson& path, const ParamValue& param_value, int device = 0);
    // runMPC: dummy obstacle (3, 3, 3), r = 0 (mpc.cpp:92-102)
    bool runMPC(MPCReturn& mpc_return, State& x0, Input& u0);
    // runMPC_ (mpc.cpp:104-190): returns SOLVED || (MAX_ITER_EXCEEDED && fewer than 5 failures in a row)
    bool runMPC_(MPCReturn& mpc_return, State& x0, Input& u0, const std::array<double, 3>& obs_position,
                 const double& obs_radius);
    void setTrack(const std::vector<double>& X, const std::vector<double>& Y, const std::vector<double>& Z,
                  const std::vector<Rot>& R);
    double getTrackLength();
    void setParam(const ParamValue& param_value);
    Status lastStatus() const { return last_status_; }
    std::array<double, 3> eePosition(const std::array<double, 7>& q) { return impl_.eePosition(q); }
    int horizon() const { return impl_.horizon(); }
    mpcc_engine* engine() { return impl_.engine(); }

   private:
    BatchMPC impl_;
    Status last_status_ = SOLVED;
};

}  // namespace mpcc_amd
