// mpc.cpp — C++ host surface (include/mpcc_mpc.hpp) over the engine's C ABI: the reference's MPC
// (cpp/src/MPC/mpc.cpp) with OsqpInterface swapped for the MI355X engine, plus the batched entry.
#include "mpcc_mpc.hpp"

#include <cstring>

#include "host_json.h"
#include "host_spline.h"

namespace mpcc_amd {

namespace {

void check(int rc, const char* what) {
    if (rc != MPCC_OK) throw Error(std::string(what) + ": " + mpcc_last_error());
}

// Params/*.json + ParamValue -> engine parameter block (params.cpp, mpc.cpp:40-52 / 204-209 semantics)
mpcc_params load(int N, double Ts, const PathToJson& path, const ParamValue& pv, bool ctor, int mask) {
    mpcc_json_paths p{};
    auto cs = [](const std::string& s) -> const char* { return s.empty() ? nullptr : s.c_str(); };
    p.param_path = cs(path.param_path);
    p.cost_path = cs(path.cost_path);
    p.bounds_path = cs(path.bounds_path);
    p.normalization_path = cs(path.normalization_path);
    p.sqp_path = cs(path.sqp_path);
    p.merged_path = cs(path.merged_path);
    std::vector<mpcc_override> ov;
    const std::pair<const char*, const std::map<std::string, double>*> secs[] = {
        {"param", &pv.param}, {"cost", &pv.cost}, {"bounds", &pv.bounds},
        {"normalization", &pv.normalization}, {"sqp", &pv.sqp}};
    for (const auto& sec : secs)
        for (const auto& kv : *sec.second) ov.push_back({sec.first, kv.first.c_str(), kv.second});
    mpcc_params out;
    check(mpcc_params_load_json(&p, ov.empty() ? nullptr : ov.data(), (int)ov.size(), ctor ? 1 : 0, N, &out),
          "mpcc_params_load_json");
    out.Ts = Ts;
    out.constraint_mask = mask;
    return out;
}

}  // namespace

PathToJson defaultPaths(const std::string& data_dir) {
    PathToJson p;
    p.merged_path = data_dir + "/params/default_params.json";
    p.track_path = data_dir + "/params/default_track.json";
    p.nn_dir = data_dir + "/nn";
    return p;
}

TrackPoints loadTrack(const std::string& track_json, const std::array<double, 3>& init_position) {
    TrackPoints t;
    try {
        const mpcc::JVal j = mpcc::json_load_file(track_json);
        std::vector<double> qx, qy, qz, qw;
        if (j.has("points")) {
            for (const auto& pt : j.at("points").arr) {
                const auto v = pt.numbers();
                if (v.size() != 7) throw Error("loadTrack: point with " + std::to_string(v.size()) + " values");
                t.X.push_back(v[0]); t.Y.push_back(v[1]); t.Z.push_back(v[2]);
                qx.push_back(v[3]); qy.push_back(v[4]); qz.push_back(v[5]); qw.push_back(v[6]);
            }
        } else {
            t.X = j.at("X").numbers();
            t.Y = j.at("Y").numbers();
            t.Z = j.at("Z").numbers();
            qx = j.at("quat_X").numbers(); qy = j.at("quat_Y").numbers();
            qz = j.at("quat_Z").numbers(); qw = j.at("quat_W").numbers();
        }
        if (t.X.empty() || t.Y.size() != t.X.size() || t.Z.size() != t.X.size() || qx.size() != t.X.size() ||
            qy.size() != qx.size() || qz.size() != qx.size() || qw.size() != qx.size())
            throw Error("loadTrack: inconsistent array lengths in " + track_json);
        const double x0 = t.X[0], y0 = t.Y[0], z0 = t.Z[0];
        for (size_t i = 0; i < t.X.size(); i++) {
            t.X[i] = t.X[i] - x0 + init_position[0];
            t.Y[i] = t.Y[i] - y0 + init_position[1];
            t.Z[i] = t.Z[i] - z0 + init_position[2];
            Rot R;
            mpcc::quat_to_rot(qx[i], qy[i], qz[i], qw[i], R.data());
            t.R.push_back(R);
        }
    } catch (const Error&) {
        throw;
    } catch (const std::exception& x) {
        throw Error(std::string("loadTrack: ") + x.what());
    }
    return t;
}

// ------------------------------------------------------------------------------------------------
BatchMPC::BatchMPC(int N, double Ts, int max_batch, const PathToJson& path, const ParamValue& param_value,
                   int device, int constraint_mask)
    : N_(N), Ts_(Ts), path_(path), mask_(constraint_mask) {
    const mpcc_params p = load(N, Ts, path, param_value, true, constraint_mask);
    mpcc_config cfg{};
    cfg.N = N;
    cfg.Ts = Ts;
    cfg.max_batch = max_batch;
    cfg.device = device;
    cfg.constraint_mask = constraint_mask;
    cfg.faithful_dead_trials = 0;
    check(mpcc_create(&cfg, &p, path.nn_dir.empty() ? nullptr : path.nn_dir.c_str(), &e_), "mpcc_create");
}

BatchMPC::~BatchMPC() {
    if (e_) mpcc_destroy(e_);
}

void BatchMPC::setTrack(const std::vector<double>& X, const std::vector<double>& Y, const std::vector<double>& Z,
                        const std::vector<Rot>& R) {
    if (Y.size() != X.size() || Z.size() != X.size() || R.size() != X.size()) throw Error("setTrack: size mismatch");
    std::vector<double> R9(9 * R.size());
    for (size_t i = 0; i < R.size(); i++) std::memcpy(&R9[9 * i], R[i].data(), 9 * sizeof(double));
    check(mpcc_set_track(e_, (int)X.size(), X.data(), Y.data(), Z.data(), R9.data()), "mpcc_set_track");
}

double BatchMPC::getTrackLength() { return mpcc_track_length(e_); }

void BatchMPC::setParam(const ParamValue& param_value) {
    const mpcc_params p = load(N_, Ts_, path_, param_value, false, mask_);
    check(mpcc_set_params(e_, &p), "mpcc_set_params");
}

void BatchMPC::runMPCBatch(int B, double* x0, const double* u0, const double* obs, double* u0_out, double* horizon,
                           int32_t* status, int32_t* ok, ComputeTime* time) {
    mpcc_timing tm{};
    check(mpcc_solve(e_, B, x0, u0, obs, u0_out, horizon, status, ok, time ? &tm : nullptr), "mpcc_solve");
    if (time) *time = {tm.set_env, tm.set_qp, tm.solve_qp, tm.get_alpha, tm.total};
}

void BatchMPC::resetWarmStart(int B) { check(mpcc_reset_warmstart(e_, B, nullptr), "mpcc_reset_warmstart"); }

std::array<double, 3> BatchMPC::eePosition(const std::array<double, 7>& q) {
    const double obs[4] = {3.0, 3.0, 3.0, 0.0};
    std::vector<double> rec(MPCC_REC_SIZE);
    check(mpcc_debug_robot_records(e_, 1, q.data(), obs, rec.data()), "mpcc_debug_robot_records");
    return {rec[0], rec[1], rec[2]};
}

// ------------------------------------------------------------------------------------------------
OcpSolver::OcpSolver(int N, double Ts, const PathToJson& path, const ParamValue& param_value, int device,
                     int constraint_mask)
    : impl_(N, Ts, 1, path, param_value, device, constraint_mask), guess_((size_t)(N + 1) * 17, 0.0) {}

void OcpSolver::setTrack(const std::vector<double>& s, const std::vector<double>& X, const std::vector<double>& Y,
                         const std::vector<double>& Z, const std::vector<Rot>& R) {
    const size_t n = s.size();
    if (X.size() != n || Y.size() != n || Z.size() != n || R.size() != n) throw Error("setTrack: size mismatch");
    std::vector<double> R9(9 * n);
    for (size_t i = 0; i < n; i++) std::memcpy(&R9[9 * i], R[i].data(), 9 * sizeof(double));
    check(mpcc_set_track_path(impl_.engine(), (int)n, s.data(), X.data(), Y.data(), Z.data(), R9.data()),
          "mpcc_set_track_path");
}

void OcpSolver::setParam(const ParamValue& param_value) { impl_.setParam(param_value); }

void OcpSolver::setEnvData(const std::array<double, 3>& obs_position, const double& obs_radius) {
    obs_[0] = obs_position[0]; obs_[1] = obs_position[1]; obs_[2] = obs_position[2]; obs_[3] = obs_radius;
}

void OcpSolver::setInitialGuess(const std::vector<OptVariables>& g) {
    const int N = impl_.horizon();
    if ((int)g.size() != N + 1) throw Error("setInitialGuess: expected N+1 stages");
    for (int k = 0; k <= N; k++) {
        const State& x = g[k].xk;
        const Input& u = g[k].uk;
        const double v[17] = {x.q1, x.q2, x.q3, x.q4, x.q5, x.q6, x.q7, x.s, x.vs,
                              u.dq1, u.dq2, u.dq3, u.dq4, u.dq5, u.dq6, u.dq7, u.dVs};
        std::memcpy(&guess_[(size_t)17 * k], v, sizeof v);
    }
}

void OcpSolver::setCurrentInput(const Input& u) {
    const double v[NU] = {u.dq1, u.dq2, u.dq3, u.dq4, u.dq5, u.dq6, u.dq7, u.dVs};
    std::memcpy(ucur_, v, sizeof v);
}

bool OcpSolver::solveOCP(std::vector<OptVariables>& opt_sol, Status* status, ComputeTime* mpc_time) {
    const int N = impl_.horizon();
    std::vector<double> sol((size_t)(N + 1) * 17);
    int32_t st = 0, ok = 0;
    mpcc_timing tm{};
    check(mpcc_solve_ocp(impl_.engine(), 1, guess_.data(), ucur_, obs_, sol.data(), &st, &ok, mpc_time ? &tm : nullptr),
          "mpcc_solve_ocp");
    opt_sol.resize(N + 1);
    for (int k = 0; k <= N; k++) {
        const double* h = &sol[(size_t)17 * k];
        opt_sol[k].xk = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]};
        opt_sol[k].uk = {h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16]};
    }
    if (status) *status = (Status)st;
    if (mpc_time) *mpc_time = {tm.set_env, tm.set_qp, tm.solve_qp, tm.get_alpha, tm.total};
    return ok != 0;
}

// ------------------------------------------------------------------------------------------------
MPC::MPC(int N, double Ts, const PathToJson& path, int device) : MPC(N, Ts, path, ParamValue{}, device) {}

MPC::MPC(int N, double Ts, const PathToJson& path, const ParamValue& param_value, int device)
    : impl_(N, Ts, 1, path, param_value, device) {}

bool MPC::runMPC(MPCReturn& mpc_return, State& x0, Input& u0) {
    return runMPC_(mpc_return, x0, u0, {3.0, 3.0, 3.0}, 0.0);  // mpc.cpp:97-100
}

bool MPC::runMPC_(MPCReturn& mpc_return, State& x0, Input& u0, const std::array<double, 3>& obs_position,
                  const double& obs_radius) {
    const int N = impl_.horizon();
    double x[NX] = {x0.q1, x0.q2, x0.q3, x0.q4, x0.q5, x0.q6, x0.q7, x0.s, x0.vs};
    const double u[NU] = {u0.dq1, u0.dq2, u0.dq3, u0.dq4, u0.dq5, u0.dq6, u0.dq7, u0.dVs};
    const double obs[4] = {obs_position[0], obs_position[1], obs_position[2], obs_radius};
    double uo[NU];
    std::vector<double> hor((size_t)(N + 1) * 17);
    int32_t st = 0, ok = 0;
    impl_.runMPCBatch(1, x, u, obs, uo, hor.data(), &st, &ok, &mpc_return.compute_time);
    x0 = {x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[8]};  // x0 is mutated (mpc.cpp:107-115)
    mpc_return.u0 = {uo[0], uo[1], uo[2], uo[3], uo[4], uo[5], uo[6], uo[7]};
    mpc_return.mpc_horizon.resize(N + 1);
    for (int k = 0; k <= N; k++) {
        const double* h = &hor[(size_t)17 * k];
        mpc_return.mpc_horizon[k].xk = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]};
        mpc_return.mpc_horizon[k].uk = {h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16]};
    }
    last_status_ = (Status)st;
    return ok != 0;
}

void MPC::setTrack(const std::vector<double>& X, const std::vector<double>& Y, const std::vector<double>& Z,
                   const std::vector<Rot>& R) {
    impl_.setTrack(X, Y, Z, R);
}

double MPC::getTrackLength() { return impl_.getTrackLength(); }

void MPC::setParam(const ParamValue& param_value) { impl_.setParam(param_value); }

}  // namespace mpcc_amd
