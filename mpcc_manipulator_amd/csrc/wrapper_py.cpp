// wrapper_py.cpp — Python module MPCC_WRAPPER with the names of the reference's Boost.Python module
// (cpp/src/MPCC_wrapper.cpp:116-417) over the MI355X engine, so that python/MPCC/MPCC.py and
// python/MPCC/robot_model.py run unchanged against it.  Eigen values are
// numpy arrays.  Differences: the horizon is read from the module attribute N when an MPC is built
// (the reference's is compile-time, config.h:36; default 10 as there); PathToJson carries nn_dir
// (default <data>/nn); engine failures raise RuntimeError.
#include <dlfcn.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl_bind.h>

#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "mpcc_mpc.hpp"

namespace py = pybind11;
using namespace mpcc_amd;
using Map = std::map<std::string, double>;
using Horizon = std::vector<OptVariables>;
PYBIND11_MAKE_OPAQUE(Map);
PYBIND11_MAKE_OPAQUE(Horizon);

namespace {

std::string g_data;  // <package>/data, from this module's location (<package>/_build/MPCC_WRAPPER*.so)

using Arr = py::array_t<double, py::array::c_style | py::array::forcecast>;

Arr vec(const double* p, size_t n) {
    Arr a(n);
    std::copy(p, p + n, a.mutable_data());
    return a;
}
Arr mat3(const double* R) {
    Arr a({3, 3});
    std::copy(R, R + 9, a.mutable_data());
    return a;
}
std::vector<double> values(const py::handle& h, size_t n, const char* what) {
    Arr a = Arr::ensure(h);
    if (!a || (size_t)a.size() != n) throw std::invalid_argument(std::string(what) + ": expected " + std::to_string(n) + " values");
    return std::vector<double>(a.data(), a.data() + n);
}
std::vector<double> values(const py::handle& h, const char* what) {
    Arr a = Arr::ensure(h);
    if (!a) throw std::invalid_argument(std::string(what) + ": expected an array");
    return std::vector<double>(a.data(), a.data() + a.size());
}
std::vector<Rot> rotations(const py::handle& seq) {
    std::vector<Rot> R;
    for (auto item : py::reinterpret_borrow<py::sequence>(seq)) {
        const auto v = values(item, 9, "rotation");
        Rot r;
        std::copy(v.begin(), v.end(), r.begin());
        R.push_back(r);
    }
    return R;
}
void check(int rc, const char* what) {
    if (rc != MPCC_OK) throw std::runtime_error(std::string(what) + ": " + mpcc_last_error());
}

// types.cpp conversions
Arr stateToVector(const State& x) {
    const double v[9] = {x.q1, x.q2, x.q3, x.q4, x.q5, x.q6, x.q7, x.s, x.vs};
    return vec(v, 9);
}
Arr inputToVector(const Input& u) {
    const double v[8] = {u.dq1, u.dq2, u.dq3, u.dq4, u.dq5, u.dq6, u.dq7, u.dVs};
    return vec(v, 8);
}
State vectorToState(const py::handle& h) {
    const auto v = values(h, 9, "vectorToState");
    return {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]};
}
Input vectorToInput(const py::handle& h) {
    const auto v = values(h, 8, "vectorToInput");
    return {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
}

// ArcLengthSpline: the spline of a set of way-points (host tables, mpcc_track_*_host)
struct Spline {
    std::vector<double> X, Y, Z, R9;
    double proj_max_dist = 0.03;
    bool built = false;
    void gen6DSpline(const py::handle& x, const py::handle& y, const py::handle& z, const py::handle& r) {
        X = values(x, "X"); Y = values(y, "Y"); Z = values(z, "Z");
        const auto R = rotations(r);
        if (Y.size() != X.size() || Z.size() != X.size() || R.size() != X.size())
            throw std::invalid_argument("gen6DSpline: size mismatch");
        R9.assign(9 * R.size(), 0.0);
        for (size_t i = 0; i < R.size(); i++) std::copy(R[i].begin(), R[i].end(), R9.begin() + 9 * i);
        built = true;
    }
    void need() const {
        if (!built) throw std::runtime_error("ArcLengthSpline: gen6DSpline first");
    }
    void eval(double s, double* p, double* d1, double* d2, double* R, double* dR) const {
        need();
        check(mpcc_track_eval_host((int)X.size(), X.data(), Y.data(), Z.data(), R9.data(), 1, &s, p, d1, d2, R, dR),
              "ArcLengthSpline");
    }
    py::dict pathData() const {  // PathData (arc_length_spline.h:49-56)
        need();
        std::vector<double> s(NSPLINE), x(NSPLINE), y(NSPLINE), z(NSPLINE), r(9 * NSPLINE);
        double L = 0;
        check(mpcc_track_build_host((int)X.size(), X.data(), Y.data(), Z.data(), R9.data(), s.data(), x.data(),
                                    y.data(), z.data(), r.data(), &L),
              "getPathData");
        py::list R;
        for (int i = 0; i < NSPLINE; i++) R.append(mat3(&r[9 * i]));
        py::dict d;
        d["X"] = vec(x.data(), NSPLINE); d["Y"] = vec(y.data(), NSPLINE); d["Z"] = vec(z.data(), NSPLINE);
        d["R"] = R; d["s"] = vec(s.data(), NSPLINE); d["n_points"] = NSPLINE;
        return d;
    }
    static constexpr int NSPLINE = 100;  // config.h:38
};

struct PathData {
    Arr X, Y, Z, s;
    py::list R;
    int n_points = 0;
};

PathData to_path_data(const Spline& sp) {
    py::dict d = sp.pathData();
    PathData p;
    p.X = d["X"].cast<Arr>(); p.Y = d["Y"].cast<Arr>(); p.Z = d["Z"].cast<Arr>(); p.s = d["s"].cast<Arr>();
    p.R = d["R"].cast<py::list>(); p.n_points = d["n_points"].cast<int>();
    return p;
}

struct TrackPos {
    Arr X, Y, Z;
    py::list R;
};

// Track (track.cpp:19-66)
struct PyTrack {
    std::string file;
    explicit PyTrack(std::string f) : file(std::move(f)) {}
    TrackPos getTrack(const py::handle& init_position) const {
        const auto p = values(init_position, 3, "getTrack");
        const TrackPoints t = loadTrack(file, {p[0], p[1], p[2]});
        TrackPos o;
        o.X = vec(t.X.data(), t.X.size()); o.Y = vec(t.Y.data(), t.Y.size()); o.Z = vec(t.Z.data(), t.Z.size());
        for (const auto& r : t.R) o.R.append(mat3(r.data()));
        return o;
    }
};

PathToJson with_nn(PathToJson p) {
    if (p.nn_dir.empty()) p.nn_dir = g_data + "/nn";
    return p;
}
int module_N() { return py::module_::import("MPCC_WRAPPER").attr("N").cast<int>(); }

// MPC (mpc.h:58-128)
struct PyMPC {
    std::unique_ptr<MPC> mpc;
    Spline track;
    double proj_max_dist = 0.03;
    PyMPC(double Ts, const PathToJson& path) : mpc(new MPC(module_N(), Ts, with_nn(path))) { init(path); }
    PyMPC(double Ts, const PathToJson& path, const ParamValue& pv) : mpc(new MPC(module_N(), Ts, with_nn(path), pv)) {
        init(path);
    }
    void init(const PathToJson& path) {
        mpcc_params p;
        check(mpcc_get_params(mpc->engine(), &p), "MPC");
        proj_max_dist = p.proj_max_dist;
        (void)path;
    }
    bool runMPC(MPCReturn& ret, State& x0, Input& u0) { return mpc->runMPC(ret, x0, u0); }
    bool runMPC_(MPCReturn& ret, State& x0, Input& u0, const py::handle& obs, double r) {
        const auto o = values(obs, 3, "obs_position");
        return mpc->runMPC_(ret, x0, u0, {o[0], o[1], o[2]}, r);
    }
    void setTrack(const py::handle& X, const py::handle& Y, const py::handle& Z, const py::handle& R) {
        track.gen6DSpline(X, Y, Z, R);
        track.proj_max_dist = proj_max_dist;
        mpc->setTrack(track.X, track.Y, track.Z, rotations(R));
    }
    Spline getTrack() const { return track; }
    double getTrackLength() { return mpc->getTrackLength(); }
    void setParam(const ParamValue& pv) {
        mpc->setParam(pv);
        mpcc_params p;
        check(mpcc_get_params(mpc->engine(), &p), "setParam");
        proj_max_dist = track.proj_max_dist = p.proj_max_dist;
    }
};

// RobotModel (robot_model.h:27-141, robot_model.cpp:354-450): frame kinematics on the GPU
// (mpcc_robot_frames).  Like the reference object it keeps the joint vector of the last
// getUpdateKinematics for the frame_id-only getters.
constexpr int EE_FRAME = 9;  // PANDA_NUM_LINKS: panda_hand_tcp
struct PyRobot {
    std::vector<double> q = std::vector<double>(7, 0.0), qdot = std::vector<double>(7, 0.0);
    struct Frame {
        double pos[3], R[9], J[42], mani, dmani[7];
    };
    Frame frame(const std::vector<double>& qv, int f) const {
        Frame o;
        check(mpcc_robot_frames(0, 1, qv.data(), f, o.pos, o.R, o.J, &o.mani, o.dmani), "RobotModel");
        return o;
    }
    Frame at(const py::handle& qh, int f) const { return frame(values(qh, 7, "joint angles"), f); }
    static Arr jac(const Frame& fr, int row0, int rows) {
        Arr a({rows, 7});
        for (int i = 0; i < rows; i++)
            for (int j = 0; j < 7; j++) a.mutable_data()[7 * i + j] = fr.J[7 * (row0 + i) + j];
        return a;
    }
    static Arr trans(const Frame& fr) {  // Affine3d as a 4x4 homogeneous matrix
        Arr a({4, 4});
        double* d = a.mutable_data();
        for (int i = 0; i < 16; i++) d[i] = 0.0;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) d[4 * i + j] = fr.R[3 * i + j];
            d[4 * i + 3] = fr.pos[i];
        }
        d[15] = 1.0;
        return a;
    }
    // getX(q) / getX(frame_id) / getX(q, frame_id) of the reference overload sets
    Frame resolve(const py::object& a, const py::object& b) const {
        if (a.is_none()) return frame(q, EE_FRAME);
        const bool scalar = !py::isinstance<py::array>(a) && !py::isinstance<py::sequence>(a);  // int / numpy int
        if (scalar && b.is_none()) return frame(q, a.cast<int>());
        return at(a, b.is_none() ? EE_FRAME : b.cast<int>());
    }
};

// SelCollNNmodel / EnvCollNNmodel (SelfCollisionModel.cpp / EnvCollisionModel.cpp): setNeuralNetwork loads a
// network of any shape from the model path; calculateMlpOutput -> (output, Jacobian wrt every input)
struct PyNN {
    std::string path;
    std::shared_ptr<mpcc_mlp> net;
    int nin = 0, nout = 0;
    explicit PyNN(std::string p) : path(std::move(p)) {}
    void setNeuralNetwork(int n_input, int n_output, const py::handle& hidden, bool is_nerf) {
        const auto h = values(hidden, "n_hidden");
        std::vector<int32_t> hs(h.size());
        for (size_t i = 0; i < h.size(); i++) hs[i] = (int32_t)h[i];
        mpcc_mlp* m = nullptr;
        check(mpcc_mlp_create(0, path.c_str(), n_input, n_output, hs.data(), (int)hs.size(), is_nerf ? 1 : 0, &m),
              "setNeuralNetwork");
        net.reset(m, mpcc_mlp_destroy);
        nin = n_input;
        nout = n_output;
    }
    py::tuple calculateMlpOutput(const py::handle& input, bool /*time_verbose*/) {
        if (!net) throw std::runtime_error("calculateMlpOutput: setNeuralNetwork first");
        const auto x = values(input, (size_t)nin, "input");
        Arr out(nout), jac({nout, nin});
        check(mpcc_mlp_eval(net.get(), 1, x.data(), out.mutable_data(), jac.mutable_data()), "calculateMlpOutput");
        return py::make_tuple(out, jac);
    }
};
struct PySelfNN : PyNN {
    using PyNN::PyNN;
};
struct PyEnvNN : PyNN {
    using PyNN::PyNN;
};

// Integrator (integrator.cpp:29-68) of the kinematic model (model.cpp:31-45)
struct PyIntegrator {
    double Ts = 0.01;
    static void f(const double* x, const double* u, double* d) {
        for (int i = 0; i < 7; i++) d[i] = u[i];
        d[7] = x[8];
        d[8] = u[7];
    }
    static State rk4(const State& s, const Input& in, double h) {
        const double x[9] = {s.q1, s.q2, s.q3, s.q4, s.q5, s.q6, s.q7, s.s, s.vs};
        const double u[8] = {in.dq1, in.dq2, in.dq3, in.dq4, in.dq5, in.dq6, in.dq7, in.dVs};
        double k1[9], k2[9], k3[9], k4[9], t[9], o[9];
        f(x, u, k1);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h / 2. * k1[i];
        f(t, u, k2);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h / 2. * k2[i];
        f(t, u, k3);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h * k3[i];
        f(t, u, k4);
        for (int i = 0; i < 9; i++) o[i] = x[i] + h * (k1[i] / 6. + k2[i] / 3. + k3[i] / 3. + k4[i] / 6.);
        return {o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]};
    }
    static State ef(const State& s, const Input& in, double h) {
        const double x[9] = {s.q1, s.q2, s.q3, s.q4, s.q5, s.q6, s.q7, s.s, s.vs};
        const double u[8] = {in.dq1, in.dq2, in.dq3, in.dq4, in.dq5, in.dq6, in.dq7, in.dVs};
        double d[9], o[9];
        f(x, u, d);
        for (int i = 0; i < 9; i++) o[i] = x[i] + h * d[i];
        return {o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]};
    }
    static State simTimeStep(const State& s, const Input& u, double ts) {
        State x = s;
        const int steps = (int)(ts / 0.001);
        for (int i = 0; i < steps; i++) x = rk4(x, u, 0.001);
        return x;
    }
};

}  // namespace

PYBIND11_MODULE(MPCC_WRAPPER, m) {
    {
        Dl_info info;
        if (dladdr((void*)&vectorToState, &info) && info.dli_fname) {
            std::string so = info.dli_fname;
            g_data = so.substr(0, so.rfind('/')) + "/../data";
        }
    }
    m.doc() = "MPCC_WRAPPER names (reference cpp/src/MPCC_wrapper.cpp) over the MI355X engine";
    m.attr("PANDA_DOF") = 7;
    m.attr("PANDA_NUM_LINKS") = 9;
    m.attr("NX") = NX;
    m.attr("NU") = NU;
    m.attr("NPC") = 11;
    m.attr("N") = 10;  // config.h:36; set MPCC_WRAPPER.N before building an MPC to change the horizon
    m.attr("INF") = 1e30;
    m.attr("N_SPLINE") = 100;
    m.attr("pkg_path") = g_data + "/";

    py::class_<State>(m, "State")
        .def(py::init<>())
        .def_readwrite("q1", &State::q1).def_readwrite("q2", &State::q2).def_readwrite("q3", &State::q3)
        .def_readwrite("q4", &State::q4).def_readwrite("q5", &State::q5).def_readwrite("q6", &State::q6)
        .def_readwrite("q7", &State::q7).def_readwrite("s", &State::s).def_readwrite("vs", &State::vs)
        .def("setZero", [](State& x) { x = State{}; })
        .def("unwrap", [](State& x, double L) { x.s = std::max(0., std::min(L, x.s)); });  // types.h:57-60
    py::class_<Input>(m, "Input")
        .def(py::init<>())
        .def_readwrite("dq1", &Input::dq1).def_readwrite("dq2", &Input::dq2).def_readwrite("dq3", &Input::dq3)
        .def_readwrite("dq4", &Input::dq4).def_readwrite("dq5", &Input::dq5).def_readwrite("dq6", &Input::dq6)
        .def_readwrite("dq7", &Input::dq7).def_readwrite("dVs", &Input::dVs)
        .def("setZero", [](Input& u) { u = Input{}; });
    py::class_<PathToJson>(m, "PathToJson")
        .def(py::init([]() { PathToJson p; p.nn_dir = g_data + "/nn"; return p; }))
        .def_readwrite("param_path", &PathToJson::param_path).def_readwrite("cost_path", &PathToJson::cost_path)
        .def_readwrite("bounds_path", &PathToJson::bounds_path).def_readwrite("track_path", &PathToJson::track_path)
        .def_readwrite("normalization_path", &PathToJson::normalization_path)
        .def_readwrite("sqp_path", &PathToJson::sqp_path).def_readwrite("nn_dir", &PathToJson::nn_dir);
    py::bind_map<Map>(m, "StringDoubleMap");
    py::class_<ParamValue>(m, "ParamValue")
        .def(py::init<>())
        .def_readwrite("param", &ParamValue::param).def_readwrite("cost", &ParamValue::cost)
        .def_readwrite("bounds", &ParamValue::bounds).def_readwrite("normalization", &ParamValue::normalization)
        .def_readwrite("sqp", &ParamValue::sqp);

    m.def("stateToVector", &stateToVector);
    m.def("inputToVector", &inputToVector);
    m.def("vectorToState", [](const py::handle& h) { return vectorToState(h); });
    m.def("vectorToInput", [](const py::handle& h) { return vectorToInput(h); });
    m.def("arrayToState", [](const py::handle& h) { return vectorToState(h); });
    m.def("arrayToInput", [](const py::handle& h) { return vectorToInput(h); });
    m.def("stateToJointVector", [](const State& x) {
        const double v[7] = {x.q1, x.q2, x.q3, x.q4, x.q5, x.q6, x.q7};
        return vec(v, 7);
    });
    m.def("inputTodJointVector", [](const Input& u) {
        const double v[7] = {u.dq1, u.dq2, u.dq3, u.dq4, u.dq5, u.dq6, u.dq7};
        return vec(v, 7);
    });

    py::class_<ComputeTime>(m, "ComputeTime")
        .def(py::init<>())
        .def_readwrite("set_qp", &ComputeTime::set_qp).def_readwrite("solve_qp", &ComputeTime::solve_qp)
        .def_readwrite("get_alpha", &ComputeTime::get_alpha).def_readwrite("set_env", &ComputeTime::set_env)
        .def_readwrite("total", &ComputeTime::total)
        .def("setZero", [](ComputeTime& t) { t = ComputeTime{}; });
    py::class_<OptVariables>(m, "OptVariables")
        .def(py::init<>())
        .def_readwrite("xk", &OptVariables::xk).def_readwrite("uk", &OptVariables::uk);
    py::bind_vector<Horizon>(m, "OptVariablesVector");
    py::class_<MPCReturn>(m, "MPCReturn")
        .def(py::init<>())
        .def_readwrite("u0", &MPCReturn::u0).def_readwrite("mpc_horizon", &MPCReturn::mpc_horizon)
        .def_readwrite("compute_time", &MPCReturn::compute_time)
        .def("setZero", [](MPCReturn& r) { r = MPCReturn{}; });

    py::class_<TrackPos>(m, "TrackPos")
        .def_readonly("X", &TrackPos::X).def_readonly("Y", &TrackPos::Y).def_readonly("Z", &TrackPos::Z)
        .def_readonly("R", &TrackPos::R);
    py::class_<PyTrack>(m, "Track").def(py::init<std::string>()).def("getTrack", &PyTrack::getTrack);
    py::class_<PathData>(m, "PathData")
        .def_readonly("X", &PathData::X).def_readonly("Y", &PathData::Y).def_readonly("Z", &PathData::Z)
        .def_readonly("R", &PathData::R).def_readonly("s", &PathData::s).def_readonly("n_points", &PathData::n_points);
    py::class_<Spline>(m, "ArcLengthSpline")
        .def(py::init<>())
        .def("gen6DSpline", &Spline::gen6DSpline)
        .def("getPathData", [](const Spline& sp) { return to_path_data(sp); })
        .def("getLength", [](const Spline& sp) { double s[1]; auto d = sp.pathData(); Arr a = d["s"].cast<Arr>(); s[0] = a.data()[a.size() - 1]; return s[0]; })
        .def("getPosition", [](const Spline& sp, double s) { double p[3]; sp.eval(s, p, nullptr, nullptr, nullptr, nullptr); return vec(p, 3); })
        .def("getDerivative", [](const Spline& sp, double s) { double p[3]; sp.eval(s, nullptr, p, nullptr, nullptr, nullptr); return vec(p, 3); })
        .def("getSecondDerivative", [](const Spline& sp, double s) { double p[3]; sp.eval(s, nullptr, nullptr, p, nullptr, nullptr); return vec(p, 3); })
        .def("getOrientation", [](const Spline& sp, double s) { double R[9]; sp.eval(s, nullptr, nullptr, nullptr, R, nullptr); return mat3(R); })
        .def("getOrientationDerivative", [](const Spline& sp, double s) { double d[3]; sp.eval(s, nullptr, nullptr, nullptr, nullptr, d); return vec(d, 3); })
        .def("projectOnSpline", [](const Spline& sp, double s, const py::handle& ee) {
            sp.need();
            const auto e = values(ee, 3, "ee_pos");
            double out = 0;
            check(mpcc_track_project_host((int)sp.X.size(), sp.X.data(), sp.Y.data(), sp.Z.data(), sp.R9.data(), 1,
                                          sp.proj_max_dist, &s, e.data(), &out),
                  "projectOnSpline");
            return out;
        });

    py::class_<PyMPC>(m, "MPC")
        .def(py::init<double, const PathToJson&>())
        .def(py::init<double, const PathToJson&, const ParamValue&>())
        .def("runMPC", &PyMPC::runMPC)
        .def("runMPC_", &PyMPC::runMPC_)
        .def("setTrack", &PyMPC::setTrack)
        .def("getTrack", &PyMPC::getTrack)
        .def("getTrackLength", &PyMPC::getTrackLength)
        .def("setParam", &PyMPC::setParam);

    using PR = PyRobot;
    const auto none = py::none();
    py::class_<PyRobot>(m, "RobotModel")
        .def(py::init<>())
        .def("getNumq", [](PR&) { return 7; })
        .def("getNumv", [](PR&) { return 7; })
        .def("getNumu", [](PR&) { return 7; })
        .def("getUpdateKinematics", [](PR& r, const py::handle& q, const py::handle& qd) {
            r.q = values(q, 7, "q");
            r.qdot = values(qd, 7, "qdot");
        })
        .def("getJointPosition", [](PR& r) { return vec(r.q.data(), 7); })
        .def("getJacobian", [](PR& r, py::object a, py::object b) { return PR::jac(r.resolve(a, b), 0, 6); },
             py::arg("q_or_frame"), py::arg("frame_id") = none)
        .def("getJacobianv", [](PR& r, py::object a, py::object b) { return PR::jac(r.resolve(a, b), 0, 3); },
             py::arg("q"), py::arg("frame_id") = none)
        .def("getJacobianw", [](PR& r, py::object a, py::object b) { return PR::jac(r.resolve(a, b), 3, 3); },
             py::arg("q"), py::arg("frame_id") = none)
        .def("getPosition", [](PR& r, int f) { return vec(r.frame(r.q, f).pos, 3); })
        .def("getEEPosition", [](PR& r, py::object q) { return vec(r.resolve(q, py::none()).pos, 3); },
             py::arg("q") = none)
        .def("getOrientation", [](PR& r, int f) { return mat3(r.frame(r.q, f).R); })
        .def("getEEOrientation", [](PR& r, py::object q) { return mat3(r.resolve(q, py::none()).R); },
             py::arg("q") = none)
        .def("getTransformation", [](PR& r, int f) { return PR::trans(r.frame(r.q, f)); })
        .def("getEETransformation", [](PR& r, py::object q) { return PR::trans(r.resolve(q, py::none())); },
             py::arg("q") = none)
        .def("getManipulability", [](PR& r, const py::handle& q, int f) { return r.at(q, f).mani; },
             py::arg("q"), py::arg("frame_id") = EE_FRAME)
        .def("getDManipulability", [](PR& r, const py::handle& q, int f) { return vec(r.at(q, f).dmani, 7); },
             py::arg("q"), py::arg("frame_id") = EE_FRAME);

    py::class_<PySelfNN>(m, "SelCollNNmodel")
        .def(py::init([]() { return PySelfNN(g_data + "/nn/self"); }))
        .def(py::init<std::string>())
        .def("setNeuralNetwork", &PyNN::setNeuralNetwork)
        .def("calculateMlpOutput", &PyNN::calculateMlpOutput, py::arg("input"), py::arg("time_verbose") = false);
    py::class_<PyEnvNN>(m, "EnvCollNNmodel")
        .def(py::init([]() { return PyEnvNN(g_data + "/nn/env"); }))
        .def(py::init<std::string>())
        .def("setNeuralNetwork", &PyNN::setNeuralNetwork)
        .def("calculateMlpOutput", &PyNN::calculateMlpOutput, py::arg("input"), py::arg("time_verbose") = false);

    // cubic_spline_rot.h utilities (cubic_spline_rot.cpp:25-95)
    m.def("getSkewMatrix", [](const py::handle& v) {
        const auto a = values(v, 3, "getSkewMatrix");
        const double S[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
        return mat3(S);
    });
    m.def("getInverseSkewVector", [](const py::handle& R) {
        const auto a = values(R, 9, "getInverseSkewVector");
        const double v[3] = {a[7], a[2], a[3]};
        return vec(v, 3);
    });
    m.def("LogMatrix", [](const py::handle& R) {
        const auto a = values(R, 9, "LogMatrix");
        double S[9];
        check(mpcc_so3_log(a.data(), S), "LogMatrix");
        return mat3(S);
    });
    m.def("ExpMatrix", [](const py::handle& S) {
        const auto a = values(S, 9, "ExpMatrix");
        double R[9];
        check(mpcc_so3_exp(a.data(), R), "ExpMatrix");
        return mat3(R);
    });

    // StateInputIndex (config.h:40-76)
    struct SII {};
    auto sii = py::class_<SII>(m, "StateInputIndex").def(py::init<>());
    const char* qn[] = {"q1", "q2", "q3", "q4", "q5", "q6", "q7", "s", "vs"};
    for (int i = 0; i < 9; i++) sii.def_property_readonly(qn[i], [i](const SII&) { return i; });
    const char* un[] = {"dq1", "dq2", "dq3", "dq4", "dq5", "dq6", "dq7", "dVs"};
    for (int i = 0; i < 8; i++) sii.def_property_readonly(un[i], [i](const SII&) { return i; });
    sii.def_property_readonly("con_selcol", [](const SII&) { return 0; });
    sii.def_property_readonly("con_sing", [](const SII&) { return 1; });
    for (int i = 1; i <= 9; i++)
        sii.def_property_readonly(("con_envcol" + std::to_string(i)).c_str(), [i](const SII&) { return i + 1; });
    m.attr("si_index") = SII{};

    py::class_<PyIntegrator>(m, "Integrator")
        .def(py::init<>())
        .def(py::init([](double Ts, const PathToJson&) { PyIntegrator i; i.Ts = Ts; return i; }))
        .def("RK4", [](const PyIntegrator&, const State& x, const Input& u, double ts) { return PyIntegrator::rk4(x, u, ts); })
        .def("EF", [](const PyIntegrator&, const State& x, const Input& u, double ts) { return PyIntegrator::ef(x, u, ts); })
        .def("simTimeStep", [](const PyIntegrator&, const State& x, const Input& u, double ts) {
            return PyIntegrator::simTimeStep(x, u, ts);
        });
}
