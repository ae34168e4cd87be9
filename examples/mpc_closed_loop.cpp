// mpc_closed_loop.cpp — the reference's closed-loop driver (cpp/src/main.cpp:55-114) on the C++ host
// surface (include/mpcc_mpc.hpp): start at the reference joint configuration, offset the track to
// the end-effector, then runMPC_ -> simTimeStep for a fixed number of control steps.
//
//   examples/mpc_closed_loop <data_dir> <steps> [ox oy oz r]   -> CSV: step, x[9], u0[8], status, ok
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "mpcc_mpc.hpp"

using namespace mpcc_amd;

// model.cpp:31-45: q' = dq, s' = vs, vs' = dVs
static void f(const double* x, const double* u, double* d) {
    for (int i = 0; i < 7; i++) d[i] = u[i];
    d[7] = x[8];
    d[8] = u[7];
}

// Integrator::RK4 / simTimeStep (integrator.cpp:29-68): ts / 1 ms sub-steps
static void sim_time_step(double* x, const double* u, double ts) {
    const int steps = (int)(ts / 0.001);
    const double h = 0.001;
    for (int s = 0; s < steps; s++) {
        double k1[9], k2[9], k3[9], k4[9], t[9];
        f(x, u, k1);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h / 2. * k1[i];
        f(t, u, k2);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h / 2. * k2[i];
        f(t, u, k3);
        for (int i = 0; i < 9; i++) t[i] = x[i] + h * k3[i];
        f(t, u, k4);
        for (int i = 0; i < 9; i++) x[i] = x[i] + h * (k1[i] / 6. + k2[i] / 3. + k3[i] / 3. + k4[i] / 6.);
    }
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <data_dir> <steps> [ox oy oz r]\n", argv[0]);
        return 2;
    }
    const std::string data = argv[1];
    const int steps = std::atoi(argv[2]);
    std::array<double, 3> obs_p{3.0, 3.0, 3.0};
    double obs_r = 0.0;
    if (argc >= 7) {
        obs_p = {std::atof(argv[3]), std::atof(argv[4]), std::atof(argv[5])};
        obs_r = std::atof(argv[6]);
    }
    try {
        const double Ts = 0.01;  // Params/config.json
        const PathToJson path = defaultPaths(data);
        MPC mpc(20, Ts, path);

        const std::array<double, 7> q0{0, 0, 0, -M_PI / 2, 0, M_PI / 2, M_PI / 4};  // main.cpp:60-61
        const TrackPoints tr = loadTrack(path.track_path, mpc.eePosition(q0));
        mpc.setTrack(tr.X, tr.Y, tr.Z, tr.R);
        std::fprintf(stderr, "track length %.9f\n", mpc.getTrackLength());

        double x[9] = {q0[0], q0[1], q0[2], q0[3], q0[4], q0[5], q0[6], 0.0, 0.0};
        Input u0;
        MPCReturn ret;
        for (int k = 0; k < steps; k++) {
            State xs{x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], x[8]};
            std::printf("%d", k);
            for (double v : x) std::printf(",%.17g", v);
            const bool ok = mpc.runMPC_(ret, xs, u0, obs_p, obs_r);
            x[7] = xs.s;  // runMPC_ updates s and vs of its state argument; the reference integrates that
            x[8] = xs.vs; // state (main.cpp:103-105)
            u0 = ret.u0;
            const double u[8] = {u0.dq1, u0.dq2, u0.dq3, u0.dq4, u0.dq5, u0.dq6, u0.dq7, u0.dVs};
            for (double v : u) std::printf(",%.17g", v);
            std::printf(",%d,%d\n", (int)mpc.lastStatus(), ok ? 1 : 0);
            sim_time_step(x, u, Ts);
            if (!ok) break;  // main.cpp:108-112
        }
    } catch (const Error& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
