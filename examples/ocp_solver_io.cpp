// ocp_solver_io.cpp — drives mpcc_amd::OcpSolver (the SolverInterface mirror) the way the reference's
// MPC::runMPC_ drives its solver_interface_ (mpc.cpp:126-136): setCurrentInput, setInitialGuess,
// setEnvData, solveOCP — one instance after another on one solver object.
//
//   examples/ocp_solver_io <data_dir> <mask> <max_iter> <in.bin> <out.bin>
//   in.bin : int32 N, int32 B, path data s[100] X[100] Y[100] Z[100] R[100*9],
//            then per instance guess[(N+1)*17], u_cur[8], obs[4]               (float64)
//   out.bin: per instance int32 status, int32 solved, opt_sol[(N+1)*17]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpcc_mpc.hpp"

using namespace mpcc_amd;

static void rd(std::FILE* f, void* p, size_t n) {
    if (std::fread(p, 1, n, f) != n) throw Error("short read");
}

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s <data_dir> <mask> <max_iter> <in.bin> <out.bin>\n", argv[0]);
        return 2;
    }
    try {
        std::FILE* in = std::fopen(argv[4], "rb");
        if (!in) throw Error("cannot open input");
        int32_t N = 0, B = 0;
        rd(in, &N, 4);
        rd(in, &B, 4);
        std::vector<double> s(100), X(100), Y(100), Z(100), R9(900);
        rd(in, s.data(), 800); rd(in, X.data(), 800); rd(in, Y.data(), 800); rd(in, Z.data(), 800);
        rd(in, R9.data(), 7200);
        std::vector<Rot> R(100);
        for (int i = 0; i < 100; i++)
            for (int a = 0; a < 9; a++) R[i][a] = R9[9 * i + a];

        ParamValue pv;
        pv.sqp["max_iter"] = std::atof(argv[3]);
        OcpSolver solver(N, 0.01, defaultPaths(argv[1]), pv, 0, std::atoi(argv[2]));
        solver.setTrack(s, X, Y, Z, R);

        std::FILE* out = std::fopen(argv[5], "wb");
        if (!out) throw Error("cannot open output");
        std::vector<double> g((size_t)(N + 1) * 17);
        for (int b = 0; b < B; b++) {
            double u[8], obs[4];
            rd(in, g.data(), g.size() * 8);
            rd(in, u, 64);
            rd(in, obs, 32);
            std::vector<OptVariables> guess(N + 1), sol;
            for (int k = 0; k <= N; k++) {
                const double* h = &g[(size_t)17 * k];
                guess[k].xk = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]};
                guess[k].uk = {h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16]};
            }
            solver.setCurrentInput({u[0], u[1], u[2], u[3], u[4], u[5], u[6], u[7]});
            solver.setInitialGuess(guess);
            solver.setEnvData({obs[0], obs[1], obs[2]}, obs[3]);
            Status st;
            ComputeTime tm;
            const int32_t ok = solver.solveOCP(sol, &st, &tm) ? 1 : 0;
            const int32_t st32 = (int32_t)st;
            std::fwrite(&st32, 4, 1, out);
            std::fwrite(&ok, 4, 1, out);
            for (int k = 0; k <= N; k++) {
                const State& x = sol[k].xk;
                const Input& v = sol[k].uk;
                const double h[17] = {x.q1, x.q2, x.q3, x.q4, x.q5, x.q6, x.q7, x.s, x.vs,
                                      v.dq1, v.dq2, v.dq3, v.dq4, v.dq5, v.dq6, v.dq7, v.dVs};
                std::fwrite(h, 8, 17, out);
            }
        }
        std::fclose(out);
        std::fclose(in);
    } catch (const Error& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
