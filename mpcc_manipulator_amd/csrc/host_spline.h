// host_spline.h — host-side construction of the arc-length parameterized 6-D track spline.
// Restates ArcLengthSpline::gen6DSpline / fitSpline (arc_length_spline.cpp:33-265) with the cubic
// spline fit of cubic_spline.cpp:65-124 and the rotation spline of cubic_spline_rot.cpp:137-238.
// Runs once per setTrack; the result is a set of flat tables uploaded to the device.
#pragma once
#include <array>
#include <vector>

namespace mpcc {

struct SplineTables {
    int n = 0;
    double delta = 0;              // x_in(1) - x_in(0) of the final regular fit
    std::vector<double> s;         // [n]  arc length of the path data (getPathData().s)
    std::vector<double> X, Y, Z;   // [n]  path data points (getPathData)
    std::vector<double> a[3], b[3], c[3], d[3];  // spline coefficients per axis ([n] each, b/d padded)
    std::vector<double> R;         // [n*9] rotation data
    std::vector<double> cr, dr;    // [n] rotation spline c, d (padded)
    std::vector<double> logv;      // [n*3] invskew(LogMatrix(R_i^T R_{i+1})) (padded)
    double length() const { return s.back(); }
};

// Build from way-points (MPC::setTrack(X, Y, Z, R)); R9 = n row-major 3x3 matrices.
SplineTables build_track_spline(int n, const double* X, const double* Y, const double* Z, const double* R9);

// Final regular fit only (arc_length_spline.cpp:245-252) from ArcLengthSpline::getPathData():
// n = N_SPLINE points, s strictly increasing.  build_track_spline ends with this call.
SplineTables build_track_from_path(int n, const double* s, const double* X, const double* Y, const double* Z,
                                   const double* R9);

// evaluation of the final tables at arc length s (any output may be null): the device formulas
void eval_tables(const SplineTables& t, double s, double* p, double* dp, double* ddp, double* R9, double* dR);
// ArcLengthSpline::projectOnSpline(s_guess, ee) (arc_length_spline.cpp:318-379), as the device
double project_tables(const SplineTables& t, double proj_max_dist, double s_guess, const double* ee);

// quaternion (x, y, z, w) -> rotation as Eigen Quaterniond::normalized().toRotationMatrix() (track.cpp:45-53)
void quat_to_rot(double qx, double qy, double qz, double qw, double* R9);

// host LogMatrix / ExpMatrix (cubic_spline_rot.cpp:44-95), exposed for tests
void host_log_vec(const double* R, double* v);
void host_exp_matrix(const double* sk, double* E);
void host_cubic_spline(int n, const double* x, const double* y, bool regular, int m, const double* xq, double* out3);
void host_rot_spline(int n, const double* x, const double* R9, bool regular, int m, const double* xq, double* Rq, double* dRq);

}  // namespace mpcc
