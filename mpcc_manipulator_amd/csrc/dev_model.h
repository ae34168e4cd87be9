// dev_model.h — device kinematics, rotation algebra and spline evaluation.
//
// Panda chain: the RBDL model of robot_model.cpp:68-319 evaluated as a product of
// [E_i^T, r_i] fixed transforms and Rz(q_i) joint rotations (RBDL SpatialTransform(E, r): E maps
// parent to child coordinates, so the child frame's rotation is E^T).  Jacobian columns are the
// geometric ones RBDL's CalcPointJacobian6D returns, reordered [Jv; Jw] (robot_model.cpp:372-375).
#pragma once
#include "dev_common.h"

namespace mpcc {

// E^T of the fixed joint frames 1..7 (robot_model.cpp:189-235) and link7->hand (:238-242, Q19:
// literal 0.707107).  Stored as the rotation R = E^T row-major.
__device__ __forceinline__ void joint_fixed_rot(int i, double* R) {
    // i = 1..8
    switch (i) {
        case 1: R[0]=1;R[1]=0;R[2]=0; R[3]=0;R[4]=1;R[5]=0; R[6]=0;R[7]=0;R[8]=1; break;
        case 2: case 5: R[0]=1;R[1]=0;R[2]=0; R[3]=0;R[4]=0;R[5]=1; R[6]=0;R[7]=-1;R[8]=0; break;
        case 3: case 4: case 6: case 7: R[0]=1;R[1]=0;R[2]=0; R[3]=0;R[4]=0;R[5]=-1; R[6]=0;R[7]=1;R[8]=0; break;
        default: R[0]=0.707107;R[1]=0.707107;R[2]=0; R[3]=-0.707107;R[4]=0.707107;R[5]=0; R[6]=0;R[7]=0;R[8]=1; break;
    }
}
__device__ __forceinline__ void joint_offset(int i, double* r) {  // robot_model.cpp:171-182
    r[0] = 0; r[1] = 0; r[2] = 0;
    switch (i) {
        case 1: r[2] = 0.333; break;
        case 3: r[1] = -0.316; break;
        case 4: r[0] = 0.0825; break;
        case 5: r[0] = -0.0825; r[1] = 0.384; break;
        case 7: r[0] = 0.088; break;
        case 8: r[2] = 0.107; break;
        default: break;
    }
}

// FK of panda_hand_tcp: position, rotation (row-major) and 6x7 Jacobian (rows 0-2 Jv, 3-5 Jw).
// want_J = false skips the Jacobian.
__device__ inline void panda_fk(const double* q, double* pos, double* Rout, double* J, bool want_J) {
    double Rc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double pc[3] = {0, 0, 0};
    double z[7][3], o[7][3];
#pragma unroll
    for (int i = 1; i <= 7; i++) {
        double r[3], E[9], Rt[9];
        joint_offset(i, r);
        pc[0] += Rc[0] * r[0] + Rc[1] * r[1] + Rc[2] * r[2];
        pc[1] += Rc[3] * r[0] + Rc[4] * r[1] + Rc[5] * r[2];
        pc[2] += Rc[6] * r[0] + Rc[7] * r[1] + Rc[8] * r[2];
        joint_fixed_rot(i, E);
        m3mul(Rc, E, Rt);
        z[i - 1][0] = Rt[2]; z[i - 1][1] = Rt[5]; z[i - 1][2] = Rt[8];
        o[i - 1][0] = pc[0]; o[i - 1][1] = pc[1]; o[i - 1][2] = pc[2];
        double s, c;
        sincos(q[i - 1], &s, &c);
        // Rc = Rt * Rz(q)
#pragma unroll
        for (int a = 0; a < 3; a++) {
            double r0 = Rt[3 * a], r1 = Rt[3 * a + 1];
            Rc[3 * a] = r0 * c + r1 * s;
            Rc[3 * a + 1] = -r0 * s + r1 * c;
            Rc[3 * a + 2] = Rt[3 * a + 2];
        }
    }
    {
        double r[3], E[9], Rt[9];
        joint_offset(8, r);
        pc[0] += Rc[0] * r[0] + Rc[1] * r[1] + Rc[2] * r[2];
        pc[1] += Rc[3] * r[0] + Rc[4] * r[1] + Rc[5] * r[2];
        pc[2] += Rc[6] * r[0] + Rc[7] * r[1] + Rc[8] * r[2];
        joint_fixed_rot(8, E);
        m3mul(Rc, E, Rt);
#pragma unroll
        for (int a = 0; a < 9; a++) Rc[a] = Rt[a];
        const double tz = 0.1034;  // hand -> hand_tcp (:182)
        pc[0] += Rc[2] * tz; pc[1] += Rc[5] * tz; pc[2] += Rc[8] * tz;
    }
    if (pos) { pos[0] = pc[0]; pos[1] = pc[1]; pos[2] = pc[2]; }
    if (Rout)
#pragma unroll
        for (int a = 0; a < 9; a++) Rout[a] = Rc[a];
    if (want_J) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            double r0 = pc[0] - o[i][0], r1 = pc[1] - o[i][1], r2 = pc[2] - o[i][2];
            J[0 * 7 + i] = z[i][1] * r2 - z[i][2] * r1;
            J[1 * 7 + i] = z[i][2] * r0 - z[i][0] * r2;
            J[2 * 7 + i] = z[i][0] * r1 - z[i][1] * r0;
            J[3 * 7 + i] = z[i][0];
            J[4 * 7 + i] = z[i][1];
            J[5 * 7 + i] = z[i][2];
        }
    }
}

// Frame of RobotModel::getPosition/getOrientation/getJacobian(frame_id) (robot_model.cpp:354-398,
// body_id_ at :310-319): 1 = panda_link0 (the base), 2..8 = panda_link1..7 (origin after joint f-1),
// 9 = panda_hand_tcp (= panda_fk).  J is the 6x7 point Jacobian at the frame origin, zero columns for
// the joints after the frame.  Any output may be null.
__device__ inline void panda_frame(const double* q, int frame, double* pos, double* Rout, double* J) {
    if (frame >= 9) {
        double Jt[42];
        panda_fk(q, pos, Rout, Jt, J != nullptr);
        if (J)
            for (int a = 0; a < 42; a++) J[a] = Jt[a];
        return;
    }
    double Rc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double pc[3] = {0, 0, 0};
    double z[7][3], o[7][3];
    const int nj = frame - 1;  // joints that move the frame
    for (int i = 1; i <= nj; i++) {
        double r[3], E[9], Rt[9];
        joint_offset(i, r);
        pc[0] += Rc[0] * r[0] + Rc[1] * r[1] + Rc[2] * r[2];
        pc[1] += Rc[3] * r[0] + Rc[4] * r[1] + Rc[5] * r[2];
        pc[2] += Rc[6] * r[0] + Rc[7] * r[1] + Rc[8] * r[2];
        joint_fixed_rot(i, E);
        m3mul(Rc, E, Rt);
        z[i - 1][0] = Rt[2]; z[i - 1][1] = Rt[5]; z[i - 1][2] = Rt[8];
        o[i - 1][0] = pc[0]; o[i - 1][1] = pc[1]; o[i - 1][2] = pc[2];
        double s, c;
        sincos(q[i - 1], &s, &c);
        for (int a = 0; a < 3; a++) {
            const double r0 = Rt[3 * a], r1 = Rt[3 * a + 1];
            Rc[3 * a] = r0 * c + r1 * s;
            Rc[3 * a + 1] = -r0 * s + r1 * c;
            Rc[3 * a + 2] = Rt[3 * a + 2];
        }
    }
    if (pos) { pos[0] = pc[0]; pos[1] = pc[1]; pos[2] = pc[2]; }
    if (Rout)
        for (int a = 0; a < 9; a++) Rout[a] = Rc[a];
    if (J)
        for (int i = 0; i < 7; i++) {
            if (i < nj) {
                const double r0 = pc[0] - o[i][0], r1 = pc[1] - o[i][1], r2 = pc[2] - o[i][2];
                J[0 * 7 + i] = z[i][1] * r2 - z[i][2] * r1;
                J[1 * 7 + i] = z[i][2] * r0 - z[i][0] * r2;
                J[2 * 7 + i] = z[i][0] * r1 - z[i][1] * r0;
                J[3 * 7 + i] = z[i][0];
                J[4 * 7 + i] = z[i][1];
                J[5 * 7 + i] = z[i][2];
            } else {
                for (int a = 0; a < 6; a++) J[a * 7 + i] = 0.0;
            }
        }
}

// Husky+Panda (MPCC_DOF = 10): planar base joints x, y (prismatic) and theta (revolute
// about z) of RobotModel::setHusky (robot_model.cpp:321-352) carry panda_link0 at MOBILE_MOUNT in the base
// frame (identity rotation).  p = [x, y, 0] + Rz(th) (mount + p_arm), R = Rz(th) R_arm; Jacobian columns
// e_x, e_y, (e_z x (p - [x, y, 0]); e_z) for the base and Rz(th)-rotated arm columns (the oracle's fk).
constexpr double MOBILE_MOUNT_Z = MPCC_MOBILE_MOUNT_Z;  // include/mpcc_engine.h
// FK of panda_hand_tcp for this build's robot: position, rotation (row-major) and the 6 x DOF Jacobian.
__device__ inline void robot_fk(const double* q, double* pos, double* Rout, double* J, bool want_J) {
    if constexpr (NBASE == 0) {
        panda_fk(q, pos, Rout, J, want_J);
    } else {
        double pa[3], Ra[9], Ja[42];
        panda_fk(q + NBASE, pa, Ra, Ja, want_J);
        double sn, cs;
        sincos(q[2], &sn, &cs);
        const double pl[3] = {0.0 + pa[0], 0.0 + pa[1], MOBILE_MOUNT_Z + pa[2]};
        const double pw[3] = {cs * pl[0] + -sn * pl[1] + 0 * pl[2], sn * pl[0] + cs * pl[1] + 0 * pl[2],
                              0 * pl[0] + 0 * pl[1] + 1 * pl[2]};
        const double p3[3] = {q[0] + pw[0], q[1] + pw[1], 0.0 + pw[2]};
        if (pos) { pos[0] = p3[0]; pos[1] = p3[1]; pos[2] = p3[2]; }
        if (Rout) {
            const double Rz[9] = {cs, -sn, 0, sn, cs, 0, 0, 0, 1};
            m3mul(Rz, Ra, Rout);
        }
        if (want_J) {
#pragma unroll
            for (int i = 0; i < 6 * DOF; i++) J[i] = 0.0;
            J[0 * DOF + 0] = 1.0;
            J[1 * DOF + 1] = 1.0;
            J[0 * DOF + 2] = -(p3[1] - q[1]);
            J[1 * DOF + 2] = p3[0] - q[0];
            J[5 * DOF + 2] = 1.0;
#pragma unroll
            for (int j = 0; j < NARM; j++) {
                const double v0 = Ja[0 * 7 + j], v1 = Ja[1 * 7 + j], v2 = Ja[2 * 7 + j];
                const double w0 = Ja[3 * 7 + j], w1 = Ja[4 * 7 + j], w2 = Ja[5 * 7 + j];
                J[0 * DOF + NBASE + j] = cs * v0 + -sn * v1 + 0 * v2;
                J[1 * DOF + NBASE + j] = sn * v0 + cs * v1 + 0 * v2;
                J[2 * DOF + NBASE + j] = 0 * v0 + 0 * v1 + 1 * v2;
                J[3 * DOF + NBASE + j] = cs * w0 + -sn * w1 + 0 * w2;
                J[4 * DOF + NBASE + j] = sn * w0 + cs * w1 + 0 * w2;
                J[5 * DOF + NBASE + j] = 0 * w0 + 0 * w1 + 1 * w2;
            }
        }
    }
}

// sqrt(det(J J^T)) with a partial-pivot LU of the 6x6 Gram matrix (robot_model.cpp:431-435;
// Eigen's MatrixXd::determinant for n > 4 is PartialPivLU).
// NC = Jacobian columns (the robot's DOF; 7 for a Panda frame query)
template <int NC = DOF>
__device__ inline double manip_from_J(const double* J) {
    double A[36];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < NC; k++) s += J[NC * i + k] * J[NC * j + k];
            A[6 * i + j] = s;
        }
    double det = 1.0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        int p = k;
        double mx = fabs(A[6 * k + k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++) {
            double v = fabs(A[6 * i + k]);
            if (v > mx) { mx = v; p = i; }
        }
        if (p != k) {
#pragma unroll
            for (int j = 0; j < 6; j++) {
                // select-based swap keeps A in registers (no dynamic indexing)
                double a0 = A[6 * k + j];
                double ap = 0;
#pragma unroll
                for (int i = k + 1; i < 6; i++) ap = (i == p) ? A[6 * i + j] : ap;
                A[6 * k + j] = ap;
#pragma unroll
                for (int i = k + 1; i < 6; i++) A[6 * i + j] = (i == p) ? a0 : A[6 * i + j];
            }
            det = -det;
        }
        double piv = A[6 * k + k];
        det *= piv;
        if (piv != 0.0) {
            double inv = 1.0 / piv;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double f = A[6 * i + k] / piv;
#pragma unroll
                for (int j = k + 1; j < 6; j++) A[6 * i + j] -= f * A[6 * k + j];
            }
            (void)inv;
        }
    }
    return sqrt(det);
}

__device__ inline double manipulability(const double* q) {
    double J[6 * DOF];
    robot_fk(q, nullptr, nullptr, J, true);
    return manip_from_J(J);
}

// ---- SO(3) log/exp (cubic_spline_rot.cpp:44-95) ----
// Symmetric 3x3 eigen-solve on the lower triangle (Eigen SelfAdjointEigenSolver reads it),
// cyclic Jacobi; only used by LogMatrix's theta = pi branch.
__device__ inline void sym_eig3(const double* Rin, double* w, double* V) {
    double A[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) A[3 * i + j] = (i >= j) ? Rin[3 * i + j] : Rin[3 * j + i];
#pragma unroll
    for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        double off = fabs(A[1]) + fabs(A[2]) + fabs(A[5]);
        if (off < 1e-300) break;
        for (int pq = 0; pq < 3; pq++) {
            int p = (pq == 2) ? 1 : 0, q = (pq == 0) ? 1 : 2;
            double apq = A[3 * p + q];
            if (fabs(apq) < 1e-300) continue;
            double theta = (A[3 * q + q] - A[3 * p + p]) / (2 * apq);
            double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
            double c = 1 / sqrt(t * t + 1), s = t * c;
            for (int k = 0; k < 3; k++) {
                double akp = A[3 * k + p], akq = A[3 * k + q];
                A[3 * k + p] = c * akp - s * akq;
                A[3 * k + q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; k++) {
                double apk = A[3 * p + k], aqk = A[3 * q + k];
                A[3 * p + k] = c * apk - s * aqk;
                A[3 * q + k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; k++) {
                double vkp = V[3 * k + p], vkq = V[3 * k + q];
                V[3 * k + p] = c * vkp - s * vkq;
                V[3 * k + q] = s * vkp + c * vkq;
            }
        }
    }
    // ascending order
    int i0 = 0, i1 = 1, i2 = 2;
    double e0 = A[0], e1 = A[4], e2 = A[8];
    if (e0 > e1) { double t = e0; e0 = e1; e1 = t; int ti = i0; i0 = i1; i1 = ti; }
    if (e1 > e2) { double t = e1; e1 = e2; e2 = t; int ti = i1; i1 = i2; i2 = ti; }
    if (e0 > e1) { double t = e0; e0 = e1; e1 = t; int ti = i0; i0 = i1; i1 = ti; }
    w[0] = e0; w[1] = e1; w[2] = e2;
    double Vs[9];
    for (int r = 0; r < 3; r++) { Vs[3 * r] = V[3 * r + i0]; Vs[3 * r + 1] = V[3 * r + i1]; Vs[3 * r + 2] = V[3 * r + i2]; }
    for (int i = 0; i < 9; i++) V[i] = Vs[i];
}

// invskew(LogMatrix(R)) (cubic_spline_rot.cpp:44-79, quirk Q10)
__device__ inline void log_vec(const double* R, double* v) {
    double tr = R[0] + R[4] + R[8];
    v[0] = v[1] = v[2] = 0.0;
    if (fabs(tr + 1.0) < 1e-6) {
        double w[3], V[9];
        sym_eig3(R, w, V);
        for (int i = 0; i < 3; i++) {
            if (fabs(w[i] - 1.0) < 1e-4) {
                double e0 = V[i], e1 = V[3 + i], e2 = V[6 + i];
                double n = sqrt(e0 * e0 + e1 * e1 + e2 * e2);
                // result = -skew(u) * pi  ->  invskew = -u * pi
                v[0] = -(e0 / n) * M_PI; v[1] = -(e1 / n) * M_PI; v[2] = -(e2 / n) * M_PI;
            }
        }
    } else if (fabs(tr - 3.0) < 1e-6) {
        // zero
    } else {
        double th = acos((tr - 1.0) / 2.0);
        double f = 1.0 / 2.0 * th / sin(th);
        v[0] = f * (R[7] - R[5]);
        v[1] = f * (R[2] - R[6]);
        v[2] = f * (R[3] - R[1]);
    }
}

// ExpMatrix(skew(v)) (cubic_spline_rot.cpp:81-95; Q11: integer 1/2 == 0 in the small-angle branch)
__device__ inline void exp_skew(const double* v, double* E) {
    double sk[9], sk2[9];
    skew3(v, sk);
    m3mul(sk, sk, sk2);
    double vn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (vn <= 1e-8) {
        double c = cos(vn);
#pragma unroll
        for (int i = 0; i < 9; i++) E[i] = ((i % 4 == 0) ? 1.0 : 0.0) + c * sk[i];
        return;
    }
    double a = sin(vn) / vn, b = (1 - cos(vn)) / (vn * vn);
#pragma unroll
    for (int i = 0; i < 9; i++) E[i] = ((i % 4 == 0) ? 1.0 : 0.0) + a * sk[i] + b * sk2[i];
}

// ---- regular cubic spline evaluation (cubic_spline.cpp:126-246, cubic_spline_rot.cpp:216-259) ----
// unwrapInput (cubic_spline.cpp, arc_length_spline.cpp): std::max(0., std::min(x, L)) — comparison
// semantics, so a NaN (0/0 Newton step at the track end, arc_length_spline.cpp:356-372) maps to 0,
// where IEEE fmin/fmax would return L and end the projection there.
__device__ __forceinline__ double spl_unwrap(const SplineView& sp, double x) {
    const double m = (sp.L < x) ? sp.L : x;
    return (0. < m) ? m : 0.;
}
__device__ __forceinline__ int spl_index(const SplineView& sp, double x) {
    if (x == sp.L) return NSPL - 1;
    return MPCC_BCHK(sp.err, (int)floor(x / sp.delta), NSPL, BC_SPLINE);
}
// position, first and second derivative of the x/y/z splines at arc length t
__device__ inline void spline_pos3(const SplineView& sp, double t, double* p, double* dp, double* ddp) {
    double x = spl_unwrap(sp, t);
    int i = spl_index(sp, x);
    const int n = NSPL;
    double xi = sp.s(i);
    double d1 = x - xi, d2 = d1 * d1, d3 = d1 * d2;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        if (i == n - 1) {
            if (p) p[a] = sp.a(a, n - 1);
            if (dp) dp[a] = 0.;
            if (ddp) ddp[a] = 2.0 * sp.c(a, n - 1);
        } else {
            double A = sp.a(a, i), B = sp.b(a, i), C = sp.c(a, i), D = sp.d(a, i);
            if (p) p[a] = A + B * d1 + C * d2 + D * d3;
            if (dp) dp[a] = B + 2.0 * C * d1 + 3.0 * D * d2;
            if (ddp) ddp[a] = 2.0 * C + 6.0 * D * d1;
        }
    }
}
__device__ inline void spline_rot(const SplineView& sp, double t, double* R, double* dR) {
    double x = spl_unwrap(sp, t);
    int i = spl_index(sp, x);
    if (i == NSPL - 1) {
        if (R)
            for (int a = 0; a < 9; a++) R[a] = sp.R(NSPL - 1)[a];
        if (dR) dR[0] = dR[1] = dR[2] = 0;
        return;
    }
    double d1 = x - sp.s(i), d2 = d1 * d1, d3 = d1 * d2;
    const double* lvp = sp.logv(i);
    double lv[3] = {lvp[0], lvp[1], lvp[2]};
    double cr = sp.cr(i), dr = sp.dr(i);
    if (R) {
        double f = cr * d2 + dr * d3;
        double v[3] = {lv[0] * f, lv[1] * f, lv[2] * f}, E[9];
        exp_skew(v, E);
        m3mul(sp.R(i), E, R);
    }
    if (dR) {
        double f = 2.0 * cr * d1 + 3.0 * dr * d2;
        dR[0] = lv[0] * f; dR[1] = lv[1] * f; dR[2] = lv[2] * f;
    }
}

// projectOnSpline (arc_length_spline.cpp:318-379).  Far branch (quirk Q12) restated with Eigen's
// scalar minCoeff semantics: NaN-masked valid entries never compare smaller, so index 0 wins.
__device__ inline double project_on_spline(const SplineView& sp, double proj_max_dist, double s_guess, const double* ee) {
    double pp[3];
    spline_pos3(sp, s_guess, pp, nullptr, nullptr);
    double s_opt = s_guess;
    double dx = ee[0] - pp[0], dy = ee[1] - pp[1], dz = ee[2] - pp[2];
    double dist = sqrt(dx * dx + dy * dy + dz * dz);
    if (dist >= proj_max_dist) {
        const int n = NSPL;
        bool any = false;
        double best = 0;
        int bi = 0;
        for (int i = 0; i < n; i++) {
            bool valid = fabs(sp.s(i) - s_guess) <= proj_max_dist;
            any |= valid;
            double ex = sp.a(0, i) - ee[0], ey = sp.a(1, i) - ee[1], ez = sp.a(2, i) - ee[2];
            double d2 = ex * ex + ey * ey + ez * ez;
            if (i == 0 || d2 < best) { best = d2; bi = i; }
        }
        s_opt = any ? sp.s(0) : sp.s(bi);
    }
    if (s_opt >= sp.L) return sp.L;
    double s_old = s_opt;
    for (int it = 0; it < 20; it++) {
        double p[3], dp[3], ddp[3];
        spline_pos3(sp, s_opt, p, dp, ddp);
        double d0 = p[0] - ee[0], d1 = p[1] - ee[1], d2 = p[2] - ee[2];
        double jac = 2.0 * d0 * dp[0] + 2.0 * d1 * dp[1] + 2.0 * d2 * dp[2];
        double hes = 2.0 * dp[0] * dp[0] + 2.0 * d0 * ddp[0] + 2.0 * dp[1] * dp[1] + 2.0 * d1 * ddp[1] +
                     2.0 * dp[2] * dp[2] + 2.0 * d2 * ddp[2];
        s_opt -= jac / hes;
        s_opt = spl_unwrap(sp, s_opt);
        if (fabs(s_old - s_opt) <= 1e-5) return s_opt;
        s_old = s_opt;
    }
    return s_guess;
}

// Integrator::RK4 (integrator.cpp:29-43) of the kinematic model (model.cpp:31-45): q' = dq, s' = vs, vs' = dVs
__device__ inline void rk4_step(const double* x, const double* u, double ts, double* out) {
    double k1[NX], k2[NX], k3[NX], k4[NX], t[NX];
#pragma unroll
    for (int j = 0; j < DOF; j++) { k1[j] = u[j]; k2[j] = u[j]; k3[j] = u[j]; k4[j] = u[j]; }
    k1[XS] = x[XVS]; k1[XVS] = u[UVS];
#pragma unroll
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts / 2. * k1[i];
    k2[XS] = t[XVS]; k2[XVS] = u[UVS];
#pragma unroll
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts / 2. * k2[i];
    k3[XS] = t[XVS]; k3[XVS] = u[UVS];
#pragma unroll
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts * k3[i];
    k4[XS] = t[XVS]; k4[XVS] = u[UVS];
#pragma unroll
    for (int i = 0; i < NX; i++) out[i] = x[i] + ts * (k1[i] / 6. + k2[i] / 3. + k3[i] / 3. + k4[i] / 6.);
}

}  // namespace mpcc
