// dev_records.h — RobotData::update of one (instance, stage) record by a group of RPT lanes (robot_data.h:55-71):
// FK, Jacobian, manipulability and its central-difference gradient.  Shared by k_records (kernels.hip) and the solo
// blocks' own records (ipm.hip k_sqp_solo, early solo blocks); included under fp-contract off in both, so the two
// are bitwise the same.
#pragma once
#include "dev_model.h"
#include "kernels.h"

namespace mpcc {

// RobotData::update (robot_data.h:55-71) of joint vector q into the SoA record at rec (stride S); the
// self-collision MLP (if masked: infinite distance) and the env MLP outputs are written by k_mlp_*.
// The central-difference term of joint i: (mu(q + delta e_i) - mu(q - delta e_i)) / (2 delta)
__device__ inline double manip_fd(const double* q, int i) {
    const double delta = 1e-4;  // robot_model.cpp:439
    double qp[DOF], qm[DOF];
#pragma unroll
    for (int j = 0; j < DOF; j++) { qp[j] = q[j] + (j == i ? delta : 0.0); qm[j] = q[j] - (j == i ? delta : 0.0); }
    const double m1 = manipulability(qp), m2 = manipulability(qm);
    return (m1 - m2) / (2 * delta);
}
// The fields of the record that do not depend on q: the collision columns of a network the constraint mask leaves
// out (infinite distance, zero gradient; k_mlp_* writes the others) and the obstacle radius.  Constant field f
// (0 <= f < rec_const_count) of lane group member u: f = u, u + nl, ... (nl lanes share the stores)
__device__ inline int rec_const_count(const DevConst& c) {
    const bool sel = c.p.constraint_mask & MPCC_CON_SELFCOL, env = c.p.constraint_mask & MPCC_CON_ENVCOL;
    return (sel ? NBASE : 1 + DOF) + (env ? 0 : 9 + 9 * DOF);
}
__device__ inline void rec_const_store(const DevConst& c, int f, double* rec, size_t S) {
    const double inf = __longlong_as_double(0x7ff0000000000000LL);
    const bool sel = c.p.constraint_mask & MPCC_CON_SELFCOL;
    const int ns = sel ? NBASE : 1 + DOF;  // self-collision fields: R_SEL (unless masked in), then R_DSEL columns
    if (f < ns) {
        if (sel) rec[(R_DSEL + f) * S] = 0.0;  // the base moves no Panda link relative to another
        else if (f == 0) rec[R_SEL * S] = inf;
        else rec[(R_DSEL + f - 1) * S] = 0.0;
        return;
    }
    f -= ns;
    if (f < 9) rec[(R_ENV + f) * S] = inf;
    else rec[(R_DENV + f - 9) * S] = 0.0;
}
// position, rotation and Jacobian of one record (RobotData::update)
__device__ inline void robot_record_q(const DevConst& c, const double (&pos)[3], const double (&R)[9],
                                     const double (&J)[6 * DOF], double* rec, size_t S) {
#pragma unroll
    for (int a = 0; a < 3; a++) rec[(R_POS + a) * S] = pos[a];
#pragma unroll
    for (int a = 0; a < 9; a++) rec[(R_ROT + a) * S] = R[a];
#pragma unroll
    for (int a = 0; a < 6 * DOF; a++) rec[(R_J + a) * S] = J[a];
}
// the whole record from one thread (k_debug_records; fd = false: without the gradient block R_DMU)
__device__ inline void robot_record(const DevConst& c, const double* q, double obs_r, double* rec, size_t S, bool fd = true) {
    double pos[3], R[9], J[6 * DOF];
    robot_fk(q, pos, R, J, true);
    robot_record_q(c, pos, R, J, rec, S);
    rec[R_MU * S] = manip_from_J(J);
    if (fd)
        for (int i = 0; i < DOF; i++) rec[(R_DMU + i) * S] = manip_fd(q, i);
    for (int f = 0; f < rec_const_count(c); f++) rec_const_store(c, f, rec, S);
    rec[R_OBSR * S] = obs_r;
}

// RPT threads per (instance, stage) record.  Every thread of the group runs ONE FK + Jacobian + manipulability
// evaluation in lockstep (the Panda: thread 0 and 15 at q, thread 1 + i at q + delta e_i, thread 1 + DOF + i at
// q - delta e_i; the mobile build: thread 1 + i at q + delta e_i, then at q - delta e_i, thread 0 at q), then
// thread 0 stores the q-dependent record, thread 1 + i the central difference of joint i (robot_model.cpp:436-447),
// and all of them the constant fields.  The record's own evaluation used to run on thread 0 beside the others'
// (a divergent branch: the wave issued both), and thread 0 alone stored the constant fields.  Same arithmetic
// per value (fp-contract off): bitwise the previous records.
constexpr bool FD_SPLIT = 2 * DOF + 1 <= 16;
constexpr int RPT = FD_SPLIT ? 16 : ((DOF + 1 <= 8) ? 8 : 16);
static_assert(DOF + 1 <= RPT, "one thread per gradient term");
// record t (instance t / (N+1), stage t mod (N+1)) by lane u of its RPT-lane group; every lane of the group calls it
// (the gradient terms are exchanged by a 16-lane shuffle), live = false evaluates without storing
__device__ inline void record_group(const DevConst& c, const DevBuffers& d, int t, int u, bool live) {
    const int S = c.S;
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    const double* g = d.guess + ((size_t)b * (N + 1) + k) * NXU;
    double q[DOF];
#pragma unroll
    for (int j = 0; j < DOF; j++) q[j] = g[j];
    const double delta = 1e-4;  // robot_model.cpp:439 (manip_fd)
    double* rec = d.rec + t;
    double pos[3], R[9], J[6 * DOF];
    if constexpr (FD_SPLIT) {
        const bool plus = u >= 1 && u <= DOF, minus = u > DOF && u <= 2 * DOF;
        const int i = plus ? u - 1 : u - 1 - DOF;
        double qq[DOF];
#pragma unroll
        for (int j = 0; j < DOF; j++)
            qq[j] = plus ? q[j] + (j == i ? delta : 0.0) : (minus ? q[j] - (j == i ? delta : 0.0) : q[j]);
        robot_fk(qq, pos, R, J, true);
        if (live && u == 0) robot_record_q(c, pos, R, J, rec, (size_t)S);  // before the Gram matrix: J dies in it
        const double mu = manip_from_J(J);
        const double mm = __shfl_down(mu, DOF, 16);  // lane 1 + i <- mu(q - delta e_i)
        if (!live) return;
        if (u == 0) rec[(size_t)R_MU * S] = mu;
        else if (u <= DOF) rec[(size_t)(R_DMU + u - 1) * S] = (mu - mm) / (2 * delta);
    } else {
        const bool fd = u >= 1 && u <= DOF;
        const int i = u - 1;
        double qq[DOF];
#pragma unroll
        for (int j = 0; j < DOF; j++) qq[j] = fd ? q[j] + (j == i ? delta : 0.0) : q[j];
        robot_fk(qq, pos, R, J, true);
        if (live && u == 0) robot_record_q(c, pos, R, J, rec, (size_t)S);
        const double m1 = manip_from_J(J);
        double m2 = 0.0;
        if (fd) {
#pragma unroll
            for (int j = 0; j < DOF; j++) qq[j] = q[j] - (j == i ? delta : 0.0);
            m2 = manipulability(qq);
        }
        if (!live) return;
        if (u == 0) rec[(size_t)R_MU * S] = m1;
        else if (fd) rec[(size_t)(R_DMU + i) * S] = (m1 - m2) / (2 * delta);
    }
    const int nc = rec_const_count(c);
    for (int f = u; f < nc; f += RPT) rec_const_store(c, f, rec, (size_t)S);
    if (u == RPT - 1) rec[(size_t)R_OBSR * S] = d.obs[4 * b + 3];
}

}  // namespace mpcc
