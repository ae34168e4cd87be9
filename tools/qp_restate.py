"""Independent restatement of the reference's SQP subproblem: QP assembly and an exact dense solve (numpy).

Written from the reference sources, not from oracle/ or the product (mpcc_manipulator_amd/), so that the
oracle's dense reference layout and the engine's QP step are checked against a second, separately derived
implementation of the hot path's assembly (VERDICT r02 "What's missing" 1):
  * OsqpInterface::setCost / setDynamics / setBounds / setPolytopicConstraints / setConstraints
    (cpp/src/Interfaces/osqp_interface.cpp:129-389) and the QP of solveOCP
    (:445, :479: min 1/2 s'Ps + q's, l - c <= A s <= u - c, OSQP's infinity 1e30);
  * Cost::getCost and its helpers (cpp/src/Cost/cost.cpp:36-357), quirks Q2 (ddz_ref = ddpos(1)),
    Q3 (|e_lag| I in d_lag_error), Q13 (unclamped weight blend), Q14 (end-deceleration target constant);
  * Constraints::getConstraints (cpp/src/Constraints/constraints.cpp:34-243), Q16 (zero terminal rows);
  * Bounds::getBoundsLX/UX/LU/UU/LddJoint/UddJoint (cpp/src/Constraints/bounds.cpp:85-128), Q1 (input
    rows on the state columns NU*i), Q15 (the 8th ddq row of a stage is a zero row);
  * Model::getLinModel (cpp/src/Model/model.cpp:47-124): the ZOH by a matrix exponential (scipy's expm,
    Pade as Eigen's MatrixFunctions);
  * the parameter files' keys (cpp/src/Params/params.cpp:24-448; cpp/Params/*.json).
Track evaluation uses tools/spline_restate.py, the independent restatement of the reference's splines.

Beyond the reference: the constraint mask of BASELINE configs[1] (rows of disabled constraint kinds become
l = -INF, u = +INF with zero Jacobian rows at k != N) and the robot-record layout of
the fixture (REC_* below: the stage data of RobotData, robot_data.h:13-31, one row per stage).

The dense solve replaces OSQP (which stops near 1e-4 and on a wall-clock limit, SURVEY finding 4) by an exact
solution: a Mehrotra predictor-corrector interior point on the dense KKT system (no stage structure), then an
active-set polish (the equality-constrained QP of the identified active set) checked against the KKT
conditions.  Test infrastructure (tools/make_qp_fixture.py, tests/test_qp_restate.py); never product code.
"""
import math
import os
import sys

import numpy as np
import scipy.linalg

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import spline_restate as sr  # noqa: E402

NX, NU, NPC, DOF, NLINK = 9, 8, 11, 7, 9  # config.h:29-34
IS, IVS, IDVS = 7, 8, 7                   # StateInputIndex s, vs, dVs (config.h:41-75)
INF = 1e30                                # config.h:37 (= OSQP_INFTY)
BIG = 1e20                                # |bound| >= BIG: infinite for the dense solve
# robot record of one stage (RobotData, robot_data.h:13-31): pos 3 | R 9 (row-major) | J 6x7 (rows Jv; Jw) |
# manipul | d_manipul 7 | sel_min_dist | d_sel 7 | obs_radius | env_min_dist 9 | d_env 9x7 (row-major)
REC_POS, REC_ROT, REC_J = 0, 3, 12
REC_MU = REC_J + 42
REC_DMU = REC_MU + 1
REC_SEL = REC_DMU + 7
REC_DSEL = REC_SEL + 1
REC_OBSR = REC_DSEL + 7
REC_ENV = REC_OBSR + 1
REC_DENV = REC_ENV + 9
REC = REC_DENV + 63
MASK_SELF, MASK_SING, MASK_ENV = 1, 2, 4


# ------------------------------------------------------------------------------------------------ params
def load_params(params_dir, Ts=None):
    """Param / CostParam / BoundsParam / NormalizationParam / SQPParam file constructors (params.cpp:24-448)
    from the reference's JSON files (cpp/Params)."""
    import json

    def rd(name):
        with open(os.path.join(params_dir, name)) as f:
            return json.load(f)
    m, c, b, n = rd("model.json"), rd("cost.json"), rd("bounds.json"), rd("normalization.json")
    cfg = rd("config.json")
    qn = [f"q{i}" for i in range(1, 8)]
    dn = [f"dq{i}" for i in range(1, 8)]
    return dict(
        Ts=float(cfg["Ts"] if Ts is None else Ts),
        # Param (model.json), params.cpp:24-51
        max_dist_proj=m["max_dist_proj"], desired_ee_velocity=m["desired_ee_velocity"],
        deacc_ratio=m["deaccelerate_ratio"], s_trust_region=m["s_trust_region"],
        tol_sing=m["tol_sing"], tol_selcol=m["tol_selcol"], tol_envcol=m["tol_envcol"],
        # CostParam (cost.json), params.cpp:88-126
        q_c=c["qC"], q_c_N_mult=c["qCNmult"], q_l=c["qL"], q_vs=c["qVs"], q_ori=c["qOri"], q_sing=c["qSing"],
        r_dq=c["rdq"], r_ddq=c["rddq"], r_dVs=c["rdVs"], q_c_red_ratio=c["qC_reduction_ratio"],
        q_l_inc_ratio=c["qL_increase_ratio"], q_ori_red_ratio=c["qOri_reduction_ratio"],
        # BoundsParam (bounds.json), params.cpp:177-241
        lx=np.array([b[k + "l"] for k in qn] + [b["sl"], b["vsl"]], float),
        ux=np.array([b[k + "u"] for k in qn] + [b["su"], b["vsu"]], float),
        lu=np.array([b[k + "l"] for k in dn] + [b["dVsl"]], float),
        uu=np.array([b[k + "u"] for k in dn] + [b["dVsu"]], float),
        lddq=np.array([b[f"ddq{i}l"] for i in range(1, 8)], float),
        uddq=np.array([b[f"ddq{i}u"] for i in range(1, 8)], float),
        # NormalizationParam (normalization.json), params.cpp:312-356
        Tx=np.array([n[k] for k in qn] + [n["s"], n["vs"]], float),
        Tu=np.array([n[k] for k in dn] + [n["dVs"]], float),
    )


PARAM_SCALARS = ["Ts", "max_dist_proj", "desired_ee_velocity", "deacc_ratio", "s_trust_region", "tol_sing",
                 "tol_selcol", "tol_envcol", "q_c", "q_c_N_mult", "q_l", "q_vs", "q_ori", "q_sing", "r_dq", "r_ddq",
                 "r_dVs", "q_c_red_ratio", "q_l_inc_ratio", "q_ori_red_ratio"]
PARAM_VECTORS = ["lx", "ux", "lu", "uu", "lddq", "uddq", "Tx", "Tu"]


def quat_to_rot(qx, qy, qz, qw):
    """Eigen Quaterniond::normalized().toRotationMatrix() (track.cpp:44-52)."""
    nrm = math.sqrt(qx * qx + qy * qy + qz * qz + qw * qw)
    x, y, z, w = qx / nrm, qy / nrm, qz / nrm, qw / nrm
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz, txx, txy, txz = tx * w, ty * w, tz * w, tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return [[1 - (tyy + tzz), txy - twz, txz + twy], [txy + twz, 1 - (txx + tzz), tyz - twx],
            [txz - twy, tyz + twx, 1 - (txx + tyy)]]


def load_track(track_json, ee_start):
    """Track(json).getTrack(ee_pos) (track.cpp:19-66): waypoints offset to the end-effector start."""
    import json
    with open(track_json) as f:
        t = json.load(f)
    X = [x - t["X"][0] + ee_start[0] for x in t["X"]]
    Y = [y - t["Y"][0] + ee_start[1] for y in t["Y"]]
    Z = [z - t["Z"][0] + ee_start[2] for z in t["Z"]]
    R = [quat_to_rot(*q) for q in zip(t["quat_X"], t["quat_Y"], t["quat_Z"], t["quat_W"])]
    return X, Y, Z, R


class Track:
    """ArcLengthSpline of the waypoints (gen6DSpline) and its getters (arc_length_spline.cpp:267-316)."""

    def __init__(self, X, Y, Z, R):
        R = [[list(map(float, r[3 * i:3 * i + 3])) for i in range(3)] if len(np.shape(r)) == 1 else
             [list(map(float, row)) for row in r] for r in R]
        path, self.fin = sr.gen6d(list(map(float, X)), list(map(float, Y)), list(map(float, Z)), R)
        self.path = path  # the final regular path data (s, X, Y, Z, R): projectOnSpline's far branch reads it
        self.length = path[0][-1]

    def ref(self, s):
        pos, d1, d2, Rr, dR = sr.evaluate(self.fin, s)
        return np.array(pos), np.array(d1), np.array(d2), np.array(Rr), np.array(dR)


# ------------------------------------------------------------------------------------------------ model
def lin_model(Ts):
    """getModelJacobian + discretizeModel (model.cpp:47-91): expm of Ts [A B g; 0] (NX+NU+1)^2."""
    A = np.zeros((NX, NX)); A[IS, IVS] = 1.0
    B = np.zeros((NX, NU)); B[:DOF, :DOF] = np.eye(DOF); B[IVS, IDVS] = 1.0
    g = np.zeros(NX)
    T = np.zeros((NX + NU + 1, NX + NU + 1))
    T[:NX, :NX] = A; T[:NX, NX:NX + NU] = B; T[:NX, NX + NU] = g
    E = scipy.linalg.expm(T * Ts)
    return E[:NX, :NX], E[:NX, NX:NX + NU], E[:NX, NX + NU]


# ------------------------------------------------------------------------------------------------ cost
def skew(v):
    """getSkewMatrix (cubic_spline_rot.cpp:25-35)."""
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def blend(x, x0, xf, y0, yf):
    """CubicSpline weight blend (cost.cpp:36-43), not clamped (Q13)."""
    t = (x - x0) / (xf - x0)
    return y0 + (yf - y0) * (3 * t ** 2 - 2 * t ** 3)


def stage_cost(P, track, x, u, rec, k, N):
    """Cost::getCost (cost.cpp:290-357) with grad and Hessian: (obj, f_x, f_u, f_xx, f_uu, f_xu)."""
    pos = rec[REC_POS:REC_POS + 3]
    Rcur = rec[REC_ROT:REC_ROT + 9].reshape(3, 3)
    J = rec[REC_J:REC_J + 42].reshape(6, 7)
    Jv, Jw = J[:3], J[3:]
    mu, dmu = rec[REC_MU], rec[REC_DMU:REC_DMU + 7]
    sel = rec[REC_SEL]
    # weight schedule :293-308
    ratio = min(sel / (P["tol_selcol"] * 2.0), mu / (P["tol_sing"] * 2.0))
    if ratio <= 1.0:
        qc = P["q_c"] * blend(ratio, 0.5, 1.0, P["q_c_red_ratio"], 1.0)
        ql = P["q_l"] * blend(ratio, 0.5, 1.0, P["q_l_inc_ratio"], 1.0)
        qo = P["q_ori"] * blend(ratio, 0.5, 1.0, P["q_ori_red_ratio"], 1.0)
    else:
        qc, ql, qo = P["q_c"], P["q_l"], P["q_ori"]
    s, vs = x[IS], x[IVS]
    pr, T, dd, Rref, dRref = track.ref(s)
    Nrm = np.array([dd[0], dd[1], dd[1]])  # getRefPoint :62-65 (Q2: ddz_ref = ddpos(1))
    # getErrorInfo :82-117
    e = pos - pr
    e_lag = T.dot(e) * T
    e_con = e - e_lag
    d_e = np.zeros((3, NX)); d_e[:, :DOF] = Jv; d_e[:, IS] = -T
    d_T = np.zeros((3, NX)); d_T[:, IS] = Nrm
    d_lag = np.outer(T, T) @ d_e + (np.outer(T, e) + np.linalg.norm(e_lag) * np.eye(3)) @ d_T  # Q3
    d_con = d_e - d_lag
    # getContouringCost :119-162
    CC0 = qc if k < N else P["q_c_N_mult"] * qc
    CC1 = ql
    s_max = track.length
    des = (P["desired_ee_velocity"] if s < s_max * P["deacc_ratio"]
           else -P["desired_ee_velocity"] / (s_max * P["deacc_ratio"]) * (s - s_max))  # Q14
    obj_c = CC0 * e_con.dot(e_con) + CC1 * e_lag.dot(e_lag) + P["q_vs"] * (vs - des) ** 2
    gx_c = 2.0 * CC0 * d_con.T @ e_con + 2.0 * CC1 * d_lag.T @ e_lag
    gx_c[IVS] += 2.0 * P["q_vs"] * (vs - des)
    hxx_c = 2.0 * CC0 * d_con.T @ d_con + 2.0 * CC1 * d_lag.T @ d_lag
    hxx_c[IVS, IVS] += 2.0 * P["q_vs"]
    # getHeadingCost :164-207
    Rbar = Rref.T @ Rcur
    L = np.array(sr.log_matrix(Rbar.tolist()))
    w = np.array([L[2, 1], L[0, 2], L[1, 0]])  # getInverseSkewVector (cubic_spline_rot.cpp:37-42)
    obj_h = qo * w.dot(w)
    wn = np.linalg.norm(w)
    if wn < 1e-8:
        Jri = np.eye(3)
    else:
        S = skew(w)
        Jri = np.eye(3) + 0.5 * S + (1.0 / w.dot(w) + (1.0 + math.cos(wn)) / (2.0 * wn * math.sin(wn))) * S @ S
    dL = np.zeros((3, NX))
    dL[:, :DOF] = Jri @ Rcur.T @ Jw
    dL[:, IS] = -Jri @ Rcur.T @ dRref
    gx_h = 2.0 * qo * dL.T @ w
    hxx_h = 2.0 * qo * dL.T @ dL
    # getInputCost :209-270
    obj_i = 0.0
    gu_i = np.zeros(NU); huu_i = np.zeros((NU, NU))
    if k != N:
        dq = u[:DOF]
        obj_i = P["r_dq"] * dq.dot(dq) + P["r_dVs"] * u[IDVS] ** 2
        gu_i[:DOF] = 2.0 * P["r_dq"] * dq
        gu_i[IDVS] = 2.0 * P["r_dVs"] * u[IDVS]
        huu_i[:DOF, :DOF] = 2.0 * P["r_dq"] * np.eye(DOF)
        huu_i[IDVS, IDVS] = 2.0 * P["r_dVs"]
    # getSingularityCost :272-288
    obj_s = -P["q_sing"] * mu
    gx_s = np.zeros(NX); gx_s[:DOF] = -P["q_sing"] * dmu
    obj = obj_c + obj_h + obj_i + obj_s
    fx = gx_c + gx_h + gx_s
    fu = gu_i
    fxx = hxx_c + hxx_h + 1e-6 * np.eye(NX)  # :353
    fuu = huu_i + 1e-6 * np.eye(NU)          # :354
    return obj, fx, fu, fxx, fuu, np.zeros((NX, NU))


# ------------------------------------------------------------------------------------------------ constraints
def rbf(delta, h):
    """getRBF (constraints.cpp:34-43)."""
    if h >= delta:
        return -math.log(h + 1)
    return -math.log(delta + 1) - 1 / (delta + 1) * (h - delta) + 1 / (2 * (delta + 1) ** 2) * (h - delta) ** 2


def drbf(delta, h):
    """getDRBF (constraints.cpp:52-61)."""
    if h >= delta:
        return -1 / (h + 1)
    return -1 / (delta + 1) + 1 / ((delta + 1) ** 2) * (h - delta)


def stage_constraints(P, x, u, rec, k, N, mask):
    """Constraints::getConstraints (constraints.cpp:192-243): c, l, u (NPC) and c_x (NPC x NX), c_u (NPC x NU)."""
    c, lo, hi = np.zeros(NPC), np.zeros(NPC), np.zeros(NPC)
    cx, cu = np.zeros((NPC, NX)), np.zeros((NPC, NU))
    if k == N:  # every row setZero (Q16)
        return c, lo, hi, cx, cu
    dq = u[:DOF]
    delta = -0.5

    def row(r, h, grad):
        c[r] = -grad.dot(dq) + rbf(delta, h)
        lo[r], hi[r] = -INF, 0.0
        cx[r, :DOF] = drbf(delta, h) * grad
        cu[r, :DOF] = -grad

    def masked(r):
        c[r], lo[r], hi[r] = 0.0, -INF, INF

    if mask & MASK_SELF:  # getSelcollConstraint :70-108 (cm -> m)
        row(0, 0.01 * rec[REC_SEL] - P["tol_selcol"] * 0.01, 0.01 * rec[REC_DSEL:REC_DSEL + 7])
    else:
        masked(0)
    if mask & MASK_SING:  # getSingularConstraint :110-147
        row(1, rec[REC_MU] - P["tol_sing"], rec[REC_DMU:REC_DMU + 7])
    else:
        masked(1)
    for m in range(NLINK):  # getEnvcollConstraint :149-190
        if mask & MASK_ENV:
            dmin = 0.01 * (rec[REC_ENV + m] - rec[REC_OBSR] * 1.2)
            row(2 + m, dmin - 0.01 * P["tol_envcol"], 0.01 * rec[REC_DENV + 7 * m:REC_DENV + 7 * m + 7])
        else:
            masked(2 + m)
    return c, lo, hi, cx, cu


# ------------------------------------------------------------------------------------------------ assembly
def sizes(N):
    """osqp_interface.h:113-117: N_var, N_eq, N_ineqb, N_ineqp, N_constr."""
    nv = NX * (N + 1) + NU * N
    neq, nib, nip = NX * (N + 1), NX * (N + 1) + 2 * NU * N, NPC * (N + 1)
    return nv, neq, nib, nip, neq + nib + nip


def assemble(P, track, guess, recs, ucur, N, mask):
    """setQP = setCost + setConstraints (osqp_interface.cpp:129-396) at the linearization point `guess`
    ((N+1) x [x(9) | u(8)], u_N unused), frozen stage records `recs` ((N+1) x REC) and the current input.
    Returns dict(obj, P, q, A, c, l, u) in the reference's dense layout."""
    nv, neq, nib, nip, nc = sizes(N)
    Tx, Tu = np.diag(P["Tx"]), np.diag(P["Tu"])
    Txi = np.diag(1.0 / P["Tx"])
    Tu7 = np.diag(P["Tu"][:DOF])
    Ts = P["Ts"]
    xs = [guess[i, :NX] for i in range(N + 1)]
    us = [guess[i, NX:] for i in range(N + 1)]
    uo = lambda i: NX * (N + 1) + NU * i  # noqa: E731  (first input column of stage i)
    # ---- setCost :129-219
    obj = 0.0
    q = np.zeros(nv)
    H = np.zeros((nv, nv))
    rddq = P["r_ddq"]  # OsqpInterface::cost_param_ (Q8: always from the file)
    for i in range(N + 1):
        ok, fx, fu, fxx, fuu, fxu = stage_cost(P, track, xs[i], us[i], recs[i], i, N)
        obj += ok
        q[NX * i:NX * i + NX] = Tx @ fx
        H[NX * i:NX * i + NX, NX * i:NX * i + NX] = Tx @ fxx @ Tx
        if i != N:
            q[uo(i):uo(i) + NU] = Tu @ fu
            H[uo(i):uo(i) + NU, uo(i):uo(i) + NU] = Tu @ fuu @ Tu
            H[NX * i:NX * i + NX, uo(i):uo(i) + NU] = Tx @ fxu @ Tu
            H[uo(i):uo(i) + NU, NX * i:NX * i + NX] = (Tx @ fxu @ Tu).T
            dqi = us[i][:DOF]
            if i != N - 1:
                d = us[i + 1][:DOF] - dqi
                obj += rddq * d.dot(d)
            if i == 0:
                g = 2.0 * rddq * (dqi - us[i + 1][:DOF])
                hii, hij = 2.0 * rddq * np.eye(DOF), -2.0 * rddq * np.eye(DOF)
            elif i == N - 1:
                g = 2.0 * rddq * (dqi - us[i - 1][:DOF])
                hii, hij = 2.0 * rddq * np.eye(DOF), None
            else:
                g = 2.0 * rddq * (2.0 * dqi - us[i + 1][:DOF] - us[i - 1][:DOF])
                hii, hij = 4.0 * rddq * np.eye(DOF), -2.0 * rddq * np.eye(DOF)
            q[uo(i):uo(i) + DOF] += Tu7 @ g
            H[uo(i):uo(i) + DOF, uo(i):uo(i) + DOF] += Tu7 @ hii @ Tu7
            if i != N - 1:
                H[uo(i):uo(i) + DOF, uo(i + 1):uo(i + 1) + DOF] += Tu7 @ hij @ Tu7
                H[uo(i + 1):uo(i + 1) + DOF, uo(i):uo(i) + DOF] += Tu7 @ hij @ Tu7
    A = np.zeros((nc, nv))
    c, lo, hi = np.zeros(nc), np.zeros(nc), np.zeros(nc)
    # ---- setDynamics :221-252 (rows [0, neq))
    Ad, Bd, gd = lin_model(Ts)
    for i in range(N + 1):
        r = NX * i
        if i == 0:
            A[0:NX, 0:NX] = np.eye(NX)
            continue
        A[r:r + NX, NX * (i - 1):NX * i] = -Txi @ Ad @ Tx
        A[r:r + NX, NX * i:NX * i + NX] = np.eye(NX)
        A[r:r + NX, uo(i - 1):uo(i - 1) + NU] = -Txi @ Bd @ Tu
        c[r:r + NX] = Txi @ (xs[i] - (Ad @ xs[i - 1] + Bd @ us[i - 1] + gd))
    # ---- setBounds :254-300 (rows [neq, neq + nib))
    b0 = neq
    L = track.length
    for i in range(N + 1):
        r = b0 + NX * i
        A[r:r + NX, NX * i:NX * i + NX] = np.eye(NX) * Tx
        c[r:r + NX] = xs[i]
        lx, ux = P["lx"].copy(), P["ux"].copy()
        lx[IS] = max(xs[i][IS] - P["s_trust_region"], 0.0)  # getBoundsLX :85-91
        ux[IS] = min(xs[i][IS] + P["s_trust_region"], L)    # getBoundsUX :97-103
        lo[r:r + NX], hi[r:r + NX] = lx, ux
        if i == N:
            continue
        r = b0 + NX * (N + 1) + NU * i  # input bounds on the state columns NU*i (Q1, :273)
        A[r:r + NU, NU * i:NU * i + NU] = np.eye(NU) * Tu
        c[r:r + NU] = us[i]
        lo[r:r + NU], hi[r:r + NU] = P["lu"], P["uu"]
        r = b0 + NX * (N + 1) + NU * N + NU * i  # ddq rows (7 of NU; the 8th stays zero, Q15)
        A[r:r + DOF, uo(i):uo(i) + DOF] = 1.0 / Ts * np.eye(DOF) * Tu7
        if i == 0:
            c[r:r + DOF] = 1.0 / Ts * us[0][:DOF]
            lo[r:r + DOF] = P["lddq"] + 1.0 / Ts * ucur[:DOF]
            hi[r:r + DOF] = P["uddq"] + 1.0 / Ts * ucur[:DOF]
        else:
            A[r:r + DOF, uo(i - 1):uo(i - 1) + DOF] = -1.0 / Ts * np.eye(DOF) * Tu7
            c[r:r + DOF] = 1.0 / Ts * (us[i][:DOF] - us[i - 1][:DOF])
            lo[r:r + DOF], hi[r:r + DOF] = P["lddq"], P["uddq"]
    # ---- setPolytopicConstraints :302-344 (rows [neq + nib, nc))
    p0 = neq + nib
    for i in range(N + 1):
        cc, cl, ch, cx, cu = stage_constraints(P, xs[i], us[i], recs[i], i, N, mask)
        r = p0 + NPC * i
        A[r:r + NPC, NX * i:NX * i + NX] = cx @ Tx
        if i != N:
            A[r:r + NPC, uo(i):uo(i) + NU] = cu @ Tu
        c[r:r + NPC], lo[r:r + NPC], hi[r:r + NPC] = cc, cl, ch
    return dict(obj=obj, P=H, q=q, A=A, c=c, l=lo, u=hi)


# ------------------------------------------------------------------------------------------------ dense solve
def solve_dense(H, q, A, lo, hi, tol=1e-13, max_it=100):
    """min 1/2 s'Hs + q's  s.t.  lo <= A s <= hi (|bound| >= BIG infinite, lo = hi an equality): Mehrotra
    predictor-corrector on the dense KKT system, then an active-set polish.  Returns (s, info)."""
    n = H.shape[0]
    zero = ~np.any(A != 0.0, axis=1)
    if np.any(zero & ((lo > 1e-12) | (hi < -1e-12))):
        raise ValueError("infeasible constant row")
    keep = ~zero
    eq = keep & (lo == hi) & (np.abs(lo) < BIG)
    up = keep & ~eq & (hi < BIG)
    dn = keep & ~eq & (lo > -BIG)
    E, e = A[eq], lo[eq]
    G = np.vstack([A[up], -A[dn]])
    h = np.concatenate([hi[up], -lo[dn]])
    m, me = G.shape[0], E.shape[0]

    def kkt_solve(D, r1, r2):
        K = np.zeros((n + me, n + me))
        K[:n, :n] = H + G.T @ (D[:, None] * G)
        K[:n, n:] = E.T
        K[n:, :n] = E
        sol = np.linalg.solve(K, np.concatenate([r1, r2]))
        return sol[:n], sol[n:]

    # start: the equality-constrained minimizer, slacks and multipliers pushed inside
    s, y = kkt_solve(np.zeros(m), -q, e)
    w = np.maximum(h - G @ s, 1.0)
    z = np.ones(m)
    it = 0
    for it in range(1, max_it + 1):
        rd = H @ s + q + E.T @ y + G.T @ z
        re = E @ s - e
        ri = G @ s + w - h
        mu = w.dot(z) / m
        scale = 1.0 + max(np.abs(q).max(), np.abs(h).max() if m else 0.0)
        if max(np.abs(rd).max(), np.abs(re).max() if me else 0.0, np.abs(ri).max()) < tol * scale and mu < 1e-15:
            break
        D = z / w
        # predictor (affine)
        rc = -w * z
        ds, dy = kkt_solve(D, -rd - G.T @ ((rc + z * ri) / w), -re)
        dw = -ri - G @ ds
        dz = (rc - z * dw) / w
        a_aff = min(1.0, _max_step(w, dw), _max_step(z, dz))
        mu_aff = (w + a_aff * dw).dot(z + a_aff * dz) / m
        sigma = (mu_aff / mu) ** 3
        # corrector
        rc = -w * z + sigma * mu - dw * dz
        ds, dy = kkt_solve(D, -rd - G.T @ ((rc + z * ri) / w), -re)
        dw = -ri - G @ ds
        dz = (rc - z * dw) / w
        a = min(1.0, 0.995 * _max_step(w, dw), 0.995 * _max_step(z, dz))
        s, y, w, z = s + a * ds, y + a * dy, w + a * dw, z + a * dz
    info = dict(ipm_iters=it, mu=float(w.dot(z) / m), polished=False)
    # polish: the equality-constrained QP of the active set (z > w), accepted if it satisfies the KKT conditions;
    # when it does not (an interior point that stalled before identifying the active set), primal-dual active-set
    # steps from there (act <- {z + (G s - h) > 0}, the semismooth Newton iteration of the complementarity
    # conditions) until the KKT conditions hold
    act = z > w

    def eqp(act):
        Ea = np.vstack([E, G[act]])
        ea = np.concatenate([e, h[act]])
        ka = Ea.shape[0]
        K = np.zeros((n + ka, n + ka))
        K[:n, :n] = H; K[:n, n:] = Ea.T; K[n:, :n] = Ea
        rhs = np.concatenate([-q, ea])
        sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
        for _ in range(2):  # iterative refinement of the (ill-conditioned) KKT solve
            sol = sol + np.linalg.lstsq(K, rhs - K @ sol, rcond=None)[0]
        sp, lam = sol[:n], sol[n:]
        return sp, lam, Ea
    stat = None
    hs = 1.0 + (np.abs(h).max() if m else 0.0)      # scales of the feasibility and stationarity tests
    ss = 1.0 + np.abs(q).max() + np.abs(H).max()
    for pd in range(40):
        sp, lam, Ea = eqp(act)
        za = lam[me:]
        feas = (G @ sp - h).max() if m else 0.0
        stat = np.abs(H @ sp + q + Ea.T @ lam).max()
        if os.environ.get("QPR_DEBUG"):
            print("pdas", pd, int(act.sum()), feas, za.min() if za.size else 0.0, stat)
        if feas <= 1e-11 * hs and (za.min() if za.size else 0.0) >= -1e-11 and stat <= 1e-12 * ss:
            info.update(polished=True, max_step_change=float(np.abs(sp - s).max()), active_set_steps=pd)
            s = sp
            break
        zf = np.zeros(m)
        zf[act] = za
        nxt = (zf + (G @ sp - h)) > 0
        if np.array_equal(nxt, act):
            break
        act = nxt
    info.update(kkt_stationarity=float(np.abs(H @ s + q + E.T @ y + G.T @ z).max()) if not info["polished"] else float(stat),
                primal_violation=float(max((G @ s - h).max() if m else 0.0, np.abs(E @ s - e).max() if me else 0.0)),
                active=int(act.sum()))
    return s, info


def _max_step(v, dv):
    neg = dv < 0
    return float(np.min(-v[neg] / dv[neg])) if np.any(neg) else np.inf


def solve_qp(qp, **kw):
    """The QP of solveOCP (:479): bounds l - c, u - c (an infinite side stays infinite)."""
    lo = np.where(qp["l"] <= -BIG, -INF, qp["l"] - qp["c"])
    hi = np.where(qp["u"] >= BIG, INF, qp["u"] - qp["c"])
    return solve_dense(qp["P"], qp["q"], qp["A"], lo, hi, **kw)
