"""Independent (test-side) restatement of the reference's parameter loaders and override rules.

Used to build the oracle's parameter block straight from JSON with Python's json module, so the
product's C++ JSON loader (mpcc_manipulator_amd/csrc/host) is checked against an independent path.

Reference semantics restated (cpp/src/Params/params.cpp, cpp/src/Interfaces/osqp_interface.cpp,
cpp/src/MPC/mpc.cpp):
* Param (model.json) overrides apply to Cost, Constraints, Bounds' s_trust_region, MPC and the
  track's projection distance (mpc.cpp:40-52, osqp_interface.cpp:50-59, arc_length_spline.cpp:28-31).
* CostParam overrides apply to Cost only; OsqpInterface::cost_param_ (r_ddq for the QP) is always
  read from the file (osqp_interface.cpp:57, quirk Q8).
* BoundsParam is always read from the file (osqp_interface.cpp:54,99: BoundsParam(path) without
  overrides).
* NormalizationParam / SQPParam overrides apply at construction only; setParam does not refresh them
  (osqp_interface.cpp:95-100).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), "mpcc_manipulator_amd", "data")
NN_DIR = os.path.join(DATA, "nn")


def load_default_sections():
    with open(os.path.join(DATA, "params", "default_params.json")) as f:
        return json.load(f)


def load_default_track():
    with open(os.path.join(DATA, "params", "default_track.json")) as f:
        pts = json.load(f)["points"]
    cols = list(zip(*pts))
    return [list(c) for c in cols]  # X, Y, Z, qx, qy, qz, qw


def quat_to_rot(qx, qy, qz, qw):
    """Eigen Quaterniond::normalized().toRotationMatrix() (track.cpp:45-53)."""
    n = (qx * qx + qy * qy + qz * qz + qw * qw) ** 0.5
    x, y, z, w = qx / n, qy / n, qz / n, qw / n
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return [[1 - (tyy + tzz), txy - twz, txz + twy],
            [txy + twz, 1 - (txx + tzz), tyz - twx],
            [txz - twy, tyz + twx, 1 - (txx + tyy)]]


def default_track_xyzr(init_position):
    """Track(json).getTrack(ee_pos) (track.cpp:19-66)."""
    X, Y, Z, qx, qy, qz, qw = load_default_track()
    X = [x - X[0] + init_position[0] for x in X]
    Y = [y - Y[0] + init_position[1] for y in Y]
    Z = [z - Z[0] + init_position[2] for z in Z]
    R = [quat_to_rot(*q) for q in zip(qx, qy, qz, qw)]
    return X, Y, Z, R


def load_mobile_sections():
    with open(os.path.join(DATA, "params", "mobile_params.json")) as f:
        return json.load(f)


def resolve(sections=None, overrides=None, N=20, Ts=None, constraint_mask=7, ctor_overrides=True, dof=7):
    """Effective per-consumer parameter values (dict keyed like OracleParams).  dof = 10: the Husky+Panda
    (base joints xb, yb, thb before the Panda joints; data/params/mobile_params.json)."""
    s = sections or (load_mobile_sections() if dof == 10 else load_default_sections())
    ov = overrides or {}
    m = dict(s["model"]); c = dict(s["cost"]); b = dict(s["bounds"])
    nrm = dict(s["normalization"]); q = dict(s["sqp"])
    m_o = {**m, **ov.get("param", {})}
    c_o = {**c, **ov.get("cost", {})}
    nrm_o = {**nrm, **ov.get("normalization", {})} if ctor_overrides else nrm
    q_o = {**q, **ov.get("sqp", {})} if ctor_overrides else q
    ts = Ts if Ts is not None else s["config"]["Ts"]
    base = ["xb", "yb", "thb"] if dof == 10 else []
    qn = base + ["q1", "q2", "q3", "q4", "q5", "q6", "q7"]
    un = ["d" + b for b in base] + ["dq1", "dq2", "dq3", "dq4", "dq5", "dq6", "dq7"]
    return dict(
        N=N, Ts=ts, constraint_mask=constraint_mask,
        proj_max_dist=m_o["max_dist_proj"], guess_max_dist=m_o["max_dist_proj"],
        desired_ee_velocity=m_o["desired_ee_velocity"], deacc_ratio=m_o["deaccelerate_ratio"],
        cost_tol_selcol=m_o["tol_selcol"], cost_tol_sing=m_o["tol_sing"],
        q_c=c_o["qC"], q_c_N_mult=c_o["qCNmult"], q_l=c_o["qL"], q_vs=c_o["qVs"], q_ori=c_o["qOri"],
        q_sing=c_o["qSing"], r_dq=c_o["rdq"], r_dVs=c_o["rdVs"],
        q_c_red_ratio=c_o["qC_reduction_ratio"], q_l_inc_ratio=c_o["qL_increase_ratio"],
        q_ori_red_ratio=c_o["qOri_reduction_ratio"],
        qp_r_ddq=c["rddq"],
        con_tol_selcol=m_o["tol_selcol"], con_tol_sing=m_o["tol_sing"], con_tol_envcol=m_o["tol_envcol"],
        s_trust_region=m_o["s_trust_region"],
        lx=[b[n + "l"] for n in qn] + [b["sl"], b["vsl"]],
        ux=[b[n + "u"] for n in qn] + [b["su"], b["vsu"]],
        lu=[b[n + "l"] for n in un] + [b["dVsl"]],
        uu=[b[n + "u"] for n in un] + [b["dVsu"]],
        lddq=[b["d" + n + "l"] for n in un],
        uddq=[b["d" + n + "u"] for n in un],
        Tx=[nrm_o[n] for n in qn] + [nrm_o["s"], nrm_o["vs"]],
        Tu=[nrm_o[n] for n in un] + [nrm_o["dVs"]],
        eps_prim=q_o["eps_prim"], eps_dual=q_o["eps_dual"], line_search_tau=q_o["line_search_tau"],
        line_search_eta=q_o["line_search_eta"], line_search_rho=q_o["line_search_rho"],
        max_iter=int(q_o["max_iter"]), line_search_max_iter=int(q_o["line_search_max_iter"]),
        do_SOC=int(bool(q_o["do_SOC"])), use_BFGS=int(bool(q_o["use_BFGS"])),
        vio_floor=1e-9,
    )
