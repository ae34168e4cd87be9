"""Independent restatement of the per-control-step driver in numpy: MPC::runMPC_ and OsqpInterface::solveOCP with
its filter line search, written from the reference sources, not from oracle/ or the product (VERDICT r03 next-round
item 4).  Builds on tools/qp_restate.py (QP assembly and an exact dense QP solve), tools/records_restate.py (stage
records) and tools/spline_restate.py (the track).

  * MPC::runMPC_ (cpp/src/MPC/mpc.cpp:104-190): s <- projectOnSpline(s, p_ee(q)), vs <- (Jv dq) . t(s); the
    guess goes invalid when the projection moved s by more than max_dist_proj; warm-start shift
    (updateInitialGuess :54-69, with Integrator::RK4 for the last state, integrator.cpp:29-39, Model::getF
    model.cpp:31-46) or cold start (generateNewInitialGuess :80-90), both followed by unwrapInitialGuess (:71-78,
    s <= L from stage 1 on); after the solve: valid flag and fail counter, and the return rule of :188;
  * ArcLengthSpline::projectOnSpline (cpp/src/Spline/arc_length_spline.cpp:318-379): the far branch's masking
    dist * mask + (1 - mask) * inf is NaN on every admissible grid point (0 * inf), so minCoeff, which keeps its
    first entry unless a later one compares smaller, returns index 0 (quirk Q12); Newton on |p(s) - p_ee|^2 with
    unwrapInput (clamp to [0, L]), at most 20 steps, tolerance 1e-5, s_guess back when it does not converge;
  * OsqpInterface::setInitialGuess / setEnvData / solveOCP / filterLineSearch / constraint_norm / deNormalizeStep
    (cpp/src/Interfaces/osqp_interface.cpp:102-127, 398-590, 759-833, 859-869): records frozen per solve (Q4), the
    positive-definiteness and NaN checks of the Hessian, a failed QP keeps the previous step (Q6), the filter that
    never resets its acceptance flag (Q5: after one rejection alpha = tau^L), the step in normalized coordinates
    de-normalized by T_x, T_u, primal_step_norm = alpha |step|_inf against eps_prim, MAX_ITER_EXCEEDED when the loop
    runs out, and the zero guess (x0 repeated, u = 0) on any exit but SOLVED (Q7).
The QP is solved exactly (the documented deviation from OSQP), and the filter's violation norm
counts per-row violations <= 1e-9 as zero (parity policy P1): an exact QP step leaves rounding-level
violations where OSQP leaves ~1e-4.  Test infrastructure only (tools/make_sqp_fixture.py, tests/test_sqp_restate.py).
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import qp_restate as qr  # noqa: E402
import records_restate as rr  # noqa: E402

NX, NU, DOF, IS, IVS, IDVS = qr.NX, qr.NU, qr.DOF, qr.IS, qr.IVS, qr.IDVS
SOLVED, MAX_ITER_EXCEEDED, NAN_HESSIAN, NON_PD_HESSIAN = 0, 1, 10, 11  # solver_interface.h Status (the ABI's values)
VIO_FLOOR = 1e-9  # parity policy P1


def load_sqp_params(params_dir):
    import json
    with open(os.path.join(params_dir, "sqp.json")) as f:
        s = json.load(f)
    return dict(eps_prim=s["eps_prim"], max_iter=s["max_iter"], ls_max=s["line_search_max_iter"],
                tau=s["line_search_tau"])


def project_on_spline(track, s_guess, ee, max_dist_proj):
    """ArcLengthSpline::projectOnSpline (arc_length_spline.cpp:318-379)."""
    sgrid, X, Y, Z = (np.asarray(v, float) for v in track.path[:4])
    L = track.length
    pos = track.ref(s_guess)[0]
    s_opt = s_guess
    dist = np.linalg.norm(ee - pos)
    if dist >= max_dist_proj:
        d2 = (X - ee[0]) ** 2 + (Y - ee[1]) ** 2 + (Z - ee[2]) ** 2
        valid = np.abs(sgrid - s_guess) <= max_dist_proj
        if not valid.any():
            s_opt = sgrid[int(np.argmin(d2))]
        else:
            # d2 * valid + (1 - valid) * inf: NaN where valid (0 * inf), inf elsewhere; minCoeff keeps index 0
            s_opt = sgrid[0]
    if s_opt >= sgrid[-1]:
        return sgrid[-1]
    s_old = s_opt
    for _ in range(20):
        p, d1, d2_, _, _ = track.ref(s_opt)
        diff = p - ee
        jac = 2.0 * diff[0] * d1[0] + 2.0 * diff[1] * d1[1] + 2.0 * diff[2] * d1[2]
        hess = (2.0 * d1[0] * d1[0] + 2.0 * diff[0] * d2_[0] + 2.0 * d1[1] * d1[1] + 2.0 * diff[1] * d2_[1]
                + 2.0 * d1[2] * d1[2] + 2.0 * diff[2] * d2_[2])
        s_opt -= jac / hess
        s_opt = max(0.0, min(s_opt, L))  # unwrapInput
        if abs(s_old - s_opt) <= 1e-5:
            return s_opt
        s_old = s_opt
    return s_guess


def rk4(x, u, ts):
    """Integrator::RK4 with Model::getF (x' = [dq, vs, dVs])."""
    def f(xv):
        o = np.zeros(NX)
        o[:DOF] = u[:DOF]
        o[IS] = xv[IVS]
        o[IVS] = u[IDVS]
        return o
    k1 = f(x)
    k2 = f(x + ts / 2.0 * k1)
    k3 = f(x + ts / 2.0 * k2)
    k4 = f(x + ts * k3)
    return x + ts * (k1 / 6.0 + k2 / 3.0 + k3 / 3.0 + k4 / 6.0)


def denormalize(step, P, N):
    """deNormalizeStep (osqp_interface.cpp:859-869) on the stacked [x_0..x_N | u_0..u_{N-1}] vector."""
    d = step.copy()
    for i in range(N + 1):
        d[NX * i:NX * i + NX] *= P["Tx"]
        if i != N:
            o = NX * (N + 1) + NU * i
            d[o:o + NU] *= P["Tu"]
    return d


def to_vec(guess, N):
    v = np.zeros(NX * (N + 1) + NU * N)
    for i in range(N + 1):
        v[NX * i:NX * i + NX] = guess[i, :NX]
        if i != N:
            v[NX * (N + 1) + NU * i:NX * (N + 1) + NU * i + NU] = guess[i, NX:]
    return v


def to_guess(v, N, uN=0.0):
    """vectorToOptvar (osqp_interface.cpp:835-845): u_N is not written; the std::vector's fresh elements are
    value-initialized, so it is 0 (never read by the QP)."""
    g = np.zeros((N + 1, NX + NU))
    for i in range(N + 1):
        g[i, :NX] = v[NX * i:NX * i + NX]
        g[i, NX:] = v[NX * (N + 1) + NU * i:NX * (N + 1) + NU * i + NU] if i != N else uN
    return g


def constraint_norm(c, lo, hi):
    """constraint_norm (osqp_interface.cpp:824-833) with the P1 floor."""
    a = np.maximum(lo - c, 0.0)
    b = np.maximum(c - hi, 0.0)
    return float(np.where(a > VIO_FLOOR, a, 0.0).sum() + np.where(b > VIO_FLOOR, b, 0.0).sum())


def solve_ocp(P, S, track, guess, recs, ucur, N, mask):
    """OsqpInterface::solveOCP (osqp_interface.cpp:398-590) without BFGS / SOC.  Returns (out guess, status,
    sqp iterations run, trace [(qp_ok, alpha, step_norm, obj, vio)])."""
    uN = 0.0
    vec = to_vec(guess, N)
    step = np.zeros_like(vec)
    filt = []
    zero = np.zeros_like(guess)
    zero[:, :NX] = guess[0, :NX]
    status, trace, it = None, [], 0
    cur = guess.copy()
    for it in range(S["max_iter"]):
        qp = qr.assemble(P, track, cur, recs, ucur, N, mask)
        H = qp["P"]
        try:
            np.linalg.cholesky(H)
        except np.linalg.LinAlgError:
            status = NON_PD_HESSIAN
            break
        if np.isnan(H).any():
            status = NAN_HESSIAN
            break
        qp_ok = True
        try:
            s_new, info = qr.solve_qp(qp)
            qp_ok = info["primal_violation"] <= 1e-9 and info["kkt_stationarity"] <= 1e-8
        except (ValueError, np.linalg.LinAlgError):
            qp_ok = False
        if qp_ok:
            step = s_new  # a failed QP leaves the previous step (Q6)
        # filterLineSearch (:759-808)
        accepted, alpha = True, 1.0
        obj_t = vio_t = None
        for _ in range(S["ls_max"]):
            trial = to_guess(vec + alpha * denormalize(step, P, N), N, uN)
            tq = qr.assemble(P, track, trial, recs, ucur, N, mask)
            f_obj, f_vio = tq["obj"], constraint_norm(tq["c"], tq["l"], tq["u"])
            if obj_t is None:
                obj_t, vio_t = f_obj, f_vio
            for fo, fv in filt:
                if f_obj >= fo and f_vio >= fv:
                    accepted = False
                    break
            if accepted:
                filt = [(fo, fv) for fo, fv in filt if f_obj > fo or f_vio > fv] + [(f_obj, f_vio)]
                break
            alpha *= S["tau"]
        vec = vec + alpha * denormalize(step, P, N)
        cur = to_guess(vec, N, uN)
        nrm = alpha * float(np.abs(step).max())
        trace.append((qp_ok, alpha, nrm, obj_t, vio_t))
        if nrm < S["eps_prim"]:
            status = SOLVED
            break
    else:
        it = S["max_iter"]
        status = MAX_ITER_EXCEEDED
    return (cur if status == SOLVED else zero), status, it, trace


def prepare(P, track, x0, u0, guess, valid, fails, N):
    """runMPC_ up to the solve (mpc.cpp:106-121): projection, vs, validity, warm-start shift or cold start.  x0 is
    updated in place; returns (guess for the solver, valid, fails)."""
    L = track.length
    last_s = x0[IS]
    q = x0[:DOF]
    ee = rr.kinematics(q)[0]
    x0[IS] = project_on_spline(track, last_s, ee, P["max_dist_proj"])
    Jv = rr.jacobian(q)[:3]
    x0[IVS] = float((Jv @ u0[:DOF]).dot(track.ref(x0[IS])[1]))
    if abs(last_s - x0[IS]) > P["max_dist_proj"]:
        valid = 0
        fails += 1
    g = guess.copy()
    if valid:
        for i in range(1, N):
            g[i - 1] = g[i]
        g[0, :NX] = x0
        g[N - 1] = g[N - 2]
        g[N, :NX] = rk4(g[N - 1, :NX], g[N - 1, NX:], P["Ts"])
        g[N, NX:] = 0.0
    else:
        g[:, :NX] = x0
        g[:, NX:] = 0.0
        valid = 1
    for i in range(1, N + 1):
        g[i, IS] = min(g[i, IS], L)
    return g, valid, fails


def run_mpc(P, S, track, nets, x0, u0, obs, guess, valid, fails, N, mask):
    """MPC::runMPC_ (mpc.cpp:104-190) for one controller.  x0 is updated in place (s, vs); returns dict with the
    horizon (the new initial guess), u0, status, the new valid flag / fail counter, the return value, the stage
    records and the SQP trace."""
    g, valid, fails = prepare(P, track, x0, u0, guess, valid, fails, N)
    recs = np.array([rr.record(g[i, :DOF], obs[:3], obs[3], nets) for i in range(N + 1)])
    out, status, it, trace = solve_ocp(P, S, track, g, recs, u0, N, mask)
    if status == SOLVED:
        valid, fails = 1, 0
    else:
        valid, fails = 0, fails + 1
    ok = status == SOLVED or (status == MAX_ITER_EXCEEDED and fails < 5)
    return dict(horizon=out, u0=out[0, NX:].copy(), status=status, valid=valid, fails=fails, ok=ok, recs=recs,
                sqp_iter=it, trace=trace, guess_in=g)
