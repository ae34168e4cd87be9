"""ctypes wrapper of the CPU parity oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
REC_SIZE = 143

D = C.c_double
DP = C.POINTER(C.c_double)
IP = C.POINTER(C.c_int)


def _params_struct(dof):
    nx, nu = dof + 2, dof + 1

    class _P(C.Structure):
        _fields_ = [
            ("N", C.c_int), ("Ts", D), ("constraint_mask", C.c_int),
            ("proj_max_dist", D), ("guess_max_dist", D),
            ("desired_ee_velocity", D), ("deacc_ratio", D), ("cost_tol_selcol", D), ("cost_tol_sing", D),
            ("q_c", D), ("q_c_N_mult", D), ("q_l", D), ("q_vs", D), ("q_ori", D), ("q_sing", D),
            ("r_dq", D), ("r_dVs", D), ("q_c_red_ratio", D), ("q_l_inc_ratio", D), ("q_ori_red_ratio", D),
            ("qp_r_ddq", D),
            ("con_tol_selcol", D), ("con_tol_sing", D), ("con_tol_envcol", D),
            ("s_trust_region", D),
            ("lx", D * nx), ("ux", D * nx), ("lu", D * nu), ("uu", D * nu), ("lddq", D * dof), ("uddq", D * dof),
            ("Tx", D * nx), ("Tu", D * nu),
            ("eps_prim", D), ("eps_dual", D), ("line_search_tau", D), ("line_search_eta", D),
            ("line_search_rho", D),
            ("max_iter", C.c_int), ("line_search_max_iter", C.c_int), ("do_SOC", C.c_int), ("use_BFGS", C.c_int),
            ("vio_floor", D),
        ]
    _P.__name__ = f"OracleParams{dof}"
    return _P


OracleParams = _params_struct(7)
OracleParamsMobile = _params_struct(10)
PARAMS = {7: OracleParams, 10: OracleParamsMobile}
LIBS = {7: "liboracle.so", 10: "liboracle_mobile.so"}


class OracleOptions(C.Structure):
    _fields_ = [("qp_mode", C.c_int), ("nthreads", C.c_int)]


def build(quiet=True):
    """Compile the oracle with its committed Makefile (gcc; no reference sources involved)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)
    return LIB_PATH


_libs = {}


def lib(dof=7):
    """The oracle build for a robot: dof 7 = Panda (liboracle.so), 10 = Husky+Panda (liboracle_mobile.so)."""
    if dof not in _libs:
        path = os.path.join(HERE, "_build", LIBS[dof])
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        OP = PARAMS[dof]
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(OP), C.c_char_p, OracleOptions]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_set_params.argtypes = [C.c_void_p, C.POINTER(OP)]
        L.oracle_set_track.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP]
        L.oracle_track_length.restype = D
        L.oracle_track_length.argtypes = [C.c_void_p]
        L.oracle_track_path.argtypes = [C.c_void_p, DP, DP, DP, DP, DP]
        L.oracle_fk.argtypes = [DP, DP, DP, DP]
        L.oracle_manipulability.restype = D
        L.oracle_manipulability.argtypes = [DP]
        L.oracle_dmanipulability.argtypes = [DP, DP]
        L.oracle_self_mlp.argtypes = [C.c_void_p, DP, DP, DP]
        L.oracle_env_mlp.argtypes = [C.c_void_p, DP, DP, DP]
        L.oracle_spline_eval.argtypes = [C.c_void_p, D, DP, DP, DP, DP, DP]
        L.oracle_project.restype = D
        L.oracle_project.argtypes = [C.c_void_p, D, DP]
        L.oracle_robot_record.argtypes = [C.c_void_p, DP, DP, D, DP]
        L.oracle_stage_cost.argtypes = [C.c_void_p, DP, DP, DP, C.c_int, DP, DP, DP, DP, DP, DP]
        L.oracle_stage_constraints.argtypes = [C.c_void_p, DP, DP, DP, C.c_int, DP, DP, DP, DP, DP]
        L.oracle_dense_qp.restype = D
        L.oracle_dense_qp.argtypes = [C.c_void_p, DP, DP, DP, DP, DP, DP, DP, DP, DP]
        L.oracle_solve_qp.restype = C.c_int
        L.oracle_solve_qp.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP, IP]
        L.oracle_solve_qp_lr.restype = C.c_int
        L.oracle_solve_qp_lr.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, C.c_int, DP, DP, DP, IP]
        L.oracle_solve_soc.restype = C.c_int
        L.oracle_solve_soc.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP, DP, IP]
        L.oracle_rk4.argtypes = [DP, DP, D, DP]
        L.oracle_sim_time_step.argtypes = [DP, DP, D, DP]
        L.oracle_run_mpc.restype = C.c_int
        L.oracle_run_mpc.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP, IP, IP, DP, DP, IP, IP, IP]
        L.oracle_cubic_spline.restype = None
        L.oracle_cubic_spline.argtypes = [C.c_int, DP, DP, C.c_int, C.c_int, DP, DP]
        L.oracle_prepare.restype = C.c_int
        L.oracle_prepare.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP, IP, IP, DP]
        L.oracle_run_mpc_trace.restype = C.c_int
        L.oracle_run_mpc_trace.argtypes = [C.c_void_p, C.c_int, DP, DP, DP, DP, IP, IP, DP, DP, IP, IP, IP, DP]
        L.oracle_rec_size.restype = C.c_int
        L.oracle_fk_frame.argtypes = [DP, C.c_int, DP, DP, DP]
        L.oracle_manip_from_J.restype = D
        L.oracle_manip_from_J.argtypes = [DP]
        L.oracle_dof.restype = C.c_int
        assert L.oracle_dof() == dof and L.oracle_rec_size() == 24 + 17 * dof
        _libs[dof] = L
    return _libs[dof]


def _dp(a):
    return a.ctypes.data_as(DP)


def _ip(a):
    return a.ctypes.data_as(IP)


def _f64(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if shape is not None:
        a = a.reshape(shape)
    return a


def make_params(d, dof=7):
    """OracleParams from a dict of resolved values (see tests/refparams.py)."""
    p = PARAMS[dof]()
    for name, _ in OracleParams._fields_:
        v = d[name]
        f = getattr(p, name)
        if hasattr(f, "__len__"):
            for i, x in enumerate(v):
                f[i] = x
        else:
            setattr(p, name, v)
    return p


class Oracle:
    def __init__(self, params: dict, nn_dir: str, qp_mode=0, nthreads=1, dof=7):
        self.dof = dof
        self.NX, self.NU = dof + 2, dof + 1
        self.NXU = self.NX + self.NU
        self.REC = 24 + 17 * dof
        self.L = lib(dof)
        self.params = dict(params)
        self._p = make_params(params, dof)
        opt = OracleOptions(qp_mode, nthreads)
        self.h = self.L.oracle_create(C.byref(self._p), nn_dir.encode() if nn_dir else None, opt)
        self.N = params["N"]

    def close(self):
        if self.h:
            self.L.oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params: dict):
        self.params = dict(params)
        self._p = make_params(params, self.dof)
        self.L.oracle_set_params(self.h, C.byref(self._p))

    def set_track(self, X, Y, Z, R):
        X, Y, Z = _f64(X), _f64(Y), _f64(Z)
        R = _f64(R).reshape(-1, 9)
        self.L.oracle_set_track(self.h, len(X), _dp(X), _dp(Y), _dp(Z), _dp(R))

    def track_length(self):
        return self.L.oracle_track_length(self.h)

    def track_path(self):
        s, X, Y, Z = (np.zeros(100) for _ in range(4))
        R = np.zeros((100, 9))
        self.L.oracle_track_path(self.h, _dp(s), _dp(X), _dp(Y), _dp(Z), _dp(R))
        return s, X, Y, Z, R.reshape(100, 3, 3)

    # ---- kinematics
    def fk(self, q):
        q = _f64(q)
        p, R, J = np.zeros(3), np.zeros(9), np.zeros(6 * self.dof)
        self.L.oracle_fk(_dp(q), _dp(p), _dp(R), _dp(J))
        return p, R.reshape(3, 3), J.reshape(6, self.dof)

    def fk_frame(self, q, frame):
        """RobotModel frame 1..9 (panda_link0..7, panda_hand_tcp): position, rotation, 6x7 Jacobian."""
        q = _f64(q)
        p, R, J = np.zeros(3), np.zeros(9), np.zeros(42)
        self.L.oracle_fk_frame(_dp(q), int(frame), _dp(p), _dp(R), _dp(J))
        return p, R.reshape(3, 3), J.reshape(6, 7)

    def manip_from_J(self, J):
        return self.L.oracle_manip_from_J(_dp(_f64(J).reshape(6 * self.dof)))

    def manipulability(self, q):
        return self.L.oracle_manipulability(_dp(_f64(q)))

    def dmanipulability(self, q):
        d = np.zeros(self.dof)
        self.L.oracle_dmanipulability(_dp(_f64(q)), _dp(d))
        return d

    def self_mlp(self, q):
        d, g = np.zeros(1), np.zeros(7)
        self.L.oracle_self_mlp(self.h, _dp(_f64(q)), _dp(d), _dp(g))
        return d[0], g

    def env_mlp(self, inp):
        d, j = np.zeros(9), np.zeros(90)
        self.L.oracle_env_mlp(self.h, _dp(_f64(inp)), _dp(d), _dp(j))
        return d, j.reshape(9, 10)

    def spline_eval(self, s):
        out = [np.zeros(3), np.zeros(3), np.zeros(3), np.zeros(9), np.zeros(3)]
        self.L.oracle_spline_eval(self.h, float(s), *[_dp(a) for a in out])
        out[3] = out[3].reshape(3, 3)
        return out

    def project(self, s, ee):
        return self.L.oracle_project(self.h, float(s), _dp(_f64(ee)))

    def robot_record(self, q, obs=(3.0, 3.0, 3.0), obs_r=0.0):
        rec = np.zeros(self.REC)
        self.L.oracle_robot_record(self.h, _dp(_f64(q)[:self.dof].copy()), _dp(_f64(obs)), float(obs_r), _dp(rec))
        return rec

    def stage_cost(self, x, u, rec, k):
        obj = np.zeros(1)
        nx, nu = self.NX, self.NU
        fx, fu, fxx, fuu, fxu = np.zeros(nx), np.zeros(nu), np.zeros(nx * nx), np.zeros(nu * nu), np.zeros(nx * nu)
        self.L.oracle_stage_cost(self.h, _dp(_f64(x)), _dp(_f64(u)), _dp(_f64(rec)), int(k), _dp(obj),
                                 _dp(fx), _dp(fu), _dp(fxx), _dp(fuu), _dp(fxu))
        return obj[0], fx, fu, fxx.reshape(nx, nx), fuu.reshape(nu, nu), fxu.reshape(nx, nu)

    def stage_constraints(self, x, u, rec, k):
        nx, nu = self.NX, self.NU
        c, l, u_, cx, cu = np.zeros(11), np.zeros(11), np.zeros(11), np.zeros(11 * nx), np.zeros(11 * nu)
        self.L.oracle_stage_constraints(self.h, _dp(_f64(x)), _dp(_f64(u)), _dp(_f64(rec)), int(k),
                                        _dp(c), _dp(l), _dp(u_), _dp(cx), _dp(cu))
        return c, l, u_, cx.reshape(11, nx), cu.reshape(11, nu)

    def nvar(self):
        return self.NXU * self.N + self.NX

    def nconstr(self):
        nx, nu, N = self.NX, self.NU, self.N
        return (N + 1) * nx + ((N + 1) * nx + 2 * N * nu) + (N + 1) * 11

    def dense_qp(self, guess, recs, u_current):
        nv, nc = self.nvar(), self.nconstr()
        P, g, A = np.zeros(nv * nv), np.zeros(nv), np.zeros(nc * nv)
        c, l, u = np.zeros(nc), np.zeros(nc), np.zeros(nc)
        obj = self.L.oracle_dense_qp(self.h, _dp(_f64(guess)), _dp(_f64(recs)), _dp(_f64(u_current)),
                                     _dp(P), _dp(g), _dp(A), _dp(c), _dp(l), _dp(u))
        return dict(obj=obj, P=P.reshape(nv, nv), g=g, A=A.reshape(nc, nv), c=c, l=l, u=u)

    def solve_qp(self, guess, recs, u_current, mode=0):
        step = np.zeros(self.nvar())
        it = np.zeros(1, dtype=np.int32)
        rc = self.L.oracle_solve_qp(self.h, int(mode), _dp(_f64(guess)), _dp(_f64(recs)),
                                    _dp(_f64(u_current)), _dp(step), _ip(it))
        return rc, step, int(it[0])

    def solve_qp_lr(self, guess, recs, u_current, lr, lrc, mode=0):
        """One QP with low-rank Hessian terms (the damped-BFGS form): lr [nlr, N+1, NXU], lrc [nlr]."""
        lr = _f64(lr).reshape(-1, self.N + 1, self.NXU)
        lrc = _f64(lrc).reshape(-1)
        step = np.zeros(self.nvar())
        it = C.c_int(0)
        rc = self.L.oracle_solve_qp_lr(self.h, int(mode), _dp(_f64(guess)), _dp(_f64(recs)), _dp(_f64(u_current)),
                                       int(lr.shape[0]), _dp(lr), _dp(lrc), _dp(step), C.byref(it))
        return rc, step, it.value

    def solve_soc(self, guess, recs, u_current, step, mode=0):
        """SecondOrderCorrection QP (osqp_interface.cpp:658-681) after the first QP's step."""
        out = np.zeros(self.nvar())
        it = np.zeros(1, dtype=np.int32)
        rc = self.L.oracle_solve_soc(self.h, int(mode), _dp(_f64(guess)), _dp(_f64(recs)), _dp(_f64(u_current)),
                                     _dp(_f64(step)), _dp(out), _ip(it))
        return rc, out, int(it[0])

    def rk4(self, x, u, ts):
        out = np.zeros(self.NX)
        self.L.oracle_rk4(_dp(_f64(x)), _dp(_f64(u)), float(ts), _dp(out))
        return out

    def sim_time_step(self, x, u, ts):
        out = np.zeros(self.NX)
        self.L.oracle_sim_time_step(_dp(_f64(x)), _dp(_f64(u)), float(ts), _dp(out))
        return out

    @staticmethod
    def cubic_spline(x, y, xq, regular=True):
        """CubicSpline (cubic_spline.cpp) fit to (x, y), evaluated at xq -> [m, 3] (y, y', y'')."""
        x, y, xq = _f64(x), _f64(y), _f64(xq)
        out = np.zeros((xq.shape[0], 3))
        lib().oracle_cubic_spline(x.shape[0], _dp(x), _dp(y), 1 if regular else 0, xq.shape[0], _dp(xq), _dp(out))
        return out

    def prepare(self, x0, u0, obs, guess, valid, fails):
        """runMPC_ up to the SQP (in place on x0, guess, valid, fails); returns the frozen records."""
        B = x0.shape[0]
        recs = np.zeros((B, self.N + 1, self.L.oracle_rec_size()))
        self.L.oracle_prepare(self.h, B, _dp(x0), _dp(_f64(u0, (B, self.NU))), _dp(_f64(obs, (B, 4))), _dp(guess),
                              _ip(valid), _ip(fails), _dp(recs))
        return recs

    def run_mpc(self, x0, u0, obs, guess, valid, fails, trace=False):
        """Batched runMPC_.  All arrays are modified in place where the reference mutates them
        (x0, guess, valid, fails).  Returns dict of outputs."""
        B = x0.shape[0]
        N = self.N
        nx, nu, nxu = self.NX, self.NU, self.NXU
        assert x0.dtype == np.float64 and x0.flags.c_contiguous and x0.shape == (B, nx)
        assert guess.dtype == np.float64 and guess.flags.c_contiguous and guess.shape == (B, N + 1, nxu)
        assert valid.dtype == np.int32 and fails.dtype == np.int32
        u0 = _f64(u0, (B, nu))
        obs = _f64(obs, (B, 4))
        u0_out = np.zeros((B, nu))
        hor = np.zeros((B, N + 1, nxu))
        status = np.zeros(B, dtype=np.int32)
        ok = np.zeros(B, dtype=np.int32)
        iters = np.zeros(B, dtype=np.int32)
        tr = np.zeros((B, 4, 8)) if trace else None
        self.L.oracle_run_mpc_trace(self.h, B, _dp(x0), _dp(u0), _dp(obs), _dp(guess), _ip(valid), _ip(fails),
                                    _dp(u0_out), _dp(hor), _ip(status), _ip(ok), _ip(iters),
                                    _dp(tr) if trace else None)
        out = dict(u0=u0_out, horizon=hor, status=status, ok=ok, sqp_iters=iters)
        if trace:
            out["trace"] = tr
        return out
