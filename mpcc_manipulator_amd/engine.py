"""ctypes bindings of libmpcc_engine.so (include/mpcc_engine.h) and the batched Engine wrapper.

The product path is HIP-only: if the shared library (or a GPU) is missing, the calls fail loudly —
there is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(PKG, "data")
NN_DIR = os.path.join(DATA, "nn")
DEFAULT_PARAMS = os.path.join(DATA, "params", "default_params.json")
DEFAULT_TRACK = os.path.join(DATA, "params", "default_track.json")
MOBILE_PARAMS = os.path.join(DATA, "params", "mobile_params.json")
LIB_PATH = os.environ.get("MPCC_ENGINE_LIB", os.path.join(PKG, "_build", "libmpcc_engine.so"))
# Robot dimensions are compile-time in the engine, as the reference's NX/NU (config.h:29-38): one library
# per robot with the same C ABI.  dof 7 = Franka Panda, dof 10 = Husky+Panda mobile manipulator.
LIB_PATHS = {7: LIB_PATH, 10: os.environ.get("MPCC_ENGINE_LIB_MOBILE", os.path.join(PKG, "_build", "libmpcc_engine_mobile.so"))}
ROBOT_DOF = {"panda": 7, "husky_panda": 10}

REC_SIZE = 143
NX, NU, PANDA_DOF, PANDA_NUM_LINKS = 9, 8, 7, 9


def dims(dof):
    """(NX, NU, NXU, REC) of a robot with dof joints: state [q, s, vs], input [dq, dVs]."""
    return dof + 2, dof + 1, 2 * dof + 3, 24 + 17 * dof

D, I32 = C.c_double, C.c_int32
DP, IP = C.POINTER(C.c_double), C.POINTER(C.c_int32)

# Status (solver_interface.h:28-42)
STATUS_NAMES = ["SOLVED", "MAX_ITER_EXCEEDED", "QP_DualInfeasibleInaccurate", "QP_PrimalInfeasibleInaccurate",
                "QP_SolvedInaccurate", "QP_MaxIterReached", "QP_PrimalInfeasible", "QP_DualInfeasible", "Sigint",
                "INVALID_SETTINGS", "NAN_HESSIAN", "NON_PD_HESSIAN"]
SOLVED, MAX_ITER_EXCEEDED = 0, 1
CON_SELFCOL, CON_SING, CON_ENVCOL = 1, 2, 4


def _params_struct(dof):
    """mpcc_params (include/mpcc_engine.h) of the library built with MPCC_DOF = dof."""
    nx, nu = dof + 2, dof + 1

    class _P(C.Structure):
        _dof = dof
        _fields_ = [
            ("N", I32), ("Ts", D), ("constraint_mask", I32),
            ("proj_max_dist", D), ("guess_max_dist", D),
            ("desired_ee_velocity", D), ("deacc_ratio", D), ("cost_tol_selcol", D), ("cost_tol_sing", D),
            ("q_c", D), ("q_c_N_mult", D), ("q_l", D), ("q_vs", D), ("q_ori", D), ("q_sing", D), ("r_dq", D),
            ("r_dVs", D), ("q_c_red_ratio", D), ("q_l_inc_ratio", D), ("q_ori_red_ratio", D),
            ("qp_r_ddq", D),
            ("con_tol_selcol", D), ("con_tol_sing", D), ("con_tol_envcol", D),
            ("s_trust_region", D),
            ("lx", D * nx), ("ux", D * nx), ("lu", D * nu), ("uu", D * nu), ("lddq", D * dof), ("uddq", D * dof),
            ("Tx", D * nx), ("Tu", D * nu),
            ("eps_prim", D), ("eps_dual", D), ("line_search_tau", D), ("line_search_eta", D), ("line_search_rho", D),
            ("max_iter", I32), ("line_search_max_iter", I32), ("do_SOC", I32), ("use_BFGS", I32),
            ("vio_floor", D),
        ]

        def as_dict(self):
            out = {}
            for name, _ in self._fields_:
                v = getattr(self, name)
                out[name] = list(v) if hasattr(v, "__len__") else v
            return out

    _P.__name__ = "MpccParams" if dof == 7 else f"MpccParams{dof}"
    return _P


PARAMS_STRUCT = {7: _params_struct(7), 10: _params_struct(10)}
MpccParams = PARAMS_STRUCT[7]


class MpccJsonPaths(C.Structure):
    _fields_ = [("param_path", C.c_char_p), ("cost_path", C.c_char_p), ("bounds_path", C.c_char_p),
                ("normalization_path", C.c_char_p), ("sqp_path", C.c_char_p), ("merged_path", C.c_char_p)]


class MpccOverride(C.Structure):
    _fields_ = [("section", C.c_char_p), ("key", C.c_char_p), ("value", D)]


class MpccConfig(C.Structure):
    _fields_ = [("N", I32), ("Ts", D), ("max_batch", I32), ("device", I32), ("constraint_mask", I32),
                ("faithful_dead_trials", I32)]


class MpccTiming(C.Structure):
    _fields_ = [("set_env", D), ("set_qp", D), ("solve_qp", D), ("get_alpha", D), ("total", D)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MpccError(RuntimeError):
    pass


_libs = {}
BUILD_BOUNDS_CHECK, BUILD_PROF = 1, 2
import weakref  # noqa: E402
LIVE_CHECKED = weakref.WeakSet()  # engines of a bounds-checked library (tests/conftest.py reads their flags)


def build_id(dof=7):
    """Hash of the sources the loaded library was compiled from (mpcc_manipulator_amd._build.source_hash)."""
    return lib(dof).mpcc_build_id().decode()


def lib(dof=7):
    """Load the engine library of a robot (dof 7: libmpcc_engine.so, 10: libmpcc_engine_mobile.so; build
    them first with mpcc_manipulator_amd._build.build())."""
    if dof in _libs:
        return _libs[dof]
    path = LIB_PATHS[dof]
    if not os.path.exists(path):
        raise MpccError(f"{os.path.basename(path)} not built ({path}); run python -m mpcc_manipulator_amd._build")
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME libamdhip64.so.7, loaded by
    # the unversioned name libamdhip64.so).  Loaded first, it satisfies the engine's libamdhip64.so.7
    # dependency; loaded after the engine had pulled in /opt/rocm's copy, it would be a second runtime
    # in the process and torch.cuda fails to initialise ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    V = C.c_void_p
    MpccParams = PARAMS_STRUCT[dof]
    sig = {
        "mpcc_abi_version": (C.c_int, []),
        "mpcc_robot_dof": (C.c_int, []),
        "mpcc_last_error": (C.c_char_p, []),
        "mpcc_params_load_json": (C.c_int, [C.POINTER(MpccJsonPaths), C.POINTER(MpccOverride), C.c_int, C.c_int,
                                            C.c_int, C.POINTER(MpccParams)]),
        "mpcc_create": (C.c_int, [C.POINTER(MpccConfig), C.POINTER(MpccParams), C.c_char_p, C.POINTER(V)]),
        "mpcc_destroy": (None, [V]),
        "mpcc_set_params": (C.c_int, [V, C.POINTER(MpccParams)]),
        "mpcc_get_params": (C.c_int, [V, C.POINTER(MpccParams)]),
        "mpcc_set_track": (C.c_int, [V, C.c_int, DP, DP, DP, DP]),
        "mpcc_track_length": (D, [V]),
        "mpcc_get_track_path": (C.c_int, [V, DP, DP, DP, DP, DP]),
        "mpcc_track_build_host": (C.c_int, [C.c_int, DP, DP, DP, DP, DP, DP, DP, DP, DP, DP]),
        "mpcc_set_warmstart": (C.c_int, [V, C.c_int, DP, IP, IP]),
        "mpcc_get_warmstart": (C.c_int, [V, C.c_int, DP, IP, IP]),
        "mpcc_reset_warmstart": (C.c_int, [V, C.c_int, C.POINTER(C.c_uint8)]),
        "mpcc_solve": (C.c_int, [V, C.c_int, DP, DP, DP, DP, DP, IP, IP, C.POINTER(MpccTiming)]),
        "mpcc_solve_device": (C.c_int, [V, C.c_int, V, V, V, V, V, V, V, V]),
        "mpcc_closed_loop": (C.c_int, [V, C.c_int, C.c_int, DP, DP, DP, DP, DP, IP, C.c_int]),
        "mpcc_set_tracks": (C.c_int, [V, C.c_int, C.c_int, DP, DP, DP, DP]),
        "mpcc_set_track_path": (C.c_int, [V, C.c_int, DP, DP, DP, DP, DP]),
        "mpcc_solve_ocp": (C.c_int, [V, C.c_int, DP, DP, DP, DP, IP, IP, C.POINTER(MpccTiming)]),
        "mpcc_sim_time_step": (C.c_int, [V, C.c_int, DP, DP, D, DP]),
        "mpcc_set_warmstart_device": (C.c_int, [V, C.c_int, V, V, V, V]),
        "mpcc_timing_begin": (C.c_int, [V]),
        "mpcc_timing_end": (C.c_int, [V, C.POINTER(MpccTiming), IP, IP]),
        "mpcc_get_solve_stats": (C.c_int, [V, C.c_int, IP, IP, IP]),
        "mpcc_debug_robot_records": (C.c_int, [V, C.c_int, DP, DP, DP]),
        "mpcc_debug_spline": (C.c_int, [V, C.c_int, DP, DP, DP, DP, DP, DP]),
        "mpcc_debug_stage_cost": (C.c_int, [V, C.c_int, DP, DP, DP, IP, DP, DP, DP, DP, DP]),
        "mpcc_debug_solve_qp": (C.c_int, [V, C.c_int, DP, DP, DP, DP, IP, IP]),
        "mpcc_debug_solve_qp_lr": (C.c_int, [V, C.c_int, DP, DP, DP, C.c_int, DP, DP, DP, IP, IP]),
        "mpcc_debug_trace_enable": (C.c_int, [V, C.c_int]),
        "mpcc_debug_workspace": (C.c_int, [V, C.c_int, DP]),
        "mpcc_debug_project": (C.c_int, [V, C.c_int, DP, DP, DP]),
        "mpcc_debug_trace_get": (C.c_int, [V, C.c_int, DP]),
        "mpcc_track_eval_host": (C.c_int, [C.c_int, DP, DP, DP, DP, C.c_int, DP, DP, DP, DP, DP, DP]),
        "mpcc_track_project_host": (C.c_int, [C.c_int, DP, DP, DP, DP, C.c_int, D, DP, DP, DP]),
        "mpcc_cubic_spline_host": (C.c_int, [C.c_int, DP, DP, C.c_int, C.c_int, DP, DP]),
        "mpcc_rot_spline_host": (C.c_int, [C.c_int, DP, DP, C.c_int, C.c_int, DP, DP, DP]),
        "mpcc_so3_log": (C.c_int, [DP, DP]),
        "mpcc_so3_exp": (C.c_int, [DP, DP]),
        "mpcc_mlp_create": (C.c_int, [C.c_int, C.c_char_p, C.c_int, C.c_int, IP, C.c_int, C.c_int, C.POINTER(V)]),
        "mpcc_mlp_eval": (C.c_int, [V, C.c_int, DP, DP, DP]),
        "mpcc_mlp_dims": (C.c_int, [V, IP, IP]),
        "mpcc_mlp_destroy": (None, [V]),
        "mpcc_robot_frames": (C.c_int, [C.c_int, C.c_int, DP, C.c_int, DP, DP, DP, DP, DP]),
        "mpcc_debug_bounds": (C.c_int, [V, C.POINTER(C.c_uint32), C.c_int]),
        "mpcc_debug_tail_solves": (C.c_int, [C.POINTER(C.c_longlong), C.c_int]),
        "mpcc_debug_order": (C.c_int, [V, IP, C.c_int]),
        "mpcc_build_id": (C.c_char_p, []),
        "mpcc_build_flags": (C.c_int, []),
        "mpcc_timing_mlp": (C.c_int, [V, C.POINTER(D), IP, C.POINTER(D), IP]),
        "mpcc_timing_sqp": (C.c_int, [V, C.POINTER(D), IP, DP]),
        "mpcc_timing_intervals": (C.c_int, [V, V, C.c_int, C.c_int, DP, DP, IP]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.mpcc_abi_version() != 1:
        raise MpccError("libmpcc_engine ABI version mismatch")
    if L.mpcc_robot_dof() != dof:
        raise MpccError(f"{path} was built for {L.mpcc_robot_dof()} joints, expected {dof}")
    _libs[dof] = L
    return L


def _check(rc, what, dof=7):
    if rc != 0:
        msg = lib(dof).mpcc_last_error().decode(errors="replace")
        raise MpccError(f"{what} failed ({rc}): {msg}")


def _f64(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return a.reshape(shape) if shape is not None else a


def _dp(a):
    return a.ctypes.data_as(DP) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(IP) if a is not None else None


# ------------------------------------------------------------------------------------------------
# Params
# ------------------------------------------------------------------------------------------------
SECTION_KEYS = {  # python/MPCC/MPCC.py:37-43 (valid ParamValue keys)
    "param": ["max_dist_proj", "desired_ee_velocity", "deaccelerate_ratio", "s_trust_region", "tol_sing",
              "tol_selcol", "tol_envcol"],
    "cost": ["qC", "qCNmult", "qL", "qVs", "qOri", "qSing", "rdq", "rddq", "rdVs", "qC_reduction_ratio",
             "qL_increase_ratio", "qOri_reduction_ratio"],
    "bounds": ["q1l", "q2l", "q3l", "q4l", "q5l", "q6l", "q7l", "sl", "vsl", "q1u", "q2u", "q3u", "q4u", "q5u",
               "q6u", "q7u", "su", "vsu", "dq1l", "dq2l", "dq3l", "dq4l", "dq5l", "dq6l", "dq7l", "dVsl", "dq1u",
               "dq2u", "dq3u", "dq4u", "dq5u", "dq6u", "dq7u", "dVsu"] +
              [f"ddq{i}{s}" for s in "lu" for i in range(1, 8)],
    "normalization": ["q1", "q2", "q3", "q4", "q5", "q6", "q7", "s", "vs", "dq1", "dq2", "dq3", "dq4", "dq5", "dq6",
                      "dq7", "dVs"],
    "sqp": ["eps_prim", "eps_dual", "line_search_tau", "line_search_eta", "line_search_rho", "max_iter",
            "line_search_max_iter", "do_SOC", "use_BFGS"],
}


def section_keys(dof=7):
    """Valid ParamValue keys per section for a robot (the mobile base adds xb, yb, thb and their rates)."""
    if dof == 7:
        return SECTION_KEYS
    base = ["xb", "yb", "thb"]
    k = {s: list(v) for s, v in SECTION_KEYS.items()}
    k["bounds"] += [f"{n}{s}" for n in base for s in "lu"] + [f"d{n}{s}" for n in base for s in "lu"] + \
        [f"dd{n}{s}" for n in base for s in "lu"]
    k["normalization"] += base + [f"d{n}" for n in base]
    return k


def load_params(N=20, paths=None, merged=None, overrides=None, ctor_semantics=True, Ts=None, dof=7):
    """Params/*.json + ParamValue overrides -> mpcc_params of the robot's library (C++ loader, host only).

    paths: dict with PathToJson keys (param_path, cost_path, bounds_path, normalization_path, sqp_path)
    overrides: {"param": {...}, "cost": {...}, ...} as the reference's ParamValue (types.h:72-79).
    merged defaults to the robot's parameter file (default_params.json / mobile_params.json) when no
    per-section paths are given."""
    if merged is None and not paths:
        merged = DEFAULT_PARAMS if dof == 7 else MOBILE_PARAMS
    keys = section_keys(dof)
    p = MpccJsonPaths()
    keep = []
    for k in ["param_path", "cost_path", "bounds_path", "normalization_path", "sqp_path"]:
        v = (paths or {}).get(k)
        if v is not None:
            b = v.encode()
            keep.append(b)
            setattr(p, k, b)
    if merged:
        p.merged_path = merged.encode()
    ov = []
    for sec, kv in (overrides or {}).items():
        if sec not in keys:
            raise ValueError(f"unknown parameter section {sec!r}; valid: {list(keys)}")
        for k, v in kv.items():
            if k not in keys[sec]:
                raise ValueError(f"keys for {sec} must be a subset of {keys[sec]}, got {k!r}")
            ov.append((sec.encode(), k.encode(), float(v)))
    arr = (MpccOverride * max(1, len(ov)))()
    for i, (s, k, v) in enumerate(ov):
        arr[i].section, arr[i].key, arr[i].value = s, k, v
    out = PARAMS_STRUCT[dof]()
    _check(lib(dof).mpcc_params_load_json(C.byref(p), arr, len(ov), int(bool(ctor_semantics)), int(N), C.byref(out)),
           "mpcc_params_load_json", dof)
    if Ts is not None:
        out.Ts = float(Ts)
    return out


def load_default_track():
    """Default way-points (reference Params/track.json): X, Y, Z arrays and quaternions (x,y,z,w)."""
    import json
    with open(DEFAULT_TRACK) as f:
        pts = np.array(json.load(f)["points"], dtype=np.float64)
    return pts[:, 0], pts[:, 1], pts[:, 2], pts[:, 3:7]


def quat_to_rot(q):
    """Eigen Quaterniond(x,y,z,w).normalized().toRotationMatrix() (track.cpp:45-53), vectorized."""
    q = np.asarray(q, dtype=np.float64)
    n = np.sqrt((q * q).sum(-1, keepdims=True))
    x, y, z, w = np.moveaxis(q / n, -1, 0)
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    R = np.stack([1 - (tyy + tzz), txy - twz, txz + twy,
                  txy + twz, 1 - (txx + tzz), tyz - twx,
                  txz - twy, tyz + twx, 1 - (txx + tyy)], -1)
    return R.reshape(q.shape[:-1] + (3, 3))


def track_from_points(X, Y, Z, quats, init_position):
    """Track::getTrack(init_position) (track.cpp:56-66): offset the way-points to the EE start."""
    X = np.asarray(X) - X[0] + init_position[0]
    Y = np.asarray(Y) - Y[0] + init_position[1]
    Z = np.asarray(Z) - Z[0] + init_position[2]
    return X, Y, Z, quat_to_rot(quats)


def build_track_host(X, Y, Z, R):
    """Host-only arc-length spline construction; returns (s, X, Y, Z, R, length)."""
    X, Y, Z = _f64(X), _f64(Y), _f64(Z)
    R = _f64(R).reshape(-1, 9)
    out = [np.zeros(100) for _ in range(4)] + [np.zeros(900), np.zeros(1)]
    _check(lib().mpcc_track_build_host(len(X), _dp(X), _dp(Y), _dp(Z), _dp(R), *[_dp(a) for a in out]),
           "mpcc_track_build_host")
    s, Xo, Yo, Zo, Ro, L = out
    return s, Xo, Yo, Zo, Ro.reshape(100, 3, 3), float(L[0])


def eval_track_host(X, Y, Z, R, s):
    """ArcLengthSpline queries on the host spline of the way-points (mpcc_track_eval_host): pos, d1, d2
    [M, 3], R [M, 3, 3], dR [M, 3] at the arc lengths s."""
    X, Y, Z = _f64(X), _f64(Y), _f64(Z)
    R = _f64(R).reshape(-1, 9)
    s = _f64(s).reshape(-1)
    M = len(s)
    pos, d1, d2, Rq, dR = np.zeros((M, 3)), np.zeros((M, 3)), np.zeros((M, 3)), np.zeros((M, 9)), np.zeros((M, 3))
    _check(lib().mpcc_track_eval_host(len(X), _dp(X), _dp(Y), _dp(Z), _dp(R), M, _dp(s), _dp(pos), _dp(d1), _dp(d2),
                                      _dp(Rq), _dp(dR)), "mpcc_track_eval_host")
    return pos, d1, d2, Rq.reshape(M, 3, 3), dR


def cubic_spline_host(x, y, xq, regular):
    """CubicSpline fit + (value, d1, d2) at xq [M] -> [M, 3] (mpcc_cubic_spline_host)."""
    x, y, xq = _f64(x), _f64(y), _f64(xq).reshape(-1)
    out = np.zeros((len(xq), 3))
    _check(lib().mpcc_cubic_spline_host(len(x), _dp(x), _dp(y), int(bool(regular)), len(xq), _dp(xq), _dp(out)),
           "mpcc_cubic_spline_host")
    return out


def rot_spline_host(x, R, xq, regular):
    """CubicSplineRot fit + (R [M, 3, 3], dR [M, 3]) at xq (mpcc_rot_spline_host)."""
    x, R, xq = _f64(x), _f64(R).reshape(-1, 9), _f64(xq).reshape(-1)
    Rq, dR = np.zeros((len(xq), 9)), np.zeros((len(xq), 3))
    _check(lib().mpcc_rot_spline_host(len(x), _dp(x), _dp(R), int(bool(regular)), len(xq), _dp(xq), _dp(Rq), _dp(dR)),
           "mpcc_rot_spline_host")
    return Rq.reshape(-1, 3, 3), dR


# ------------------------------------------------------------------------------------------------
# Engine
# ------------------------------------------------------------------------------------------------
class Engine:
    """B independent MPCC controllers on one MI355X (one runMPC_ per instance per solve call)."""

    def __init__(self, params: MpccParams, max_batch: int, device: int = 0, nn_dir: str = NN_DIR,
                 constraint_mask: int = -1, faithful_dead_trials: bool = False):
        self.dof = getattr(type(params), "_dof", 7)  # the robot of the params struct picks the library
        self.NX, self.NU, self.NXU, self.REC = dims(self.dof)
        self.L = lib(self.dof)
        cfg = MpccConfig(int(params.N), float(params.Ts), int(max_batch), int(device), int(constraint_mask),
                         int(bool(faithful_dead_trials)))
        h = C.c_void_p()
        _check(self.L.mpcc_create(C.byref(cfg), C.byref(params), nn_dir.encode() if nn_dir else None, C.byref(h)),
               "mpcc_create", self.dof)
        self.h = h
        self.N = int(params.N)
        self.max_batch = int(max_batch)
        self.device = int(device)
        if self.L.mpcc_build_flags() & BUILD_BOUNDS_CHECK:
            LIVE_CHECKED.add(self)

    def close(self):
        if getattr(self, "h", None):
            self.L.mpcc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        _check(rc, what, self.dof)

    @property
    def params(self):
        p = PARAMS_STRUCT[self.dof]()
        self._check(self.L.mpcc_get_params(self.h, C.byref(p)), "mpcc_get_params")
        return p

    def set_params(self, params: MpccParams):
        self._check(self.L.mpcc_set_params(self.h, C.byref(params)), "mpcc_set_params")

    def set_track(self, X, Y, Z, R):
        X, Y, Z = _f64(X), _f64(Y), _f64(Z)
        R = _f64(R).reshape(-1, 9)
        self._check(self.L.mpcc_set_track(self.h, len(X), _dp(X), _dp(Y), _dp(Z), _dp(R)), "mpcc_set_track")

    def set_tracks(self, X, Y, Z, R):
        """One track per instance (mpcc_set_tracks): X, Y, Z [B, n], R [B, n, 3, 3]."""
        X, Y, Z = _f64(X), _f64(Y), _f64(Z)
        B, n = X.shape
        R = _f64(R).reshape(B, n, 9)
        self._check(self.L.mpcc_set_tracks(self.h, B, n, _dp(X), _dp(Y), _dp(Z), _dp(R)), "mpcc_set_tracks")

    def set_track_path(self, s, X, Y, Z, R):
        """SolverInterface::setTrack(ArcLengthSpline): from getPathData() (100 regular points)."""
        s, X, Y, Z = _f64(s), _f64(X), _f64(Y), _f64(Z)
        R = _f64(R).reshape(-1, 9)
        self._check(self.L.mpcc_set_track_path(self.h, len(s), _dp(s), _dp(X), _dp(Y), _dp(Z), _dp(R)),
               "mpcc_set_track_path")

    def track_length(self):
        return self.L.mpcc_track_length(self.h)

    def track_path(self):
        s, X, Y, Z, R = np.zeros(100), np.zeros(100), np.zeros(100), np.zeros(100), np.zeros(900)
        self._check(self.L.mpcc_get_track_path(self.h, _dp(s), _dp(X), _dp(Y), _dp(Z), _dp(R)), "mpcc_get_track_path")
        return s, X, Y, Z, R.reshape(100, 3, 3)

    def set_warmstart(self, guess, valid, fails):
        B = guess.shape[0]
        g = _f64(guess, (B, self.N + 1, self.NXU))
        v = np.ascontiguousarray(valid, dtype=np.int32)
        f = np.ascontiguousarray(fails, dtype=np.int32)
        self._check(self.L.mpcc_set_warmstart(self.h, B, _dp(g), _ip(v), _ip(f)), "mpcc_set_warmstart")

    def get_warmstart(self, B):
        g = np.zeros((B, self.N + 1, self.NXU))
        v = np.zeros(B, np.int32)
        f = np.zeros(B, np.int32)
        self._check(self.L.mpcc_get_warmstart(self.h, B, _dp(g), _ip(v), _ip(f)), "mpcc_get_warmstart")
        return g, v, f

    def reset_warmstart(self, B, mask=None):
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
        self._check(self.L.mpcc_reset_warmstart(self.h, B, m.ctypes.data_as(C.POINTER(C.c_uint8)) if m is not None else None),
               "mpcc_reset_warmstart")

    def solve(self, x0, u0, obs, timing=False):
        """Batched runMPC_ on host arrays.  x0 [B,NX] is updated in place (s, vs), as the reference
        mutates its State argument.  Returns dict(u0, horizon, status, ok[, timing])."""
        B = x0.shape[0]
        assert x0.dtype == np.float64 and x0.flags.c_contiguous and x0.shape == (B, self.NX)
        u0 = _f64(u0, (B, self.NU))
        obs = _f64(obs, (B, 4))
        u_out = np.zeros((B, self.NU))
        hor = np.zeros((B, self.N + 1, self.NXU))
        st = np.zeros(B, np.int32)
        ok = np.zeros(B, np.int32)
        tm = MpccTiming()
        self._check(self.L.mpcc_solve(self.h, B, _dp(x0), _dp(u0), _dp(obs), _dp(u_out), _dp(hor), _ip(st), _ip(ok),
                                 C.byref(tm) if timing else None), "mpcc_solve")
        out = dict(u0=u_out, horizon=hor, status=st, ok=ok)
        if timing:
            out["timing"] = tm.as_dict()
        return out

    def closed_loop(self, x0, u0, obs, steps, graph=True):
        """main.cpp:100-114 on the device for B instances (mpcc_closed_loop).  Returns dict(x [steps+1,B,9],
        u [steps,B,8], status [steps,B] (-1 after an instance stopped), x_final, u_final)."""
        B = x0.shape[0]
        x = _f64(x0, (B, self.NX)).copy()
        u = _f64(u0, (B, self.NU)).copy()
        obs = _f64(obs, (B, 4))
        xt = np.zeros((steps + 1, B, self.NX)); ut = np.zeros((steps, B, self.NU)); stt = np.zeros((steps, B), np.int32)
        self._check(self.L.mpcc_closed_loop(self.h, B, int(steps), _dp(x), _dp(u), _dp(obs), _dp(xt), _dp(ut), _ip(stt),
                                       int(bool(graph))), "mpcc_closed_loop")
        return dict(x=xt, u=ut, status=stt, x_final=x, u_final=u)

    def solve_ocp(self, guess, u_cur, obs):
        """SolverInterface::setInitialGuess/setCurrentInput/setEnvData/solveOCP for B instances
        (solver_interface.h:44-54).  Returns dict(opt_sol [B,N+1,17], status, solved)."""
        B = guess.shape[0]
        guess = _f64(guess, (B, self.N + 1, self.NXU))
        u_cur = _f64(u_cur, (B, self.NU))
        obs = _f64(obs, (B, 4))
        sol = np.zeros((B, self.N + 1, self.NXU))
        st = np.zeros(B, np.int32)
        ok = np.zeros(B, np.int32)
        self._check(self.L.mpcc_solve_ocp(self.h, B, _dp(guess), _dp(u_cur), _dp(obs), _dp(sol), _ip(st), _ip(ok), None),
               "mpcc_solve_ocp")
        return dict(opt_sol=sol, status=st, solved=ok)

    def _dev_ptr(self, t, name, dtype, shape, required=False):
        """data_ptr() of a device tensor after checking what the kernels assume of it: dtype, this
        engine's device, contiguity and (leading) shape.  A wrong tensor would otherwise make the
        kernels read or write out of bounds in HBM."""
        import torch
        if t is None:
            if required:
                raise MpccError(f"{name} is required")
            return None
        if not isinstance(t, torch.Tensor):
            raise MpccError(f"{name}: expected a torch tensor on the device, got {type(t).__name__}")
        if t.dtype != dtype:
            raise MpccError(f"{name}: dtype {t.dtype}, expected {dtype}")
        if t.device.type != "cuda" or t.device.index != self.device:
            raise MpccError(f"{name}: on {t.device}, the engine is on cuda:{self.device}")
        if not t.is_contiguous():
            raise MpccError(f"{name}: not contiguous")
        if tuple(t.shape[:len(shape)]) != tuple(shape) or t.numel() != int(np.prod(shape)):
            raise MpccError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
        return C.c_void_p(t.data_ptr())

    def _stream_handle(self, stream):
        """The torch stream the call is ordered on: 'stream', else torch's current stream on the engine's
        device.  torch's default stream has handle 0, which the ABI reads as the engine's stream; that
        stream is a blocking stream, so it is ordered with the default stream's work."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        h = stream.cuda_stream
        return C.c_void_p(h) if h else None

    def solve_device(self, B, x0, u0, obs, u_out=None, horizon=None, status=None, ok=None, stream=None):
        """Batched runMPC_ on device-resident torch tensors (float64 / int32), asynchronous on 'stream'
        (default: torch's current stream)."""
        import torch
        B = int(B)
        if not 1 <= B <= self.max_batch:
            raise MpccError(f"B = {B} outside [1, {self.max_batch}]")
        f64, i32 = torch.float64, torch.int32
        a = [self._dev_ptr(x0, "x0", f64, (B, self.NX), True), self._dev_ptr(u0, "u0", f64, (B, self.NU), True),
             self._dev_ptr(obs, "obs", f64, (B, 4), True), self._dev_ptr(u_out, "u_out", f64, (B, self.NU)),
             self._dev_ptr(horizon, "horizon", f64, (B, self.N + 1, self.NXU)), self._dev_ptr(status, "status", i32, (B,)),
             self._dev_ptr(ok, "ok", i32, (B,))]
        s = self._stream_handle(stream)
        self._check(self.L.mpcc_solve_device(self.h, B, *a, s), "mpcc_solve_device")

    def set_warmstart_device(self, B, guess, valid, fails, stream=None):
        """Device-to-device warm start of instances [0, B) (float64 guess [B, N+1, NXU], int32 valid/fails)."""
        import torch
        B = int(B)
        if not 0 <= B <= self.max_batch:
            raise MpccError(f"B = {B} outside [0, {self.max_batch}]")
        a = [self._dev_ptr(guess, "guess", torch.float64, (B, self.N + 1, self.NXU)),
             self._dev_ptr(valid, "valid", torch.int32, (B,)), self._dev_ptr(fails, "fails", torch.int32, (B,))]
        s = self._stream_handle(stream)
        self._check(self.L.mpcc_set_warmstart_device(self.h, B, *a, s), "mpcc_set_warmstart_device")

    def timing_begin(self):
        self._check(self.L.mpcc_timing_begin(self.h), "mpcc_timing_begin")

    def timing_end(self):
        t = MpccTiming()
        nc = C.c_int32()
        ni = C.c_int32()
        self._check(self.L.mpcc_timing_end(self.h, C.byref(t), C.byref(nc), C.byref(ni)), "mpcc_timing_end")
        return t.as_dict(), nc.value, ni.value

    def timing_mlp(self):
        """After timing_end: {kernel: (total seconds, launches)} of k_mlp_self / k_mlp_env in that window."""
        ss, se = C.c_double(), C.c_double()
        ns, ne = C.c_int32(), C.c_int32()
        self._check(self.L.mpcc_timing_mlp(self.h, C.byref(ss), C.byref(ns), C.byref(se), C.byref(ne)),
                    "mpcc_timing_mlp")
        return {"k_mlp_self": (ss.value, ns.value), "k_mlp_env": (se.value, ne.value)}

    def timing_sqp(self):
        """After timing_end: (summed launch seconds, launches, phase fractions [set_qp, solve_qp, get_alpha, step]) of
        the fused SQP kernel; the fractions split its span over the ComputeTime fields (0 launches: staged path)."""
        sp = C.c_double()
        n = C.c_int32()
        fr = np.zeros(4)
        self._check(self.L.mpcc_timing_sqp(self.h, C.byref(sp), C.byref(n), _dp(fr)), "mpcc_timing_sqp")
        return sp.value, n.value, fr

    TIMING_KINDS = {"qp": 0, "k_mlp_self": 1, "k_mlp_env": 2}

    def timing_intervals(self, kind="qp", anchor=None, max_n=4096):
        """After timing_end: (start_ms, end_ms) arrays of one kernel's launches in the window ("qp": the QP solve,
        "k_mlp_self", "k_mlp_env"), relative to the first event of `anchor`'s window (default: this engine)."""
        a = (anchor or self).h
        while True:
            s, t = np.zeros(max_n), np.zeros(max_n)
            n = C.c_int32()
            self._check(self.L.mpcc_timing_intervals(self.h, a, self.TIMING_KINDS[kind], int(max_n), _dp(s), _dp(t),
                                                     C.byref(n)), "mpcc_timing_intervals")
            if n.value <= max_n:
                return s[:n.value], t[:n.value]
            max_n = n.value  # more launches than the buffer held (e.g. the staged loop: one per SQP iteration)

    def solve_stats(self, B):
        a, b, c = np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(B, np.int32)
        self._check(self.L.mpcc_get_solve_stats(self.h, int(B), _ip(a), _ip(b), _ip(c)), "mpcc_get_solve_stats")
        return dict(sqp_iter=a, ipm_iters=b, qp_status=c)

    def sim_time_step(self, x, u, ts):
        B = x.shape[0]
        x = _f64(x, (B, self.NX))
        u = _f64(u, (B, self.NU))
        out = np.zeros((B, self.NX))
        self._check(self.L.mpcc_sim_time_step(self.h, B, _dp(x), _dp(u), float(ts), _dp(out)), "mpcc_sim_time_step")
        return out

    # ---- stage-level entry points (parity tests)
    def robot_records(self, q, obs):
        q = _f64(q).reshape(-1, self.dof)
        M = q.shape[0]
        obs = _f64(obs, (M, 4))
        rec = np.zeros((M, self.REC))
        self._check(self.L.mpcc_debug_robot_records(self.h, M, _dp(q), _dp(obs), _dp(rec)), "mpcc_debug_robot_records")
        return rec

    def spline_eval(self, s):
        s = _f64(s).reshape(-1)
        M = s.shape[0]
        pos, d1, d2, R, dR = np.zeros((M, 3)), np.zeros((M, 3)), np.zeros((M, 3)), np.zeros((M, 9)), np.zeros((M, 3))
        self._check(self.L.mpcc_debug_spline(self.h, M, _dp(s), _dp(pos), _dp(d1), _dp(d2), _dp(R), _dp(dR)),
               "mpcc_debug_spline")
        return pos, d1, d2, R.reshape(M, 3, 3), dR

    def stage_cost(self, x, u, rec, k):
        nx, nu = self.NX, self.NU
        x = _f64(x).reshape(-1, nx)
        M = x.shape[0]
        u = _f64(u, (M, nu))
        rec = _f64(rec, (M, self.REC))
        k = np.ascontiguousarray(k, dtype=np.int32).reshape(M)
        obj, fx, fu = np.zeros(M), np.zeros((M, nx)), np.zeros((M, nu))
        fxx, fuu = np.zeros((M, nx * nx)), np.zeros((M, nu * nu))
        self._check(self.L.mpcc_debug_stage_cost(self.h, M, _dp(x), _dp(u), _dp(rec), _ip(k), _dp(obj), _dp(fx), _dp(fu),
                                            _dp(fxx), _dp(fuu)), "mpcc_debug_stage_cost")
        return obj, fx, fu, fxx.reshape(M, nx, nx), fuu.reshape(M, nu, nu)

    def solve_qp(self, guess, rec, u_cur):
        B = guess.shape[0]
        g = _f64(guess, (B, self.N + 1, self.NXU))
        r = _f64(rec, (B, self.N + 1, self.REC))
        u = _f64(u_cur, (B, self.NU))
        nv = self.NXU * self.N + self.NX
        step = np.zeros((B, nv))
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        self._check(self.L.mpcc_debug_solve_qp(self.h, B, _dp(g), _dp(r), _dp(u), _dp(step), _ip(st), _ip(it)),
               "mpcc_debug_solve_qp")
        return step, st, it

    def solve_qp_lr(self, guess, rec, u_cur, lr, lrc):
        """One QP with low-rank Hessian terms sum_j lrc_j u_j u_j^T (the damped-BFGS QP form, 32-lane solver):
        lr [nlr, N+1, NXU], lrc [nlr]; the same terms for every instance."""
        B = guess.shape[0]
        g = _f64(guess, (B, self.N + 1, self.NXU))
        r = _f64(rec, (B, self.N + 1, self.REC))
        u = _f64(u_cur, (B, self.NU))
        lr = _f64(lr).reshape(-1, self.N + 1, self.NXU)
        lrc = _f64(lrc).reshape(-1)
        step = np.zeros((B, self.NXU * self.N + self.NX))
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        self._check(self.L.mpcc_debug_solve_qp_lr(self.h, B, _dp(g), _dp(r), _dp(u), int(lr.shape[0]), _dp(lr), _dp(lrc),
                                                  _dp(step), _ip(st), _ip(it)), "mpcc_debug_solve_qp_lr")
        return step, st, it

    def project(self, s_guess, ee):
        """projectOnSpline for M (s_guess, ee) pairs (arc_length_spline.cpp:318-379)."""
        sg = _f64(np.atleast_1d(s_guess))
        M = sg.shape[0]
        e = _f64(ee, (M, 3))
        out = np.zeros(M)
        self._check(self.L.mpcc_debug_project(self.h, M, _dp(sg), _dp(e), _dp(out)), "mpcc_debug_project")
        return out

    def tail_solves(self, reset=True):
        """QP solves finished in tail mode (csrc/ipm_tail.h) since the last reset, over the whole process."""
        v = C.c_longlong()
        self._check(self.L.mpcc_debug_tail_solves(C.byref(v), 1 if reset else 0), "mpcc_debug_tail_solves")
        return int(v.value)

    def order(self, n):
        """k_sqp's instance per 16-lane group slot of the last fused solve (-1: empty; csrc/kernels.hip k_order)."""
        out = np.zeros(n, dtype=np.int32)
        got = self.L.mpcc_debug_order(self.h, out.ctypes.data_as(C.POINTER(C.c_int)), n)
        if got < 0:
            self._check(got, "mpcc_debug_order")
        return out[:got]

    def bounds_flags(self, clear=True):
        """Bounds-checked build (MPCC_BOUNDS_CHECK): OR of the index-violation bits recorded by every kernel since
        the last clear (0 = every computed index in range; bits: csrc/dev_common.h BC_*)."""
        f = C.c_uint32(0)
        self._check(self.L.mpcc_debug_bounds(self.h, C.byref(f), 1 if clear else 0), "mpcc_debug_bounds")
        return int(f.value)

    def workspace(self, B):
        """Interior-point workspace of the last solve, [B, N+1, 816] (Panda; 2048 for the mobile build)."""
        out = np.zeros((B, self.N + 1, 816 if self.dof == 7 else 2048))
        self._check(self.L.mpcc_debug_workspace(self.h, B, _dp(out)), "mpcc_debug_workspace")
        return out

    def trace_enable(self, on=True):
        """Record per-SQP-iteration decisions of the next solves (test instrumentation)."""
        self._check(self.L.mpcc_debug_trace_enable(self.h, 1 if on else 0), "mpcc_debug_trace_enable")

    def trace_get(self, B):
        """[B, 4, 8]: qp status, ipm iters, trial obj, trial vio, accepted, |step|_inf, alpha, alpha*|step|_inf."""
        out = np.zeros((B, 4, 8))
        self._check(self.L.mpcc_debug_trace_get(self.h, B, _dp(out)), "mpcc_debug_trace_get")
        return out
