"""Python controller API mirroring the reference's python/MPCC/MPCC.py (class MPCC) on top of the
HIP engine, plus BatchMPCC for B independent controllers per call.

Reference surface (python/MPCC/MPCC.py:10-114, cpp/src/MPCC_wrapper.cpp:116-417):
    MPCC().setParam(param_value: dict)                      MPCC.py:33-55
    MPCC().setTrack(state)                                  MPCC.py:57-73
    MPCC().getSplinePath() -> (position, rotation, s)       MPCC.py:75-81
    MPCC().getRefPose(s) -> (position, rotation)            MPCC.py:83-85
    MPCC().getContourError(s, ee_posi) -> float             MPCC.py:87-89
    MPCC().runMPC(state, input, obs_position, obs_radius)
        -> (status, updated_state, u0, horizon, compute_time)  MPCC.py:92-114
"""
import json

import numpy as np

from .engine import (DEFAULT_PARAMS, NN_DIR, PANDA_DOF, PANDA_NUM_LINKS, SECTION_KEYS, Engine, NX, NU, load_default_track,
                     load_params, quat_to_rot, track_from_points)


def load_track_file(path):
    """Way-points from a track JSON: the reference's layout (X, Y, Z, quat_X..quat_W; track.cpp:19-54)
    or this repo's points layout."""
    with open(path) as f:
        t = json.load(f)
    if "points" in t:
        pts = np.asarray(t["points"], dtype=np.float64)
        return pts[:, 0], pts[:, 1], pts[:, 2], pts[:, 3:7]
    q = np.stack([t["quat_X"], t["quat_Y"], t["quat_Z"], t["quat_W"]], -1)
    return np.asarray(t["X"], float), np.asarray(t["Y"], float), np.asarray(t["Z"], float), q


class BatchMPCC:
    """B independent MPC controllers (mpc.h:58-128 state per instance) solved together on one GPU."""

    def __init__(self, batch, N=20, param_value=None, paths=None, merged=DEFAULT_PARAMS, device=0, constraint_mask=7,
                 max_iter=None, nn_dir=NN_DIR, faithful_dead_trials=False):
        ov = {k: dict(v) for k, v in (param_value or {}).items()}
        if max_iter is not None:
            ov.setdefault("sqp", {})["max_iter"] = max_iter
        self._paths, self._merged, self._ov = paths, merged, ov
        self.params = load_params(N, paths=paths, merged=merged, overrides=ov, ctor_semantics=True)
        self.params.constraint_mask = constraint_mask
        self.engine = Engine(self.params, max_batch=batch, device=device, nn_dir=nn_dir,
                             constraint_mask=constraint_mask, faithful_dead_trials=faithful_dead_trials)
        self.batch = batch
        self.N = N
        self.Ts = self.params.Ts
        self.track_set = False

    def setParam(self, param_value: dict):
        """MPC::setParam (mpc.cpp:204-209): Cost/Constraints/Bounds/MPC params refresh; normalization,
        SQP and the track's projection distance keep their construction values."""
        for key, value in param_value.items():
            if key not in SECTION_KEYS:
                raise AssertionError(f"List of Parameters must be a subset of {list(SECTION_KEYS)}, but got {key}")
            bad = set(value) - set(SECTION_KEYS[key])
            if bad:
                raise AssertionError(f"Keys for {key} must be a subset of {SECTION_KEYS[key]}, but got {sorted(bad)}")
        p = load_params(self.N, paths=self._paths, merged=self._merged, overrides=param_value, ctor_semantics=False)
        p.Ts = self.params.Ts
        p.constraint_mask = self.params.constraint_mask
        p.proj_max_dist = self.params.proj_max_dist          # ArcLengthSpline::param_ is not refreshed
        for name in ["Tx", "Tu"]:                             # NormalizationParam not refreshed
            setattr(p, name, getattr(self.params, name))
        for name in ["eps_prim", "eps_dual", "line_search_tau", "line_search_eta", "line_search_rho", "max_iter",
                     "line_search_max_iter", "do_SOC", "use_BFGS"]:  # SQPParam not refreshed
            setattr(p, name, getattr(self.params, name))
        self.engine.set_params(p)
        self.params = p

    def setTrackPoints(self, X, Y, Z, R):
        """MPC::setTrack(X, Y, Z, R) (mpc.cpp:192-197)."""
        self.engine.set_track(X, Y, Z, R)
        self.track_set = True

    def getTrackLength(self):
        return self.engine.track_length()

    def run(self, x0, u0, obs=None, timing=False):
        assert self.track_set, "Set Track first!"
        B = x0.shape[0]
        if obs is None:
            obs = np.tile(np.array([3.0, 3.0, 3.0, 0.0]), (B, 1))  # runMPC dummy obstacle (mpc.cpp:97-99)
        return self.engine.solve(x0, u0, obs, timing=timing)


class MPCC:
    """Single-controller API with the reference Python class's method names and return values."""

    def __init__(self, N=20, param_value=None, paths=None, merged=DEFAULT_PARAMS, track_path=None, device=0,
                 constraint_mask=7, max_iter=None, nn_dir=NN_DIR):
        self._b = BatchMPCC(1, N=N, param_value=param_value, paths=paths, merged=merged, device=device,
                            constraint_mask=constraint_mask, max_iter=max_iter, nn_dir=nn_dir)
        self.engine = self._b.engine
        self.Ts = self._b.Ts
        self.pred_horizon = N
        self.robot_dof = PANDA_DOF
        self.num_links = PANDA_NUM_LINKS
        self.track_path = track_path
        self.track_set = False

    def getEEPosition(self, q):
        rec = self.engine.robot_records(np.asarray(q, float)[:7], np.array([[3.0, 3.0, 3.0, 0.0]]))
        return rec[0, 0:3].copy()

    def setParam(self, param_value: dict) -> None:
        self._b.setParam(param_value)

    def setTrack(self, state: np.ndarray) -> None:
        state = np.asarray(state, dtype=np.float64)
        assert state.size == NX, f"State size {state.size} does not match expected size {NX}"
        self.init_state = state
        ee = self.getEEPosition(state[:PANDA_DOF])
        if self.track_path:
            X, Y, Z, q = load_track_file(self.track_path)
        else:
            X, Y, Z, q = load_default_track()
        X, Y, Z, R = track_from_points(X, Y, Z, q, ee)
        self._b.setTrackPoints(X, Y, Z, R)
        self.spline_path = self.engine.track_path()
        self.track_set = True

    def getSplinePath(self):
        assert self.track_set, "Set Track first!"
        s, X, Y, Z, R = self.spline_path
        return np.stack([X, Y, Z], axis=1), R, s

    def getRefPose(self, path_parameter: float):
        assert self.track_set, "Set Track first!"
        s = self.spline_path[0]
        assert s.min() - 1e-3 <= path_parameter <= s.max() + 1e-3, \
            f"Path parameter must be in [{s.min(), s.max()}] and your input is {path_parameter}"
        pos, _, _, R, _ = self.engine.spline_eval(np.array([path_parameter]))
        return pos[0], R[0]

    def getContourError(self, s: float, ee_posi: np.ndarray) -> float:
        ref, _ = self.getRefPose(s)
        return float(np.linalg.norm(ref - ee_posi))

    def runMPC(self, state: np.ndarray, input: np.ndarray, obs_position=np.array([3, 3, 3]), obs_radius: float = 0):
        assert self.track_set, "Set Track first!"
        assert np.asarray(state).size == NX, f"State size {np.asarray(state).size} does not match expected size {NX}"
        x0 = np.asarray(state, dtype=np.float64).reshape(1, NX).copy()
        u0 = np.asarray(input, dtype=np.float64).reshape(1, NU)
        obs = np.concatenate([np.asarray(obs_position, float).reshape(3), [float(obs_radius)]]).reshape(1, 4)
        out = self.engine.solve(x0, u0, obs, timing=True)
        horizon = [{"state": out["horizon"][0, k, :NX].copy(), "input": out["horizon"][0, k, NX:].copy()}
                   for k in range(self.pred_horizon + 1)]
        t = out["timing"]
        compute_time = {"total": t["total"], "set_qp": t["set_qp"], "solve_qp": t["solve_qp"],
                        "get_alpha": t["get_alpha"], "set_env": t["set_env"]}
        return bool(out["ok"][0]), x0[0].copy(), out["u0"][0].copy(), horizon, compute_time
