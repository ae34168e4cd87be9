"""Husky+Panda mobile manipulator (BASELINE configs[3]): the engine built with
MPCC_DOF = 10 (libmpcc_engine_mobile.so) against the oracle built with ORC_DOF = 10 (liboracle_mobile.so).

Parity here is "parity unpinned": the reference defines the base joints (RobotModel::setHusky,
robot_model.cpp:321-352) but never mounts the Panda on them and fixes NX/NU at compile time for the Panda
(config.h:29-38), so no reference output exists for this robot.  The oracle restates the reference's
algorithm for the 10-joint chain (mount, MLP inputs in the arm frame: DESIGN.md §11); both sides share that
definition.  Tolerances are the Panda's: records 1e-10 relative (FD gradient 1e-7), QP
step 1e-8, status exact, optimal inputs 1e-6.
"""
import ctypes as C

import numpy as np
import pytest

import refparams as rp
from helpers import SEED, batch_from_pool, make_oracle, oracle_pool
from helpers import Q0_MOBILE
from test_host_abi import declared_functions

DOF, NX, NU, NXU, REC = 10, 12, 11, 23, 194
OBS = (0.62, 0.28, 0.75, 5.0)  # near the arm's reach from the start pose (EE at ~(0.55, 0, 0.87))


def _mobile_lib(built_lib):
    import os
    return os.path.join(os.path.dirname(built_lib), "libmpcc_engine_mobile.so")


# ---------------------------------------------------------------- CPU: the library and its host entries
def test_mobile_library_exports_and_dims(built_lib):
    L = C.CDLL(_mobile_lib(built_lib))
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    L.mpcc_robot_dof.restype = C.c_int
    assert L.mpcc_robot_dof() == DOF
    import mpcc_manipulator_amd as m
    assert m.lib(7).mpcc_robot_dof() == 7 and m.lib(10).mpcc_robot_dof() == 10


@pytest.mark.parametrize("ctor", [True, False])
def test_mobile_params_loader(built_lib, ctor):
    """The C++ loader of the mobile build reads mobile_params.json with the base joints (xb, yb, thb) first,
    as the Python restatement of the reference's loaders does (tests/refparams.py, dof = 10)."""
    import mpcc_manipulator_amd as m
    ov = {"cost": {"qC": 321.0}, "normalization": {"xb": 2.0, "q1": 3.0}, "bounds": {}}
    p = m.load_params(N=30, overrides=ov, ctor_semantics=ctor, dof=10).as_dict()
    r = rp.resolve(N=30, overrides=ov, ctor_overrides=ctor, dof=10)
    for k, v in r.items():
        if k == "constraint_mask":
            continue
        if isinstance(v, list):
            assert np.array_equal(np.array(p[k], float), np.array(v, float)), k
        else:
            assert float(p[k]) == float(v), (k, p[k], v)
    assert len(p["Tx"]) == NX and len(p["Tu"]) == NU and len(p["lddq"]) == DOF
    with pytest.raises(ValueError):
        m.load_params(N=30, overrides={"bounds": {"xbl": -1.0}}, dof=7)  # base keys exist only for dof 10


# ---------------------------------------------------------------- GPU parity
N30 = 30


@pytest.fixture(scope="module")
def mobile(built_lib, oracle_lib):
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=N30, max_iter=2, mask=7, dof=10, nthreads=16)
    params = m.load_params(N=N30, overrides={"sqp": {"max_iter": 2}}, dof=10)
    eng = m.Engine(params, max_batch=512, constraint_mask=7)
    eng.set_track(*track)
    pool = oracle_pool(o, 40, obs=OBS)
    return m, o, eng, track, pool


def _obstacles(rng, B):
    return np.column_stack([np.full(B, OBS[0]), np.full(B, OBS[1]), rng.uniform(OBS[2] - 0.1, OBS[2] + 0.1, B),
                            np.full(B, OBS[3])])


@pytest.mark.gpu
def test_mobile_robot_records(mobile):
    """FK / Jacobian of the base + arm chain, manipulability and its FD gradient, both MLPs (the env network
    with the arm-frame obstacle and its chain rule onto the base joints)."""
    m, o, eng, track, pool = mobile
    rng = np.random.default_rng(SEED + 100)
    M = 64
    q = Q0_MOBILE + rng.normal(0, 0.3, size=(M, DOF))
    obs = _obstacles(rng, M)
    rec = eng.robot_records(q, obs)
    r_mu, r_dmu, r_sel = 12 + 6 * DOF, 13 + 6 * DOF, 13 + 7 * DOF
    for i in range(M):
        ro = o.robot_record(q[i], obs[i, :3], obs[i, 3])
        assert np.allclose(rec[i, :r_dmu], ro[:r_dmu], rtol=1e-11, atol=1e-13), i   # FK, R, J, mu
        assert np.allclose(rec[i, r_dmu:r_sel], ro[r_dmu:r_sel], rtol=1e-7, atol=1e-9), i  # FD gradient of mu
        assert np.allclose(rec[i, r_sel:], ro[r_sel:], rtol=1e-10, atol=1e-10), i  # MLPs + Jacobians
    # the base columns of the env Jacobian are live (chain rule through the arm-frame obstacle)
    r_denv = 24 + 8 * DOF
    base_cols = rec[:, r_denv:].reshape(M, 9, DOF)[:, :, :3]
    assert np.abs(base_cols).max() > 1e-3


@pytest.mark.gpu
def test_mobile_stage_cost(mobile):
    m, o, eng, track, pool = mobile
    rng = np.random.default_rng(SEED + 101)
    M = 40
    x = np.zeros((M, NX)); u = rng.normal(0, 0.2, (M, NU))
    x[:, :DOF] = Q0_MOBILE + rng.normal(0, 0.1, (M, DOF))
    x[:, DOF] = rng.uniform(0, o.track_length(), M)
    x[:, DOF + 1] = rng.uniform(-0.2, 0.3, M)
    k = rng.integers(0, N30 + 1, M).astype(np.int32)
    recs = np.stack([o.robot_record(x[i, :DOF], OBS[:3], OBS[3]) for i in range(M)])
    obj, fx, fu, fxx, fuu = eng.stage_cost(x, u, recs, k)
    for i in range(M):
        oo, ofx, ofu, ofxx, ofuu, _ = o.stage_cost(x[i], u[i], recs[i], int(k[i]))
        assert abs(obj[i] - oo) <= 1e-10 * max(1.0, abs(oo)), i
        assert np.allclose(fx[i], ofx, rtol=1e-9, atol=1e-9), i
        assert np.allclose(fu[i], ofu, rtol=1e-12, atol=1e-14), i
        assert np.allclose(fxx[i], ofxx, rtol=1e-9, atol=1e-8), i
        assert np.allclose(np.diag(fuu[i]), np.diag(ofuu), rtol=1e-12), i


@pytest.mark.gpu
def test_mobile_qp_step(mobile):
    """One QP of the SQP (the 32-lane interior point of ipm_wide.hip) vs the oracle's solve_struct_ipm."""
    m, o, eng, track, pool = mobile
    rng = np.random.default_rng(SEED + 102)
    B = 24
    T = len(pool["x0"])
    guess = np.zeros((B, N30 + 1, NXU)); recs = np.zeros((B, N30 + 1, REC)); ucur = np.zeros((B, NU))
    for b in range(B):
        t = 3 + (b * 7) % (T - 4)
        g = pool["guess"][t + 1].copy()
        g[:, :DOF] += rng.normal(0, 0.01, (N30 + 1, DOF))
        g[:N30, NX:] += rng.normal(0, 0.05, (N30, NU))
        guess[b] = g
        ucur[b] = pool["u0"][t + 1]
        for k in range(N30 + 1):
            recs[b, k] = o.robot_record(g[k, :DOF], OBS[:3], OBS[3])
    step, st, it = eng.solve_qp(guess, recs, ucur)
    for b in range(B):
        rc, so, ito = o.solve_qp(guess[b], recs[b], ucur[b], mode=0)
        assert st[b] == rc, (b, st[b], rc)
        if rc == 0:
            assert abs(int(it[b]) - int(ito)) <= 1, (b, it[b], ito)
            assert np.max(np.abs(step[b] - so)) < 1e-8, (b, np.max(np.abs(step[b] - so)))


def _run_both(eng, o, x0, u0, obs, guess, valid, fails):
    B = x0.shape[0]
    eng.set_warmstart(guess, valid, fails)
    xg = x0.copy()
    outg = eng.solve(xg, u0, obs)
    gg, vg, fg = eng.get_warmstart(B)
    xo = x0.copy(); go = guess.copy(); vo = valid.copy(); fo = fails.copy()
    outo = o.run_mpc(xo, u0, obs, go, vo, fo)
    return (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo)


@pytest.mark.gpu
def test_mobile_batch_parity(mobile):
    """configs[3] settings (N = 30, the full cost and constraint set, per-instance obstacles) on 512
    instances: status exact, optimal inputs <= 1e-6, x0 update <= 1e-9, controller state exact."""
    m, o, eng, track, pool = mobile
    rng = np.random.default_rng(SEED + 103)
    B = 512
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=_obstacles(rng, B))
    (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo) = _run_both(eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.mean(outo["status"] == 0) > 0.9
    assert np.abs(outg["horizon"][:, :-1, NX:] - outo["horizon"][:, :-1, NX:]).max() <= 1e-6
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    assert np.abs(xg - xo).max() <= 1e-9
    assert np.array_equal(vg, vo) and np.array_equal(fg, fo) and np.array_equal(outg["ok"], outo["ok"])


@pytest.mark.gpu
def test_mobile_closed_loop(mobile):
    """The reference driver loop (main.cpp:100-114) for one controller, 25 steps, engine vs oracle."""
    m, o, eng, track, pool = mobile
    x = np.zeros((1, NX)); x[0, :DOF] = Q0_MOBILE
    u = np.zeros((1, NU)); ob = np.array([OBS])
    eng.reset_warmstart(1)
    go = np.zeros((1, N30 + 1, NXU)); vo = np.zeros(1, np.int32); fo = np.zeros(1, np.int32)
    for step in range(25):
        xg = x.copy(); xo = x.copy()
        outg = eng.solve(xg, u, ob)
        outo = o.run_mpc(xo, u, ob, go, vo, fo)
        assert outg["status"][0] == outo["status"][0], step
        assert np.abs(outg["u0"] - outo["u0"]).max() <= 1e-6, step
        assert np.abs(xg - xo).max() <= 1e-9, step
        u = outo["u0"].copy()
        x[0] = o.sim_time_step(xo[0], u[0], o.params["Ts"])
    xs = eng.sim_time_step(x, u, o.params["Ts"])
    assert np.allclose(xs[0], o.sim_time_step(x[0], u[0], o.params["Ts"]), rtol=0, atol=1e-14)


@pytest.mark.gpu
def test_mobile_config3_full_scale(mobile):
    """configs[3] at full size (B = 32,768, N = 30, full constraint set): (1) instance independence — a
    random subset re-solved alone is bitwise its rows of the full batch; (2) every output finite with a
    valid status; (3) a seeded 32-instance sample matches the oracle (status exact, u <= 1e-6)."""
    m, o, eng_small, track, pool = mobile
    B = 32768
    rng = np.random.default_rng(SEED + 32768)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=_obstacles(rng, B))
    eng = m.Engine(m.load_params(N=N30, overrides={"sqp": {"max_iter": 2}}, dof=10), max_batch=B, constraint_mask=7)
    eng.set_track(*track)
    eng.set_warmstart(guess, valid, fails)
    xf = x0.copy()
    full = eng.solve(xf, u0, obs)
    gf, vf, ff = eng.get_warmstart(B)
    assert np.all(np.isfinite(full["horizon"])) and np.all(np.isfinite(xf))
    assert set(np.unique(full["status"]).tolist()) <= {0, 1, 10, 11}
    assert np.mean(full["status"] == 0) > 0.97, np.bincount(full["status"])  # bench configs[3]: 99.96% SOLVED
    sub = np.sort(rng.choice(B, 128, replace=False))
    eng.set_warmstart(guess[sub], valid[sub], fails[sub])
    xs = x0[sub].copy()
    part = eng.solve(xs, u0[sub], obs[sub])
    gs, vs, fs = eng.get_warmstart(len(sub))
    assert np.array_equal(part["status"], full["status"][sub])
    assert np.array_equal(part["horizon"], full["horizon"][sub]) and np.array_equal(xs, xf[sub])
    assert np.array_equal(gs, gf[sub]) and np.array_equal(vs, vf[sub]) and np.array_equal(fs, ff[sub])
    smp = sub[:32]
    xo = x0[smp].copy(); go = guess[smp].copy(); vo = valid[smp].copy(); fo = fails[smp].copy()
    outo = o.run_mpc(xo, u0[smp], obs[smp], go, vo, fo)
    assert np.array_equal(outo["status"], full["status"][smp])
    assert np.abs(outo["horizon"][:, :-1, NX:] - full["horizon"][smp, :-1, NX:]).max() <= 1e-6
    eng.close()


def test_mobile_mount_is_compiled_in(built_lib, tmp_path):
    """robot.mount of the parameter file must equal the library's compiled mount (MPCC_MOBILE_MOUNT_Z): an edited
    mount is refused instead of silently ignored."""
    import json
    import mpcc_manipulator_amd as m
    with open(m.engine.MOBILE_PARAMS) as f:
        d = json.load(f)
    assert d["robot"]["mount"] == [0.0, 0.0, 0.35]
    m.load_params(N=30, dof=10)  # the shipped file loads
    d["robot"]["mount"] = [0.0, 0.0, 0.40]
    p = tmp_path / "mobile_params_mount.json"
    p.write_text(json.dumps(d))
    with pytest.raises(m.MpccError, match="mount"):
        m.load_params(N=30, merged=str(p), dof=10)
