"""The per-control-step driver and the stage records pinned independently of the oracle (VERDICT r03 next-round
item 4).

tests/golden/sqp_restate.npz holds 64 controllers (N = 20, 2 SQP iterations; 32 with configs[1]'s rows, 32 with
all 11 rows and the main_w_sim.py obstacle; joint noise 0.005 / 0.03 rad, cold starts) whose runMPC_ outputs were
computed by tools/sqp_restate.py: numpy restatements of MPC::runMPC_ (projection, vs update, warm-start shift and
validity, mpc.cpp:54-190), OsqpInterface::solveOCP with its filter line search (osqp_interface.cpp:398-590,
759-833; quirks Q5-Q7) and, in tools/records_restate.py, the RBDL kinematics of setPanda (robot_model.cpp:68-319,
366-450) and both collision networks read from the reference's parameter text files (SelfCollisionModel.cpp:140-250,
EnvCollisionModel.cpp:137-247).  They import neither oracle/ nor the product (tools/make_sqp_fixture.py).

CPU: the oracle's stage records equal the restated ones; the oracle's runMPC_ equals the restated one (status, SQP
iterations, filter decisions and the valid / fail bookkeeping exact, inputs <= 1e-8, x0 <= 1e-12).
GPU: the engine's runMPC_ equals it (status exact, inputs <= 1e-6, the north star's bar).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
FIX = os.path.join(ROOT, "tests", "golden", "sqp_restate.npz")
REC_FIELDS = {"pos": (0, 3), "R": (3, 12), "J": (12, 54), "mu": (54, 55), "dmu": (55, 62), "d_self": (62, 63),
              "dd_self": (63, 70), "obs_r": (70, 71), "d_env": (71, 80), "dd_env": (80, 143)}


@pytest.fixture(scope="module")
def fx():
    f = np.load(FIX, allow_pickle=False)
    return {k: f[k] for k in f.files}


def _inputs(fx, mask):
    p = f"m{mask}_in_"
    return (fx[p + "x0"].copy(), fx[p + "u0"].copy(), fx[p + "obs"].copy(), fx[p + "guess"].copy(),
            fx[p + "valid"].copy(), fx[p + "fails"].copy())


def _oracle(fx, mask):
    from helpers import make_oracle
    o, Po, _ = make_oracle(N=int(fx["N"]), max_iter=2, mask=mask)
    assert float(Po["Ts"]) == float(fx["param_Ts"]) and int(fx["sqp_max_iter"]) == 2
    for k in ("Tx", "Tu", "lx", "ux", "lu", "uu", "lddq", "uddq"):
        assert np.array_equal(np.asarray(Po[k], float), fx["param_" + k]), k
    o.set_track(fx["X"], fx["Y"], fx["Z"], fx["R"].reshape(-1, 3, 3))
    return o


def test_fixture_coverage(fx):
    """Both masks, filter rejections (alpha = tau^5 = 1/32), cold starts, MAX_ITER exits and active collision rows."""
    alphas = np.concatenate([fx["m2_alpha"].ravel(), fx["m7_alpha"].ravel()])
    assert np.sum(np.isclose(alphas, 1 / 32)) >= 5
    assert np.sum(fx["m2_in_valid"] == 0) + np.sum(fx["m7_in_valid"] == 0) >= 2
    assert np.sum(fx["m2_status"] == 1) >= 1  # MAX_ITER_EXCEEDED: the zero guess of Q7
    assert np.all(fx["m2_u0"][fx["m2_status"] != 0] == 0)
    # with the obstacle, some env-collision rows bind: c = -grad^T dq + RBF(d - r) is near its bound 0 at the solution
    assert np.min(fx["m7_recs"][:, :-1, 71:80]) < 20.0


def test_restatement_reproduces(fx):
    """tools/sqp_restate.py computes two stored controllers again (guards the fixture and the restatement)."""
    import qp_restate as qr
    import records_restate as rr
    import sqp_restate as srs
    if not os.path.isdir("/root/reference/cpp/NNmodel"):
        pytest.skip("the reference's network parameter files are not on this machine")
    P = {k[6:]: (float(v) if v.ndim == 0 else v) for k, v in fx.items() if k.startswith("param_")}
    S = {k[4:]: (float(v) if k != "sqp_max_iter" and k != "sqp_ls_max" else int(v)) for k, v in fx.items()
         if k.startswith("sqp_")}
    track = qr.Track(fx["X"], fx["Y"], fx["Z"], fx["R"])
    nets = rr.load_networks("/root/reference")
    x0, u0, obs, guess, valid, fails = _inputs(fx, 2)
    for i in (3, 10):
        x = x0[i].copy()
        r = srs.run_mpc(P, S, track, nets, x, u0[i], obs[i], guess[i], int(valid[i]), int(fails[i]), int(fx["N"]), 2)
        assert r["status"] == fx["m2_status"][i] and r["sqp_iter"] == fx["m2_sqp_iter"][i]
        assert np.abs(r["horizon"] - fx["m2_horizon"][i]).max() <= 1e-10
        assert np.abs(r["recs"] - fx["m2_recs"][i]).max() <= 1e-12


@pytest.mark.parametrize("mask", [2, 7])
def test_oracle_records_match_restatement(fx, oracle_lib, mask):
    """RobotData of every stage of the shifted guess (the joints the restatement evaluated, stage_q): FK, J, mu and
    both networks within max(1e-10 relative, 1e-12 absolute); the central-difference gradient of mu <= 1e-9 absolute
    (it divides rounding by 2e-4)."""
    o = _oracle(fx, mask)
    recs, qs, obs = fx[f"m{mask}_recs"], fx[f"m{mask}_stage_q"], fx[f"m{mask}_in_obs"]
    B, S = recs.shape[:2]
    worst = {k: 0.0 for k in REC_FIELDS}
    for b in range(B):
        for k in range(S):
            r = o.robot_record(qs[b, k], tuple(obs[b, :3]), float(obs[b, 3]))
            for name, (lo, hi) in REC_FIELDS.items():
                if mask == 2 and name in ("d_self", "dd_self", "d_env", "dd_env"):
                    continue  # configs[1]'s mask: the engine and the oracle skip both networks
                a, e = r[lo:hi], recs[b, k, lo:hi]
                # excess over the bar: max(1e-10 |e|, 1e-12), 1e-9 absolute for the FD gradient
                bar = np.full(e.shape, 1e-9) if name == "dmu" else np.maximum(1e-10 * np.abs(e), 1e-12)
                worst[name] = max(worst[name], float((np.abs(a - e) / bar).max()))
    o.close()
    for name, err in worst.items():
        assert err <= 1.0, (name, err)


@pytest.mark.parametrize("mask", [2, 7])
def test_oracle_run_mpc_matches_restatement(fx, oracle_lib, mask):
    o = _oracle(fx, mask)
    x0, u0, obs, guess, valid, fails = _inputs(fx, mask)
    out = o.run_mpc(x0, u0, obs, guess, valid, fails, trace=True)
    p = f"m{mask}_"
    assert np.array_equal(out["status"], fx[p + "status"])
    assert np.array_equal(out["sqp_iters"], fx[p + "sqp_iter"])
    assert np.array_equal(valid, fx[p + "valid_out"]) and np.array_equal(fails, fx[p + "fails_out"])
    assert np.array_equal(out["ok"].astype(bool), fx[p + "ok"].astype(bool))
    assert np.abs(x0 - fx[p + "x0_out"]).max() <= 1e-12
    # the filter's decisions: alpha of every SQP iteration run
    ran = ~np.isnan(fx[p + "alpha"])
    assert np.array_equal(out["trace"][:, :2, 6][ran], fx[p + "alpha"][ran])
    assert np.abs(out["horizon"][:, :-1, 9:] - fx[p + "horizon"][:, :-1, 9:]).max() <= 1e-8
    assert np.abs(out["horizon"][:, :, :9] - fx[p + "horizon"][:, :, :9]).max() <= 1e-8
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mask", [2, 7])
def test_engine_run_mpc_matches_restatement(fx, built_lib, mask):
    """The HIP engine's runMPC_ (k_prepare, k_records, the MLP kernels, k_setqp, k_sqp, k_finalize) on the
    fixture's controllers: status and bookkeeping exact, optimal inputs <= 1e-6 (north star)."""
    import mpcc_manipulator_amd as m
    x0, u0, obs, guess, valid, fails = _inputs(fx, mask)
    B = x0.shape[0]
    eng = m.Engine(m.load_params(N=int(fx["N"]), overrides={"sqp": {"max_iter": 2}}), max_batch=B, constraint_mask=mask)
    eng.set_track(fx["X"], fx["Y"], fx["Z"], fx["R"].reshape(-1, 3, 3))
    eng.set_warmstart(guess, valid, fails)
    out = eng.solve(x0, u0, obs)
    g, v, f = eng.get_warmstart(B)
    eng.close()
    p = f"m{mask}_"
    assert np.array_equal(out["status"], fx[p + "status"])
    assert np.array_equal(v, fx[p + "valid_out"]) and np.array_equal(f, fx[p + "fails_out"])
    assert np.abs(x0 - fx[p + "x0_out"]).max() <= 1e-9
    assert np.abs(out["horizon"][:, :-1, 9:] - fx[p + "horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(out["u0"] - fx[p + "u0"]).max() <= 1e-6
