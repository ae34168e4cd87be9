"""Damped BFGS (SQPParam use_BFGS; osqp_interface.cpp:437-453 gate, 540-555 multiplier/step bookkeeping,
683-715 BFGSUpdate) on the GPU against the oracle, SURVEY §8(a23)/(f)4, DESIGN.md §4.2.

The engine holds the QP Hessian of SQP iteration >= 1 as the iteration-0 stage Hessians plus 2 low-rank terms
per update and solves with the Woodbury identity around the Riccati recursion (ipm_wide.hip, both robots);
the oracle does the same in its structured mode and is cross-checked against the reference's dense in-place
update in tests/test_oracle.py::test_bfgs_layouts_agree.  Cold-started controllers (valid = 0) take a
second SQP iteration, so every batch below exercises BFGS-updated QPs.  Tolerances as DESIGN.md §5.2:
status exact, optimal inputs <= 1e-6.
"""
import numpy as np
import pytest

from helpers import SEED, batch_from_pool, make_oracle, oracle_pool

pytestmark = pytest.mark.gpu
OV = {"sqp": {"max_iter": 3, "use_BFGS": 1}}


def _run(m, eng, o, x0, u0, obs, guess, valid, fails):
    eng.set_warmstart(guess, valid, fails)
    xg = x0.copy()
    outg = eng.solve(xg, u0, obs)
    stats = eng.solve_stats(x0.shape[0])
    outo = o.run_mpc(x0.copy(), u0, obs, guess.copy(), valid.copy(), fails.copy())
    return xg, outg, stats, outo


def _lowrank_terms(o, rng, nlr):
    """Smooth random low-rank terms for one QP (horizon layout): positive coefficients plus a small negative
    one, the sign pattern of a BFGS update (-Bs Bs^T / sBs + r r^T / sr)."""
    N, nxu = o.N, o.NXU
    lr = rng.normal(0, 1, (nlr, N + 1, nxu))
    lr[:, N, o.NX:] = 0.0  # no u_N
    lr = np.cumsum(lr, axis=1) / np.sqrt(N + 1)
    lrc = np.array([1.0 if j % 2 else -0.02 for j in range(nlr)]) / np.maximum(1.0, (lr ** 2).reshape(nlr, -1).sum(1))
    return lr, lrc


@pytest.mark.parametrize("nlr", [1, 2, 4, 6, 12, 28])
def test_lowrank_qp_step(built_lib, oracle_lib, nlr):
    """One QP with low-rank Hessian terms (the BFGS QP form) on the 32-lane interior point with the Woodbury
    correction, against the oracle's structured (Riccati + Woodbury) and dense-Hessian solves.  nlr > 4: the
    extended path (Woodbury columns and the capacitance LU in memory), up to LRX = 28 terms (max_iter 15)."""
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=7, nthreads=16)
    pool = oracle_pool(o, 40, obs=(0.48, 0.218, 0.521, 5.0))
    eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=16, constraint_mask=7)
    eng.set_track(*track)
    rng = np.random.default_rng(SEED + 730 + nlr)
    B, N = 12, 20
    guess = np.zeros((B, N + 1, 17)); recs = np.zeros((B, N + 1, 143)); ucur = np.zeros((B, 8))
    for b in range(B):
        t = 3 + (b * 3) % 30
        guess[b] = pool["guess"][t + 1]
        ucur[b] = pool["u0"][t + 1]
        for k in range(N + 1):
            recs[b, k] = o.robot_record(guess[b, k, :7], (0.48, 0.218, 0.521), 5.0)
    lr, lrc = _lowrank_terms(o, rng, nlr)
    step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
    for b in range(B):
        rc0, s0, _ = o.solve_qp_lr(guess[b], recs[b], ucur[b], lr, lrc, mode=0)
        rc1, s1, _ = o.solve_qp_lr(guess[b], recs[b], ucur[b], lr, lrc, mode=1)
        assert st[b] == rc0, (b, st[b], rc0)
        if rc0 == 0:
            assert np.abs(step[b] - s0).max() < 1e-8, (b, np.abs(step[b] - s0).max())
            if rc1 == 0:
                assert np.abs(s0 - s1).max() < 1e-7
    base, _, _ = eng.solve_qp(guess, recs, ucur)
    assert np.abs(base - step).max() > 1e-6  # the terms change the solution
    eng.close()


@pytest.mark.parametrize("mask,B", [(2, 512), (7, 256)])
def test_bfgs_batch_parity(built_lib, oracle_lib, mask, B):
    """The reference's own sqp.json with use_BFGS switched on: max_iter 100, eps_prim 0.1 (sqp.json:2-5)."""
    import mpcc_manipulator_amd as m
    OV = {"sqp": {"use_BFGS": 1}}
    o, P, track = make_oracle(N=20, max_iter=None, mask=mask, overrides=OV, nthreads=16)
    assert P["use_BFGS"] == 1 and P["max_iter"] == 100 and P["eps_prim"] == 0.1
    ob = (0.48, 0.218, 0.521, 5.0)
    pool = oracle_pool(o, 120, obs=ob if mask == 7 else (3.0, 3.0, 3.0, 0.0))
    rng = np.random.default_rng(SEED + 700 + mask)
    obs = np.tile(ob, (B, 1)) if mask == 7 else None
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=obs)
    valid[::4] = 0  # a quarter cold-started: BFGS-updated second QPs
    eng = m.Engine(m.load_params(N=20, overrides=OV), max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    xg, outg, stats, outo = _run(m, eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.array_equal(stats["sqp_iter"], outo["sqp_iters"])
    assert np.sum(outo["sqp_iters"] >= 1) >= B // 8
    assert np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    # the update is live: the exact-Hessian SQP (use_BFGS = 0) gives different inputs
    eng2 = m.Engine(m.load_params(N=20), max_batch=B, constraint_mask=mask)
    eng2.set_track(*track)
    eng2.set_warmstart(guess, valid, fails)
    out2 = eng2.solve(x0.copy(), u0, obs)
    assert np.abs(out2["horizon"][:, :-1, 9:] - outg["horizon"][:, :-1, 9:]).max() > 1e-6
    eng.close(); eng2.close()


def test_bfgs_set_params_toggle(built_lib, oracle_lib):
    """mpcc_set_params turning use_BFGS on switches the engine to the BFGS kernel and allocates its state on the
    fly; the result equals that of an engine created with the option."""
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=3, mask=2, overrides=OV, nthreads=16)
    pool = oracle_pool(o, 60)
    B = 64
    rng = np.random.default_rng(SEED + 710)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng)
    valid[::2] = 0
    e1 = m.Engine(m.load_params(N=20, overrides=OV), max_batch=B, constraint_mask=2)
    e2 = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 3}}), max_batch=B, constraint_mask=2)
    p2 = m.load_params(N=20, overrides=OV)
    p2.constraint_mask = 2  # the engine's constraint set (its NN weights were not loaded at create)
    e2.set_params(p2)
    outs = []
    for e in (e1, e2):
        e.set_track(*track)
        e.set_warmstart(guess, valid, fails)
        outs.append(e.solve(x0.copy(), u0, obs))
    assert np.array_equal(outs[0]["status"], outs[1]["status"])
    assert np.array_equal(outs[0]["horizon"], outs[1]["horizon"])
    e1.close(); e2.close()


def test_bfgs_mobile_parity(built_lib, oracle_lib):
    """The same option on the Husky+Panda build (configs[3] settings, N = 30, full constraint set)."""
    import mpcc_manipulator_amd as m
    ov = OV
    o, P, track = make_oracle(N=30, max_iter=3, mask=7, dof=10, overrides=ov, nthreads=16)
    obs_xyz = (0.62, 0.28, 0.75, 5.0)
    pool = oracle_pool(o, 30, obs=obs_xyz)
    B = 96
    rng = np.random.default_rng(SEED + 720)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=np.tile(obs_xyz, (B, 1)))
    valid[::3] = 0
    eng = m.Engine(m.load_params(N=30, overrides=ov, dof=10), max_batch=B, constraint_mask=7)
    eng.set_track(*track)
    xg, outg, stats, outo = _run(m, eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.sum(outo["sqp_iters"] >= 1) >= B // 6
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    eng.close()


def test_bfgs_with_soc_parity(built_lib, oracle_lib):
    """Both SQP variants at once (use_BFGS and do_SOC): the correction QP keeps the BFGS Hessian, and the
    multiplier estimate comes from whichever QP produced the step (osqp_interface.cpp:506-555)."""
    import mpcc_manipulator_amd as m
    ov = {"sqp": {"max_iter": 3, "use_BFGS": 1, "do_SOC": 1}}
    o, P, track = make_oracle(N=20, max_iter=3, mask=2, overrides=ov, nthreads=16)
    assert P["use_BFGS"] == 1 and P["do_SOC"] == 1
    pool = oracle_pool(o, 80)
    B = 256
    rng = np.random.default_rng(SEED + 740)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng)
    valid[::4] = 0
    eng = m.Engine(m.load_params(N=20, overrides=ov), max_batch=B, constraint_mask=2)
    eng.set_track(*track)
    xg, outg, stats, outo = _run(m, eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.array_equal(stats["sqp_iter"], outo["sqp_iters"])
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    eng.close()


@pytest.mark.parametrize("mask,B", [(2, 256), (7, 128)])
def test_bfgs_max_iter_10_parity(built_lib, oracle_lib, mask, B):
    """use_BFGS at max_iter 10: with eps_prim 1e-4 many controllers run 4+ SQP iterations, so
    their QPs hold 6..18 low-rank terms and go through the extended Woodbury path; status, SQP iterations and
    the horizon as in test_bfgs_batch_parity."""
    import mpcc_manipulator_amd as m
    ov = {"sqp": {"max_iter": 10, "use_BFGS": 1, "eps_prim": 1e-4}}
    o, P, track = make_oracle(N=20, max_iter=10, mask=mask, overrides=ov, nthreads=16)
    assert P["use_BFGS"] == 1 and P["max_iter"] == 10
    ob = (0.48, 0.218, 0.521, 5.0)
    pool = oracle_pool(o, 100, obs=ob if mask == 7 else (3.0, 3.0, 3.0, 0.0))
    rng = np.random.default_rng(SEED + 750 + mask)
    obs = np.tile(ob, (B, 1)) if mask == 7 else None
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=obs)
    valid[::4] = 0
    eng = m.Engine(m.load_params(N=20, overrides=ov), max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    xg, outg, stats, outo = _run(m, eng, o, x0, u0, obs, guess, valid, fails)
    assert np.sum(outo["sqp_iters"] >= 4) >= B // 16, np.bincount(outo["sqp_iters"])  # > LRM terms in play
    assert np.array_equal(outg["status"], outo["status"])
    assert np.array_equal(stats["sqp_iter"], outo["sqp_iters"])
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    eng.close()


@pytest.mark.parametrize("mask,B", [(2, 64), (7, 32)])
def test_bfgs_restart_parity(built_lib, oracle_lib, mask, B):
    """More updates than the LRX = 28 low-rank terms hold: with eps_prim 3e-3 BFGS-SQP runs past 15 iterations, and
    the update of iteration 15 (and 29) restarts the quasi-Newton matrix from that iteration's exact Hessian (ipm_wide.hip
    bfgs_pre; the oracle's solve_ocp BFGS_MAX_TERMS).  No error for the batch; status, SQP iterations
    and the horizon as in test_bfgs_batch_parity."""
    import mpcc_manipulator_amd as m
    ov = {"sqp": {"max_iter": 40, "use_BFGS": 1, "eps_prim": 3e-3}}
    o, P, track = make_oracle(N=20, max_iter=40, mask=mask, overrides=ov, nthreads=16)
    ob = (0.48, 0.218, 0.521, 5.0)
    pool = oracle_pool(o, 60, obs=ob if mask == 7 else (3.0, 3.0, 3.0, 0.0))
    rng = np.random.default_rng(SEED + 760 + mask)
    obs = np.tile(ob, (B, 1)) if mask == 7 else None
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=obs, qnoise=0.02)
    valid[::2] = 0
    eng = m.Engine(m.load_params(N=20, overrides=ov), max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    xg, outg, stats, outo = _run(m, eng, o, x0, u0, obs, guess, valid, fails)
    # restarts in play: controllers that converge on a restarted Hessian, others that run into MAX_ITER
    assert np.sum((outo["sqp_iters"] >= 15) & (outo["status"] == 0)) >= B // 8, np.bincount(outo["sqp_iters"])
    assert np.any(outo["status"] == 1)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.array_equal(stats["sqp_iter"], outo["sqp_iters"])
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    eng.close()
