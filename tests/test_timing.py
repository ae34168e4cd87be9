"""The reference's ComputeTime fields (osqp_interface.cpp:548-564: set_qp, solve_qp, get_alpha, total) from the
engine: the fused k_sqp span split by its waves' phase clocks (csrc/engine.cpp split_sqp), the staged path's
per-launch spans, and a timing window that mixes both (the staged k_ipm spans must survive the split)."""
import numpy as np
import pytest

from helpers import SEED, batch_from_pool

pytestmark = pytest.mark.gpu


def _pool():
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = np.load(os.path.join(root, "mpcc_manipulator_amd", "data", "bench_pool_n20_mask2.npz"), allow_pickle=False)
    return {k: f[k] for k in f.files}


def _track(m, eng):
    X, Y, Z, q = m.load_default_track()
    ee = eng.robot_records(np.array([[0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4]]), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    return m.track_from_points(X, Y, Z, q, ee)


def _check_fields(t):
    for k in ("set_qp", "solve_qp", "get_alpha", "total"):
        assert t[k] >= 0.0, (k, t)
    assert t["solve_qp"] > 0.0 and t["total"] > 0.0
    assert t["set_qp"] + t["solve_qp"] + t["get_alpha"] <= t["total"] * 1.02 + 1e-5, t


def test_fused_split_sync_and_live(built_lib):
    """One synchronous call with timing and one live window over 3 calls: the three QP-side fields stay within
    total, and the four phase fractions of k_sqp sum to 1."""
    import mpcc_manipulator_amd as m
    B = 512
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=B, constraint_mask=2)
    eng.set_track(*_track(m, eng))
    rng = np.random.default_rng(SEED + 900)
    x0, u0, obs, guess, valid, fails = batch_from_pool(_pool(), B, rng, qnoise=0.005)
    eng.set_warmstart(guess, valid, fails)
    out = eng.solve(x0.copy(), u0, obs, timing=True)
    _check_fields(out["timing"])
    eng.set_warmstart(guess, valid, fails)
    eng.timing_begin()
    for _ in range(3):
        eng.solve(x0.copy(), u0, obs)
    t, ncalls, nipm = eng.timing_end()
    assert ncalls == 3
    _check_fields(t)
    span, n, fr = eng.timing_sqp()
    assert n >= 3 and span > 0.0
    assert np.all(fr >= 0.0) and abs(fr.sum() - 1.0) < 1e-9, fr
    assert t["solve_qp"] == pytest.approx(span * fr[1], rel=1e-9, abs=1e-12)
    eng.close()


def test_mixed_window_keeps_staged_spans(built_lib, monkeypatch):
    """A staged engine (MPCC_STAGED_SQP=1: k_setqp / k_ipm / k_trial per SQP iteration) whose params switch to
    use_BFGS (always the fused 32-lane kernel) inside one timing window: solve_qp is the staged k_ipm spans plus
    the fused span's solve fraction, not the latter alone."""
    import mpcc_manipulator_amd as m
    monkeypatch.setenv("MPCC_STAGED_SQP", "1")
    B = 256
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=B, constraint_mask=2)
    eng.set_track(*_track(m, eng))
    rng = np.random.default_rng(SEED + 901)
    x0, u0, obs, guess, valid, fails = batch_from_pool(_pool(), B, rng, qnoise=0.005)
    # the staged solve alone: its k_ipm spans
    eng.set_warmstart(guess, valid, fails)
    eng.timing_begin()
    eng.solve(x0.copy(), u0, obs)
    ta, _, nipm_a = eng.timing_end()
    assert eng.timing_sqp()[1] == 0 and nipm_a >= 1
    staged = ta["solve_qp"]
    assert staged > 0.0
    # staged, then fused (BFGS) in one window
    eng.set_warmstart(guess, valid, fails)
    eng.timing_begin()
    eng.solve(x0.copy(), u0, obs)
    bfgs = eng.params  # the engine's params (constraint mask 2), with use_BFGS switched on
    bfgs.use_BFGS = 1
    eng.set_params(bfgs)
    eng.set_warmstart(guess, valid, fails)
    eng.solve(x0.copy(), u0, obs)
    tb, ncalls, _ = eng.timing_end()
    span, n, fr = eng.timing_sqp()
    assert ncalls == 2 and n == 1 and span > 0.0
    _check_fields(tb)
    staged_b = tb["solve_qp"] - span * fr[1]
    assert staged_b > 0.25 * staged, (tb, span, fr, staged)
    eng.close()
