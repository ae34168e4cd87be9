"""The filter line search's rejection branch (osqp_interface.cpp:759-808, quirk Q5), exercised and asserted.

filterLineSearch never resets is_alpha_accepted, so once the trial at alpha = 1 is rejected by the filter the
remaining ls_max - 1 halvings run without a test and the step is taken with alpha = tau^ls_max = 0.5^5 = 1/32
(osqp_interface.cpp:767-806).  The benchmark batches almost never reach that branch (their instances solve in one
SQP iteration), so these batches use larger joint noise on the closed-loop pool (q + N(0, 0.02 rad)): about one
instance in ten takes it.  The oracle's per-iteration trace names the rejected instances; the engine's trace
(mpcc_debug_trace_*) must show the same alpha, acceptance and trial filter values for every instance.
"""
import numpy as np
import pytest

from helpers import SEED, batch_from_pool, make_oracle, oracle_pool

QNOISE = 0.02
OBS7 = (0.48, 0.218, 0.521, 5.0)


def _batch(mask, B):
    obs = (3.0, 3.0, 3.0, 0.0) if mask == 2 else OBS7
    o, P, track = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16)
    pool = oracle_pool(o, 100, obs=obs)
    rng = np.random.default_rng(SEED + 77 + mask)
    x0, u0, ob, g, v, f = batch_from_pool(pool, B, rng, qnoise=QNOISE, obs=np.tile(obs, (B, 1)))
    return o, track, (x0, u0, ob, g, v, f)


def _rejected(trace):
    return np.any(trace[:, :, 6] == 1.0 / 32.0, axis=1)


@pytest.mark.parametrize("mask", [2, 7])
def test_oracle_batch_takes_the_rejection_branch(oracle_lib, mask):
    """The oracle trace: alpha is 1 or exactly tau^5 = 1/32 (never an intermediate halving, Q5); a rejection
    batch has dozens of instances on the 1/32 branch, and they still end SOLVED or MAX_ITER_EXCEEDED."""
    o, track, (x0, u0, ob, g, v, f) = _batch(mask, 512)
    out = o.run_mpc(x0.copy(), u0, ob, g.copy(), v.copy(), f.copy(), trace=True)
    tr = out["trace"]
    ran = tr[:, :, 4] != 0  # accepted flag column is 1 or -1 for an iteration that ran (0 otherwise)
    alphas = np.unique(tr[:, :, 6][tr[:, :, 6] != 0])
    assert set(alphas.tolist()) <= {1.0, 1.0 / 32.0}, alphas
    rej = _rejected(tr)
    assert rej.sum() >= 25, int(rej.sum())
    assert set(np.unique(out["status"][rej]).tolist()) <= {0, 1}
    assert ran.any()
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mask", [2, 7])
def test_engine_rejection_branch_matches_oracle(built_lib, oracle_lib, mask):
    """Engine vs oracle on the rejection batch: per instance and SQP iteration the same QP status, filter
    decision and alpha (bit-exact), trial objective / violation at alpha = 1 within 1e-9 relative; then the
    usual outputs (status exact, u <= 1e-6) for the rejected instances and the whole batch."""
    import mpcc_manipulator_amd as m
    B = 512
    o, track, (x0, u0, ob, g, v, f) = _batch(mask, B)
    out_o = o.run_mpc(x0.copy(), u0, ob, g.copy(), v.copy(), f.copy(), trace=True)
    tro = out_o["trace"]
    rej = _rejected(tro)
    assert rej.sum() >= 25
    eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    eng.set_warmstart(g, v, f)
    eng.trace_enable(True)
    out_g = eng.solve(x0.copy(), u0, ob)
    trg = eng.trace_get(B)
    eng.trace_enable(False)
    assert np.array_equal(_rejected(trg), rej)
    for col in (0, 4, 6):  # qp status, accepted, alpha
        assert np.array_equal(trg[:, :, col], tro[:, :, col]), col
    for col in (2, 3):  # trial objective and violation at alpha = 1 (the filter's inputs)
        a, b = trg[:, :, col], tro[:, :, col]
        assert np.all(np.abs(a - b) <= 1e-9 * np.maximum(1.0, np.abs(b))), col
    assert np.array_equal(out_g["status"], out_o["status"])
    assert np.abs(out_g["u0"][rej] - out_o["u0"][rej]).max() <= 1e-6
    assert np.abs(out_g["horizon"][:, :-1, 9:] - out_o["horizon"][:, :-1, 9:]).max() <= 1e-6
    eng.close()
    o.close()
