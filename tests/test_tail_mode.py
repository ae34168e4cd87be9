"""Tail mode of the fused interior point (csrc/ipm_tail.h): the last running instance of a wave
takes all four 16-lane groups.  It computes the same expressions in the same order as the normal path, so every
output must be bitwise the MPCC_TAIL=0 engine's; the runs must also have used it.  Reference: the QP solve it
belongs to replaces OSQP inside solveOCP (osqp_interface.cpp:398-590)."""
import os

import numpy as np
import pytest

from helpers import batch_from_pool, make_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x4D504343


def _bench_pool():
    f = np.load(os.path.join(ROOT, "mpcc_manipulator_amd", "data", "bench_pool_n20_mask2.npz"), allow_pickle=False)
    return {k: f[k] for k in f.files}


def _solve(monkeypatch, tail, params, mask, track, batch, staged=False):
    import mpcc_manipulator_amd as m
    monkeypatch.setenv("MPCC_TAIL", "1" if tail else "0")
    if staged:
        monkeypatch.setenv("MPCC_STAGED_SQP", "1")
    x0, u0, obs, guess, valid, fails = batch
    B = x0.shape[0]
    eng = m.Engine(params, max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    eng.tail_solves(reset=True)
    eng.set_warmstart(guess, valid, fails)
    x = x0.copy()
    out = eng.solve(x, u0, obs)
    n_tail = eng.tail_solves(reset=True)
    ws = eng.get_warmstart(B)
    st = eng.solve_stats(B)
    eng.close()
    return x, out, ws, st, n_tail


def _assert_bitwise(a, b):
    xa, oa, wa, sa, _ = a
    xb, ob, wb, sb, _ = b
    assert np.array_equal(xa.view(np.int64), xb.view(np.int64))
    for k in oa:
        assert np.array_equal(np.asarray(oa[k]).view(np.uint8), np.asarray(ob[k]).view(np.uint8)), k
    for u, v in zip(wa, wb):
        assert np.array_equal(np.asarray(u).view(np.uint8), np.asarray(v).view(np.uint8))
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k


OBS = (0.48, 0.218, 0.521, 5.0)  # main_w_sim.py:42-45's obstacle (bench.py --config 1-all-rows)


@pytest.mark.gpu
@pytest.mark.parametrize("mask,B,qnoise,soc,staged", [
    (2, 4096, 0.005, 0, False),   # configs[1], the bench pool and noise
    (2, 1024, 0.02, 0, False),    # filter rejections, restarts
    (2, 512, 0.005, 1, False),    # second-order correction: two QPs per SQP iteration
    (2, 512, 0.005, 0, True),     # staged path (k_ipm)
    (0, 512, 0.005, 0, False),    # no polytopic row
    (3, 512, 0.005, 0, False),    # self collision + singularity: two polytopic rows
    (7, 2048, 0.005, 0, False),   # the reference's default rows (11 poly rows, wide-poly variant), obstacle
    (7, 512, 0.02, 0, False),     # wide-poly with filter rejections and restarts
    (7, 256, 0.005, 1, True),     # wide-poly, staged path with the correction
])
def test_tail_mode_bitwise(built_lib, monkeypatch, mask, B, qnoise, soc, staged):
    import mpcc_manipulator_amd as m
    ov = {"sqp": {"max_iter": 2, "do_SOC": soc}}
    params = m.load_params(N=20, overrides=ov)
    eng = m.Engine(params, max_batch=1, constraint_mask=mask)
    X, Y, Z, q = m.load_default_track()
    ee = eng.robot_records(np.array([[0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4]]), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    eng.close()
    track = m.track_from_points(X, Y, Z, q, ee)
    rng = np.random.default_rng(SEED + 41)
    batch = batch_from_pool(_bench_pool(), B, rng, qnoise=qnoise, obs=np.tile(OBS, (B, 1)) if mask == 7 else None)
    on = _solve(monkeypatch, True, params, mask, track, batch, staged)
    off = _solve(monkeypatch, False, params, mask, track, batch, staged)
    assert off[4] == 0
    assert on[4] > 0, "tail mode was not used"
    _assert_bitwise(on, off)


@pytest.mark.gpu
@pytest.mark.parametrize("mask,B", [(2, 2048), (7, 1024)])
def test_tail_mode_against_oracle(built_lib, oracle_lib, monkeypatch, mask, B):
    """The instances that finished in tail mode (the cold-started ones of the bench pool, two QPs; with the default
    rows the slowest QP of each wave) against the oracle: status exact, inputs <= 1e-6 (north star), x0 update
    <= 1e-9."""
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16)
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    pool = _bench_pool()
    rng = np.random.default_rng(SEED + 43)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, qnoise=0.005,
                                                      obs=np.tile(OBS, (B, 1)) if mask == 7 else None)
    xg, outg, (gg, vg, fg), st, n_tail = _solve(monkeypatch, True, params, mask, track, (x0, u0, obs, guess, valid, fails))
    assert n_tail > 0
    xo, go, vo, fo = x0.copy(), guess.copy(), valid.copy(), fails.copy()
    outo = o.run_mpc(xo, u0, obs, go, vo, fo)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(xg - xo).max() <= 1e-9
    assert np.array_equal(vg, vo) and np.array_equal(fg, fo)
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mask,B,cold_every", [(2, 4096, 64), (0, 512, 8), (3, 512, 8), (2, 512, 1)])
def test_early_solo_bitwise(built_lib, monkeypatch, mask, B, cold_every):
    """Early solo blocks (engine.cpp run_batch): the solo instances' records by a k_records launch over
    them alone, their first QP records inside k_sqp_solo, the other instances' records and QP records by launches
    that skip them.  Every output equals the old launch order's (MPCC_EARLY_SOLO=0), cold_every 1: more cold starts
    than solo blocks.  Reference: mpc.cpp:79-89, the cold-start path these controllers take."""
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=1, constraint_mask=mask)
    X, Y, Z, q = m.load_default_track()
    ee = eng.robot_records(np.array([[0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4]]), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    eng.close()
    track = m.track_from_points(X, Y, Z, q, ee)
    rng = np.random.default_rng(SEED + 44)
    x0, u0, obs, guess, valid, fails = batch_from_pool(_bench_pool(), B, rng, qnoise=0.005)
    valid[::cold_every] = 0
    res = {}
    for early in ("0", "1"):
        monkeypatch.setenv("MPCC_EARLY_SOLO", early)
        eng = m.Engine(params, max_batch=B, constraint_mask=mask)
        eng.set_track(*track)
        eng.set_warmstart(guess, valid, fails)
        x = x0.copy()
        out = eng.solve(x, u0, obs)
        res[early] = (x, out, eng.get_warmstart(B), eng.solve_stats(B), 0)
        eng.close()
    _assert_bitwise(res["1"], res["0"])


@pytest.mark.gpu
@pytest.mark.parametrize("mask,B,cold_every", [(2, 4096, 64), (3, 512, 8), (2, 512, 1), (7, 1024, 16)])
def test_solo_waves_bitwise(built_lib, monkeypatch, mask, B, cold_every):
    """Solo waves and solo blocks (csrc/kernels.hip k_order): k_sqp gives the first 64
    cold-started controllers a wave each (MPCC_SOLO=1) or, in k_sqp_solo, a block of two waves whose second joins the
    tail-mode solves (MPCC_SOLO=2, the default); the instance -> wave map and the number of groups on a tail-mode solve change
    nothing in an instance's arithmetic, so every output equals the MPCC_SOLO=0 engine's.  cold_every 1: every
    controller cold, past the cap."""
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=1, constraint_mask=mask)
    X, Y, Z, q = m.load_default_track()
    ee = eng.robot_records(np.array([[0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4]]), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    eng.close()
    track = m.track_from_points(X, Y, Z, q, ee)
    rng = np.random.default_rng(SEED + 43)
    x0, u0, obs, guess, valid, fails = batch_from_pool(_bench_pool(), B, rng, qnoise=0.005,
                                                      obs=np.tile(OBS, (B, 1)) if mask == 7 else None)
    valid[::cold_every] = 0
    nsl = 4 * ((B + 3) // 4 + 64)  # kernels.h order_slots: the map, then k_prepare's cold flags
    res, orders = {}, {}
    for solo in (2, 1, 0):
        monkeypatch.setenv("MPCC_SOLO", str(solo))
        eng = m.Engine(params, max_batch=B, constraint_mask=mask)
        eng.set_track(*track)
        eng.set_warmstart(guess, valid, fails)
        x = x0.copy()
        out = eng.solve(x, u0, obs)
        res[solo] = (x, out, eng.get_warmstart(B), eng.solve_stats(B), 0)
        orders[solo] = eng.order(nsl + B)
        eng.close()
    _assert_bitwise(res[1], res[0])
    _assert_bitwise(res[2], res[0])
    for solo in (1, 2):
        sl, flags = orders[solo][:nsl].reshape(-1, 4), orders[solo][nsl:]
        cold = np.nonzero(flags)[0]  # k_prepare's cold starts: the host's plus projection resets
        assert set(np.nonzero(valid == 0)[0]) <= set(cold)
        ns = min(len(cold), 64)
        assert np.array_equal(sl[:ns, 0], cold[:ns]) and np.all(sl[:ns, 1:] == -1)  # the first 64 cold starts alone
        used = sl[sl >= 0]
        assert np.array_equal(np.sort(used), np.arange(B))  # every instance exactly once
