"""GPU parity tests: HIP engine (through the C ABI) vs the CPU oracle on the same seeded inputs.

Tolerances: stage records / spline / cost terms <= 1e-10 relative (1e-12 absolute
floor; the manipulability FD gradient divides rounding noise by 2e-4 and gets 1e-9 absolute);
QP steps <= 1e-8; optimal control sequence u_0..u_{N-1} <= 1e-6 absolute (north star);
Status bit-exact, and no instance may take a different discrete branch (projection, warm-start
validity, filter decisions, eps_prim test): the stage kernels follow the oracle's operation order
without FMA contraction, and parity policies P1 (violation noise floor) and P2 (Riccati breakdown at a
converged iterate) are shared by both sides.
"""
import os

import numpy as np
import pytest

from helpers import Q0, SEED, batch_from_pool, make_oracle, max_rel, oracle_pool

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def setup20(built_lib, oracle_lib):
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=7)
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=256, constraint_mask=7)
    eng.set_track(*track)
    pool = oracle_pool(o, 120)
    return m, o, eng, pool


def test_track_tables(setup20):
    m, o, eng, pool = setup20
    s, X, Y, Z, R = eng.track_path()
    so, Xo, Yo, Zo, Ro = o.track_path()
    assert np.array_equal(s, so) and np.array_equal(X, Xo) and np.array_equal(R, Ro)
    assert eng.track_length() == o.track_length()


def test_spline_eval(setup20):
    m, o, eng, pool = setup20
    L = o.track_length()
    sv = np.concatenate([np.linspace(0, L, 301), [0.0, L, L * 0.5, -0.1, L + 0.1]])
    pos, d1, d2, R, dR = eng.spline_eval(sv)
    for i, s in enumerate(sv):
        p, dp, ddp, Ro, dRo = o.spline_eval(s)
        assert np.allclose(pos[i], p, rtol=1e-12, atol=1e-13)
        assert np.allclose(d1[i], dp, rtol=1e-11, atol=1e-12)
        assert np.allclose(d2[i], ddp, rtol=1e-10, atol=1e-10)
        assert np.allclose(R[i], Ro, rtol=1e-12, atol=1e-13)
        assert np.allclose(dR[i], dRo, rtol=1e-11, atol=1e-12)


def test_set_track_path_equivalent(setup20):
    """mpcc_set_track_path (SolverInterface::setTrack(ArcLengthSpline) via getPathData()) reproduces
    the tables of mpcc_set_track on the way-points bit for bit (the reference's final regular fit)."""
    m, o, eng, pool = setup20
    eng2 = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=4, constraint_mask=7)
    eng2.set_track_path(*eng.track_path())
    assert eng2.track_length() == eng.track_length()
    L = eng.track_length()
    sv = np.concatenate([np.linspace(0, L, 257), [-0.1, L + 0.1]])
    for a, b in zip(eng.spline_eval(sv), eng2.spline_eval(sv)):
        assert np.array_equal(a, b)
    with pytest.raises(m.MpccError):
        s, X, Y, Z, R = eng.track_path()
        eng2.set_track_path(s[:50], X[:50], Y[:50], Z[:50], R[:50])
    eng2.close()


def test_projection(setup20):
    """projectOnSpline (arc_length_spline.cpp:318-379) incl. the far branch (Q12) and the 0/0 Newton step
    at the track end that the reference's unwrapInput maps to s = 0."""
    m, o, eng, pool = setup20
    rng = np.random.default_rng(SEED + 7)
    L = o.track_length()
    M = 400
    sg = rng.uniform(0, L, M)
    base = np.array([o.spline_eval(s)[0] for s in sg])
    off = rng.normal(0, 1, (M, 3))
    off *= (rng.choice([0.005, 0.02, 0.05, 0.12], M) / np.linalg.norm(off, axis=1))[:, None]
    ee = base + off
    sgpu = eng.project(sg, ee)
    so = np.array([o.project(sg[i], ee[i]) for i in range(M)])
    assert np.abs(sgpu - so).max() <= 1e-9, np.abs(sgpu - so).max()
    # the benchmark-pool cases that once diverged (far branch, Newton cycling through s = L)
    x = pool["x0"][5:60]
    ee2 = np.array([o.fk(q[:7])[0] for q in x])
    s2 = np.clip(x[:, 7] + 0.1, 0, L)
    assert np.abs(eng.project(s2, ee2) - np.array([o.project(s2[i], ee2[i]) for i in range(len(s2))])).max() <= 1e-9


def test_robot_records(setup20):
    m, o, eng, pool = setup20
    rng = np.random.default_rng(SEED)
    M = 48
    q = Q0 + rng.normal(0, 0.3, size=(M, 7))
    obs = np.column_stack([np.full(M, 0.48), np.full(M, 0.218), rng.uniform(0.421, 0.621, M), np.full(M, 5.0)])
    rec = eng.robot_records(q, obs)
    for i in range(M):
        ro = o.robot_record(q[i], obs[i, :3], obs[i, 3])
        assert np.allclose(rec[i, :55], ro[:55], rtol=1e-11, atol=1e-13), i          # FK, R, J, mu
        assert np.allclose(rec[i, 55:62], ro[55:62], rtol=1e-7, atol=1e-9), i        # FD gradient of mu
        assert np.allclose(rec[i, 62:], ro[62:], rtol=1e-10, atol=1e-10), i          # MLP distances + Jacobians


def test_stage_cost(setup20):
    m, o, eng, pool = setup20
    rng = np.random.default_rng(SEED + 1)
    M = 40
    N = o.N
    x = np.zeros((M, 9)); u = rng.normal(0, 0.2, (M, 8))
    x[:, :7] = Q0 + rng.normal(0, 0.1, (M, 7))
    x[:, 7] = rng.uniform(0, o.track_length(), M)
    x[:, 8] = rng.uniform(-0.2, 0.3, M)
    k = rng.integers(0, N + 1, M).astype(np.int32)
    recs = np.stack([o.robot_record(x[i, :7]) for i in range(M)])
    obj, fx, fu, fxx, fuu = eng.stage_cost(x, u, recs, k)
    for i in range(M):
        oo, ofx, ofu, ofxx, ofuu, _ = o.stage_cost(x[i], u[i], recs[i], int(k[i]))
        assert abs(obj[i] - oo) <= 1e-10 * max(1.0, abs(oo)), i
        assert np.allclose(fx[i], ofx, rtol=1e-9, atol=1e-9), i
        assert np.allclose(fu[i], ofu, rtol=1e-12, atol=1e-14), i
        assert np.allclose(fxx[i], ofxx, rtol=1e-9, atol=1e-8), i
        assert np.allclose(np.diag(fuu[i]), np.diag(ofuu), rtol=1e-12), i


def _qp_cases(o, pool, B, rng, scale):
    N = o.N
    T = len(pool["x0"])
    guess = np.zeros((B, N + 1, 17))
    recs = np.zeros((B, N + 1, 143))
    ucur = np.zeros((B, 8))
    for b in range(B):
        t = 5 + (b * 7) % (T - 6)
        g = pool["guess"][t + 1].copy()
        g[:, :7] += rng.normal(0, 0.01 * scale, (N + 1, 7))
        g[:N, 9:] += rng.normal(0, 0.05 * scale, (N, 8))
        guess[b] = g
        ucur[b] = pool["u0"][t + 1]
        for k in range(N + 1):
            recs[b, k] = o.robot_record(g[k, :7])
    return guess, recs, ucur


@pytest.mark.parametrize("scale", [1.0, 4.0])
def test_qp_step(setup20, scale):
    m, o, eng, pool = setup20
    rng = np.random.default_rng(SEED + 2)
    B = 24
    guess, recs, ucur = _qp_cases(o, pool, B, rng, scale)
    step, st, it = eng.solve_qp(guess, recs, ucur)
    for b in range(B):
        rc, so, ito = o.solve_qp(guess[b], recs[b], ucur[b], mode=0)
        assert st[b] == rc, (b, st[b], rc)
        assert it[b] == ito, (b, it[b], ito)  # IPM iterations of both attempts (scaled start + restart)
        if rc == 0:
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


def test_solve_batch_parity(setup20):
    m, o, eng, pool = setup20
    rng = np.random.default_rng(SEED + 3)
    B = 200
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, qnoise=0.005)
    (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo) = _run_both(eng, o, x0, u0, obs, guess, valid, fails)
    assert np.allclose(xg, xo, rtol=0, atol=1e-9)
    same = outg["status"] == outo["status"]
    flips = int(np.sum(~same))
    assert flips == 0, f"status flips {flips}"
    ok = same & (outo["status"] == 0)
    du = np.abs(outg["horizon"][ok, :-1, 9:] - outo["horizon"][ok, :-1, 9:]).max()
    assert du <= 1e-6, du
    assert np.abs(outg["u0"][same] - outo["u0"][same]).max() <= 1e-6
    assert np.abs(outg["horizon"][same] - outo["horizon"][same]).max() <= 1e-6
    assert np.array_equal(vg[same], vo[same]) and np.array_equal(fg[same], fo[same])
    assert np.array_equal(outg["ok"][same], outo["ok"][same])


def test_closed_loop_single(setup20):
    """B = 1 closed loop from the reference's start state (main.cpp:60-63, 100-114), 60 steps."""
    m, o, eng, pool = setup20
    N = o.N
    x = np.zeros((1, 9)); x[0, :7] = Q0
    u = np.zeros((1, 8)); ob = np.array([[3.0, 3.0, 3.0, 0.0]])
    eng.reset_warmstart(1)
    go = np.zeros((1, N + 1, 17)); vo = np.zeros(1, np.int32); fo = np.zeros(1, np.int32)
    for step in range(60):
        xg = x.copy(); xo = x.copy()
        outg = eng.solve(xg, u, ob)
        outo = o.run_mpc(xo, u, ob, go, vo, fo)
        assert outg["status"][0] == outo["status"][0], step
        assert np.abs(outg["u0"] - outo["u0"]).max() <= 1e-6, step
        assert np.abs(xg - xo).max() <= 1e-9, step
        u = outo["u0"].copy()
        x[0] = o.sim_time_step(xo[0], u[0], o.params["Ts"])  # the mutated state (main.cpp:103-105)


@pytest.mark.parametrize("mask,B", [(2, 4096), (7, 1024)])
def test_benchmark_batch_parity(built_lib, oracle_lib, mask, B):
    """configs[1] at full size (B = 4096, bounds + singularity rows) and the full constraint set:
    every instance's status and optimal input sequence match the oracle (1e-6, north star)."""
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16)
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    pool = oracle_pool(o, 400)
    rng = np.random.default_rng(SEED + 11)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, qnoise=0.005)
    (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo) = _run_both(eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(xg - xo).max() <= 1e-9
    assert np.array_equal(vg, vo) and np.array_equal(fg, fo)
    eng.close()


# ---------------------------------------------------------------- second-order correction
@pytest.mark.parametrize("mask,B,staged", [(2, 1024, False), (7, 256, False), (7, 256, True)])
def test_soc_batch_parity(built_lib, oracle_lib, monkeypatch, mask, B, staged):
    """do_SOC = 1 (SecondOrderCorrection, osqp_interface.cpp:506-535, 658-681): a second QP with the first
    QP's P, q, A and the bounds at x + step shifted by A step, in the fused k_sqp and in the staged
    loop (k_soc + k_ipm), against the oracle (status exact, inputs 1e-6)."""
    import mpcc_manipulator_amd as m
    if staged:
        monkeypatch.setenv("MPCC_STAGED_SQP", "1")
    ov = {"sqp": {"max_iter": 2, "do_SOC": 1}}
    o, P, track = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16, overrides=ov)
    assert P["do_SOC"] == 1
    params = m.load_params(N=20, overrides=ov)
    eng = m.Engine(params, max_batch=B, constraint_mask=mask)
    eng.set_track(*track)
    pool = oracle_pool(o, 200, obs=(0.48, 0.218, 0.521, 5.0) if mask == 7 else (3.0, 3.0, 3.0, 0.0))
    rng = np.random.default_rng(SEED + 17)
    obs = None
    if mask == 7:
        obs = np.column_stack([np.full(B, 0.48), np.full(B, 0.218), rng.uniform(0.421, 0.621, B), np.full(B, 5.0)])
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, qnoise=0.005, obs=obs)
    (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo) = _run_both(eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.array_equal(vg, vo) and np.array_equal(fg, fo)
    # the correction is live: the same batch without it gives different inputs
    o2, _, _ = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16)
    out2 = o2.run_mpc(x0.copy(), u0, obs, guess.copy(), valid.copy(), fails.copy())
    assert np.abs(out2["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() > 1e-6
    eng.close()


# ---------------------------------------------------------------- the closed loop on the device
def test_device_closed_loop(setup20):
    """main.cpp:100-114 on the device for B instances (mpcc_closed_loop) against the oracle's loop:
    runMPC_, then simTimeStep of the state runMPC_ updated, an instance stopping when runMPC_ returns
    false.  Status at every step exact, inputs <= 1e-6, states <= 1e-8; the hipGraph replay is bitwise
    the plain launch sequence."""
    m, o, eng, pool = setup20
    B, steps = 48, 25
    rng = np.random.default_rng(SEED + 9)
    z = rng.uniform(0.421, 0.621, B)
    obs = np.column_stack([np.full(B, 0.48), np.full(B, 0.218), z, np.full(B, 5.0)])
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=obs)
    eng.set_warmstart(guess, valid, fails)
    rg = eng.closed_loop(x0, u0, obs, steps, graph=True)
    eng.set_warmstart(guess, valid, fails)
    rp = eng.closed_loop(x0, u0, obs, steps, graph=False)
    for key in ("x", "u", "status", "x_final", "u_final"):
        assert np.array_equal(rg[key], rp[key]), key
    x, u = x0.copy(), u0.copy()
    g, v, f = guess.copy(), valid.copy(), fails.copy()
    alive = np.ones(B, bool)
    for k in range(steps):
        assert np.abs(rg["x"][k] - x).max() <= 1e-8, k
        xin = x.copy()
        out = o.run_mpc(xin, u, obs, g, v, f)
        assert np.array_equal(rg["status"][k], np.where(alive, out["status"], -1)), k
        go = alive & (out["ok"] != 0)
        u[go] = out["u0"][go]
        for b in np.where(go)[0]:
            x[b] = o.sim_time_step(xin[b], u[b], o.params["Ts"])
        alive = go
        assert np.abs(rg["u"][k] - u).max() <= 1e-6, k
    assert np.abs(rg["x"][steps] - x).max() <= 1e-8
    assert np.array_equal(rg["x_final"], rg["x"][steps])


# ---------------------------------------------------------------- a track per instance
def _track_variant(track, theta, scale):
    """The default way-points rotated by theta about z through their start point and scaled about it
    (rotations follow: R' = Rz R), as a different path for another controller of the batch."""
    X, Y, Z, R = (np.asarray(a, float) for a in track)
    c, sn = np.cos(theta), np.sin(theta)
    Rz = np.array([[c, -sn, 0], [sn, c, 0], [0, 0, 1]])
    P = np.stack([X - X[0], Y - Y[0], Z - Z[0]], 1) @ Rz.T * scale
    return X[0] + P[:, 0], Y[0] + P[:, 1], Z[0] + P[:, 2], np.einsum("ij,njk->nik", Rz, R.reshape(-1, 3, 3))


def test_per_instance_tracks(built_lib, oracle_lib):
    """mpcc_set_tracks: instance b follows its own path.  Four track variants interleaved over 64
    instances, each instance's state pool from the oracle's closed loop on its own track; every
    instance matches the oracle holding that track (status, u <= 1e-6, x0 update, controller state).
    Per-instance copies of one track are bitwise the shared track; a batch larger than the number of
    tracks is refused."""
    import mpcc_manipulator_amd as m
    V, B, N = 4, 64, 20
    base_o, P, track = make_oracle(N=N, max_iter=2, mask=7)
    variants = [_track_variant(track, th, sc) for th, sc in [(0.0, 1.0), (-0.1, 1.05), (-0.2, 0.9), (0.1, 0.95)]]
    orcs, pools = [], []
    for X, Y, Z, R in variants:
        o, _, _ = make_oracle(N=N, max_iter=2, mask=7)
        o.set_track(X, Y, Z, R)
        orcs.append(o)
        pools.append(oracle_pool(o, 30))
    rng = np.random.default_rng(SEED + 31)
    inst = [batch_from_pool(pools[v], B // V, rng) for v in range(V)]
    order = np.arange(B) % V                      # instance b -> variant b % V
    pick = lambda j: np.stack([inst[order[b]][j][b // V] for b in range(B)])
    x0, u0, obs, guess, valid, fails = (pick(j) for j in range(6))
    n = len(variants[0][0])
    TX = np.stack([variants[v][0] for v in order]); TY = np.stack([variants[v][1] for v in order])
    TZ = np.stack([variants[v][2] for v in order]); TR = np.stack([variants[v][3] for v in order])
    eng = m.Engine(m.load_params(N=N, overrides={"sqp": {"max_iter": 2}}), max_batch=2 * B, constraint_mask=7)
    eng.set_tracks(TX, TY, TZ, TR)
    eng.set_warmstart(guess, valid, fails)
    xg = x0.copy()
    outg = eng.solve(xg, u0, obs)
    gg, vg, fg = eng.get_warmstart(B)
    for v in range(V):
        sel = np.where(order == v)[0]
        xo = x0[sel].copy(); go = guess[sel].copy(); vo = valid[sel].copy(); fo = fails[sel].copy()
        outo = orcs[v].run_mpc(xo, u0[sel], obs[sel], go, vo, fo)
        assert np.array_equal(outg["status"][sel], outo["status"]), v
        assert np.abs(outg["horizon"][sel] - outo["horizon"]).max() <= 1e-6, v
        assert np.abs(xg[sel] - xo).max() <= 1e-9, v
        assert np.array_equal(vg[sel], vo) and np.array_equal(fg[sel], fo), v
    with pytest.raises(m.MpccError):
        eng.solve(np.zeros((B + 1, 9)), np.zeros((B + 1, 8)), np.tile([3.0, 3.0, 3.0, 0.0], (B + 1, 1)))
    # per-instance copies of one track == the shared track, bitwise
    X, Y, Z, R = variants[1]
    eng.set_tracks(np.tile(X, (B, 1)), np.tile(Y, (B, 1)), np.tile(Z, (B, 1)), np.tile(R, (B, 1, 1, 1)))
    eng.set_warmstart(guess, valid, fails)
    xa = x0.copy(); a = eng.solve(xa, u0, obs)
    eng.set_track(X, Y, Z, R)
    eng.set_warmstart(guess, valid, fails)
    xb = x0.copy(); b2 = eng.solve(xb, u0, obs)
    assert np.array_equal(a["horizon"], b2["horizon"]) and np.array_equal(xa, xb)
    assert np.array_equal(a["status"], b2["status"])
    eng.close()


# ---------------------------------------------------------------- configs[2]: N = 40, both MLPs, obstacles
def _obstacles(rng, B):
    """main_w_sim.py:42-45 scenario: xyz = (0.48, 0.218, z), z ~ U[0.421, 0.621], r = 5 cm."""
    z = rng.uniform(0.421, 0.621, B)
    return np.column_stack([np.full(B, 0.48), np.full(B, 0.218), z, np.full(B, 5.0)])


@pytest.fixture(scope="module")
def setup40(built_lib, oracle_lib):
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=40, max_iter=2, mask=7, nthreads=16)
    pool = oracle_pool(o, 120, obs=(0.48, 0.218, 0.521, 5.0))
    return m, o, track, pool


def test_config2_parity(setup40):
    """BASELINE configs[2] shape (N = 40, self + env collision rows, per-instance obstacles): status,
    optimal input sequence (1e-6), x0 update and controller state match the oracle per instance."""
    m, o, track, pool = setup40
    B = 512
    rng = np.random.default_rng(SEED + 40)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=_obstacles(rng, B))
    eng = m.Engine(m.load_params(N=40, overrides={"sqp": {"max_iter": 2}}), max_batch=B, constraint_mask=7)
    eng.set_track(*track)
    (xg, outg, gg, vg, fg), (xo, outo, go, vo, fo) = _run_both(eng, o, x0, u0, obs, guess, valid, fails)
    assert np.array_equal(outg["status"], outo["status"])
    assert np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(outg["horizon"] - outo["horizon"]).max() <= 1e-6
    assert np.abs(xg - xo).max() <= 1e-9
    assert np.array_equal(vg, vo) and np.array_equal(fg, fo) and np.array_equal(outg["ok"], outo["ok"])
    eng.close()


def test_config2_full_scale(setup40):
    """configs[2] at full size (B = 65,536, N = 40): size-independent properties.
    (1) instance independence: a random subset re-solved alone is bitwise identical to its rows of the
    full batch (outputs, x0 update, warm-start state); (2) every output finite with a valid status;
    (3) a seeded sample of 64 instances matches the oracle (status, u <= 1e-6)."""
    m, o, track, pool = setup40
    B = 65536
    rng = np.random.default_rng(SEED + 65536)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng, obs=_obstacles(rng, B))
    params = m.load_params(N=40, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=B, constraint_mask=7)
    eng.set_track(*track)
    eng.set_warmstart(guess, valid, fails)
    xf = x0.copy()
    full = eng.solve(xf, u0, obs)
    gf, vf, ff = eng.get_warmstart(B)
    assert np.all(np.isfinite(full["horizon"])) and np.all(np.isfinite(xf))
    assert set(np.unique(full["status"]).tolist()) <= {0, 1, 10, 11}
    assert np.mean(full["status"] == 0) > 0.97, np.bincount(full["status"])  # bench configs[2]: 99.5% SOLVED
    sub = np.sort(rng.choice(B, 256, replace=False))
    eng.set_warmstart(guess[sub], valid[sub], fails[sub])
    xs = x0[sub].copy()
    part = eng.solve(xs, u0[sub], obs[sub])
    gs, vs, fs = eng.get_warmstart(len(sub))
    assert np.array_equal(part["status"], full["status"][sub])
    assert np.array_equal(part["horizon"], full["horizon"][sub]) and np.array_equal(xs, xf[sub])
    assert np.array_equal(gs, gf[sub]) and np.array_equal(vs, vf[sub]) and np.array_equal(fs, ff[sub])
    smp = sub[:64]
    xo = x0[smp].copy(); go = guess[smp].copy(); vo = valid[smp].copy(); fo = fails[smp].copy()
    outo = o.run_mpc(xo, u0[smp], obs[smp], go, vo, fo)
    assert np.array_equal(outo["status"], full["status"][smp])
    assert np.abs(outo["horizon"][:, :-1, 9:] - full["horizon"][smp, :-1, 9:]).max() <= 1e-6
    eng.close()


# ---------------------------------------------------------------- committed golden vectors
def _gold(name):
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name), allow_pickle=False)


def test_golden_records_gpu(setup20):
    m, o, eng, pool = setup20
    g = _gold("records.npz")
    rec = eng.robot_records(g["q"], g["obs"])
    assert np.allclose(rec[:, :55], g["rec"][:, :55], rtol=1e-11, atol=1e-13)
    assert np.allclose(rec[:, 55:62], g["rec"][:, 55:62], rtol=1e-7, atol=1e-9)
    assert np.allclose(rec[:, 62:], g["rec"][:, 62:], rtol=1e-10, atol=1e-10)


def test_golden_qp_step_gpu(setup20):
    m, o, eng, pool = setup20
    g = _gold("qp_step.npz")
    step, st, it = eng.solve_qp(g["guess"], g["rec"], g["ucur"])
    assert np.array_equal(st, g["status"])
    assert np.abs(step - g["step"]).max() < 1e-8


def test_golden_batch_mask2_gpu(built_lib, oracle_lib):
    import mpcc_manipulator_amd as m
    g = _gold("batch_mask2.npz")
    o, P, track = make_oracle(N=20, max_iter=2, mask=2)
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=64, constraint_mask=2)
    eng.set_track(*track)
    eng.set_warmstart(g["guess"], g["valid"], g["fails"])
    xg = g["x0"].copy()
    out = eng.solve(xg, g["u0"], g["obs"])
    assert np.array_equal(out["status"], g["status"])
    assert np.abs(out["horizon"][:, :-1, 9:] - g["horizon"][:, :-1, 9:]).max() <= 1e-6
    assert np.abs(xg - g["x0_out"]).max() <= 1e-9
    eng.close()


def test_solve_ocp_plugin_boundary(built_lib, oracle_lib):
    """mpcc_solve_ocp (the SolverInterface::solveOCP granularity, solver_interface.h:44-54): given the
    guess the reference MPC would pass after its own projection and shift (here: the oracle's
    runMPC_ prefix), it returns the same opt_sol and status as the full runMPC_ path, and as the fixture."""
    import mpcc_manipulator_amd as m
    g = _gold("batch_mask2.npz")
    o, P, track = make_oracle(N=20, max_iter=2, mask=2)
    xo, go, vo, fo = g["x0"].copy(), g["guess"].copy(), g["valid"].copy(), g["fails"].copy()
    o.prepare(xo, g["u0"], g["obs"], go, vo, fo)           # MPC side: projection + warm start (mpc.cpp:104-124)
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=64, constraint_mask=2)
    eng.set_track(*track)
    res = eng.solve_ocp(go, g["u0"], g["obs"])
    assert np.array_equal(res["status"], g["status"])
    assert np.array_equal(res["solved"], (g["status"] == 0).astype(np.int32))
    assert np.abs(res["opt_sol"][:, :-1, 9:] - g["horizon"][:, :-1, 9:]).max() <= 1e-6
    eng.set_warmstart(g["guess"], g["valid"], g["fails"])
    full = eng.solve(g["x0"].copy(), g["u0"], g["obs"])
    assert np.array_equal(full["status"], res["status"])
    assert np.abs(full["horizon"] - res["opt_sol"]).max() <= 1e-12
    eng.close()


def test_cpp_ocp_solver_plugin(built_lib, oracle_lib, tmp_path):
    """mpcc_amd::OcpSolver (SolverInterface mirror; examples/ocp_solver_io.cpp drives it as MPC::runMPC_
    drives solver_interface_) on the golden configs[1] batch, one instance at a time on one solver:
    status, solveOCP's bool and opt_sol match the fixture (u <= 1e-6)."""
    import subprocess
    g = _gold("batch_mask2.npz")
    o, P, track = make_oracle(N=20, max_iter=2, mask=2)
    xo, go, vo, fo = g["x0"].copy(), g["guess"].copy(), g["valid"].copy(), g["fails"].copy()
    o.prepare(xo, g["u0"], g["obs"], go, vo, fo)
    B, N = go.shape[0], 20
    s, X, Y, Z, R = o.track_path()
    blob = [np.array([N, B], np.int32).tobytes()] + [np.asarray(a, np.float64).tobytes() for a in (s, X, Y, Z, R)]
    for b in range(B):
        blob += [go[b].tobytes(), np.asarray(g["u0"][b], np.float64).tobytes(), g["obs"][b].tobytes()]
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(b"".join(blob))
    exe = os.path.join(os.path.dirname(built_lib), "ocp_solver_io")
    r = subprocess.run([exe, os.path.join(ROOT, "mpcc_manipulator_amd", "data"), "2", "2", str(fin), str(fout)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    raw = fout.read_bytes()
    rec = 8 + (N + 1) * 17 * 8
    assert len(raw) == B * rec
    for b in range(B):
        st, ok = np.frombuffer(raw[b * rec:b * rec + 8], np.int32)
        sol = np.frombuffer(raw[b * rec + 8:(b + 1) * rec], np.float64).reshape(N + 1, 17)
        assert st == g["status"][b] and ok == (st == 0), b
        assert np.abs(sol[:-1, 9:] - g["horizon"][b, :-1, 9:]).max() <= 1e-6, b


def test_golden_closed_loop_gpu(setup20):
    """The engine drives the 60-step closed loop of the fixture (status and u0 at every step)."""
    m, o, eng, pool = setup20
    g = _gold("closed_loop_n20.npz")
    eng.reset_warmstart(1)
    for step in range(g["x"].shape[0]):
        x = g["x"][step:step + 1].copy()
        u = g["u0"][step - 1:step].copy() if step else np.zeros((1, 8))
        out = eng.solve(x, u, g["obs"][None, :])
        assert out["status"][0] == g["status"][step], step
        assert np.abs(out["u0"][0] - g["u0"][step]).max() <= 1e-6, step


def test_cpp_mpc_closed_loop_golden(built_lib):
    """The C++ host surface (mpcc_amd::MPC, examples/mpc_closed_loop.cpp: the reference main.cpp loop)
    reproduces the golden closed loop: status at every step, u0 within 1e-6, states within 1e-6."""
    import subprocess
    g = _gold("closed_loop_n20.npz")
    exe = os.path.join(os.path.dirname(built_lib), "mpc_closed_loop")
    steps = g["x"].shape[0]
    r = subprocess.run([exe, os.path.join(ROOT, "mpcc_manipulator_amd", "data"), str(steps)] +
                       [repr(float(v)) for v in g["obs"]], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = np.array([[float(v) for v in line.split(",")] for line in r.stdout.strip().splitlines()])
    assert rows.shape == (steps, 1 + 9 + 8 + 2)
    assert np.abs(rows[:, 1:10] - g["x"]).max() <= 1e-6
    assert np.abs(rows[:, 10:18] - g["u0"]).max() <= 1e-6
    assert np.array_equal(rows[:, 18].astype(np.int32), g["status"])
