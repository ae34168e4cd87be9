"""Shared test helpers: oracle setup, closed-loop state pools, comparison utilities."""
import numpy as np

import refparams as rp

Q0 = np.array([0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4])  # main.cpp:60-61
SEED = 0x4D504343


# start configuration of the Husky+Panda (configs[3]): base at the origin, arm at the reference's Q0
Q0_MOBILE = np.concatenate([[0.0, 0.0, 0.0], Q0])


def make_oracle(N=20, max_iter=2, mask=7, qp_mode=0, nthreads=1, overrides=None, dof=7):
    from oracle.pyoracle import Oracle
    P = rp.resolve(N=N, constraint_mask=mask, overrides=overrides, dof=dof)
    if max_iter is not None:
        P["max_iter"] = max_iter
    o = Oracle(P, rp.NN_DIR, qp_mode=qp_mode, nthreads=nthreads, dof=dof)
    pee, _, _ = o.fk(Q0_MOBILE if dof == 10 else Q0)
    X, Y, Z, R = rp.default_track_xyzr(pee)
    o.set_track(X, Y, Z, np.array(R))
    return o, P, (X, Y, Z, np.array(R))


def oracle_pool(o, steps, obs=(3.0, 3.0, 3.0, 0.0)):
    if o.dof != 7:
        return oracle_pool_dof(o, steps, obs)
    """Closed loop (main.cpp:100-114): runMPC_ (which mutates x0's s, vs) then simTimeStep of the
    mutated state.  Returns per-step controller inputs (x0 before projection, u0, obs, warm start
    (guess, valid, fails) before the call)."""
    N = o.N
    x = np.zeros((1, 9)); x[0, :7] = Q0
    u = np.zeros((1, 8))
    ob = np.array([obs], dtype=np.float64)
    guess = np.zeros((1, N + 1, 17)); valid = np.zeros(1, np.int32); fails = np.zeros(1, np.int32)
    pool = dict(x0=[], u0=[], guess=[], valid=[], fails=[], status=[])
    for _ in range(steps):
        pool["x0"].append(x[0].copy()); pool["u0"].append(u[0].copy())
        pool["guess"].append(guess[0].copy()); pool["valid"].append(valid[0]); pool["fails"].append(fails[0])
        xin = x.copy()
        out = o.run_mpc(xin, u, ob, guess, valid, fails)
        pool["status"].append(out["status"][0])
        u = out["u0"].copy()
        x[0] = o.sim_time_step(xin[0], u[0], o.params["Ts"])
    return {k: np.array(v) for k, v in pool.items()}


def batch_from_pool(pool, B, rng, qnoise=0.005, obs=None):
    """Config-2/3 instances: pool step t = i mod T, q += N(0, qnoise) on the joints."""
    T = len(pool["x0"])
    idx = np.arange(B) % T
    x0 = pool["x0"][idx].copy()
    dof = x0.shape[1] - 2
    x0[:, :dof] += rng.normal(0.0, qnoise, size=(B, dof))
    u0 = pool["u0"][idx].copy()
    guess = pool["guess"][idx].copy()
    valid = pool["valid"][idx].astype(np.int32).copy()
    fails = pool["fails"][idx].astype(np.int32).copy()
    if obs is None:
        obs = np.tile(np.array([3.0, 3.0, 3.0, 0.0]), (B, 1))
    return x0, u0, np.ascontiguousarray(obs, dtype=np.float64), guess, valid, fails


def max_rel(a, b, floor=1e-12):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor))) if a.size else 0.0


def oracle_pool_dof(o, steps, obs=(3.0, 3.0, 3.0, 0.0)):
    """oracle_pool for any robot (state [q(DOF), s, vs]); the start is Q0_MOBILE for the 10-DOF model."""
    N, nx, nu, dof = o.N, o.NX, o.NU, o.dof
    x = np.zeros((1, nx)); x[0, :dof] = Q0_MOBILE if dof == 10 else Q0
    u = np.zeros((1, nu))
    ob = np.array([obs], dtype=np.float64)
    guess = np.zeros((1, N + 1, o.NXU)); valid = np.zeros(1, np.int32); fails = np.zeros(1, np.int32)
    pool = dict(x0=[], u0=[], guess=[], valid=[], fails=[], status=[])
    for _ in range(steps):
        pool["x0"].append(x[0].copy()); pool["u0"].append(u[0].copy())
        pool["guess"].append(guess[0].copy()); pool["valid"].append(valid[0]); pool["fails"].append(fails[0])
        xin = x.copy()
        out = o.run_mpc(xin, u, ob, guess, valid, fails)
        pool["status"].append(out["status"][0])
        u = out["u0"].copy()
        x[0] = o.sim_time_step(xin[0], u[0], o.params["Ts"])
    return {k: np.array(v) for k, v in pool.items()}
