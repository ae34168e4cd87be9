"""Generate the golden fixtures under tests/golden/ from the oracle (CPU restatement of the reference).

The reference pins almost no numeric outputs of the hot path; these fixtures freeze
the oracle's outputs at its pinned state (KAT- and property-checked, tests/test_oracle.py) so that
(a) the oracle cannot drift silently and (b) the GPU engine is checked against committed vectors.

    python tools/make_golden.py            # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import Q0, SEED, batch_from_pool, make_oracle, oracle_pool  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def closed_loop(o, steps, obs):
    N = o.N
    x = np.zeros((1, 9)); x[0, :7] = Q0
    u = np.zeros((1, 8))
    ob = np.array([obs])
    g = np.zeros((1, N + 1, 17)); v = np.zeros(1, np.int32); f = np.zeros(1, np.int32)
    xs, us, st = [], [], []
    for _ in range(steps):
        xs.append(x[0].copy())
        xin = x.copy()
        out = o.run_mpc(xin, u, ob, g, v, f)
        st.append(out["status"][0])
        u = out["u0"].copy()
        us.append(u[0].copy())
        x[0] = o.sim_time_step(xin[0], u[0], o.params["Ts"])  # the state runMPC mutated (main.cpp:103-105)
    return np.array(xs), np.array(us), np.array(st, np.int32)


def main():
    os.makedirs(OUT, exist_ok=True)
    from oracle import pyoracle
    pyoracle.build()
    o, P, track = make_oracle(N=20, max_iter=2, mask=7)
    rng = np.random.default_rng(SEED)

    # 1. closed loop from the reference start state (main.cpp:60-63, 100-114), obstacle of main_w_sim.py
    xs, us, st = closed_loop(o, 60, (0.48, 0.218, 0.521, 5.0))
    np.savez_compressed(os.path.join(OUT, "closed_loop_n20.npz"), x=xs, u0=us, status=st,
                        obs=np.array([0.48, 0.218, 0.521, 5.0]))

    # 2. robot records (FK, J, manipulability + FD gradient, both MLPs) at seeded configurations
    q = Q0 + rng.normal(0, 0.3, (16, 7))
    obs = np.column_stack([np.full(16, 0.48), np.full(16, 0.218), rng.uniform(0.421, 0.621, 16), np.full(16, 5.0)])
    rec = np.stack([o.robot_record(q[i], obs[i, :3], obs[i, 3]) for i in range(16)])
    np.savez_compressed(os.path.join(OUT, "records.npz"), q=q, obs=obs, rec=rec)

    # 3. stage cost (value, gradient, Hessian) at seeded (x, u, k)
    M = 16
    x = np.zeros((M, 9)); x[:, :7] = Q0 + rng.normal(0, 0.1, (M, 7))
    x[:, 7] = rng.uniform(0, o.track_length(), M); x[:, 8] = rng.uniform(-0.2, 0.3, M)
    u = rng.normal(0, 0.2, (M, 8))
    k = rng.integers(0, 21, M).astype(np.int32)
    recs = np.stack([o.robot_record(x[i, :7]) for i in range(M)])
    res = [o.stage_cost(x[i], u[i], recs[i], int(k[i])) for i in range(M)]
    np.savez_compressed(os.path.join(OUT, "stage_cost.npz"), x=x, u=u, k=k, rec=recs,
                        obj=np.array([r[0] for r in res]), fx=np.stack([r[1] for r in res]),
                        fu=np.stack([r[2] for r in res]), fxx=np.stack([r[3] for r in res]),
                        fuu=np.stack([r[4] for r in res]))

    # 4. QP steps (the OSQP replacement) on closed-loop warm starts
    pool = oracle_pool(o, 40)
    N = 20
    G, Rr, U, S, ST = [], [], [], [], []
    for t in range(5, 37, 8):
        g = pool["guess"][t + 1].copy()
        g[:, :7] += rng.normal(0, 0.01, (N + 1, 7))
        g[:N, 9:] += rng.normal(0, 0.05, (N, 8))
        r = np.stack([o.robot_record(g[kk, :7]) for kk in range(N + 1)])
        rc, s, it = o.solve_qp(g, r, pool["u0"][t + 1], mode=0)
        G.append(g); Rr.append(r); U.append(pool["u0"][t + 1]); S.append(s); ST.append(rc)
    np.savez_compressed(os.path.join(OUT, "qp_step.npz"), guess=np.stack(G), rec=np.stack(Rr), ucur=np.stack(U),
                        step=np.stack(S), status=np.array(ST, np.int32))

    # 5. a configs[1]-style batch (bounds + singularity rows), runMPC_ per instance
    o2, _, _ = make_oracle(N=20, max_iter=2, mask=2)
    pool2 = oracle_pool(o2, 200)
    x0, u0, obsb, guess, valid, fails = batch_from_pool(pool2, 64, np.random.default_rng(SEED + 21))
    xo = x0.copy(); go = guess.copy(); vo = valid.copy(); fo = fails.copy()
    out = o2.run_mpc(xo, u0, obsb, go, vo, fo)
    np.savez_compressed(os.path.join(OUT, "batch_mask2.npz"), x0=x0, u0=u0, obs=obsb, guess=guess, valid=valid,
                        fails=fails, x0_out=xo, status=out["status"], u0_out=out["u0"], horizon=out["horizon"],
                        valid_out=vo, fails_out=fo)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)), "bytes")


if __name__ == "__main__":
    main()
