"""QP-level probe of selected benchmark instances: the first SQP QP solved by the engine (k_ipm through
mpcc_debug_solve_qp) and by the oracle (Riccati and dense layouts) on identical inputs (oracle
prepare = runMPC_ up to the SQP).  Reports QP objective, feasibility and iteration counts.

    python tools/qp_probe.py --batch 4096 --mask 2 --idx 981 571 966
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def qp_eval(q, s):
    obj = 0.5 * s @ q["P"] @ s + q["g"] @ s
    As = q["A"] @ s
    vio = np.maximum(q["l"] - q["c"] - As, 0).max(initial=0) + 0 * np.maximum(As - (q["u"] - q["c"]), 0).max(initial=0)
    vu = np.maximum(As - (q["u"] - q["c"]), 0).max(initial=0)
    return obj, max(vio, vu)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--mask", type=int, default=2)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--pool", type=int, default=400)
    ap.add_argument("--idx", type=int, nargs="+", required=True)
    args = ap.parse_args()
    from helpers import SEED, batch_from_pool, make_oracle, oracle_pool
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=args.N, max_iter=2, mask=args.mask)
    params = m.load_params(N=args.N, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=len(args.idx), constraint_mask=args.mask)
    eng.set_track(*track)
    pool = oracle_pool(o, args.pool)
    rng = np.random.default_rng(SEED + 11)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, args.batch, rng)
    sel = np.array(args.idx)
    xs, gs, vs, fs = x0[sel].copy(), guess[sel].copy(), valid[sel].copy(), fails[sel].copy()
    recs = o.prepare(xs, u0[sel], obs[sel], gs, vs, fs)
    stg, stat_g, it_g = eng.solve_qp(gs, recs, u0[sel])
    np.set_printoptions(precision=6, linewidth=160)
    for j, i in enumerate(sel):
        q = o.dense_qp(gs[j], recs[j], u0[i])
        line = [f"inst {i}:"]
        for name, (rc, s, it) in (("gpu", (int(stat_g[j]), stg[j], int(it_g[j]))),
                                  ("ric", o.solve_qp(gs[j], recs[j], u0[i], mode=0)),
                                  ("dense", o.solve_qp(gs[j], recs[j], u0[i], mode=1))):
            if rc == 0:
                ob, vi = qp_eval(q, s)
                line.append(f"{name}: st {rc} it {it} qpobj {ob:.10g} vio {vi:.2e} |s| {np.abs(s).max():.6g}")
            else:
                line.append(f"{name}: st {rc} it {it}")
        print("  ".join(line))
        if stat_g[j] == 0:
            rc, s, it = o.solve_qp(gs[j], recs[j], u0[i], mode=1)
            if rc == 0:
                d = np.abs(stg[j] - s)
                print(f"   max|gpu - dense| {d.max():.3e} at {int(d.argmax())}")


if __name__ == "__main__":
    main()
