"""Large-batch parity scan: HIP engine vs the CPU oracle on the benchmark workload.

Reports status flips (instances whose SQP takes a different discrete branch) and the max |du| over
instances with equal status.  Test infrastructure: imports oracle/ (never on the product path).

    python tools/parity_scan.py --batch 4096 --mask 2
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--mask", type=int, default=2)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--pool", type=int, default=400)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--qnoise", type=float, default=0.005)
    ap.add_argument("--show", type=int, default=12)
    args = ap.parse_args()
    from helpers import SEED, batch_from_pool, make_oracle, oracle_pool
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=args.N, max_iter=2, mask=args.mask, nthreads=args.threads)
    params = m.load_params(N=args.N, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=args.batch, constraint_mask=args.mask)
    eng.set_track(*track)
    pool = oracle_pool(o, args.pool)
    rng = np.random.default_rng(SEED + 11)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, args.batch, rng, qnoise=args.qnoise)
    eng.set_warmstart(guess, valid, fails)
    eng.trace_enable(True)
    xg = x0.copy()
    outg = eng.solve(xg, u0, obs)
    trg = eng.trace_get(args.batch)
    sg = eng.solve_stats(args.batch)
    xo = x0.copy(); go = guess.copy(); vo = valid.copy(); fo = fails.copy()
    outo = o.run_mpc(xo, u0, obs, go, vo, fo, trace=True)
    tro = outo["trace"]
    same = outg["status"] == outo["status"]
    ok = same & (outo["status"] == 0)
    du = float(np.abs(outg["horizon"][same, :-1, 9:] - outo["horizon"][same, :-1, 9:]).max()) if same.any() else 0.0
    du_ok = float(np.abs(outg["horizon"][ok, :-1, 9:] - outo["horizon"][ok, :-1, 9:]).max()) if ok.any() else 0.0
    flips = np.nonzero(~same)[0]
    dmax = np.abs(outg["horizon"][:, :-1, 9:] - outo["horizon"][:, :-1, 9:]).reshape(args.batch, -1).max(axis=1)
    branch = np.nonzero(same & (dmax > 1e-6))[0]
    # near-tie check: the oracle's dense-layout QP (same algorithm, different rounding) on those instances
    sel = np.concatenate([flips, branch]).astype(int)
    dense_agree = None
    if sel.size:
        od, _, _ = make_oracle(N=args.N, max_iter=2, mask=args.mask, qp_mode=1, nthreads=args.threads)
        xd = x0[sel].copy(); gd = guess[sel].copy(); vd = valid[sel].copy(); fd = fails[sel].copy()
        outd = od.run_mpc(xd, u0[sel], obs[sel], gd, vd, fd)
        dd = np.abs(outd["horizon"][:, :-1, 9:] - outo["horizon"][sel, :-1, 9:]).reshape(sel.size, -1).max(axis=1)
        dense_agree = {"oracle_dense_vs_riccati_differs": int(np.sum((outd["status"] != outo["status"][sel]) | (dd > 1e-6))),
                       "of": int(sel.size),
                       "gpu_matches_dense": int(np.sum((outd["status"] == outg["status"][sel]) &
                                                       (np.abs(outd["horizon"][:, :-1, 9:] - outg["horizon"][sel, :-1, 9:]).reshape(sel.size, -1).max(axis=1) <= 1e-6)))}
    sel = np.concatenate([flips, branch]).astype(int)
    res = {"batch": args.batch, "mask": args.mask, "flips": int(flips.size),
           "flip_pairs": [[int(outg["status"][i]), int(outo["status"][i])] for i in flips[:20]],
           "max_du_same_status": du, "branch_diffs_same_status": int(branch.size),
           "sqp_iter_pairs": [[int(sg["sqp_iter"][i]), int(outo["sqp_iters"][i])] for i in sel[:20]] if sel.size else [],
           "near_tie_check": dense_agree, "max_du_solved": du_ok,
           "gpu_status_hist": np.bincount(outg["status"], minlength=12).tolist(),
           "oracle_status_hist": np.bincount(outo["status"], minlength=12).tolist(),
           "gpu_ipm_iters_mean": float(sg["ipm_iters"].mean()), "gpu_ipm_iters_max": int(sg["ipm_iters"].max())}
    print(json.dumps(res))
    np.set_printoptions(linewidth=200, precision=17)
    for i in sel[:args.show]:
        print(f"--- instance {i}: gpu status {outg['status'][i]} oracle {outo['status'][i]} du {dmax[i]:.3g} "
              f"valid_in {valid[i]} x0_in s {x0[i, 7]:.12g} | gpu s,vs {xg[i, 7]:.15g} {xg[i, 8]:.15g} | "
              f"oracle s,vs {xo[i, 7]:.15g} {xo[i, 8]:.15g}")
        for itr in range(3):
            print("  it", itr, "gpu   ", trg[i, itr].tolist())
            print("  it", itr, "oracle", tro[i, itr].tolist())


if __name__ == "__main__":
    main()
