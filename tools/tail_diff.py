"""Where tail mode (csrc/ipm_tail.h) and the normal interior point differ on one batch: per instance the SQP trace
(QP status, IPM iterations, trial objective / violation, alpha) and the outputs of MPCC_TAIL=1 vs MPCC_TAIL=0.

    python tools/tail_diff.py [--batch 4096 --mask 2 --qnoise 0.005]
"""
import argparse
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
    ap.add_argument("--qnoise", type=float, default=0.005)
    ap.add_argument("--staged", action="store_true")
    args = ap.parse_args()
    import mpcc_manipulator_amd as m
    from helpers import batch_from_pool
    f = np.load(os.path.join(ROOT, "mpcc_manipulator_amd", "data", "bench_pool_n20_mask2.npz"), allow_pickle=False)
    pool = {k: f[k] for k in f.files}
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    e1 = m.Engine(params, max_batch=1, constraint_mask=args.mask)
    X, Y, Z, q = m.load_default_track()
    ee = e1.robot_records(np.array([[0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4]]), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    e1.close()
    track = m.track_from_points(X, Y, Z, q, ee)
    rng = np.random.default_rng(0x4D504343 + 41)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, args.batch, rng, qnoise=args.qnoise)
    if args.staged:
        os.environ["MPCC_STAGED_SQP"] = "1"
    res = {}
    for tail in (1, 0):
        os.environ["MPCC_TAIL"] = str(tail)
        B = args.batch
        eng = m.Engine(params, max_batch=B, constraint_mask=args.mask)
        eng.set_track(*track)
        eng.trace_enable(True)
        eng.tail_solves(reset=True)
        eng.set_warmstart(guess, valid, fails)
        x = x0.copy()
        out = eng.solve(x, u0, obs)
        res[tail] = dict(x=x, out=out, tr=eng.trace_get(B), st=eng.solve_stats(B), n=eng.tail_solves(reset=True))
        eng.close()
    a, b = res[1], res[0]
    print("tail solves:", a["n"], b["n"])
    du = np.abs(a["out"]["u0"] - b["out"]["u0"]).max(axis=1)
    bad = np.nonzero(np.any(a["out"]["u0"].view(np.int64) != b["out"]["u0"].view(np.int64), axis=1))[0]
    print("instances with u0 bits different:", len(bad), "max |du0|", float(du.max()))
    trd = np.any(a["tr"].view(np.int64) != b["tr"].view(np.int64), axis=(1, 2)) if a["tr"].ndim == 3 else None
    if trd is not None:
        print("instances with a trace difference:", int(trd.sum()))
    for i in bad[:12]:
        print(i, "ipm", a["st"]["ipm_iters"][i], b["st"]["ipm_iters"][i], "sqp", a["st"]["sqp_iter"][i], b["st"]["sqp_iter"][i],
              "status", a["out"]["status"][i], b["out"]["status"][i], "du0 %.3g" % du[i])
        ta, tb = a["tr"][i], b["tr"][i]
        for it in range(ta.shape[0]):
            if np.any(ta[it] != tb[it]):
                print("   it", it, "tail", np.array2string(ta[it], precision=17), "\n         ", np.array2string(tb[it], precision=17))


if __name__ == "__main__":
    main()
