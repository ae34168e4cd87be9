"""One low-rank QP (tests/test_bfgs.py::test_lowrank_qp_step setup, instance 0) on the GPU (a library built with
-DMPCC_IPM_TRACE: per-iteration printf) and in the oracle (MPCC_ORACLE_IPM_DEBUG=1): where the two interior
points part.  python tools/lr_debug.py NLR"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    nlr = int(sys.argv[1])
    import mpcc_manipulator_amd as m
    from helpers import SEED, make_oracle, oracle_pool
    from test_bfgs import _lowrank_terms
    o, P, track = make_oracle(N=20, max_iter=2, mask=7, nthreads=1)
    pool = oracle_pool(o, 40, obs=(0.48, 0.218, 0.521, 5.0))
    eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=16, constraint_mask=7)
    eng.set_track(*track)
    rng = np.random.default_rng(SEED + 730 + nlr)
    B, N = 1, 20
    guess = np.zeros((B, N + 1, 17)); recs = np.zeros((B, N + 1, 143)); ucur = np.zeros((B, 8))
    t = 3
    guess[0] = pool["guess"][t + 1]
    ucur[0] = pool["u0"][t + 1]
    for k in range(N + 1):
        recs[0, k] = o.robot_record(guess[0, k, :7], (0.48, 0.218, 0.521), 5.0)
    lr, lrc = _lowrank_terms(o, rng, nlr)
    step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
    print("gpu status", st[0], "iters", it[0], flush=True)
    rc0, s0, it0 = o.solve_qp_lr(guess[0], recs[0], ucur[0], lr, lrc, mode=0)
    print("oracle status", rc0, "iters", it0, "max|dstep|", float(np.abs(step[0] - s0).max()), flush=True)


if __name__ == "__main__":
    main()
