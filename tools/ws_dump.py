"""Dump the k_ipm workspace after one QP solve (debug builds capped at one IPM iteration), for
field-by-field comparison of two kernel variants.  Usage: MPCC_ENGINE_LIB=... python tools/ws_dump.py out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import SEED, make_oracle, oracle_pool  # noqa: E402
import mpcc_manipulator_amd as m  # noqa: E402

MASK = int(os.environ.get("WS_MASK", "7"))
o, P, track = make_oracle(N=20, max_iter=2, mask=MASK)
params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
eng = m.Engine(params, max_batch=8, constraint_mask=MASK)
eng.set_track(*track)
pool = oracle_pool(o, 40)
rng = np.random.default_rng(SEED + 2)
B, N = 4, 20
guess = np.zeros((B, N + 1, 17)); recs = np.zeros((B, N + 1, 143)); ucur = np.zeros((B, 8))
for b in range(B):
    t = 5 + b * 7
    g = pool["guess"][t + 1].copy()
    g[:, :7] += rng.normal(0, 0.01, (N + 1, 7)); g[:N, 9:] += rng.normal(0, 0.05, (N, 8))
    guess[b] = g; ucur[b] = pool["u0"][t + 1]
    for k in range(N + 1):
        recs[b, k] = o.robot_record(g[k, :7])
step, st, it = eng.solve_qp(guess, recs, ucur)
ws = eng.workspace(B)
np.savez(sys.argv[1], ws=ws, step=step, st=st, it=it)
print("status", st, "iters", it)
