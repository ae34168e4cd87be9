"""Per-iteration trace of one low-rank QP: engine built with -DMPCC_IPM_TRACE vs the oracle's IPM debug log
(debugging aid, GPU box).  Usage: lr_trace.py CASE (unit-v | base1)"""
import os
import sys

os.environ["MPCC_ORACLE_IPM_DEBUG"] = "1"
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import SEED, make_oracle, oracle_pool  # noqa: E402

import mpcc_manipulator_amd as m  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "unit-v"
o, P, track = make_oracle(N=20, max_iter=2, mask=7, nthreads=1)
pool = oracle_pool(o, 40, obs=(0.48, 0.218, 0.521, 5.0))
eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=16, constraint_mask=7)
eng.set_track(*track)
N, B = 20, 1
guess = np.zeros((B, N + 1, 17)); recs = np.zeros((B, N + 1, 143)); ucur = np.zeros((B, 8))
guess[0] = pool["guess"][4]
ucur[0] = pool["u0"][4]
for k in range(N + 1):
    recs[0, k] = o.robot_record(guess[0, k, :7], (0.48, 0.218, 0.521), 5.0)
rng = np.random.default_rng(SEED)
base = rng.normal(0, 1, (4, N + 1, 17))
base[:, N, 9:] = 0
base = np.cumsum(base, axis=1) / np.sqrt(N + 1)
nrm = (base ** 2).reshape(4, -1).sum(1)
if case == "unit-v":
    lr = np.zeros((1, N + 1, 17)); lr[0, 10, 9] = 1.0; lrc = np.array([0.5])
else:
    lr = base[:1]; lrc = np.array([1.0]) / max(1.0, nrm[0])
step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
print("gpu status", st[0], "iters", it[0], flush=True)
rc0, s0, i0 = o.solve_qp_lr(guess[0], recs[0], ucur[0], lr, lrc, mode=0)
print("oracle status", rc0, "iters", i0, flush=True)
