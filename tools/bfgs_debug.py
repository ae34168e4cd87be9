"""Per-iteration SQP trace of the damped-BFGS option, engine vs oracle (debugging aid, GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import SEED, batch_from_pool, make_oracle, oracle_pool  # noqa: E402

import mpcc_manipulator_amd as m  # noqa: E402

OV = {"sqp": {"max_iter": 3, "use_BFGS": 1}}
mask, B = int(sys.argv[1]) if len(sys.argv) > 1 else 2, 64
o, P, track = make_oracle(N=20, max_iter=3, mask=mask, overrides=OV, nthreads=16)
pool = oracle_pool(o, 120)
rng = np.random.default_rng(SEED + 700 + mask)
x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng)
valid[::4] = 0
eng = m.Engine(m.load_params(N=20, overrides=OV), max_batch=B, constraint_mask=mask)
eng.set_track(*track)
eng.trace_enable(True)
eng.set_warmstart(guess, valid, fails)
outg = eng.solve(x0.copy(), u0, obs)
tg = eng.trace_get(B)
outo = o.run_mpc(x0.copy(), u0, obs, guess.copy(), valid.copy(), fails.copy(), trace=True)
to = outo["trace"]
d = np.abs(outg["horizon"] - outo["horizon"]).reshape(B, -1).max(1)
print("max du per instance:", np.round(d, 9).tolist())
print("sqp iters", outo["sqp_iters"].tolist())
for i in np.argsort(-d)[:3]:
    print("instance", i, "du", d[i])
    for it in range(3):
        print("  gpu", np.array2string(tg[i, it], precision=6), "\n  orc", np.array2string(to[i, it], precision=6))
