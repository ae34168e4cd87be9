"""MLP outputs of the engine (k_mlp_self / k_mlp_env) vs the oracle on seeded inputs: exact-equality
counts and max relative difference per record field group.  GPU box: python tools/mlp_check.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import Q0, SEED, make_oracle  # noqa: E402
import mpcc_manipulator_amd as m  # noqa: E402

o, P, track = make_oracle(N=20, max_iter=2, mask=7)
eng = m.Engine(m.load_params(N=20), max_batch=8, constraint_mask=7)
rng = np.random.default_rng(SEED + 77)
M = 257
q = Q0 + rng.normal(0, 0.4, (M, 7))
obs = np.column_stack([np.full(M, 0.48), np.full(M, 0.218), rng.uniform(0.421, 0.621, M), np.full(M, 5.0)])
rg = eng.robot_records(q, obs)
ro = np.stack([o.robot_record(q[i], obs[i, :3], obs[i, 3]) for i in range(M)])
for name, sl in [("self d", slice(62, 63)), ("self grad", slice(63, 70)), ("env d", slice(71, 80)), ("env jac", slice(80, 143))]:
    a, b = rg[:, sl], ro[:, sl]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    print(f"{name:10s} exact {np.mean(a == b) * 100:6.2f}%  max rel {rel.max():.3e}")
