"""Low-rank QP (damped-BFGS form) engine vs oracle for several term counts / signs (debugging aid, GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import SEED, make_oracle, oracle_pool  # noqa: E402

import mpcc_manipulator_amd as m  # noqa: E402

mask = int(sys.argv[1]) if len(sys.argv) > 1 else 7
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
o, P, track = make_oracle(N=20, max_iter=2, mask=mask, nthreads=16)
pool = oracle_pool(o, 40, obs=(0.48, 0.218, 0.521, 5.0))
eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=16, constraint_mask=mask)
eng.set_track(*track)
N = 20
guess = np.zeros((B, N + 1, 17)); recs = np.zeros((B, N + 1, 143)); ucur = np.zeros((B, 8))
for b in range(B):
    t = 3 + (b * 3) % 30
    guess[b] = pool["guess"][t + 1]
    ucur[b] = pool["u0"][t + 1]
    for k in range(N + 1):
        recs[b, k] = o.robot_record(guess[b, k, :7], (0.48, 0.218, 0.521), 5.0)
rng = np.random.default_rng(SEED)
base = rng.normal(0, 1, (4, N + 1, 17))
base[:, N, 9:] = 0
base = np.cumsum(base, axis=1) / np.sqrt(N + 1)
nrm = (base ** 2).reshape(4, -1).sum(1)
from test_bfgs import _lowrank_terms  # noqa: E402
def show(tag, lr, lrc):
    step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
    out = []
    for b in range(B):
        rc0, s0, i0 = o.solve_qp_lr(guess[b], recs[b], ucur[b], lr, lrc, mode=0)
        out.append((int(st[b]), rc0, int(it[b]), i0, float(np.abs(step[b] - s0).max()) if rc0 == 0 and st[b] == 0 else -1))
    print(tag, out, flush=True)
show("zero-u", np.zeros((1, N + 1, 17)), np.array([1.0]))
show("tiny-c", base[:1], np.array([1e-30]))
u1 = np.zeros((1, N + 1, 17)); u1[0, 10, 0] = 1.0
show("unit-y", u1, np.array([0.5]))
u2 = np.zeros((1, N + 1, 17)); u2[0, 10, 9] = 1.0
show("unit-v", u2, np.array([0.5]))
for nlr in (1, 2):
    lr, lrc = _lowrank_terms(o, np.random.default_rng(SEED + 730 + nlr), nlr)
    step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
    out = []
    for b in range(B):
        rc0, s0, i0 = o.solve_qp_lr(guess[b], recs[b], ucur[b], lr, lrc, mode=0)
        out.append((int(st[b]), rc0, int(it[b]), i0, float(np.abs(step[b] - s0).max()) if rc0 == 0 and st[b] == 0 else -1))
    print("test-like", nlr, lrc, out, flush=True)
for nlr, signs in [(1, "+"), (2, "++"), (2, "-+"), (3, "+++"), (3, "-+-"), (4, "++++"), (4, "-+-+"), (4, "+-+-")]:
    lr = base[:nlr]
    lrc = np.array([(1.0 if c == "+" else -0.02) for c in signs]) / np.maximum(1.0, nrm[:nlr])
    step, st, it = eng.solve_qp_lr(guess, recs, ucur, lr, lrc)
    res = []
    for b in range(B):
        rc0, s0, i0 = o.solve_qp_lr(guess[b], recs[b], ucur[b], lr, lrc, mode=0)
        res.append((int(st[b]), rc0, int(it[b]), i0, float(np.abs(step[b] - s0).max()) if rc0 == 0 and st[b] == 0 else -1))
    print(nlr, signs, res, flush=True)
