import sys, os, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
from helpers import SEED, batch_from_pool, make_oracle, oracle_pool
import mpcc_manipulator_amd as m
o, P, track = make_oracle(N=20, max_iter=2, mask=2)
params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
eng = m.Engine(params, max_batch=16, constraint_mask=2)
eng.set_track(*track)
pool = oracle_pool(o, 400)
rng = np.random.default_rng(SEED + 11)
x0, u0, obs, guess, valid, fails = batch_from_pool(pool, 4096, rng)
idx = [979, 1782, 175, 176, 966, 967, 1394, 0, 1, 2]
sg = x0[idx, 7]
ee = np.array([o.fk(x0[i, :7])[0] for i in idx])
sgpu = eng.project(sg, ee)
for j, i in enumerate(idx):
    so = o.project(sg[j], ee[j])
    pp = o.spline_eval(sg[j])[0]
    print(i, "s_guess", sg[j], "dist", np.linalg.norm(ee[j] - pp), "gpu", sgpu[j], "oracle", so)
print("proj_max_dist engine", params.proj_max_dist, "oracle", P.get("proj_max_dist"))

def newton(ev, s, e, L):
    out = []
    s_old = s
    for it in range(20):
        p, dp, ddp = ev(s)
        d = p - e
        jac = 2.0 * d[0] * dp[0] + 2.0 * d[1] * dp[1] + 2.0 * d[2] * dp[2]
        hes = 2.0 * dp[0] * dp[0] + 2.0 * d[0] * ddp[0] + 2.0 * dp[1] * dp[1] + 2.0 * d[1] * ddp[1] + 2.0 * dp[2] * dp[2] + 2.0 * d[2] * ddp[2]
        s = s - jac / hes
        s = max(0.0, min(s, L))
        out.append((s, jac, hes))
        if abs(s_old - s) <= 1e-5:
            break
        s_old = s
    return out

def ev_o(s):
    p, dp, ddp, _, _ = o.spline_eval(s)
    return np.array(p), np.array(dp), np.array(ddp)

def ev_g(s):
    p, d1, d2, _, _ = eng.spline_eval(np.array([s]))
    return p[0], d1[0], d2[0]

L = o.track_length()
e = ee[0]
to = newton(ev_o, 0.0, e, L)
tg = newton(ev_g, 0.0, e, L)
for k in range(max(len(to), len(tg))):
    a = to[k] if k < len(to) else None
    b = tg[k] if k < len(tg) else None
    print(k, "oracle", a, "gpu", b)
