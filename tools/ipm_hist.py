"""IPM iteration distribution of the benchmark workload, on the oracle (CPU): the QP solves of one
configs[1] step (bench.py's instances: pool step i mod 1000, q + N(0, 0.005), bench.py's seed).

A k_sqp launch lasts as long as its slowest wave, so the tail of this distribution (per instance: the
sum over its SQP iterations; per wave: the max over its 4 instances) sets the kernel time.

    python tools/ipm_hist.py [--batch 4096 --threads 8]
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
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mask", type=int, default=2)
    ap.add_argument("--pool", type=int, default=400, help="closed-loop pool steps when no committed pool exists")
    ap.add_argument("--obstacles", action="store_true", help="configs[2] obstacles (main_w_sim.py:42-45)")
    args = ap.parse_args()
    from helpers import make_oracle, oracle_pool
    o, P, track = make_oracle(N=args.N, max_iter=2, mask=args.mask, nthreads=args.threads)
    path = os.path.join(ROOT, "mpcc_manipulator_amd", "data", f"bench_pool_n{args.N}_mask{args.mask}.npz")
    if os.path.exists(path):
        f = np.load(path, allow_pickle=False)
        pool = {k: f[k] for k in f.files}
    else:
        pool = oracle_pool(o, args.pool, obs=(0.48, 0.218, 0.521, 5.0) if args.obstacles else (3.0, 3.0, 3.0, 0.0))
    B = args.batch
    rng = np.random.default_rng(0x4D504343)
    idx = np.arange(B) % len(pool["x0"])
    x0 = pool["x0"][idx].copy()
    x0[:, :7] += rng.normal(0.0, 0.005, size=(B, 7))
    u0 = pool["u0"][idx].copy()
    guess = np.ascontiguousarray(pool["guess"][idx])
    valid = pool["valid"][idx].astype(np.int32)
    fails = pool["fails"][idx].astype(np.int32)
    obs = np.tile(np.array([3.0, 3.0, 3.0, 0.0]), (B, 1))
    if args.obstacles:
        obs = np.column_stack([np.full(B, 0.48), np.full(B, 0.218), rng.uniform(0.421, 0.621, B), np.full(B, 5.0)])
    out = o.run_mpc(x0, u0, obs, guess, valid, fails, trace=True)
    tr = out["trace"]
    it1 = tr[:, 0, 1].astype(int)
    it2 = np.where(out["sqp_iters"] >= 1, tr[:, 1, 1], 0).astype(int)
    tot = it1 + it2
    wave = tot.reshape(-1, 4).max(axis=1)
    print("first QP iterations: mean %.2f max %d" % (it1.mean(), it1.max()))
    print("per instance total:  mean %.2f p99 %d max %d" % (tot.mean(), np.percentile(tot, 99), tot.max()))
    print("per wave max:        mean %.2f max %d" % (wave.mean(), wave.max()))
    print("histogram (total iterations: instances):",
          {int(k): int(v) for k, v in zip(*np.unique(tot, return_counts=True))})
    worst = np.argsort(-tot)[:10]
    print("worst (instance, it1, it2, sqp_iters, qp status 1, 2):",
          [(int(i), int(it1[i]), int(it2[i]), int(out["sqp_iters"][i]), int(tr[i, 0, 0]), int(tr[i, 1, 0])) for i in worst])


if __name__ == "__main__":
    main()
