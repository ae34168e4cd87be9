"""Timing driver for the collision-MLP kernels (k_mlp_self / k_mlp_env) at configs[2] scale: robot
records for M (instance, stage) samples, repeated; run under rocprofv3 --kernel-trace --stats for the
per-kernel durations.  Also writes the records (gpurun_out/mlp_records_<tag>.npy) for a bitwise
comparison between engine builds.  GPU box:
    rocprofv3 --kernel-trace --stats -d gpurun_out/mlp -- python3 tools/mlp_bench.py --tag new
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpcc_manipulator_amd as m  # noqa: E402

Q0 = np.array([0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=65536 * 41 // 8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default="run")
    args = ap.parse_args()
    M = args.samples
    eng = m.Engine(m.load_params(N=20), max_batch=8, constraint_mask=7)
    rng = np.random.default_rng(0x4D504343)
    q = Q0 + rng.normal(0, 0.4, (M, 7))
    obs = np.column_stack([np.full(M, 0.48), np.full(M, 0.218), rng.uniform(0.421, 0.621, M), np.full(M, 5.0)])
    for _ in range(args.reps):
        rec = eng.robot_records(q, obs)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"mlp_records_{args.tag}.npy"), rec[:4096, 62:143])
    print("samples", M, "records", rec.shape)


if __name__ == "__main__":
    main()
