"""Collision-MLP records of the loaded engine library for seeded inputs, saved for a bitwise comparison between two
builds (A/B of mlp.hip variants that must not change a bit: LDS rings, block shapes).  GPU box:

    python tools/mlp_bitwise.py gpurun_out/a.npz [M ...]
    MPCC_ENGINE_LIB=.../_ab/X/libmpcc_engine.so python tools/mlp_bitwise.py gpurun_out/b.npz
    python tools/mlp_bitwise.py --compare gpurun_out/a.npz gpurun_out/b.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        ok = True
        for k in a.files:
            eq = np.array_equal(a[k].view(np.uint64), b[k].view(np.uint64))
            print(f"{k}: {a[k].shape} bitwise {'equal' if eq else 'DIFFERENT'}")
            ok = ok and eq
        sys.exit(0 if ok else 1)
    import mpcc_manipulator_amd as m
    out = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:]] or [4096, 300000]  # short launches (two-wave env blocks) and long ones
    eng = m.Engine(m.load_params(N=20), max_batch=8, constraint_mask=7)
    rng = np.random.default_rng(0x4D504343 + 91)
    q0 = np.array([0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4])
    res = {}
    for M in sizes:
        q = q0 + rng.normal(0, 0.4, (M, 7))
        obs = np.column_stack([np.full(M, 0.48), np.full(M, 0.218), rng.uniform(0.421, 0.621, M), np.full(M, 5.0)])
        rec = eng.robot_records(q, obs)
        res[f"M{M}"] = rec[:, 62:143].copy()  # self distance + gradient, env distances + Jacobian
    eng.close()
    np.savez(out, **res)
    print("saved", out, {k: v.shape for k, v in res.items()})


if __name__ == "__main__":
    main()
