"""Where a solo wave's time goes (k_sqp, profiling build): cycles per SQP-loop phase of the waves holding one
instance (the cold starts), per wave.
    MPCC_PROF_BUILD=1 python -m mpcc_manipulator_amd._build
    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so python tools/solo_prof.py --batch 2048
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    args = ap.parse_args()
    import mpcc_manipulator_amd as m
    from mpcc_manipulator_amd.engine import lib
    L = lib()
    f = L.mpcc_debug_solo_prof
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    params = m.load_params(20, overrides={"sqp": {"max_iter": 2}})
    params.constraint_mask = 2
    pool, track = bench.make_pool(m, params, 2, 1000, 0)
    B = args.batch
    eng = m.Engine(params, max_batch=B, device=0, constraint_mask=2)
    eng.set_track(*track)
    rng = np.random.default_rng(bench.SEED)
    idx = np.arange(B) % len(pool["x0"])
    x0 = pool["x0"][idx].copy()
    x0[:, :7] += rng.normal(0, 0.005, (4096 if B <= 4096 else B, 7))[:B]
    a = (x0, pool["u0"][idx], np.tile([3., 3., 3., 0.], (B, 1)))
    ws = (pool["guess"][idx], pool["valid"][idx].astype(np.int32), pool["fails"][idx].astype(np.int32))
    buf = (C.c_ulonglong * 8)()
    for _ in range(3):
        f(buf, 1)
        eng.set_warmstart(*ws)
        eng.solve(*[v.copy() for v in a])
    f(buf, 0)
    v = np.frombuffer(buf, dtype=np.uint64).astype(float)
    nw = max(1.0, v[5])
    names = ["setqp", "qp_solve", "trial", "accept", "step_and_rest"]
    print(json.dumps({"solo_waves": int(v[5]), "sqp_iters_per_wave": v[6] / nw,
                      "kcycles_per_wave": {n: round(v[i] / nw / 1e3, 2) for i, n in enumerate(names)},
                      "kcycles_total_per_wave": round(v[:5].sum() / nw / 1e3, 2)}))
    eng.close()


if __name__ == "__main__":
    main()
