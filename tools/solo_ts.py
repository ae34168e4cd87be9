"""Timeline of the solo blocks (k_sqp_solo) of one configs[1] group solve: per cold-started instance, the time from the
block's entry to the end of its first QP records, and of each SQP iteration's QP records / QP solve / line search and step
(s_memrealtime, 100 MHz).  Needs an engine built with -DMPCC_SOLO_TS (tools/ab_build.sh NAME -DMPCC_SOLO_TS=1).

    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_ab/NAME/libmpcc_engine.so python tools/solo_ts.py --batch 2048
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
    f = L.mpcc_debug_solo_ts
    f.argtypes = [C.POINTER(C.c_ulonglong)]
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
    buf = (C.c_ulonglong * (64 * 8))()
    for _ in range(4):
        eng.set_warmstart(*ws)
        eng.solve(*[v.copy() for v in a])
    assert f(buf) == 0
    ts = np.frombuffer(buf, dtype=np.uint64).reshape(64, 8).astype(np.int64)
    names = ["prep_done", "qp_records_0", "qp_0", "step_0", "qp_records_1", "qp_1", "step_1"]
    out = []
    for r in range(64):
        if ts[r, 0] == 0:
            continue
        row = {n: round((ts[r, i + 1] - ts[r, 0]) / 100.0, 1) if ts[r, i + 1] >= ts[r, 0] else None
               for i, n in enumerate(names)}
        out.append({"block": r, "us_from_entry": row})
    print(json.dumps({"batch": B, "solo_blocks": out}))
    eng.close()


if __name__ == "__main__":
    main()
