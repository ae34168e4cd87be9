"""Cycle accounting of k_ipm sections (profiling build: MPCC_PROF_BUILD=1 python -m mpcc_manipulator_amd._build).

    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so python tools/ipm_prof.py --batch 512
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

SECTIONS = ["setup", "fload", "factor_rest", "pred_fwd", "corr_bwd", "corr_fwd", "-", "-", "f_update", "f_slots_g0", "f_Y_Hb_F_Gm", "f_chol_solves", "f_stores", "f_P"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[256, 512, 1024, 4096])
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mask", type=int, default=2)
    ap.add_argument("--obstacles", action="store_true", help="bench.py's obstacle scenario (--config 1-all-rows / 2)")
    args = ap.parse_args()
    import torch
    import mpcc_manipulator_amd as m
    from mpcc_manipulator_amd.engine import lib
    L = lib()
    prof = getattr(L, "mpcc_debug_ipm_prof", None)
    params = m.load_params(args.N, overrides={"sqp": {"max_iter": 2}})
    params.constraint_mask = args.mask
    oxyz = (0.48, 0.218, 0.521)
    pool, track = bench.make_pool(m, params, args.mask, 1000, 0, (*oxyz, 5.0) if args.obstacles else (3., 3., 3., 0.))
    for B in args.batch:
        eng = m.Engine(params, max_batch=B, device=0, constraint_mask=args.mask)
        eng.set_track(*track)
        x0, u0, obs, g, v, f = bench.batch_inputs(pool, B, 7, args.obstacles, oxyz)
        args_ = (x0, u0, obs)
        ws = (g, v, f)
        for rep in range(3):
            eng.set_warmstart(*ws)
            if rep == 2 and prof:
                buf = (C.c_ulonglong * 16)()
                prof(buf, 1)
                if getattr(L, "mpcc_debug_tail_prof", None):
                    L.mpcc_debug_tail_prof((C.c_ulonglong * 16)(), 1)
            eng.timing_begin()
            out = eng.solve(*[a.copy() for a in args_])
            tm, ncalls, nipm = eng.timing_end()
        res = {"batch": B, "solve_qp_ms": tm["solve_qp"] * 1e3, "ipm_launches": nipm, "total_ms": tm["total"] * 1e3}
        if prof:
            buf = (C.c_ulonglong * 16)()
            prof(buf, 0)
            n_inst, n_it = buf[7], buf[6]
            res["instances"] = n_inst
            res["ipm_iters"] = n_it
            res["kcycles_per_iter"] = {s: round(buf[i] / max(1, n_it) / 1e3, 2) for i, s in enumerate(SECTIONS) if s != "-"}
        tp = getattr(L, "mpcc_debug_tail_prof", None)
        if tp:
            tb = (C.c_ulonglong * 16)()
            tp(tb, 1)
            nt = max(1, tb[7])
            res["tail_iters"] = int(tb[7])
            res["tail_kcycles_per_iter"] = {s: round(tb[i] / nt / 1e3, 2) for i, s in enumerate(
                ["f_A", "f_B_rest", "f_C", "f_D", "pred_D", "corr_bwd", "corr_fwd", "-", "fB_Y_F_Gm", "fB_chol",
                 "fB_u_export", "fB_hb", "fB_P", "pred_A_loads", "pred_B_chain", "pred_C_slots"]) if s != "-"}
        print(json.dumps(res), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
