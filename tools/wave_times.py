"""Per-wave start / end times of one k_sqp launch (profiling build, s_memrealtime at 100 MHz), against the
wave's IPM iteration count: how long the bulk of a launch runs and how much of it is the tail.

    MPCC_PROF_BUILD=1 python -m mpcc_manipulator_amd._build
    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_prof/libmpcc_engine.so python tools/wave_times.py --batch 2048 4096
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
    ap.add_argument("--batch", type=int, nargs="+", default=[2048, 4096])
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mask", type=int, default=2)
    ap.add_argument("--obstacles", action="store_true", help="bench.py's obstacle scenario (--config 1-all-rows / 2)")
    args = ap.parse_args()
    import mpcc_manipulator_amd as m
    from mpcc_manipulator_amd.engine import lib
    L = lib()
    wt = L.mpcc_debug_wave_times
    params = m.load_params(args.N, overrides={"sqp": {"max_iter": 2}})
    params.constraint_mask = args.mask
    oxyz = (0.48, 0.218, 0.521)
    pool, track = bench.make_pool(m, params, args.mask, 1000, 0, (*oxyz, 5.0) if args.obstacles else (3., 3., 3., 0.))
    for B in args.batch:
        eng = m.Engine(params, max_batch=B, device=0, constraint_mask=args.mask)
        eng.set_track(*track)
        x0, u0, obs, g, v, f = bench.batch_inputs(pool, B, 7, args.obstacles, oxyz)
        a = (x0, u0, obs)
        ws = (g, v, f)
        for _ in range(3):
            eng.set_warmstart(*ws)
            eng.solve(*[v.copy() for v in a])
        solo = os.environ.get("MPCC_SOLO", "1") != "0"
        nw = (B + 3) // 4 + (64 if solo else 0)  # solo waves: the group slots map through eng.order
        slots = eng.order(4 * nw).reshape(-1, 4) if solo else np.arange(4 * nw).reshape(-1, 4)
        slots = np.where(slots < B, slots, -1)
        buf = (C.c_ulonglong * (2 * nw))()
        assert wt(buf, nw) == nw
        t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
        live = (slots >= 0).any(axis=1)  # waves with an instance (empty ones exit at once)
        st, en = t[:nw][live], t[nw:][live]
        slots = slots[live]
        t0 = st.min()
        st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0  # 100 MHz -> us
        stats = eng.solve_stats(B)
        ib = (C.c_int * B)()
        assert L.mpcc_debug_inst_ipm_iters(ib, B) == B
        its = np.frombuffer(ib, dtype=np.int32)  # IPM iterations summed over the instance's QPs
        it = np.where(slots >= 0, its[np.maximum(slots, 0)], 0)
        sq = np.where(slots >= 0, stats["sqp_iter"][np.maximum(slots, 0)], 0)
        nw = len(slots)
        wmax = it.max(axis=1)
        res = {"batch": B, "waves": nw, "launch_us": float(en_us.max()), "start_spread_us": float(st_us.max()),
               "end_quantiles_us": {q: float(np.percentile(en_us, q)) for q in (10, 50, 90, 99, 99.9, 100)},
               "waves_running_at_us": {int(x): int(((st_us <= x) & (en_us > x)).sum()) for x in
                                      np.linspace(0, en_us.max(), 12)}}
        by = {}
        for k in np.unique(wmax):
            sel = wmax == k
            by[int(k)] = {"waves": int(sel.sum()), "mean_end_us": round(float(en_us[sel].mean()), 1),
                          "max_end_us": round(float(en_us[sel].max()), 1), "two_qp": int((sq[sel].max(axis=1) >= 1).sum())}
        res["by_wave_max_ipm_iters"] = by
        print(json.dumps(res), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
