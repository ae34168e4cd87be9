"""Single-controller latency (B = 1, configs[1] settings): one control step (runMPC_ + simTimeStep) of
the device closed loop with and without hipGraph replay, and a host-buffer mpcc_solve call.
The reference budget is one sample period, Ts = 10 ms (Params/config.json).   python tools/latency.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mpcc_manipulator_amd as m  # noqa: E402


def main(steps=300):
    params = m.load_params(20, overrides={"sqp": {"max_iter": 2}})
    params.constraint_mask = 2
    pool, track = bench.make_pool(m, params, 2, 1000, 0)
    eng = m.Engine(params, max_batch=1, device=0, constraint_mask=2)
    eng.set_track(*track)
    x0 = np.zeros((1, 9)); x0[0, :7] = bench.Q0
    u0 = np.zeros((1, 8)); obs = np.array([[3.0, 3.0, 3.0, 0.0]])
    res = {}
    for graph in (False, True):
        eng.reset_warmstart(1)
        eng.closed_loop(x0, u0, obs, 5, graph=graph)  # warm up
        eng.reset_warmstart(1)
        t0 = time.perf_counter()
        out = eng.closed_loop(x0, u0, obs, steps, graph=graph)
        dt = time.perf_counter() - t0
        res["graph" if graph else "launches"] = dt / steps * 1e3
        res["solved_" + ("graph" if graph else "launches")] = int(np.sum(out["status"] == 0))
    eng.reset_warmstart(1)
    x = x0.copy(); u = u0.copy(); ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        o = eng.solve(x, u, obs)
        ts.append(time.perf_counter() - t0)
        u = o["u0"]
    res["host_solve_ms_median"] = float(np.median(ts) * 1e3)
    print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()})


if __name__ == "__main__":
    main()
