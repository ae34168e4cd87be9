"""Benchmark state pool: the reference's closed loop from x0 = [q0, 0, 0]
(main.cpp:60-63, 100-114) at configs[1] settings (N=20, bounds + singularity rows, 2 SQP iterations),
1000 control steps; per step the controller inputs (x0 before projection, u0, warm start).

Written to mpcc_manipulator_amd/data/bench_pool_n20_mask2.npz (synthetic input data for bench.py, so
the timed k_ipm launches are the only ones of that kernel in a profile of the bench command).
The closed loop is run with the oracle; the engine reproduces it (tests/test_gpu_parity.py).

    python tools/make_bench_pool.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_oracle, oracle_pool  # noqa: E402


def main(steps=1000, N=20, mask=2):
    o, P, track = make_oracle(N=N, max_iter=2, mask=mask)
    pool = oracle_pool(o, steps)
    out = os.path.join(ROOT, "mpcc_manipulator_amd", "data", f"bench_pool_n{N}_mask{mask}.npz")
    np.savez_compressed(out, x0=pool["x0"], u0=pool["u0"], guess=pool["guess"],
                        valid=pool["valid"].astype(np.int32), fails=pool["fails"].astype(np.int32),
                        status=pool["status"].astype(np.int32))
    print(out, os.path.getsize(out), "bytes; solved", int(np.sum(pool["status"] == 0)), "/", steps)


if __name__ == "__main__":
    main()
