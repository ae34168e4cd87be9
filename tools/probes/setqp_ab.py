"""Engine outputs of the filter-rejection batch (tests/test_filter_rejection.py, mask 2) from two engine libraries,
each in its own process: trace columns, status, horizon; compared bitwise and against the oracle.

    python tools/probes/setqp_ab.py LIB_A LIB_B
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mpcc_manipulator_amd as m
    from test_filter_rejection import _batch
    o, track, (x0, u0, ob, g, v, f) = _batch(2, 512)
    out_o = o.run_mpc(x0.copy(), u0, ob, g.copy(), v.copy(), f.copy(), trace=True)
    eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=512, constraint_mask=2)
    eng.set_track(*track)
    eng.set_warmstart(g, v, f)
    eng.trace_enable(True)
    out_g = eng.solve(x0.copy(), u0, ob)
    trg = eng.trace_get(512)
    np.savez(out, trace=trg, status=out_g["status"], horizon=out_g["horizon"], otrace=out_o["trace"],
             ostatus=out_o["status"], ohorizon=out_o["horizon"])


if __name__ == "__main__":
    if len(sys.argv) == 2:
        run(sys.argv[1])
        sys.exit(0)
    res = []
    for i, lib in enumerate(sys.argv[1:3]):
        out = os.path.join(ROOT, "gpurun_out", f"setqp_ab_{i}.npz")
        subprocess.run([sys.executable, __file__, out], check=True, env=dict(os.environ, MPCC_ENGINE_LIB=lib))
        res.append(np.load(out))
    a, b = res
    for i, r in enumerate(res):
        d = np.abs(r["trace"][:, :, 2] - r["otrace"][:, :, 2]) / np.maximum(1.0, np.abs(r["otrace"][:, :, 2]))
        w = np.unravel_index(np.argmax(d), d.shape)
        print(f"lib {i}: trial-objective rel diff vs oracle max {d.max():.3e} at {w}, engine {r['trace'][w][2]!r} "
              f"oracle {r['otrace'][w][2]!r}, trace row {r['trace'][w].tolist()} oracle row {r['otrace'][w].tolist()}")
        print(f"lib {i}: status equal {np.array_equal(r['status'], r['ostatus'])}, horizon max diff "
              f"{np.abs(r['horizon'] - r['ohorizon']).max():.3e}")
    print("A vs B: trace bitwise", np.array_equal(a["trace"].view(np.int64), b["trace"].view(np.int64)),
          "horizon bitwise", np.array_equal(a["horizon"].view(np.int64), b["horizon"].view(np.int64)),
          "horizon max diff", float(np.abs(a["horizon"] - b["horizon"]).max()))
