"""Bitwise check of the mobile build's two-pass env MLP (mlp.hip ENV_SPLIT) against the one-tile form: the stage
records (both MLPs, value and every Jacobian column) of the same seeded samples from the regular mobile library and
from a variant built with -DMPCC_ENV_SPLIT=0 (mpcc_manipulator_amd/_ab/envsplit0), each in its own process.

    python tools/probes/env_split_bitwise.py            # runs both and compares

The variant library (built in this container, it travels to the GPU box with the tree):

    cd mpcc_manipulator_amd && mkdir -p _ab/envsplit0 && \\
    hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I ../include -I csrc -ffp-contract=off -DMPCC_DOF=10 \\
          -Dmpcc=mpcc_m10 -DMPCC_ENV_SPLIT=0 -c csrc/mlp.hip -o _ab/envsplit0/mlp_mobile.o && \\
    hipcc --offload-arch=gfx950 -shared -fPIC -o _ab/envsplit0/libmpcc_engine_mobile.so _build/kernels_mobile.o \\
          _build/ipm_wide_mobile.o _ab/envsplit0/mlp_mobile.o _build/nn_generic_mobile.o _build/engine_mobile.o \\
          _build/host_params_mobile.o _build/host_spline_mobile.o
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def records(out):
    sys.path.insert(0, ROOT)
    import mpcc_manipulator_amd as m
    rng = np.random.default_rng(2024)
    M = 8192
    eng = m.Engine(m.load_params(N=30, dof=10), max_batch=64, constraint_mask=7)
    q0 = np.array([0.3, -0.2, 0.4, 0.0, -0.3, 0.0, -2.0, 0.0, 1.8, 0.8])
    q = q0 + rng.normal(0, 0.4, size=(M, 10))
    obs = np.column_stack([rng.uniform(-0.5, 1.0, M), rng.uniform(-0.5, 0.8, M), rng.uniform(0.2, 0.9, M),
                           np.full(M, 0.05)])
    np.save(out, eng.robot_records(q, obs))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        records(sys.argv[1])
        sys.exit(0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    a, b = os.path.join(ROOT, "gpurun_out", "env_split1.npy"), os.path.join(ROOT, "gpurun_out", "env_split0.npy")
    subprocess.run([sys.executable, __file__, a], check=True)
    env = dict(os.environ, MPCC_ENGINE_LIB_MOBILE=os.path.join(ROOT, "mpcc_manipulator_amd", "_ab", "envsplit0",
                                                                "libmpcc_engine_mobile.so"))
    subprocess.run([sys.executable, __file__, b], check=True, env=env)
    ra, rb = np.load(a), np.load(b)
    diff = np.argwhere(ra.view(np.int64) != rb.view(np.int64))
    print({"samples": ra.shape[0], "fields": ra.shape[1], "bitwise_equal": bool(diff.size == 0),
           "differing_entries": int(diff.shape[0]), "max_abs_diff": float(np.nanmax(np.abs(ra - rb)))})
    sys.exit(0 if diff.size == 0 else 1)
