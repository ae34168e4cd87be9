"""Multi-rank bench path (BASELINE configs[4]) and the per-GPU share of configs[4].

CPU tests: `bench.py --gpus N` refuses to run on fewer GPUs than asked and refuses a launcher whose
WORLD_SIZE disagrees with --gpus (it used to run one rank on GPU 0 and report n_gpus = 1).

GPU tests:
  * a 2-rank rehearsal of `bench.py --gpus 2` (MPCC_BENCH_REHEARSE=1: both ranks on GPU 0, gloo) runs
    the HIP engine on each rank's contiguous shard and all-gathers u0; the gathered u0 is bitwise the
    one-process solve of the same global batch (instances are independent, mpc.h:119-127);
  * configs[4]'s per-GPU share (B = 65,536, N = 20, bounds + singularity rows) at full size with the
    size-independent properties of test_config2_full_scale plus a seeded oracle sample;
  * the device entry points reject tensors the kernels would read out of bounds.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import SEED, batch_from_pool, make_oracle, oracle_pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run_bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "MPCC_BENCH_REHEARSE"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_refuses_missing_gpus():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _run_bench(["--gpus", str(n), "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr


def test_bench_refuses_world_mismatch():
    r = _run_bench(["--gpus", "1", "--steps", "1"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"},
                   timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_matches_single_process(built_lib, tmp_path):
    """2 ranks x 256 instances (gloo rehearsal on GPU 0) == 1 rank x 512 instances, bitwise."""
    u2, u1 = str(tmp_path / "u2.npy"), str(tmp_path / "u1.npy")
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--pool-steps", "1000"]
    r2 = _run_bench(["--gpus", "2", "--batch", "256", "--dump-u0", u2] + common, {"MPCC_BENCH_REHEARSE": "1"})
    assert r2.returncode == 0, r2.stderr[-3000:]
    line = json.loads(r2.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 512 and line["value"] > 0
    r1 = _run_bench(["--gpus", "1", "--batch", "512", "--dump-u0", u1] + common)
    assert r1.returncode == 0, r1.stderr[-3000:]
    a, b = np.load(u2), np.load(u1)
    assert a.shape == b.shape == (512, 8)
    assert np.array_equal(a, b), float(np.abs(a - b).max())


@pytest.mark.gpu
def test_config4_share_full_scale(built_lib, oracle_lib):
    """configs[4]'s per-GPU share at full size: B = 65,536, N = 20, mask 2 (configs[1] settings).
    (1) instance independence: a random subset re-solved alone is bitwise its rows of the full batch;
    (2) every output finite with a valid status; (3) a seeded 64-instance sample matches the oracle
    (status exact, u <= 1e-6, x0 update <= 1e-9, controller state exact)."""
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=2, nthreads=16)
    pool = oracle_pool(o, 200)
    B = 65536
    rng = np.random.default_rng(SEED + 524288)
    x0, u0, obs, guess, valid, fails = batch_from_pool(pool, B, rng)
    eng = m.Engine(m.load_params(N=20, overrides={"sqp": {"max_iter": 2}}), max_batch=B, constraint_mask=2)
    eng.set_track(*track)
    eng.set_warmstart(guess, valid, fails)
    xf = x0.copy()
    full = eng.solve(xf, u0, obs)
    gf, vf, ff = eng.get_warmstart(B)
    assert np.all(np.isfinite(full["horizon"])) and np.all(np.isfinite(xf))
    assert set(np.unique(full["status"]).tolist()) <= {0, 1, 10, 11}
    assert np.mean(full["status"] == 0) > 0.99
    sub = np.sort(rng.choice(B, 256, replace=False))
    eng.set_warmstart(guess[sub], valid[sub], fails[sub])
    xs = x0[sub].copy()
    part = eng.solve(xs, u0[sub], obs[sub])
    gs, vs, fs = eng.get_warmstart(len(sub))
    assert np.array_equal(part["status"], full["status"][sub])
    assert np.array_equal(part["horizon"], full["horizon"][sub]) and np.array_equal(xs, xf[sub])
    assert np.array_equal(gs, gf[sub]) and np.array_equal(vs, vf[sub]) and np.array_equal(fs, ff[sub])
    smp = sub[:64]
    xo = x0[smp].copy(); go = guess[smp].copy(); vo = valid[smp].copy(); fo = fails[smp].copy()
    outo = o.run_mpc(xo, u0[smp], obs[smp], go, vo, fo)
    assert np.array_equal(outo["status"], full["status"][smp])
    assert np.abs(outo["horizon"][:, :-1, 9:] - full["horizon"][smp, :-1, 9:]).max() <= 1e-6
    assert np.abs(xo - xf[smp]).max() <= 1e-9
    assert np.array_equal(vo, vf[smp]) and np.array_equal(fo, ff[smp])
    eng.close()


@pytest.mark.gpu
def test_device_entry_points_check_tensors(built_lib):
    import torch
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
    eng = m.Engine(params, max_batch=8, constraint_mask=2)
    X, Y, Z, q = m.load_default_track()
    eng.set_track(*m.track_from_points(X, Y, Z, q, np.array([0.5545, 0.0, 0.5211])))
    dev = torch.device("cuda", 0)
    x0 = torch.zeros((8, 9), dtype=torch.float64, device=dev)
    u0 = torch.zeros((8, 8), dtype=torch.float64, device=dev)
    obs = torch.zeros((8, 4), dtype=torch.float64, device=dev)
    bad = [
        dict(x0=x0.float()),                                   # wrong dtype
        dict(x0=x0[:4]),                                       # fewer rows than B
        dict(u0=torch.zeros((8, 16), dtype=torch.float64, device=dev)[:, ::2]),  # not contiguous
        dict(obs=obs.cpu()),                                   # host tensor
    ]
    for kw in bad:
        a = dict(x0=x0, u0=u0, obs=obs)
        a.update(kw)
        with pytest.raises(m.MpccError):
            eng.solve_device(8, a["x0"], a["u0"], a["obs"])
    with pytest.raises(m.MpccError):
        eng.solve_device(9, x0, u0, obs)  # more than max_batch
    with pytest.raises(m.MpccError):
        eng.set_warmstart_device(8, torch.zeros((8, 21, 17), dtype=torch.float32, device=dev), None, None)
    eng.solve_device(8, x0, u0, obs)  # the well-formed call still runs
    torch.cuda.synchronize()
    eng.close()


RCCL_WORLD1 = r"""
import os, sys, json
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["MPCC_ROOT"])
sys.path.insert(0, os.path.join(os.environ["MPCC_ROOT"], "tests"))
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["MPCC_PORT"], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
import mpcc_manipulator_amd as m
from mpcc_manipulator_amd.distributed import check_equal_shards, gather_u0, max_over_ranks
from helpers import Q0
dev = torch.device("cuda", 0)
B = 64
params = m.load_params(N=20, overrides={"sqp": {"max_iter": 2}})
eng = m.Engine(params, max_batch=B, constraint_mask=2)
X, Y, Z, q = m.load_default_track()
eng.set_track(*m.track_from_points(X, Y, Z, q, np.array([0.5545, 0.0, 0.5211])))
rng = np.random.default_rng(7)
x0 = np.zeros((B, 9)); x0[:, :7] = Q0 + rng.normal(0, 0.002, (B, 7))
xd = torch.from_numpy(x0).to(dev)
u0 = torch.zeros((B, 8), dtype=torch.float64, device=dev)
obs = torch.tensor([[3.0, 3.0, 3.0, 0.0]] * B, dtype=torch.float64, device=dev)
uo = torch.empty((B, 8), dtype=torch.float64, device=dev)
check_equal_shards(B, device=dev)  # all_reduce over RCCL
eng.solve_device(B, xd, u0, obs, uo)
torch.cuda.synchronize()
out = torch.full((B, 8), float("nan"), dtype=torch.float64, device=dev)
g = gather_u0(uo, 1, out=out)  # all_gather_into_tensor over RCCL
t = max_over_ranks(1.25, device=dev)
torch.cuda.synchronize()
ok = g.data_ptr() == out.data_ptr() and torch.equal(out, uo) and t == 1.25 and bool(torch.isfinite(uo).all())
print(json.dumps({"ok": bool(ok), "backend": dist.get_backend(), "max_abs_u0": float(uo.abs().max())}))
eng.close()
dist.destroy_process_group()
"""


@pytest.mark.gpu
def test_rccl_world1_gather(built_lib):
    """The RCCL ("nccl") branch of the multi-GPU path, executed: a world-size-1 process group on GPU 0 runs
    check_equal_shards (all_reduce), gather_u0 (all_gather_into_tensor of the engine's u0) and max_over_ranks
    through RCCL; the gathered u0 equals the solve's output bitwise.  2+ ranks over RCCL need one GPU per rank
    (the driver's 8-GPU runs)."""
    env = dict(os.environ, MPCC_ROOT=ROOT, MPCC_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", RCCL_WORLD1], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"] and res["backend"] == "nccl", res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
