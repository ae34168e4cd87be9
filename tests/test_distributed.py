"""Multi-process path on CPU (gloo, world_size 2): sharding + u0 gather reproduce the unsharded run.

Each rank solves its contiguous shard (the oracle stands in for the GPU engine here — test
infrastructure only) and the u0 blocks are all-gathered exactly as bench.py does over RCCL; rank 0
checks the gathered result bitwise against the unsharded solve.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpcc_manipulator_amd.distributed import gather_u0, max_over_ranks, shard_bounds


def test_shard_bounds_partition():
    for n in (0, 1, 7, 4096, 524288, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert sum(c for _, c in spans) == n
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        sys.path.insert(0, os.path.dirname(here))
        from helpers import SEED, batch_from_pool, make_oracle, oracle_pool
        o, _, _ = make_oracle(N=20, max_iter=2, mask=2)
        pool = oracle_pool(o, 30)
        x0, u0, obs, guess, valid, fails = batch_from_pool(pool, n_total, np.random.default_rng(SEED))
        start, count = shard_bounds(n_total, rank, world)
        sl = slice(start, start + count)
        out = o.run_mpc(x0[sl].copy(), u0[sl], obs[sl], guess[sl].copy(), valid[sl].copy(), fails[sl].copy())
        u_all = gather_u0(torch.from_numpy(out["u0"]), world)
        t = max_over_ranks(float(rank))
        if rank == 0:
            full = o.run_mpc(x0.copy(), u0, obs, guess.copy(), valid.copy(), fails.copy())
            result_q.put((bool(np.array_equal(u_all.numpy(), full["u0"])), t))
    finally:
        dist.destroy_process_group()


def test_sharded_solve_matches_unsharded(oracle_lib):
    world, n_total = 2, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    equal, tmax = q.get(timeout=10)
    assert equal
    assert tmax == 1.0
