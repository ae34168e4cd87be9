"""Sub-batch pipelining probe: configs[1] (B = 4096 total, N = 20, mask 2) as S independent engines of B/S
instances, each stepping on its own HIP stream, so that one sub-batch's next control step can start while another
finishes its interior-point tail.  Prints solves/s for each S and checks that the outputs equal the S = 1 solve
bitwise (instances are independent, mpc.h:119-127).

    python tools/pipeline_probe.py --subs 1 2 4 --steps 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subs", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timing", action="store_true", help="engines in live-timing mode (HIP events around launches)")
    args = ap.parse_args()
    import torch
    import mpcc_manipulator_amd as m
    B, N, mask = args.batch, 20, 2
    params = m.load_params(N, overrides={"sqp": {"max_iter": 2}})
    params.constraint_mask = mask
    pool, track = bench.make_pool(m, params, mask, 1000, 0)
    rng = np.random.default_rng(bench.SEED)
    idx = np.arange(B) % len(pool["x0"])
    x0 = pool["x0"][idx].copy()
    x0[:, :7] += rng.normal(0.0, 0.005, size=(B, 7))
    u0, g, v, f = pool["u0"][idx], pool["guess"][idx], pool["valid"][idx].astype(np.int32), pool["fails"][idx].astype(np.int32)
    obs = np.tile(np.array([3.0, 3.0, 3.0, 0.0]), (B, 1))
    dev = torch.device("cuda", 0)
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    ref = None
    res = {}
    for S in args.subs:
        Bs = B // S
        engs, st, bufs = [], [], []
        for s in range(S):
            sl = slice(s * Bs, (s + 1) * Bs)
            e = m.Engine(params, max_batch=Bs, device=0, constraint_mask=mask)
            e.set_track(*track)
            engs.append(e)
            st.append(torch.cuda.Stream(dev))
            bufs.append(dict(x0p=T(x0[sl]), x0=T(x0[sl]), u0=T(u0[sl]), obs=T(obs[sl]), g=T(g[sl]),
                             v=T(v[sl], torch.int32), f=T(f[sl], torch.int32),
                             uo=torch.empty((Bs, 8), dtype=torch.float64, device=dev)))

        def step():
            for s in range(S):
                b = bufs[s]
                with torch.cuda.stream(st[s]):
                    b["x0"].copy_(b["x0p"])
                    engs[s].set_warmstart_device(Bs, b["g"], b["v"], b["f"], stream=st[s])
                    engs[s].solve_device(Bs, b["x0"], b["u0"], b["obs"], b["uo"], stream=st[s])
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if args.timing:
            for e in engs:
                e.timing_begin()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if args.timing:
            busy = []
            for e in engs:
                e.timing_end()
                a, b = e.timing_intervals("qp", anchor=engs[0], max_n=4 * args.steps + 8)
                busy.append((a, b))
            res_busy = bench.union_length(np.concatenate([a for a, _ in busy]), np.concatenate([b for _, b in busy]))
        u = torch.cat([b["uo"] for b in bufs]).cpu().numpy()
        if ref is None:
            ref = u
        res[S] = {"solves_per_s": B * args.steps / dt, "ms_per_step": dt / args.steps * 1e3,
                  "bitwise_equal_to_S1": bool(np.array_equal(u, ref))}
        if args.timing:
            res[S]["qp_busy_ms_per_step"] = res_busy / args.steps
        print(json.dumps({"S": S, **res[S]}), flush=True)
        for e in engs:
            e.close()


if __name__ == "__main__":
    main()
