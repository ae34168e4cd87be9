"""Why two controller groups on two torch streams overlap in tools/pipeline_probe.py but ran back to back in
bench.py (round-3 r03e: 2 x 2.75 ms per step).  configs[1] (B = 4096, N = 20, mask 2) as 2 engines of 2048
instances; each variant times 20 steps and reports ms/step and the union of the QP-solve launch intervals.

  bench_order   engines first, then two consecutive torch.cuda.Stream()s (bench.py's order)
  interleaved   engine, stream, engine, stream (pipeline_probe.py's order)
  spaced        engines, then stream, an unused stream, stream
  fresh_each    engines, then a torch pool stream per group taken after 3 unused ones
  after_s1      interleaved, after one S = 1 engine + stream has solved once and been closed
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    import mpcc_manipulator_amd as m
    B, N, mask, S, steps = 4096, 20, 2, 2, 20
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
    Bs = B // S
    variant = sys.argv[1]
    engs, st = [], []
    if variant == "after_s1":  # pipeline_probe.py's history: an S = 1 engine and stream used and closed first
        e1 = m.Engine(params, max_batch=B, device=0, constraint_mask=mask)
        e1.set_track(*track)
        s1 = torch.cuda.Stream(dev)
        with torch.cuda.stream(s1):
            e1.set_warmstart_device(B, T(g), T(v, torch.int32), T(f, torch.int32), stream=s1)
            e1.solve_device(B, T(x0), T(u0), T(obs), torch.empty((B, 8), dtype=torch.float64, device=dev), stream=s1)
        torch.cuda.synchronize()
        e1.close()
        variant_eff = "interleaved"
    else:
        variant_eff = variant
    if variant_eff == "interleaved":
        for s in range(S):
            engs.append(m.Engine(params, max_batch=Bs, device=0, constraint_mask=mask))
            st.append(torch.cuda.Stream(dev))
    else:
        engs = [m.Engine(params, max_batch=Bs, device=0, constraint_mask=mask) for _ in range(S)]
        if variant_eff == "bench_order":
            st = [torch.cuda.Stream(dev) for _ in range(S)]
        elif variant_eff == "spaced":
            st.append(torch.cuda.Stream(dev))
            torch.cuda.Stream(dev)
            st.append(torch.cuda.Stream(dev))
        elif variant_eff == "fresh_each":
            for s in range(S):
                for _ in range(3):
                    torch.cuda.Stream(dev)
                st.append(torch.cuda.Stream(dev))
        else:
            raise SystemExit(f"unknown variant {variant}")
    for e in engs:
        e.set_track(*track)
    bufs = []
    for s in range(S):
        sl = slice(s * Bs, (s + 1) * Bs)
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
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for e in engs:
        e.timing_begin()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    iv = []
    for e in engs:
        e.timing_end()
        iv.append(e.timing_intervals("qp", anchor=engs[0], max_n=4 * steps + 8))
    busy = bench.union_length(np.concatenate([a for a, _ in iv]), np.concatenate([b for _, b in iv]))
    print(json.dumps({"variant": variant, "ms_per_step": dt / steps * 1e3, "solves_per_s": B * steps / dt,
                      "qp_busy_ms_per_step": busy / steps,
                      "streams": [hex(s.cuda_stream) for s in st], "priority_range": torch.cuda.Stream.priority_range(),
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)


if __name__ == "__main__":
    main()
