"""Benchmark: MPCC solves/sec (7-DOF Panda, N=20, 2 SQP iterations) — BASELINE.json configs[1].
Other BASELINE configs as presets (--config 2, 3; parity cases, not the headline line).

One step = one batched MPC::runMPC_ (cpp/src/MPC/mpc.cpp:104-190) over B independent controllers per
GPU (default B = 4096, bounds + singularity rows: constraint_mask = 2), inputs resident in HBM; for
N > 1 GPUs every rank solves its own B instances (weak scaling) and the optimal inputs u0 are gathered
over RCCL each step.  Prints one JSON line (rank 0).

    python bench.py [--gpus N --steps K --warmup W --batch B]
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense peak (matrix = vector, spec) — the roof of the FP64 solve kernels
SEED = 0x4D504343
METRIC = "MPCC solves/sec (whole node), 7-DOF Panda N=20, 2 SQP iters; 1/2/4/8 GPU"  # BASELINE.json metric
Q0 = np.array([0, 0, 0, -np.pi / 2, 0, np.pi / 2, np.pi / 4])


def q_start(dof):
    """Start joints of the reference's main.cpp:60-61 (the mobile base at the origin for dof 10)."""
    return Q0 if dof == 7 else np.concatenate([np.zeros(dof - 7), Q0])


def batch_inputs(pool, B, dof, obstacles, obs_xyz, start=0, world=1):
    """The bench's instances: pool step t = (global index) mod T, q += N(0, 0.005); the noise
    is drawn for the global batch, so instance i gets the same input whatever the number of ranks.  Obstacles:
    main_w_sim.py:42-45's scenario, xyz = (0.48, 0.218, z), z ~ U[z0 - 0.1, z0 + 0.1], r = 5 cm, or the dummy
    obstacle of MPC::runMPC (mpc.cpp:97-100).  Returns x0, u0, obs, guess, valid, fails of this rank's block."""
    rng = np.random.default_rng(SEED)
    T = len(pool["x0"])
    idx = (np.arange(B) + start) % T
    x0 = pool["x0"][idx].copy()
    x0[:, :dof] += rng.normal(0.0, 0.005, size=(B * world, dof))[start:start + B]
    u0 = pool["u0"][idx].copy()
    guess = pool["guess"][idx].copy()
    valid = pool["valid"][idx].astype(np.int32)
    fails = pool["fails"][idx].astype(np.int32)
    if obstacles:
        z = rng.uniform(obs_xyz[2] - 0.1, obs_xyz[2] + 0.1, B * world)[start:start + B]
        obs = np.column_stack([np.full(B, obs_xyz[0]), np.full(B, obs_xyz[1]), z, np.full(B, 5.0)])
    else:
        obs = np.tile(np.array([3.0, 3.0, 3.0, 0.0]), (B, 1))
    return x0, u0, obs, guess, valid, fails


def find_pmc(kname, B, N, mask, dof, override=None, prof_dir=None):
    """The committed PMC summary of this workload (tools/pmc_summary.py): the first pmc_traffic_<kernel>*.json
    whose kernel, batch, horizon, constraint mask and DOF match, with the per-launch counters of the summary it
    names ("source"), or None."""
    prof_dir = prof_dir or os.path.join(ROOT, "profiles")
    tpaths = [override] if override else sorted(glob.glob(os.path.join(prof_dir, f"pmc_traffic_{kname}*.json")))
    for tpath in tpaths:
        if not os.path.exists(tpath):
            continue
        with open(tpath) as f:
            tr = json.load(f)
        if (tr.get("batch") == B and tr.get("N") == N and tr.get("mask") == mask
                and tr.get("kernel", "k_ipm") == kname and tr.get("dof", 7) == dof):
            src = os.path.join(ROOT, tr["source"]) if tr.get("source") else None
            if src and os.path.exists(src):
                with open(src) as f:
                    tr["counters"] = json.load(f).get("counters_avg_per_launch", {})
            tr["file"] = os.path.relpath(tpath, ROOT)
            return tr
    return None


def find_traffic(kname, B, N, mask, dof, override=None, prof_dir=None):
    """HBM bytes per launch from the matching PMC summary (find_pmc), or None."""
    tr = find_pmc(kname, B, N, mask, dof, override, prof_dir)
    return tr.get("hbm_bytes_per_launch") if tr else None


def pmc_fp64_flops(counters):
    """FP64 flops per launch from the PMC counters: 64 lanes x (ADD + MUL + 2 FMA) VALU wave instructions (an upper
    bound: lanes masked off inside a 16-lane group are counted) plus, when the profile has it, the FP64 matrix-core
    work (SQ_INSTS_VALU_MFMA_MOPS_F64, in units of 512 flops: 4 per v_mfma_f64_16x16x4f64 of 2048); or None."""
    if not counters or "SQ_INSTS_VALU_FMA_F64" not in counters:
        return None
    valu = 64.0 * (counters["SQ_INSTS_VALU_ADD_F64"] + counters["SQ_INSTS_VALU_MUL_F64"] +
                   2.0 * counters["SQ_INSTS_VALU_FMA_F64"])
    return valu + 512.0 * counters.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)


def union_length(starts, ends):
    """Length of the union of the intervals [starts[i], ends[i]]."""
    tot, cur_s, cur_e = 0.0, None, None
    for a, b in sorted(zip(starts, ends)):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    return tot + ((cur_e - cur_s) if cur_e is not None else 0.0)


HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E peak (spec), MI355X_MICROARCH.md


def qs_doubles(dof):
    """Doubles of one stage's QP record (csrc/dev_common.h QS: NX = DOF + 2, NU = DOF + 1, 11 polytopic rows of
    2 DOF + 1, padded to whole 128-byte lines): 336 for the Panda, 480 for the Husky+Panda."""
    nx, nu, npc = dof + 2, dof + 1, 11
    ylb = (nx * nx + nx + 2 * nu + nx + 15) // 16 * 16
    obj = ylb + 2 * nx + 2 * dof + 1 + npc * (2 * dof + 1) + 1
    return (obj + 1 + 15) // 16 * 16


def mlp_flops_per_sample(which, dof=7):
    """value + the DOF forward-mode Jacobian columns of one collision-MLP sample.
    self: 21 -> 256 -> 64 -> 1; env: 30 -> 256 x 4 -> 9 (F_self 0.285, F_env 3.21 MFLOP for the Panda)."""
    if which == "k_mlp_self":
        return 2 * (256 * 21 + 64 * 256 + 64 + dof * 256 * 3 + dof * 64 * 256 + dof * 64)
    return 2 * (256 * 30 + 3 * 256 ** 2 + 9 * 256 + dof * 256 * 3 + dof * 3 * 256 ** 2 + dof * 9 * 256)


def algorithmic_qp_flops(N, dof=7):
    """SURVEY.md §8(d) F_qp per SQP iteration (condensing + Cholesky + solves; inequality handling is
    solver overhead and not credited): 2(96N^3 + 324N^2) + 616N^2 + n^3/3 + 4n^2, n = 8N for the Panda,
    i.e. 2(NU^2 NX N^3 / 6 + NX^2 NU N^2 / 2) + NPC NU DOF N^2 + n^3/3 + 4n^2 with n = NU N for any robot."""
    nx, nu = dof + 2, dof + 1
    n = nu * N
    return 2 * (nu * nu * nx / 6 * N ** 3 + nx * nx * nu / 2 * N ** 2) + 11 * nu * dof * N ** 2 + n ** 3 / 3 + 4 * n ** 2


def make_pool(m, params, mask, steps, device, pool_obs=(3.0, 3.0, 3.0, 0.0)):
    """State pool of the reference closed loop (main.cpp:100-114): the committed file for configs[1]
    (tools/make_bench_pool.py), else a B = 1 closed loop on the GPU.  Returns (pool, track)."""
    N = params.N
    eng = m.Engine(params, max_batch=1, device=device, constraint_mask=mask)
    dof, nx, nu = eng.dof, eng.NX, eng.NU
    ee = eng.robot_records(q_start(dof), np.array([[3.0, 3.0, 3.0, 0.0]]))[0, :3]
    X, Y, Z, q = m.load_default_track()
    track = m.track_from_points(X, Y, Z, q, ee)
    path = os.path.join(ROOT, "mpcc_manipulator_amd", "data", f"bench_pool_n{N}_mask{mask}.npz")
    if dof == 7 and os.path.exists(path):
        f = np.load(path, allow_pickle=False)
        if f["x0"].shape[0] >= steps:
            eng.close()
            return {k: f[k][:steps] for k in f.files}, track
    eng.set_track(*track)
    from mpcc_manipulator_amd.integrator import sim_time_step
    x = np.zeros((1, nx)); x[0, :dof] = q_start(dof)
    u = np.zeros((1, nu))
    obs = np.array([pool_obs])
    pool = {k: [] for k in ["x0", "u0", "guess", "valid", "fails", "status"]}
    for _ in range(steps):
        g, v, fl = eng.get_warmstart(1)
        pool["x0"].append(x[0].copy()); pool["u0"].append(u[0].copy())
        pool["guess"].append(g[0]); pool["valid"].append(v[0]); pool["fails"].append(fl[0])
        xin = x.copy()
        out = eng.solve(xin, u, obs)
        pool["status"].append(out["status"][0])
        u = out["u0"].copy()
        x = eng.sim_time_step(xin, u, params.Ts) if dof != 7 else sim_time_step(xin, u, params.Ts)  # main.cpp:103-105
    eng.close()
    return {k: np.array(v) for k, v in pool.items()}, track


def cpu_info():
    """Host CPU of this run: logical CPUs of the machine (nproc), the CPUs this process may use (its
    affinity mask / the box's share), the OpenMP thread cap of the environment and the lscpu model name."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": os.cpu_count(), "usable": usable, "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "model": model}


def cpu_baseline(params_dict, track, x0, u0, obs, guess, valid, fails, threads, sample, budget_s, latency_n=200,
                 dof=7, latency_budget_s=10.0):
    """The oracle (CPU restatement of the reference algorithm, oracle/) on a bounded sample of the same
    workload: repeated passes over the first `sample` instances (each pass from the same inputs, so
    every pass is one full runMPC_ per instance), OpenMP over instances, until `budget_s` seconds of
    CPU work.  Then the single-controller latency BASELINE.md §2 asks for: `latency_n` solves one at a
    time on one thread (ms per runMPC_, against the Ts = 10 ms real-time budget of config.json:4).
    Test infrastructure used only as the reported baseline."""
    from oracle.pyoracle import Oracle
    o = Oracle(params_dict, os.path.join(ROOT, "mpcc_manipulator_amd", "data", "nn"), qp_mode=0, nthreads=threads, dof=dof)
    o.set_track(*track)
    n = min(sample, x0.shape[0])
    o.run_mpc(x0[:2].copy(), u0[:2], obs[:2], guess[:2].copy(), valid[:2].copy(), fails[:2].copy())  # warm caches
    done, dt, passes = 0, 0.0, 0
    while dt < budget_s and passes < 1000:
        xs, gs, vs, fs = x0[:n].copy(), guess[:n].copy(), valid[:n].copy(), fails[:n].copy()
        t0 = time.perf_counter()
        o.run_mpc(xs, u0[:n], obs[:n], gs, vs, fs)
        dt += time.perf_counter() - t0
        done += n
        passes += 1
    o.close()
    o1 = Oracle(params_dict, os.path.join(ROOT, "mpcc_manipulator_amd", "data", "nn"), qp_mode=0, nthreads=1, dof=dof)
    o1.set_track(*track)
    lat = []
    for i in range(min(latency_n, x0.shape[0])):
        if sum(lat) > latency_budget_s:
            break
        xs, gs, vs, fs = x0[i:i + 1].copy(), guess[i:i + 1].copy(), valid[i:i + 1].copy(), fails[i:i + 1].copy()
        t0 = time.perf_counter()
        o1.run_mpc(xs, u0[i:i + 1], obs[i:i + 1], gs, vs, fs)
        lat.append(time.perf_counter() - t0)
    o1.close()
    lat = np.array(lat) * 1e3
    return done / dt, n, passes, dt, {"mean_ms": float(lat.mean()), "p99_ms": float(np.percentile(lat, 99)),
                                      "max_ms": float(lat.max()), "solves": int(lat.size), "budget_ms": 10.0}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`python bench.py --gpus N` outside a launcher: start N ranks (one process per GPU) as child
    processes before this process touches the GPU, with the env torch.distributed.run would set, and
    exit with the worst child exit code.  Rank 0 writes the JSON line to our stdout."""
    import torch
    rehearse = os.environ.get("MPCC_BENCH_REHEARSE", "0") == "1"
    ndev = torch.cuda.device_count()  # counts devices without initialising the GPU
    if not rehearse and ndev < n:
        print(f"bench.py: --gpus {n} requested but {ndev} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [None] * n
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if any(c not in (None, 0) for c in codes):  # one rank failed: stop the others (exact PIDs)
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.kill()
                    codes[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [c for c in codes if c != 0]
    sys.exit(bad[0] if bad else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="1", choices=["1", "2", "3", "1-all-rows"],
                    help="BASELINE configs[i] preset: 1 = B 4096, N 20, mask 2 (the metric); "
                         "2 = B 65536, N 40, mask 7, per-instance obstacles (parity case, timing only); "
                         "3 = Husky+Panda 10-DOF mobile manipulator, B 32768, N 30, mask 7 (full cost and constraint "
                         "set), per-instance obstacles (parity case, timing only); "
                         "1-all-rows = configs[1]'s B 4096, N 20 with the reference's default rows (all 11: self + "
                         "singularity + 9 env collision, config.h:34) and the main_w_sim.py:42-45 obstacles")
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--mask", type=int, default=None, help="polytopic rows: 1 self, 2 singularity, 4 env (configs[1] = 2)")
    ap.add_argument("--max-iter", type=int, default=2)
    ap.add_argument("--pool-steps", type=int, default=1000)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="OpenMP threads of the CPU baseline (default: the CPUs this process may use, capped by OMP_NUM_THREADS)")
    ap.add_argument("--cpu-sample", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline budget (bounded sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-all-cores", action="store_true",
                    help="also time the oracle on every CPU of the affinity mask (cpu_baseline.all_cores, kind "
                         "'measured'); default: the estimate from the job's CPU share")
    ap.add_argument("--traffic", default=None, help="PMC traffic summary (default profiles/pmc_traffic_<kernel>.json)")
    ap.add_argument("--dump-u0", default=None, help="rank 0 writes the last step's gathered u0 [world*B, 8] (.npy)")
    ap.add_argument("--sub-batches", type=int, default=2,
                    help="controller groups per GPU, each an engine of B/S instances stepping on its own HIP stream, so "
                         "one group's next control step overlaps another's interior-point tail (1: one engine)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args.gpus)
    preset = {"1": dict(batch=4096, N=20, mask=2), "2": dict(batch=65536, N=40, mask=7),
              "3": dict(batch=32768, N=30, mask=7, pool_steps=300),
              "1-all-rows": dict(batch=4096, N=20, mask=7)}[args.config]
    dof = 10 if args.config == "3" else 7
    obstacles = args.config in ("2", "3", "1-all-rows")
    if args.config == "3" and args.pool_steps == 1000:
        args.pool_steps = preset.pop("pool_steps")
    preset.pop("pool_steps", None)
    for k, v in preset.items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    # MPCC_BENCH_REHEARSE=1: every rank on GPU 0 over gloo — rehearses the multi-rank path (sharding,
    # u0 gather, max-over-ranks timing, aggregation) on a one-GPU box; real runs use one GPU per rank
    # over RCCL ("nccl")
    rehearse = os.environ.get("MPCC_BENCH_REHEARSE", "0") == "1"
    if rehearse:
        local = 0
    # Every controller group's stream needs a hardware queue of its own, or the groups' kernels run back to back:
    # HIP multiplexes all streams onto GPU_MAX_HW_QUEUES queues (4 by default) and torch's stream pool, created
    # whole at the first torch.cuda.Stream(), lands consecutive pool streams on one queue (measured:
    # tools/probes/stream_overlap.py, profiles/r03g_stream_overlap.log, r03h_stream_overlap.log).  Read by HIP when it
    # initialises, below.
    hwq = min(32, max(8, 2 * args.sub_batches + 4))
    if args.sub_batches > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < hwq:
        os.environ["GPU_MAX_HW_QUEUES"] = str(hwq)
    import torch
    if torch.cuda.device_count() <= local:
        print(f"bench.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import mpcc_manipulator_amd as m
    from mpcc_manipulator_amd.distributed import check_equal_shards, gather_u0, max_over_ranks, shard_bounds

    N, B = args.N, args.batch
    params = m.load_params(N, overrides={"sqp": {"max_iter": args.max_iter}}, dof=dof)
    params.constraint_mask = args.mask
    nx, nu, nxu, _ = m.dims(dof)
    # obstacle scenario: main_w_sim.py:42-45 for the Panda; for the mobile manipulator the same kind of
    # obstacle near the arm's reach from its start pose (its EE starts 0.35 m higher, on the base)
    obs_xyz = (0.48, 0.218, 0.521) if dof == 7 else (0.62, 0.28, 0.75)
    pool_obs = (*obs_xyz, 5.0) if obstacles else (3.0, 3.0, 3.0, 0.0)
    pool, track = make_pool(m, params, args.mask, args.pool_steps, local, pool_obs)
    S = args.sub_batches
    if S < 1 or B % S:
        print(f"bench.py: --sub-batches {S} must divide the batch {B}", file=sys.stderr)
        sys.exit(2)
    Bs = B // S
    engs = [m.Engine(params, max_batch=Bs, device=local, constraint_mask=args.mask) for _ in range(S)]
    for e in engs:
        e.set_track(*track)
    eng = engs[0]

    start, _ = shard_bounds(B * world, rank, world)  # contiguous instance block of this rank
    x0, u0, obs, guess, valid, fails = batch_inputs(pool, B, dof, obstacles, obs_xyz, start, world)

    dev = torch.device("cuda", local)
    t = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
    x0_p, u0_d, obs_d = t(x0), t(u0), t(obs)
    g_p, v_p, f_p = t(guess), t(valid, torch.int32), t(fails, torch.int32)
    # runMPC_ updates x0 (s, vs) in place, so every step gets its own copy of the inputs, made before any timing
    # (no input-restore copy inside the timed region)
    x0_steps = [x0_p.clone() for _ in range(args.warmup + args.steps)]
    # u0 outputs double-buffered by step parity: with N > 1 ranks the gather of step i reads its buffer on the
    # gather stream while step i + 1 writes the other one
    u_out = [torch.empty((B, nu), dtype=torch.float64, device=dev) for _ in range(2)]
    hor = torch.empty((B, N + 1, nxu), dtype=torch.float64, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    ok = torch.empty(B, dtype=torch.int32, device=dev)
    u_all = [torch.empty((world * B, nu), dtype=torch.float64, device=dev) for _ in range(2)] if world > 1 else None
    # Each controller group (engine s: instances [s Bs, (s+1) Bs)) steps on its own stream: the warm-start restore
    # and the engine's kernels on the step's own x0 copy, so every step reads the inputs it restored and group s only
    # waits for its own previous step.  The u0 gather (RCCL, N > 1 ranks) runs on a third stream after all groups
    # of the step; it needs every rank's u0 of that step, nothing of the next one.
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    gstream = torch.cuda.Stream(dev)
    done = [[torch.cuda.Event() for _ in range(S)] for _ in range(2)]
    gathered = [torch.cuda.Event() for _ in range(2)]
    sl = [slice(s_ * Bs, (s_ + 1) * Bs) for s_ in range(S)]
    nstep = [0]

    def step():
        i = nstep[0]
        buf = i % 2
        for s_ in range(S):
            st_ = streams[s_]
            with torch.cuda.stream(st_):
                if world > 1 and i >= 2:
                    st_.wait_event(gathered[buf])  # the gather of step i - 2 has read this u0 buffer
                engs[s_].set_warmstart_device(Bs, g_p[sl[s_]], v_p[sl[s_]], f_p[sl[s_]], stream=st_)
                engs[s_].solve_device(Bs, x0_steps[i][sl[s_]], u0_d[sl[s_]], obs_d[sl[s_]], u_out[buf][sl[s_]], hor[sl[s_]],
                                      status[sl[s_]], ok[sl[s_]], stream=st_)
                done[buf][s_].record(st_)
        if world > 1:
            with torch.cuda.stream(gstream):
                for s_ in range(S):
                    gstream.wait_event(done[buf][s_])
                gather_u0(u_out[buf], world, out=u_all[buf])  # RCCL all-gather of u0 over xGMI
                gathered[buf].record(gstream)
        nstep[0] += 1

    if world > 1:
        check_equal_shards(B, device=dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for e in engs:
        e.timing_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    last = (nstep[0] - 1) % 2
    tms = [e.timing_end() for e in engs]
    tmlps = [e.timing_mlp() for e in engs]
    tsqp = [e.timing_sqp() for e in engs]  # the fused kernel's spans (timing_end splits them over set_qp/solve_qp/get_alpha)
    # the QP-solve launches of all groups, as intervals on engine 0's clock (its window's first event, recorded
    # before any group's first kernel of the timed region): their union is the time the kernel family ran
    nq = max(x[2] for x in tms)  # QP-solve launches of the timed steps per engine (the staged loop: one per SQP iteration)
    ivs = [e.timing_intervals("qp", anchor=engs[0], max_n=nq + 8) for e in engs]
    ivs_env = [e.timing_intervals("k_mlp_env", anchor=engs[0], max_n=4 * args.steps + 8) for e in engs]
    if world > 1:
        elapsed = max_over_ranks(elapsed, device=dev)
    tm = {k: sum(x[0][k] for x in tms) for k in tms[0][0]}  # summed over groups
    ncalls = tms[0][1]
    nipm = sum(x[2] for x in tms)
    tmlp = {k: (sum(x[k][0] for x in tmlps), sum(x[k][1] for x in tmlps)) for k in tmlps[0]}

    st = status.cpu().numpy()
    stats_g = [e.solve_stats(Bs) for e in engs]
    stats = {k: np.concatenate([sg[k] for sg in stats_g]) for k in stats_g[0]}
    solved = float(np.mean(st == 0))
    value = B * world * args.steps / elapsed
    ms = elapsed / args.steps * 1e3

    # Roofline of the dominant kernel, by measured time per step: k_sqp (the SQP loop with its interior-point
    # QP solves, 16 lanes per instance; k_ipm alone when the staged SQP loop is selected, MPCC_STAGED_SQP=1) or,
    # with the collision networks on (configs[2]), k_mlp_env.  Launch durations are HIP events on the engine
    # stream around those launches alone, over the timed steps.
    kname = "k_ipm" if os.environ.get("MPCC_STAGED_SQP", "0") == "1" else "k_sqp"
    nsqp = sum(x[1] for x in tsqp)
    # mean duration of one launch (B/S instances): the fused kernel's span, or the staged path's k_ipm launches
    t_ipm = sum(x[0] for x in tsqp) / nsqp if nsqp else tm["solve_qp"] / max(1, nipm)
    # QP solves per step: an instance solves min(sqp_iter + 1, max_iter) QPs (a SOLVED exit at SQP
    # iteration i has solved i + 1); the launches are credited with the QPs they actually solved
    qps = int(np.minimum(stats["sqp_iter"] + 1, args.max_iter).sum())
    flops_step = qps * algorithmic_qp_flops(N, dof)
    flops = flops_step * ncalls / max(1, nipm)  # per launch, on average
    # time the kernel ran: the union of all groups' launch intervals (S = 1: the sum of launch durations)
    busy = union_length(np.concatenate([a for a, _ in ivs]), np.concatenate([b for _, b in ivs])) * 1e-3
    # per launch (the contract's figure): the algorithmic flops one launch is credited with over its mean duration;
    # the S groups' launches overlap, so the chip-wide figure over the union of their intervals is reported beside it
    achieved = flops / t_ipm / 1e12 if t_ipm > 0 else 0.0
    achieved_union = flops_step * ncalls / busy / 1e12 if busy > 0 else achieved
    pmc = find_pmc(kname, Bs, N, args.mask, dof, args.traffic)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    pflops = pmc_fp64_flops(pmc.get("counters")) if pmc else None
    # the stage records one launch must move at least: every instance's QP record and step, read / written once per
    # QP solved (QS + NX + NU doubles per stage), against which the counted traffic is compared
    rec_io = (qps / max(1, S)) * (N + 1) * (qs_doubles(dof) + dof + 2 + dof + 1) * 8.0
    # k_sqp is a latency-bound FP64 kernel: VALU + DPP for the stage recursions, the matrix cores for P = Hb - U^T U
    # (and the poly Gram blocks of the wide variants); its roof is the FP64 peak (78.6 TFLOP/s for vector and matrix
    # alike on MI355X), its work the SURVEY's condensed-dense F_qp per QP actually solved; the PMC-counted FP64 flops
    # it executed (VALU and MFMA) and its counter-measured HBM traffic (not algorithmic bytes: mostly the interior
    # point's streamed workspace) are reported beside it
    roof = {"kernel": kname, "bound": "valu+mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
            "achieved_union": achieved_union, "frac_union": achieved_union / FP64_PEAK_TFLOPS,
            "counter_hbm_frac": (traffic * nipm / busy / HBM_PEAK_BPS) if traffic and busy > 0 else None,
            "record_io_bytes_per_launch": rec_io,
            "traffic_over_record_io": (traffic / rec_io) if traffic and rec_io > 0 else None,
            "pmc_fp64_flops_per_launch": pflops,
            "pmc_fp64_frac": (pflops / t_ipm / 1e12 / FP64_PEAK_TFLOPS) if pflops and t_ipm > 0 else None,
            "pmc_source": pmc.get("file") if pmc else None,
            "avg_launch_ms": t_ipm * 1e3, "launches_timed": nipm, "concurrent_groups": S,
            "busy_ms_per_step": busy / max(1, ncalls) * 1e3, "algorithmic_flops_per_launch": flops,
            "work": "F_qp (SURVEY 8(d), condensed-dense QP) x QPs solved; frac per launch (mean launch duration), "
                    "frac_union over the union of the S groups' concurrent launches",
            "qp_solves_per_step": qps}
    t_env, n_env = tmlp["k_mlp_env"]
    busy_env = union_length(np.concatenate([a for a, _ in ivs_env]), np.concatenate([b for _, b in ivs_env])) * 1e-3
    # the collision MLPs of this configuration (mask bits 1, 4), each against the FP64 MFMA roof: mean launch
    # duration and the fraction over it (one launch = the B/S (N + 1) samples of a group)
    mlps = {}
    for kn in ("k_mlp_self", "k_mlp_env"):
        t_k, n_k = tmlp[kn]
        if n_k:
            fl_k = Bs * (N + 1) * mlp_flops_per_sample(kn, dof)
            mlps[kn] = {"avg_launch_ms": t_k / n_k * 1e3, "launches_timed": n_k,
                        "frac": fl_k / (t_k / n_k) / 1e12 / FP64_PEAK_TFLOPS}
    if mlps:
        roof["mlp"] = mlps
    if n_env and busy_env > busy:  # the env MLP ran longer than the QP solve (configs[2])
        t_l = t_env / n_env
        samples = Bs * (N + 1)
        fl = samples * mlp_flops_per_sample("k_mlp_env", dof)
        pm = find_pmc("k_mlp_env", Bs, N, args.mask, dof)
        tr = pm.get("hbm_bytes_per_launch") if pm else None
        ach = fl / t_l / 1e12  # per launch, as for k_sqp; the union of the groups' launches beside it
        ach_u = fl * n_env / busy_env / 1e12
        roof = {"kernel": "k_mlp_env", "bound": "mfma", "achieved": ach, "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS, "traffic": tr,
                "achieved_union": ach_u, "frac_union": ach_u / FP64_PEAK_TFLOPS,
                "counter_hbm_frac": (tr * n_env / busy_env / HBM_PEAK_BPS) if tr else None, "avg_launch_ms": t_l * 1e3,
                "launches_timed": n_env, "concurrent_groups": S, "busy_ms_per_step": busy_env / max(1, ncalls) * 1e3,
                "algorithmic_flops_per_launch": fl,
                "work": "F_env (SURVEY 8(d): value + DOF Jacobian columns) x B/S (N+1) samples per launch, over the "
                        "union of the launches' intervals",
                "k_sqp": {"avg_launch_ms": t_ipm * 1e3, "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                          "busy_ms_per_step": busy / max(1, ncalls) * 1e3}, "mlp": mlps}

    # PCIe-inclusive rate (host buffers in and out through mpcc_solve): a diagnostic, never `value`
    pcie = None
    if rank == 0 and world == 1:  # one group's engine, its instances through host buffers
        reps = 5
        xh = np.ascontiguousarray(x0[sl[0]])
        dt_h = 0.0
        for r in range(reps + 1):
            eng.set_warmstart_device(Bs, g_p[sl[0]], v_p[sl[0]], f_p[sl[0]], stream=streams[0])
            torch.cuda.synchronize()
            xs = xh.copy()
            t1 = time.perf_counter()
            eng.solve(xs, u0[sl[0]], obs[sl[0]])
            if r:
                dt_h += time.perf_counter() - t1
        pcie = Bs * reps / dt_h

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            pd = params.as_dict()
            ci = cpu_info()
            threads = args.cpu_threads or min(ci["usable"], ci["omp_num_threads"] or ci["usable"])
            args.cpu_threads = threads
            v, n, passes, dt, lat = cpu_baseline(pd, track, x0, u0, obs, guess, valid, fails, threads,
                                                 args.cpu_sample, args.cpu_seconds, dof=dof)
            # the machine's other cores: the GPU box gives one GPU's job a CPU share (OMP_NUM_THREADS = 16 there,
            # set by the harness, which asks jobs to keep their pools within it), so by default the all-core figure is
            # the measured per-thread rate times nproc, stated as an estimate, with the measured 1 -> `threads`
            # scaling efficiency beside it.  --cpu-all-cores measures it instead (a second oracle leg on every CPU of
            # the affinity mask), for a machine the run owns.
            rate1 = 1e3 / lat["mean_ms"]
            allc = {"value": v / threads * ci["nproc"], "cores": ci["nproc"], "kind": "estimate",
                    "efficiency_vs_1thread": v / (threads * rate1),
                    "basis": f"measured {threads}-thread rate x {ci['nproc']}/{threads} (linear; instances are "
                             f"independent, one per thread; measured {threads}-thread efficiency against the "
                             f"single-thread latency run ({rate1:.1f} solves/s): {v / (threads * rate1):.2f})"}
            if args.cpu_all_cores and ci["usable"] > threads:
                va, na, pa, dta, _ = cpu_baseline(pd, track, x0, u0, obs, guess, valid, fails, ci["usable"],
                                                  args.cpu_sample, args.cpu_seconds, latency_n=1, dof=dof,
                                                  latency_budget_s=0.0)
                allc = {"value": va, "cores": ci["usable"], "kind": "measured",
                        "sample": f"{pa} passes over the first {na} instances ({pa * na} solves, {dta:.1f} s), "
                                  f"OpenMP {ci['usable']} threads"}
            cpu = {"value": v, "unit": "solves/s", "cores": threads, "kind": "port", "host": ci,
                   "all_cores": allc, "latency_1thread": lat,
                   "sample": f"{passes} passes over the first {n} instances of the same workload "
                             f"({passes * n} runMPC_ solves, {dt:.1f} s; oracle = CPU restatement of the "
                             f"reference algorithm with OSQP replaced by an exact IPM, OpenMP {args.cpu_threads} threads)"}
        except Exception as e:  # baseline is reported, never the target
            print(f"cpu baseline failed: {e}", file=sys.stderr)

    if rank == 0:
        # per controller group and step: the S groups' phases run concurrently, so the sum over groups would
        # exceed the wall time per step
        phases = {k: round(v / max(1, ncalls) / S * 1e3, 4) for k, v in tm.items()}
        phases.update({k: round(v[0] / max(1, ncalls) / S * 1e3, 4) for k, v in tmlp.items() if v[1]})
        fr = np.mean([x[2] for x in tsqp], axis=0) if nsqp else np.zeros(4)
        print(json.dumps({"phase_ms_per_group_step": phases,
                          "sqp_phase_frac": dict(zip(["set_qp", "solve_qp", "get_alpha", "step"], np.round(fr, 4).tolist())),
                          "groups": S, "solved_frac": solved,
                          "sqp_iter_hist": np.bincount(stats["sqp_iter"], minlength=3).tolist(),
                          "ipm_iters_mean": float(stats["ipm_iters"].mean()),
                          "pcie_inclusive_solves_per_s": pcie}), file=sys.stderr)
        line = {
            "metric": METRIC,
            "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (closed-loop state pool on the default track, q + N(0, 0.005 rad))",
            "config": {"workload": {
                "1": f"configs[1]: batch={B}/GPU Panda MPCC instances, N={N}, bounds+singularity constraints "
                     f"(mask={args.mask}), {args.max_iter} SQP iters",
                "2": f"configs[2]: batch={B}/GPU Panda MPCC instances, N={N}, self+env collision NN constraints "
                     f"(mask={args.mask}), per-instance obstacles, {args.max_iter} SQP iters",
                "3": f"configs[3]: batch={B}/GPU Husky+Panda 10-DOF mobile manipulator MPCC instances, N={N}, full cost "
                     f"and constraint set (mask={args.mask}: self + singularity + env collision NN rows), per-instance "
                     f"obstacles, {args.max_iter} SQP iters",
                "1-all-rows": f"configs[1] shape with the reference's default rows: batch={B}/GPU Panda MPCC instances, "
                              f"N={N}, all 11 polytopic rows incl. both collision NNs (mask={args.mask}), per-instance "
                              f"obstacles, {args.max_iter} SQP iters"}[args.config],
                       "batch_per_gpu": B, "global_batch": B * world, "horizon": N, "sqp_iters": args.max_iter,
                       "sub_batches": S, "instances_per_engine": Bs,
                       "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "parallelism": f"instance-sharded x{world}" + ((", gloo rehearsal, all ranks on GPU 0" if rehearse else
                                                                  ", RCCL all_gather(u0)") if world > 1 else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if args.dump_u0 and rank == 0:
        np.save(args.dump_u0, (u_all[last] if world > 1 else u_out[last]).cpu().numpy())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
