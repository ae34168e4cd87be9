"""Summarize a round profile (tools/profile_round.sh) into profiles/:
  <round>_kernel_stats.csv        rocprofv3 --stats of the bench command (per-kernel time)
  <round>_<kernel>_pmc.json       counters of the dominant kernel per benchmark-size launch (averaged)
  pmc_traffic_<kernel>.json       HBM bytes per launch of that kernel (read by bench.py)
FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half of the bytes of wide
coalesced reads, so it is doubled (MI355X_MICROARCH.md §HBM).

    python tools/pmc_summary.py gpurun_out/prof r01 --batch 4096 --N 20 --kernel k_sqp
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_pmc(d, name):
    f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))
    if not f:
        return {}
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        agg[int(r["Dispatch_Id"])].update({"grid": int(r["Grid_Size"]), "kernel": r["Kernel_Name"],
                                           r["Counter_Name"]: float(r["Counter_Value"])})
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("round")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--mask", type=int, default=2, help="constraint mask of the profiled run (bench.py matches it)")
    ap.add_argument("--dof", type=int, default=7, help="robot DOF of the profiled build (10: mobile)")
    ap.add_argument("--kernel", default="k_sqp")
    ap.add_argument("--ipw", type=int, default=4, help="instances per wavefront (4 Panda, 2 mobile build)")
    ap.add_argument("--ns", default="mpcc", help="kernel namespace (mpcc_m10 for the mobile build)")
    ap.add_argument("--grid", type=int, default=None,
                    help="grid size (threads) of the profiled launches (default: batch / ipw waves; k_sqp with solo "
                         "waves launches 64 more)")
    ap.add_argument("--traffic-name", default=None,
                    help="traffic file name under profiles/ (default pmc_traffic_<kernel>.json, read by bench.py)")
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(args.dir, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{args.round}_kernel_stats.csv"))
    grid = args.grid or (args.batch + args.ipw - 1) // args.ipw * 64
    merged = collections.defaultdict(dict)
    for p in ("p1", "p2", "p3", "p4", "p5"):
        for k, v in load_pmc(args.dir, p).items():
            if v["grid"] == grid and (v["kernel"].startswith(f"void {args.ns}::{args.kernel}<")  # template kernels
                                      or v["kernel"].startswith(f"{args.ns}::{args.kernel}(")):
                merged[p + ":" + str(k)] = v
    per = collections.defaultdict(list)
    for key, v in merged.items():
        for c, x in v.items():
            if c not in ("grid", "kernel"):
                per[c].append(x)
    avg = {c: sum(x) / len(x) for c, x in per.items()}
    out = {"kernel": args.kernel, "batch": args.batch, "N": args.N, "launches_averaged": len(per.get("FETCH_SIZE", [])),
           "counters_avg_per_launch": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rd = 2.0 * avg["FETCH_SIZE"] * 1024.0
        wr = avg["WRITE_SIZE"] * 1024.0
        out["hbm_read_bytes_per_launch"] = rd
        out["hbm_write_bytes_per_launch"] = wr
        out["hbm_bytes_per_launch"] = rd + wr
        with open(os.path.join(prof, args.traffic_name or f"pmc_traffic_{args.kernel}.json"), "w") as f:
            json.dump({"kernel": args.kernel, "batch": args.batch, "N": args.N, "mask": args.mask, "dof": args.dof, "hbm_bytes_per_launch": rd + wr,
                       "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                       "source": f"profiles/{args.round}_{args.kernel}_pmc.json"}, f, indent=1)
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: avg.get(k, 0) / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")}
    with open(os.path.join(prof, f"{args.round}_{args.kernel}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
