"""Per-stream timeline of a rocprofv3 kernel trace (bench.py under `rocprofv3 --kernel-trace`): for each queue, the
kernels of the last control steps with their durations and the gaps before them, and the mean duration / gap per
kernel name over the timed steps.  Shows where a controller group's period goes besides its QP solve.

    python tools/trace_timeline.py gpurun_out/s3/trace [--steps 20] [--kernel-prefix mpcc]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=20, help="timed steps at the end of the trace")
    ap.add_argument("--show", type=int, default=1, help="steps printed in full per queue")
    args = ap.parse_args()
    f = glob.glob(os.path.join(args.dir, "*kernel_trace.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    for q, ks in sorted(byq.items()):
        ks.sort()
        # a control step of a group ends with its finalize kernel
        ends = [i for i, k in enumerate(ks) if k[2].endswith("k_finalize")]
        if len(ends) < args.steps + 1:
            continue
        first = ends[-args.steps - 1] + 1
        seg = ks[first:ends[-1] + 1]
        per = collections.defaultdict(lambda: [0.0, 0.0, 0])
        prev_end = ks[first - 1][1]
        for s, e, n in seg:
            per[n][0] += (e - s) * 1e-3
            per[n][1] += max(0, s - prev_end) * 1e-3
            per[n][2] += 1
            prev_end = e
        span = (seg[-1][1] - ks[first - 1][1]) * 1e-3 / args.steps
        print(f"queue {q}: {len(seg)} kernels over {args.steps} steps, {span:.1f} us per step")
        for n, (dur, gap, cnt) in sorted(per.items(), key=lambda kv: -kv[1][0]):
            print(f"  {n:45s} x{cnt / args.steps:4.1f}/step  {dur / cnt:9.1f} us  gap before {gap / cnt:7.1f} us")
        last = ends[-args.show - 1] + 1
        prev_end = ks[last - 1][1]
        for s, e, n in ks[last:ends[-1] + 1]:
            print(f"    +{(s - prev_end) * 1e-3:7.1f} us gap  {n:45s} {(e - s) * 1e-3:9.1f} us")
            prev_end = e


if __name__ == "__main__":
    main()
