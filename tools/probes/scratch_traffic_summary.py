"""Summary of tools/probes/scratch_traffic_probe.hip under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate
passes): counter bytes (the counters are in KiB) against each kernel's algorithmic bytes.

    python tools/probes/scratch_traffic_summary.py gpurun_out/r03y > profiles/r03y_scratch_traffic_probe.json
"""
import collections
import csv
import json
import os
import sys


def main():
    d = sys.argv[1]
    known = {}
    with open(os.path.join(d, "probe_fetch.log")) as f:
        for line in f:
            if line.startswith("{"):
                r = json.loads(line)
                known[r["kernel"]] = r
    agg = collections.defaultdict(float)
    for name in ("fetch", "write"):
        with open(os.path.join(d, name, f"{name}_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0]
                agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]) * 1024.0
    out = {}
    for k, kn in known.items():
        fs, ws = agg[(k, "FETCH_SIZE")], agg[(k, "WRITE_SIZE")]
        out[k] = {"read_bytes": kn["read_bytes"], "write_bytes": kn["write_bytes"], "FETCH_SIZE_bytes": fs,
                  "WRITE_SIZE_bytes": ws, "read_bytes_over_FETCH_SIZE": kn["read_bytes"] / fs,
                  "write_bytes_over_WRITE_SIZE": kn["write_bytes"] / ws}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
