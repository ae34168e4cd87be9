"""Convert the reference's run-time DATA files into this repo's data directory.

This is a one-off import tool (run in the build container, where the read-only reference
checkout exists at /root/reference).  It copies no source code: it parses

* the MLP parameter text files  ``cpp/NNmodel/{self,env}/parameter/{weight,bias}_<i>.txt``
  (row-major whitespace-separated decimals, read by the reference into ``double`` with
  ``operator>>`` — SelfCollisionModel.cpp:19-58) and stores them as raw little-endian
  float64 blobs (``data/nn/<net>/<name>.f64``) plus a manifest with the shapes; Python's
  ``float()`` and libstdc++'s ``strtod`` are both correctly rounded, so the doubles are
  bit-identical to what the reference loads;
* the parameter JSON files ``cpp/Params/{model,cost,bounds,normalization,sqp,config}.json``
  into one merged ``data/params/default_params.json`` (same keys, one section per file);
* the default track ``cpp/Params/track.json`` into ``data/params/default_track.json`` as a
  list of ``[x, y, z, qx, qy, qz, qw]`` points.

The loaders in ``mpcc_manipulator_amd`` read both this layout and the reference's own
file layout (``PathToJson``), so a user can point the engine at their existing Params/.
"""
import json
import os
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/cpp"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "mpcc_manipulator_amd", "data")

# network name -> (n_input (before NeRF), n_output, hidden sizes); osqp_interface.cpp:35-43
NETS = {"self": (7, 1, [256, 64]), "env": (10, 9, [256, 256, 256, 256])}


def read_numbers(path):
    with open(path) as f:
        return np.array([float(t) for t in f.read().split()], dtype=np.float64)


def main():
    os.makedirs(os.path.join(OUT, "params"), exist_ok=True)
    for net, (n_in, n_out, hidden) in NETS.items():
        d_out = os.path.join(OUT, "nn", net)
        os.makedirs(d_out, exist_ok=True)
        dims = [3 * n_in] + hidden + [n_out]  # NeRF input = [x, sin x, cos x]
        manifest = {"n_input": n_in, "n_output": n_out, "hidden": hidden, "nerf": True,
                    "layers": []}
        for i in range(len(dims) - 1):
            w = read_numbers(os.path.join(REF, "NNmodel", net, "parameter", f"weight_{i}.txt"))
            b = read_numbers(os.path.join(REF, "NNmodel", net, "parameter", f"bias_{i}.txt"))
            assert w.size == dims[i + 1] * dims[i], (net, i, w.size)
            assert b.size == dims[i + 1], (net, i, b.size)
            w.astype("<f8").tofile(os.path.join(d_out, f"weight_{i}.f64"))
            b.astype("<f8").tofile(os.path.join(d_out, f"bias_{i}.f64"))
            manifest["layers"].append({"rows": dims[i + 1], "cols": dims[i],
                                       "weight": f"weight_{i}.f64", "bias": f"bias_{i}.f64"})
        with open(os.path.join(d_out, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)

    merged = {}
    for sec in ["model", "cost", "bounds", "normalization", "sqp", "config"]:
        with open(os.path.join(REF, "Params", sec + ".json")) as f:
            merged[sec] = json.load(f)
    with open(os.path.join(OUT, "params", "default_params.json"), "w") as f:
        json.dump(merged, f, indent=2, sort_keys=True)

    with open(os.path.join(REF, "Params", "track.json")) as f:
        t = json.load(f)
    keys = ["X", "Y", "Z", "quat_X", "quat_Y", "quat_Z", "quat_W"]
    pts = [list(p) for p in zip(*[t[k] for k in keys])]
    with open(os.path.join(OUT, "params", "default_track.json"), "w") as f:
        f.write('{"format": "points_xyz_qxqyqzqw", "points": [\n')
        f.write(",\n".join(json.dumps(p) for p in pts))
        f.write("\n]}\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
