"""Write mpcc_manipulator_amd/data/Params/ in the reference's file layout (cpp/Params/: config.json with
relative paths, model.json, cost.json, bounds.json, normalization.json, sqp.json, track.json with
X, Y, Z, quat_X..quat_W arrays) from this repo's merged data (data/params/default_params.json,
default_track.json), so that code written against the reference (python/MPCC/MPCC.py: pkg_path +
"Params/config.json") finds its files under MPCC_WRAPPER.pkg_path.     python tools/make_params_dir.py"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "mpcc_manipulator_amd", "data")


def main():
    with open(os.path.join(DATA, "params", "default_params.json")) as f:
        merged = json.load(f)
    with open(os.path.join(DATA, "params", "default_track.json")) as f:
        pts = json.load(f)["points"]
    out = os.path.join(DATA, "Params")
    os.makedirs(out, exist_ok=True)
    cfg = dict(merged["config"])
    cfg.update({"model_path": "Params/model.json", "cost_path": "Params/cost.json", "bounds_path": "Params/bounds.json",
                "track_path": "Params/track.json", "normalization_path": "Params/normalization.json",
                "sqp_path": "Params/sqp.json"})
    files = {"config.json": cfg, "model.json": merged["model"], "cost.json": merged["cost"], "bounds.json": merged["bounds"],
             "normalization.json": merged["normalization"], "sqp.json": merged["sqp"],
             "track.json": {k: [p[i] for p in pts] for i, k in enumerate(["X", "Y", "Z", "quat_X", "quat_Y", "quat_Z", "quat_W"])}}
    for name, obj in files.items():
        with open(os.path.join(out, name), "w") as f:
            json.dump(obj, f, indent=2)
            f.write("\n")
    print("wrote", sorted(files))


if __name__ == "__main__":
    main()
