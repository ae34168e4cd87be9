"""Golden fixture of the track spline tables from the independent restatement tools/spline_restate.py
(not from oracle/ or the product): tests/golden/track_tables.npz.

Two tracks: the reference's default track (Params/track.json, offset to the end-effector start
(0.5545, 0, 0.5211) = the reference's own KAT at q0, python/main_utils.py:50-52, as Track::getTrack does,
track.cpp:56-66) and a helix with irregular point spacing and a rotation turning about a varying axis.
Stored per track: way-points, the final regular path data (getPathData) and the five evaluations at 67
arc lengths (inside, at the grid points, at both ends and outside [0, L]).

    python tools/make_spline_fixture.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import refparams  # noqa: E402  (test-side JSON restatement; independent of oracle/ and the product)
import spline_restate as sr  # noqa: E402


def helix_track():
    rng = np.random.default_rng(0x5EED)
    t = np.sort(np.concatenate([[0.0, 1.0], rng.uniform(0, 1, 38)]))
    X = (0.4 + 0.15 * np.cos(3 * t)).tolist()
    Y = (0.15 * np.sin(3 * t)).tolist()
    Z = (0.3 + 0.4 * t).tolist()
    R = []
    for ti in t:
        ax = np.array([np.sin(2 * ti), np.cos(2 * ti), 0.5])
        ax /= np.linalg.norm(ax)
        R.append(sr.exp_matrix(sr.skew((ax * 1.2 * ti).tolist())))
    return X, Y, Z, R


def main():
    out = {}
    X, Y, Z, R = refparams.default_track_xyzr([0.5545, 0.0, 0.5211])
    tracks = {"default": (X, Y, Z, R), "helix": helix_track()}
    for name, (X, Y, Z, R) in tracks.items():
        (s, Xf, Yf, Zf, Rf), fin = sr.gen6d(X, Y, Z, R)
        L = s[-1]
        sq = np.concatenate([np.linspace(0, L, 61), [s[37], s[50], L, 0.0, -0.05, L + 0.05]])
        ev = [sr.evaluate(fin, float(v)) for v in sq]
        out[f"{name}_X"], out[f"{name}_Y"], out[f"{name}_Z"] = np.array(X), np.array(Y), np.array(Z)
        out[f"{name}_R"] = np.array(R).reshape(-1, 9)
        out[f"{name}_path_s"], out[f"{name}_path_X"] = np.array(s), np.array(Xf)
        out[f"{name}_path_Y"], out[f"{name}_path_Z"] = np.array(Yf), np.array(Zf)
        out[f"{name}_path_R"] = np.array(Rf).reshape(-1, 9)
        out[f"{name}_sq"] = sq
        out[f"{name}_pos"] = np.array([e[0] for e in ev])
        out[f"{name}_d1"] = np.array([e[1] for e in ev])
        out[f"{name}_d2"] = np.array([e[2] for e in ev])
        out[f"{name}_Rq"] = np.array([e[3] for e in ev]).reshape(-1, 9)
        out[f"{name}_dR"] = np.array([e[4] for e in ev])
    path = os.path.join(ROOT, "tests", "golden", "track_tables.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, "L =", out["default_path_s"][-1], out["helix_path_s"][-1])


if __name__ == "__main__":
    main()
