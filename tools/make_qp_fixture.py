"""Generate tests/golden/qp_dense.npz: dense reference-layout QPs assembled and solved by tools/qp_restate.py.

Inputs (linearization points) come from the oracle's closed loop on the default track, the way the engine
meets them: the shifted warm start of a pool step with joint noise, its frozen stage records (the oracle's
RobotData restatement, pinned by the reference FK/Jacobian KATs) and the current input.  Everything the
assembly and the solve compute is tools/qp_restate.py's (written from the reference sources; it imports
neither oracle/ nor the product).  Parameters are read from the reference's own JSON files
(/root/reference/cpp/Params) and the track from its track.json, offset to the end-effector start.

    python tools/make_qp_fixture.py [--ref /root/reference]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import qp_restate as qr  # noqa: E402

N = 20
SEED = 0x4D504343
OBS = (0.48, 0.218, 0.521, 5.0)  # main_w_sim.py:42-45


def coo(M):
    r, c = np.nonzero(M)
    return r.astype(np.int32), c.astype(np.int32), M[r, c]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "qp_dense.npz"))
    args = ap.parse_args()
    from helpers import Q0, make_oracle, oracle_pool  # inputs only (linearization points and stage records)

    P = qr.load_params(os.path.join(args.ref, "cpp", "Params"))
    cases = []
    for mask, obs, label in ((2, (3.0, 3.0, 3.0, 0.0), "mask2"), (7, OBS, "mask7")):
        o, Po, _ = make_oracle(N=N, max_iter=2, mask=mask)
        ee = o.fk(Q0)[0]
        X, Y, Z, R = qr.load_track(os.path.join(args.ref, "cpp", "Params", "track.json"), ee)
        o.set_track(X, Y, Z, np.array(R))
        pool = oracle_pool(o, 60, obs=obs)
        rng = np.random.default_rng(SEED + mask)
        for j in range(12):
            t = 3 + 4 * j  # the warm start the engine meets at pool step t + 1
            g = pool["guess"][t + 1].copy()
            noise = (0.002, 0.01, 0.03)[j % 3]
            g[:, :7] += rng.normal(0, noise, (N + 1, 7))
            g[:N, 9:] += rng.normal(0, noise, (N, 8))
            recs = np.stack([o.robot_record(g[k, :7], obs[:3], obs[3]) for k in range(N + 1)])
            cases.append(dict(mask=mask, label=f"{label}_t{t + 1}_n{noise}", guess=g, recs=recs,
                              ucur=pool["u0"][t + 1].copy(), X=np.array(X), Y=np.array(Y), Z=np.array(Z),
                              R=np.array(R).reshape(-1, 9)))
        o.close()
    track = qr.Track(cases[0]["X"], cases[0]["Y"], cases[0]["Z"], cases[0]["R"])
    out = {"N": np.int32(N), "n_cases": np.int32(len(cases)), "X": cases[0]["X"], "Y": cases[0]["Y"],
           "Z": cases[0]["Z"], "R": cases[0]["R"]}
    for k in qr.PARAM_SCALARS:
        out["param_" + k] = np.float64(P[k])
    for k in qr.PARAM_VECTORS:
        out["param_" + k] = P[k]
    for i, cs in enumerate(cases):
        assert np.array_equal(cs["X"], out["X"]) and np.array_equal(cs["R"], out["R"])
        qp = qr.assemble(P, track, cs["guess"], cs["recs"], cs["ucur"], N, cs["mask"])
        s, info = qr.solve_qp(qp)
        pr, pc, pv = coo(qp["P"])
        ar, ac, av = coo(qp["A"])
        pre = f"c{i}_"
        out.update({pre + "mask": np.int32(cs["mask"]), pre + "guess": cs["guess"], pre + "recs": cs["recs"],
                    pre + "ucur": cs["ucur"], pre + "obj": np.float64(qp["obj"]), pre + "q": qp["q"],
                    pre + "c": qp["c"], pre + "l": qp["l"], pre + "u": qp["u"], pre + "P_r": pr, pre + "P_c": pc,
                    pre + "P_v": pv, pre + "A_r": ar, pre + "A_c": ac, pre + "A_v": av, pre + "step": s,
                    pre + "active": np.int32(info["active"])})
        print(f"{i:2d} {cs['label']:22s} obj {qp['obj']:.6g} ipm {info['ipm_iters']} polished {info['polished']} "
              f"active {info['active']} viol {info['primal_violation']:.1e} stat {info['kkt_stationarity']:.1e}")
    np.savez_compressed(args.out, **out)
    print("wrote", args.out, os.path.getsize(args.out), "bytes")


if __name__ == "__main__":
    main()
