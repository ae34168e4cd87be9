"""Localize a difference between tail mode (csrc/ipm_tail.h) and the normal interior point: one QP per call
(mpcc_debug_solve_qp, B = 1, so the instance runs in tail mode from its first iteration when MPCC_TAIL=1), both
modes, after the same number of iterations (a library built with -DMPCC_DBG_IPM_STOP=K by tools/build_variant.sh),
then the first workspace field and stage that differ.

    for K in 1 2 3: bash tools/build_variant.sh stopK "-DMPCC_DBG_IPM_STOP=K"
    MPCC_ENGINE_LIB=mpcc_manipulator_amd/_build_vstopK/libmpcc_engine.so python tools/tail_ws_diff.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIELDS = ["SL", "LL", "SU", "LU", "ZX", "ZV"] + [f"KR{i}" for i in range(8)] + ["GVK", "AX", "AV", "GX"] + \
         [f"FI{i}" for i in range(4)] + ["SP", "LP", "PZ", "PA", "PD", "DX", "DV"] + [f"-{i}" for i in range(29, 35)] + \
         ["gx", "gv", "pv", "fv", "dvr", "cP", "wd", "pnew", "kff", "Pc0", "LF35", "dinv7", "u0", "kc0", "Y0", "Fc0"]


FIELDS2 = FIELDS[:29] + ["LF0", "LF1", "LF2"] + [f"u{i}" for i in range(8)] + [f"kc{i}" for i in range(8)]


def main():
    import mpcc_manipulator_amd as m
    f = np.load(os.path.join(ROOT, "tests", "golden", "qp_dense.npz"), allow_pickle=False)
    d = {k: f[k] for k in f.files}
    N = int(d["N"])
    for i in range(int(d["n_cases"])):
        p = f"c{i}_"
        mask = int(d[p + "mask"])
        if mask != 2:
            continue
        res = {}
        names = FIELDS2 if os.environ.get("DBG2") else FIELDS
        for tail in (1, 0):
            os.environ["MPCC_TAIL"] = str(tail)
            eng = m.Engine(m.load_params(N=N, overrides={"sqp": {"max_iter": 2}}), max_batch=1, constraint_mask=mask)
            eng.set_track(d["X"], d["Y"], d["Z"], d["R"].reshape(-1, 3, 3))
            step, st, it = eng.solve_qp(d[p + "guess"][None], d[p + "recs"][None], d[p + "ucur"][None])
            res[tail] = (step, st, it, eng.workspace(1)[0].reshape(N + 1, 51, 16)[:, :len(names), :].copy())
            eng.close()
        (s1, st1, it1, w1), (s0, st0, it0, w0) = res[1], res[0]
        same_step = np.array_equal(s1.view(np.int64), s0.view(np.int64))
        line = f"case {i}: it {it1[0]} {it0[0]} st {st1[0]} {st0[0]} step bitwise {same_step} max|dstep| {np.abs(s1 - s0).max():.3g}"
        diff = w1.view(np.int64) != w0.view(np.int64)
        if diff.any():
            bad = [(names[fi], int(np.nonzero(diff[:, fi, :].any(axis=1))[0][-1]), int(np.sum(diff[:, fi, :])),
                    float(np.abs(w1[:, fi, :] - w0[:, fi, :]).max())) for fi in range(len(names)) if diff[:, fi, :].any()]
            if os.environ.get("DBG2"):  # the lane-0 copy of L and 1/L_jj: which entries differ, stage by stage
                lf1, lf0 = w1[:, 29:32, :].reshape(N + 1, 48), w0[:, 29:32, :].reshape(N + 1, 48)
                for kk in range(N, -1, -1):
                    dd = np.nonzero(lf1[kk].view(np.int64) != lf0[kk].view(np.int64))[0]
                    if dd.size:
                        line += f" | stage {kk} L/dinv entries {dd.tolist()[:8]}"
                        break
            line += " | fields differing (name, highest stage, count, max):" + str(bad)
        print(line, flush=True)


if __name__ == "__main__":
    main()
