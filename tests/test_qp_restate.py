"""The QP of one SQP iteration pinned independently of the oracle (VERDICT r02 "What's missing" 1).

tests/golden/qp_dense.npz holds 24 linearization points (N = 20; 12 with BASELINE configs[1]'s bounds +
singularity rows, 12 with all 11 rows and the main_w_sim.py obstacle) with the dense reference-layout QP
(P, q, A, c, l, u of osqp_interface.cpp:129-389) and its exact solution, both computed by tools/qp_restate.py:
a numpy restatement written from the reference's osqp_interface.cpp, cost.cpp, constraints.cpp, bounds.cpp and
model.cpp that imports neither oracle/ nor the product, with parameters read from the reference's own
cpp/Params/*.json (tools/make_qp_fixture.py).

CPU: the fixture reproduces from its inputs; the oracle's dense layout equals it entry for entry (<= 1e-12);
the oracle's structured (Riccati) and dense QP solves equal its solution (<= 1e-8).
GPU: the engine's QP solve (the 16-lane interior point of ipm.hip) equals the fixture's solution (<= 1e-8).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
FIX = os.path.join(ROOT, "tests", "golden", "qp_dense.npz")


@pytest.fixture(scope="module")
def fixture():
    f = np.load(FIX, allow_pickle=False)
    d = {k: f[k] for k in f.files}
    N = int(d["N"])
    nv = 17 * N + 9
    nc = 45 * N + 29
    cases = []
    for i in range(int(d["n_cases"])):
        p = f"c{i}_"
        Pm = np.zeros((nv, nv)); Pm[d[p + "P_r"], d[p + "P_c"]] = d[p + "P_v"]
        A = np.zeros((nc, nv)); A[d[p + "A_r"], d[p + "A_c"]] = d[p + "A_v"]
        cases.append(dict(mask=int(d[p + "mask"]), guess=d[p + "guess"], recs=d[p + "recs"], ucur=d[p + "ucur"],
                          obj=float(d[p + "obj"]), P=Pm, q=d[p + "q"], A=A, c=d[p + "c"], l=d[p + "l"], u=d[p + "u"],
                          step=d[p + "step"]))
    params = {k[6:]: d[k] for k in d if k.startswith("param_")}
    params = {k: (float(v) if v.ndim == 0 else v) for k, v in params.items()}
    return dict(N=N, cases=cases, params=params, track=(d["X"], d["Y"], d["Z"], d["R"]))


def test_fixture_covers_both_masks_and_active_sets(fixture):
    masks = [c["mask"] for c in fixture["cases"]]
    assert masks.count(2) == 12 and masks.count(7) == 12
    # the solutions sit on bounds and collision rows, not only in the interior
    act = []
    for c in fixture["cases"]:
        lo, hi = c["l"] - c["c"], c["u"] - c["c"]
        r = c["A"] @ c["step"]
        fin_hi, fin_lo = c["u"] < 1e20, c["l"] > -1e20
        act.append(int(np.sum(fin_hi & (np.abs(r - hi) < 1e-9) & (lo != hi)) + np.sum(fin_lo & (np.abs(r - lo) < 1e-9) & (lo != hi))))
    assert sum(a > 5 for a in act) >= 6, act


def test_fixture_reproduces_from_inputs(fixture):
    """tools/qp_restate.py assembles and solves the stored QPs again (guards the fixture and the restatement)."""
    import qp_restate as qr
    P, N = fixture["params"], fixture["N"]
    track = qr.Track(*fixture["track"])
    for c in fixture["cases"][::5]:
        qp = qr.assemble(P, track, c["guess"], c["recs"], c["ucur"], N, c["mask"])
        for k in ("P", "q", "A", "c", "l", "u"):
            assert np.array_equal(qp[k], c[k]), k
        s, info = qr.solve_qp(qp)
        assert info["polished"] and np.abs(s - c["step"]).max() < 1e-10


def _oracle(fixture, mask):
    from helpers import make_oracle
    o, Po, _ = make_oracle(N=fixture["N"], max_iter=2, mask=mask)
    # the oracle's parameters (this repo's JSON re-serialization) are the reference files' values
    pr = fixture["params"]
    for k_or, k_fx in (("Ts", "Ts"), ("s_trust_region", "s_trust_region"), ("q_c", "q_c"), ("qp_r_ddq", "r_ddq"),
                       ("cost_tol_sing", "tol_sing"), ("cost_tol_selcol", "tol_selcol"), ("con_tol_envcol", "tol_envcol")):
        assert float(Po[k_or]) == pr[k_fx], k_or
    for k in ("Tx", "Tu", "lx", "ux", "lu", "uu", "lddq", "uddq"):
        assert np.array_equal(np.asarray(Po[k], float), pr[k]), k
    X, Y, Z, R = fixture["track"]
    o.set_track(X, Y, Z, R.reshape(-1, 3, 3))
    return o


@pytest.mark.parametrize("mask", [2, 7])
def test_oracle_dense_layout_matches_restatement(fixture, oracle_lib, mask):
    """oracle_dense_qp (the oracle's verbatim reference layout) == the independent restatement, <= 1e-12."""
    o = _oracle(fixture, mask)
    n = 0
    for c in fixture["cases"]:
        if c["mask"] != mask:
            continue
        d = o.dense_qp(c["guess"], c["recs"], c["ucur"])
        assert abs(d["obj"] - c["obj"]) <= 1e-12 * max(1.0, abs(c["obj"]))
        for k, ref in (("P", c["P"]), ("g", c["q"]), ("A", c["A"]), ("c", c["c"])):
            err = np.abs(d[k] - ref).max() / max(1.0, np.abs(ref).max())
            assert err <= 1e-12, (k, err)
        for k in ("l", "u"):
            inf = np.abs(c[k]) >= 1e20
            assert np.array_equal(np.abs(d[k]) >= 1e20, inf), k
            assert np.array_equal(np.sign(d[k][inf]), np.sign(c[k][inf])), k
            assert np.abs(d[k][~inf] - c[k][~inf]).max() <= 1e-12, k
        n += 1
    assert n == 12
    o.close()


@pytest.mark.parametrize("mask", [2, 7])
def test_oracle_qp_solutions_match_restatement(fixture, oracle_lib, mask):
    """The oracle's structured Riccati interior point (mode 0, what the engine restates) and its dense-layout
    solve (mode 1) reach the restatement's exact solution, <= 1e-8."""
    o = _oracle(fixture, mask)
    for c in fixture["cases"]:
        if c["mask"] != mask:
            continue
        for mode in (0, 1):
            rc, s, _ = o.solve_qp(c["guess"], c["recs"], c["ucur"], mode=mode)
            assert rc == 0, (mode, rc)
            assert np.abs(s - c["step"]).max() < 1e-8, (mode, np.abs(s - c["step"]).max())
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mask", [2, 7])
def test_engine_qp_step_matches_restatement(fixture, built_lib, mask):
    """The engine's QP solve (ipm.hip, through the C ABI's mpcc_debug_solve_qp) reaches the independent
    restatement's exact solution of the reference-layout QP, <= 1e-8."""
    import mpcc_manipulator_amd as m
    N = fixture["N"]
    cs = [c for c in fixture["cases"] if c["mask"] == mask]
    eng = m.Engine(m.load_params(N=N, overrides={"sqp": {"max_iter": 2}}), max_batch=len(cs), constraint_mask=mask)
    X, Y, Z, R = fixture["track"]
    eng.set_track(X, Y, Z, R.reshape(-1, 3, 3))
    step, st, it = eng.solve_qp(np.stack([c["guess"] for c in cs]), np.stack([c["recs"] for c in cs]),
                                np.stack([c["ucur"] for c in cs]))
    assert np.all(st == 0), st
    for b, c in enumerate(cs):
        assert np.abs(step[b] - c["step"]).max() < 1e-8, (b, np.abs(step[b] - c["step"]).max())
    eng.close()
