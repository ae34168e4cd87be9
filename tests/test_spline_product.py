"""The product's track spline construction (host, csrc/host_spline.cpp through the C ABI) against
(1) a fixture from an independent restatement (tools/spline_restate.py -> tests/golden/track_tables.npz,
written from the reference sources, not from oracle/ or the product), and
(2) the reference's own spline tests, ported to run on the product (cpp/include/Tests/spline_test.h:31-239,
same thresholds).  CPU only: the track tables are built on the host (mpcc_track_build_host).
"""
import os

import numpy as np
import pytest

from helpers import SEED

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def m(built_lib):
    import mpcc_manipulator_amd as mm
    return mm


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(ROOT, "tests", "golden", "track_tables.npz"), allow_pickle=False)


@pytest.mark.parametrize("name", ["default", "helix"])
def test_track_tables_match_independent_restatement(m, gold, name):
    X, Y, Z, R = (gold[f"{name}_{k}"] for k in "XYZR")
    s, Xo, Yo, Zo, Ro, L = m.build_track_host(X, Y, Z, R.reshape(-1, 3, 3))
    assert np.allclose(s, gold[f"{name}_path_s"], rtol=1e-13, atol=1e-15)
    for a, k in ((Xo, "X"), (Yo, "Y"), (Zo, "Z")):
        assert np.allclose(a, gold[f"{name}_path_{k}"], rtol=1e-13, atol=1e-15), k
    assert np.allclose(Ro.reshape(-1, 9), gold[f"{name}_path_R"], rtol=1e-12, atol=1e-14)
    assert abs(L - gold[f"{name}_path_s"][-1]) <= 1e-14
    pos, d1, d2, Rq, dR = m.eval_track_host(X, Y, Z, R.reshape(-1, 3, 3), gold[f"{name}_sq"])
    assert np.allclose(pos, gold[f"{name}_pos"], rtol=1e-12, atol=1e-14)
    assert np.allclose(d1, gold[f"{name}_d1"], rtol=1e-10, atol=1e-12)
    assert np.allclose(d2, gold[f"{name}_d2"], rtol=1e-8, atol=1e-9)
    assert np.allclose(Rq.reshape(-1, 9), gold[f"{name}_Rq"], rtol=1e-12, atol=1e-14)
    assert np.allclose(dR, gold[f"{name}_dR"], rtol=1e-10, atol=1e-12)


def test_spline_cos(m):
    """spline_test.h:31-83 (TestSpline): natural cubic spline of cos on 50 regular points in [0, pi], checked at
    100 points: mean errors of value <= 1e-4, derivative <= 1e-3, second derivative <= 1e-1."""
    NT, NV = 50, 100
    x = np.linspace(0, np.pi, NT)
    xt = np.linspace(0, np.pi, NV)
    out = m.cubic_spline_host(x, np.cos(x), xt, regular=True)
    assert np.linalg.norm(out[:, 0] - np.cos(xt)) / NV <= 1e-4
    assert np.linalg.norm(out[:, 1] + np.sin(xt)) / NV <= 1e-3
    assert np.linalg.norm(out[:, 2] + np.cos(xt)) / NV <= 1e-1


def _rot_zyx(r, p, y):
    """AngleAxis(y, Z) * AngleAxis(p, Y) * AngleAxis(r, X) (spline_test.h:116-118)."""
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def test_spline_rot(m, built_lib):
    """spline_test.h:85-168 (TestSplineRot): rotation spline through roll 0, 60, 120, 180, 120, 60, 0 deg at
    x = 0..6 (irregular fit), checked at 25 points: the first-order prediction Exp(dR dx) R(x) of R(x + 0.01)
    has a summed Log error < 1e-2."""
    import sys
    sys.path.insert(0, os.path.dirname(built_lib))
    import MPCC_WRAPPER as W
    x = np.arange(7.0)
    roll = np.array([0, 60, 120, 180, 120, 60, 0]) * np.pi / 180
    R = np.array([_rot_zyx(r, 0, 0) for r in roll])
    xt = np.linspace(0, 6, 6 * 3 + 7)
    Rt, dRt = m.rot_spline_host(x, R, xt, regular=False)
    Rr, _ = m.rot_spline_host(x, R, xt + 0.01, regular=False)
    err = 0.0
    for i in range(len(xt)):
        est = W.ExpMatrix(W.getSkewMatrix(dRt[i] * 0.01)) @ Rt[i]
        err += np.linalg.norm(W.getInverseSkewVector(W.LogMatrix(Rr[i].T @ est)))
    assert err < 1e-2, err


def test_arc_length_spline_half_circle(m):
    """spline_test.h:170-239 (TestArcLengthSpline): 50 randomly spaced points on a half circle (ends fixed),
    gen6DSpline, then 200 validation points: ||error|| / 200 <= 0.03."""
    NT, NV = 50, 200
    rng = np.random.default_rng(SEED + 170)
    phi = np.sort(rng.uniform(0, np.pi, NT))
    phi[0], phi[-1] = 0.0, np.pi
    X, Y, Z = np.zeros(NT), np.cos(phi), np.sin(phi)
    R = np.tile(np.eye(3), (NT, 1, 1))
    phiv = np.linspace(0, np.pi, NV)
    pos = m.eval_track_host(X, Y, Z, R, phiv)[0]
    err = np.sqrt(pos[:, 0] ** 2 + (pos[:, 1] - np.cos(phiv)) ** 2 + (pos[:, 2] - np.sin(phiv)) ** 2)
    assert np.linalg.norm(err) / NV <= 0.03
