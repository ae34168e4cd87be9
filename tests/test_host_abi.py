"""CPU tests of the C ABI library (include/mpcc_engine.h) — host-only entry points, no GPU.

* the shared library loads and exports every function the header declares;
* the Params JSON loader (host_params.cpp) equals an independent Python restatement of the
  reference's loaders and override rules (tests/refparams.py), for constructor and setParam semantics;
* the host arc-length spline build (host_spline.cpp) is bit-identical to the oracle's track tables;
* the product path fails loudly on a machine without a GPU (no CPU fallback).
"""
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

import refparams as rp
from helpers import Q0, make_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpcc_engine.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mpcc_[a-z0-9_]+)\s*\(", src)))


def test_header_functions_exported(built_lib):
    L = C.CDLL(built_lib)
    names = declared_functions()
    assert len(names) >= 25, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version(built_lib):
    import mpcc_manipulator_amd as m
    L = m.lib()
    v = L.mpcc_abi_version()
    assert v >= 1


def _params_dict(p):
    d = p.as_dict()
    for k, v in d.items():
        if isinstance(v, list):
            d[k] = [float(x) for x in v]
    return d


@pytest.mark.parametrize("ctor", [True, False])
def test_params_loader_matches_reference_semantics(built_lib, ctor):
    import mpcc_manipulator_amd as m
    ov = {"param": {"max_dist_proj": 0.05, "s_trust_region": 0.3},
          "cost": {"qC": 123.0, "rddq": 7.0},
          "normalization": {"q1": 3.5, "dVs": 4.0},
          "sqp": {"max_iter": 3, "eps_prim": 0.2}}
    p = _params_dict(m.load_params(N=20, overrides=ov, ctor_semantics=ctor))
    r = rp.resolve(N=20, overrides=ov, ctor_overrides=ctor)
    for k, v in r.items():
        if k in ("constraint_mask",):
            continue
        got = p[k]
        if isinstance(v, list):
            assert np.array_equal(np.array(got, float), np.array(v, float)), k
        else:
            assert float(got) == float(v), (k, got, v)
    # quirk Q8: the QP's r_ddq never sees the override; Cost's weights do
    assert p["qp_r_ddq"] == rp.load_default_sections()["cost"]["rddq"]
    assert p["q_c"] == 123.0


def test_params_loader_rejects_unknown_keys(built_lib):
    import mpcc_manipulator_amd as m
    with pytest.raises(ValueError):
        m.load_params(N=20, overrides={"cost": {"not_a_key": 1.0}})
    with pytest.raises(ValueError):
        m.load_params(N=20, overrides={"nonsense": {"qC": 1.0}})


def test_params_loader_bad_path(built_lib):
    import mpcc_manipulator_amd as m
    with pytest.raises(m.MpccError):
        m.load_params(N=20, merged="/nonexistent/params.json")


def test_host_track_tables_match_oracle(built_lib, oracle_lib):
    import mpcc_manipulator_amd as m
    o, P, track = make_oracle(N=20, max_iter=2, mask=7)
    X, Y, Z, R = track
    s, Xh, Yh, Zh, Rh, L = m.build_track_host(X, Y, Z, R)
    so, Xo, Yo, Zo, Ro = o.track_path()
    assert np.array_equal(s, so) and np.array_equal(Xh, Xo) and np.array_equal(Yh, Yo) and np.array_equal(Zh, Zo)
    assert np.array_equal(Rh.reshape(-1), np.asarray(Ro).reshape(-1))
    assert L == o.track_length()


def test_default_track_offset(built_lib, oracle_lib):
    """Track::getTrack (track.cpp:56-66): way-points offset so that the path starts at the EE."""
    import mpcc_manipulator_amd as m
    o, _, _ = make_oracle(N=20, max_iter=2, mask=7)
    ee = o.fk(Q0)[0]
    X, Y, Z, q = m.load_default_track()
    Xo, Yo, Zo, R = m.track_from_points(X, Y, Z, q, ee)
    assert np.allclose([Xo[0], Yo[0], Zo[0]], ee)
    Xr, Yr, Zr, Rr = rp.default_track_xyzr(ee)
    assert np.allclose(Xo, Xr) and np.allclose(Yo, Yr) and np.allclose(Zo, Zr)
    assert np.allclose(R, np.array(Rr))


def test_quaternion_rotation_orthonormal(built_lib):
    import mpcc_manipulator_amd as m
    rng = np.random.default_rng(3)
    R = m.quat_to_rot(rng.normal(size=(50, 4)))
    assert np.allclose(np.einsum("nij,nkj->nik", R, R), np.eye(3), atol=1e-12)
    assert np.allclose(np.linalg.det(R), 1.0)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_engine_fails_loudly_without_gpu(built_lib):
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20)
    with pytest.raises(m.MpccError):
        m.Engine(params, max_batch=4, constraint_mask=2)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
@pytest.mark.parametrize("max_iter", [3, 10, 15, 16, 100])
def test_bfgs_passes_validation(built_lib, max_iter):
    """Damped BFGS (osqp_interface.cpp:683-715) takes any max_iter, the reference sqp.json's 100 included: past
    LRX = 28 low-rank terms the quasi-Newton matrix restarts from that iteration's exact Hessian,
    so validation accepts it and without a GPU creation fails only at the device."""
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20, overrides={"sqp": {"use_BFGS": 1.0, "max_iter": max_iter}})
    assert params.use_BFGS == 1
    with pytest.raises(m.MpccError) as e:
        m.Engine(params, max_batch=4, constraint_mask=2)
    assert "max_iter" not in str(e.value)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_soc_passes_validation(built_lib):
    """do_SOC (SecondOrderCorrection, osqp_interface.cpp:506-535, 658-681) is supported: parameter
    validation accepts it, and without a GPU creation fails only at the device."""
    import mpcc_manipulator_amd as m
    params = m.load_params(N=20, overrides={"sqp": {"do_SOC": 1.0}})
    assert params.do_SOC == 1
    with pytest.raises(m.MpccError) as e:
        m.Engine(params, max_batch=4, constraint_mask=2)
    assert "not supported" not in str(e.value)


def test_host_integrator_matches_oracle(built_lib, oracle_lib):
    """integrator.py (Integrator::simTimeStep, integrator.cpp:55-68) vs the oracle, batched."""
    from mpcc_manipulator_amd.integrator import sim_time_step
    o, _, _ = make_oracle(N=20, max_iter=2, mask=7)
    rng = np.random.default_rng(9)
    x = rng.normal(size=(6, 9)); u = rng.normal(size=(6, 8))
    xs = sim_time_step(x, u, 0.01)
    for i in range(6):
        assert np.allclose(xs[i], o.sim_time_step(x[i], u[i], 0.01), rtol=0, atol=1e-15)


def test_cpp_surface_exported(built_lib):
    """The C++ host mirror (include/mpcc_mpc.hpp) is compiled into the same library."""
    import subprocess
    syms = subprocess.run(["nm", "-DC", built_lib], capture_output=True, text=True, check=True).stdout
    for s in ("mpcc_amd::MPC::runMPC_(", "mpcc_amd::MPC::setTrack(", "mpcc_amd::MPC::setParam(",
              "mpcc_amd::BatchMPC::runMPCBatch(", "mpcc_amd::loadTrack(", "mpcc_amd::defaultPaths("):
        assert s in syms, s


@pytest.mark.skipif(torch.cuda.device_count() > 0, reason="checks the no-GPU failure path")
def test_cpp_example_fails_loudly_without_gpu(built_lib):
    """examples/mpc_closed_loop on a machine without a GPU exits 1 with the HIP error (no fallback)."""
    import subprocess
    exe = os.path.join(os.path.dirname(built_lib), "mpc_closed_loop")
    r = subprocess.run([exe, os.path.join(ROOT, "mpcc_manipulator_amd", "data"), "1"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1
    assert "mpcc_create" in r.stderr and r.stdout == ""
