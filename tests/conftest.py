import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def built_lib():
    """The engine libraries, built in-tree if stale, and proven to be compiled from this tree's csrc/ and
    include/ (mpcc_build_id() = _build.source_hash()), so a GPU run cannot pass on a library of other sources."""
    from mpcc_manipulator_amd import _build, engine
    path = _build.build()
    want = _build.source_hash()
    for dof in (7, 10):
        if os.environ.get("MPCC_ENGINE_LIB" if dof == 7 else "MPCC_ENGINE_LIB_MOBILE"):
            continue  # an explicitly chosen variant library (tools/bounds_check.sh, bench variants)
        got = engine.build_id(dof)
        assert got == want, f"{engine.LIB_PATHS[dof]} was built from other sources ({got}) than this tree ({want})"
    return path


@pytest.fixture(autouse=True)
def _bounds_check_engines():
    """With a bounds-checked engine library loaded (MPCC_BOUNDS_CHECK builds), every test ends by asserting
    that no kernel computed an index outside its buffer."""
    yield
    if "mpcc_manipulator_amd.engine" not in sys.modules:
        return
    from mpcc_manipulator_amd import engine
    for e in list(engine.LIVE_CHECKED):
        if getattr(e, "h", None):
            f = e.bounds_flags(clear=True)
            assert f == 0, f"bounds-checked kernel index violation bits {f:#x} (csrc/dev_common.h BC_*)"


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle
