"""The interior point's algorithm constants are stated three times: the oracle (oracle/mpcc_oracle.cpp), the 16-lane
engine (csrc/ipm.hip, with its tail mode) and the 32-lane engine (csrc/ipm_wide.hip).  Engine-vs-oracle parity rests on
all three taking the same branches (stopping tests, start point, iteration caps, fraction to the boundary; DESIGN.md
§3.2, §5.3), so a constant changed in one place and not the others would show up only as rounding-level drift.  CPU
only: this reads the sources."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "mpcc_oracle.cpp")
IPM = os.path.join(ROOT, "mpcc_manipulator_amd", "csrc", "ipm.hip")
WIDE = os.path.join(ROOT, "mpcc_manipulator_amd", "csrc", "ipm_wide.hip")

NAMES = ("IPM_TOL_MU", "IPM_TOL_P", "IPM_TOL_STEP", "IPM_TOL_FB", "IPM_DIV", "IPM_TAU", "IPM_S0", "IPM_L0",
         "IPM_MAX_IT", "IPM_MAX_IT_SCALED")


def _constants(path):
    """name -> value of the constexpr (or the default of the MPCC_* macro it is set from) in a source file"""
    src = open(path).read()
    macros = {m.group(1): m.group(2) for m in re.finditer(r"#define\s+(MPCC_\w+)\s+([0-9.eE+-]+)", src)}
    out = {}
    for decl in re.finditer(r"constexpr\s+(?:double|int)\s+([^;]+);", src):
        for part in decl.group(1).split(","):
            m = re.match(r"\s*(IPM_\w+)\s*=\s*([\w.+-]+)\s*$", part)
            if not m or m.group(1) in out:  # the first definition: the default build's (debug overrides follow it)
                continue
            v = macros.get(m.group(2), m.group(2))
            try:
                out[m.group(1)] = float(v)
            except ValueError:
                pass
    return out


def test_ipm_constants_agree():
    o, n, w = _constants(ORACLE), _constants(IPM), _constants(WIDE)
    for name in NAMES:
        assert name in o, name
        assert n.get(name) == o[name], (name, n.get(name), o[name])
        assert w.get(name) == o[name], (name, w.get(name), o[name])
    # the round-6 stopping tests: QPs solved to ~2e-10 in u
    assert (o["IPM_TOL_MU"], o["IPM_TOL_STEP"]) == (1e-12, 3e-9)
