"""Guard of the round-2 memory fault's cause: the fused kernels once copied the whole by-value
DevConst into every lane's private segment (a reference to a by-value kernel parameter) and read it back through
reloaded generic pointers.  The fix names the arguments in place (kernels.h kernarg_const).  This test reads the
gfx950 kernel descriptors of both engine libraries (the AMDGPU metadata note of each code object in the offload
bundle) and fails if any kernel's per-lane private segment could hold such a copy, or if the interior-point kernels'
frames grow past their post-fix sizes.  CPU only: it inspects the built code objects."""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
# sizeof(DevConst) at this revision: the kernel-argument segment of k_ipm<9> (DevConst + DevBuffers, then the 256
# bytes of HIP's hidden arguments) minus DevBuffers (30 pointers and the low-rank stride, 248 bytes).  Any private
# segment this large could hold a copy.
DEVCONST_BYTES = 3288
DEVBUFFERS_BYTES = 248
PANDA_NARROW_MAX = 1740   # 1.7 KB: k_sqp / k_ipm of ipm.hip (16-lane interior point, tail mode included)
WIDE_MAX = 2400           # 2.3 KB: the 32-lane kernels of ipm_wide.hip (mobile build, damped BFGS incl. the extended low-rank path)


def _descriptors(lib, tmp):
    work = os.path.join(tmp, os.path.basename(lib) + ".d")
    os.makedirs(work, exist_ok=True)
    local = os.path.join(work, os.path.basename(lib))
    shutil.copy(lib, local)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=work, check=True,
                   capture_output=True)
    out = {}
    for f in sorted(os.listdir(work)):
        if not f.endswith("gfx950"):
            continue
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(work, f)], check=True,
                               capture_output=True, text=True).stdout
        # one YAML map per kernel ("  - .agpr_count: ..."); keys are sorted, so .group_segment_fixed_size and
        # .kernarg_segment_size come before .name: collect the map, then file it under its name
        cur = {}
        for line in notes.splitlines():
            if line.startswith("  - ."):  # a kernel's map (its .args entries are indented further)
                cur = {}
            m = re.match(r"(?:  - |    )\.(\w+):\s+(\S+)", line)
            if not m:
                continue
            if m.group(1) == "name":
                out[m.group(2)] = cur
            elif m.group(1) in ("private_segment_fixed_size", "kernarg_segment_size", "group_segment_fixed_size",
                                "vgpr_count"):
                cur[m.group(1)] = int(m.group(2))
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-readelf")), reason="ROCm LLVM tools not installed")
def test_no_private_devconst_copy(built_lib, tmp_path):
    from mpcc_manipulator_amd import engine
    libs = {7: engine.LIB_PATHS[7], 10: engine.LIB_PATHS[10]}
    seen = {"narrow": 0, "wide": 0}
    for dof, lib in libs.items():
        d = _descriptors(lib, str(tmp_path))
        kern = {k: v for k, v in d.items() if k.startswith(("_ZN4mpcc", "_ZN8mpcc_m10"))}
        assert kern, f"no kernel descriptors found in {lib}"
        for name, v in kern.items():
            priv = v.get("private_segment_fixed_size", 0)
            assert priv < DEVCONST_BYTES, f"{name}: {priv}-byte private segment could hold a DevConst copy"
            if re.search(r"\d+k_(sqp|sqp_solo|ipm)I", name):  # k_sqp, k_sqp_solo, k_ipm (mangled: <len>k_...I<args>)
                # ipm_wide.hip's kernels carry a bool template argument (ILb0/ILb1 after the row count)
                wide = dof == 10 or re.search(r"ILi\d+ELb[01]E", name) is not None
                lim = WIDE_MAX if wide else PANDA_NARROW_MAX
                seen["wide" if wide else "narrow"] += 1
                assert priv <= lim, f"{name}: private segment {priv} > {lim} bytes (DESIGN.md §3.4)"
        # the DevConst size the bound is derived from
        if dof == 7:
            ka = [v["kernarg_segment_size"] for k, v in kern.items() if k.startswith("_ZN4mpcc5k_ipmILi9E")]
            assert ka and ka[0] - DEVBUFFERS_BYTES - 256 == DEVCONST_BYTES
            # the self-collision MLP at two waves per SIMD; the two-wave env blocks two per CU
            # beside the interior point's waves
            selfk = [v for k, v in kern.items() if k.startswith("_ZN4mpcc10k_mlp_self")]
            assert selfk and selfk[0]["vgpr_count"] <= 256
            env2 = [v for k, v in kern.items() if k.startswith("_ZN4mpcc9k_mlp_envILi2E")]
            assert env2 and env2[0]["group_segment_fixed_size"] <= 80 * 1024
            # k_records at four waves per SIMD: the record is stored before the Gram matrix of the manipulability
            # (holding pos, R and J through it took 194 registers)
            recs = [v for k, v in kern.items() if k.startswith("_ZN4mpcc9k_records")]
            assert recs and recs[0]["vgpr_count"] <= 128
    assert seen["narrow"] >= 12 and seen["wide"] >= 8
