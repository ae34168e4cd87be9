"""In-tree build of libmpcc_engine.so (hipcc, gfx950).  Used by __graft_entry__.build() and tests.

The shared library is written to mpcc_manipulator_amd/_build/ (git-ignored; travels to the GPU box
with the repository snapshot)."""
import concurrent.futures as cf
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
PROF = os.environ.get("MPCC_PROF_BUILD", "0") == "1"  # cycle-accounting variant (tools/ipm_prof.py)
# bounds-checked variant: every computed workspace / record / ring / LDS / spline index is tested and clamped,
# violations are recorded per lane (dev_common.h MPCC_BCHK, mpcc_debug_bounds); tests load it through
# MPCC_ENGINE_LIB / MPCC_ENGINE_LIB_MOBILE (tools/bounds_check.sh)
BCHK = os.environ.get("MPCC_BOUNDS_CHECK", "0") == "1"
BUILD = os.path.join(PKG, "_build_prof" if PROF else ("_build_bchk" if BCHK else "_build"))
LIB = os.path.join(BUILD, "libmpcc_engine.so")
SOURCES = ["kernels.hip", "ipm.hip", "ipm_wide.hip", "mlp.hip", "nn_generic.hip", "engine.cpp", "host_params.cpp",
           "host_spline.cpp", "mpc.cpp"]
# The Husky+Panda mobile manipulator (BASELINE configs[3]): the same sources built with the
# robot's compile-time dimensions (as the reference's config.h NX/NU), its own 32-lane interior point and
# namespace, into a second library with the same C ABI.
MOBILE_LIB = os.path.join(BUILD, "libmpcc_engine_mobile.so")
MOBILE_SOURCES = ["kernels.hip", "ipm_wide.hip", "mlp.hip", "nn_generic.hip", "engine.cpp", "host_params.cpp",
                  "host_spline.cpp"]
MOBILE_FLAGS = ["-DMPCC_DOF=10", "-Dmpcc=mpcc_m10"]
ARCH = os.environ.get("MPCC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# The stage kernels (projection, kinematics, records, QP assembly, line-search trials) follow the
# oracle's operation order without FMA contraction, so their discrete decisions (projection Newton,
# warm-start validity, filter comparisons) see the same values as the reference CPU arithmetic.
FILE_FLAGS = {"kernels.hip": ["-ffp-contract=off"], "mlp.hip": ["-ffp-contract=off"], "nn_generic.hip": ["-ffp-contract=off"]}


def source_hash():
    """Build provenance: sha256 (first 16 hex digits) over the product sources and headers (csrc/, include/),
    file names and contents in sorted order.  Compiled into the libraries as mpcc_build_id(); the tests check
    that the library they load was built from the tree they run in (tests/conftest.py built_lib)."""
    import hashlib
    h = hashlib.sha256()
    for d in (CSRC, os.path.join(ROOT, "include")):
        for f in sorted(os.listdir(d)):
            p = os.path.join(d, f)
            if os.path.isfile(p) and f.endswith((".h", ".hpp", ".hip", ".cpp")):
                h.update(f.encode() + b"\0")
                with open(p, "rb") as fh:
                    h.update(fh.read())
                h.update(b"\0")
    return h.hexdigest()[:16]


BUILD_ID = source_hash()
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
          "-I", CSRC, "-Wno-unused-result"] + (["-DMPCC_IPM_PROF"] if PROF else []) + \
         (["-DMPCC_BOUNDS_CHECK"] if BCHK else [])


def _compile(src, variant=""):
    path = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + variant + ".o")
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    inc = os.path.join(ROOT, "include")
    deps += [os.path.join(inc, h) for h in os.listdir(inc)]
    idf = []
    if src == "engine.cpp":  # carries mpcc_build_id(): rebuilt whenever any product source changes
        deps += [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
        idf = [f'-DMPCC_BUILD_ID="{BUILD_ID}"']
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    lang = ["-x", "hip"] if src.endswith(".cpp") else []
    extra = MOBILE_FLAGS if variant == "_mobile" else []
    cmd = [HIPCC] + CFLAGS + extra + idf + lang + FILE_FLAGS.get(src, []) + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def _link(lib, objs, verbose):
    if not (os.path.exists(lib) and os.path.getmtime(lib) >= max(os.path.getmtime(o) for o in objs)):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("built", lib)


def build(verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    jobs = [(s, "") for s in SOURCES] + ([] if PROF else [(s, "_mobile") for s in MOBILE_SOURCES])
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(lambda j: _compile(*j), jobs))
    _link(LIB, objs[:len(SOURCES)], verbose)
    if not PROF:
        _link(MOBILE_LIB, objs[len(SOURCES):], verbose)
    build_examples(verbose)
    build_python_module(verbose)
    return LIB


def build_python_module(verbose=False):
    """MPCC_WRAPPER (csrc/wrapper_py.cpp, pybind11): the reference's Python module names over the
    engine, written next to libmpcc_engine.so (rpath $ORIGIN)."""
    import sysconfig
    import pybind11
    src = os.path.join(CSRC, "wrapper_py.cpp")
    out = os.path.join(BUILD, "MPCC_WRAPPER" + sysconfig.get_config_var("EXT_SUFFIX"))
    deps = [src, LIB] + [os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))]
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-I", os.path.join(ROOT, "include"),
           "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], src, "-o", out,
           "-L", BUILD, "-lmpcc_engine", "-Wl,-rpath,$ORIGIN", "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"MPCC_WRAPPER build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", out)
    return out


EXAMPLES = os.path.join(ROOT, "examples")


def build_examples(verbose=False):
    """C++ programs on the host surface (include/mpcc_mpc.hpp), linked against the engine with g++."""
    out = []
    for src in sorted(os.listdir(EXAMPLES)) if os.path.isdir(EXAMPLES) else []:
        if not src.endswith(".cpp"):
            continue
        exe = os.path.join(BUILD, os.path.splitext(src)[0])
        path = os.path.join(EXAMPLES, src)
        deps = [path, LIB] + [os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))]
        if not (os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(d) for d in deps)):
            cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), path, "-o", exe,
                   "-L", BUILD, "-lmpcc_engine", "-Wl,-rpath,$ORIGIN"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"example build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            if verbose:
                print("built", exe)
        out.append(exe)
    return out


if __name__ == "__main__":
    build(verbose=True)
