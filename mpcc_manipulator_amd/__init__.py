"""mpcc_manipulator_amd — MI355X-native batched MPCC solve engine.

Hot path: the reference's per-control-step SQP solve MPC::runMPC_ (JunHeonYoon/MPCC_manipulator,
cpp/src/MPC/mpc.cpp:104-190) for thousands of independent controllers per launch, as hand-written
HIP kernels for gfx950 behind the C ABI in include/mpcc_engine.h (libmpcc_engine.so).
"""
from .engine import (CON_ENVCOL, CON_SELFCOL, CON_SING, DEFAULT_PARAMS, MOBILE_PARAMS, NN_DIR, REC_SIZE, SOLVED,
                     STATUS_NAMES, Engine, MpccError, MpccParams, build_track_host, cubic_spline_host, dims,
                     eval_track_host, lib, load_default_track, load_params, quat_to_rot, rot_spline_host,
                     track_from_points)
from .mpcc import MPCC, BatchMPCC, load_track_file

__all__ = ["Engine", "MPCC", "BatchMPCC", "MpccParams", "MpccError", "load_params", "load_default_track",
           "load_track_file", "track_from_points", "quat_to_rot", "build_track_host", "eval_track_host",
           "cubic_spline_host", "rot_spline_host", "lib", "STATUS_NAMES",
           "SOLVED", "CON_SELFCOL", "CON_SING", "CON_ENVCOL", "NN_DIR", "DEFAULT_PARAMS", "MOBILE_PARAMS", "REC_SIZE",
           "dims"]
