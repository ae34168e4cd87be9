"""bench.py host logic (no GPU): the roofline's traffic comes only from a PMC summary of the same workload."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(d, name, **kw):
    rec = {"kernel": "k_sqp", "batch": 4096, "N": 20, "mask": 2, "dof": 7, "hbm_bytes_per_launch": 1.0}
    rec.update(kw)
    with open(os.path.join(d, name), "w") as f:
        json.dump(rec, f)


def test_find_traffic_matches_workload(tmp_path):
    import bench
    d = str(tmp_path)
    _write(d, "pmc_traffic_k_sqp.json", hbm_bytes_per_launch=8.97e9)
    _write(d, "pmc_traffic_k_sqp_c1all.json", mask=7, hbm_bytes_per_launch=14.7e9)
    _write(d, "pmc_traffic_k_sqp_cfg3.json", batch=32768, N=30, mask=7, dof=10, hbm_bytes_per_launch=7.2e11)
    assert bench.find_traffic("k_sqp", 4096, 20, 2, 7, prof_dir=d) == 8.97e9
    assert bench.find_traffic("k_sqp", 4096, 20, 7, 7, prof_dir=d) == 14.7e9
    assert bench.find_traffic("k_sqp", 32768, 30, 7, 10, prof_dir=d) == 7.2e11
    # another batch, horizon, mask, DOF or kernel has no measured traffic
    assert bench.find_traffic("k_sqp", 65536, 20, 2, 7, prof_dir=d) is None
    assert bench.find_traffic("k_sqp", 4096, 40, 2, 7, prof_dir=d) is None
    assert bench.find_traffic("k_sqp", 32768, 30, 7, 7, prof_dir=d) is None
    assert bench.find_traffic("k_ipm", 4096, 20, 2, 7, prof_dir=d) is None


def test_find_traffic_ignores_unlabelled_summaries(tmp_path):
    import bench
    d = str(tmp_path)
    with open(os.path.join(d, "pmc_traffic_k_sqp.json"), "w") as f:
        json.dump({"kernel": "k_sqp", "batch": 4096, "N": 20, "hbm_bytes_per_launch": 1e10}, f)  # no mask
    assert bench.find_traffic("k_sqp", 4096, 20, 2, 7, prof_dir=d) is None


def test_committed_configs1_summary_is_found():
    import bench
    assert bench.find_traffic("k_sqp", 4096, 20, 2, 7) is not None


def test_union_length_of_launch_intervals():
    """bench.union_length: the time a kernel family ran when several groups' launches overlap."""
    import bench
    assert bench.union_length([], []) == 0.0
    assert bench.union_length([0.0], [2.0]) == 2.0
    assert bench.union_length([0.0, 1.0, 5.0], [2.0, 3.0, 6.0]) == 4.0       # [0,3] + [5,6]
    assert bench.union_length([5.0, 0.0], [6.0, 10.0]) == 10.0               # nested, unsorted
    assert bench.union_length([-1.0, 0.0], [0.5, 0.25]) == 1.5               # times before the anchor


def test_record_io_size_matches_qp_record_layout():
    """The roofline's record-I/O bytes use the QP record size of csrc/dev_common.h (QS, whole 128-byte lines): 336
    doubles for the Panda (its static_assert), 480 for the Husky+Panda."""
    import bench
    assert bench.qs_doubles(7) == 336 and bench.qs_doubles(10) == 480
