"""bench.py's roofline fields (CPU): SURVEY.md 8(d)'s literal bytes, the
Infinity-Cache-resident share and the counter-based bound label."""
import numpy as np

import bench


def test_literal_bytes_exact_and_qg():
    # counters [q, 8]: c[0] distances, c[4] edges (exact) / code blocks (qg), c[3] exact distances (qg)
    c = np.zeros((3, 8))
    c[:, 0] = [100, 200, 300]
    c[:, 4] = [10, 20, 30]
    c[:, 3] = [5, 5, 5]
    dp, nq, k = 128, 3, 10
    assert bench.literal_bytes(c, dp, nq, k, False, 128) == 600 * dp * 4 + 60 * 4 + nq * (dp * 4 + k * 8)
    # NGTQG: blocks * 8 * Me + ADC distances * 4 + exact rows * Dp * 4 + per query Dp * 4 + k * 8
    assert bench.literal_bytes(c, dp, nq, k, True, 128) == 60 * 8 * 128 + 600 * 4 + 15 * dp * 4 + nq * (dp * 4 + k * 8)


def test_ic_share():
    assert bench.ic_share(None, 100.0) == 0.0
    assert bench.ic_share({"filter_copy_fits_infinity_cache": False, "filter_copy_bytes": 50.0}, 100.0) == 0.0
    assert bench.ic_share({"filter_copy_fits_infinity_cache": True, "filter_copy_bytes": 88.0}, 100.0) == 0.88


def test_bound_from_counters():
    w = 1000.0
    assert bench.bound_from_counters({"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 560, "SQ_ACTIVE_INST_VALU": 100}) == "latency"
    assert bench.bound_from_counters({"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 300, "SQ_ACTIVE_INST_VALU": 600}) == "valu"
    assert bench.bound_from_counters({"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 300, "SQ_ACTIVE_INST_VALU": 100}) == "hbm"
    # most algorithmic bytes from an Infinity-Cache-resident table (the C2 filter copy)
    assert bench.bound_from_counters({"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 495, "SQ_ACTIVE_INST_VALU": 100},
                                     0.90) == "infinity-cache"
    assert bench.bound_from_counters({"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 560, "SQ_ACTIVE_INST_VALU": 100},
                                     0.90) == "latency"


def test_run_reaped_terminates_leftovers(tmp_path):
    """A child's own leftovers (here a background sleep it does not wait for)
    are terminated with its process group once it exits."""
    import time
    pidfile = tmp_path / "pid"
    rc, out, _ = bench.run_reaped(["bash", "-c", "sleep 60 & echo $! > %s; echo done" % pidfile], 30,
                                  capture_stderr=True, what="test child")
    assert rc == 0 and out.strip() == "done"
    pid = int(pidfile.read_text())
    for _ in range(50):
        try:
            with open("/proc/%d/stat" % pid) as f:
                state = f.read().rsplit(")", 1)[1].split()[0]
        except OSError:
            break
        if state == "Z":
            break
        time.sleep(0.1)
    else:
        raise AssertionError("the leftover sleep survived its group")


def test_bound_issue_from_clocked_pass():
    """A SIMD issuing in >= 0.7 of its measured cycles is issue-bound even when
    its waves wait on memory most of the time (the other waves fill in)."""
    w = 1000.0
    cn = {"SQ_WAVE_CYCLES": w, "SQ_WAIT_ANY": 650, "SQ_ACTIVE_INST_VALU": 150}
    assert bench.bound_from_counters(cn, 0.0, {"simd_issue_util": 0.78}) == "issue"
    assert bench.bound_from_counters(cn, 0.0, {"simd_issue_util": 0.58}) == "latency"
    assert bench.bound_from_counters(cn, 0.0, None) == "latency"


def test_pick_expansion():
    sw = [{"result_expansion": 2.0, "epsilon": 0.106, "recall_at_10": 0.955, "kernel_ms": 85.0},
          {"result_expansion": 3.0, "epsilon": 0.098, "recall_at_10": 0.955, "kernel_ms": 77.5},
          {"result_expansion": 4.0, "epsilon": 0.093, "recall_at_10": 0.957, "kernel_ms": 79.2},
          {"result_expansion": 6.0, "epsilon": 0.085, "recall_at_10": 0.955, "kernel_ms": 76.5}]
    # 3.0 is within 3 % of the fastest (6.0): the tie goes to the default
    assert bench.pick_expansion(sw, 0.95)["result_expansion"] == 3.0
    # a clear winner is taken
    sw[3]["kernel_ms"] = 60.0
    assert bench.pick_expansion(sw, 0.95)["result_expansion"] == 6.0
    # one below the target is skipped while another reaches it
    sw[3]["recall_at_10"] = 0.94
    assert bench.pick_expansion(sw, 0.95)["result_expansion"] == 3.0


def test_traffic_entries_carry_clocked_passes():
    """The four timed lines' traffic.json entries (the ones bench.py attaches
    to C2, ANNG, qg and C3) hold both clocked counter passes: the SIMD issue
    figures and the texture address units' busy share, each a fraction of
    the GRBM-measured cycles."""
    import json
    import os
    t = json.load(open(os.path.join(os.path.dirname(bench.__file__), "profiles", "traffic.json")))
    clocked = [e for e in t["entries"] if "simd_issue" in e]
    assert len(clocked) == 4
    for e in clocked:
        ta = e["texture_address"]
        assert 0.0 < ta["ta_busy_frac"] < 1.0 and 0.0 < ta["vmem_per_cu_cycle"] < 1.0
        assert 0.0 < e["simd_issue"]["simd_valu_util"] <= e["simd_issue"]["simd_issue_util"]
