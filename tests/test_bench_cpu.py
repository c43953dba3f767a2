"""bench.py host logic on the CPU: device selection per rank and the roofline labelling."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pick_device_refuses_stacked_rccl_ranks():
    """Under RCCL each rank needs its own GPU: WORLD_SIZE > visible devices is refused instead of
    stacking ranks with local % device_count."""
    assert bench.pick_device(0, 1, "nccl", 0) == 0
    assert [bench.pick_device(r, 8, "nccl", 8) for r in range(8)] == list(range(8))
    with pytest.raises(SystemExit, match="one rank per GPU"):
        bench.pick_device(1, 2, "nccl", 1)
    with pytest.raises(SystemExit):
        bench.pick_device(0, 8, "nccl", 4)  # rank 0 fits, but the job as a whole does not
    # the gloo rehearsal shares one device
    assert [bench.pick_device(r, 8, "gloo", 1) for r in range(8)] == [0] * 8


def test_setup_dist_refuses_before_touching_gpu(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setattr(bench, "BACKEND", "nccl")

    class A:
        gpus = 2
    with pytest.raises(SystemExit, match="one rank per GPU"):
        bench.setup_dist(A())  # no GPU in this container: 0 devices


def test_rollout_roofline_residency():
    """bound 'hbm' only for a working set beyond the 256 MiB Infinity Cache."""
    small = dict(ev_s=20 * 25e-6, wall=20 * 26e-6, n=65536, k=64, settle_ms=60.0,
                 working_set=38 * 65536 * 64 + 65536 * 40)
    r = bench.rollout_roofline(small, 20, None)
    assert r["bound"] == "issue" and r["resident"] == "infinity-cache"
    assert abs(r["achieved"] - 38 * 65536 * 64 / 25e-6 / 1e9) < 1e-6
    # both clocks carried: frac (= frac_events) from the events, frac_wall from ms_per_step's
    assert r["frac"] == r["frac_events"]
    assert abs(r["frac_wall"] - 38 * 65536 * 64 / 26e-6 / 1e9 / 8000.0) < 1e-9
    big = dict(small, working_set=8 * 38 * 65536 * 64)
    assert bench.rollout_roofline(big, 20, None)["bound"] == "hbm"
    rec = {"hbm_bytes_per_launch": 2.0e8, "source": "profiles/r04/pmc.json (box)"}
    t = bench.rollout_roofline(big, 20, rec)
    assert t["traffic"] == 2.0e8 and "profiles/r04/pmc.json" in t["traffic_source"]


def test_pmc_summary_steps_per_launch():
    """Issue counters are normalised per env step: K of the rollout key, with or without the
    ring-launches suffix (round 4 parsed every key as K = 1)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_summary
    assert pmc_summary.steps_of("k_rollout@65536x64") == 64
    assert pmc_summary.steps_of("k_rollout@65536x64r8") == 64
    assert pmc_summary.steps_of("k_rollout_ws@4194304x16") == 16
    assert pmc_summary.steps_of("k_step@65536") == 1
    assert pmc_summary.steps_of("k_rollout@65536x0") == 1
