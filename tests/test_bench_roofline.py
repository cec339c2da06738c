"""CPU tests of bench.py's roofline block: `bound` is the
resource with the largest MEASURED fraction, never a hard-coded "hbm"; the
kernel's requested bytes are priced against the L2, never against HBM; every
frac is <= 1 for the profiles this repo commits."""
import json
import os

import pytest

from conftest import ROOT

import bench  # noqa: E402  (numpy-only at import)


def test_bound_is_the_measured_limiter():
    pmc = {"hbm_bytes_per_launch": 1.16e8, "valu_insts_per_launch": 1.9e8, "cycles_per_launch": 7.7e5,
           "trace_kernel_avg_us": 320.0}
    r = bench.roofline_of(1.8e9, 0.33, pmc)
    assert r["bound"] == "valu_issue"
    assert r["frac"] == r["issue_frac"] == pytest.approx(1.9e8 / (512 * 7.7e5), abs=1e-4)
    assert r["unit"].startswith("G VALU")
    assert r["l2_frac"] == pytest.approx(1.8e9 / 0.33e-3 / 1e9 / bench.L2_PEAK_GBS, abs=1e-4)
    assert r["hbm_frac"] == pytest.approx(1.16e8 / 0.33e-3 / 1e9 / bench.HBM_PEAK_GBS, abs=1e-4)


def test_hbm_bound_and_l2_without_pmc():
    r = bench.roofline_of(1.0e9, 1.0, {"hbm_bytes_per_launch": 7.0e9, "valu_insts_per_launch": 1e6,
                                       "cycles_per_launch": 1e9})
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert r["frac"] == pytest.approx(7.0 / 8.0, abs=1e-4)
    r = bench.roofline_of(2.0e9, 0.1, None)  # requested bytes far above the HBM peak
    assert r["bound"] == "l2" and r["frac"] == r["l2_frac"] < 1.0
    assert r["traffic"] is None and r["hbm_frac"] is None


def test_committed_profiles_give_fracs_at_most_one():
    """Every PMC entry committed in profiles/pmc_summary.json, priced with its
    own rocprof kernel duration, yields a roofline whose fractions are <= 1."""
    pj = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
    assert pj["entries"]
    for e in pj["entries"]:
        us = e["trace_kernel_avg_us"]
        r = bench.roofline_of(1.8e9, us * 1e-3, e)
        for k in ("frac", "hbm_frac", "l2_frac", "issue_frac"):
            assert r[k] is None or 0.0 <= r[k] <= 1.0, (e["config"], k, r[k])


def test_build_stage_rooflines():
    """Per-stage build roofline: algorithmic bytes from
    the §8(d) share, measured bytes and fractions of 8 TB/s, the limiter."""
    import bench
    pmc = {"build_stages": {"topo_refit": {"us": 80.0, "hbm_bytes": 3.2e8, "algo_bytes_per_prim": 256},
                            "crossing": {"us": 15.0, "hbm_bytes": 2.0e7, "algo_bytes_per_prim": 0},
                            "k0_k1": {"us": 20.0, "hbm_bytes": 8.0e7, "algo_bytes_per_prim": 84}}}
    r = bench.build_stage_rooflines(pmc, 1_000_000)
    assert r["limiter"] == "topo_refit"
    t = r["topo_refit"]
    assert abs(t["frac"] - 256e6 / 80e-6 / 8e12) < 1e-3
    assert abs(t["hbm_frac_measured"] - 3.2e8 / 80e-6 / 8e12) < 1e-3
    assert abs(t["traffic_vs_algo"] - 3.2e8 / 256e6) < 1e-3
    assert r["crossing"]["frac"] is None and r["crossing"]["traffic"] == 2.0e7
    assert bench.build_stage_rooflines(None, 10) is None
