"""bench.py's roofline pieces that need no GPU: the committed PMC summary of
the current sources is found by its source hash, and the extension's issue
roofline is priced against the row kernel's own time."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_pmc_profile_matches_sources():
    """A PMC summary stamped with these sources' hash is committed, so the
    round-end bench line carries measured traffic (null otherwise)."""
    prof = bench.pmc_profile("C3", 1)
    if prof is None:   # sources changed since the last profile: the bench line says so
        pytest.skip(f"no profiles/*/C3_pmc.json with src_hash {bench.src_hash()}")
    assert prof["traffic_bytes_seed_extend"] > 0
    assert bench.pmc_profile("C3", 2) is None   # per-rank shares are not profiled


def test_issue_roofline_uses_the_row_kernel_time():
    iss = {"valu": 65.4e9, "salu": 37.1e9, "valu_peak_g_per_s": 1228.8, "valu_per_wave_step": 142.7,
           "kernel": "extend_rows_kernel", "kernel_ms": 84.5, "kernel_ms_source": "stats.csv"}
    r = bench.issue_roofline(iss, 92.0)
    assert r["kernel_ms"] == 84.5 and r["kernel_ms_source"] == "stats.csv"
    assert abs(r["achieved"] - 65.4e9 / 84.5e-3 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / 1228.8) < 1e-3
    # without the kernel's own time: the live extension time, named as such
    del iss["kernel_ms"]
    r = bench.issue_roofline(iss, 92.0)
    assert r["kernel_ms"] == 92.0 and "live" in r["kernel_ms_source"]


def test_committed_summary_has_the_row_kernel_time():
    prof = bench.pmc_profile("C3", 1)
    if prof is None:
        pytest.skip(f"no profiles/*/C3_pmc.json with src_hash {bench.src_hash()}")
    iss = prof.get("issue") or {}
    assert iss.get("kernel") == "extend_rows_kernel" and iss.get("kernel_ms", 0) > 0
    stats = os.path.join(ROOT, iss["kernel_ms_source"])
    assert os.path.exists(stats)
    json.dumps(bench.issue_roofline(iss, 92.0))
