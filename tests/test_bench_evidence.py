"""bench.py's roofline block and the committed PMC records it reads
(profiles/r02/pmc_*.json).  Host logic only: no GPU.

The measured candidates (hbm, valu) are used only when the PMC record was
taken on the same library build (build_id); otherwise the block falls back
to the L2 record-byte bound and reports traffic null."""
import json
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


COUNTS = {"node_tests": 10_000_000, "triangle_tests": 2_000_000}
WAVES = {"node_steps": 800_000, "triangle_steps": 180_000}
NPX = 1920 * 1080


def pmc_record(build_id):
    return {"build_id": build_id, "hbm_bytes_per_launch": 50_000_000,
            "valu_insts_per_launch": 60_000_000, "salu_insts_per_launch": 9_000_000}


def test_fresh_pmc_adds_measured_candidates():
    r = bench.roofline_block(0.1, COUNTS, WAVES, NPX, pmc_record("abc"), "abc", 1.0)
    assert r["traffic"] == 50_000_000
    # 60M wave-instructions in 0.1 ms = 600 Ginst/s against the VALU issue peak
    assert r["bound"] == "valu_issue"
    assert r["achieved"] == pytest.approx(600.0)
    assert r["frac"] == pytest.approx(600.0 / bench.VALU_PEAK_GINST, rel=1e-4)


def test_stale_pmc_is_ignored():
    r = bench.roofline_block(0.1, COUNTS, WAVES, NPX, pmc_record("old"), "new", 1.0)
    assert r["traffic"] is None
    assert r["bound"] == "l2"
    uniq = bench.PNODE_BYTES * WAVES["node_steps"] + bench.SLOT_BYTES * WAVES["triangle_steps"] \
        + bench.PIXEL_BYTES * NPX
    assert r["achieved"] == pytest.approx(uniq / 1e-4 / 1e9, rel=1e-4)


def test_shard_fraction_scales_per_launch_figures():
    full = bench.roofline_block(0.1, COUNTS, WAVES, NPX, pmc_record("a"), "a", 1.0)
    half = bench.roofline_block(0.05, COUNTS, WAVES, NPX, pmc_record("a"), "a", 0.5)
    assert half["traffic"] == full["traffic"] // 2
    assert half["frac"] == pytest.approx(full["frac"], rel=1e-3)


def test_no_pmc_and_no_wave_steps_is_unmeasured():
    """GI / wavefront walks count no wave steps: without a PMC record of the
    benched build no bound can be named."""
    r = bench.roofline_block(0.1, COUNTS, {}, NPX, None, "a", 1.0)
    assert r["bound"] is None and r["frac"] is None and r["measured"] is False
    assert r["s8d_work_rate"]["bytes_per_launch"] > 0
    r = bench.roofline_block(0.1, COUNTS, {}, NPX, pmc_record("a"), "a", 1.0)
    assert r["bound"] in ("valu_issue", "hbm") and r["measured"] is True


def test_no_pmc_falls_back_to_l2():
    r = bench.roofline_block(0.1, COUNTS, WAVES, NPX, None, "a", 1.0)
    assert r["bound"] == "l2" and r["traffic"] is None


@pytest.mark.parametrize("config,size", [("c2", (1920, 1080)), ("c5", (3840, 2160))])
def test_committed_pmc_records_are_well_formed(config, size):
    path = ROOT / "profiles" / "r02" / f"pmc_{config}.json"
    d = json.loads(path.read_text())
    assert d["config"] == config and tuple(d["size"]) == size
    assert len(d["build_id"]) == 16
    assert d["hbm_bytes_per_launch"] > 0 and d["valu_insts_per_launch"] > 0
    loaded = bench.load_pmc(str(path), config, *size)
    assert loaded is not None and loaded["build_id"] == d["build_id"]
    # a record for another frame size is not applied
    assert bench.load_pmc(str(path), config, 64, 64) is None
