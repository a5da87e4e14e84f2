"""bench.py's roofline traffic: the PMC bytes per launch of the timed k_wf_step instances
(COUNT=false), weighted by their dispatch counts (scripts/summarize_traffic.py).  Kernel names of
round 3's profiles carry a sixth template argument (the removed entry cull: CULL=true instances
are not timed)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _write(tmp_path, entries):
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "traffic.json").write_text(json.dumps({"64x64x4x8x1": entries}))


def test_weighted_by_dispatches(tmp_path, monkeypatch):
    _write(tmp_path, {
        "k_wf_step_bf<true, true, true, false, false, false>": {"hbm_bytes_per_launch": 200.0, "dispatches": 8},
        "k_wf_step_bf<false, true, true, false, false, false>": {"hbm_bytes_per_launch": 100.0, "dispatches": 9},
        "k_wf_step_bf<true, true, true, false, false, true>": {"hbm_bytes_per_launch": 1000.0, "dispatches": 1},
        "k_wf_step_bf<true, true, true, true, false, false>": {"hbm_bytes_per_launch": 9e9, "dispatches": 8},   # COUNT
        "k_wf_step_bf<true, true, true, false, true, false>": {"hbm_bytes_per_launch": 9e9, "dispatches": 1},   # CULL
        "k_wf_accum": {"hbm_bytes_per_launch": 9e9, "dispatches": 1},
    })
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got, src = bench.load_traffic(("k_wf_step_bf<",), 64, 64, 4, 8, 1)
    assert got == (200.0 * 8 + 100.0 * 9 + 1000.0) / 18
    assert src.startswith("profiles/traffic.json[64x64x4x8x1]")


def test_weighted_five_argument_names(tmp_path, monkeypatch):
    """k_wf_step_bf<EXT, LDS, rcp, COUNT, GEN> (round 4): the GEN launch is timed, COUNT is not."""
    _write(tmp_path, {
        "k_wf_step_bf<true, true, true, false, false>": {"hbm_bytes_per_launch": 200.0, "dispatches": 8},
        "k_wf_step_bf<false, true, true, false, false>": {"hbm_bytes_per_launch": 100.0, "dispatches": 9},
        "k_wf_step_bf<true, true, true, false, true>": {"hbm_bytes_per_launch": 1000.0, "dispatches": 1},
        "k_wf_step_bf<true, true, true, true, false>": {"hbm_bytes_per_launch": 9e9, "dispatches": 8},
    })
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got, _ = bench.load_traffic(("k_wf_step_bf<",), 64, 64, 4, 8, 1)
    assert got == (200.0 * 8 + 100.0 * 9 + 1000.0) / 18


def test_unweighted_without_counts(tmp_path, monkeypatch):
    _write(tmp_path, {
        "k_wf_step_bf<true, true, true, false, false>": {"hbm_bytes_per_launch": 200.0},
        "k_wf_step_bf<false, true, true, false, false>": {"hbm_bytes_per_launch": 100.0},
        "k_wf_step_bf<true, true, true, false, true>": {"hbm_bytes_per_launch": 9e9},
        "k_wf_step_bf<true, true, true, true, false>": {"hbm_bytes_per_launch": 9e9},
        "k_wf_trace<true, 17, false>": {"hbm_bytes_per_launch": 7.0},
        "k_wf_trace<true, 17, true>": {"hbm_bytes_per_launch": 9e9},
    })
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.load_traffic("k_wf_step_bf<", 64, 64, 4, 8, 1)[0] == 150.0
    assert bench.load_traffic("k_wf_trace", 64, 64, 4, 8, 1)[0] == 7.0
    assert bench.load_traffic("k_wf_trace", 32, 32, 4, 8, 1) is None


def test_valu_field_and_metric_name(tmp_path, monkeypatch):
    _write(tmp_path, {
        "k_wf_step_bf<true, true, true, false, false, false>": {"hbm_bytes_per_launch": 1.0, "valu_issue": 0.7,
                                                               "dispatches": 3},
        "k_wf_step_bf<false, true, true, false, false, false>": {"hbm_bytes_per_launch": 1.0, "valu_issue": 0.5,
                                                                "dispatches": 1},
        "k_wf_step_bf<false, true, true, true, false, false>": {"hbm_bytes_per_launch": 1.0, "valu_issue": 0.1,
                                                               "dispatches": 9},
    })
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    v, _ = bench.load_traffic("k_wf_step_bf<", 64, 64, 4, 8, 1, field="valu_issue")
    assert abs(v - (0.7 * 3 + 0.5) / 4) < 1e-12
    assert bench.metric_name("CornellBox-Glossy", 1024, 1024, 16) == "Msamples/s (paths/s) CornellBox-Glossy 1024x1024 depth 16"
