"""bench.py's roofline traffic: the PMC bytes per launch of the timed k_wf_step instances
(COUNT=false), weighted by their dispatch counts (scripts/summarize_traffic.py).  Kernel names of
round 3's profiles carry a sixth template argument (the removed entry cull: CULL=true instances
are not timed)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _write(tmp_path, entries, key="CornellBox|reference|64x64x4x8x1"):
    (tmp_path / "profiles").mkdir(exist_ok=True)
    (tmp_path / "profiles" / "traffic.json").write_text(json.dumps({key: entries}))


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
    got, src = bench.load_traffic(("k_wf_step_bf<",), "CornellBox", "reference", 64, 64, 4, 8, 1)
    assert got == (200.0 * 8 + 100.0 * 9 + 1000.0) / 18
    assert src.startswith("profiles/traffic.json[64x64x4x8x1]")
    # another scene or tree at the same size, spp and depth does not get this scene's PMC
    assert bench.load_traffic(("k_wf_step_bf<",), "CornellBox-Mirror", "reference", 64, 64, 4, 8, 1) is None
    assert bench.load_traffic(("k_wf_step_bf<",), "CornellBox", "sah", 64, 64, 4, 8, 1) is None


def test_weighted_five_argument_names(tmp_path, monkeypatch):
    """k_wf_step_bf<EXT, LDS, rcp, COUNT, GEN> (round 4): the GEN launch is timed, COUNT is not."""
    _write(tmp_path, {
        "k_wf_step_bf<true, true, true, false, false>": {"hbm_bytes_per_launch": 200.0, "dispatches": 8},
        "k_wf_step_bf<false, true, true, false, false>": {"hbm_bytes_per_launch": 100.0, "dispatches": 9},
        "k_wf_step_bf<true, true, true, false, true>": {"hbm_bytes_per_launch": 1000.0, "dispatches": 1},
        "k_wf_step_bf<true, true, true, true, false>": {"hbm_bytes_per_launch": 9e9, "dispatches": 8},
    })
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got, _ = bench.load_traffic(("k_wf_step_bf<",), "CornellBox", "reference", 64, 64, 4, 8, 1)
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
    assert bench.load_traffic("k_wf_step_bf<", "CornellBox", "reference", 64, 64, 4, 8, 1)[0] == 150.0
    assert bench.load_traffic("k_wf_trace", "CornellBox", "reference", 64, 64, 4, 8, 1)[0] == 7.0
    assert bench.load_traffic("k_wf_trace", "CornellBox", "reference", 32, 32, 4, 8, 1) is None


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
    v, _ = bench.load_traffic("k_wf_step_bf<", "CornellBox", "reference", 64, 64, 4, 8, 1, field="valu_issue")
    assert abs(v - (0.7 * 3 + 0.5) / 4) < 1e-12
    assert bench.metric_name("CornellBox-Glossy", 1024, 1024, 16) == "Msamples/s (paths/s) CornellBox-Glossy 1024x1024 depth 16"


def test_plain_key_only_for_the_scene_it_names(tmp_path, monkeypatch):
    """Entries written before the qualified keys (round 5): used only for the scene their source names,
    on the reference tree."""
    _write(tmp_path, {"_source": "rocprofv3 ... (CornellBox.xml 64x64 4spp depth 8, rr 0.9)",
                      "k_wf_step_bf<true, true, true, false, false>": {"hbm_bytes_per_launch": 5.0, "dispatches": 1}},
           key="64x64x4x8x1")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.load_traffic("k_wf_step_bf<", "CornellBox", "reference", 64, 64, 4, 8, 1)[0] == 5.0
    assert bench.load_traffic("k_wf_step_bf<", "CornellBox-Glossy", "reference", 64, 64, 4, 8, 1) is None
    assert bench.load_traffic("k_wf_step_bf<", "CornellBox", "sah", 64, 64, 4, 8, 1) is None


def test_valu_exec_per_kernel_family(tmp_path, monkeypatch):
    """roofline.valu_exec: timed instances only (the counted render's are left out), summed per kernel
    family with their dispatches, density x lane use per family, the step weighted by the families'
    warm-up times; shade instances map to k_wf_shade_ext / _shadow as the bench names them."""
    def v(act, thr, grbm):
        return {"valu_counters": {"SQ_ACTIVE_INST_VALU": act, "SQ_THREAD_CYCLES_VALU": thr, "GRBM_GUI_ACTIVE": grbm},
                "dispatches": 1}
    _write(tmp_path, {
        "k_wf_trace_pre<false, 277, false, 128u, 4>": v(128.0, 64.0 * 128.0 * 0.5, 4.0),  # density k*128/(128*4)
        "k_wf_trace_pre<false, 277, true, 128u, 4>": v(1e9, 1e9, 1.0),                   # COUNT: left out
        "k_wf_leafpass<true>": v(64.0, 64.0 * 64.0, 4.0),
        "k_wf_shade<true, false>": v(32.0, 64.0 * 32.0 * 0.25, 4.0),
        "k_wf_shade<true, true>": v(1e9, 1e9, 1.0),                                       # COUNT: left out
    }, key="MedievalBoat|reference|64x64x4x16x1")
    (tmp_path / "profiles" / "valu_calibration.json").write_text(json.dumps({"k_active": 4.0}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got = bench.load_valu_exec("MedievalBoat", "reference", 64, 64, 4, 16, 1,
                               {"k_wf_trace": 1.0, "k_wf_leafpass": 1.0, "k_wf_shade_ext": 2.0})
    k = got["kernels"]
    assert abs(k["k_wf_trace"]["issue_density"] - 1.0) < 1e-12 and abs(k["k_wf_trace"]["frac"] - 0.5) < 1e-12
    assert abs(k["k_wf_leafpass"]["frac"] - 0.5) < 1e-12
    assert abs(k["k_wf_shade_ext"]["frac"] - 0.0625) < 1e-12
    assert abs(got["frac"] - (0.5 + 0.5 + 2 * 0.0625) / 4) < 1e-3  # (rounded to 4 places)
    assert bench.load_valu_exec("MedievalBoat", "sah", 64, 64, 4, 16, 1, {"k_wf_trace": 1.0}) is None
