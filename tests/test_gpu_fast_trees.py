"""GPU vs oracle, bit for bit, on the trees the perf story leans on beyond the reference scenes:

* the fast SAH tree (pt_bvh_build_sah; SURVEY.md §8(f) row 2, src/ts-util/bvh.ts:25-187 is the
  reference's builder it replaces) on CornellBox-Glossy 1024^2 (depth 16, 8 frames) and
  MedievalBoat 1920x1080 (depth 16, 4 frames);
* the Cornell-sized synthetic scenes of the BVH sweep (scripts/synth_scene.py, seed 1234,
  BASELINE.json north_star) on the reference's tree: 1,000 and 12,500 triangles (1024^2,
  depth 8, 8 frames, three bands), 100,000 (one band, 8 frames; with and without the traversal
  kernel's pooled leaf turns) and 1,000,000 (one band, 2 frames: the reference builder's
  depth cap of 16 keeps even this tree at <= 32,767 internal nodes), plus 12,500 on the SAH tree.
The bands are rows that see light (the light at rows ~190-210; the random triangles shade the
rest of the box more and more as N grows).

The product renders the WHOLE image through AUTO at the default batch target and at 8 M-path
batches (identical bits), and 16-row bands of it are compared with the C oracle
(oracle/pt_oracle.c: the literal restatement of src/wgsl-util/intersection-logic.wgsl:1-215)
rendering the same rows of the same packed buffers.  These trees run k_wf_trace's code paths that
the reference scenes do not reach: deep stacks, leaf sizes of the SAH builder (<= 8), the
synthetic reference trees' many mid-size leaves (1M: ~30+ entries per leaf).
"""
import os
import sys

import pytest

import pt_amd
from conftest import ROOT, SCENES, pack_with_node
from test_gpu_bench_config import assert_same_bits
from test_gpu_config_bands import _render_bands

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import synth_scene  # noqa: E402

pytestmark = pytest.mark.gpu

SYNTH_BANDS = [(192, 208), (320, 336), (504, 520)]  # the light, the upper box, the centre


@pytest.fixture(scope="module")
def sah_packed(tmp_path_factory):
    base = tmp_path_factory.mktemp("sah")
    out = {}
    for s in ("CornellBox-Glossy", "MedievalBoat"):
        out[s] = pack_with_node(os.path.join(SCENES, "scene_assets", s + ".xml"), str(base / s), "--bvh", "sah",
                                "--native-bvh")
    return out


@pytest.fixture(scope="module")
def synth_packed(tmp_path_factory):
    cache = {}

    def get(n, bvh="reference", light_grid=1):
        if (n, bvh, light_grid) not in cache:
            root = tmp_path_factory.mktemp(f"synth{n}")
            xml = synth_scene.write(n, str(root), light_grid)
            cache[(n, bvh, light_grid)] = pack_with_node(xml, str(root / "packed"), "--native-bvh", "--bvh", bvh)
        return cache[(n, bvh, light_grid)]
    return get


def _trace_kernel_ran(profs):
    assert all("k_wf_trace" in p for p in profs), profs


def test_sah_glossy_1024_depth16_rows_bitexact(sah_packed):
    _, profs = _render_bands(sah_packed["CornellBox-Glossy"], 1024, 1024, 8, 16, [(260, 276), (500, 516), (900, 916)])
    _trace_kernel_ran(profs)


def test_sah_boat_1080p_depth16_rows_bitexact(sah_packed):
    p = sah_packed["MedievalBoat"]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        assert s.info["max_leaf"] <= 8  # no big leaves on the SAH tree: lean16 turns, leaf entries pooled in runs of 2
    _, profs = _render_bands(p, 1920, 1080, 4, 16, [(680, 696), (560, 576)])
    _trace_kernel_ran(profs)


@pytest.mark.parametrize("n", [1000, 12500])
def test_synthetic_reference_tree_rows_bitexact(synth_packed, n):
    _, profs = _render_bands(synth_packed(n), 1024, 1024, 8, 8, SYNTH_BANDS)
    _trace_kernel_ran(profs)


def test_synthetic_12500_sah_rows_bitexact(synth_packed):
    _, profs = _render_bands(synth_packed(12500, "sah"), 1024, 1024, 8, 8, SYNTH_BANDS)
    _trace_kernel_ran(profs)


def test_synthetic_100k_band_bitexact(synth_packed, ptopts):
    p = synth_packed(100000)
    img, profs = _render_bands(p, 1024, 1024, 8, 8, [(192, 208)])
    _trace_kernel_ran(profs)
    ptopts.set("leaf_pool", "0")  # the same render with each lane walking its own leaf pairs
    img2, _ = _render_bands(p, 1024, 1024, 8, 8, [(192, 208)])
    assert_same_bits(img2, img, "leaf_pool=0 vs default (pooled leaf turns)")


def test_synthetic_1m_band_bitexact(synth_packed):
    p = synth_packed(1000000)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        assert s.info["nodes"] <= 32767 and s.info["max_stack"] <= 17  # bvh.ts's depth cap of 16
    _, profs = _render_bands(p, 1024, 1024, 2, 8, [(256, 272)])
    _trace_kernel_ran(profs)


@pytest.mark.parametrize("bvh", ["sah", "reference"])
def test_many_emitters_rows_bitexact(synth_packed, bvh):
    """A finely meshed light (synth_scene LIGHT_GRID 12: 288 emissive triangles) over the 1,000-triangle
    synthetic scene: on the fast tree all 288 sit in ONE leaf under the root, which the pruning never
    skips (advisor r04: round 4 gave them an SAH subtree), and the bands through the light and the box
    must see it, bit-exact against the oracle on both trees."""
    p = synth_packed(1000, bvh, 12)
    if bvh == "sah":
        left = int(p.bvh_data[6 + 2])
        assert p.bvh_data[left] == 1.0 and int(p.bvh_data[left + 4]) // 4 == 288
    _, profs = _render_bands(p, 1024, 1024, 4, 8, SYNTH_BANDS)
    _trace_kernel_ran(profs)


def test_many_emitters_10k_rows_bitexact(synth_packed):
    """A light of 10,082 emissive triangles (LIGHT_GRID 71) over the 1,000-triangle synthetic scene on
    the fast tree (advisor r05): every one sits in the emitter leaf under the root, which is >= 128
    entries, so it gets chunks (option leaf_bvh) and the big-leaf machinery by default — the leaf
    pass or the cooperative turns, as the probe decides — and every shadow ray meets it.  Rows
    through the light and the box, bit-exact against the oracle (at 256^2 so the oracle's 10k-test
    shadow rays stay cheap)."""
    p = synth_packed(1000, "sah", 71)
    left = int(p.bvh_data[6 + 2])
    assert p.bvh_data[left] == 1.0 and int(p.bvh_data[left + 4]) // 4 == 2 * 71 * 71
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        assert max(n for _, n, _ in s.leaf_bvhs()) == 2 * 71 * 71  # the emitter leaf has chunks
    _, profs = _render_bands(p, 256, 256, 2, 8, [(48, 56), (80, 88)])
    _trace_kernel_ran(profs)
