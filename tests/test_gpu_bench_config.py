"""Parity pinned at the benchmarked configurations (BASELINE.json configs[0..1]) and a
noise-calibrated per-pixel L2 comparison with the reference's own renders.

* The bench's default pipeline (AUTO: fused wavefront k_wf_step_bf, camera paths made in its
  first launch, the batch in parts on their own streams, region queues) renders CornellBox
  1024^2, depth 8, frames 0..255 — exactly the bench step — and bands of rows of that
  accumulator are compared bit for bit with the C oracle (oracle/pt_oracle.c) rendering the
  same rows (po_render's y0/y1).  No transitivity through the megakernel.
* Config 1 (CornellBox 256^2, 16 spp, depth 4) against the oracle over the whole image.
* The reference renders (scenes/student_outputs/final/*.png, 512^2, tone-mapped u8, unknown
  wall-clock seeds) are independent noisy estimates of the same image.  With K disjoint salt
  sets at the .ini's spp, d(GPU_k, ref) (per-pixel RMS over u8 RGB) must lie within the
  spread of d(GPU_a, GPU_b) between our own independent renders: the ratio
  d(GPU, ref) / d(GPU_a, GPU_b) is stated in DESIGN.md §4 with the tolerance below.  The same
  on 4x4 block means (noise averaged down 4x, so an estimator bias weighs ~16x more).
"""
import os

import numpy as np
import pytest

import oracle
import pt_amd
from conftest import SCENES

pytestmark = pytest.mark.gpu

ENV_KEYS = ("PT_KERNEL", "PT_TRAV", "PT_LDS", "PT_FASTRCP", "PT_WF_TRACE_BLOCKS", "PT_NODE_BIAS",
            "PT_DUAL", "PT_MAILBOX", "PT_MB_UID_ORDER", "PT_BF", "PT_BF_SLOTS", "PT_FUSE", "PT_PARTS",
            "PT_FUSE_GEN", "PT_WF_PATHS", "PT_BIG_LEAF", "PT_BF_STACKLESS", "PT_SORT", "PT_LEAF_POOL", "PT_POOL_RUN", "PT_REGEN")
ORACLE_THREADS = 16  # the GPU box's CPU share


@pytest.fixture
def clean_env(ptopts):
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    return ptopts


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_same_bits(gpu, ref, what):
    bad = np.argwhere(bits(gpu) != bits(ref))
    assert len(bad) == 0, f"{what}: {len(bad)} mismatches, first {bad[:4].tolist()}"


# ---------------------------------------------------------------------------------------------
# BASELINE.json configs[1]: CornellBox 1024^2, 256 spp, depth 8 — the bench step itself
# ---------------------------------------------------------------------------------------------
BANDS = [(96, 112), (504, 520), (1000, 1016)]  # light + ceiling, image centre (boxes), floor


def test_bench_config_rows_bitexact_vs_oracle(packed, clean_env):
    p = packed["CornellBox"]
    meta = p.meta_for(1024, 1024)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.profile_enable(True)
        gpu = s.render(meta, 0, 256, 1, 8, pt_amd.MODE_AUTO)
        prof = s.profile_read()
        s.profile_enable(False)
    assert "k_wf_step" in prof and "k_regen" not in prof, prof  # the bench's pipeline ran
    for y0, y1 in BANDS:
        ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 256, 1, 8, y0=y0, y1=y1, nthreads=ORACLE_THREADS)
        assert_same_bits(gpu[y0:y1], ref, f"rows {y0}..{y1}")
    assert float(gpu.mean()) > 0.0


def test_config1_256_16spp_depth4_vs_oracle(packed, clean_env):
    """BASELINE.json configs[0]: 256^2 x 16 spp = 2^20 paths, so AUTO takes the wavefront."""
    p = packed["CornellBox"]
    meta = p.meta_for(256, 256)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.profile_enable(True)
        gpu, gc = s.render(meta, 0, 16, 1, 4, pt_amd.MODE_AUTO, counters=True)
        plain = s.render(meta, 0, 16, 1, 4, pt_amd.MODE_AUTO)
        prof = s.profile_read()
        s.profile_enable(False)
    assert "k_wf_step" in prof, prof
    ref, rc = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 16, 1, 4, nthreads=ORACLE_THREADS)
    assert_same_bits(gpu, ref, "counted build")
    assert_same_bits(plain, ref, "uncounted build")
    assert gc == rc, (gc, rc)


@pytest.mark.parametrize("parts", ["1", "2", "4"])
def test_multi_batch_ragged_parts_vs_oracle(packed, clean_env, parts):
    """Several wavefront batches in one call (PT_WF_PATHS smaller than the call's paths), a
    ragged last batch with fewer frames than parts, accumulation across batches."""
    p = packed["CornellBox"]
    meta = p.meta_for(64, 64)
    clean_env.set("PT_KERNEL", "wavefront")
    clean_env.set("PT_WF_PATHS", "12288")  # 3 frames per batch: 7 frames = 3 + 3 + 1
    clean_env.set("PT_PARTS", parts)
    init = np.random.default_rng(7).uniform(0, 1, (64, 64, 3)).astype(np.float32)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        gpu = s.render(meta, 2, 7, 3, 8, pt_amd.MODE_AUTO, accum=init.copy())
    ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 2, 7, 3, 8, acc=init.copy())
    assert_same_bits(gpu, ref, f"parts={parts}")


# ---------------------------------------------------------------------------------------------
# noise-calibrated per-pixel L2 against the reference's own renders
# ---------------------------------------------------------------------------------------------
FINAL = ["cornell_box_full_lighting", "cornell_box_direct_lighting_only", "cornell_box_full_lighting_low_probability",
         "mirror", "glossy", "refraction"]
K_SETS = 4  # disjoint salt sets: frames s * 1000 + [0, spp) (all < 16787: no seed overlap between pixels)
# stated tolerance: d(GPU_k, ref) <= L2_TOL x the largest d(GPU_a, GPU_b) among our own renders,
# per pixel and on 4x4 block means (measured ratios in DESIGN.md §4)
L2_TOL = 1.05


def rms(a, b):
    return float(np.sqrt(np.mean((a[..., :3].astype(np.float64) - b[..., :3].astype(np.float64)) ** 2)))


def block4(img):
    h, w = img.shape[:2]
    return img[..., :3].astype(np.float64).reshape(h // 4, 4, w // 4, 4, 3).mean(axis=(1, 3))


@pytest.mark.parametrize("name", FINAL)
def test_per_pixel_l2_within_noise_of_reference_png(name):
    from PIL import Image
    ini = os.path.join(SCENES, "scene_files", "final", name + ".ini")
    packed = pt_amd.load_scene(ini, web_root=SCENES)
    spp = int(packed.settings["samplesPerPixel"])
    ref = np.array(Image.open(os.path.join(SCENES, "student_outputs", "final", name + ".png")))
    with pt_amd.Scene(packed.triangle_data, packed.bvh_data) as s:
        ours = [s.render_image(packed.meta, k * 1000, spp, 1, 16) for k in range(K_SETS)]
    assert ref.shape == ours[0].shape
    pairs = [(a, b) for a in range(K_SETS) for b in range(a + 1, K_SETS)]
    out = {}
    for label, f in (("pixel", lambda x: x), ("block4", block4)):
        self_d = [rms(f(ours[a]), f(ours[b])) for a, b in pairs]
        ref_d = [rms(f(o), f(ref)) for o in ours]
        ratio = max(ref_d) / max(self_d)
        out[label] = (min(self_d), max(self_d), min(ref_d), max(ref_d), ratio)
        print(f"{name} {label}: self {min(self_d):.3f}..{max(self_d):.3f} ref {min(ref_d):.3f}..{max(ref_d):.3f} "
              f"ratio {ratio:.4f}")
    for label, (_, _, _, _, ratio) in out.items():
        assert ratio <= L2_TOL, (label, out)
