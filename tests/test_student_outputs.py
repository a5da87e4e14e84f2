"""Statistical parity with the reference's OWN renders (scenes/student_outputs/**.png: the WGSL
path tracer's 512x512 outputs for each .ini, tone-mapped by program-raymarch.ts:295-316 with
unknown wall-clock RNG seeds).  Same seeds are impossible, so images are compared on
32x32-pixel block means of the tone-mapped u8 channels, where 50+ spp of Monte Carlo noise
averages out.  This is the only check that ties the numerics to the reference's actual
execution (the oracle restates it; the GPU matches the oracle bit for bit).

Stated tolerances (u8 levels, per channel): global mean within 3, block means within 2.5 on
average (MAD) — measured margins are recorded in DESIGN.md §4.
"""
import os

import numpy as np
import pytest
from PIL import Image

from conftest import SCENES

MILESTONE = pytest.mark.xfail(strict=False, reason="rendered by the milestone-era shader (submission-milestone.md), "
                              "not by the final src/ code this build restates; reported for information")
CONFIGS = [
    ("final", "cornell_box_full_lighting"),
    ("final", "cornell_box_direct_lighting_only"),
    ("final", "cornell_box_full_lighting_low_probability"),
    ("final", "mirror"),
    ("final", "glossy"),
    ("final", "refraction"),
    pytest.param("milestone", "cornell_box_milestone", marks=MILESTONE),
    pytest.param("milestone", "sphere_milestone", marks=MILESTONE),
]
# measured on MI355X (round 1): global <= 1.57, block MAD <= 0.93 over the six final configs
TOL_GLOBAL, TOL_BLOCK_MAD = 3.0, 2.5


def block_means(img, b):
    h, w = img.shape[:2]
    return img[: h // b * b, : w // b * b, :3].astype(np.float64).reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def compare(ours, ref, b):
    g = np.abs(ours[..., :3].reshape(-1, 3).mean(0) - ref[..., :3].reshape(-1, 3).mean(0))
    bm = np.abs(block_means(ours, b) - block_means(ref, b))
    return float(g.max()), float(bm.mean()), float(bm.max())


@pytest.mark.gpu
@pytest.mark.parametrize("group,name", CONFIGS)
def test_gpu_render_matches_reference_png(group, name):
    import pt_amd
    ini = os.path.join(SCENES, "scene_files", group, name + ".ini")
    packed = pt_amd.load_scene(ini, web_root=SCENES)
    r = pt_amd.program_entry(packed, max_depth=16)
    ref = np.array(Image.open(os.path.join(SCENES, "student_outputs", group, name + ".png")))
    assert ref.shape == r["rgba"].shape
    gdiff, mad, bmax = compare(r["rgba"], ref, 32)
    print(f"{group}/{name}: global {gdiff:.2f} block MAD {mad:.2f} block max {bmax:.2f}")
    assert gdiff < TOL_GLOBAL and mad < TOL_BLOCK_MAD, (gdiff, mad, bmax)


@pytest.mark.parametrize("name", ["cornell_box_full_lighting", "cornell_box_direct_lighting_only"])
def test_oracle_matches_reference_png_lowres(name):
    """CPU: the oracle at 128x128, 8 spp against the reference PNG block-averaged 4x (looser bound:
    fewer samples and a different pixel footprint)."""
    import oracle
    import scene_oracle as so
    sc = so.ini_file_to_ini_scene(so.parse_ini_file(open(os.path.join(SCENES, "scene_files", "final", name + ".ini")).read()))
    with open(os.path.join(SCENES, sc["IO"]["scene"].lstrip("/"))) as f:
        cam, _ = so.load_scene_xml(f.read())
    _, ps = so.load_scene(os.path.join(SCENES, sc["IO"]["scene"].lstrip("/")), os.path.join(SCENES, "scene_assets"))
    st = dict(sc["Settings"], imageWidth=128, imageHeight=128)
    meta = so.make_meta(so.screen_dimension(st), cam, st)
    acc, _ = oracle.render(ps.triangle_data, ps.bvh_data, meta, 0, 8, 1, 16, nthreads=8)
    ours = oracle.tonemap(acc, 8).reshape(128, 128, 4)
    ref = np.array(Image.open(os.path.join(SCENES, "student_outputs", "final", name + ".png")))
    ref4 = block_means(ref, 4)
    gdiff, mad, bmax = compare(ours.astype(np.float64), np.concatenate([ref4, np.full(ref4.shape[:2] + (1,), 255.0)], -1), 8)
    assert gdiff < 2 * TOL_GLOBAL and mad < 2 * TOL_BLOCK_MAD, (gdiff, mad, bmax)
