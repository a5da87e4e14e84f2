#!/usr/bin/env python3
"""Diagnostic: where does d(GPU, reference PNG) exceed the noise level?  Renders each final .ini at
its spp under K disjoint salt sets plus one high-spp render, writes the u8 images to
gpurun_out/l2_diag/<name>.npz (ours[K], hi, ref) for offline analysis."""
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brown-cs2240-path-tracer_amd"))
import pt_amd  # noqa: E402

SCENES = os.path.join(ROOT, "scenes")
out_dir = os.path.join(ROOT, "gpurun_out", "l2_diag")
os.makedirs(out_dir, exist_ok=True)
names = sys.argv[1:] or ["cornell_box_full_lighting", "mirror"]
for name in names:
    packed = pt_amd.load_scene(os.path.join(SCENES, "scene_files", "final", name + ".ini"), web_root=SCENES)
    spp = int(packed.settings["samplesPerPixel"])
    ref = np.array(Image.open(os.path.join(SCENES, "student_outputs", "final", name + ".png")))
    with pt_amd.Scene(packed.triangle_data, packed.bvh_data) as s:
        ours = np.stack([s.render_image(packed.meta, k * 1000, spp, 1, 16) for k in range(4)])
        hi = s.render_image(packed.meta, 8000, 8192, 1, 16)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), ours=ours, hi=hi, ref=ref, spp=spp)
    print(name, "saved", flush=True)
