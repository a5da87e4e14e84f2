"""Driver of scripts/leaf_visit_stats.c (diagnostic, test infrastructure): dumps a scene's packed
buffers and meta through the oracle's loader, builds the harness and runs it.

    python3 scripts/leaf_visit_stats.py MedievalBoat 1920 1080 [frames] [depth] [min_entries] [row_step]
(ALL_MESHES=1: every primitive of the scene, as --all-meshes; PROBE=n: n of the library's probe rays
instead of the render's; PROBE_GRID=g: the camera probe's g x g pixel-centre rays and their bounces,
pt_leafbvh.cpp probe_pre_leaves — run either with frames 0)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import scene_oracle as so  # noqa: E402


def main():
    name, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    frames = sys.argv[4] if len(sys.argv) > 4 else "1"
    depth = sys.argv[5] if len(sys.argv) > 5 else "16"
    min_entries = sys.argv[6] if len(sys.argv) > 6 else "128"
    step = sys.argv[7] if len(sys.argv) > 7 else "8"
    assets = os.path.join(ROOT, "scenes", "scene_assets")
    all_meshes = os.environ.get("ALL_MESHES") == "1"
    camera, p = so.load_scene(os.path.join(assets, name + ".xml"), assets, all_meshes=all_meshes)
    settings = {"samplesPerPixel": 1, "pathContinuationProb": 0.9, "directLightingOnly": False}
    d = "/tmp/leafstats"
    os.makedirs(d, exist_ok=True)
    np.asarray(p.triangle_data, np.float32).tofile(os.path.join(d, "tri.bin"))
    np.asarray(p.bvh_data, np.float32).tofile(os.path.join(d, "bvh.bin"))
    so.make_meta([W, H], camera, settings).tofile(os.path.join(d, "meta.bin"))
    exe = os.path.join(d, "leaf_visit_stats")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "scripts", "leaf_visit_stats.c"), "-lm"])
    subprocess.check_call([exe, d, frames, depth, min_entries, step, os.environ.get("PROBE", "0"),
                           os.environ.get("PROBE_GRID", "0")])


if __name__ == "__main__":
    main()
