#!/usr/bin/env python3
"""In-process A/B of render options (pt_set_option switches read by every render call, csrc/pt_capi.hip
launch_opts; keys as "kernel" or the old spelling "PT_KERNEL").  Each variant renders the same workload; results must be
bit-identical to the first variant's; times are medians of --reps renders, variants interleaved.
usage: env_ab.py [--scene S --width W --height H --spp N --depth D --reps R] 'A=1,B=2' 'A=0' ..."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brown-cs2240-path-tracer_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--synthetic", type=int, default=0, help="bench.py's N-triangle synthetic scene instead of --scene")
    ap.add_argument("--bvh", default="reference", help="reference | sah (bench.py --bvh)")
    ap.add_argument("--all-meshes", action="store_true", help="every primitive of the scene (bench.py --all-meshes)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--profile", action="store_true", help="one more render per variant with per-launch events")
    ap.add_argument("--scene-opt", action="append", default=[],
                    help="NAME=VALUE set while the scene is created (options pt_scene_create reads, e.g. leaf_bvh=128)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    import bench
    import pt_amd
    with tempfile.TemporaryDirectory() as td:
        tri, bvh, meta = bench.pack_scene(a.scene, td, a.width, a.height, a.spp, a.synthetic, bvh=a.bvh,
                                          all_meshes=a.all_meshes)
    W, H = int(meta[0]), int(meta[1])
    for kv in a.scene_opt:
        pt_amd.set_option(*kv.split("=", 1))
    scene = pt_amd.Scene(tri, bvh)
    pt_amd.reset_options()
    st = torch.cuda.Stream()
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    variants = [dict(kv.split("=", 1) for kv in v.split(",") if kv) for v in a.variants]
    times = {i: [] for i in range(len(variants))}
    ref = None
    for rep in range(a.reps + 1):
        order = list(range(len(variants))) if rep % 2 == 0 else list(reversed(range(len(variants))))
        for i in order:
            pt_amd.reset_options()
            for k, v in variants[i].items():
                pt_amd.set_option(k, v)
            with torch.cuda.stream(st):
                acc.zero_()
                st.synchronize()
                t = time.perf_counter()
                scene.render_async(meta, 0, a.spp, 1, a.depth, pt_amd.MODE_AUTO, acc.data_ptr(), st.cuda_stream)
                st.synchronize()
                dt = time.perf_counter() - t
            scene.check()
            if rep > 0:
                times[i].append(dt)
            out = acc.cpu().numpy()
            if ref is None:
                ref = out.copy()
            elif not np.array_equal(ref.view(np.uint32), out.view(np.uint32)):
                print(json.dumps({"variant": a.variants[i], "error": "result differs from variant 0",
                                  "mismatches": int((ref != out).sum())}), flush=True)
    for i, v in enumerate(a.variants):
        ms = float(np.median(times[i])) * 1e3
        rec = {"variant": v, "scene": a.scene, "ms": round(ms, 3), "msamples_s": round(W * H * a.spp / ms / 1e3, 1)}
        if a.profile:
            pt_amd.reset_options()
            for k, v in variants[i].items():
                pt_amd.set_option(k, v)
            scene.profile_enable(True)
            with torch.cuda.stream(st):
                acc.zero_()
                scene.render_async(meta, 0, a.spp, 1, a.depth, pt_amd.MODE_AUTO, acc.data_ptr(), st.cuda_stream)
            st.synchronize()
            rec["kernels"] = {k: {kk: round(vv, 4) for kk, vv in d.items()} for k, d in scene.profile_read().items()}
            scene.profile_enable(False)
        print(json.dumps(rec), flush=True)
    scene.close()


if __name__ == "__main__":
    main()
