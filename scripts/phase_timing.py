#!/usr/bin/env python3
"""Where the fused kernel's time goes: shader-clock cycles per phase of bf_step_batch, from a
diagnostic build (make -C brown-cs2240-path-tracer_amd/csrc OUT_DIR=/root/repo/ab/phase
EXTRA=-DPT_PHASE_TIMING=1 /root/repo/ab/phase/libpt_hip.so), driven through the C ABI.

usage: phase_timing.py [LIB] [--scene CornellBox] [--res 1024] [--spp 16] [--depth 8]
Prints one JSON line per queue (extension / shadow): cycles per 64-entry batch per phase and
each phase's share.  s_memtime waits for its own scalar load, so the marks cost a little and
the split (not the total) is what this measures.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ["load_ray_cull", "phase1_brute_force", "phase2_replay", "shading", "append_store"]
WAVES, SLOTS = 16384, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "ab", "phase", "libpt_hip.so"))
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    import torch  # one HIP runtime for the process (see pt_amd/_lib.py)
    torch.cuda.init()
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["node", os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "node", "bin", "pt-pack.js"),
                        os.path.join(ROOT, "scenes", "scene_assets", a.scene + ".xml"), td, "--width", str(a.res),
                        "--height", str(a.res)], check=True, capture_output=True)
        tri = np.fromfile(os.path.join(td, "triangle_data.f32"), np.float32)
        bvh = np.fromfile(os.path.join(td, "bvh_data.f32"), np.float32)
        meta = np.fromfile(os.path.join(td, "meta.f32"), np.float32)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L = ctypes.CDLL(os.path.abspath(a.lib), mode=os.RTLD_LOCAL)
    L.pt_scene_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p)]
    L.pt_render.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.pt_last_error.restype = ctypes.c_char_p
    L.pt_debug_phase_read.argtypes = [ctypes.c_void_p]
    h = ctypes.c_void_p()
    assert L.pt_scene_create(p(tri), tri.size, p(bvh), bvh.size, 0, ctypes.byref(h)) == 0, L.pt_last_error()
    acc = np.zeros((a.res, a.res, 3), np.float32)
    buf = np.zeros(WAVES * SLOTS, np.uint64)
    assert L.pt_render(h, p(meta), 0, 2, 1, a.depth, 0, p(acc), None) == 0, L.pt_last_error()  # warm-up
    assert L.pt_debug_phase_read(p(buf)) > 0
    acc[:] = 0
    assert L.pt_render(h, p(meta), 0, a.spp, 1, a.depth, 0, p(acc), None) == 0, L.pt_last_error()
    assert L.pt_debug_phase_read(p(buf)) > 0
    t = buf.reshape(WAVES, SLOTS).sum(axis=0).astype(np.float64)
    for q, off in (("extension", 0), ("shadow", 8)):
        batches = t[off + 5]
        cyc = t[off:off + 5]
        tot = cyc.sum()
        print(json.dumps({"queue": q, "scene": a.scene, "res": a.res, "spp": a.spp, "batches": int(batches),
                          "cycles_per_batch": {k: round(c / max(batches, 1), 1) for k, c in zip(PHASES, cyc)},
                          "share": {k: round(c / max(tot, 1), 3) for k, c in zip(PHASES, cyc)}}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
