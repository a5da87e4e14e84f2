#!/usr/bin/env python3
"""Per-phase statistics of the fused kernel k_wf_step_bf (verdict r05 item 2): a diagnostic build
(make -C brown-cs2240-path-tracer_amd/csrc EXTRA=-DPT_PHASE_STATS=1 OUT_DIR=<dir>) times each wave's
phases with s_memtime and counts, per phase, loop iterations and active lanes (pt_wavefront.hip
PhaseAcc).  This script renders the bench workload through that library (same sources, so the same
build id) and prints per instance (extension / shadow) and phase: the share of the waves' wall
cycles, iterations per 64-path batch and the lane use (active lanes / 64 per iteration).

usage: phase_stats.py DIAG_LIB [--scene CornellBox --res 1024 --spp 256 --depth 8]"""
import argparse
import ctypes
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "brown-cs2240-path-tracer_amd"))
sys.path.insert(0, ROOT)
PHASES = ["load", "phase1", "phase1_full", "replay", "replay_leaf", "shade", "append"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=8)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, pt_amd/_lib.py)
    import pt_amd._lib as L
    L._LIB_FILE = os.path.abspath(a.lib)
    import bench
    import pt_amd
    lib = L.load_library()
    lib.pt_phase_stats_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    with tempfile.TemporaryDirectory() as td:
        tri, bvh, meta = bench.pack_scene(a.scene, td, a.res, a.res, a.spp)
    scene = pt_amd.Scene(tri, bvh)
    acc = np.zeros((a.res, a.res, 3), np.float32)
    scene.render(meta, 0, min(a.spp, 8), 1, a.depth, pt_amd.MODE_AUTO, accum=acc)  # warm-up
    buf = np.zeros((2, len(PHASES), 3), np.uint64)
    assert lib.pt_phase_stats_read(buf.ctypes.data, 1) == 0
    acc[:] = 0
    scene.render(meta, 0, a.spp, 1, a.depth, pt_amd.MODE_AUTO, accum=acc)
    assert lib.pt_phase_stats_read(buf.ctypes.data, 1) == 0
    scene.close()
    out = {"scene": a.scene, "res": a.res, "spp": a.spp, "depth": a.depth, "instances": {}}
    for ext, name in ((1, "extension"), (0, "shadow")):
        b = buf[ext].astype(np.float64)
        batches = b[PHASES.index("shade"), 1]  # one path-logic sample per batch
        timed = [p for p in PHASES if p not in ("phase1_full", "replay_leaf")]
        total = sum(b[PHASES.index(p), 0] for p in timed)
        inst = {"batches": int(batches), "cycles_per_batch": round(total / max(batches, 1), 1), "phases": {}}
        for i, p in enumerate(PHASES):
            cyc, it, ln = b[i]
            inst["phases"][p] = {
                "share_of_wave_cycles": round(cyc / total, 4) if p in timed and total else None,
                "iterations_per_batch": round(it / max(batches, 1), 3),
                "lane_use": round(ln / (64.0 * it), 4) if it else None}
        out["instances"][name] = inst
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
