#!/usr/bin/env python3
"""Turn statistics of the traversal kernel k_wf_trace (verdict r05 items 1 and 4): a diagnostic build
(make -C brown-cs2240-path-tracer_amd/csrc EXTRA=-DPT_TRACE_STATS=1 OUT_DIR=<dir>) times each lean
traversal turn with s_memtime and counts its participating lanes (pt_device.h trav_step_lean,
Counters::ts).  Renders the workload through that library (same sources, same build id) and prints
per queue (extension / shadow) and kind: turns, the share of the loop's wall cycles, and the lane use
(participating lanes / 64 per turn):
  node   — node turns (lanes in node state that step)
  leaf   — leaf turns (lanes in leaf state whose pairs are pooled or walked)
  big    — cooperative / chunk turns of a parked big leaf (count only)
  none   — loop iterations with nothing to step (refill waits)
  poolrun— the pool's test rounds: lanes holding a run of RUN entries
  loop   — every loop iteration (cycles = the whole loop; lanes = lanes holding a ray)
  blocked— iterations with idle lanes whose next window waits for the hit ring (a straggler of an
           old window holds its flush); lanes = the idle ones
  starved— iterations with idle lanes and no window left for the wave (the launch's tail)
usage: trace_stats.py DIAG_LIB [--scene CornellBox-Glossy | --synthetic N] [--res 1024 --spp 8 --depth 16]
       [--opt NAME=VALUE ...]"""
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
KINDS = ["node", "leaf", "big", "none", "poolrun", "loop", "blocked", "starved"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="CornellBox-Glossy")
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=16)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, pt_amd/_lib.py)
    import pt_amd._lib as L
    L._LIB_FILE = os.path.abspath(a.lib)
    import bench
    import pt_amd
    lib = L.load_library()
    lib.pt_trace_stats_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    with tempfile.TemporaryDirectory() as td:
        tri, bvh, meta = bench.pack_scene(a.scene, td, a.res, a.res, a.spp, a.synthetic)
    scene = pt_amd.Scene(tri, bvh)
    for kv in a.opt:
        pt_amd.set_option(*kv.split("=", 1))
    acc = np.zeros((a.res, a.res, 3), np.float32)
    scene.render(meta, 0, 1, 1, a.depth, pt_amd.MODE_AUTO, accum=acc)  # warm-up
    buf = np.zeros((2, len(KINDS), 3), np.uint64)
    assert lib.pt_trace_stats_read(buf.ctypes.data, 1) == 0
    acc[:] = 0
    scene.render(meta, 0, a.spp, 1, a.depth, pt_amd.MODE_AUTO, accum=acc)
    assert lib.pt_trace_stats_read(buf.ctypes.data, 1) == 0
    scene.close()
    out = {"scene": f"synthetic-{a.synthetic}" if a.synthetic else a.scene, "res": a.res, "spp": a.spp,
           "depth": a.depth, "options": a.opt, "queues": {}}
    for q, name in ((0, "extension"), (1, "shadow")):
        b = buf[q].astype(np.float64)
        loop = b[KINDS.index("loop"), 0]
        qo = {}
        for i, k in enumerate(KINDS):
            cyc, n, ln = b[i]
            qo[k] = {"turns": int(n), "share_of_loop_cycles": round(cyc / loop, 4) if loop and k in ("node", "leaf") else None,
                     "lane_use": round(ln / (64.0 * n), 4) if n else None}
        out["queues"][name] = qo
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
