#!/usr/bin/env python3
"""A/B the render kernels (PT_KERNEL variants) on one workload, interleaved in one process.

Usage: python scripts/perf_variants.py [--scene CornellBox] [--res 1024] [--spp 64] [--depth 8]
       [--rounds 3] [--variants literal,regen,regen_lds]
Prints one JSON line per variant: median/min kernel ms and Msamples/s.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "brown-cs2240-path-tracer_amd")
sys.path.insert(0, PKG)


VARIANTS = {
    "auto": {},
    "literal": {"PT_KERNEL": "literal"},
    "mega_nested": {"PT_KERNEL": "mega", "PT_TRAV": "nested"},
    "mega_flat_global": {"PT_KERNEL": "mega", "PT_TRAV": "flat1", "PT_LDS": "0"},
    "mega_flat_lds": {"PT_KERNEL": "mega", "PT_TRAV": "flat1"},
    "mega_pred_lds": {"PT_KERNEL": "mega", "PT_TRAV": "pred"},
    "mega_lean_lds": {"PT_KERNEL": "mega", "PT_TRAV": "lean"},
    "mega_lean_global": {"PT_KERNEL": "mega", "PT_TRAV": "lean", "PT_LDS": "0"},
    "wavefront_global": {"PT_KERNEL": "wavefront", "PT_TRAV": "flat1", "PT_LDS": "0"},
    "wavefront_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "flat1"},
    "wavefront_pred_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "pred"},
    "wavefront_lean_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean"},
    "wavefront_lean_global": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean", "PT_LDS": "0"},
    "wavefront_lean2_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean2"},
    "wavefront_lean4_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean4"},
    "wavefront_lean8_lds": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8"},
    "mega_lean2_lds": {"PT_KERNEL": "mega", "PT_TRAV": "lean2"},
    "mega_lean_fastrcp": {"PT_KERNEL": "mega", "PT_TRAV": "lean", "PT_FASTRCP": "1"},
    "wavefront_lean4_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean4", "PT_FASTRCP": "1"},
    "wavefront_lean8_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_FASTRCP": "1"},
    "wavefront_lean8_div": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_FASTRCP": "0"},
    "wavefront_lean16_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_FASTRCP": "1"},
    "wf_lean8_bias2": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_NODE_BIAS": "2"},
    "wf_lean8_bias4": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_NODE_BIAS": "4"},
    "wf_lean16_bias2": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "2"},
    "wf_lean16_bias4": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "4"},
    "wf_lean16_bias8": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "8"},
    "wf_lean16_bias16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "16"},
    "wf_lean16_bias64": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "64"},
    "wf_lean32_bias8": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean32", "PT_NODE_BIAS": "8"},
    "wf_lean32_bias16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean32", "PT_NODE_BIAS": "16"},
    "wf_lean32_bias64": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean32", "PT_NODE_BIAS": "64"},
    "wf_lean8_bias16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_NODE_BIAS": "16"},
    "mega_lean2_bias2": {"PT_KERNEL": "mega", "PT_TRAV": "lean2", "PT_NODE_BIAS": "2"},
    "mega_lean2_bias4": {"PT_KERNEL": "mega", "PT_TRAV": "lean2", "PT_NODE_BIAS": "4"},
    "mega_lean_bias2": {"PT_KERNEL": "mega", "PT_TRAV": "lean", "PT_NODE_BIAS": "2"},
    "mega_lean2_bias8": {"PT_KERNEL": "mega", "PT_TRAV": "lean2", "PT_NODE_BIAS": "8"},
    "mega_lean4_bias4": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_NODE_BIAS": "4"},
    "mega_lean4_bias8": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_NODE_BIAS": "8"},
    "mega_lean2_bias4_fast": {"PT_KERNEL": "mega", "PT_TRAV": "lean2", "PT_NODE_BIAS": "4", "PT_FASTRCP": "1"},
    "mega_lean4_bias8_fast": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_NODE_BIAS": "8", "PT_FASTRCP": "1"},
    "mega_lean4_bias16_fast": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_NODE_BIAS": "16", "PT_FASTRCP": "1"},
    "mega_lean2_bias8_fast": {"PT_KERNEL": "mega", "PT_TRAV": "lean2", "PT_NODE_BIAS": "8", "PT_FASTRCP": "1"},
    "wf_bf": {"PT_KERNEL": "wavefront"},
    "wf_bf_nofuse": {"PT_KERNEL": "wavefront", "PT_FUSE": "0"},
    "wf_bf_nofuse_2blk": {"PT_KERNEL": "wavefront", "PT_FUSE": "0", "PT_WF_TRACE_BLOCKS": "512"},
    "wf_gen": {"PT_KERNEL": "wavefront", "PT_FUSE_GEN": "1"},
    "wf_nogen": {"PT_KERNEL": "wavefront", "PT_FUSE_GEN": "0"},
    "wf_parts4": {"PT_KERNEL": "wavefront", "PT_PARTS": "4"},
    "wf_parts3": {"PT_KERNEL": "wavefront", "PT_PARTS": "3"},
    "wf_parts4_16M": {"PT_KERNEL": "wavefront", "PT_PARTS": "4", "PT_WF_PATHS": "16777216"},
    "wf_bf_single": {"PT_KERNEL": "wavefront", "PT_DUAL": "0"},
    "wf_bf_32M_single": {"PT_KERNEL": "wavefront", "PT_DUAL": "0", "PT_WF_PATHS": "33554432"},
    "wf_bf_16M": {"PT_KERNEL": "wavefront", "PT_WF_PATHS": "16777216"},
    "wf_bf_32M": {"PT_KERNEL": "wavefront", "PT_WF_PATHS": "33554432"},
    "wf_bf_3blk": {"PT_KERNEL": "wavefront", "PT_WF_TRACE_BLOCKS": "768"},
    "wf_bf_2blk": {"PT_KERNEL": "wavefront", "PT_WF_TRACE_BLOCKS": "512"},
    "wf_bf_div": {"PT_KERNEL": "wavefront", "PT_FASTRCP": "0"},
    "wf_nomb": {"PT_KERNEL": "wavefront", "PT_MAILBOX": "0"},
    "wf_mb16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16"},
    "wf_mb32": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean32"},
    "wf_mb32_bias16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean32", "PT_NODE_BIAS": "16"},
    "wf_mb8": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8"},
    "wf_mb4": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean4"},
    "wf_mb16_bias4": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "4"},
    "wf_mb8_bias4": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_NODE_BIAS": "4"},
    "wf_mb8_bias2": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_NODE_BIAS": "2"},
    "wf_mb16_bias16": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "16"},
}


def set_variant(v):
    import pt_amd
    pt_amd.reset_options()  # the library's options (pt_set_option), not the environment
    for k, val in VARIANTS[v].items():
        pt_amd.set_option(k, val)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="mega_flat_lds,wavefront_lds")
    args = ap.parse_args()
    import torch

    import pt_amd

    H = args.height or args.res
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["node", os.path.join(PKG, "node", "bin", "pt-pack.js"),
                        os.path.join(ROOT, "scenes", "scene_assets", args.scene + ".xml"), td, "--width",
                        str(args.res), "--height", str(H)], check=True)
        tri = np.fromfile(os.path.join(td, "triangle_data.f32"), np.float32)
        bvh = np.fromfile(os.path.join(td, "bvh_data.f32"), np.float32)
        meta = np.fromfile(os.path.join(td, "meta.f32"), np.float32)
    W, H = int(meta[0]), int(meta[1])
    scene = pt_amd.Scene(tri, bvh)
    st = torch.cuda.Stream()
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    variants = args.variants.split(",")
    times = {v: [] for v in variants}
    ref = None
    for r in range(args.rounds + 1):
        for v in variants:
            set_variant(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                acc.zero_()
                e0.record(st)
                scene.render_async(meta, 0, args.spp, 1, args.depth, 0, acc.data_ptr(), st.cuda_stream)
                e1.record(st)
            e1.synchronize()
            if r > 0:
                times[v].append(e0.elapsed_time(e1))
            out = acc.cpu().numpy()
            if ref is None:
                ref = out.copy()
            elif not np.array_equal(out.view(np.uint32), ref.view(np.uint32)):
                print(json.dumps({"variant": v, "error": "result differs from first variant"}), flush=True)
    n = W * H * args.spp
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"scene": args.scene, "res": [W, H], "spp": args.spp, "depth": args.depth, "variant": v,
                          "ms_median": round(float(np.median(t)), 3), "ms_min": round(float(t.min()), 3),
                          "msamples_s": round(n / (np.median(t) * 1e-3) / 1e6, 1)}), flush=True)
    scene.close()


if __name__ == "__main__":
    main()
