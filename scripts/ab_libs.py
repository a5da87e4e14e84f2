#!/usr/bin/env python3
"""A/B two (or more) builds of libpt_hip.so in ONE process on the same GPU, interleaved, so
box-to-box clock differences cancel.  Each library is loaded privately (RTLD_LOCAL) and driven
through the C ABI only.

usage: ab_libs.py LIB[@ENV=VAL,ENV=VAL] ... [--scene CornellBox] [--res 1024] [--spp 64] [--depth 8]
                 [--rounds 5] [--mode 0]
The optional @OPT list is set around that variant's renders through the library's own
pt_set_option (keys "kernel" or "PT_KERNEL"; builds older than the option API read PT_* environment
variables instead), so one build can be compared with itself under different switches.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scene", default="CornellBox")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--all-meshes", action="store_true", help="every primitive of the scene (pt-pack --all-meshes)")
    ap.add_argument("--async-torch", action="store_true", help="pt_render_async on a torch stream (as bench.py)")
    ap.add_argument("--counters", action="store_true",
                    help="after the timed rounds, one counted render per variant; print its work counters")
    a = ap.parse_args()
    import torch  # one HIP runtime for the process (see pt_amd/_lib.py)
    torch.cuda.init()
    with tempfile.TemporaryDirectory() as td:
        if a.scene.startswith("synthetic-"):  # scripts/synth_scene.py: N triangles in the Cornell box
            sys.path.insert(0, os.path.join(ROOT, "scripts"))
            import synth_scene
            xml = synth_scene.write(int(a.scene.split("-")[1]), td)
        else:
            xml = os.path.join(ROOT, "scenes", "scene_assets", a.scene + ".xml")
        subprocess.run(["node", os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "node", "bin", "pt-pack.js"),
                        xml, td, "--width", str(a.res), "--height", str(a.res)] + (["--all-meshes"] if a.all_meshes else []),
                       check=True, capture_output=True)
        tri = np.fromfile(os.path.join(td, "triangle_data.f32"), np.float32)
        bvh = np.fromfile(os.path.join(td, "bvh_data.f32"), np.float32)
        meta = np.fromfile(os.path.join(td, "meta.f32"), np.float32)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    runs = []
    loaded = {}

    def with_env(L, env, fn):
        if hasattr(L, "pt_set_option"):  # the option API
            name = lambda k: (k[3:].lower() if k.startswith("PT_") else k).encode()  # noqa: E731
            L.pt_set_option.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
            for k, v in env.items():
                assert L.pt_set_option(name(k), v.encode()) == 0, L.pt_last_error()
            try:
                return fn()
            finally:
                for k in env:
                    L.pt_set_option(name(k), None)
        old = {k: os.environ.get(k) for k in env}  # older builds: PT_* environment variables
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    for spec in a.libs:
        path, _, envs = spec.partition("@")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        if path not in loaded:
            loaded[path] = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
        L = loaded[path]
        L.pt_scene_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p)]
        L.pt_render.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.pt_last_error.restype = ctypes.c_char_p
        L.pt_render_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        h = ctypes.c_void_p()
        assert L.pt_scene_create(p(tri), tri.size, p(bvh), bvh.size, 0, ctypes.byref(h)) == 0, L.pt_last_error()
        acc = np.zeros((a.res, a.res, 3), np.float32)
        rc = with_env(L, env, lambda: L.pt_render(h, p(meta), 0, a.spp, 1, a.depth, a.mode, p(acc), None))  # warm-up
        assert rc == 0, L.pt_last_error()
        runs.append({"lib": spec, "L": L, "h": h, "acc": acc, "ms": [], "ref": acc.copy(), "env": env})
    if a.async_torch:
        for r in runs:
            r["stream"] = torch.cuda.Stream()
            r["dacc"] = torch.zeros((a.res, a.res, 3), dtype=torch.float32, device="cuda")
    for _ in range(a.rounds):
        for r in runs:
            if a.async_torch:
                st = r["stream"]
                with torch.cuda.stream(st):
                    r["dacc"].zero_()
                st.synchronize()
                t = time.perf_counter()
                rc = with_env(r["L"], r["env"], lambda: r["L"].pt_render_async(r["h"], p(meta), 0, a.spp, 1, a.depth, a.mode,
                                                                      ctypes.c_void_p(r["dacc"].data_ptr()), None,
                                                                      ctypes.c_void_p(st.cuda_stream)))
                st.synchronize()
            else:
                r["acc"][:] = 0
                t = time.perf_counter()
                rc = with_env(r["L"], r["env"], lambda: r["L"].pt_render(r["h"], p(meta), 0, a.spp, 1, a.depth, a.mode,
                                                                 p(r["acc"]), None))
            assert rc == 0
            r["ms"].append((time.perf_counter() - t) * 1e3)
    if a.async_torch:
        for r in runs:
            r["ref"] = r["dacc"].cpu().numpy()
    base = runs[0]["ref"]
    if a.counters:  # pt_counters (include/pt_hip.h): six uint64
        names = ("samples", "ext_queries", "shadow_queries", "nodes", "tri_tests", "box_tests")
        for r in runs:
            c = (ctypes.c_uint64 * 6)()
            acc = np.zeros((a.res, a.res, 3), np.float32)
            rc = with_env(r["L"], r["env"], lambda: r["L"].pt_render(r["h"], p(meta), 0, a.spp, 1, a.depth, a.mode,
                                                             p(acc), ctypes.cast(c, ctypes.c_void_p)))
            assert rc == 0
            print(json.dumps({"lib": r["lib"], "counters": dict(zip(names, map(int, c)))}), flush=True)
    for r in runs:
        ms = float(np.median(r["ms"]))
        print(json.dumps({"lib": r["lib"], "ms_median": round(ms, 3), "msamples_s": round(a.res * a.res * a.spp / ms / 1e3, 1),
                          "same_bits_as_first": bool(np.array_equal(r["ref"].view(np.uint32), base.view(np.uint32)))}),
              flush=True)


if __name__ == "__main__":
    main()
