#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/.

  hash_kat.json           hash1u / hash1 / hash2 (hash.wgsl:1-28) on fixed inputs, computed
                          here with plain Python integers (mod 2^32) and numpy f32 rounding,
                          independently of the C oracle.
  survey_scene_stats.json scene/BVH statistics from SURVEY.md §8's table, which the survey
                          derived with its own throwaway restatement of parse-obj.ts + bvh.ts
                          + packer.ts (independent of this repo's code).  Typed in, not computed.
  packed_sha256.json      SHA-256 + lengths of the packed buffers the Node host emits for each
                          scene (regression pin; tests also check them against the Python oracle).
  cornell32_radiance.npz  oracle per-pixel radiance, CornellBox 32x32, t = 0..3, depth 16,
                          plus the meta block used (regression pin for oracle and GPU).

Run from the repo root: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

M32 = 0xFFFFFFFF
KAT_INPUTS = [0, 1, 2, 3, 7, 11, 17, 42, 1000, 16787, 65535, 65536, 123456789, 2**31 - 1, 2**31, 2**32 - 1,
              0xDEADBEEF, 0x9E3779B9, 3141592653]


def mix(n: int) -> int:
    n = ((n << 13) & M32) ^ n
    return (n * ((n * n * 15731 + 789221) & M32) + 1376312589) & M32


def hash1u(n: int) -> int:
    return mix(n) & 0x7FFFFFFF


def hash1(n: int) -> float:
    return float(np.float32(1.0) - np.float32(np.float32(mix(n) & 0x7FFFFFFF) / np.float32(2147483648.0)))


def hash2(n: int):
    m = mix(n)
    kx, ky = (m * m) & M32, (m * ((m * 16807) & M32)) & M32
    return [float(np.float32(np.float32(kx & 0x7FFFFFFF) / np.float32(2147483648.0))),
            float(np.float32(np.float32(ky & 0x7FFFFFFF) / np.float32(2147483648.0)))]


SURVEY_STATS = {
    # tris, verts, BVH nodes / leaves, leaf refs, max leaf, bvh floats, tri floats excl. vn+pad
    "CornellBox": {"tris": 36, "verts": 72, "nodes": 21, "leaves": 11, "refs": 164, "max_leaf": 20, "bvh_len": 1019,
                   "tri_len_no_vn_pad": 496},
    "CornellBox-Mirror": {"tris": 36, "verts": 72, "nodes": 21, "leaves": 11, "refs": 164, "max_leaf": 20,
                          "bvh_len": 1019},
    "CornellBox-Glossy": {"tris": 1112, "verts": 578, "nodes": 777, "leaves": 389, "refs": 5223, "max_leaf": 50,
                          "bvh_len": 34107},
    "MedievalBoat": {"tris": 12573, "verts": 15222, "nodes": 5661, "leaves": 2831, "refs": 52090, "max_leaf": 3791,
                     "bvh_len": 304603, "vn_len": 9268 * 3},
}

SCENES = ["CornellBox", "CornellBox-Mirror", "CornellBox-Glossy", "CornellBox-Sphere", "MedievalBoat"]


def node_pack(scene, out, *extra):
    subprocess.run(["node", os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "node", "bin", "pt-pack.js"),
                    os.path.join(ROOT, "scenes", "scene_assets", scene + ".xml"), out, *extra], check=True)
    tri = np.fromfile(os.path.join(out, "triangle_data.f32"), np.float32)
    bvh = np.fromfile(os.path.join(out, "bvh_data.f32"), np.float32)
    meta = np.fromfile(os.path.join(out, "meta.f32"), np.float32)
    return tri, bvh, meta


def main():
    kat = {"inputs": KAT_INPUTS, "hash1u": [hash1u(n) for n in KAT_INPUTS], "hash1": [hash1(n) for n in KAT_INPUTS],
           "hash2": [hash2(n) for n in KAT_INPUTS]}
    with open(os.path.join(HERE, "hash_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    with open(os.path.join(HERE, "survey_scene_stats.json"), "w") as f:
        json.dump(SURVEY_STATS, f, indent=1)
    sha = {}
    with tempfile.TemporaryDirectory() as td:
        for s in SCENES:
            tri, bvh, _ = node_pack(s, os.path.join(td, s))
            sha[s] = {"triangle_len": int(tri.size), "bvh_len": int(bvh.size),
                      "triangle_sha256": hashlib.sha256(tri.tobytes()).hexdigest(),
                      "bvh_sha256": hashlib.sha256(bvh.tobytes()).hexdigest()}
        tri, bvh, meta = node_pack("CornellBox", os.path.join(td, "c32"), "--width", "32", "--height", "32")
    with open(os.path.join(HERE, "packed_sha256.json"), "w") as f:
        json.dump(sha, f, indent=1)
    import oracle
    rad = np.stack([oracle.frame(tri, bvh, meta, t, 16)[0] for t in range(4)])
    np.savez_compressed(os.path.join(HERE, "cornell32_radiance.npz"), meta=meta, radiance=rad, salts=np.arange(4))
    print("golden fixtures written")


if __name__ == "__main__":
    main()
