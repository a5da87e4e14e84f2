"""Python-side counterpart of the reference host entry (src/index.ts:24-186 -> programEntry).

Scene loading stays in the reference's language: `load_scene` runs the Node host's packer
(node/bin/pt-pack.js: INI/XML/OBJ/MTL -> f64 BVH -> packed buffers + the 48-float meta
block).  `program_entry` then renders all samplesPerPixel frames on the GPU and applies the
display transform, like programEntry's render_loop (program-raymarch.ts:226-335).
"""
from __future__ import annotations

import json
import os
import subprocess
import tempfile
from dataclasses import dataclass

import numpy as np

from ._lib import MODE_AUTO, Scene, tonemap

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACK_JS = os.path.join(_PKG_ROOT, "node", "bin", "pt-pack.js")


@dataclass
class PackedScene:
    """SceneObjectPacked (data-structs.ts:46-50) + the meta block and settings it renders with."""
    triangle_data: np.ndarray
    bvh_data: np.ndarray
    meta: np.ndarray
    settings: dict
    io: dict

    @property
    def screen_dimension(self):
        return [int(self.meta[0]), int(self.meta[1])]


def load_scene(src: str, width: int | None = None, height: int | None = None, spp: int | None = None,
               rr: float | None = None, direct_only: bool = False, web_root: str | None = None) -> PackedScene:
    """Pack a .ini or .xml scene with the Node host; optional overrides of the INI settings."""
    extra = []
    for flag, v in (("--width", width), ("--height", height), ("--spp", spp), ("--rr", rr), ("--web-root", web_root)):
        if v is not None:
            extra += [flag, str(v)]
    if direct_only:
        extra.append("--direct-only")
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["node", PACK_JS, src, td, *extra], check=True, capture_output=True)
        tri = np.fromfile(os.path.join(td, "triangle_data.f32"), np.float32)
        bvh = np.fromfile(os.path.join(td, "bvh_data.f32"), np.float32)
        meta = np.fromfile(os.path.join(td, "meta.f32"), np.float32)
        with open(os.path.join(td, "scene.json")) as f:
            info = json.load(f)
    return PackedScene(tri, bvh, meta, info["settings"], info["io"])


def program_entry(packed: PackedScene, device: int = 0, max_depth: int = 16, mode: int = MODE_AUTO, frame0: int = 0,
                  spp: int | None = None, counters: bool = False, vertex_normals: bool = False) -> dict:
    """Render spp (default samplesPerPixel) frames; returns accum [H,W,3] f32, rgba [H,W,4] u8 and the work
    counters (None unless asked for: they run the kernels' counting builds)."""
    n = int(spp if spp is not None else packed.settings["samplesPerPixel"])
    with Scene(packed.triangle_data, packed.bvh_data, device=device) as s:
        if vertex_normals:
            s.set_vertex_normals(True)
        if counters:
            accum, cnt = s.render(packed.meta, frame0, n, 1, max_depth, mode, counters=True)
        else:
            accum, cnt = s.render(packed.meta, frame0, n, 1, max_depth, mode), None
    return {"accum": accum, "sample_runs": n, "rgba": tonemap(accum, n), "counters": cnt}
