#!/usr/bin/env python3
"""Synthetic Cornell-box-sized scenes for the BVH-size sweep (BASELINE.json
north_star "Cornell-box-sized synthetic BVHs"): N triangles in the Cornell box's bounds — the
box itself (CornellBox-Original.obj: walls, two boxes, the light; 36 triangles) plus N - 36
random triangles, centres uniform in the box, edges ~1.2 N^(-1/3), from
numpy.random.default_rng(1234) — under CornellBox.xml's camera.  Written as OBJ + MTL + scene
XML in the reference's formats, so the product's Node host packs them like any scene.

usage: synth_scene.py N OUT_ROOT [LIGHT_GRID]  ->  OUT_ROOT/scene_assets/synth_N.xml (+ models/synth_N.obj/.mtl)

LIGHT_GRID = g > 1 replaces the light's quad with a g x g grid of cells, two emissive triangles each
(a finely meshed area light: 2 g^2 emitters; files synth_N_lg.*), for the fast tree's emitter leaf.
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORNELL = os.path.join(ROOT, "scenes", "scene_assets", "models", "CornellBox", "CornellBox-Original")
LO, HI = np.array([-0.99, 0.0, -1.04]), np.array([0.99, 1.99, 0.99])

XML = """<scenefile>
\t<cameradata>
\t\t<pos x="0" y="1" z="3.6"/>
\t\t<up x="0" y="1" z="0"/>
\t\t<focus x="0" y="1" z="0"/>
\t\t<heightangle v="45"/>
\t</cameradata>
\t<object type="tree" name="root">
\t\t<transblock>
\t\t\t<translate x="0" y="0" z="0"/>
\t\t\t<object type="primitive" name="mesh" filename="models/synth_{n}.obj">
\t\t\t</object>
\t\t</transblock>
\t</object>
</scenefile>
"""


LIGHT_QUAD = np.array([[-0.24, 1.98, 0.16], [-0.24, 1.98, -0.22], [0.23, 1.98, -0.22], [0.23, 1.98, 0.16]])


def _light_grid(g: int, nverts: int):
    """OBJ lines of the light quad (CornellBox-Original.obj's `f -4 -3 -2 -1`, corners LIGHT_QUAD)
    as g x g cells of two triangles with the quad's winding; vertex numbers from nverts + 1."""
    a, b, c, d = LIGHT_QUAD
    vs, fs = [], []
    for i in range(g + 1):
        for j in range(g + 1):
            u, w = i / g, j / g
            vs.append((1 - u) * ((1 - w) * a + w * b) + u * ((1 - w) * d + w * c))
    num = lambda i, j: nverts + 1 + i * (g + 1) + j  # noqa: E731
    for i in range(g):
        for j in range(g):
            fs.append("f %d %d %d" % (num(i, j), num(i, j + 1), num(i + 1, j + 1)))
            fs.append("f %d %d %d" % (num(i, j), num(i + 1, j + 1), num(i + 1, j)))
    return ["\n".join("v %.6f %.6f %.6f" % tuple(p) for p in vs), "g light", "usemtl light", "\n".join(fs)]


def write(n: int, out_root: str, light_grid: int = 1) -> str:
    assets = os.path.join(out_root, "scene_assets")
    os.makedirs(os.path.join(assets, "models"), exist_ok=True)
    with open(CORNELL + ".obj") as f:
        base = f.read()
    tag = f"{n}_l{light_grid}" if light_grid > 1 else f"{n}"
    if light_grid > 1:  # the light's one quad face goes; its grid is appended after the random triangles
        cut = base.rindex("f -4 -3 -2 -1")
        base = base[:cut] + base[cut + len("f -4 -3 -2 -1"):]
    with open(CORNELL + ".mtl") as f:
        mtl = f.read()
    m = max(0, n - 36)
    rng = np.random.default_rng(1234)
    c = rng.uniform(LO, HI, size=(m, 3))
    s = 1.2 * max(n, 1) ** (-1.0 / 3.0)
    v = c[:, None, :] + rng.uniform(-s, s, size=(m, 3, 3))
    lines = [base.rstrip("\n"), "", "## synthetic triangles", "usemtl synth"]
    if m:
        lines.append("\n".join("v %.6f %.6f %.6f" % tuple(p) for p in v.reshape(-1, 3)))
        # relative indices: each face is the three vertices just written before it... absolute is simpler
        # vertex lines "v x y z" or "v<TAB>x ..." (the light's; round 4 counted only the first
        # form, 24 of 72, so 16 random faces took Cornell vertices: fixed in round 5)
        nbase = len(re.findall(r"^v\s", base, re.M))
        idx = nbase + 1 + 3 * np.arange(m)
        lines.append("\n".join("f %d %d %d" % (i, i + 1, i + 2) for i in idx))
    if light_grid > 1:
        nverts = len(re.findall(r"^v\s", base, re.M)) + 3 * m
        lines += _light_grid(light_grid, nverts)
    with open(os.path.join(assets, "models", f"synth_{tag}.obj"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(assets, "models", f"synth_{tag}.mtl"), "w") as f:
        f.write(mtl.rstrip("\n") + "\n\nnewmtl synth\n  Ns 10.0000\n  Ni 1.0000\n  illum 2\n  Ka 0.5 0.5 0.5\n"
                "  Kd 0.5 0.5 0.5\n  Ks 0 0 0\n  Ke 0 0 0\n")
    xml = os.path.join(assets, f"synth_{tag}.xml")
    with open(xml, "w") as f:
        f.write(XML.format(n=tag))
    return xml


if __name__ == "__main__":
    print(write(int(sys.argv[1]), sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1))
