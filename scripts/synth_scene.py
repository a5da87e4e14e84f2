#!/usr/bin/env python3
"""Synthetic Cornell-box-sized scenes for the BVH-size sweep (BASELINE.json
north_star "Cornell-box-sized synthetic BVHs"): N triangles in the Cornell box's bounds — the
box itself (CornellBox-Original.obj: walls, two boxes, the light; 36 triangles) plus N - 36
random triangles, centres uniform in the box, edges ~1.2 N^(-1/3), from
numpy.random.default_rng(1234) — under CornellBox.xml's camera.  Written as OBJ + MTL + scene
XML in the reference's formats, so the product's Node host packs them like any scene.

usage: synth_scene.py N OUT_ROOT   ->  OUT_ROOT/scene_assets/synth_N.xml (+ models/synth_N.obj/.mtl)
"""
import os
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


def write(n: int, out_root: str) -> str:
    assets = os.path.join(out_root, "scene_assets")
    os.makedirs(os.path.join(assets, "models"), exist_ok=True)
    with open(CORNELL + ".obj") as f:
        base = f.read()
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
        nbase = base.count("\nv ") + (1 if base.startswith("v ") else 0)
        idx = nbase + 1 + 3 * np.arange(m)
        lines.append("\n".join("f %d %d %d" % (i, i + 1, i + 2) for i in idx))
    with open(os.path.join(assets, "models", f"synth_{n}.obj"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(assets, "models", f"synth_{n}.mtl"), "w") as f:
        f.write(mtl.rstrip("\n") + "\n\nnewmtl synth\n  Ns 10.0000\n  Ni 1.0000\n  illum 2\n  Ka 0.5 0.5 0.5\n"
                "  Kd 0.5 0.5 0.5\n  Ks 0 0 0\n  Ke 0 0 0\n")
    xml = os.path.join(assets, f"synth_{n}.xml")
    with open(xml, "w") as f:
        f.write(XML.format(n=n))
    return xml


if __name__ == "__main__":
    print(write(int(sys.argv[1]), sys.argv[2]))
