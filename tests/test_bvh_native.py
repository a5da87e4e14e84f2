"""Native BVH build (pt_bvh_build, csrc/pt_bvh.cpp) — CPU only.

The packed BVH is part of the parity contract (traversal order and exit-distance pruning depend
on its topology), so the C++ build must be byte-identical to the reference's JS build
(src/ts-util/bvh.ts + src/packer.ts), here checked against two independent restatements:
the Python oracle (oracle/scene_oracle.py, f64, numpy) and the Node host (node/lib/bvh.js).
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import pt_amd
import scene_oracle as so
from conftest import ALL_SCENES, PACK_JS, SCENES

XMLS = [os.path.join(SCENES, "scene_assets", s + ".xml") for s in ALL_SCENES]


def oracle_inputs(xml_path):
    """f64 vertices and (i0, i1, i2, mat) records of the first primitive, as index.ts builds them."""
    with open(xml_path) as f:
        _, prims = so.load_scene_xml(f.read())
    p = prims[0]
    path = os.path.join(SCENES, "scene_assets", p["path"].lstrip("/").split("/", 1)[1])
    obj = open(path).read()
    mtl = open(path[:-3] + "mtl").read() if os.path.exists(path[:-3] + "mtl") else ""
    g = so.parse_obj(obj, mtl, p["ctm"])
    recs = []
    for mat_i, o in enumerate(g["objects"]):
        ind = o["indices"]
        for i in range(0, len(ind), 3):
            recs.append([int(ind[i]), int(ind[i + 1]), int(ind[i + 2]), mat_i])
    return np.array(g["vertices"], np.float64).reshape(-1, 3), np.array(recs, np.int32), (obj, mtl, p["ctm"])


@pytest.mark.parametrize("xml", XMLS, ids=[os.path.basename(x)[:-4] for x in XMLS])
def test_native_bvh_equals_oracle(xml):
    verts, recs, (obj, mtl, ctm) = oracle_inputs(xml)
    native = pt_amd.bvh_build(verts, recs)
    ref = so.pack_primitive(obj, mtl, ctm).bvh_data.astype(np.float32)
    assert native.tobytes() == ref.tobytes()


@pytest.mark.parametrize("xml", XMLS, ids=[os.path.basename(x)[:-4] for x in XMLS])
def test_node_native_bvh_flag_equals_js_build(xml):
    with tempfile.TemporaryDirectory() as td:
        for flag, sub in (([], "js"), (["--native-bvh"], "native")):
            subprocess.run(["node", PACK_JS, xml, os.path.join(td, sub), *flag], check=True, capture_output=True)
        a = open(os.path.join(td, "js", "bvh_data.f32"), "rb").read()
        b = open(os.path.join(td, "native", "bvh_data.f32"), "rb").read()
    assert a == b and len(a) > 0


@pytest.mark.parametrize("n,seed", [(1, 0), (17, 1), (300, 2), (3000, 3)])
def test_native_bvh_random_meshes(n, seed):
    """Random soups (overlapping, degenerate-ish triangles, coincident coordinates) against the
    oracle's builder: exercises deep trees, the depth-16 cap and 'split separated nothing' leaves."""
    rng = np.random.default_rng(seed)
    nv = 3 * n
    centers = np.repeat(rng.uniform(-3, 3, (n, 3)), 3, axis=0)
    verts = np.round(centers + rng.uniform(-0.2, 0.2, (nv, 3)), 2)  # coincident coordinates are common
    verts[::7] = verts[0]                                           # and some shared far vertices
    recs = np.concatenate([np.arange(1, nv + 1, dtype=np.int32).reshape(-1, 3),
                           rng.integers(0, 4, (n, 1), dtype=np.int32)], axis=1)
    native = pt_amd.bvh_build(verts, recs)
    bmin, bmax = so.bounds_of_vec3(verts.tolist())
    tri = verts[recs[:, :3] - 1]
    root = so.build_bvh(tri.min(axis=1), tri.max(axis=1), bmin, bmax)
    ref = so.pack_bvh(root, bmin, bmax, recs.astype(np.float64)).astype(np.float32)
    assert native.tobytes() == ref.tobytes()


def test_native_bvh_rejects_bad_input():
    with pytest.raises(pt_amd.PtError):
        pt_amd.bvh_build(np.zeros((3, 3)), np.array([[1, 2, 4, 0]], np.int32))  # vertex index out of range
    with pytest.raises(pt_amd.PtError):
        pt_amd.bvh_build(np.zeros((3, 3)), np.array([[0, 1, 2, 0]], np.int32))  # 0 is not 1-based
