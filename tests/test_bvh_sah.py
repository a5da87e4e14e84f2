"""The fast tree (pt_bvh_build_sah, csrc/pt_bvh.cpp; SURVEY.md §8(f) row 2's flagged mode) and the
synthetic sweep scenes (scripts/synth_scene.py; BASELINE.json north_star) — CPU only.

The SAH tree gives up the reference's topology (src/ts-util/bvh.ts:25-187 duplicates triangles that
straddle a split; this builder puts each in one leaf), but it must still be a valid tree in the
reference's packed layout (src/packer.ts:83-137) for the unchanged traversal
(src/wgsl-util/intersection-logic.wgsl:1-215) to find every closest hit the oracle finds:
  * every input triangle record (i0, i1, i2, material) in exactly one leaf;
  * leaves of at most kSahMaxLeaf = 8 entries, except at the depth cap (kSahMaxDepth = 28, root 1)
    and the emitter leaf of pt_bvh_build_sah2 (all flagged triangles in one leaf under the root);
  * every child box (the parent's [o+5..10] / [o+11..16]) contains the f32 vertices of every
    triangle below that child, and the outer bounds [0..5] contain all of them;
  * every non-empty child box has a positive extent on every axis (ray-bbox-intersection.wgsl's
    `tmax > max(tmin, 0)` never enters a flat box; the builder pads by one f32 ulp);
  * pre-order layout: an internal node's left child follows it at o + 17 (packer.ts:112).
The GPU renders on these buffers are compared with the oracle bit for bit in
tests/test_gpu_fast_trees.py.
"""
import hashlib
import os
import sys
import tempfile

import numpy as np
import pytest

import pt_amd
import scene_oracle as so
from conftest import ALL_SCENES, ROOT, SCENES

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import synth_scene  # noqa: E402

K_MAX_LEAF, K_MAX_DEPTH = 8, 28


def walk_packed(bvh):
    """Leaves of a packed BVH: list of (entries [n, 4] int, box lo, box hi, depth) — the box is the
    one the leaf's parent stores for it — and the internal nodes' (box lo, box hi, subtree leaves)."""
    leaves, inner = [], []

    def child_box(o, side):
        b = bvh[o + 5 + 6 * side: o + 11 + 6 * side]
        return b[:3], b[3:]

    def visit(o, lo, hi, depth):
        assert bvh[o] in (0.0, 1.0)
        if bvh[o] == 1.0:
            n = int(bvh[o + 4])
            assert n % 4 == 0 and bvh[o + 2] == -1 and bvh[o + 3] == -1
            leaves.append((bvh[o + 17: o + 17 + n].reshape(-1, 4).astype(np.int64), lo, hi, depth))
            return [len(leaves) - 1]
        assert bvh[o + 4] == -2 and int(bvh[o + 2]) == o + 17  # pre-order: left child right after
        below = []
        for side in (0, 1):
            clo, chi = child_box(o, side)
            below += visit(int(bvh[o + 2 + side]), clo, chi, depth + 1)
        inner.append((lo, hi, below))
        return below

    visit(6, bvh[0:3], bvh[3:6], 1)
    return leaves, inner


def check_sah(verts64, recs, bvh, emitter_leaf=False):
    leaves, inner = walk_packed(bvh)
    first_leaf_free = emitter_leaf and bvh[int(bvh[6 + 2])] == 1.0  # the root's left child, a leaf
    v32 = verts64.astype(np.float32)
    got = np.concatenate([e for e, _, _, _ in leaves])
    # every triangle record in exactly one leaf
    key = lambda a: np.sort(a.view([("", a.dtype)] * 4).reshape(-1))  # noqa: E731
    assert got.shape == recs.shape
    assert np.array_equal(key(np.ascontiguousarray(got)), key(np.ascontiguousarray(recs.astype(np.int64))))
    for i, (e, lo, hi, depth) in enumerate(leaves):
        assert len(e) <= K_MAX_LEAF or depth >= K_MAX_DEPTH or (i == 0 and first_leaf_free), (len(e), depth)
        if len(e):
            p = v32[e[:, :3].reshape(-1) - 1]
            assert np.all(p >= lo) and np.all(p <= hi), "a leaf's box must contain its triangles"
            # positive extent on every axis: the slab test never enters a zero-thickness box
            assert np.all(lo < hi), "a leaf box must not be flat (coplanar axis-aligned triangles)"
    for lo, hi, below in inner:
        e = np.concatenate([leaves[i][0] for i in below])
        if len(e):
            p = v32[e[:, :3].reshape(-1) - 1]
            assert np.all(p >= lo) and np.all(p <= hi), "an internal box must contain its subtree"
    assert np.all(v32 >= bvh[0:3]) and np.all(v32 <= bvh[3:6])
    return leaves


def scene_inputs(xml_path, assets):
    with open(xml_path) as f:
        _, prims = so.load_scene_xml(f.read())
    p = prims[0]
    path = os.path.join(assets, p["path"].lstrip("/").split("/", 1)[1])
    obj = open(path).read()
    mtl = open(path[:-3] + "mtl").read() if os.path.exists(path[:-3] + "mtl") else ""
    g = so.parse_obj(obj, mtl, p["ctm"])
    recs = []
    for mat_i, o in enumerate(g["objects"]):
        ind = o["indices"]
        for i in range(0, len(ind), 3):
            recs.append([int(ind[i]), int(ind[i + 1]), int(ind[i + 2]), mat_i])
    return np.array(g["vertices"], np.float64).reshape(-1, 3), np.array(recs, np.int32)


def emitter_flags(xml_path, assets):
    """Per material id: sum(Ke) > 0 (program-raymarch.wgsl:136), as the Node host flags them."""
    with open(xml_path) as f:
        _, prims = so.load_scene_xml(f.read())
    p = prims[0]
    path = os.path.join(assets, p["path"].lstrip("/").split("/", 1)[1])
    mtl = open(path[:-3] + "mtl").read() if os.path.exists(path[:-3] + "mtl") else ""
    g = so.parse_obj(open(path).read(), mtl, p["ctm"])
    return np.array([1 if sum(o["material"]["Ke"]) > 0 else 0 for o in g["objects"]], np.uint8)


def check_isolated(verts, recs, flags):
    """pt_bvh_build_sah2: the emitters' triangles in the root's left child as ONE leaf however many
    they are (a leaf child of the root is never pruned, intersection-logic.wgsl:47-176), the rest on
    the right; still a valid SAH tree over all triangles."""
    bvh = pt_amd.bvh_build(verts, recs, sah=True, isolate=flags)
    check_sah(verts, recs, bvh, emitter_leaf=True)
    lit = recs[flags[recs[:, 3]] != 0]
    left = int(bvh[6 + 2])
    if 0 < len(lit) < len(recs):
        assert bvh[left] == 1.0, "the emitters form one leaf under the root"
        got = bvh[left + 17: left + 17 + int(bvh[left + 4])].reshape(-1, 4).astype(np.int64)
        assert sorted(map(tuple, got)) == sorted(map(tuple, lit.astype(np.int64)))
    return bvh


@pytest.mark.parametrize("scene", ALL_SCENES)
def test_sah_emitters_under_the_root(scene):
    assets = os.path.join(SCENES, "scene_assets")
    xml = os.path.join(assets, scene + ".xml")
    verts, recs = scene_inputs(xml, assets)
    flags = emitter_flags(xml, assets)
    assert flags.any()  # every scene has its light
    check_isolated(verts, recs, flags)
    # no flags: pt_bvh_build_sah itself
    assert np.array_equal(pt_amd.bvh_build(verts, recs, sah=True, isolate=np.zeros_like(flags)).view(np.uint32),
                          pt_amd.bvh_build(verts, recs, sah=True).view(np.uint32))


@pytest.mark.parametrize("n", [1000, 12500])
def test_sah_emitters_under_the_root_synthetic(n, tmp_path):
    xml = synth_scene.write(n, str(tmp_path))
    assets = os.path.join(str(tmp_path), "scene_assets")
    verts, recs = scene_inputs(xml, assets)
    check_isolated(verts, recs, emitter_flags(xml, assets))


def test_sah_many_emitters_one_leaf():
    """A finely meshed area light (a quad split into 2 x 12 x 12 = 288 emissive triangles) above a
    floor of 200 triangles: all 288 in the one leaf under the root (advisor r04: round 4 built them
    an SAH subtree, whose internal nodes the exit-distance pruning can skip)."""
    g = 12
    xs = np.linspace(-0.25, 0.25, g + 1)
    lv = np.array([[x, 1.98, z] for z in xs for x in xs], np.float64)
    idx = lambda i, j: i * (g + 1) + j + 1  # noqa: E731
    light = [[idx(i, j), idx(i, j + 1), idx(i + 1, j), 1] for i in range(g) for j in range(g)]
    light += [[idx(i, j + 1), idx(i + 1, j + 1), idx(i + 1, j), 1] for i in range(g) for j in range(g)]
    rng = np.random.default_rng(3)
    fl = rng.uniform(-1, 1, (200, 3, 3)) * [1, 0.01, 1]
    verts = np.concatenate([lv, fl.reshape(-1, 3)])
    base = len(lv)
    floor = [[base + 3 * k + 1, base + 3 * k + 2, base + 3 * k + 3, 0] for k in range(200)]
    recs = np.array(light + floor, np.int32)
    flags = np.array([0, 1], np.uint8)
    bvh = check_isolated(verts, recs, flags)
    left = int(bvh[6 + 2])
    assert int(bvh[left + 4]) // 4 == 288


def test_node_sah_pack_isolates_emitters(tmp_path):
    """The Node host's --bvh sah packs through pt_bvh_build_sah2 with the emitter flags."""
    from conftest import pack_with_node
    assets = os.path.join(SCENES, "scene_assets")
    xml = os.path.join(assets, "CornellBox-Glossy.xml")
    p = pack_with_node(xml, str(tmp_path / "p"), "--bvh", "sah")
    verts, recs = scene_inputs(xml, assets)
    want = pt_amd.bvh_build(verts, recs, sah=True, isolate=emitter_flags(xml, assets))
    assert np.array_equal(p.bvh_data.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("scene", ALL_SCENES)
def test_sah_tree_structure_reference_scenes(scene):
    assets = os.path.join(SCENES, "scene_assets")
    verts, recs = scene_inputs(os.path.join(assets, scene + ".xml"), assets)
    leaves = check_sah(verts, recs, pt_amd.bvh_build(verts, recs, sah=True))
    # the reference's own tree holds every triangle at least once, some of them many times
    ref = pt_amd.bvh_build(verts, recs)
    assert sum(len(e) for e, _, _, _ in walk_packed(ref)[0]) >= len(recs) == sum(len(e) for e, _, _, _ in leaves)


@pytest.mark.parametrize("n", [36, 1000, 12500])
def test_sah_tree_structure_synthetic(n, tmp_path):
    xml = synth_scene.write(n, str(tmp_path))
    verts, recs = scene_inputs(xml, os.path.join(str(tmp_path), "scene_assets"))
    assert len(recs) == max(n, 36)
    check_sah(verts, recs, pt_amd.bvh_build(verts, recs, sah=True))


def test_sah_tree_degenerate_inputs():
    """Coincident centroids (the builder halves the list), a single triangle (the layout needs an
    internal root: two leaves), and triangles at geometrically shrinking scales (a deep,
    unbalanced tree)."""
    rng = np.random.default_rng(5)
    # 40 copies of one triangle: every centroid equal
    verts = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float64)
    recs = np.array([[1, 2, 3, k % 3] for k in range(40)], np.int32)
    check_sah(verts, recs, pt_amd.bvh_build(verts, recs, sah=True))
    check_sah(verts, recs[:1], pt_amd.bvh_build(verts, recs[:1], sah=True))
    # triangles at geometrically shrinking scales: a deep, unbalanced tree
    m = 400
    c = np.stack([2.0 ** -(np.arange(m) / 8.0), np.zeros(m), np.zeros(m)], 1)
    tri = c[:, None, :] + rng.uniform(-1e-3, 1e-3, (m, 3, 3)) * (2.0 ** -(np.arange(m) / 8.0))[:, None, None]
    verts = tri.reshape(-1, 3)
    recs = np.stack([3 * np.arange(m) + 1, 3 * np.arange(m) + 2, 3 * np.arange(m) + 3, np.zeros(m, int)], 1).astype(np.int32)
    leaves = check_sah(verts, recs, pt_amd.bvh_build(verts, recs, sah=True))
    assert max(d for _, _, _, d in leaves) <= K_MAX_DEPTH + 1


def test_sah_rejects_bad_indices():
    verts = np.zeros((3, 3), np.float64)
    with pytest.raises(pt_amd.PtError):
        pt_amd.bvh_build(verts, np.array([[1, 2, 4, 0]], np.int32), sah=True)
    with pytest.raises(pt_amd.PtError):
        pt_amd.bvh_build(verts, np.array([[0, 1, 2, 0]], np.int32), sah=True)


# ---------------------------------------------------------------------------------------------
# scripts/synth_scene.py: the sweep's scenes are a pure function of N (rng seed 1234)
# ---------------------------------------------------------------------------------------------
def _synth_digest(n, root):
    xml = synth_scene.write(n, root)
    h = hashlib.sha256()
    for f in (xml, os.path.join(root, "scene_assets", "models", f"synth_{n}.obj"),
              os.path.join(root, "scene_assets", "models", f"synth_{n}.mtl")):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


@pytest.mark.parametrize("n", [36, 1000, 12500])
def test_synth_scene_deterministic(n):
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        assert _synth_digest(n, a) == _synth_digest(n, b)


def test_synth_scene_contents():
    """N triangles: the Cornell box's 36 (walls, boxes, light: the light stays the only emitter)
    plus N - 36 random ones inside the box's bounds, edges ~1.2 N^(-1/3)."""
    with tempfile.TemporaryDirectory() as td:
        xml = synth_scene.write(1000, td)
        verts, recs = scene_inputs(xml, os.path.join(td, "scene_assets"))
        assert len(recs) == 1000
        extra = verts[recs[36:, :3].reshape(-1) - 1]
        s = 1.2 * 1000 ** (-1.0 / 3.0)
        assert np.all(extra >= synth_scene.LO - s) and np.all(extra <= synth_scene.HI + s)
        tri = extra.reshape(-1, 3, 3)
        edge = np.linalg.norm(tri[:, 1] - tri[:, 0], axis=1)
        assert 0.2 * s < np.median(edge) < 2.0 * s
