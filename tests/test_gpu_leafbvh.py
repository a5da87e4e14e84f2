"""Leaf chunks (csrc/pt_leafbvh.cpp, pt_device.h chunk_leaf): a big leaf's entries tested chunk by
chunk, skipping chunks that provably hold no hit below the bound, must end exactly where the
reference's sequential strict-< loop over all the leaf's entries ends — same entry, same t bits —
for every ray and closest-t-so-far — walked for one ray at a time (chunk_leaf) and by the walk that
the rays parked at one leaf share (chunk_leaf_multi, 16 interleaved lanes per walk).
pt_selftest_leaf runs them on the device for four ray
families, including rays grazing the entries' planes (where the triangle test's rounding, which
the skip rule bounds, is largest) and rays leaving the surfaces as the path tracer's bounces do.  Renders through the walk are checked against the oracle by
test_gpu_parity.py (the leaf variants, the boat frames) and test_gpu_config_bands.py (the boat
band at 1920x1080)."""
import numpy as np
import pytest

import pt_amd

pytestmark = pytest.mark.gpu

NRAYS = 1 << 15


def _check(s, label, nrays=NRAYS):
    leaves = s.leaf_bvhs()
    assert leaves, f"{label}: no leaf BVH"
    stats = []
    for li, (rec0, n, nodes) in enumerate(leaves):
        for mode in range(8):  # + 4: the walk several parked rays share (chunk_leaf_multi)
            out = s.selftest_leaf(li, mode, 1234 + 17 * li, nrays)
            bad = np.flatnonzero(np.any(out[:, :2] != out[:, 2:4], axis=1))
            assert bad.size == 0, (f"{label} leaf {li} ({n} entries) mode {mode}: {bad.size} rays differ, first "
                                   f"{out[bad[:4]].tolist()}")
            if mode < 4:
                hits = int((out[:, 0] >= 0).sum())
                stats.append((li, n, nodes, mode, hits, float(out[:, 4].mean()), float(out[:, 5].mean())))
    for li, n, nchunks, mode, hits, tests, opened in stats if len(stats) <= 64 else []:
        steps = -(-nchunks // 64) + 8 * -(-opened // 64)
        print(f"{label} leaf {li}: {n} entries {nchunks} chunks mode {mode}: {hits}/{nrays} taken, "
              f"{tests:.1f} tests, {opened:.1f} open chunks per ray: ~{steps:.0f} wave-steps "
              f"(cooperative turn: {-(-n // 64)})")
    if len(stats) > 64:
        print(f"{label}: {len(leaves)} leaves x 4 ray families, {nrays} rays each: identical")
    return stats


def test_leaf_walk_equals_loop_boat(packed, ptopts):
    ptopts.set("leaf_bvh", "64")
    p = packed["MedievalBoat"]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        stats = _check(s, "boat")
    # the 7327-entry leaf: chunk checks + open chunks take well under the cooperative turn's
    # n / 64 wave-steps (a regression guard on the grouping)
    big = [st for st in stats if st[1] > 7000]
    assert big and all(-(-st[2] // 64) + 8 * -(-st[6] // 64) < 0.7 * (st[1] / 64) for st in big), big


@pytest.mark.parametrize("scene", ["CornellBox", "CornellBox-Glossy", "CornellBox-Sphere"])
def test_leaf_walk_equals_loop_small_leaves(packed, ptopts, scene):
    """Every leaf of >= 2 entries with a leaf BVH: the Cornell boxes' axis-aligned walls give
    rays exactly parallel to an entry's plane and to a node's box faces."""
    ptopts.set("leaf_bvh", "2")
    p = packed[scene]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        _check(s, scene, nrays=1 << 13)


def test_leaf_bvh_option(packed, ptopts):
    p = packed["MedievalBoat"]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:  # default: leaves of >= 128 entries
        assert sorted(n for _, n, _ in s.leaf_bvhs()) == [132, 206, 219, 238, 275, 520, 7327]
    ptopts.set("leaf_bvh", "0")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        assert s.leaf_bvhs() == []
    ptopts.set("leaf_bvh", "1000")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        assert [n for _, n, _ in s.leaf_bvhs()] == [7327]


# ---------------------------------------------------------------------------------------------
# The leaf pass's own walks (pt_leafpass.hip: resolve_leaf, resolve_leaf_pairs with and without its
# second check) against the sequential strict-< loop, on the device, for the same four ray families
# — grazing rays included, where pass_box_skip's rounding slack (A', B' x 1.00001 rounded up, planes
# in t by FMA, the running best as a finite bound) is tightest (verdict r05: the rule had no targeted
# device test).  Every key must equal the loop's first entry of the smallest t and its t bits.
# ---------------------------------------------------------------------------------------------
PASS_METHODS = {0: "resolve_leaf, one ray per lane", 1: "resolve_leaf, 8 rays x 8 lanes",
                2: "pair walk, cone check only", 3: "pair walk + second check (entries' normals)"}


def _check_pass(s, label, nrays=NRAYS):
    """Every pre-resolvable leaf of the scene (the 8 largest), every method and ray family."""
    done = []
    b = 0
    while True:
        try:
            s.selftest_leaf(b, 16, 1, 64)
        except pt_amd.PtError:
            break  # past the last leaf
        for method, what in PASS_METHODS.items():
            for fam in range(4):
                try:
                    out = s.selftest_leaf(b, 16 + (method << 2 | fam), 4321 + 31 * b + fam, nrays)
                except pt_amd.PtError as e:
                    assert method >= 2 and "pass chunks" in str(e), e
                    break  # this leaf has no pass chunks (below option leaf_bvh)
                bad = np.flatnonzero(np.any(out[:, :2] != out[:, 2:4], axis=1))
                assert bad.size == 0, (f"{label} pre leaf {b} {what} family {fam}: {bad.size} of {nrays} rays "
                                       f"differ, first {out[bad[:4]].tolist()}")
                done.append((b, method, fam, int((out[:, 0] >= 0).sum())))
        b += 1
    print(f"{label}: {b} pre-resolvable leaves, {len(done)} (leaf, method, family) cases of {nrays} rays identical")
    return b, done


def test_leaf_pass_equals_loop_boat(packed, ptopts):
    p = packed["MedievalBoat"]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:  # default leaf_bvh: chunks on leaves >= 128
        nb, done = _check_pass(s, "boat")
    assert nb == 8
    # the pair walks ran on the chunked leaves (7 of the 8 have >= 128 entries), with rays that hit
    pairs = [d for d in done if d[1] >= 2]
    assert len({d[0] for d in pairs}) == 7 and all(d[3] > 0 for d in pairs if d[2] in (1, 2)), pairs


def test_leaf_pass_equals_loop_cornellbox2_all_meshes(ptopts, tmp_path):
    """CornellBox2 with every mesh (the box's walls around the boat), chunks on every leaf of >= 16
    entries, so the pass's walks meet the walls' axis-aligned planes as well as the boat's."""
    import os
    from conftest import SCENES, pack_with_node
    p = pack_with_node(os.path.join(SCENES, "scene_assets", "CornellBox2.xml"), str(tmp_path / "cb2"),
                       "--all-meshes", "--native-bvh")
    ptopts.set("leaf_bvh", "16")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        nb, done = _check_pass(s, "CornellBox2 all meshes")
    assert nb == 8 and len({d[0] for d in done if d[1] >= 2}) == 8, done
