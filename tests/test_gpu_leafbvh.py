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
