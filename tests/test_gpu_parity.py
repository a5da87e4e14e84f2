"""GPU parity: the HIP core (through the C ABI) against the CPU oracle on identical inputs.

Bar: bit-exact.  The numeric contract (pt_math.h / oracle/pt_oracle.c header) pins every
implementation-defined WGSL operation, so per-pixel radiance, accumulators and work counters
must match the oracle exactly, not within a tolerance.
"""
import numpy as np
import pytest

import oracle
import pt_amd

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(1234)
# kernel variants (environment read by the C ABI on every call)
KERNELS = {
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
    "mega_lean2_lds": {"PT_KERNEL": "mega", "PT_TRAV": "lean2"},
    "mega_lean_fastrcp": {"PT_KERNEL": "mega", "PT_TRAV": "lean", "PT_FASTRCP": "1"},
    "wavefront_lean4_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean4", "PT_FASTRCP": "1"},
    "wavefront_lean8_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_FASTRCP": "1"},
    "wavefront_lean8_div": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean8", "PT_FASTRCP": "0"},
    "wavefront_lean16_fastrcp": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_FASTRCP": "1"},
    # one trace block (8 waves): long per-wave window sequences, hit-ring wrap-around, many
    # write-backs — the multi-window path full-size renders take, at oracle-checkable sizes
    "wavefront_1block": {"PT_KERNEL": "wavefront", "PT_WF_TRACE_BLOCKS": "1"},
    "wavefront_lean16_majority_div": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_NODE_BIAS": "1",
                                      "PT_FASTRCP": "0"},
    "mega_lean4_majority": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_NODE_BIAS": "1"},
    "wavefront_single_stream": {"PT_KERNEL": "wavefront", "PT_DUAL": "0"},
    "wavefront_dual_1block": {"PT_KERNEL": "wavefront", "PT_DUAL": "1", "PT_WF_TRACE_BLOCKS": "1"},
    "wavefront_nomailbox": {"PT_KERNEL": "wavefront", "PT_MAILBOX": "0"},
    "wavefront_mailbox_rev": {"PT_KERNEL": "wavefront", "PT_MB_UID_ORDER": "reverse"},
    "wavefront_mb_lean16_rev": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean16", "PT_MB_UID_ORDER": "reverse"},
    "wavefront_bf_nofuse": {"PT_KERNEL": "wavefront", "PT_FUSE": "0"},
    "wavefront_4parts": {"PT_KERNEL": "wavefront", "PT_PARTS": "4"},
    "wavefront_3parts_nofuse": {"PT_KERNEL": "wavefront", "PT_PARTS": "3", "PT_FUSE": "0"},
    "wavefront_bf_step_3blocks": {"PT_KERNEL": "wavefront", "PT_WF_TRACE_BLOCKS": "3"},
    "wavefront_bf_nofuse_1block": {"PT_KERNEL": "wavefront", "PT_FUSE": "0", "PT_WF_TRACE_BLOCKS": "1"},
    "wavefront_bf_global_noslots": {"PT_KERNEL": "wavefront", "PT_LDS": "0", "PT_BF_SLOTS": "0"},
    "wavefront_bf_2slots_div": {"PT_KERNEL": "wavefront", "PT_BF_SLOTS": "2", "PT_FASTRCP": "0"},
    "wavefront_mailbox_lean4_global": {"PT_KERNEL": "wavefront", "PT_TRAV": "lean4", "PT_LDS": "0"},
    "wavefront_3blocks_flat1": {"PT_KERNEL": "wavefront", "PT_TRAV": "flat1", "PT_WF_TRACE_BLOCKS": "3"},
    # camera paths made in the first fused launch (GEN) or by k_wf_generate
    "wavefront_gen": {"PT_KERNEL": "wavefront", "PT_FUSE_GEN": "1"},
    "wavefront_nogen": {"PT_KERNEL": "wavefront", "PT_FUSE_GEN": "0"},
    # big leaves tested by the whole wave (default from 128 entries: the boat; forced onto small leaves
    # here so every scene runs many cooperative turns), and off
    "wavefront_big8": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "8", "PT_MAILBOX": "0"},
    "wavefront_big4_lean8_div": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "4", "PT_TRAV": "lean8", "PT_FASTRCP": "0",
                                 "PT_MAILBOX": "0"},
    "wavefront_nobig": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "0"},
    "mega_big8": {"PT_KERNEL": "mega", "PT_BIG_LEAF": "8"},
    "mega_nobig": {"PT_KERNEL": "mega", "PT_BIG_LEAF": "0"},
    # brute-force replay: the stack walk instead of the stackless pre-order walk (the default)
    "wavefront_bf_stack_replay": {"PT_KERNEL": "wavefront", "PT_BF_STACKLESS": "0"},
    # traversal pipeline: survivors grouped by 8 / 64 / 512 coherence keys per shade block (queue order only; 512 is the default)
    "wavefront_sort8": {"PT_KERNEL": "wavefront", "PT_SORT": "8"},
    # the traversal kernel's hit ring forced to 128 / 256 entries (default: 256 when it costs no block)
    "wavefront_ring128": {"PT_KERNEL": "wavefront", "PT_TRACE_RING": "128", "PT_MAILBOX": "0"},
    "wavefront_ring256_1block": {"PT_KERNEL": "wavefront", "PT_TRACE_RING": "256", "PT_MAILBOX": "0",
                                 "PT_WF_TRACE_BLOCKS": "1"},
    # camera batches dealt to the fused kernel's regions by a permutation (option region_perm), with
    # the camera paths made by the first fused launch or by k_wf_generate, and on 3 blocks (24 regions)
    "wavefront_region_perm": {"PT_KERNEL": "wavefront", "PT_REGION_PERM": "1"},
    "wavefront_region_perm_nofusegen_3blocks": {"PT_KERNEL": "wavefront", "PT_REGION_PERM": "1", "PT_FUSE_GEN": "0",
                                                "PT_WF_TRACE_BLOCKS": "3"},
    # short queues in windows below 32 entries (option trace_sparse=n; default 4): n = 1 on the full
    # grid (windows of 1..4 entries), on 3 blocks (the last depths only); n = 8 on one block; off
    "wavefront_trace_sparse_off": {"PT_KERNEL": "wavefront", "PT_TRACE_SPARSE": "0", "PT_MAILBOX": "0"},
    "wavefront_trace_sparse": {"PT_KERNEL": "wavefront", "PT_TRACE_SPARSE": "1", "PT_MAILBOX": "0"},
    "wavefront_trace_sparse_3blocks": {"PT_KERNEL": "wavefront", "PT_TRACE_SPARSE": "1", "PT_MAILBOX": "0",
                                       "PT_WF_TRACE_BLOCKS": "3"},
    "wavefront_trace_sparse8_1block": {"PT_KERNEL": "wavefront", "PT_TRACE_SPARSE": "8", "PT_MAILBOX": "0",
                                       "PT_WF_TRACE_BLOCKS": "1"},
    # leaf BVHs (option leaf_bvh, read at scene creation; default off): on every leaf of >= 4 / >= 2
    # entries (every scene, Cornell boxes with mailbox=0; the boat's 7327-entry leaf too), and on the
    # megakernel's big-leaf path
    "wavefront_leaf4": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "4", "PT_MAILBOX": "0"},
    "wavefront_leaf2_div_1block": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "2", "PT_MAILBOX": "0", "PT_FASTRCP": "0",
                                   "PT_WF_TRACE_BLOCKS": "1"},
    "mega_leaf4_lean4": {"PT_KERNEL": "mega", "PT_TRAV": "lean4", "PT_FASTRCP": "1", "PT_LEAF_BVH": "4",
                         "PT_MAILBOX": "0"},
    "wavefront_nosort_nomailbox": {"PT_KERNEL": "wavefront", "PT_SORT": "0", "PT_MAILBOX": "0"},
    "wavefront_sort64": {"PT_KERNEL": "wavefront", "PT_SORT": "64"},
    "wavefront_sort512_nomailbox": {"PT_KERNEL": "wavefront", "PT_SORT": "512", "PT_MAILBOX": "0"},
    "wavefront_sort64_nomailbox_1block": {"PT_KERNEL": "wavefront", "PT_SORT": "64", "PT_MAILBOX": "0",
                                          "PT_WF_TRACE_BLOCKS": "1"},
    # the traversal kernel's leaf turns pooled over the wave (lean_leaf_pool; on by default) and not (each lane walks its own pair, lean_leaf_loop), and pooled on one block
    "wavefront_nopool_nomailbox": {"PT_KERNEL": "wavefront", "PT_LEAF_POOL": "0", "PT_MAILBOX": "0"},
    "wavefront_pool_nomailbox_1block": {"PT_KERNEL": "wavefront", "PT_LEAF_POOL": "1", "PT_MAILBOX": "0",
                                        "PT_WF_TRACE_BLOCKS": "1"},
    # runs of 2 entries (the default where leaves reference >= 32 Ki triangles and no leaf is big)
    "wavefront_pool_run2_nomailbox": {"PT_KERNEL": "wavefront", "PT_POOL_RUN": "2", "PT_MAILBOX": "0"},
    "wavefront_pool_run2_1block": {"PT_KERNEL": "wavefront", "PT_POOL_RUN": "2", "PT_WF_TRACE_BLOCKS": "1"},
    # the traversal kernel on one block with the big-leaf turns forced onto small leaves
    "wavefront_big4_1block": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "4", "PT_MAILBOX": "0",
                              "PT_WF_TRACE_BLOCKS": "1"},
    # big leaves resolved before the traversal (k_wf_leafpass; AUTO runs it where the scene's probe
    # finds the leaves' box filters predict their visits — the variants above with big_leaf / leaf_bvh
    # forced small take that choice on the 8 largest leaves of every scene; here leaf_pre=1 forces
    # it): on one block (each wave's LDS rings wrap and flush partial batches), and off (leaf_pre=0)
    # — the cooperative turns and chunk walks inside k_wf_trace
    "wavefront_big8_leafpass_1block": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "8", "PT_MAILBOX": "0",
                                       "PT_LEAF_BLOCKS": "1", "PT_LEAF_PRE": "1"},
    "wavefront_big8_nopre": {"PT_KERNEL": "wavefront", "PT_BIG_LEAF": "8", "PT_MAILBOX": "0", "PT_LEAF_PRE": "0"},
    "wavefront_leaf4_nopre": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "4", "PT_MAILBOX": "0", "PT_LEAF_PRE": "0"},
    "wavefront_leaf2_div_nopre_1block": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "2", "PT_MAILBOX": "0",
                                         "PT_FASTRCP": "0", "PT_LEAF_PRE": "0", "PT_WF_TRACE_BLOCKS": "1"},
    # the leaf pass with leaf BVHs forced small (the 8 largest leaves of every scene), on one block;
    # its pair walk of the chunked leaves at every batch size (option leaf_pairs=2; by default only
    # full batches of 64 rays take it) and never (leaf_pairs=0)
    "wavefront_leaf2_div_leafpass_1block": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "2", "PT_MAILBOX": "0",
                                            "PT_FASTRCP": "0", "PT_LEAF_BLOCKS": "1", "PT_LEAF_PRE": "1"},
    "wavefront_leaf4_pairs_always": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "4", "PT_MAILBOX": "0", "PT_LEAF_PAIRS": "2",
                                     "PT_LEAF_PRE": "1"},
    "wavefront_leaf2_pairs_always_1block": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "2", "PT_MAILBOX": "0",
                                            "PT_LEAF_PAIRS": "2", "PT_LEAF_BLOCKS": "1", "PT_LEAF_PRE": "1"},
    "wavefront_leaf4_nopairs": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "4", "PT_MAILBOX": "0", "PT_LEAF_PAIRS": "0",
                                "PT_LEAF_PRE": "1"},
    # the pair walk without its second check of the open chunks by the entries' own normals
    # (option leaf_refine=0), at every batch size
    "wavefront_leaf4_pairs_norefine": {"PT_KERNEL": "wavefront", "PT_LEAF_BVH": "4", "PT_MAILBOX": "0",
                                       "PT_LEAF_PAIRS": "2", "PT_LEAF_PRE": "1", "PT_LEAF_REFINE": "0"},
    # leaf remainders (option leaf_skip, on by default on scenes without mailbox: every variant above
    # that keeps big_leaf >= 64 runs them on Glossy, the sphere and the boat) off, and on with the
    # lane-per-pair leaf turns, the megakernel and one block
    "wavefront_noskip": {"PT_KERNEL": "wavefront", "PT_LEAF_SKIP": "0"},
    "wavefront_skip_nopool_lean4": {"PT_KERNEL": "wavefront", "PT_LEAF_SKIP": "1", "PT_LEAF_POOL": "0", "PT_TRAV": "lean4"},
    "mega_skip_lean16": {"PT_KERNEL": "mega", "PT_LEAF_SKIP": "1", "PT_TRAV": "lean16"},
    "wavefront_skip_1block_run2": {"PT_KERNEL": "wavefront", "PT_LEAF_SKIP": "1", "PT_WF_TRACE_BLOCKS": "1",
                                   "PT_POOL_RUN": "2"},
    # runs of 4 (the default only on trees with big leaves since round 6)
    "wavefront_run4": {"PT_KERNEL": "wavefront", "PT_POOL_RUN": "4", "PT_MAILBOX": "0"},
    # node steps per node turn of the lean traversal (option node_steps; wavefront default 4, megakernel 1)
    "wavefront_nodesteps1": {"PT_KERNEL": "wavefront", "PT_NODE_STEPS": "1", "PT_MAILBOX": "0"},
    "wavefront_nodesteps2": {"PT_KERNEL": "wavefront", "PT_NODE_STEPS": "2", "PT_MAILBOX": "0"},
    "wavefront_nodesteps8_nopool": {"PT_KERNEL": "wavefront", "PT_NODE_STEPS": "8", "PT_MAILBOX": "0",
                                    "PT_LEAF_POOL": "0"},
    "mega_nodesteps4": {"PT_KERNEL": "mega", "PT_NODE_STEPS": "4"},
    # streaming regeneration in the fused kernel (option regen = camera batches per region admitted by
    # each extension launch; small grids so that the regions hold many camera batches)
    "wavefront_regen8_1block": {"PT_KERNEL": "wavefront", "PT_REGEN": "8", "PT_WF_TRACE_BLOCKS": "1"},
    "wavefront_regen3_2blocks_noperm": {"PT_KERNEL": "wavefront", "PT_REGEN": "3", "PT_WF_TRACE_BLOCKS": "2",
                                        "PT_REGION_PERM": "0"},
    "wavefront_regen1_1block_1part": {"PT_KERNEL": "wavefront", "PT_REGEN": "1", "PT_WF_TRACE_BLOCKS": "1",
                                      "PT_PARTS": "1"},
    "wavefront_regen64": {"PT_KERNEL": "wavefront", "PT_REGEN": "64"},
    "wavefront_nodesteps3_big8_1block": {"PT_KERNEL": "wavefront", "PT_NODE_STEPS": "3", "PT_MAILBOX": "0",
                                         "PT_BIG_LEAF": "8", "PT_WF_TRACE_BLOCKS": "1"},
    "mega_nodesteps2_lean4": {"PT_KERNEL": "mega", "PT_NODE_STEPS": "2", "PT_TRAV": "lean4"},
}


ENV_KEYS = ("PT_KERNEL", "PT_TRAV", "PT_LDS", "PT_FASTRCP", "PT_WF_TRACE_BLOCKS", "PT_NODE_BIAS",
            "PT_DUAL", "PT_MAILBOX", "PT_MB_UID_ORDER", "PT_BF", "PT_BF_SLOTS", "PT_FUSE", "PT_PARTS",
            "PT_FUSE_GEN", "PT_WF_PATHS", "PT_BIG_LEAF", "PT_TRACE_WATCHDOG", "PT_REDUCE", "PT_BF_STACKLESS",
            "PT_SORT", "PT_TRACE_SPARSE", "PT_LEAF_BVH", "PT_LEAF_WALK", "PT_REGION_PERM", "PT_TRACE_RING", "PT_LEAF_POOL", "PT_REGEN",
            "PT_POOL_RUN", "PT_LEAF_PRE", "PT_LEAF_BLOCKS", "PT_LEAF_PAIRS",
            "PT_LEAF_REFINE", "PT_LEAF_SKIP", "PT_NODE_STEPS")


@pytest.fixture(params=list(KERNELS))
def kernel(request, ptopts):
    """Every kernel variant must give the same bits."""
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    for k, v in KERNELS[request.param].items():
        ptopts.set(k, v)
    return request.param


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def same_bits(a, b):
    """Bitwise equality, treating every NaN as equal to every NaN."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((bits(a) == bits(b)) | both_nan))


def mismatch_report(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    bad = np.argwhere(~((bits(a) == bits(b)) | (np.isnan(a) & np.isnan(b))))
    return f"{len(bad)} mismatches; first {bad[:5].tolist()}: gpu {a[tuple(bad[0])] if len(bad) else None} " \
           f"oracle {b[tuple(bad[0])] if len(bad) else None}"


# ---------------------------------------------------------------------------------------------
# pinned math on device == oracle restatement
# ---------------------------------------------------------------------------------------------
def _inputs(fn, n=4096):
    if fn in ("sin", "cos", "tan"):
        x = np.concatenate([RNG.uniform(0, 2 * np.pi, n), RNG.uniform(-20, 20, n // 4), [0.0, -0.0, 0.785398, 1e-30]])
    elif fn == "acos":
        x = np.concatenate([RNG.uniform(0, 1, n), RNG.uniform(-1, 1, n // 4), [0.0, 0.5, 1.0, -1.0, -0.5]])
    elif fn == "log2":
        x = np.concatenate([RNG.uniform(0, 1, n), 10 ** RNG.uniform(-44, 30, n // 4), [1.0, 2.0, 0.0, 1e-45]])
    elif fn == "exp2":
        x = np.concatenate([RNG.uniform(-130, 130, n), RNG.uniform(-1, 1, n // 4), [0.0, -127.0, 127.0, -126.5]])
    else:
        x = RNG.uniform(0, 1, n)
    return x.astype(np.float32)


@pytest.mark.parametrize("fn", ["sin", "cos", "tan", "acos", "log2", "exp2"])
def test_math_unary_bitexact(fn):
    x = _inputs(fn)
    gpu = pt_amd.selftest_math(fn, x)
    ref = oracle.math_fn(fn, x)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)


def test_math_pow_bitexact():
    x = np.concatenate([RNG.uniform(0, 1, 4096), [0.0, 1.0, 1e-3, 0.999]]).astype(np.float32)
    y = np.concatenate([RNG.choice([5.0, 10.0, 40.0, 200.0, 1000.0], 4096), [40, 40, 40, 1000]]).astype(np.float32)
    gpu = pt_amd.selftest_math("pow", x, y)
    ref = np.array([oracle.lib().po_powf(float(a), float(b)) for a, b in zip(x, y)], np.float32)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)


def test_math_div_sqrt_correctly_rounded():
    a = (RNG.standard_normal(8192) * 10 ** RNG.uniform(-30, 30, 8192)).astype(np.float32)
    b = (RNG.standard_normal(8192) * 10 ** RNG.uniform(-30, 30, 8192)).astype(np.float32)
    assert same_bits(pt_amd.selftest_math("div", a, b), a / b)
    s = np.abs(a)
    assert same_bits(pt_amd.selftest_math("sqrt", s), np.sqrt(s))


def test_math_minmax_nan_handling():
    nan = np.float32(np.nan)
    a = np.array([nan, 1.0, nan, -0.0, 3.0], np.float32)
    b = np.array([2.0, nan, nan, 0.0, -3.0], np.float32)
    mn = pt_amd.selftest_math("min", a, b)
    mx = pt_amd.selftest_math("max", a, b)
    assert mn[0] == 2.0 and mn[1] == 1.0 and np.isnan(mn[2]) and mn[4] == -3.0
    assert mx[0] == 2.0 and mx[1] == 1.0 and np.isnan(mx[2]) and mx[4] == 3.0


def test_rcp_rn_exhaustive():
    """The triangle test's division-free 1/det (pt_math.h rcp_rn: v_rcp_f32 + one Newton FMA
    step) equals IEEE 1.0f/x for EVERY float with 2^-126 <= |x| <= 2^126 (checked on the device,
    4.3e9 inputs); above 2^126 the hardware reciprocal flushes, which is why scenes with
    max |e1||e2| >= 2^124 keep the division (SceneView::fast_rcp)."""
    assert pt_amd.selftest_rcp() == (0, 0)                                  # 2^-126 .. 2^125
    assert pt_amd.selftest_rcp(-1, 0x7E000000, 0x7E800000) == (0, 0)        # 2^125 .. 2^126
    assert pt_amd.selftest_rcp(-1, 0x7E800000, 0x7F7FFFFF)[0] > 0           # above 2^126: flushed
    assert pt_amd.selftest_rcp(0)[0] > 0                                    # the check can fail


def test_hash_bitexact():
    n = np.concatenate([RNG.integers(0, 2**32, 20000, dtype=np.uint64), [0, 1, 2**31 - 1, 2**32 - 1]]).astype(np.uint32)
    x = n.view(np.float32)
    g1u = pt_amd.selftest_math("hash1u", x).view(np.uint32)
    assert np.array_equal(g1u, np.array([oracle.hash1u(int(v)) for v in n], np.uint32))
    g1 = pt_amd.selftest_math("hash1", x)
    assert same_bits(g1, np.array([oracle.hash1(int(v)) for v in n], np.float32))
    g2 = np.stack([pt_amd.selftest_math("hash2x", x), pt_amd.selftest_math("hash2y", x)], 1)
    assert same_bits(g2, np.array([oracle.hash2(int(v)) for v in n], np.float32))


# ---------------------------------------------------------------------------------------------
# one reference dispatch (pt_frame) == oracle po_frame, per pixel, bit for bit
# ---------------------------------------------------------------------------------------------
FRAME_CASES = [
    # scene, W, H, salts, max_depth
    ("CornellBox", 48, 40, (0, 1, 977), 16),
    ("CornellBox", 33, 17, (5,), 8),
    ("CornellBox-Mirror", 40, 40, (0, 3), 16),
    ("CornellBox-Glossy", 40, 32, (0, 11), 16),
    ("CornellBox-Sphere", 40, 32, (0, 2), 16),
    ("MedievalBoat", 24, 16, (0,), 16),
]


@pytest.mark.parametrize("scene,W,H,salts,depth", FRAME_CASES)
def test_frame_bitexact(packed, kernel, scene, W, H, salts, depth):
    p = packed[scene]
    meta = p.meta_for(W, H)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        for t in salts:
            gpu = s.frame(meta, t, depth)
            ref, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, t, depth)
            assert same_bits(gpu, ref), f"{scene} t={t} kernel={kernel}: " + mismatch_report(gpu, ref)


@pytest.mark.parametrize("rr,direct", [(0.9, False), (0.1, False), (0.9, True)])
def test_frame_settings_bitexact(packed, kernel, rr, direct):
    p = packed["CornellBox"]
    meta = p.meta_for(40, 40, rr=rr, direct_only=direct)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        gpu = s.frame(meta, 42, 16)
    ref, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, 42, 16)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)


# ---------------------------------------------------------------------------------------------
# accumulation over frames (pt_render) == oracle po_render, and counters
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene,W,H,frame0,nframes,stride,depth", [
    ("CornellBox", 64, 48, 0, 8, 1, 8),
    ("CornellBox", 32, 32, 3, 5, 4, 16),
    ("CornellBox-Glossy", 32, 32, 1, 4, 2, 16),
    ("CornellBox-Sphere", 32, 32, 0, 4, 1, 16),
])
def test_render_accum_bitexact(packed, kernel, scene, W, H, frame0, nframes, stride, depth):
    p = packed[scene]
    meta = p.meta_for(W, H)
    init = RNG.uniform(0, 1, (H, W, 3)).astype(np.float32)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        gpu, gc = s.render(meta, frame0, nframes, stride, depth, pt_amd.MODE_MEGAKERNEL, accum=init.copy(), counters=True)
        # the uncounted build of every kernel (the one the bench times) separately
        plain = s.render(meta, frame0, nframes, stride, depth, pt_amd.MODE_MEGAKERNEL, accum=init.copy())
    ref, rc = oracle.render(p.triangle_data, p.bvh_data, meta, frame0, nframes, stride, depth, acc=init.copy())
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)
    assert same_bits(plain, ref), mismatch_report(plain, ref)
    assert gc == rc, (gc, rc)


def test_scene_info_matches_survey(packed):
    with pt_amd.Scene(packed["CornellBox"].triangle_data, packed["CornellBox"].bvh_data) as s:
        info = s.info
    # js-geometry's construction-time strides: 33 nodes / 17 leaves (16 internal), 247 leaf
    # refs, max leaf 16 (SURVEY.md §8's 21 / 11 / 164 / 20 read the strides live); light = 2 triangles
    assert info["nodes"] == 16 and info["leaves"] == 17 and info["leaf_refs"] == 247 and info["max_leaf"] == 16
    assert info["emissive_tris"] == 2 and info["materials"] == 8 and info["vertices"] == 72


def test_render_async_torch_stream(packed):
    torch = pytest.importorskip("torch")
    p = packed["CornellBox"]
    meta = p.meta_for(64, 64)
    acc = torch.zeros((64, 64, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.render_async(meta, 0, 4, 1, 8, pt_amd.MODE_MEGAKERNEL, acc.data_ptr(), st.cuda_stream)
        st.synchronize()
        host = s.render(meta, 0, 4, 1, 8, pt_amd.MODE_MEGAKERNEL)
    assert same_bits(acc.cpu().numpy(), host)


def test_invalid_scene_rejected():
    tri = np.zeros(32, np.float32)
    bvh = np.zeros(64, np.float32)
    with pytest.raises(pt_amd.PtError) as e:
        pt_amd.Scene(tri, bvh)
    assert e.value.code == -2


# ---------------------------------------------------------------------------------------------
# kernel timing (pt_profile_*) and the AUTO policy (megakernel below 2^20 paths per call)
# ---------------------------------------------------------------------------------------------
def test_profile_records_every_launch(packed, ptopts):
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    ptopts.set("PT_FUSE_GEN", "0")  # camera paths from k_wf_generate (the GEN form: below)
    p = packed["CornellBox"]
    meta = p.meta_for(64, 64)
    depth = 8
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.profile_enable(True)
        s.render(meta, 0, 4, 1, depth, pt_amd.MODE_MEGAKERNEL)
        mega = s.profile_read()
        s.profile_enable(True)
        s.render(meta, 0, 4, 1, depth, pt_amd.MODE_WAVEFRONT)
        wf = s.profile_read()
        s.profile_enable(False)
        s.render(meta, 0, 1, 1, depth, pt_amd.MODE_WAVEFRONT)
        assert s.profile_read() == {}
    assert set(mega) == {"k_regen"} and mega["k_regen"]["launches"] == 1
    # CornellBox is a mailbox scene: fused trace + shade, one launch per half and step; one batch
    # (4 frames of 64^2 fit) in two halves on two streams (dual-stream wavefront)
    assert set(wf) == {"k_wf_generate", "k_wf_step", "k_wf_accum"}
    assert wf["k_wf_step"]["launches"] == 2 * 2 * (depth + 1)
    assert wf["k_wf_generate"]["launches"] == 2 and wf["k_wf_accum"]["launches"] == 1
    ptopts.set("PT_FUSE_GEN", "1")  # the first step launch makes the camera paths
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.profile_enable(True)
        s.render(meta, 0, 4, 1, depth, pt_amd.MODE_WAVEFRONT)
        wfg = s.profile_read()
    assert set(wfg) == {"k_wf_step", "k_wf_accum"}
    assert wfg["k_wf_step"]["launches"] == 2 * 2 * (depth + 1) and wfg["k_wf_accum"]["launches"] == 1
    ptopts.set("PT_FUSE", "0")  # separate trace and shade kernels
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.profile_enable(True)
        s.render(meta, 0, 4, 1, depth, pt_amd.MODE_WAVEFRONT)
        wf2 = s.profile_read()
    assert set(wf2) == {"k_wf_generate", "k_wf_trace", "k_wf_shade_ext", "k_wf_shade_shadow", "k_wf_accum"}
    assert wf2["k_wf_trace"]["launches"] == 2 * 2 * (depth + 1)
    assert wf2["k_wf_shade_ext"]["launches"] == wf2["k_wf_shade_shadow"]["launches"] == 2 * (depth + 1)
    for v in list(mega.values()) + list(wf.values()) + list(wfg.values()) + list(wf2.values()):
        assert 0.0 < v["min_ms"] <= v["avg_ms"] <= v["max_ms"] and v["total_ms"] > 0.0


def test_auto_mode_picks_pipeline_by_size(packed, ptopts):
    """AUTO (pt_capi.hip launch_opts): the wavefront pipeline at every size on mailbox scenes (the
    fused kernel) and on scenes with cooperative big leaves, from 2^19 paths on the others."""
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)

    def kernels(name, W, H, nframes):
        p = packed[name]
        with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
            s.profile_enable(True)
            s.render(p.meta_for(W, H), 0, nframes, 1, 2, pt_amd.MODE_AUTO)
            prof = s.profile_read()
            s.profile_enable(False)
        return prof

    small = kernels("CornellBox", 64, 64, 2)
    assert "k_wf_step" in small and "k_regen" not in small  # mailbox scene: fused trace + shade
    glossy_small = kernels("CornellBox-Glossy", 64, 64, 2)
    assert "k_regen" in glossy_small and "k_wf_trace" not in glossy_small
    glossy_large = kernels("CornellBox-Glossy", 512, 512, 2)  # 2^19 paths
    assert "k_wf_trace" in glossy_large and "k_regen" not in glossy_large
    boat_small = kernels("MedievalBoat", 32, 24, 1)  # big leaves: cooperative turns in the wavefront
    assert "k_wf_trace" in boat_small and "k_regen" not in boat_small


def test_auto_large_render_matches_megakernel(packed, ptopts):
    """At the AUTO switch point the wavefront result equals the megakernel's bit for bit
    (both equal the oracle on the smaller cases above)."""
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    p = packed["CornellBox"]
    meta = p.meta_for(512, 512)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        a = s.render(meta, 0, 4, 1, 8, pt_amd.MODE_AUTO)
        m = s.render(meta, 0, 4, 1, 8, pt_amd.MODE_MEGAKERNEL)
    assert same_bits(a, m), mismatch_report(a, m)


# ---------------------------------------------------------------------------------------------
# mailboxed traversal: exact ties between distinct leaf entries
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="session")
def packed_tie(tmp_path_factory):
    """CornellBox with the back wall duplicated under another material (same vertex indices,
    so both entries give bit-identical t on every back-wall hit).  The reference keeps the
    first of the two in leaf order; the mailboxed leaf loop tests entries in uid order and
    must resolve the tie the same way (PT_MB_UID_ORDER=reverse puts the duplicate first)."""
    import os
    import shutil
    from conftest import SCENES, pack_with_node
    base = tmp_path_factory.mktemp("tie")
    src = os.path.join(SCENES, "scene_assets")
    dst = base / "scene_assets"  # the Node loader resolves '/scene_assets/...' under the web root
    dst.mkdir()
    shutil.copy(os.path.join(src, "CornellBox.xml"), dst / "CornellBox.xml")
    mdir = dst / "models" / "CornellBox"
    mdir.mkdir(parents=True)
    shutil.copy(os.path.join(src, "models", "CornellBox", "CornellBox-Original.mtl"), mdir)
    with open(os.path.join(src, "models", "CornellBox", "CornellBox-Original.obj")) as f:
        obj = f.read()
    with open(mdir / "CornellBox-Original.obj", "w") as f:
        f.write(obj + "\ng backWallTwin\nusemtl leftWall\nf 9 10 11 12\n")
    return pack_with_node(str(dst / "CornellBox.xml"), str(base / "packed"))


@pytest.mark.parametrize("env", [{}, {"PT_MB_UID_ORDER": "reverse"}, {"PT_MAILBOX": "0"},
                                 {"PT_MB_UID_ORDER": "reverse", "PT_BF_SLOTS": "1"},
                                 {"PT_TRAV": "lean16", "PT_MB_UID_ORDER": "reverse"},
                                 {"PT_FUSE": "0", "PT_MB_UID_ORDER": "reverse"},
                                 {"PT_BF_STACKLESS": "0", "PT_MB_UID_ORDER": "reverse"}],
                         ids=["bf", "bf_reverse_uids", "no_mailbox", "bf_reverse_1slot", "mb_lean16_reverse",
                              "bf_nofuse_reverse", "bf_stack_reverse"])
def test_mailbox_exact_ties(packed_tie, ptopts, env):
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    ptopts.set("PT_KERNEL", "wavefront")
    for k, v in env.items():
        ptopts.set(k, v)
    p = packed_tie
    meta = p.meta_for(48, 40)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        gpu = s.frame(meta, 3, 8)
        acc, gc = s.render(meta, 0, 3, 1, 8, pt_amd.MODE_WAVEFRONT, counters=True)
    ref, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, 3, 8)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)
    racc, rc = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 3, 1, 8)
    assert same_bits(acc, racc), mismatch_report(acc, racc)
    assert gc == rc, (gc, rc)


# ---------------------------------------------------------------------------------------------
# vertex-normal mode: the reference's commented-out smooth-normal branch
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("scene,W,H", [("CornellBox-Glossy", 40, 32), ("CornellBox-Sphere", 40, 32),
                                       ("MedievalBoat", 24, 16), ("CornellBox", 32, 24)])
@pytest.mark.parametrize("env", [{"PT_KERNEL": "mega"}, {"PT_KERNEL": "wavefront"},
                                 {"PT_KERNEL": "wavefront", "PT_FUSE": "0"}], ids=["mega", "wavefront", "wf_nofuse"])
def test_vertex_normals_bitexact(packed, ptopts, scene, W, H, env):
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    for k, v in env.items():
        ptopts.set(k, v)
    p = packed[scene]
    meta = p.meta_for(W, H)
    oracle.set_vertex_normals(True)
    try:
        ref, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, 5, 16)
        racc, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 3, 1, 8)
    finally:
        oracle.set_vertex_normals(False)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.set_vertex_normals(True)
        gpu = s.frame(meta, 5, 16)
        acc = s.render(meta, 0, 3, 1, 8, pt_amd.MODE_AUTO)
        s.set_vertex_normals(False)
        flat = s.frame(meta, 5, 16)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)
    assert same_bits(acc, racc), mismatch_report(acc, racc)
    plain, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, 5, 16)
    assert same_bits(flat, plain)  # switching back restores the reference's normals
    if scene != "CornellBox":  # scenes with vertex normals shade differently
        assert not same_bits(gpu, plain)


def test_large_image_single_part_matches_megakernel(packed, ptopts):
    """4096^2 (config 5's image): more pixels than the default batch target, so the batch holds
    two frames, one per part on its own stream (and with PT_PARTS=1 one part holding both); the
    fused wavefront still equals the megakernel bit for bit (both equal the oracle on the small
    cases)."""
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    p = packed["CornellBox"]
    meta = p.meta_for(4096, 4096)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        a = s.render(meta, 0, 2, 1, 2, pt_amd.MODE_WAVEFRONT)
        ptopts.set("PT_PARTS", "1")
        a1 = s.render(meta, 0, 2, 1, 2, pt_amd.MODE_WAVEFRONT)
        ptopts.unset("PT_PARTS")
        m = s.render(meta, 0, 2, 1, 2, pt_amd.MODE_MEGAKERNEL)
    assert same_bits(a, m), mismatch_report(a, m)
    assert same_bits(a1, m), mismatch_report(a1, m)


def test_fuse_gen_full_size(packed, ptopts):
    """Camera paths from k_wf_generate or made in the first fused launch give the same bits at the
    bench's image size (1024^2, 2 frames, the full depth)."""
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    ptopts.set("PT_KERNEL", "wavefront")
    p = packed["CornellBox"]
    meta = p.meta_for(1024, 1024)
    out = {}
    for gen in ("0", "1"):
        ptopts.set("PT_FUSE_GEN", gen)
        with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
            out[gen] = s.render(meta, 0, 2, 1, -1, pt_amd.MODE_WAVEFRONT)
    assert same_bits(out["0"], out["1"]), mismatch_report(out["0"], out["1"])


# ---------------------------------------------------------------------------------------------
# multi-mesh scene (Node host --all-meshes): CornellBox2 = Cornell box + MedievalBoat
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="session")
def packed_multi(tmp_path_factory):
    from conftest import SCENES, pack_with_node
    import os
    return pack_with_node(os.path.join(SCENES, "scene_assets", "CornellBox2.xml"),
                          str(tmp_path_factory.mktemp("multi") / "cb2"), "--all-meshes", "--native-bvh")


@pytest.mark.parametrize("env", [{}, {"PT_KERNEL": "wavefront"}, {"PT_KERNEL": "mega"}])
def test_multi_mesh_frame_bitexact(packed_multi, ptopts, env):
    for k in ENV_KEYS:
        ptopts.unset(k, raising=False)
    for k, v in env.items():
        ptopts.set(k, v)
    p = packed_multi
    meta = p.meta_for(32, 24)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        gpu = s.frame(meta, 5, 8)
    ref, _ = oracle.frame(p.triangle_data, p.bvh_data, meta, 5, 8)
    assert same_bits(gpu, ref), mismatch_report(gpu, ref)
