"""pt_render_multi (the C ABI's multi-GPU entry): frames dealt round-robin over one
scene per device, partial f32 accumulators reduced onto the first scene's device.

The box has one GPU, so the multi-device orchestration runs with repeated devices (several scenes
on device 0: one host thread each, then the ORDERED reduction: partials added in device order).
That reduction is deterministic, so it is pinned bit for bit against the oracle's per-shard
renders summed in the same order; n = 1 is pt_render exactly, and through a one-rank RCCL
communicator (option reduce=rccl) too.  The RCCL reduction over distinct devices changes only the
summation order of the same partials; the driver's 8-GPU node runs it.
"""
import numpy as np
import pytest

import oracle
import pt_amd

pytestmark = pytest.mark.gpu


@pytest.fixture
def env(ptopts):
    for k in ("PT_KERNEL", "PT_REDUCE", "PT_PARTS", "PT_WF_PATHS"):
        ptopts.unset(k, raising=False)
    return ptopts


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_single_device_list_is_pt_render(packed, env):
    p = packed["CornellBox"]
    meta = p.meta_for(256, 256)
    init = np.random.default_rng(3).uniform(0, 1, (256, 256, 3)).astype(np.float32)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        a, ca = pt_amd.render_multi([s], meta, 0, 20, 1, 8, accum=init.copy(), counters=True)
        b, cb = s.render(meta, 0, 20, 1, 8, accum=init.copy(), counters=True)
    assert np.array_equal(bits(a), bits(b)) and ca == cb


@pytest.mark.timeout(240, method="thread")  # a stuck collective ends the run with its stacks, not a hang
def test_rccl_one_rank_is_pt_render(packed, env):
    """The RCCL branch on the one-GPU box: option reduce=rccl sends a one-device list through it —
    librccl loaded, ncclCommInitAll over one device, the ncclReduce (a copy onto itself), the
    communicator released — and the bits are pt_render's."""
    p = packed["CornellBox"]
    meta = p.meta_for(128, 128)
    init = np.random.default_rng(5).uniform(0, 1, (128, 128, 3)).astype(np.float32)
    env.set("PT_REDUCE", "rccl")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        try:
            a, ca = pt_amd.render_multi([s], meta, 0, 9, 1, 8, accum=init.copy(), counters=True)
            a2, _ = pt_amd.render_multi([s], meta, 0, 9, 1, 8, accum=init.copy(), counters=True)  # cached communicator
        finally:
            pt_amd.release_communicators()
        b, cb = s.render(meta, 0, 9, 1, 8, accum=init.copy(), counters=True)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(bits(a2), bits(b)) and ca == cb


@pytest.mark.parametrize("n,mode", [(2, pt_amd.MODE_AUTO), (3, pt_amd.MODE_MEGAKERNEL), (4, pt_amd.MODE_WAVEFRONT)])
def test_repeated_device_ordered_reduction_vs_oracle(packed, env, n, mode):
    p = packed["CornellBox"]
    W = H = 64
    meta = p.meta_for(W, H)
    frame0, nframes, stride, depth = 3, 11, 2, 8
    init = np.random.default_rng(5).uniform(0, 1, (H, W, 3)).astype(np.float32)
    scenes = [pt_amd.Scene(p.triangle_data, p.bvh_data, device=0) for _ in range(n)]
    try:
        got, cnt = pt_amd.render_multi(scenes, meta, frame0, nframes, stride, depth, mode, accum=init.copy(),
                                       counters=True)
    finally:
        for s in scenes:
            s.close()
    # oracle: shard g renders frames i = g, g + n, ... (k = frame0 + i * stride) onto init (g = 0) or zero,
    # then the partials are added in device order
    parts, total = [], {}
    for g in range(n):
        cnt_g = len(range(g, nframes, n))
        acc, c = oracle.render(p.triangle_data, p.bvh_data, meta, frame0 + g * stride, cnt_g, n * stride, depth,
                               acc=init.copy() if g == 0 else np.zeros_like(init))
        parts.append(acc)
        for k, v in c.items():
            total[k] = total.get(k, 0) + v
    want = parts[0].copy()
    for g in range(1, n):
        want += parts[g]
    assert np.array_equal(bits(got), bits(want))
    assert cnt == total
    # and within f32 rounding of the single-device render of all frames
    ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, frame0, nframes, stride, depth, acc=init.copy())
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_rccl_mode_rejects_repeated_devices(packed, env):
    p = packed["CornellBox"]
    env.set("PT_REDUCE", "rccl")
    scenes = [pt_amd.Scene(p.triangle_data, p.bvh_data, device=0) for _ in range(2)]
    try:
        with pytest.raises(pt_amd.PtError):
            pt_amd.render_multi(scenes, p.meta_for(32, 32), 0, 2, 1, 4)
    finally:
        for s in scenes:
            s.close()


@pytest.mark.timeout(240, method="thread")  # a stuck collective ends the run with its stacks, not a hang
@pytest.mark.parametrize("ndev", [2, 8])
def test_rccl_reduce_distinct_devices_vs_oracle(packed, env, ndev):
    """The RCCL branch of pt_render_multi (ncclCommInitAll + ONE ncclReduce): the same partials as
    the ordered reduction in another summation order, so within f32 rounding of the oracle's
    ordered sum; the counters are exact.  Communicators are released afterwards."""
    if pt_amd.device_count() < ndev:
        pytest.skip(f"the RCCL reduction over {ndev} distinct GPUs needs {ndev} visible (the driver's 8-GPU node)")
    n = ndev
    p = packed["CornellBox"]
    W = H = 64
    meta = p.meta_for(W, H)
    frame0, nframes, stride, depth = 1, 13, 1, 8
    env.set("PT_REDUCE", "rccl")
    scenes = [pt_amd.Scene(p.triangle_data, p.bvh_data, device=g) for g in range(n)]
    try:
        got, cnt = pt_amd.render_multi(scenes, meta, frame0, nframes, stride, depth, accum=np.zeros((H, W, 3), np.float32),
                                       counters=True)
    finally:
        for s in scenes:
            s.close()
        pt_amd.release_communicators()
    parts, total = [], {}
    for g in range(n):
        acc, c = oracle.render(p.triangle_data, p.bvh_data, meta, frame0 + g * stride, len(range(g, nframes, n)),
                               n * stride, depth)
        parts.append(acc)
        for k, v in c.items():
            total[k] = total.get(k, 0) + v
    want = parts[0].copy()
    for g in range(1, n):
        want += parts[g]
    assert np.allclose(got, want, rtol=1e-6, atol=1e-6)
    assert cnt == total
