"""Device-side failure reporting on the asynchronous path (pt_render_async + pt_scene_check).

A wavefront traversal wave that exceeds its watchdog limit leaves a flag instead of hanging
(k_wf_trace, kTraceWatchdog); PT_TRACE_WATCHDOG lowers the limit so the report can be forced.
The asynchronous call cannot report it itself; pt_scene_check (after the render) and the next
call on the scene (once the render has completed) must, and the flag must then be cleared.
"""
import numpy as np
import pytest

import oracle
import pt_amd

pytestmark = pytest.mark.gpu

KEYS = ("PT_KERNEL", "PT_TRAV", "PT_TRACE_WATCHDOG", "PT_WF_PATHS", "PT_PARTS", "PT_FUSE", "PT_BF", "PT_MAILBOX")


@pytest.fixture
def env(ptopts):
    for k in KEYS:
        ptopts.unset(k, raising=False)
    ptopts.set("PT_KERNEL", "wavefront")
    return ptopts


def _torch():
    return pytest.importorskip("torch")


def test_async_watchdog_reported_by_scene_check(packed, env):
    torch = _torch()
    p = packed["CornellBox-Glossy"]  # > 64 distinct entries: the traversal kernel k_wf_trace
    meta = p.meta_for(64, 64)
    acc = torch.zeros((64, 64, 3), dtype=torch.float32, device="cuda")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        env.set("PT_TRACE_WATCHDOG", "4")
        s.render_async(meta, 0, 2, 1, 8, pt_amd.MODE_WAVEFRONT, acc.data_ptr(), 0)  # returns without a report
        with pytest.raises(pt_amd.PtError) as e:
            s.check()
        assert "gave up" in str(e.value) and e.value.code == -4
        s.check()  # reported once, then cleared
        env.unset("PT_TRACE_WATCHDOG")
        good = s.render(meta, 0, 2, 1, 8, pt_amd.MODE_WAVEFRONT)
    ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 2, 1, 8)
    assert np.array_equal(good.view(np.uint32), ref.view(np.uint32))


def test_async_watchdog_reported_by_next_call(packed, env):
    torch = _torch()
    p = packed["CornellBox-Glossy"]
    meta = p.meta_for(64, 64)
    acc = torch.zeros((64, 64, 3), dtype=torch.float32, device="cuda")
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        env.set("PT_TRACE_WATCHDOG", "4")
        s.render_async(meta, 0, 2, 1, 8, pt_amd.MODE_WAVEFRONT, acc.data_ptr(), 0)
        torch.cuda.synchronize()
        env.unset("PT_TRACE_WATCHDOG")
        with pytest.raises(pt_amd.PtError) as e:  # the completed render's flag surfaces here
            s.render_async(meta, 0, 2, 1, 8, pt_amd.MODE_WAVEFRONT, acc.data_ptr(), 0)
        assert "gave up" in str(e.value)
        acc.zero_()
        s.render_async(meta, 0, 2, 1, 8, pt_amd.MODE_WAVEFRONT, acc.data_ptr(), 0)
        s.check()
    ref, _ = oracle.render(p.triangle_data, p.bvh_data, meta, 0, 2, 1, 8)
    assert np.array_equal(acc.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_blocking_render_reports_watchdog(packed, env):
    p = packed["CornellBox-Glossy"]
    meta = p.meta_for(48, 48)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        env.set("PT_TRACE_WATCHDOG", "4")
        with pytest.raises(pt_amd.PtError):
            s.render(meta, 0, 1, 1, 8, pt_amd.MODE_WAVEFRONT)
        env.unset("PT_TRACE_WATCHDOG")
        s.render(meta, 0, 1, 1, 8, pt_amd.MODE_WAVEFRONT)  # cleared: renders again
