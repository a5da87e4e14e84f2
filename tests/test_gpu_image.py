"""On-device display transform (pt_tonemap_async, pt_render_image)
against the host pt_tonemap (program-raymarch.ts:295-316 in JS double semantics): same bytes."""
import numpy as np
import pytest

import pt_amd

pytestmark = pytest.mark.gpu


def device_tonemap(s, acc, runs):
    torch = pytest.importorskip("torch")
    d_acc = torch.from_numpy(np.ascontiguousarray(acc, np.float32)).cuda()
    npix = acc.size // 3
    d_rgba = torch.zeros(npix * 4, dtype=torch.uint8, device="cuda")
    s.tonemap_async(d_acc.data_ptr(), npix, runs, d_rgba.data_ptr(), 0)
    torch.cuda.synchronize()
    return d_rgba.cpu().numpy().reshape(acc.shape[:-1] + (4,))


@pytest.mark.parametrize("runs", [1, 7, 256])
def test_device_tonemap_equals_host(packed, runs):
    rng = np.random.default_rng(runs)
    acc = rng.exponential(0.7 * runs, (97, 131, 3)).astype(np.float32)
    acc[0, :8] = 0.0                                   # black
    acc[1, :8] = np.float32(3.0e38)                    # overflow to inf in lum + 1
    acc[2, :8] = rng.uniform(0, 1e-30, (8, 3))         # tiny / subnormal ratios
    acc[3, :8] = np.float32(runs) * np.float32(255.0)  # ToInt32 far above 255 -> clamp
    p = packed["CornellBox"]
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        dev = device_tonemap(s, acc, runs)
    host = pt_amd.tonemap(acc, runs).reshape(dev.shape)
    assert np.array_equal(dev, host), int((dev != host).sum())


@pytest.mark.parametrize("mode", [pt_amd.MODE_MEGAKERNEL, pt_amd.MODE_WAVEFRONT])
def test_render_image_equals_render_then_host_tonemap(packed, mode):
    p = packed["CornellBox"]
    meta = p.meta_for(96, 64)
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        img, c1 = s.render_image(meta, 0, 8, 1, 8, mode, counters=True)
        acc, c2 = s.render(meta, 0, 8, 1, 8, mode, counters=True)
    assert np.array_equal(img, pt_amd.tonemap(acc, 8).reshape(img.shape))
    assert c1 == c2


@pytest.mark.parametrize("n", [0, 3, 4, 1023, 3 * 96 * 64, 3 * 1024 * 1024 + 2])
def test_readback_to_pinned_host(packed, n):
    """pt_readback_async (the accumulator to pinned host memory, program-raymarch.ts:262-293): the
    same bytes as the device buffer, any length (a tail of < 4 floats included)."""
    torch = pytest.importorskip("torch")
    p = packed["CornellBox"]
    src = torch.arange(n, dtype=torch.float32, device="cuda") * 0.5 - 3.0
    dst = torch.full((max(n, 1),), -7.0, dtype=torch.float32).pin_memory()
    st = torch.cuda.Stream()
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        s.readback_async(src.data_ptr(), n, dst.data_ptr(), st.cuda_stream)
        st.synchronize()
        assert torch.equal(dst[:n], src.cpu())
        if n == 0:
            assert float(dst[0]) == -7.0
            return
        # pageable host memory is refused, not read through
        pageable = torch.zeros(max(n, 4), dtype=torch.float32)
        with pytest.raises(pt_amd.PtError):
            s.readback_async(src.data_ptr(), n, pageable.data_ptr(), st.cuda_stream)
