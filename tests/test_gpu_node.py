"""GPU: the Node host's render path (programEntry through the N-API addon, node/lib/program-entry.js;
the pt-render.js CLI) gives the same bits as the Python/C path on the same packed scene."""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import pt_amd
from conftest import PKG, SCENES, pack_with_node

pytestmark = pytest.mark.gpu
INI = os.path.join(SCENES, "scene_files", "final", "cornell_box_full_lighting.ini")
W, H, SPP = 64, 48, 6

NODE_SCRIPT = r"""
const fs = require('fs');
const host = require(process.argv[1]);
(async () => {
    const s = host.load_scene_from_ini(process.argv[2], { web_root: process.argv[3], quiet: true });
    const S = s.scene_description.Settings;
    S.imageWidth = %d; S.imageHeight = %d; S.samplesPerPixel = %d;
    const dim = host.screen_dimension(S);
    const a = await host.programEntry(dim, s.primitive_data, s.camera_data, s.scene_description,
                                      { maxDepth: 8, mode: 'megakernel', chunk: 4, counters: true });
    const b = await host.programEntry(dim, s.primitive_data, s.camera_data, s.scene_description,
                                      { maxDepth: 8, mode: 'wavefront', imageOnly: true, counters: true });
    const c = await host.programEntry(dim, s.primitive_data, s.camera_data, s.scene_description,
                                      { maxDepth: 8, mode: 'wavefront' });
    const out = process.argv[4];
    fs.writeFileSync(out + '/accum.f32', Buffer.from(a.accum.buffer));
    fs.writeFileSync(out + '/rgba.u8', Buffer.from(a.rgba.buffer));
    fs.writeFileSync(out + '/rgba_image.u8', Buffer.from(b.rgba.buffer));
    fs.writeFileSync(out + '/accum_fast.f32', Buffer.from(c.accum.buffer));
    if (c.counters !== null) throw Error('counters without asking');
    fs.writeFileSync(out + '/counters.json', JSON.stringify([a.counters, b.counters]));
})().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
""" % (W, H, SPP)


def test_node_program_entry_matches_python_path():
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["node", "-e", NODE_SCRIPT, os.path.join(PKG, "node"), INI, SCENES, td], check=True,
                       capture_output=True, timeout=300)
        acc = np.fromfile(os.path.join(td, "accum.f32"), np.float32).reshape(H, W, 3)
        rgba = np.fromfile(os.path.join(td, "rgba.u8"), np.uint8).reshape(H, W, 4)
        rgba_img = np.fromfile(os.path.join(td, "rgba_image.u8"), np.uint8).reshape(H, W, 4)
        acc_fast = np.fromfile(os.path.join(td, "accum_fast.f32"), np.float32).reshape(H, W, 3)
        c_node = json.load(open(os.path.join(td, "counters.json")))
        p = pack_with_node(INI, os.path.join(td, "packed"), "--web-root", SCENES, "--width", str(W), "--height", str(H),
                           "--spp", str(SPP))
    with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
        ref, c = s.render(p.meta, 0, SPP, 1, 8, pt_amd.MODE_MEGAKERNEL, counters=True)
    assert acc.tobytes() == ref.tobytes()                       # chunked (4 + 2 frames) == one call
    assert acc_fast.tobytes() == ref.tobytes()                  # uncounted wavefront build, same bits
    assert np.array_equal(rgba, pt_amd.tonemap(ref, SPP))
    assert np.array_equal(rgba_img, rgba)                        # device tone map, wavefront pipeline
    assert c_node[0] == c and c_node[1] == c


def test_pt_render_cli_writes_png():
    from PIL import Image
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["node", os.path.join(PKG, "node", "bin", "pt-render.js"), INI, "--web-root", SCENES,
                            "--out-root", td, "--spp", "2", "--max-depth", "4"], check=True, capture_output=True,
                           text=True, timeout=300)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        img = np.array(Image.open(info["output"]))
    assert img.shape == (info["height"], info["width"], 4) and info["spp"] == 2
    assert img[..., 3].min() == 255 and img[..., :3].mean() > 10


NODE_MULTI = r"""
const fs = require('fs');
const host = require(process.argv[1]);
(async () => {
    const s = host.load_scene_from_ini(process.argv[2], { web_root: process.argv[3], quiet: true });
    const S = s.scene_description.Settings;
    S.imageWidth = %d; S.imageHeight = %d; S.samplesPerPixel = %d;
    const dim = host.screen_dimension(S);
    const a = await host.programEntry(dim, s.primitive_data, s.camera_data, s.scene_description,
                                      { maxDepth: 8, devices: [0, 0, 0], counters: true });
    fs.writeFileSync(process.argv[4] + '/accum_multi.f32', Buffer.from(a.accum.buffer));
    // one job per scene at a time: a second render on a busy scene is rejected, not raced
    const pt = host.native();
    const sc = pt.sceneCreate(s.primitive_data[0].triangle_data, s.primitive_data[0].bvh_data, 0);
    const meta = host.make_meta(dim, s.camera_data, s.scene_description, 0);
    const acc = new Float32Array(dim[0] * dim[1] * 3);
    const p1 = pt.render(sc, meta, 0, 4, 1, 8, 0, acc, false);
    let busy = null;
    try { await pt.render(sc, meta, 0, 4, 1, 8, 0, new Float32Array(acc.length), false); } catch (e) { busy = e.message; }
    let busy_sync = null;
    try { pt.renderSync(sc, meta, 0, 1, 1, 8, 0, new Float32Array(acc.length), false); } catch (e) { busy_sync = e.message; }
    let busy_destroy = null;
    try { pt.sceneDestroy(sc); } catch (e) { busy_destroy = e.message; }
    await p1;
    pt.sceneDestroy(sc);
    let gone = null;
    try { pt.sceneInfo(sc); } catch (e) { gone = e.message; }
    fs.writeFileSync(process.argv[4] + '/busy.json', JSON.stringify({busy, busy_sync, busy_destroy, gone, counters: a.counters}));
})().catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
""" % (W, H, SPP)


def test_node_multi_device_and_busy_scene():
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["node", "-e", NODE_MULTI, os.path.join(PKG, "node"), INI, SCENES, td], check=True,
                       capture_output=True, timeout=300)
        acc = np.fromfile(os.path.join(td, "accum_multi.f32"), np.float32).reshape(H, W, 3)
        info = json.load(open(os.path.join(td, "busy.json")))
        p = pack_with_node(INI, os.path.join(td, "packed"), "--web-root", SCENES, "--width", str(W), "--height", str(H),
                           "--spp", str(SPP))
    scenes = [pt_amd.Scene(p.triangle_data, p.bvh_data) for _ in range(3)]
    try:
        ref, c = pt_amd.render_multi(scenes, p.meta, 0, SPP, 1, 8, counters=True)
    finally:
        for s in scenes:
            s.close()
    assert acc.tobytes() == ref.tobytes()
    assert info["counters"] == c
    for k in ("busy", "busy_sync", "busy_destroy"):
        assert info[k] and "busy" in info[k], info
    assert info["gone"] and "destroyed" in info["gone"]
