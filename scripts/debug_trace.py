#!/usr/bin/env python3
"""Render one configuration through the wavefront and report (watchdog snapshot on failure)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "brown-cs2240-path-tracer_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402

import pt_amd  # noqa: E402
import tempfile  # noqa: E402

from conftest import SCENES, pack_with_node  # noqa: E402

W, H, F, D = (int(v) for v in sys.argv[1:5])
p = pack_with_node(os.path.join(SCENES, "scene_assets", "CornellBox.xml"), tempfile.mkdtemp())
with pt_amd.Scene(p.triangle_data, p.bvh_data) as s:
    t = time.time()
    try:
        acc = s.render(p.meta_for(W, H), 0, F, 1, D, pt_amd.MODE_WAVEFRONT)
        print(f"ok {W}x{H}x{F} depth {D}: mean {float(np.mean(acc)):.4f} in {time.time() - t:.2f}s", flush=True)
    except pt_amd.PtError as e:
        print(f"FAILED {W}x{H}x{F} depth {D}: {e}", flush=True)
        sys.exit(1)
