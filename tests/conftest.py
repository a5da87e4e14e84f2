"""Shared fixtures.  `gpu`-marked tests need an MI355X (run on the GPU box via gpurun)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "brown-cs2240-path-tracer_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "scenes")
PACK_JS = os.path.join(PKG, "node", "bin", "pt-pack.js")
ALL_SCENES = ["CornellBox", "CornellBox-Mirror", "CornellBox-Glossy", "CornellBox-Sphere", "MedievalBoat"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu on the GPU box)")


class Packed:
    def __init__(self, d):
        self.dir = d
        self.triangle_data = np.fromfile(os.path.join(d, "triangle_data.f32"), np.float32)
        self.bvh_data = np.fromfile(os.path.join(d, "bvh_data.f32"), np.float32)
        self.meta = np.fromfile(os.path.join(d, "meta.f32"), np.float32)
        with open(os.path.join(d, "scene.json")) as f:
            self.info = json.load(f)

    def meta_for(self, W, H, rr=None, direct_only=None):
        """Same camera at another resolution: the fields program-raymarch.ts:79-92 derives from W, H."""
        m = self.meta.copy()
        m[0], m[1] = W, H
        m[8], m[9] = np.float32(1 / W), np.float32(1 / H)
        m[10] = np.float32(W / H)
        if rr is not None:
            m[45] = rr
        if direct_only is not None:
            m[46] = 1.0 if direct_only else -1.0
        return m


class PtOptions:
    """pt_set_option switches for one test (the library reads no environment variable).  Keys may
    use the old environment spelling ("PT_KERNEL") or the option name ("kernel")."""

    def set(self, name, value):
        import pt_amd
        pt_amd.set_option(name, value)

    def unset(self, name, raising=False):
        import pt_amd
        pt_amd.set_option(name, None)


@pytest.fixture
def ptopts():
    """Every option at its default before and after the test."""
    import pt_amd
    pt_amd.reset_options()
    yield PtOptions()
    pt_amd.reset_options()


def pack_with_node(src: str, out_dir: str, *extra) -> Packed:
    """Run the product's Node scene pipeline (node/bin/pt-pack.js)."""
    subprocess.run(["node", PACK_JS, src, out_dir, *extra], check=True, capture_output=True)
    return Packed(out_dir)


@pytest.fixture(scope="session")
def packed(tmp_path_factory):
    """dict scene name -> Packed (512x512 meta, rr 0.9) produced by the Node host."""
    base = tmp_path_factory.mktemp("packed")
    out = {}
    for s in ALL_SCENES:
        out[s] = pack_with_node(os.path.join(SCENES, "scene_assets", s + ".xml"), str(base / s))
    return out
