"""The camera probe behind AUTO's choice of the leaf pass (pt_leafbvh.cpp probe_pre_leaves, host code;
render_impl runs the pass when the probe's visited leaf work is >= pre_ratio % of the filtered work).
scripts/probe_harness.cpp builds a two-leaf tree by hand: a big leaf A under an inner node, and a wall
leaf B under the root.  With the wall between the camera and A, every camera ray that passes A's box
filter is stopped by the reference's exit-distance pruning before it reaches A (a pass would resolve A
for nothing); with the wall behind the camera every ray that passes the filter visits A.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("no hipcc")
    exe = str(tmp_path_factory.mktemp("probe") / "probe_harness")
    csrc = os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "csrc")
    subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O2", "-std=c++17", "-I", csrc,
                    os.path.join(ROOT, "scripts", "probe_harness.cpp"), os.path.join(csrc, "pt_leafbvh.cpp"),
                    "-o", exe], check=True, capture_output=True)
    return exe


def test_probe_counts_filter_passes_and_visits(harness):
    out = subprocess.run([harness], check=True, capture_output=True, text=True).stdout.split("\n")
    (walled_pass, walled_visit), (open_pass, open_visit) = [tuple(map(int, line.split())) for line in out[:2]]
    # 32 x 32 camera rays; A (4 x 4 at z = -5) covers the central (0.4 / 0.5)^2 of the view: 26^2 rays
    assert walled_pass == 676
    assert walled_visit == 0  # the wall's hit prunes the inner node: the pass would be wasted
    # no wall in front: primary rays and the bounces / shadow rays that pass the filter all visit A
    assert open_pass == open_visit >= 676
