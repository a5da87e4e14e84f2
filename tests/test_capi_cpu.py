"""C ABI checks that need no GPU: the library loads, exports every symbol include/pt_hip.h
declares, reports errors the documented way, and its host-side tone map matches the oracle."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle
import pt_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pt_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("pt_scene_create", "pt_scene_destroy", "pt_render", "pt_render_async", "pt_frame", "pt_tonemap",
              "pt_last_error"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(pt_amd.lib_path())
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", pt_amd.lib_path()], capture_output=True, text=True).stdout
    for f in declared_functions():
        assert re.search(rf"\bT {f}\b", out), f


def test_kernels_built_for_gfx950():
    """The fat binary embedded in libpt_hip.so carries gfx950 code objects only."""
    data = open(pt_amd.lib_path(), "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_abi_version():
    assert pt_amd.abi_version() == 3 == pt_amd.ABI_VERSION


def test_build_id_is_this_trees_source_hash():
    """The library carries the SHA-256 of its sources (csrc/Makefile); pt_amd refuses another."""
    assert re.fullmatch(r"[0-9a-f]{64}", pt_amd.build_id())
    assert pt_amd.build_id() == pt_amd.source_hash()


def test_no_environment_switches_in_the_library():
    """Kernel selection is explicit (pt_set_option): the library reads no environment variable."""
    csrc = os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h", ".cpp")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f
    out = subprocess.run(["nm", "-D", "--undefined-only", pt_amd.lib_path()], capture_output=True, text=True).stdout
    assert not re.search(r"\bgetenv\b", out)


def test_options_set_get_reset_and_validate():
    pt_amd.reset_options()
    try:
        assert pt_amd.get_option("kernel") == ""
        pt_amd.set_option("kernel", "wavefront")
        pt_amd.set_option("PT_TRAV", "lean8")  # the old environment spelling maps to the option
        pt_amd.set_option("parts", 3)
        assert (pt_amd.get_option("kernel"), pt_amd.get_option("trav"), pt_amd.get_option("parts")) == \
            ("wavefront", "lean8", "3")
        with pt_amd.options(kernel="mega", sort=64):
            assert pt_amd.get_option("kernel") == "mega" and pt_amd.get_option("sort") == "64"
        assert pt_amd.get_option("kernel") == "wavefront" and pt_amd.get_option("sort") == ""
        pt_amd.set_option("kernel", None)
        assert pt_amd.get_option("kernel") == ""
        for name, value in (("nosuch", "1"), ("kernel", "fast"), ("parts", "x"), ("lds", "2"), ("parts", "-1"),
                            ("trav", ""), ("reduce", "nccl")):
            with pytest.raises(pt_amd.PtError) as e:
                pt_amd.set_option(name, value)
            assert e.value.code == -1
    finally:
        pt_amd.reset_options()
    assert pt_amd.get_option("trav") == "" and pt_amd.get_option("parts") == ""


def test_layout_options():
    """The queue-layout and stack switches are options like the others:
    flags that take 0/1 and reject anything else; the batch target is an integer; the
    experiments removed in round 4 are unknown names."""
    pt_amd.reset_options()
    try:
        for name in ("packet", "persist", "regen_bf", "cull", "tiles", "scatter", "batch_pipe",
                     "trace_dyn", "stagger", "pipe", "ifif", "stack16"):
            with pytest.raises(pt_amd.PtError):
                pt_amd.set_option(name, "1")
        pt_amd.set_option("regen", 64)  # round 6: the fused kernel's streaming regeneration (an integer)
        assert pt_amd.get_option("regen") == "64"
        with pytest.raises(pt_amd.PtError):
            pt_amd.set_option("regen", "x")
        for name in ("region_perm",):
            pt_amd.set_option(name, 0)
            assert pt_amd.get_option(name) == "0"
            pt_amd.set_option(name, 1)
            with pytest.raises(pt_amd.PtError):
                pt_amd.set_option(name, "2")
        pt_amd.set_option("wf_paths", 8 << 20)
        assert pt_amd.get_option("wf_paths") == str(8 << 20)
        with pytest.raises(pt_amd.PtError):
            pt_amd.set_option("wf_paths", "lots")
        for run in (2, 4):  # pooled leaf turns: runs of 2 or 4 entries
            pt_amd.set_option("pool_run", run)
            assert pt_amd.get_option("pool_run") == str(run)
        for bad in ("0", "1", "3", "8", "-2"):
            with pytest.raises(pt_amd.PtError):
                pt_amd.set_option("pool_run", bad)
    finally:
        pt_amd.reset_options()


def test_kernel_time_struct_matches_header():
    # pt_kernel_time: name[32], launches, total/min/max/busy ms
    assert ctypes.sizeof(pt_amd._lib.KernelTime) == 32 + 8 + 4 * 8
    assert "busy_ms" in open(HEADER).read()


def test_no_load_time_environment_change():
    """Loading the library changes nothing in the process environment; pt_set_hw_queues is the
    explicit opt-in, effective only before the library touches HIP."""
    code = (
        "import ctypes, os, sys\n"
        "os.environ.pop('GPU_MAX_HW_QUEUES', None)\n"
        f"L = ctypes.CDLL({pt_amd.lib_path()!r})\n"
        "assert 'GPU_MAX_HW_QUEUES' not in os.environ\n"
        "libc = ctypes.CDLL(None); libc.getenv.restype = ctypes.c_char_p\n"
        "assert libc.getenv(b'GPU_MAX_HW_QUEUES') is None\n"
        "assert L.pt_set_hw_queues(0) == -1 and L.pt_set_hw_queues(99) == -1\n"
        "assert L.pt_set_hw_queues(8) == 0 and libc.getenv(b'GPU_MAX_HW_QUEUES') == b'8'\n"
        "n = ctypes.c_int(0); assert L.pt_device_count(ctypes.byref(n)) == 0\n"
        "assert L.pt_set_hw_queues(4) == -1  # the runtime is up now\n"
    )
    env = dict(os.environ, PT_AMD_NO_TORCH="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr


def test_scene_check_rejects_null():
    lib = pt_amd.load_library()
    assert lib.pt_scene_check(None) == -1
    assert b"null" in lib.pt_last_error()


def test_errors_without_gpu():
    if pt_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pt_amd.PtError) as e:
        pt_amd.Scene(np.zeros(64, np.float32), np.zeros(64, np.float32))
    assert e.value.code == -5  # PT_ERR_NODEVICE
    assert "device" in str(e.value)


def test_invalid_arguments():
    lib = pt_amd.load_library()
    assert lib.pt_scene_create(None, 0, None, 0, 0, None) == -1
    assert b"null" in lib.pt_last_error()
    assert lib.pt_tonemap(None, 0, 1, None) == -1


def test_tonemap_matches_oracle():
    rng = np.random.default_rng(5)
    acc = (rng.exponential(2.0, (37, 41, 3)) * rng.integers(1, 64)).astype(np.float32)
    acc[0, 0] = [np.nan, -1.0, 1e12]
    for runs in (1, 7, 50):
        got = pt_amd.tonemap(acc, runs).reshape(-1)
        want = oracle.tonemap(acc, runs)
        assert np.array_equal(got, want)


def test_render_multi_argument_checks():
    lib = pt_amd.load_library()
    meta = np.zeros(48, np.float32)
    acc = np.zeros(3, np.float32)
    assert lib.pt_render_multi(None, 2, meta.ctypes.data_as(ctypes.c_void_p), 0, 1, 1, 8, 0,
                               acc.ctypes.data_as(ctypes.c_void_p), None) == -1
    arr = (ctypes.c_void_p * 2)(None, None)
    assert lib.pt_render_multi(arr, 2, meta.ctypes.data_as(ctypes.c_void_p), 0, 1, 1, 8, 0,
                               acc.ctypes.data_as(ctypes.c_void_p), None) == -1
    assert lib.pt_render_multi(arr, 0, meta.ctypes.data_as(ctypes.c_void_p), 0, 1, 1, 8, 0,
                               acc.ctypes.data_as(ctypes.c_void_p), None) == -1
