"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/_build/libpt_oracle.so (the C restatement of the
reference's WGSL path tracer, oracle/pt_oracle.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpt_oracle.so")
_LIB_V4_PATH = os.path.join(_HERE, "_build", "libpt_oracle_v4.so")
FLAGS = {_LIB_PATH: "-O3 -march=x86-64-v3 -ffp-contract=off", _LIB_V4_PATH: "-O3 -march=x86-64-v4 -ffp-contract=off"}
_lib = None
_lib_path = None


def _has_avx512() -> bool:
    """x86-64-v4's AVX-512 subsets (F, BW, CD, DQ, VL) on this host's CPU."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    return {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"} <= fl
    except OSError:
        pass
    return False


def lib_flags() -> str:
    """Compiler flags of the oracle build lib() loaded (bench.py's cpu_baseline reports them)."""
    lib()
    return FLAGS[_lib_path]


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("samples", "ext_queries", "shadow_queries", "nodes", "tri_tests", "box_tests")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib, _lib_path
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or not os.path.exists(_LIB_V4_PATH):
            build()
        _lib_path = _LIB_V4_PATH if _has_avx512() and os.environ.get("PT_ORACLE_V3") != "1" else _LIB_PATH
        L = ctypes.CDLL(_lib_path)
        f, u32, i32, p = ctypes.c_float, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        for n in ("po_sinf", "po_cosf", "po_tanf", "po_acosf", "po_log2f", "po_exp2f"):
            getattr(L, n).restype = f; getattr(L, n).argtypes = [f]
        L.po_powf.restype = f; L.po_powf.argtypes = [f, f]
        L.po_hash1u.restype = u32; L.po_hash1u.argtypes = [u32]
        L.po_hash1.restype = f; L.po_hash1.argtypes = [u32]
        L.po_hash2.restype = None; L.po_hash2.argtypes = [u32, p]
        L.po_view_half_h.restype = f; L.po_view_half_h.argtypes = [p]
        L.po_frame.restype = None
        L.po_frame.argtypes = [p, u32, p, u32, p, u32, u32, u32, i32, p, p, i32]
        L.po_render.restype = None
        L.po_render.argtypes = [p, u32, p, u32, p, u32, u32, u32, u32, u32, i32, p, p, i32]
        L.po_ray_bbox.restype = f; L.po_ray_bbox.argtypes = [p, p, p, p]
        L.po_intersect.restype = i32; L.po_intersect.argtypes = [p, u32, p, u32, p, p, p, p]
        L.po_tonemap.restype = None; L.po_tonemap.argtypes = [p, ctypes.c_uint64, u32, p]
        L.po_set_vertex_normals.restype = None; L.po_set_vertex_normals.argtypes = [i32]
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def hash1u(n: int) -> int:
    return int(lib().po_hash1u(n & 0xFFFFFFFF))


def hash1(n: int) -> float:
    return float(lib().po_hash1(n & 0xFFFFFFFF))


def hash2(n: int):
    out = np.zeros(2, np.float32)
    lib().po_hash2(n & 0xFFFFFFFF, _ptr(out))
    return out


def frame(tri, bvh, meta, salt: int, max_depth: int = 16, y0: int = 0, y1: int | None = None, nthreads: int = 0):
    """One reference dispatch (1 spp) with t = salt: returns (radiance[H', W, 3], counters)."""
    tri, bvh, meta = _f32(tri), _f32(bvh), _f32(meta)
    W, H = int(meta[0]), int(meta[1])
    y1 = H if y1 is None else y1
    out = np.zeros((y1 - y0, W, 3), np.float32)
    c = Counters()
    lib().po_frame(_ptr(tri), tri.size, _ptr(bvh), bvh.size, _ptr(meta), y0, y1, salt, max_depth, _ptr(out),
                   ctypes.byref(c), nthreads)
    return out, c.as_dict()


def render(tri, bvh, meta, frame0: int, nframes: int, stride: int = 1, max_depth: int = 16, acc=None,
           y0: int = 0, y1: int | None = None, nthreads: int = 0):
    """Accumulate frames k = frame0 + i*stride (t_k = k) into acc (f32, host loop semantics)."""
    tri, bvh, meta = _f32(tri), _f32(bvh), _f32(meta)
    W, H = int(meta[0]), int(meta[1])
    y1 = H if y1 is None else y1
    if acc is None:
        acc = np.zeros((y1 - y0, W, 3), np.float32)
    assert acc.dtype == np.float32 and acc.flags.c_contiguous and acc.size == (y1 - y0) * W * 3
    c = Counters()
    lib().po_render(_ptr(tri), tri.size, _ptr(bvh), bvh.size, _ptr(meta), y0, y1, frame0, nframes, stride, max_depth,
                    _ptr(acc), ctypes.byref(c), nthreads)
    return acc, c.as_dict()


def intersect(tri, bvh, p, d):
    tri, bvh = _f32(tri), _f32(bvh)
    p4, d4 = _f32(list(p) + [1.0] * (4 - len(p))), _f32(list(d) + [0.0] * (4 - len(d)))
    out = np.zeros(8, np.float32)
    c = Counters()
    hit = lib().po_intersect(_ptr(tri), tri.size, _ptr(bvh), bvh.size, _ptr(p4), _ptr(d4), _ptr(out), ctypes.byref(c))
    return bool(hit), out, c.as_dict()


def ray_bbox(p, d, mn, mx) -> float:
    p4, d4 = _f32(list(p) + [1.0] * (4 - len(p))), _f32(list(d) + [0.0] * (4 - len(d)))
    return float(lib().po_ray_bbox(_ptr(p4), _ptr(d4), _ptr(_f32(mn)), _ptr(_f32(mx))))


def tonemap(acc, sample_runs: int):
    acc = _f32(acc)
    npix = acc.size // 3
    out = np.zeros(npix * 4, np.uint8)
    lib().po_tonemap(_ptr(acc), npix, sample_runs, _ptr(out))
    return out


def math_fn(name: str, x):
    """Vectorised access to the pinned f32 transcendentals (po_sinf, po_acosf, ...)."""
    fn = getattr(lib(), "po_" + name + "f")
    return np.array([fn(float(v)) for v in np.asarray(x, np.float32)], np.float32)


def set_vertex_normals(on: bool):
    """Vertex-normal mode (the reference's commented-out branch, intersection-logic.wgsl:81-108):
    process-wide switch of the oracle library."""
    lib().po_set_vertex_normals(1 if on else 0)
