"""ctypes binding of include/pt_hip.h (libpt_hip.so, built in-tree by csrc/Makefile)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_FILE = os.path.join(_PKG_ROOT, "lib", "libpt_hip.so")

ABI_VERSION = 3  # include/pt_hip.h PT_ABI_VERSION
_CSRC = os.path.join(_PKG_ROOT, "csrc")
# csrc/Makefile BUILD_SRCS: the sources whose SHA-256 the library carries as pt_build_id()
_BUILD_SRCS = ["pt_kernels.hip", "pt_wavefront.hip", "pt_leafpass.hip", "pt_image.hip", "pt_capi.hip", "pt_math.h", "pt_layout.h",
               "pt_device.h", "pt_path.h", "pt_kernels.h", "../../include/pt_hip.h", "pt_bvh.cpp", "pt_leafbvh.h",
               "pt_leafbvh.cpp", "pt_leafskip.cpp", "Makefile"]
MODE_AUTO, MODE_MEGAKERNEL, MODE_WAVEFRONT = 0, 1, 2
MATH_FNS = ["sin", "cos", "tan", "acos", "log2", "exp2", "pow", "sqrt", "div", "hash1u", "hash1", "hash2x",
            "hash2y", "min", "max"]

_STATUS = {0: "PT_OK", -1: "PT_ERR_INVALID", -2: "PT_ERR_SCENE", -3: "PT_ERR_NOMEM", -4: "PT_ERR_HIP",
           -5: "PT_ERR_NODEVICE"}


class PtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_STATUS.get(code, code)}: {msg}")
        self.code = code


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("samples", "ext_queries", "shadow_queries", "nodes", "tri_tests", "box_tests")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class SceneInfo(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_uint32), ("leaves", ctypes.c_uint32), ("leaf_refs", ctypes.c_uint32),
                ("max_leaf", ctypes.c_uint32), ("max_stack", ctypes.c_uint32), ("materials", ctypes.c_uint32),
                ("emissive_tris", ctypes.c_uint32), ("vertices", ctypes.c_uint32), ("device_bytes", ctypes.c_uint64)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class KernelTime(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_uint64), ("total_ms", ctypes.c_double),
                ("min_ms", ctypes.c_double), ("max_ms", ctypes.c_double), ("busy_ms", ctypes.c_double)]


_lib = None


def lib_path() -> str:
    return _LIB_FILE


def _bind_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64.so (SONAME libamdhip64.so.7, like /opt/rocm's).
    Loading libpt_hip.so first would pull /opt/rocm's runtime and torch would then load a
    second HIP/HSA runtime that finds no GPU.  Importing torch first makes libpt_hip.so bind to
    the runtime already in the process, so device pointers and streams are shared with torch.
    PT_AMD_NO_TORCH=1 skips this (standalone use on /opt/rocm's runtime)."""
    if os.environ.get("PT_AMD_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def source_hash() -> str:
    """SHA-256 of the library's sources as csrc/Makefile computes it (names sorted, contents
    concatenated); pt_build_id() of a library built from this tree returns the same digest."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(_BUILD_SRCS):
        with open(os.path.join(_CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def load_library():
    """Load libpt_hip.so; raise if it was not built, or was built from other sources than the
    tree it sits in (no silent fallback, no stale binary)."""
    global _lib
    if _lib is not None:
        return _lib
    _bind_torch_hip_runtime()
    if not os.path.exists(_LIB_FILE):
        raise PtError(-4, f"{_LIB_FILE} not built (run __graft_entry__.build() or make -C csrc)")
    L = ctypes.CDLL(_LIB_FILE)
    if L.pt_abi_version() != ABI_VERSION:
        raise PtError(-1, f"{_LIB_FILE} has ABI {L.pt_abi_version()}, this binding expects {ABI_VERSION} (rebuild)")
    L.pt_build_id.restype = ctypes.c_char_p
    built, here = L.pt_build_id().decode(), source_hash()
    if built != here:
        raise PtError(-1, f"{_LIB_FILE} was built from other sources (build id {built[:16]}, tree {here[:16]}): "
                          f"run __graft_entry__.build()")
    p, i, u32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_size_t
    L.pt_abi_version.restype = i
    L.pt_last_error.restype = ctypes.c_char_p
    L.pt_device_count.argtypes = [ctypes.POINTER(i)]
    L.pt_scene_create.argtypes = [p, sz, p, sz, i, ctypes.POINTER(p)]
    L.pt_scene_destroy.argtypes = [p]
    L.pt_scene_destroy.restype = None
    L.pt_scene_get_info.argtypes = [p, ctypes.POINTER(SceneInfo)]
    L.pt_render.argtypes = [p, p, u32, u32, u32, i, i, p, p]
    L.pt_render_async.argtypes = [p, p, u32, u32, u32, i, i, p, p, p]
    L.pt_frame.argtypes = [p, p, u32, i, p]
    L.pt_frame_async.argtypes = [p, p, u32, i, p, p]
    L.pt_tonemap.argtypes = [p, sz, u32, p]
    L.pt_selftest_math.argtypes = [i, i, p, p, p, sz]
    L.pt_profile_enable.argtypes = [p, i]
    L.pt_profile_select.argtypes = [p, ctypes.c_char_p]
    L.pt_selftest_rcp.argtypes = [i, i, u32, u32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(u32)]
    L.pt_bvh_build.argtypes = [p, sz, p, sz, p, sz, ctypes.POINTER(sz)]
    L.pt_bvh_build_sah.argtypes = [p, sz, p, sz, p, sz, ctypes.POINTER(sz)]
    L.pt_bvh_build_sah2.argtypes = [p, sz, p, sz, p, sz, p, sz, ctypes.POINTER(sz)]
    L.pt_tonemap_async.argtypes = [p, p, sz, u32, p, p]
    L.pt_readback_async.argtypes = [p, p, sz, p, p]
    L.pt_render_image.argtypes = [p, p, u32, u32, u32, i, i, p, p]
    L.pt_profile_read.argtypes = [p, ctypes.POINTER(KernelTime), i, ctypes.POINTER(i)]
    L.pt_scene_set_vertex_normals.argtypes = [p, i]
    L.pt_scene_check.argtypes = [p]
    L.pt_render_multi.argtypes = [ctypes.POINTER(p), i, p, u32, u32, u32, i, i, p, p]
    L.pt_set_hw_queues.argtypes = [i]
    L.pt_selftest_valu.argtypes = [i, i, i, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.pt_set_option.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.pt_get_option.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz]
    L.pt_reset_options.argtypes = []
    L.pt_reset_options.restype = None
    i32p = ctypes.POINTER(ctypes.c_int32)
    L.pt_scene_leaf_bvh.argtypes = [p, i, i32p, i32p, i32p]
    L.pt_selftest_leaf.argtypes = [p, i, i, u32, u32, p]
    for fn in ("pt_scene_leaf_bvh", "pt_selftest_leaf", "pt_selftest_valu", "pt_set_option", "pt_get_option", "pt_release_communicators", "pt_scene_check", "pt_set_hw_queues", "pt_render_multi", "pt_bvh_build_sah", "pt_bvh_build_sah2", "pt_device_count", "pt_scene_create", "pt_scene_get_info", "pt_render", "pt_render_async", "pt_frame",
               "pt_frame_async", "pt_tonemap", "pt_selftest_math", "pt_profile_enable", "pt_profile_select", "pt_profile_read", "pt_selftest_rcp", "pt_bvh_build", "pt_tonemap_async", "pt_readback_async", "pt_render_image",
               "pt_scene_set_vertex_normals"):
        getattr(L, fn).restype = i
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise PtError(rc, load_library().pt_last_error().decode(errors="replace"))


def abi_version() -> int:
    return int(load_library().pt_abi_version())


def build_id() -> str:
    return load_library().pt_build_id().decode()


def _opt_name(name: str) -> str:
    """Option keys: the C names ("kernel", "trav", ...); the old environment spellings
    ("PT_KERNEL") are accepted and mapped."""
    return name[3:].lower() if name.startswith("PT_") else name


def set_option(name: str, value) -> None:
    """pt_set_option: process-wide kernel-selection switch (value None = default)."""
    v = None if value is None else str(value).encode()
    _check(load_library().pt_set_option(_opt_name(name).encode(), v))


def get_option(name: str) -> str:
    buf = ctypes.create_string_buffer(64)
    _check(load_library().pt_get_option(_opt_name(name).encode(), buf, 64))
    return buf.value.decode()


def reset_options() -> None:
    load_library().pt_reset_options()


class options:
    """Context manager: `with pt_amd.options(kernel="wavefront", trav="lean16"): ...` sets the
    options for the block and restores the previous values after it."""

    def __init__(self, mapping=None, **kv):
        self.kv = {_opt_name(k): v for k, v in {**(mapping or {}), **kv}.items()}
        self.saved = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.saved[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *a):
        for k, v in self.saved.items():
            set_option(k, v or None)


def release_communicators() -> None:
    """pt_release_communicators: destroy the RCCL communicators pt_render_multi cached."""
    _check(load_library().pt_release_communicators())


def set_hw_queues(n: int = 8):
    """Explicit opt-in (pt_set_hw_queues): ask HIP for n hardware queues per process.  Only
    effective before the HIP runtime starts in this process (before torch touches the GPU);
    the library itself never changes the environment."""
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(load_library().pt_device_count(ctypes.byref(n)))
    return n.value


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Scene:
    """One `SceneObjectPacked` resident on one GPU (program-raymarch.ts:109-131)."""

    def __init__(self, triangle_data, bvh_data, device: int = 0):
        self._lib = load_library()
        self.triangle_data = _f32(triangle_data)
        self.bvh_data = _f32(bvh_data)
        self.device = device
        h = ctypes.c_void_p()
        _check(self._lib.pt_scene_create(_ptr(self.triangle_data), self.triangle_data.size, _ptr(self.bvh_data),
                                         self.bvh_data.size, device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_vertex_normals(self, enable: bool = True):
        """Vertex-normal shading (pt_scene_set_vertex_normals; off = the reference's behaviour)."""
        _check(self._lib.pt_scene_set_vertex_normals(self._h, 1 if enable else 0))

    @property
    def info(self) -> dict:
        inf = SceneInfo()
        _check(self._lib.pt_scene_get_info(self._h, ctypes.byref(inf)))
        return inf.as_dict()

    def leaf_bvhs(self) -> list:
        """pt_scene_leaf_bvh: (first record, entries, nodes) of every leaf BVH of the scene."""
        out, k = [], 0
        while True:
            a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
            if self._lib.pt_scene_leaf_bvh(self._h, k, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) != 0:
                return out
            out.append((a.value, b.value, c.value))
            k += 1

    def selftest_leaf(self, leaf: int, mode: int, seed: int, nrays: int) -> np.ndarray:
        """pt_selftest_leaf: [nrays, 6] int32 — the sequential loop's (position or -1, t bits), the
        walk's, the walk's entry tests and nodes (mode + 4: the shared multi-ray walk, no counts)."""
        out = np.zeros((nrays, 6), np.int32)
        _check(self._lib.pt_selftest_leaf(self._h, leaf, mode, seed, nrays, _ptr(out)))
        return out

    def render(self, meta, frame0: int, nframes: int, stride: int = 1, max_depth: int = -1, mode: int = MODE_AUTO,
               accum: np.ndarray | None = None, counters: bool = False):
        """Host-buffer render (blocking). Returns accum [H, W, 3] (and counters if requested)."""
        meta = _f32(meta)
        W, H = int(meta[0]), int(meta[1])
        if accum is None:
            accum = np.zeros((H, W, 3), np.float32)
        if accum.dtype != np.float32 or not accum.flags.c_contiguous or accum.size != W * H * 3:
            raise ValueError("accum must be a contiguous float32 array of H*W*3 elements")
        c = Counters()
        _check(self._lib.pt_render(self._h, _ptr(meta), frame0, nframes, stride, max_depth, mode, _ptr(accum),
                                   ctypes.byref(c) if counters else None))
        return (accum, c.as_dict()) if counters else accum

    def render_async(self, meta, frame0: int, nframes: int, stride: int, max_depth: int, mode: int, d_accum_ptr: int,
                     stream_ptr: int = 0, d_counters_ptr: int = 0):
        """Device render into a caller-owned device buffer (e.g. a torch.cuda tensor's data_ptr())."""
        meta = _f32(meta)
        _check(self._lib.pt_render_async(self._h, _ptr(meta), frame0, nframes, stride, max_depth, mode,
                                         ctypes.c_void_p(d_accum_ptr), ctypes.c_void_p(d_counters_ptr or None),
                                         ctypes.c_void_p(stream_ptr or None)))

    def render_image(self, meta, frame0: int, nframes: int, stride: int = 1, max_depth: int = -1,
                     mode: int = MODE_AUTO, counters: bool = False):
        """programEntry's displayed image in one call: RGBA u8 [H, W, 4] (device tone map)."""
        meta = _f32(meta)
        W, H = int(meta[0]), int(meta[1])
        out = np.zeros((H, W, 4), np.uint8)
        c = Counters()
        _check(self._lib.pt_render_image(self._h, _ptr(meta), frame0, nframes, stride, max_depth, mode, _ptr(out),
                                         ctypes.byref(c) if counters else None))
        return (out, c.as_dict()) if counters else out

    def readback_async(self, d_src_ptr: int, n: int, h_dst_ptr: int, stream_ptr: int = 0):
        """n floats from device memory to pinned host memory on `stream` (pt_readback_async)."""
        _check(self._lib.pt_readback_async(self._h, ctypes.c_void_p(d_src_ptr), n, ctypes.c_void_p(h_dst_ptr),
                                           ctypes.c_void_p(stream_ptr or None)))

    def tonemap_async(self, d_accum_ptr: int, npix: int, sample_runs: int, d_rgba_ptr: int, stream_ptr: int = 0):
        """Device tone map between caller-owned device buffers (e.g. torch tensors)."""
        _check(self._lib.pt_tonemap_async(self._h, ctypes.c_void_p(d_accum_ptr), npix, sample_runs,
                                          ctypes.c_void_p(d_rgba_ptr), ctypes.c_void_p(stream_ptr or None)))

    def check(self):
        """Wait for this scene's renders and raise if one failed on the device (pt_scene_check:
        a wavefront traversal wave that gave up at its watchdog limit)."""
        _check(self._lib.pt_scene_check(self._h))

    def profile_enable(self, enable: bool = True):
        """Bracket every kernel launch of this scene with HIP events (discards earlier records)."""
        _check(self._lib.pt_profile_enable(self._h, 1 if enable else 0))

    def profile_select(self, kernel: str | None = None):
        """Record only `kernel` ("k_wf_trace", "k_regen", ...); None = every kernel."""
        _check(self._lib.pt_profile_select(self._h, kernel.encode() if kernel else None))

    def profile_read(self) -> dict:
        """{kernel name: {"launches", "total_ms", "avg_ms", "min_ms", "max_ms", "busy_ms"}} since
        profile_enable(); busy_ms = union of the launches' intervals (parts on several streams overlap)."""
        buf = (KernelTime * 16)()
        n = ctypes.c_int(0)
        _check(self._lib.pt_profile_read(self._h, buf, 16, ctypes.byref(n)))
        out = {}
        for k in buf[: n.value]:
            out[k.name.decode()] = {"launches": int(k.launches), "total_ms": k.total_ms,
                                    "avg_ms": k.total_ms / max(1, k.launches), "min_ms": k.min_ms, "max_ms": k.max_ms,
                                    "busy_ms": k.busy_ms}
        return out

    def frame(self, meta, t: int, max_depth: int = -1) -> np.ndarray:
        """One reference dispatch: raw radiance [H, W, 3] for RNG salt t."""
        meta = _f32(meta)
        W, H = int(meta[0]), int(meta[1])
        out = np.zeros((H, W, 3), np.float32)
        _check(self._lib.pt_frame(self._h, _ptr(meta), t, max_depth, _ptr(out)))
        return out


def render_multi(scenes, meta, frame0: int, nframes: int, stride: int = 1, max_depth: int = -1,
                 mode: int = MODE_AUTO, accum: np.ndarray | None = None, counters: bool = False):
    """pt_render_multi: one image over several Scenes (one per device, repeats allowed), frames dealt
    round-robin, partial accumulators reduced onto scenes[0]'s device (RCCL, or PT_REDUCE=ordered)."""
    meta = _f32(meta)
    W, H = int(meta[0]), int(meta[1])
    if accum is None:
        accum = np.zeros((H, W, 3), np.float32)
    if accum.dtype != np.float32 or not accum.flags.c_contiguous or accum.size != W * H * 3:
        raise ValueError("accum must be a contiguous float32 array of H*W*3 elements")
    handles = (ctypes.c_void_p * len(scenes))(*[s._h.value for s in scenes])
    c = Counters()
    _check(load_library().pt_render_multi(handles, len(scenes), _ptr(meta), frame0, nframes, stride, max_depth, mode,
                                          _ptr(accum), ctypes.byref(c) if counters else None))
    return (accum, c.as_dict()) if counters else accum


def tonemap(accum, sample_runs: int) -> np.ndarray:
    """program-raymarch.ts:295-316 display transform -> RGBA u8 [..., 4]."""
    acc = _f32(accum)
    npix = acc.size // 3
    out = np.zeros(npix * 4, np.uint8)
    _check(load_library().pt_tonemap(_ptr(acc), npix, sample_runs, _ptr(out)))
    return out.reshape(acc.shape[:-1] + (4,)) if acc.ndim >= 2 else out


def selftest_math(fn: str, a, b=None, device: int = 0) -> np.ndarray:
    a = _f32(a).reshape(-1)
    b = _f32(np.zeros_like(a) if b is None else b).reshape(-1)
    out = np.zeros_like(a)
    _check(load_library().pt_selftest_math(device, MATH_FNS.index(fn), _ptr(a), _ptr(b), _ptr(out), a.size))
    return out


def selftest_rcp(steps: int = -1, lo_bits: int = 0x00800000, hi_bits: int = 0x7E000000, device: int = 0):
    """(mismatches, failing input bits) of the core's reciprocal vs IEEE 1/x for every float whose
    magnitude bits lie in [lo_bits, hi_bits] (default 2^-126..2^125), both signs."""
    L = load_library()
    m = ctypes.c_uint64(0)
    b = ctypes.c_uint32(0)
    _check(L.pt_selftest_rcp(device, steps, lo_bits, hi_bits, ctypes.byref(m), ctypes.byref(b)))
    return int(m.value), int(b.value)


def selftest_valu(iters: int = 20000, reps: int = 5, packed: int = 0, device: int = 0):
    """pt_selftest_valu: (ms of the timed launches, FMA wave-instructions they issued; packed 1:
    v_pk_fma_f32, 2: packed and plain chains interleaved)."""
    ms = ctypes.c_double(0.0)
    n = ctypes.c_uint64(0)
    _check(load_library().pt_selftest_valu(device, iters, reps, int(packed), ctypes.byref(ms), ctypes.byref(n)))
    return float(ms.value), int(n.value)


def bvh_build(vertices, tris, sah: bool = False, isolate=None) -> np.ndarray:
    """Native BVH build + pack (host only, no GPU): vertices f64 [n, 3] (post-CTM), tris
    int32 [m, 4] = (i0, i1, i2, material) with 1-based vertex indices -> packed bvh_data (f32).
    sah=True: the fast binned-SAH tree (pt_bvh_build_sah), same layout, not the reference's tree;
    isolate: per material id a flag (the emitters) — their triangles go under the root's left child
    (pt_bvh_build_sah2)."""
    L = load_library()
    v = np.ascontiguousarray(vertices, dtype=np.float64).reshape(-1)
    t = np.ascontiguousarray(tris, dtype=np.int32).reshape(-1)
    if sah and isolate is not None:
        iso = np.ascontiguousarray(isolate, dtype=np.uint8).reshape(-1)

        def fn(vp, nv, tp, nt, op, cap, nref):
            return L.pt_bvh_build_sah2(vp, nv, tp, nt, _ptr(iso), iso.size, op, cap, nref)
    else:
        fn = L.pt_bvh_build_sah if sah else L.pt_bvh_build
    n = ctypes.c_size_t(0)
    _check(fn(_ptr(v), v.size // 3, _ptr(t), t.size // 4, None, 0, ctypes.byref(n)))
    out = np.empty(n.value, np.float32)
    _check(fn(_ptr(v), v.size // 3, _ptr(t), t.size // 4, _ptr(out), out.size, ctypes.byref(n)))
    return out
