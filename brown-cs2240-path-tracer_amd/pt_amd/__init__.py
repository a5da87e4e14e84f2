"""pt_amd — Python host binding of the MI355X path-tracing core (libpt_hip.so).

Mirrors the reference's render-path interface (src/program-raymarch.ts:50-54,
`programEntry(screenDimension, ctx, primitive_data, camera_data, scene_description)`)
for Python callers: `Scene` wraps one uploaded `SceneObjectPacked`
(triangle_data + bvh_data, src/ts-util/data-structs.ts:46-50), `Scene.render`
is the render_loop of program-raymarch.ts:226-335 without per-frame readback,
`tonemap` is its display transform (:295-316).

The product path never falls back to CPU code: if libpt_hip.so is missing or
no GPU is visible, calls raise `PtError`.
"""
from ._lib import (  # noqa: F401
    ABI_VERSION,
    MODE_AUTO,
    MODE_MEGAKERNEL,
    MODE_WAVEFRONT,
    Counters,
    PtError,
    Scene,
    SceneInfo,
    abi_version,
    build_id,
    bvh_build,
    device_count,
    get_option,
    lib_path,
    load_library,
    options,
    release_communicators,
    render_multi,
    reset_options,
    selftest_math,
    selftest_rcp,
    selftest_valu,
    set_hw_queues,
    set_option,
    source_hash,
    tonemap,
)
from .host import PackedScene, load_scene, program_entry  # noqa: F401
