/*
 * pt_hip.h — C ABI of the MI355X (gfx950) path-tracing core.
 *
 * Drop-in boundary for the reference's render path (Kauhentus/brown-cs2240-path-tracer):
 * everything behind `programEntry(screenDimension, ctx, primitive_data, camera_data,
 * scene_description)` (src/program-raymarch.ts:50-54) — the WebGPU device/buffer setup
 * (:71-213), the per-frame dispatch + readback + host accumulation loop (:226-335) and the
 * WGSL megakernel it dispatches (src/program-raymarch.wgsl:35-303 with
 * the src/wgsl-util WGSL files) — is replaced by the calls below.  Inputs are the reference's own
 * packed buffers, bit for bit: `SceneObjectPacked.triangle_data` / `.bvh_data`
 * (src/ts-util/data-structs.ts:46-50, produced by src/packer.ts:4-137) and the 48-float
 * meta block (src/program-raymarch.ts:79-92; layout SURVEY.md §8a A2).
 *
 * Conventions: plain pointers and sizes, no torch/HIP types in signatures (streams are
 * `void*` = hipStream_t).  Every function returns PT_OK (0) or a negative pt_status; the
 * message is available from pt_last_error() (thread-local).  Calls on one scene are not
 * re-entrant; distinct scenes may be used from distinct threads.  Ownership: the library
 * owns all device memory of a scene; the caller owns every buffer it passes in.
 *
 * RNG salts: the reference salts each dispatch with the wall-clock `time_elapsed` in ms
 * (program-raymarch.ts:227,246 -> meta[11]); here frame k of a render is salted with
 * t_k = u32(f32(k)) so results are reproducible.  meta[11] is ignored.
 */
#ifndef PT_HIP_H
#define PT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 3

typedef enum {
    PT_OK = 0,
    PT_ERR_INVALID = -1,  /* bad argument (null pointer, zero size, bad meta) */
    PT_ERR_SCENE = -2,    /* malformed packed buffers (see pt_last_error) */
    PT_ERR_NOMEM = -3,    /* device or host allocation failed */
    PT_ERR_HIP = -4,      /* HIP runtime error */
    PT_ERR_NODEVICE = -5  /* no gfx950 device / bad device ordinal */
} pt_status;

typedef enum {
    PT_MODE_AUTO = 0,       /* wavefront at every size on <= 64-entry (mailbox) and big-leaf scenes, else from 2^19 paths (W*H*nframes); megakernel below */
    PT_MODE_MEGAKERNEL = 1, /* one lane per pixel, frames looped in-lane */
    PT_MODE_WAVEFRONT = 2   /* SoA path/ray queues, per-bounce kernels, wave64 compaction */
} pt_mode;

/* Work counters (optional). A "sample" is one camera path with all its bounces
 * and shadow rays; queries count closest-hit traversals. */
typedef struct {
    uint64_t samples;
    uint64_t ext_queries;
    uint64_t shadow_queries;
    uint64_t nodes;      /* BVH nodes popped (each tests 2 child boxes) */
    uint64_t tri_tests;
    uint64_t box_tests;
} pt_counters;

typedef struct {
    uint32_t nodes;        /* internal nodes (root included) */
    uint32_t leaves;
    uint32_t leaf_refs;    /* triangle references in leaves (duplicates included) */
    uint32_t max_leaf;
    uint32_t max_stack;    /* deepest traversal stack the tree can produce */
    uint32_t materials;
    uint32_t emissive_tris;/* Ntri of sample_area_lights */
    uint32_t vertices;
    uint64_t device_bytes; /* HBM held by the scene */
} pt_scene_info;

typedef struct pt_scene pt_scene;

/* Per-kernel launch timing (pt_profile_read). */
typedef struct {
    char name[32];     /* "k_regen", "k_wf_trace", "k_wf_shade_ext", ... */
    uint64_t launches;
    double total_ms;   /* sum over launches of the HIP-event time around each launch */
    double min_ms;
    double max_ms;
    double busy_ms;    /* GPU time during which at least one launch of the kernel ran: the union of the
                          launches' event intervals (launches on several streams overlap, so this is
                          <= total_ms; bytes / busy_ms is the kernel's achieved rate) */
} pt_kernel_time;

/* ABI version of the loaded library (== PT_ABI_VERSION when headers match). */
int pt_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char* pt_last_error(void);

/* Number of visible HIP devices. */
int pt_device_count(int* count_out);

/* Upload a scene.  Replaces the storage-buffer creation of program-raymarch.ts:109-131
 * (bindings 3 and 10).  Validates the packed layouts and re-encodes them for the device
 * (brown-cs2240-path-tracer_amd/csrc/pt_layout.h).  device: HIP ordinal. */
int pt_scene_create(const float* triangle_data, size_t triangle_len, const float* bvh_data, size_t bvh_len,
                    int device, pt_scene** scene_out);
void pt_scene_destroy(pt_scene* scene);
int pt_scene_get_info(const pt_scene* scene, pt_scene_info* info_out);

/* Vertex-normal shading (off by default = the reference's behaviour): the
 * hit normal of a triangle whose third index i2 = (idx2 - 1) * 3 < vn_range (triangle_data[6])
 * becomes normalize(w*n0 + u*n1 + v*n2) with the test's barycentrics and the normals at
 * vn_start + (idx - 1) * 3 (triangle_data[5]) — ray_triangle_intersection_vertex_normals
 * (src/wgsl-util/ray-triangle-intersection.wgsl:44-87), which the reference calls only from
 * commented-out code (src/wgsl-util/intersection-logic.wgsl:81-108).  Changes results on scenes
 * with vertex normals.  Applies to later renders of the scene. */
int pt_scene_set_vertex_normals(pt_scene* scene, int enable);

/* Render frames k = frame0 + i*frame_stride, i < nframes, each 1 spp per pixel, and add
 * clamp(L) (v >= 0 ? v : 0, NaN -> 0) into accum in frame order — the render_loop of
 * program-raymarch.ts:226-335 without the per-frame readback.  accum: host f32
 * [H][W][3], in/out.  max_depth: the literal 16 of `while(depth <= 16)`
 * (program-raymarch.wgsl:118); pass -1 for 16.  counters: nullable.  Blocking. */
int pt_render(pt_scene* scene, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
              int max_depth, int mode, float* accum, pt_counters* counters);

/* Same on device memory, asynchronous on `stream` (hipStream_t; NULL = default stream).
 * d_accum: device f32 [H][W][3] in/out.  d_counters: device pt_counters or NULL (added to).
 * A device-side failure of an earlier asynchronous render of this scene (a traversal wave that
 * gave up, see pt_scene_check) is reported by the next call once that render has completed:
 * this call then fails with PT_ERR_HIP and renders nothing. */
int pt_render_async(pt_scene* scene, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
                    int max_depth, int mode, float* d_accum, pt_counters* d_counters, void* stream);

/* Completion check of the asynchronous calls: waits for every render of the scene to finish
 * (blocking) and reports a device-side failure of any of them — a wavefront traversal wave that
 * gave up after its watchdog limit leaves a flag instead of hanging, and the accumulators of
 * that render are invalid — as PT_ERR_HIP with the wave's state in pt_last_error().  The flag is
 * cleared.  The blocking calls (pt_render, pt_frame, pt_render_image) check it themselves. */
int pt_scene_check(pt_scene* scene);

/* Explicit opt-in (no load-time side effect): ask HIP for `n` hardware queues per process by
 * setting GPU_MAX_HW_QUEUES, which the HIP runtime reads once, when it starts.  Call before any
 * HIP use in the process (the first pt_* call that touches a device starts it); afterwards it
 * has no effect and returns PT_ERR_INVALID.  Hosts that put many streams of their own beside the
 * wavefront's two part streams (e.g. torch) want 8 so the parts do not share a queue. */
int pt_set_hw_queues(int n);

/* Options (process-wide; the library reads no environment variable).  Every value renders the
 * same bits — the parity suite checks each — so they choose kernels and batch shapes only; the
 * defaults are the measured best.  value NULL = back to the default; unknown names and malformed
 * values fail with PT_ERR_INVALID.  Render calls read the options when they start.
 *   "kernel"        auto | mega | wavefront | literal    pipeline (auto = PT_MODE_* and the scene)
 *   "trav"          nested|flat1|pred|lean|lean2|lean4|lean8|lean16|lean32   traversal flavour
 *   "lds" "fastrcp" "dual" "fuse" "fuse_gen" "bf" "mailbox" "bf_stackless" "region_perm"
 *   "leaf_walk" "leaf_pool" "leaf_skip"                                     0 | 1 switches
 *   "parts" "sort" "node_bias" "big_leaf" "bf_slots" "wf_paths" "wf_trace_blocks" "trace_sparse"
 *   "trace_ring" "trace_watchdog" "node_steps" "regen"                      integers
 *                                       (node_steps 1..8: node steps per node turn of the lean
 *                                        traversal; regen: camera batches per region admitted by
 *                                        every extension launch of the fused kernel, 0 = off)
 *   "mb_uid_order"  forward | reverse   (read by pt_scene_create: uid numbering of mailbox scenes)
 *   "leaf_bvh"      integer             (read by pt_scene_create: leaves with a leaf BVH, >= this many entries)
 *   "pool_run"      2 | 4               (entries per run of the pooled leaf turns; default per scene)
 *   "leaf_pre"      0 | 1 | 2           (big leaves resolved before the traversal: never, always,
 *                                        2 = default: where the scene's probe finds it pays)
 *   "pre_ratio"     integer percent     (leaf_pre=2's bar: visited / filtered leaf work, default 50)
 *   "leaf_blocks" "leaf_pairs"          integers (the leaf pass's grid; its pair walk: 0 | 1 | 2)
 *   "leaf_refine"   0 | 1               (the pair walk's second check with the entries' normals)
 *   "reduce"        rccl | ordered      (pt_render_multi's reduction)
 * DESIGN.md §6 describes each.  pt_get_option writes the current value ("" = default) into buf. */
int pt_set_option(const char* name, const char* value);
int pt_get_option(const char* name, char* buf, size_t cap);
void pt_reset_options(void);

/* Destroys the RCCL communicators pt_render_multi made (they are cached per device list; the
 * library also destroys them when the process exits).  Not concurrent with pt_render_multi. */
int pt_release_communicators(void);

/* Identity of the build: the SHA-256 of the sources it was compiled from (csrc/Makefile), so a
 * host can refuse a library that was not built from the tree it runs in. */
const char* pt_build_id(void);

/* Multi-GPU render of one image (the `n_gpus` of §8(b)): scenes[g] is the same
 * packed scene uploaded to device g (pt_scene_create per device, any devices, repeats allowed).
 * Frames k = frame0 + i*frame_stride (i < nframes) are dealt round-robin: scene g renders the i
 * with i % n == g (frame-interleaved: every device sees the same mix of path lengths), each into
 * an f32 accumulator on its own device (scenes[0]'s starts from accum, the others from zero), on
 * one host thread per device; the partial accumulators are then summed onto scenes[0]'s device
 * and copied to accum (host f32 [H][W][3], in/out).
 * Reduction (option "reduce"): "rccl" (default when the devices are distinct and
 * librccl.so.1 loads) = ONE ncclReduce(sum, f32) to device 0 over a communicator made once per
 * device list (ncclCommInitAll, single process) — the summation order is RCCL's; "ordered" (and
 * always with repeated devices) = peer copies added on device 0 in device order,
 * deterministic.  n == 1 is exactly pt_render (with option reduce=rccl: the render and a one-rank
 * RCCL communicator's reduce, the same bits).  counters: nullable, summed over devices.
 * Blocking; the scenes must not be in use by other calls meanwhile. */
int pt_render_multi(pt_scene* const* scenes, int n, const float meta[48], uint32_t frame0, uint32_t nframes,
                    uint32_t frame_stride, int max_depth, int mode, float* accum, pt_counters* counters);

/* One reference dispatch: radiance[H][W][3] = radiance() of every pixel for RNG salt t
 * (the resultMatrix of program-raymarch.wgsl:82-84, before host clamping). */
int pt_frame(pt_scene* scene, const float meta[48], uint32_t t, int max_depth, float* radiance);
int pt_frame_async(pt_scene* scene, const float meta[48], uint32_t t, int max_depth, float* d_radiance, void* stream);

/* Display transform of program-raymarch.ts:295-316 on the host (JS double semantics):
 * raw = acc/sample_runs, lum = mean(raw), out = raw * (lum/(lum+1))^0.01, u8 = ToInt32(out*255)
 * clamped; rgba[i*4+3] = 255. */
int pt_tonemap(const float* accum, size_t npix, uint32_t sample_runs, uint8_t* rgba_out);

/* The same display transform on the device (double, as the JS): d_accum f32 [npix][3] ->
 * d_rgba u8 [npix][4], asynchronous on `stream` (hipStream_t; NULL = default), on the scene's
 * device. */
int pt_tonemap_async(pt_scene* scene, const float* d_accum, size_t npix, uint32_t sample_runs, uint8_t* d_rgba,
                     void* stream);

/* The accumulator (or any n floats) from device memory to PINNED host memory, asynchronous on
 * `stream`: the reference maps its accumulation buffer back to the host after every frame
 * (program-raymarch.ts:262-293).  A copy kernel of a few blocks, so that a readback pipelined
 * with the next render holds few of its CU slots (the runtime's blit copy holds ~512 blocks for
 * the whole PCIe transfer).  Both pointers 16-byte aligned; h_dst must be page-locked
 * (hipHostMalloc / torch pin_memory), else PT_ERR_INVALID. */
int pt_readback_async(pt_scene* scene, const float* d_src, size_t n, float* h_dst, void* stream);

/* programEntry's result in one call: render frames frame0 + i*stride (i < nframes) into a
 * zeroed accumulator and return the displayed image (tone map with sample_runs = nframes)
 * as host RGBA u8 [H][W][4] — only the image crosses PCIe.  counters: nullable.  Blocking. */
int pt_render_image(pt_scene* scene, const float meta[48], uint32_t frame0, uint32_t nframes, uint32_t frame_stride,
                    int max_depth, int mode, uint8_t* rgba_out, pt_counters* counters);

/* Native BVH build (host only, no GPU): the reference's f64 builder
 * (src/ts-util/bvh.ts:14-188) and packer (src/packer.ts:83-137) in C++, byte-identical to them.
 * vertices: x,y,z per vertex in double — the values the host's JS holds after the CTM, not the
 * f32 copies in triangle_data; tris: (i0, i1, i2, material) per triangle, vertex indices
 * 1-based as in the OBJ.  Writes the packed bvh_data floats; *bvh_len = their count.  bvh_cap
 * = 0 asks for the size only; a smaller non-zero bvh_cap fails with PT_ERR_INVALID. */
int pt_bvh_build(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count, float* bvh_out,
                 size_t bvh_cap, size_t* bvh_len);

/* Fast BVH build (SURVEY.md §8(f) row 2's flagged mode; gives up topology parity with the
 * reference's builder): binned SAH over triangle centroids, each triangle in one leaf of at most 8
 * (depth-capped), tight child boxes, written in the same packed layout (src/packer.ts:83-137) so the
 * unchanged traversal runs on it.  Same arguments and size query as pt_bvh_build; fails with
 * PT_ERR_INVALID when the packed buffer would exceed 2^24 floats (offsets are stored as f32). */
int pt_bvh_build_sah(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count, float* bvh_out,
                     size_t bvh_cap, size_t* bvh_len);

/* pt_bvh_build_sah with the triangles of flagged materials (isolate_material[m] != 0 for material
 * id m < material_count; hosts flag the emitters, sum(Ke) > 0) in the root's left child — ONE leaf
 * however many they are, which the traversal tests whenever a ray meets its box (leaf children are
 * never pruned), so the exit-distance pruning of intersection-logic.wgsl:178-181 cannot hide the
 * lights — and the rest of the scene in its right child.  material_count = 0: exactly
 * pt_bvh_build_sah. */
int pt_bvh_build_sah2(const double* vertices, size_t vertex_count, const int32_t* tris, size_t tri_count,
                      const uint8_t* isolate_material, size_t material_count, float* bvh_out, size_t bvh_cap,
                      size_t* bvh_len);

/* Kernel timing (no counterpart in the reference, which has no GPU timing): while enabled,
 * every kernel the scene launches is bracketed by two HIP events on the launch stream (no
 * synchronisation, a few microseconds per launch).  enable != 0 also discards earlier
 * records.  pt_profile_read waits for the recorded events and writes per-kernel totals
 * (at most max_entries; *n_out = entries written). */
int pt_profile_enable(pt_scene* scene, int enable);
/* Record only the launches of one kernel ("k_wf_trace", ...; NULL = all, the default): fewer
 * events in the stream when only one kernel's duration is wanted. */
int pt_profile_select(pt_scene* scene, const char* kernel);
int pt_profile_read(pt_scene* scene, pt_kernel_time* out, int max_entries, int* n_out);

/* Numerics self-test: out[i] = f(a[i], b[i]) evaluated ON THE DEVICE with the core's
 * pinned f32 math (fn ids: 0 sin, 1 cos, 2 tan, 3 acos, 4 log2, 5 exp2, 6 pow, 7 sqrt,
 * 8 div, 9 hash1u, 10 hash1, 11 hash2.x, 12 hash2.y, 13 min, 14 max; hash inputs are the
 * bit patterns of a[i]). */
int pt_selftest_math(int device, int fn, const float* a, const float* b, float* out, size_t n);

/* Exhaustive self-test of the core's division-free reciprocal (pt_math.h rcp_rn, used by the
 * triangle test for 1/det): compares it with IEEE 1.0f/x on the device for every float x whose
 * magnitude bit pattern lies in [lo_bits, hi_bits] (< 0x80000000), both signs.  steps: Newton
 * steps (0..2), -1 = the core's own.  *mismatches = number of differing results;
 * *failing_bits = one failing input (nullable). */
int pt_selftest_rcp(int device, int steps, uint32_t lo_bits, uint32_t hi_bits, uint64_t* mismatches,
                    uint32_t* failing_bits);

/* VALU issue calibration: `reps` timed launches (after one untimed) of a kernel whose threads run 8
 * independent v_fma_f32 chains (packed 1: v_pk_fma_f32, two FMAs per lane each; 2: packed and plain
 * chains interleaved 1 : 2; 32 instructions
 * per iteration, `iters` iterations, no memory operation) at 8 waves per SIMD — the SIMDs issue VALU
 * at their peak rate.  *ms_out = the timed launches' event time; *fma_wave_instr_out (nullable) =
 * their FMA wave-instructions.  Profiled with rocprofv3 PMC it pins the counter formula for the
 * fraction of VALU issue (scripts/calibrate_valu.sh). */
int pt_selftest_valu(int device, int iters, int reps, int packed, double* ms_out, uint64_t* fma_wave_instr_out);

/* Leaf chunks (option leaf_bvh, read by pt_scene_create: leaves of at least that many entries,
 * default 128, 0 = none): leaf `leaf`'s first record, entries and chunks.
 * PT_ERR_INVALID past the last one. */
int pt_scene_leaf_bvh(const pt_scene* scene, int leaf, int32_t* first_record, int32_t* entries, int32_t* nodes);

/* Leaf chunk stress test: nrays rays of family `mode` (0 near the leaf's entries, uniform
 * directions; 1 aimed at them; 2 grazing their planes; 3 leaving their surfaces), each tested
 * against chunked leaf `leaf` by the reference's sequential loop over all entries and by the
 * chunk scheme the traversal uses, with the same closest-t-so-far.  out (host, nrays x 6): loop
 * (position taken or -1, t bits), chunks (position or -1, t bits), entries tested and chunks
 * opened.  mode + 4: the same families through the walk that several rays parked at one leaf share
 * (chunk_leaf_multi), out columns 4-5 zero.  mode 16 + (method << 2 | family): `leaf` indexes the
 * scene's leaves the leaf pass can resolve (the 8 largest; PT_ERR_INVALID past the last) and the
 * pass's own code resolves them — method 0 resolve_leaf one ray per lane, 1 resolve_leaf 8 rays per
 * wave, 2 the (ray, chunk) pair walk without its second check, 3 with it (methods 2-3 need the
 * leaf's pass chunks: PT_ERR_INVALID without) — out columns 2-3 = its key as (position or -1, t
 * bits), 4-5 zero.  Blocking. */
int pt_selftest_leaf(pt_scene* scene, int leaf, int mode, uint32_t seed, uint32_t nrays, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* PT_HIP_H */
