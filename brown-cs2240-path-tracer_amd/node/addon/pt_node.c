/*
 * pt_node.c — N-API addon (N-API v8, Node >= 12.22) binding include/pt_hip.h for the Node
 * host.  This is the thin layer between the reference-shaped JS API (node/lib/program-entry.js,
 * replacing src/program-raymarch.ts:50-357) and libpt_hip.so.  Typed arrays are passed
 * through without copies; render() runs as napi_async_work off the event loop and resolves a
 * Promise (the reference's mapAsync().then chain, program-raymarch.ts:273).  Errors become JS
 * Error objects carrying pt_last_error().
 */
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/pt_hip.h"

#define CHECK_NAPI(env, call)                                                  \
    do {                                                                       \
        if ((call) != napi_ok) {                                               \
            napi_throw_error((env), NULL, "N-API call failed: " #call);        \
            return NULL;                                                       \
        }                                                                      \
    } while (0)

static napi_value throw_pt(napi_env env, int rc) {
    char buf[512];
    snprintf(buf, sizeof buf, "pt_hip error %d: %s", rc, pt_last_error());
    napi_throw_error(env, NULL, buf);
    return NULL;
}

static int get_f32(napi_env env, napi_value v, float** data, size_t* len) {
    bool is_ta = false;
    if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return 0;
    napi_typedarray_type t;
    void* p;
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off) != napi_ok || t != napi_float32_array) return 0;
    *data = (float*)p;
    return 1;
}

static int get_u8(napi_env env, napi_value v, uint8_t** data, size_t* len) {
    bool is_ta = false;
    if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return 0;
    napi_typedarray_type t;
    void* p;
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off) != napi_ok ||
        (t != napi_uint8_array && t != napi_uint8_clamped_array))
        return 0;
    *data = (uint8_t*)p;
    return 1;
}

static int get_i32(napi_env env, napi_value v, int32_t* out) { return napi_get_value_int32(env, v, out) == napi_ok; }
static int get_u32(napi_env env, napi_value v, uint32_t* out) { return napi_get_value_uint32(env, v, out) == napi_ok; }

/* A JS scene handle: the library's scene plus the addon's job guard.  Calls on one pt_scene are
 * not re-entrant (include/pt_hip.h), and render()/renderImage() run on libuv worker threads, so
 * a second job on a scene whose job is still running is rejected (busy), and so are
 * renderSync()/frame()/sceneDestroy() while one runs.  All of these checks run on the JS thread,
 * which also clears `busy` when the job completes: no locking needed. */
typedef struct {
    pt_scene* s;
    int busy;
} scene_box;

static void scene_finalize(napi_env env, void* data, void* hint) {
    (void)env; (void)hint;
    scene_box* b = (scene_box*)data;
    if (b->s) pt_scene_destroy(b->s);
    free(b);
}

static scene_box* get_box(napi_env env, napi_value v) {
    void* p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
    return (scene_box*)p;
}

/* the live scene of a handle: NULL (and a pending JS error) if destroyed or busy */
static pt_scene* get_scene(napi_env env, napi_value v) {
    scene_box* b = get_box(env, v);
    if (!b) return NULL;
    if (!b->s) { napi_throw_error(env, NULL, "scene was destroyed (sceneDestroy)"); return NULL; }
    if (b->busy) { napi_throw_error(env, NULL, "scene is busy: a render job on it has not completed"); return NULL; }
    return b->s;
}

static int pending_exception(napi_env env) {
    bool p = false;
    return napi_is_exception_pending(env, &p) == napi_ok && p;
}

static napi_value counters_obj(napi_env env, const pt_counters* c) {
    napi_value o, v;
    napi_create_object(env, &o);
    const char* names[6] = {"samples", "ext_queries", "shadow_queries", "nodes", "tri_tests", "box_tests"};
    const uint64_t vals[6] = {c->samples, c->ext_queries, c->shadow_queries, c->nodes, c->tri_tests, c->box_tests};
    for (int i = 0; i < 6; ++i) {
        napi_create_double(env, (double)vals[i], &v);
        napi_set_named_property(env, o, names[i], v);
    }
    return o;
}

/* abiVersion() -> number */
static napi_value js_abi_version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value r;
    CHECK_NAPI(env, napi_create_int32(env, pt_abi_version(), &r));
    return r;
}

/* setOption(name, value | null) — pt_set_option (kernel-selection switches; null = default) */
static napi_value js_set_option(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    char name[64], value[64];
    size_t n = 0;
    if (argc < 1 || napi_get_value_string_utf8(env, argv[0], name, sizeof name, &n) != napi_ok) {
        napi_throw_type_error(env, NULL, "setOption(name: string, value: string | number | null)");
        return NULL;
    }
    const char* v = NULL;
    napi_valuetype t = napi_undefined;
    if (argc >= 2) CHECK_NAPI(env, napi_typeof(env, argv[1], &t));
    if (t == napi_string) {
        if (napi_get_value_string_utf8(env, argv[1], value, sizeof value, &n) != napi_ok) return NULL;
        v = value;
    } else if (t == napi_number) {
        int64_t x = 0;
        CHECK_NAPI(env, napi_get_value_int64(env, argv[1], &x));
        snprintf(value, sizeof value, "%lld", (long long)x);
        v = value;
    } else if (t != napi_null && t != napi_undefined) {
        napi_throw_type_error(env, NULL, "setOption: value must be a string, a number or null");
        return NULL;
    }
    int rc = pt_set_option(name, v);
    if (rc) return throw_pt(env, rc);
    return NULL;
}

/* deviceCount() -> number */
static napi_value js_device_count(napi_env env, napi_callback_info info) {
    (void)info;
    int n = 0;
    int rc = pt_device_count(&n);
    if (rc) return throw_pt(env, rc);
    napi_value r;
    CHECK_NAPI(env, napi_create_int32(env, n, &r));
    return r;
}

/* sceneCreate(triangle_data: Float32Array, bvh_data: Float32Array, device: number) -> external */
static napi_value js_scene_create(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    float *tri, *bvh;
    size_t tl, bl;
    int32_t dev = 0;
    if (argc < 2 || !get_f32(env, argv[0], &tri, &tl) || !get_f32(env, argv[1], &bvh, &bl) ||
        (argc > 2 && !get_i32(env, argv[2], &dev))) {
        napi_throw_type_error(env, NULL, "sceneCreate(Float32Array triangle_data, Float32Array bvh_data, device?)");
        return NULL;
    }
    pt_scene* s = NULL;
    int rc = pt_scene_create(tri, tl, bvh, bl, dev, &s);
    if (rc) return throw_pt(env, rc);
    scene_box* b = (scene_box*)calloc(1, sizeof(scene_box));
    if (!b) { pt_scene_destroy(s); napi_throw_error(env, NULL, "out of memory"); return NULL; }
    b->s = s;
    napi_value ext;
    if (napi_create_external(env, b, scene_finalize, NULL, &ext) != napi_ok) {
        pt_scene_destroy(s);
        free(b);
        napi_throw_error(env, NULL, "napi_create_external failed");
        return NULL;
    }
    /* V8 cannot see device memory: tell it, so that dropped scenes are collected */
    pt_scene_info si;
    if (pt_scene_get_info(s, &si) == PT_OK) {
        int64_t adj = 0;
        napi_adjust_external_memory(env, (int64_t)si.device_bytes, &adj);
    }
    return ext;
}

/* sceneDestroy(scene): free the scene's device memory now (the handle becomes unusable); throws
 * while a render job on it runs */
static napi_value js_scene_destroy(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    scene_box* b = argc ? get_box(env, argv[0]) : NULL;
    if (!b) { napi_throw_type_error(env, NULL, "sceneDestroy(scene)"); return NULL; }
    if (b->busy) { napi_throw_error(env, NULL, "scene is busy: a render job on it has not completed"); return NULL; }
    if (b->s) {
        pt_scene_info si;
        int have = pt_scene_get_info(b->s, &si) == PT_OK;
        pt_scene_destroy(b->s);
        b->s = NULL;
        if (have) {
            int64_t adj = 0;
            napi_adjust_external_memory(env, -(int64_t)si.device_bytes, &adj);
        }
    }
    return NULL;
}

/* sceneInfo(scene) -> object */
static napi_value js_scene_info(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    pt_scene* s = argc ? get_scene(env, argv[0]) : NULL;
    if (!s) { if (!pending_exception(env)) napi_throw_type_error(env, NULL, "sceneInfo(scene)"); return NULL; }
    pt_scene_info si;
    int rc = pt_scene_get_info(s, &si);
    if (rc) return throw_pt(env, rc);
    napi_value o, v;
    napi_create_object(env, &o);
#define SET(name) napi_create_double(env, (double)si.name, &v); napi_set_named_property(env, o, #name, v);
    SET(nodes) SET(leaves) SET(leaf_refs) SET(max_leaf) SET(max_stack) SET(materials) SET(emissive_tris) SET(vertices)
    SET(device_bytes)
#undef SET
    return o;
}

typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref refs[3]; /* scene, meta, accum kept alive while the worker runs */
    scene_box* box;   /* busy while the job runs */
    pt_scene* scene;
    float meta[48];
    uint32_t frame0, nframes, stride;
    int32_t max_depth, mode;
    float* accum;
    uint8_t* rgba; /* renderImage: the displayed image instead of the accumulator */
    pt_counters counters;
    int want_counters; /* optional last argument (default true): counting builds of the kernels */
    int rc;
    char err[512];
} render_job;

static void render_execute(napi_env env, void* data) {
    (void)env;
    render_job* j = (render_job*)data;
    pt_counters* c = j->want_counters ? &j->counters : NULL;
    j->rc = j->rgba ? pt_render_image(j->scene, j->meta, j->frame0, j->nframes, j->stride, j->max_depth, j->mode, j->rgba, c)
                    : pt_render(j->scene, j->meta, j->frame0, j->nframes, j->stride, j->max_depth, j->mode, j->accum, c);
    if (j->rc) snprintf(j->err, sizeof j->err, "pt_hip error %d: %s", j->rc, pt_last_error());
}

static void render_complete(napi_env env, napi_status status, void* data) {
    render_job* j = (render_job*)data;
    if (j->box) j->box->busy = 0;
    if (status == napi_ok && j->rc == 0) {
        napi_value none;
        napi_get_null(env, &none);
        napi_resolve_deferred(env, j->deferred, j->want_counters ? counters_obj(env, &j->counters) : none);
    } else {
        napi_value msg, e;
        napi_create_string_utf8(env, j->rc ? j->err : "render cancelled", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &e);
        napi_reject_deferred(env, j->deferred, e);
    }
    for (int i = 0; i < 3; ++i) napi_delete_reference(env, j->refs[i]);
    napi_delete_async_work(env, j->work);
    free(j);
}

/* optional boolean argv[8]: work counters wanted (default true) */
static int parse_want_counters(napi_env env, size_t argc, napi_value* argv, render_job* j) {
    bool want = true;
    if (argc > 8) {
        napi_valuetype t;
        if (napi_typeof(env, argv[8], &t) != napi_ok) return 0;
        if (t != napi_undefined && napi_get_value_bool(env, argv[8], &want) != napi_ok) return 0;
    }
    j->want_counters = want ? 1 : 0;
    return 1;
}

/* parse (scene, meta, frame0, nframes, stride, maxDepth, mode, accum[, counters]) */
static int parse_render_args(napi_env env, napi_callback_info info, render_job* j, napi_value argv[9]) {
    size_t argc = 9;
    if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok || argc < 8) return 0;
    if (!parse_want_counters(env, argc, argv, j)) return 0;
    float* meta;
    size_t ml, al;
    j->box = get_box(env, argv[0]);
    j->scene = get_scene(env, argv[0]);
    if (!j->scene || !get_f32(env, argv[1], &meta, &ml) || ml < 48) return 0;
    memcpy(j->meta, meta, sizeof j->meta);
    if (!get_u32(env, argv[2], &j->frame0) || !get_u32(env, argv[3], &j->nframes) || !get_u32(env, argv[4], &j->stride) ||
        !get_i32(env, argv[5], &j->max_depth) || !get_i32(env, argv[6], &j->mode) || !get_f32(env, argv[7], &j->accum, &al))
        return 0;
    if (al != (size_t)j->meta[0] * (size_t)j->meta[1] * 3) return 0;
    return 1;
}

/* render(scene, meta, frame0, nframes, stride, maxDepth, mode, accum[, counters=true]) -> Promise<counters|null> */
static napi_value js_render(napi_env env, napi_callback_info info) {
    napi_value argv[9];
    render_job* j = (render_job*)calloc(1, sizeof(render_job));
    if (!j) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    if (!parse_render_args(env, info, j, argv)) {
        free(j);
        if (!pending_exception(env))
            napi_throw_type_error(env, NULL,
                                  "render(scene, Float32Array meta[48], frame0, nframes, stride, maxDepth, mode, "
                                  "Float32Array accum[W*H*3], counters?)");
        return NULL;
    }
    j->box->busy = 1;
    napi_value promise, name;
    CHECK_NAPI(env, napi_create_promise(env, &j->deferred, &promise));
    napi_create_reference(env, argv[0], 1, &j->refs[0]);
    napi_create_reference(env, argv[1], 1, &j->refs[1]);
    napi_create_reference(env, argv[7], 1, &j->refs[2]);
    napi_create_string_utf8(env, "pt_render", NAPI_AUTO_LENGTH, &name);
    CHECK_NAPI(env, napi_create_async_work(env, NULL, name, render_execute, render_complete, j, &j->work));
    CHECK_NAPI(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* renderMulti([scene, ...], meta, frame0, nframes, stride, maxDepth, mode, accum[, counters=true])
 * -> Promise<counters|null>: one image over one scene per device (pt_render_multi: frames dealt
 * round-robin, partial accumulators reduced onto the first scene's device) */
#define PT_NODE_MAX_DEVICES 64
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref refs[3]; /* scene array, meta, accum */
    scene_box* boxes[PT_NODE_MAX_DEVICES];
    pt_scene* scenes[PT_NODE_MAX_DEVICES];
    int n;
    float meta[48];
    uint32_t frame0, nframes, stride;
    int32_t max_depth, mode;
    float* accum;
    pt_counters counters;
    int want_counters;
    int rc;
    char err[512];
} multi_job;

static void multi_execute(napi_env env, void* data) {
    (void)env;
    multi_job* j = (multi_job*)data;
    j->rc = pt_render_multi(j->scenes, j->n, j->meta, j->frame0, j->nframes, j->stride, j->max_depth, j->mode, j->accum,
                            j->want_counters ? &j->counters : NULL);
    if (j->rc) snprintf(j->err, sizeof j->err, "pt_hip error %d: %s", j->rc, pt_last_error());
}

static void multi_complete(napi_env env, napi_status status, void* data) {
    multi_job* j = (multi_job*)data;
    for (int i = 0; i < j->n; ++i) j->boxes[i]->busy = 0;
    if (status == napi_ok && j->rc == 0) {
        napi_value none;
        napi_get_null(env, &none);
        napi_resolve_deferred(env, j->deferred, j->want_counters ? counters_obj(env, &j->counters) : none);
    } else {
        napi_value msg, e;
        napi_create_string_utf8(env, j->rc ? j->err : "render cancelled", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &e);
        napi_reject_deferred(env, j->deferred, e);
    }
    for (int i = 0; i < 3; ++i) napi_delete_reference(env, j->refs[i]);
    napi_delete_async_work(env, j->work);
    free(j);
}

static napi_value js_render_multi(napi_env env, napi_callback_info info) {
    size_t argc = 9;
    napi_value argv[9];
    multi_job* j = (multi_job*)calloc(1, sizeof(multi_job));
    if (!j) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    int ok = napi_get_cb_info(env, info, &argc, argv, NULL, NULL) == napi_ok && argc >= 8;
    bool is_arr = false;
    uint32_t n = 0;
    if (ok) ok = napi_is_array(env, argv[0], &is_arr) == napi_ok && is_arr &&
                 napi_get_array_length(env, argv[0], &n) == napi_ok && n >= 1 && n <= PT_NODE_MAX_DEVICES;
    for (uint32_t i = 0; ok && i < n; ++i) {
        napi_value e;
        ok = napi_get_element(env, argv[0], i, &e) == napi_ok && (j->boxes[i] = get_box(env, e)) != NULL &&
             (j->scenes[i] = get_scene(env, e)) != NULL;
        for (uint32_t k = 0; ok && k < i; ++k) ok = j->boxes[k] != j->boxes[i];
    }
    j->n = (int)n;
    float* meta = NULL;
    size_t ml = 0, al = 0;
    if (ok) {
        bool want = true;
        if (argc > 8) {
            napi_valuetype t;
            ok = napi_typeof(env, argv[8], &t) == napi_ok && (t == napi_undefined || napi_get_value_bool(env, argv[8], &want) == napi_ok);
        }
        j->want_counters = want ? 1 : 0;
    }
    if (ok) ok = get_f32(env, argv[1], &meta, &ml) && ml >= 48;
    if (ok) {
        memcpy(j->meta, meta, sizeof j->meta);
        ok = get_u32(env, argv[2], &j->frame0) && get_u32(env, argv[3], &j->nframes) && get_u32(env, argv[4], &j->stride) &&
             get_i32(env, argv[5], &j->max_depth) && get_i32(env, argv[6], &j->mode) && get_f32(env, argv[7], &j->accum, &al) &&
             al == (size_t)j->meta[0] * (size_t)j->meta[1] * 3;
    }
    if (!ok) {
        free(j);
        if (!pending_exception(env))
            napi_throw_type_error(env, NULL,
                                  "renderMulti([scene, ...] (distinct handles, <= 64), Float32Array meta[48], frame0, "
                                  "nframes, stride, maxDepth, mode, Float32Array accum[W*H*3], counters?)");
        return NULL;
    }
    for (int i = 0; i < j->n; ++i) j->boxes[i]->busy = 1;
    napi_value promise, name;
    CHECK_NAPI(env, napi_create_promise(env, &j->deferred, &promise));
    napi_create_reference(env, argv[0], 1, &j->refs[0]);
    napi_create_reference(env, argv[1], 1, &j->refs[1]);
    napi_create_reference(env, argv[7], 1, &j->refs[2]);
    napi_create_string_utf8(env, "pt_render_multi", NAPI_AUTO_LENGTH, &name);
    CHECK_NAPI(env, napi_create_async_work(env, NULL, name, multi_execute, multi_complete, j, &j->work));
    CHECK_NAPI(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* renderImage(scene, meta, frame0, nframes, stride, maxDepth, mode, Uint8Array rgba[W*H*4][, counters=true])
 * -> Promise<counters|null>:
 * programEntry's displayed image, tone-mapped on the device (pt_render_image) */
static napi_value js_render_image(napi_env env, napi_callback_info info) {
    size_t argc = 9;
    napi_value argv[9];
    render_job* j = (render_job*)calloc(1, sizeof(render_job));
    if (!j) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    float* meta;
    size_t ml = 0, il = 0;
    int ok = napi_get_cb_info(env, info, &argc, argv, NULL, NULL) == napi_ok && argc >= 8 &&
             parse_want_counters(env, argc, argv, j);
    if (ok) {
        j->box = get_box(env, argv[0]);
        j->scene = get_scene(env, argv[0]);
        ok = j->scene && get_f32(env, argv[1], &meta, &ml) && ml >= 48;
    }
    if (ok) {
        memcpy(j->meta, meta, sizeof j->meta);
        ok = get_u32(env, argv[2], &j->frame0) && get_u32(env, argv[3], &j->nframes) && get_u32(env, argv[4], &j->stride) &&
             get_i32(env, argv[5], &j->max_depth) && get_i32(env, argv[6], &j->mode) && get_u8(env, argv[7], &j->rgba, &il) &&
             il == (size_t)j->meta[0] * (size_t)j->meta[1] * 4;
    }
    if (!ok) {
        free(j);
        if (!pending_exception(env))
            napi_throw_type_error(env, NULL,
                                  "renderImage(scene, Float32Array meta[48], frame0, nframes, stride, maxDepth, mode, "
                                  "Uint8Array rgba[W*H*4])");
        return NULL;
    }
    j->box->busy = 1;
    napi_value promise, name;
    CHECK_NAPI(env, napi_create_promise(env, &j->deferred, &promise));
    napi_create_reference(env, argv[0], 1, &j->refs[0]);
    napi_create_reference(env, argv[1], 1, &j->refs[1]);
    napi_create_reference(env, argv[7], 1, &j->refs[2]);
    napi_create_string_utf8(env, "pt_render_image", NAPI_AUTO_LENGTH, &name);
    CHECK_NAPI(env, napi_create_async_work(env, NULL, name, render_execute, render_complete, j, &j->work));
    CHECK_NAPI(env, napi_queue_async_work(env, j->work));
    return promise;
}

/* renderSync(...same...) -> counters */
static napi_value js_render_sync(napi_env env, napi_callback_info info) {
    napi_value argv[9];
    render_job j;
    memset(&j, 0, sizeof j);
    if (!parse_render_args(env, info, &j, argv)) {
        if (!pending_exception(env))
            napi_throw_type_error(env, NULL, "renderSync(scene, meta, frame0, nframes, stride, maxDepth, mode, accum)");
        return NULL;
    }
    int rc = pt_render(j.scene, j.meta, j.frame0, j.nframes, j.stride, j.max_depth, j.mode, j.accum,
                       j.want_counters ? &j.counters : NULL);
    if (rc) return throw_pt(env, rc);
    napi_value none;
    napi_get_null(env, &none);
    return j.want_counters ? counters_obj(env, &j.counters) : none;
}

/* frame(scene, meta, t, maxDepth, out Float32Array[W*H*3]) */
static napi_value js_frame(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    float *meta, *out;
    size_t ml, ol;
    uint32_t t;
    int32_t md;
    pt_scene* s = argc >= 5 ? get_scene(env, argv[0]) : NULL;
    if (!s || !get_f32(env, argv[1], &meta, &ml) || ml < 48 || !get_u32(env, argv[2], &t) || !get_i32(env, argv[3], &md) ||
        !get_f32(env, argv[4], &out, &ol) || ol != (size_t)meta[0] * (size_t)meta[1] * 3) {
        if (!pending_exception(env)) napi_throw_type_error(env, NULL, "frame(scene, meta, t, maxDepth, Float32Array out[W*H*3])");
        return NULL;
    }
    int rc = pt_frame(s, meta, t, md, out);
    if (rc) return throw_pt(env, rc);
    return NULL;
}

/* tonemap(accum Float32Array, sampleRuns, out Uint8Array[npix*4]) */
static napi_value js_tonemap(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    float* acc;
    uint8_t* out;
    size_t al, ol;
    uint32_t runs;
    if (argc < 3 || !get_f32(env, argv[0], &acc, &al) || !get_u32(env, argv[1], &runs) || !get_u8(env, argv[2], &out, &ol) ||
        ol != al / 3 * 4) {
        napi_throw_type_error(env, NULL, "tonemap(Float32Array accum, sampleRuns, Uint8Array out)");
        return NULL;
    }
    int rc = pt_tonemap(acc, al / 3, runs, out);
    if (rc) return throw_pt(env, rc);
    return NULL;
}

/* bvhBuild(Float64Array vertices, Int32Array tris (i0,i1,i2,mat)[, sah=false[, Uint8Array isolate]])
 * -> Float32Array bvh_data (native twin of node/lib/bvh.js + packer.js:pack_bvh, byte-identical; sah:
 * the fast binned-SAH mode, pt_bvh_build_sah, same layout, not the reference's tree; isolate: per
 * material a flag — the emitters — whose triangles go under the root's left child,
 * pt_bvh_build_sah2) */
static napi_value js_bvh_build(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bool sah = false;
    if (argc > 2) {
        napi_valuetype t;
        if (napi_typeof(env, argv[2], &t) != napi_ok || (t != napi_undefined && napi_get_value_bool(env, argv[2], &sah) != napi_ok)) {
            napi_throw_type_error(env, NULL, "bvhBuild(Float64Array vertices, Int32Array tris, sah?, isolate?)");
            return NULL;
        }
    }
    const uint8_t* iso = NULL;
    size_t niso = 0;
    if (argc > 3) {
        napi_valuetype t;
        napi_typedarray_type ti;
        void* di = NULL;
        size_t oi;
        napi_value abi;
        if (napi_typeof(env, argv[3], &t) != napi_ok ||
            (t != napi_undefined && (napi_get_typedarray_info(env, argv[3], &ti, &niso, &di, &abi, &oi) != napi_ok ||
                                     ti != napi_uint8_array))) {
            napi_throw_type_error(env, NULL, "bvhBuild(..., isolate: Uint8Array of material flags)");
            return NULL;
        }
        iso = (const uint8_t*)di;
    }
    napi_typedarray_type t0, t1;
    size_t n0 = 0, n1 = 0, off;
    void *d0 = NULL, *d1 = NULL;
    napi_value ab;
    if (argc < 2 || napi_get_typedarray_info(env, argv[0], &t0, &n0, &d0, &ab, &off) != napi_ok ||
        napi_get_typedarray_info(env, argv[1], &t1, &n1, &d1, &ab, &off) != napi_ok || t0 != napi_float64_array ||
        t1 != napi_int32_array || n0 % 3 || n1 % 4) {
        napi_throw_type_error(env, NULL, "bvhBuild(Float64Array vertices, Int32Array tris)");
        return NULL;
    }
    size_t len = 0;
    int rc = !sah ? pt_bvh_build((const double*)d0, n0 / 3, (const int32_t*)d1, n1 / 4, NULL, 0, &len)
                  : pt_bvh_build_sah2((const double*)d0, n0 / 3, (const int32_t*)d1, n1 / 4, iso, iso ? niso : 0, NULL, 0, &len);
    if (rc) return throw_pt(env, rc);
    napi_value buf, arr;
    void* data = NULL;
    CHECK_NAPI(env, napi_create_arraybuffer(env, len * sizeof(float), &data, &buf));
    rc = !sah ? pt_bvh_build((const double*)d0, n0 / 3, (const int32_t*)d1, n1 / 4, (float*)data, len, &len)
              : pt_bvh_build_sah2((const double*)d0, n0 / 3, (const int32_t*)d1, n1 / 4, iso, iso ? niso : 0, (float*)data,
                                  len, &len);
    if (rc) return throw_pt(env, rc);
    CHECK_NAPI(env, napi_create_typedarray(env, napi_float32_array, len, buf, 0, &arr));
    return arr;
}

/* profileEnable(scene, bool): bracket every kernel launch of the scene with HIP events */
static napi_value js_profile_enable(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    pt_scene* s = argc ? get_scene(env, argv[0]) : NULL;
    bool on = true;
    if (!s || (argc > 1 && napi_get_value_bool(env, argv[1], &on) != napi_ok)) {
        if (!pending_exception(env)) napi_throw_type_error(env, NULL, "profileEnable(scene, enable)");
        return NULL;
    }
    int rc = pt_profile_enable(s, on ? 1 : 0);
    if (rc) return throw_pt(env, rc);
    return NULL;
}

/* sceneSetVertexNormals(scene, enable): vertex-normal shading (pt_scene_set_vertex_normals) */
static napi_value js_scene_set_vertex_normals(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    pt_scene* s = argc ? get_scene(env, argv[0]) : NULL;
    bool on = true;
    if (!s || (argc > 1 && napi_get_value_bool(env, argv[1], &on) != napi_ok)) {
        if (!pending_exception(env)) napi_throw_type_error(env, NULL, "sceneSetVertexNormals(scene, enable)");
        return NULL;
    }
    int rc = pt_scene_set_vertex_normals(s, on ? 1 : 0);
    if (rc) return throw_pt(env, rc);
    return NULL;
}

/* profileRead(scene) -> {kernel: {launches, totalMs, minMs, maxMs, busyMs}} */
static napi_value js_profile_read(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    pt_scene* s = argc ? get_scene(env, argv[0]) : NULL;
    if (!s) { if (!pending_exception(env)) napi_throw_type_error(env, NULL, "profileRead(scene)"); return NULL; }
    pt_kernel_time kt[16];
    int n = 0;
    int rc = pt_profile_read(s, kt, 16, &n);
    if (rc) return throw_pt(env, rc);
    napi_value o, k, v;
    napi_create_object(env, &o);
    for (int i = 0; i < n; ++i) {
        napi_create_object(env, &k);
        napi_create_double(env, (double)kt[i].launches, &v); napi_set_named_property(env, k, "launches", v);
        napi_create_double(env, kt[i].total_ms, &v); napi_set_named_property(env, k, "totalMs", v);
        napi_create_double(env, kt[i].min_ms, &v); napi_set_named_property(env, k, "minMs", v);
        napi_create_double(env, kt[i].max_ms, &v); napi_set_named_property(env, k, "maxMs", v);
        napi_create_double(env, kt[i].busy_ms, &v); napi_set_named_property(env, k, "busyMs", v);
        napi_set_named_property(env, o, kt[i].name, k);
    }
    return o;
}

static napi_value init(napi_env env, napi_value exports) {
    napi_property_descriptor props[] = {
        {"abiVersion", NULL, js_abi_version, NULL, NULL, NULL, napi_enumerable, NULL},
        {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_enumerable, NULL},
        {"setOption", NULL, js_set_option, NULL, NULL, NULL, napi_enumerable, NULL},
        {"sceneCreate", NULL, js_scene_create, NULL, NULL, NULL, napi_enumerable, NULL},
        {"sceneInfo", NULL, js_scene_info, NULL, NULL, NULL, napi_enumerable, NULL},
        {"sceneDestroy", NULL, js_scene_destroy, NULL, NULL, NULL, napi_enumerable, NULL},
        {"render", NULL, js_render, NULL, NULL, NULL, napi_enumerable, NULL},
        {"renderSync", NULL, js_render_sync, NULL, NULL, NULL, napi_enumerable, NULL},
        {"renderMulti", NULL, js_render_multi, NULL, NULL, NULL, napi_enumerable, NULL},
        {"renderImage", NULL, js_render_image, NULL, NULL, NULL, napi_enumerable, NULL},
        {"frame", NULL, js_frame, NULL, NULL, NULL, napi_enumerable, NULL},
        {"tonemap", NULL, js_tonemap, NULL, NULL, NULL, napi_enumerable, NULL},
        {"profileEnable", NULL, js_profile_enable, NULL, NULL, NULL, napi_enumerable, NULL},
        {"profileRead", NULL, js_profile_read, NULL, NULL, NULL, napi_enumerable, NULL},
        {"bvhBuild", NULL, js_bvh_build, NULL, NULL, NULL, napi_enumerable, NULL},
        {"sceneSetVertexNormals", NULL, js_scene_set_vertex_normals, NULL, NULL, NULL, napi_enumerable, NULL},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
