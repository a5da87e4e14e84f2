'use strict';
// programEntry counterpart (src/program-raymarch.ts:50-357) on the HIP core.
//   * meta block: program-raymarch.ts:55-92 (48 f32, layout SURVEY.md §8a A2)
//   * scene buffers: pt_scene_create replaces the storage buffers of :109-131
//   * render_loop (:226-335): all spp frames in one device call (or `chunk`-sized calls
//     reporting progress), t_k = k instead of the wall-clock ms, host accumulation moved
//     onto the device; the display transform (:295-316) is `tonemap`.
const { camera_matrices } = require('./geometry');
const { load } = require('./addon');

const MODE = { auto: 0, megakernel: 1, wavefront: 2 };

/** program-raymarch.ts:55-92 */
function make_meta(screenDimension, camera_data, scene_description, time_elapsed) {
    const [W, H] = screenDimension;
    const screen_dimension_inv = [1 / W, 1 / H];
    const camera_position = camera_data.pos;
    const camera_look = camera_data.focus.sub_v(camera_position).normalize();
    const FOV = camera_data.heightangle;
    const focal_length = 1;
    const aspect_ratio = W / H;
    const { world_to_cam, cam_to_world } = camera_matrices(camera_position, camera_look, camera_data.up);
    const s = scene_description.Settings;
    return new Float32Array([
        W, H, focal_length, FOV * Math.PI / 180, ...camera_position.toArray(), 1,
        ...screen_dimension_inv, aspect_ratio, time_elapsed || 0,
        ...world_to_cam, ...cam_to_world,
        s.samplesPerPixel, s.pathContinuationProb, s.directLightingOnly ? 1 : -1, 0,
    ]);
}

/**
 * programEntry(screenDimension, primitive_data, camera_data, scene_description, options?)
 *   -> Promise<{accum: Float32Array(W*H*3), sample_runs, rgba: Uint8ClampedArray(W*H*4), counters, scene_info}>
 * options: {device=0, devices=[...] (several GPUs: pt_render_multi), maxDepth=16, mode='auto', frame0=0, chunk=spp,
 *           onFrames(done, total), imageOnly=false,
 *           vertexNormals=false (the reference's commented-out smooth-normal branch; changes results),
 *           counters=false (work counters: the kernels' counting builds, slower; counters is null without)}
 * imageOnly: render and tone-map on the device in one call and return only {rgba, counters, ...}
 * (no accumulator crosses PCIe; pt_render_image).
 * As in the reference only primitive_data[0] is rendered (program-raymarch.wgsl:31,33).
 */
async function programEntry(screenDimension, primitive_data, camera_data, scene_description, options) {
    const o = Object.assign({ device: 0, maxDepth: 16, mode: 'auto', frame0: 0 }, options || {});
    const pt = load();
    const [W, H] = screenDimension;
    const meta = make_meta(screenDimension, camera_data, scene_description, 0);
    const mode = typeof o.mode === 'number' ? o.mode : MODE[o.mode];
    if (mode === undefined) throw Error(`unknown mode ${o.mode}`);
    if (o.devices && o.devices.length > 1) return programEntryMulti(pt, meta, W, H, primitive_data, scene_description, o, mode);
    const scene = pt.sceneCreate(primitive_data[0].triangle_data, primitive_data[0].bvh_data,
                                 o.devices && o.devices.length ? o.devices[0] : o.device);
    // the scene's device memory (scene + wavefront state) is released when the call ends, not
    // when V8 happens to collect the handle
    try {
        if (o.vertexNormals) pt.sceneSetVertexNormals(scene, true);
        const spp = scene_description.Settings.samplesPerPixel;
        const chunk = Math.max(1, o.chunk || spp);
        const scene_info = pt.sceneInfo(scene);
        if (o.imageOnly) {
            const rgba = new Uint8ClampedArray(W * H * 4);
            const c = await pt.renderImage(scene, meta, o.frame0, spp, 1, o.maxDepth, mode, new Uint8Array(rgba.buffer),
                                           !!o.counters);
            return { accum: null, sample_runs: spp, rgba, counters: c, scene_info };
        }
        const accum = new Float32Array(W * H * 3);
        const counters = { samples: 0, ext_queries: 0, shadow_queries: 0, nodes: 0, tri_tests: 0, box_tests: 0 };
        for (let done = 0; done < spp; done += chunk) {
            const n = Math.min(chunk, spp - done);
            const c = await pt.render(scene, meta, o.frame0 + done, n, 1, o.maxDepth, mode, accum, !!o.counters);
            if (c) for (const k of Object.keys(counters)) counters[k] += c[k];
            if (o.onFrames) o.onFrames(done + n, spp);
        }
        const rgba = new Uint8ClampedArray(W * H * 4);
        pt.tonemap(accum, spp, rgba);
        return { accum, sample_runs: spp, rgba, counters: o.counters ? counters : null, scene_info };
    } finally {
        pt.sceneDestroy(scene);
    }
}

// options.devices = [d0, d1, ...]: the scene on every device, frames dealt round-robin and the
// partial accumulators reduced onto d0 (pt_render_multi: RCCL over xGMI for distinct devices)
async function programEntryMulti(pt, meta, W, H, primitive_data, scene_description, o, mode) {
    const scenes = [];
    try {
        for (const d of o.devices) scenes.push(pt.sceneCreate(primitive_data[0].triangle_data, primitive_data[0].bvh_data, d));
        if (o.vertexNormals) for (const s of scenes) pt.sceneSetVertexNormals(s, true);
        const spp = scene_description.Settings.samplesPerPixel;
        const scene_info = pt.sceneInfo(scenes[0]);
        const accum = new Float32Array(W * H * 3);
        const counters = await pt.renderMulti(scenes, meta, o.frame0, spp, 1, o.maxDepth, mode, accum, !!o.counters);
        if (o.onFrames) o.onFrames(spp, spp);
        const rgba = new Uint8ClampedArray(W * H * 4);
        pt.tonemap(accum, spp, rgba);
        return { accum, sample_runs: spp, rgba, counters: o.counters ? counters : null, scene_info, devices: o.devices.slice() };
    } finally {
        for (const s of scenes) pt.sceneDestroy(s);
    }
}

module.exports = { programEntry, make_meta, MODE };
