#!/usr/bin/env node
'use strict';
// pt-pack: scene (.ini or .xml) -> packed buffers on disk, for non-JS callers (Python
// bench/tests).  Writes <out>/triangle_data.f32, <out>/bvh_data.f32 (little-endian f32,
// the reference's SceneObjectPacked) and <out>/scene.json (meta[48], screenDimension,
// camera, settings) plus <out>/meta.f32.  Usage: pt-pack.js <scene.ini|scene.xml> <out_dir> [--web-root DIR]
//                            [--width W --height H --spp N --rr P --direct-only --native-bvh --all-meshes]
// --native-bvh builds the BVH with the library's C++ builder (pt_bvh_build, byte-identical).
// --all-meshes packs every primitive of the scene into one (the reference packs the first only).
// --bvh sah builds the fast binned-SAH tree (same layout, not the reference's topology).
const fs = require('fs');
const path = require('path');
const host = require('..');

function main(argv) {
    const args = { _: [] };
    for (let i = 0; i < argv.length; i++) {
        const a = argv[i];
        if (a === '--direct-only') args.direct_only = true;
        else if (a === '--native-bvh') args.native_bvh = true;
        else if (a === '--all-meshes') args.all_meshes = true;
        else if (a.startsWith('--')) args[a.slice(2).replace(/-/g, '_')] = argv[++i];
        else args._.push(a);
    }
    if (args._.length < 2) { console.error('usage: pt-pack.js <scene.ini|scene.xml> <out_dir> [options]'); process.exit(2); }
    const [src, out] = args._;
    const opts = { web_root: args.web_root, quiet: true, native_bvh: !!args.native_bvh, all_meshes: !!args.all_meshes,
                   bvh: args.bvh || 'reference' };
    if (opts.bvh !== 'reference' && opts.bvh !== 'sah') { console.error('--bvh reference|sah'); process.exit(2); }
    let loaded;
    if (src.endsWith('.ini')) loaded = host.load_scene_from_ini(src, opts);
    else {
        loaded = host.load_scene_xml_file(src, opts);
        loaded.scene_description = { IO: { scene: src, output: '' }, Settings: {
            directLightingOnly: false, imageWidth: 512, imageHeight: 512, numDirectLightingSamples: 1,
            pathContinuationProb: 0.9, samplesPerPixel: 16 } };
    }
    const S = loaded.scene_description.Settings;
    if (args.width) S.imageWidth = parseInt(args.width);
    if (args.height) S.imageHeight = parseInt(args.height);
    if (args.spp) S.samplesPerPixel = parseInt(args.spp);
    if (args.rr) S.pathContinuationProb = parseFloat(args.rr);
    if (args.direct_only) S.directLightingOnly = true;
    const screenDimension = host.screen_dimension(S);
    const meta = host.make_meta(screenDimension, loaded.camera_data, loaded.scene_description, 0);
    fs.mkdirSync(out, { recursive: true });
    const p = loaded.primitive_data[0];
    const wr = (name, ta) => fs.writeFileSync(path.join(out, name), Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength));
    wr('triangle_data.f32', p.triangle_data);
    wr('bvh_data.f32', p.bvh_data);
    wr('meta.f32', meta);  // binary too: JSON cannot carry -0.0
    fs.writeFileSync(path.join(out, 'scene.json'), JSON.stringify({
        meta: Array.from(meta), screenDimension, settings: S, io: loaded.scene_description.IO,
        camera: { pos: loaded.camera_data.pos.toArray(), focus: loaded.camera_data.focus.toArray(),
            up: loaded.camera_data.up.toArray(), heightangle: loaded.camera_data.heightangle },
        triangle_len: p.triangle_data.length, bvh_len: p.bvh_data.length, meshes: loaded.meshes, bvh: opts.bvh,
    }, null, 1));
}
main(process.argv.slice(2));
