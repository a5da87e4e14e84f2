#!/usr/bin/env node
'use strict';
// pt-render: the reference's browser entry (src/index.ts) as a CLI.  Loads the .ini,
// renders samplesPerPixel frames on the GPU, writes the tone-mapped PNG to IO.output
// (relative to --out-root, default cwd).  Usage: pt-render.js <scene.ini> [--web-root DIR]
// [--out-root DIR] [--max-depth D] [--mode auto|megakernel|wavefront] [--device N] [--spp N]
// [--vertex-normals 1] (smooth shading from the OBJ normals: the reference's commented-out branch)
// [--counters 1] (work counters in the JSON line; runs the kernels' counting builds)
const fs = require('fs');
const path = require('path');
const host = require('..');

async function main(argv) {
    const args = { _: [] };
    for (let i = 0; i < argv.length; i++) {
        if (argv[i].startsWith('--')) args[argv[i].slice(2).replace(/-/g, '_')] = argv[++i];
        else args._.push(argv[i]);
    }
    if (!args._.length) { console.error('usage: pt-render.js <scene.ini> [options]'); process.exit(2); }
    const t0 = Date.now();
    const s = host.load_scene_from_ini(args._[0], { web_root: args.web_root, quiet: true });
    if (args.spp) s.scene_description.Settings.samplesPerPixel = parseInt(args.spp);
    const t1 = Date.now();
    const r = await host.programEntry(s.screenDimension, s.primitive_data, s.camera_data, s.scene_description, {
        device: parseInt(args.device || '0'), maxDepth: parseInt(args.max_depth || '16'), mode: args.mode || 'auto',
        vertexNormals: args.vertex_normals === '1', counters: args.counters === '1',
    });
    const t2 = Date.now();
    const [W, H] = s.screenDimension;
    const out = path.join(args.out_root || '.', s.scene_description.IO.output || 'out.png');
    fs.mkdirSync(path.dirname(out), { recursive: true });
    fs.writeFileSync(out, host.encode_png(r.rgba, W, H));
    const samples = W * H * r.sample_runs;
    console.log(JSON.stringify({ output: out, width: W, height: H, spp: r.sample_runs, scene_ms: t1 - t0,
        render_ms: t2 - t1, msamples_per_s: samples / ((t2 - t1) / 1000) / 1e6, counters: r.counters }));
}
main(process.argv.slice(2)).catch((e) => { console.error(e.stack || String(e)); process.exit(1); });
