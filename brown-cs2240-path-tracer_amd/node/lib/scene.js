'use strict';
// Scene loading: INI -> XML (camera + object tree) -> first mesh -> OBJ/MTL -> packed
// triangle buffer + f64 BVH -> packed BVH.  Mirrors src/index.ts:24-176 (browser XHR
// replaced by fs; the canvas is gone).  Like the reference, only the FIRST primitive
// of the traversal is packed (index.ts:116) unless opts.all_meshes merges them all.
const fs = require('fs');
const path = require('path');
const { parse_ini_file, ini_file_to_ini_scene } = require('./parse-ini');
const { xml2js } = require('./xml');
const { Vertex, mat4_matmul, mat4_scale, mat4_translate } = require('./geometry');
const { bounds_of_vec3, chunk_into_3, mat4_rot_axis } = require('./math');
const { parse_obj } = require('./parse-obj');
const { pack_bvh, pack_scene_object_group } = require('./packer');
const { BVH } = require('./bvh');

const as_array = (x) => (Array.isArray(x) ? x : [x]);

/** load-file.ts:1-14 counterpart: a web-root path ('/scene_assets/...') or a filesystem
 * path -> file text; rejects like the reference's 404 ("file error"). */
function make_loader(web_root) {
    return (p) => {
        const candidates = [path.join(web_root, p.replace(/^\/+/, '')), p];
        for (const c of candidates) if (fs.existsSync(c) && fs.statSync(c).isFile()) return fs.readFileSync(c, 'utf8');
        throw Error(`file error: ${p}`);
    };
}

/** index.ts:30-113: camera + primitive list (with CTMs) from the scene XML text. */
function parse_scene_xml(scene_xml) {
    const scene_root = xml2js(scene_xml)['scenefile'];
    if (!scene_root) throw Error('not a <scenefile>');
    const cd = scene_root['cameradata'];
    const a3 = (a) => new Vertex(parseFloat(a.x), parseFloat(a.y), parseFloat(a.z));
    const camera_data = {
        focus: a3(cd.focus._attributes),
        heightangle: parseFloat(cd.heightangle._attributes.v),
        pos: a3(cd.pos._attributes),
        up: a3(cd.up._attributes),
    };
    const final_primitives = [];
    const traverse = (obj, ctm) => {
        if (obj._attributes.type === 'tree') {
            const objects = as_array(obj.object).filter((o) => o !== undefined);
            const final_objects = objects.map((o) => traverse(o, ctm));
            if (obj.transblock) {
                as_array(obj.transblock).forEach((tb) => {
                    let new_ctm = ctm;
                    if (tb.rotate) {
                        const at = tb.rotate._attributes;
                        new_ctm = mat4_matmul(mat4_rot_axis(parseFloat(at.x), parseFloat(at.y), parseFloat(at.z),
                            parseFloat(at.angle)), new_ctm);
                    }
                    if (tb.scale) {
                        const at = tb.scale._attributes;
                        new_ctm = mat4_matmul(mat4_scale(parseFloat(at.x), parseFloat(at.y), parseFloat(at.z)), new_ctm);
                    }
                    if (tb.translate) {
                        const at = tb.translate._attributes;
                        new_ctm = mat4_matmul(mat4_translate(parseFloat(at.x), parseFloat(at.y), parseFloat(at.z)), new_ctm);
                    }
                    const inner = as_array(tb.object).map((o) => traverse(o, new_ctm));
                    final_objects.push(...inner);
                });
            }
            return { type: 'tree', name: obj._attributes.name, child_objects: final_objects, ctm };
        } else if (obj._attributes.type === 'primitive') {
            const primitive = {
                type: 'primitive', name: obj._attributes.name,
                data: { path: '/scene_assets/' + obj._attributes.filename }, child_objects: [], ctm,
            };
            final_primitives.push(primitive);
            return primitive;
        }
        throw Error('unknown type of object ' + obj._attributes.type + ' to parse');
    };
    as_array(scene_root.object).map((o) => traverse(o, mat4_scale(1, 1, 1)));
    return { camera_data, final_primitives };
}

/** index.ts:128-161 for one primitive: SceneObjectPacked {triangle_data, bvh_data, bounds}. */
function pack_primitive(obj_data, mtl_data, ctm, opts) {
    return pack_group(parse_obj(obj_data, mtl_data, ctm), opts);
}

/** Several primitives (each parsed with its own CTM, parse-obj.ts:24's transform included) as ONE
 * SceneObjectGroup: vertices concatenated, a later mesh's 1-based indices shifted by the vertices
 * before it, objects (and their materials) in primitive order — so the emissive slots are the first
 * four emissive objects over all meshes (packer.ts:65-68).  Vertex normals are laid out per vertex
 * (each mesh's list cut or zero-padded to 3 per vertex) so that vn_start + (index - 1) * 3 still
 * finds a vertex's normal (intersection-logic.wgsl:81-97). */
function merge_groups(groups) {
    const out = { vertices: [], vertex_normals: [], objects: [] };
    for (const g of groups) {
        const base = out.vertices.length / 3;
        const nv = g.vertices.length / 3;
        // an index loop, not push(...g.vertices): spreading a large mesh as call arguments exceeds
        // V8's argument limit (RangeError)
        for (let i = 0; i < g.vertices.length; i++) out.vertices.push(g.vertices[i]);
        for (let i = 0; i < 3 * nv; i++) out.vertex_normals.push(i < g.vertex_normals.length ? g.vertex_normals[i] : 0);
        for (const o of g.objects) out.objects.push(Object.assign({}, o, { indices: o.indices.map((v) => v + base) }));
    }
    return out;
}

/** SceneObjectGroup -> SceneObjectPacked (index.ts:130-161). */
function pack_group(intermediate, opts) {
    for (const o of intermediate.objects)
        if (!o.material) throw TypeError(`material '${o.name}' is not defined in the MTL file`);
    const packed_array = pack_scene_object_group(intermediate);
    const vertices = intermediate.vertices;
    const bvh_bounds = bounds_of_vec3(chunk_into_3(vertices));
    const bvh_objects = [];
    intermediate.objects.forEach((o, mat_i) => {
        const ind = o.indices;
        for (let i = 0; i < ind.length; i += 3) {
            const i0 = (ind[i] - 1) * 3, i1 = (ind[i + 1] - 1) * 3, i2 = (ind[i + 2] - 1) * 3;
            const tri = [vertices.slice(i0, i0 + 3), vertices.slice(i1, i1 + 3), vertices.slice(i2, i2 + 3)];
            bvh_objects.push({ obj: [ind[i], ind[i + 1], ind[i + 2], mat_i], bounds: bounds_of_vec3(tri) });
        }
    });
    // native_bvh: the same build in C++ (pt_bvh_build), byte-identical, for big meshes; bvh 'sah':
    // the fast binned-SAH tree (pt_bvh_build_sah2) in the same layout — not the reference's topology —
    // with the emitters (sum(Ke) > 0, program-raymarch.wgsl:136) in a leaf under the root, where the
    // exit-distance pruning of the unchanged traversal cannot hide them
    if (opts && (opts.native_bvh || opts.bvh === 'sah')) {
        const tris = new Int32Array(bvh_objects.length * 4);
        bvh_objects.forEach((o, t) => tris.set(o.obj, 4 * t));
        const emit = Uint8Array.from(intermediate.objects.map((o) => {
            const ke = o.material.Ke || [0, 0, 0];
            return ke[0] + ke[1] + ke[2] > 0 ? 1 : 0;
        }));
        const bvh_data = require('./addon').load().bvhBuild(Float64Array.from(vertices), tris, opts.bvh === 'sah',
                                                             opts.bvh === 'sah' ? emit : undefined);
        return { triangle_data: packed_array, bvh_data, bounds: bvh_bounds };
    }
    const bvh = new BVH(bvh_objects, bvh_bounds, opts);
    return { triangle_data: packed_array, bvh_data: pack_bvh(bvh), bounds: bvh_bounds };
}

/** index.ts:173-176 */
function screen_dimension(settings) {
    const x_res = settings.imageWidth;
    const aspect_ratio = x_res / settings.imageHeight;
    const round_4 = (n) => Math.floor(n / 4) * 4;
    return [round_4(x_res), round_4(x_res / aspect_ratio)];
}

/**
 * index.ts:24-176 without the canvas: returns the four arguments programEntry takes
 * (screenDimension, primitive_data, camera_data, scene_description).
 * opts.web_root: directory that plays the web server root ('/scene_assets/...' resolve under it).
 */
function load_scene_from_ini(ini_path, opts) {
    opts = opts || {};
    const web_root = opts.web_root || path.resolve(path.dirname(ini_path), '..', '..');
    const load_file = make_loader(web_root);
    const scene_description = ini_file_to_ini_scene(parse_ini_file(fs.readFileSync(ini_path, 'utf8')));
    const loaded = load_scene_xml_file(scene_description.IO.scene, Object.assign({}, opts, { web_root, load_file }));
    return Object.assign(loaded, { screenDimension: screen_dimension(scene_description.Settings), scene_description });
}

/** Scene XML (web-root path or fs path) -> {primitive_data, camera_data}. */
function load_scene_xml_file(scene_path, opts) {
    opts = opts || {};
    const web_root = opts.web_root || path.resolve(path.dirname(scene_path), '..');
    const load_file = opts.load_file || make_loader(web_root);
    const { camera_data, final_primitives } = parse_scene_xml(load_file(scene_path));
    const popts = { quiet: opts.quiet !== false, native_bvh: !!opts.native_bvh, bvh: opts.bvh };
    const parse = (p) => {
        if (!p.data) throw Error('mesh primitive missing its data');
        const obj_data = load_file(p.data.path);
        let mtl_data;
        try { mtl_data = load_file(p.data.path.slice(0, -3) + 'mtl'); } catch (e) { mtl_data = ''; }
        return parse_obj(obj_data, mtl_data, p.ctm);
    };
    // opts.all_meshes: every primitive of the scene in one packed scene (SURVEY.md §8(f) row 1); the
    // default is the reference's first primitive only (index.ts:116)
    const primitive_data = opts.all_meshes
        ? [pack_group(merge_groups(final_primitives.map(parse)), popts)]
        : final_primitives.slice(0, 1).map((p) => pack_group(parse(p), popts));
    return { primitive_data, camera_data, meshes: opts.all_meshes ? final_primitives.length : Math.min(1, final_primitives.length) };
}

module.exports = { parse_scene_xml, pack_primitive, pack_group, merge_groups, screen_dimension, load_scene_from_ini,
                   load_scene_xml_file };
