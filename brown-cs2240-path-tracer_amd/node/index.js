'use strict';
// Node host of the MI355X path-tracing core.  Same module surface as the reference's
// TypeScript host (src/index.ts, src/packer.ts, src/ts-util/*.ts, src/program-raymarch.ts),
// with programEntry rendering through the HIP core (N-API addon -> libpt_hip.so).
const { parse_ini_file, ini_file_to_ini_scene } = require('./lib/parse-ini');
const { parse_obj } = require('./lib/parse-obj');
const { BVH } = require('./lib/bvh');
const { pack_scene_object_group, pack_bvh } = require('./lib/packer');
const { mat4_rot_axis, bounds_of_vec3, chunk_into_3, bounds_bounds_intersection_3d, bounds_surface_area } = require('./lib/math');
const geometry = require('./lib/geometry');
const { xml2js } = require('./lib/xml');
const scene = require('./lib/scene');
const { programEntry, make_meta, MODE } = require('./lib/program-entry');
const { encode_png } = require('./lib/png');
const addon = require('./lib/addon');

module.exports = {
    parse_ini_file, ini_file_to_ini_scene, parse_obj, BVH, pack_scene_object_group, pack_bvh,
    mat4_rot_axis, bounds_of_vec3, chunk_into_3, bounds_bounds_intersection_3d, bounds_surface_area,
    Vertex: geometry.Vertex, Bounds: geometry.Bounds, xml2js,
    parse_scene_xml: scene.parse_scene_xml, pack_primitive: scene.pack_primitive,
    screen_dimension: scene.screen_dimension, load_scene_from_ini: scene.load_scene_from_ini,
    load_scene_xml_file: scene.load_scene_xml_file,
    programEntry, make_meta, MODE, encode_png, native: addon.load,
};
