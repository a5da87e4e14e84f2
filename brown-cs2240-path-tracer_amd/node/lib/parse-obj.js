'use strict';
// OBJ + MTL -> SceneObjectGroup.  Mirrors src/ts-util/parse-obj.ts:4-150.
const { mat3_tranpose, mat3_vecmul, mat4_invert, mat4_to_mat3, mat4_vecmul } = require('./geometry');

const last = (a) => a[a.length - 1];

function parse_obj(obj_data, mtl_data, ctm) {
    const object_groups = { vertices: [], vertex_normals: [], objects: [{ name: 'default', indices: [] }] };
    const ctm_inv = mat4_invert(ctm);
    const vm = mat3_tranpose(mat4_to_mat3(ctm_inv));

    for (const raw_line of obj_data.split('\n')) {
        const line = raw_line.replace(/\s+/g, ' ').replace(/#.*$/, '').trim();
        if (line.length === 0) continue;
        if (line[0] === '#') continue;
        else if (line.slice(0, 2) === 'v ') {
            const data = line.slice(2).trim().split(' ').map(parseFloat);
            const t = mat3_vecmul(vm, data);  // parse-obj.ts:24 (translation dropped, as in the reference)
            object_groups.vertices.push(t[0], t[1], t[2]);
        } else if (line.slice(0, 3) === 'vn ') {
            const data = line.slice(3).trim().split(' ').map(parseFloat);
            const t = mat4_vecmul(ctm, data.concat([1.0]));
            object_groups.vertex_normals.push(t[0], t[1], t[2]);
        } else if (line.slice(0, 2) === 'f ') {
            const num_vertices = object_groups.vertices.length / 3;
            const raw_indices = line.slice(2).trim().split(' ').map((triplet) => {
                const i = parseInt(triplet.split('/')[0]);
                if (i > 0) return i;
                return num_vertices + i + 1;
            });
            const cur = last(object_groups.objects);
            if (raw_indices.length === 3) cur.indices.push(...raw_indices);
            else if (raw_indices.length === 4) {
                cur.indices.push(raw_indices[0], raw_indices[1], raw_indices[2]);
                cur.indices.push(raw_indices[0], raw_indices[2], raw_indices[3]);
            } else throw Error('5+ sides encountered');
        } else if (line.slice(0, 6) === 'usemtl') {
            object_groups.objects.push({ name: line.split(' ')[1], indices: [] });
        }
    }
    object_groups.objects = object_groups.objects.filter((o) => o.indices.length > 0);

    const material_map = {};
    let cur_mtl_name = 'default';
    for (const raw_line of mtl_data.split('\n')) {
        const line = raw_line.replace(/\s+/g, ' ').replace(/#.*$/, '').trim();
        if (line.length === 0) continue;
        else if (line[0] === '#') continue;
        else if (line.slice(0, 6) === 'newmtl') {
            cur_mtl_name = line.split(' ')[1];
            material_map[cur_mtl_name] = { Ns: 0, Ni: 0, illum: 0, Ka: [0, 0, 0], Kd: [0, 0, 0], Ks: [0, 0, 0], Ke: [0, 0, 0] };
        } else if (line.slice(0, 2) === 'Ns') material_map[cur_mtl_name]['Ns'] = parseFloat(line.split(' ')[1]);
        else if (line.slice(0, 2) === 'Ni') material_map[cur_mtl_name]['Ni'] = parseFloat(line.split(' ')[1]);
        else if (line.slice(0, 5) === 'illum') material_map[cur_mtl_name]['illum'] = parseFloat(line.split(' ')[1]);
        else if (line.slice(0, 2) === 'Ka') material_map[cur_mtl_name]['Ka'] = line.split(' ').slice(1, 4).map(parseFloat);
        else if (line.slice(0, 2) === 'Kd') material_map[cur_mtl_name]['Kd'] = line.split(' ').slice(1, 4).map(parseFloat);
        else if (line.slice(0, 2) === 'Ks') material_map[cur_mtl_name]['Ks'] = line.split(' ').slice(1, 4).map(parseFloat);
        else if (line.slice(0, 2) === 'Ke') material_map[cur_mtl_name]['Ke'] = line.split(' ').slice(1, 4).map(parseFloat);
    }
    object_groups.objects.forEach((obj) => { obj.material = material_map[obj.name]; });
    return object_groups;
}

module.exports = { parse_obj };
