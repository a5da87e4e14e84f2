'use strict';
// Buffer packing.  Mirrors src/packer.ts:4-137 (layouts: SURVEY.md §8a A15/A16).

/** packer.ts:4-81 — triangle buffer: 16-float header, vertices, (i0,i1,i2,objId) per
 * triangle (1-based), 15-float materials, vertex normals, zero padding (1..16 floats). */
function pack_scene_object_group(g) {
    const object_indices = g.objects.map((o, id) => {
        const ni = [];
        for (let i = 0; i < o.indices.length; i += 3) ni.push(o.indices[i], o.indices[i + 1], o.indices[i + 2], id);
        return ni;
    });
    const object_indices_flat = [].concat(...object_indices);
    const emissive_object_ids = g.objects
        .map((o, i) => (o.material.Ke.some((n) => n > 0) ? i : -1))
        .filter((i) => i !== -1);
    const object_sizes = object_indices.map((ind) => ind.length);
    const object_offsets = object_sizes.reduce((a, v) => { a.push(a[a.length - 1] + v); return a; },
        [16 + g.vertices.length]).slice(0, -1);
    const emissive_offsets = emissive_object_ids.map((i) => [object_offsets[i], object_offsets[i] + object_sizes[i]]);

    const pack_material = (m) => [m.Ns, m.Ni, m.illum, ...m.Ka, ...m.Kd, ...m.Ks, ...m.Ke];
    const packed_materials = [].concat(...g.objects.map((o) => pack_material(o.material)));

    let group = [
        g.vertices.length / 3,
        g.objects.length,
        16,
        16 + g.vertices.length,
        16 + g.vertices.length + object_indices_flat.length,
        16 + g.vertices.length + object_indices_flat.length + packed_materials.length,
        g.vertex_normals.length,
        0,
        ...(emissive_offsets[0] ? emissive_offsets[0] : [-1, -1]),
        ...(emissive_offsets[1] ? emissive_offsets[1] : [-1, -1]),
        ...(emissive_offsets[2] ? emissive_offsets[2] : [-1, -1]),
        ...(emissive_offsets[3] ? emissive_offsets[3] : [-1, -1]),
    ].concat(g.vertices).concat(object_indices_flat).concat(packed_materials).concat(g.vertex_normals);
    const missing_offset = 16 - (group.length % 16);
    group = group.concat(new Array(missing_offset).fill(0));
    return new Float32Array(group);
}

/** packer.ts:83-137 — BVH buffer: 6-float outer bounds, then pre-order nodes of 17 floats
 * (is_leaf, axis, left ptr, right ptr, float count | -2, left AABB, right AABB) + leaf payload. */
function pack_bvh(bvh) {
    const result = [...bvh.outer_bounds.min.toArray(), ...bvh.outer_bounds.max.toArray()];
    const recurse = (node) => {
        const is_leaf = node.is_leaf;
        const children = is_leaf ? [].concat(...node.objects.map((o) => o.obj)) : [];
        const cur_offset = result.length;
        const left_node_offset = cur_offset + 5 + 12 + children.length;
        const right_node_offset_index = cur_offset + 3;
        result.push(
            is_leaf ? 1 : 0,
            node.axis,
            is_leaf ? -1 : left_node_offset,
            -1,
            is_leaf ? children.length : -2,
            ...(node.left_child ? node.left_child.bounds.min.toArray() : [0, 0, 0]),
            ...(node.left_child ? node.left_child.bounds.max.toArray() : [0, 0, 0]),
            ...(node.right_child ? node.right_child.bounds.min.toArray() : [0, 0, 0]),
            ...(node.right_child ? node.right_child.bounds.max.toArray() : [0, 0, 0]),
        );
        for (let i = 0; i < children.length; i++) result.push(children[i]);
        if (!is_leaf && node.left_child) recurse(node.left_child);
        if (!is_leaf && node.right_child) {
            result[right_node_offset_index] = result.length;
            recurse(node.right_child);
        }
    };
    recurse(bvh.root);
    return new Float32Array(result);
}

module.exports = { pack_scene_object_group, pack_bvh };
