'use strict';
// f64 BVH builder.  Mirrors src/ts-util/bvh.ts:14-188: longest axis (ties x > y > z),
// 18 split candidates 0.05..0.9000000000000002, cost |nL - avg| + |nR - avg| (first
// minimum wins), inclusive overlap assigns a triangle to BOTH children, leaf if <= 16
// objects or no reduction, max depth 16 (root depth 1).  Topology is part of the
// parity contract: traversal order and pruning depend on it (SURVEY.md §8a A4/A17).
const { Bounds } = require('./geometry');
const { bounds_bounds_intersection_3d, bounds_surface_area } = require('./math');

const MAX_DEPTH = 16;
const MAX_OBJ_PER_NODE = 16;

function split_box(b, axis, coord, low) {
    const box = new Bounds(b.min.clone(), b.max.clone());
    const key = axis === 0 ? 'x' : axis === 1 ? 'y' : 'z';
    if (low) box.max[key] = coord; else box.min[key] = coord;
    return box;
}

class BVH {
    constructor(objects, outer_bounds, opts) {
        this.objects = objects;
        this.outer_bounds = outer_bounds;
        this.quiet = !!(opts && opts.quiet);
        this.construct();
    }

    construct() {
        const stats = { nodes: 0, leaves: 0 };
        const recurse = (node, _axis, depth) => {
            stats.nodes += 1;
            if (depth >= MAX_DEPTH) { node.is_leaf = true; stats.leaves += 1; return; }
            const nb = node.bounds;
            let axis;
            if (nb.stride_x >= nb.stride_y && nb.stride_x >= nb.stride_z) axis = 0;
            else if (nb.stride_y >= nb.stride_x && nb.stride_y >= nb.stride_z) axis = 1;
            else axis = 2;
            const lo = axis === 0 ? nb.min.x : axis === 1 ? nb.min.y : nb.min.z;
            const hi = axis === 0 ? nb.max.x : axis === 1 ? nb.max.y : nb.max.z;

            let split = 0.5;
            const split_step = 0.05;
            let cost = Infinity;
            bounds_surface_area(nb);  // parent_sa: computed but unused by the cost (bvh.ts:193)
            for (let s = split_step; s <= 1.0 - split_step; s += split_step) {
                const w0 = s, w1 = 1.0 - s;
                const c = w0 * hi + w1 * lo;
                const low_box = split_box(nb, axis, c, true);
                const high_box = split_box(nb, axis, c, false);
                let num_low = 0, num_high = 0;
                for (const o of node.objects) {
                    if (bounds_bounds_intersection_3d(o.bounds, low_box)) num_low += 1;
                    if (bounds_bounds_intersection_3d(o.bounds, high_box)) num_high += 1;
                }
                const avg_num = (num_low + num_high) * 0.5;
                const cur_cost = Math.abs(num_low - avg_num) + Math.abs(num_high - avg_num);
                if (cur_cost < cost) { split = s; cost = cur_cost; }
            }
            const c = split * hi + (1.0 - split) * lo;
            const left_bounds = split_box(nb, axis, c, true);
            const right_bounds = split_box(nb, axis, c, false);
            const left_objects = node.objects.filter((o) => bounds_bounds_intersection_3d(o.bounds, left_bounds));
            const right_objects = node.objects.filter((o) => bounds_bounds_intersection_3d(o.bounds, right_bounds));

            node.left_child = { is_leaf: false, axis: -1, bounds: left_bounds, objects: left_objects };
            if (left_objects.length <= MAX_OBJ_PER_NODE || left_objects.length === node.objects.length) {
                node.left_child.is_leaf = true; stats.nodes += 1; stats.leaves += 1;
            } else recurse(node.left_child, axis, depth + 1);

            node.right_child = { is_leaf: false, axis: -1, bounds: right_bounds, objects: right_objects };
            if (right_objects.length <= MAX_OBJ_PER_NODE || right_objects.length === node.objects.length) {
                node.right_child.is_leaf = true; stats.nodes += 1; stats.leaves += 1;
            } else recurse(node.right_child, axis, depth + 1);
        };
        this.root = { is_leaf: false, axis: 0, bounds: this.outer_bounds, objects: this.objects };
        recurse(this.root, 0, 1);
        this.stats = stats;
        if (!this.quiet) {
            console.error(`Constructing BVH with ${this.objects.length} objects`);
            console.error(`    Finished with ${stats.nodes} nodes created`);
            console.error(`    Contains ${stats.leaves} leaf nodes`);
        }
    }
}

module.exports = { BVH, MAX_DEPTH, MAX_OBJ_PER_NODE };
