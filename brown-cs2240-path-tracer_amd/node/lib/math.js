'use strict';
// src/ts-util/math.ts:3-56
const { Bounds, Vertex } = require('./geometry');

/** math.ts:3-12 — theta in radians (the reference passes the XML's degrees unchanged) */
function mat4_rot_axis(x, y, z, theta) {
    const ct = Math.cos(theta);
    const st = Math.sin(theta);
    return [
        ct + x * x * (1 - ct), x * y * (1 - ct) + z * st, x * z * (1 - ct) - y * st, 0,
        x * y * (1 - ct) - z * st, ct + y * y * (1 - ct), y * z * (1 - ct) + x * st, 0,
        x * z * (1 - ct) + y * st, y * z * (1 - ct) - x * st, ct + z * z * (1 - ct), 0,
        0, 0, 0, 1,
    ];
}

/** math.ts:14-34 */
function bounds_of_vec3(vertices) {
    const min = vertices[0].slice(0);
    const max = vertices[0].slice(0);
    for (const v of vertices) {
        if (v[0] <= min[0]) min[0] = v[0];
        if (v[0] >= max[0]) max[0] = v[0];
        if (v[1] <= min[1]) min[1] = v[1];
        if (v[1] >= max[1]) max[1] = v[1];
        if (v[2] <= min[2]) min[2] = v[2];
        if (v[2] >= max[2]) max[2] = v[2];
    }
    return new Bounds(new Vertex(min[0], min[1], min[2]), new Vertex(max[0], max[1], max[2]));
}

/** math.ts:36-43 */
function chunk_into_3(array) {
    if (array.length % 3 !== 0) throw Error("Attempted to chunk non-3 multiple length array into 3's");
    const result = [];
    for (let i = 0; i < array.length; i += 3) result.push([array[i], array[i + 1], array[i + 2]]);
    return result;
}

/** math.ts:45-49 (inclusive overlap) */
function bounds_bounds_intersection_3d(b1, b2) {
    return (b2.min.x <= b1.max.x && b1.min.x <= b2.max.x) &&
        (b2.min.y <= b1.max.y && b1.min.y <= b2.max.y) &&
        (b2.min.z <= b1.max.z && b1.min.z <= b2.max.z);
}

/** math.ts:51-56 */
function bounds_surface_area(b) {
    const sx = b.stride_x, sy = b.stride_y, sz = b.stride_z;
    return 2 * (sx * sy + sy * sz + sx * sz);
}

module.exports = { mat4_rot_axis, bounds_of_vec3, chunk_into_3, bounds_bounds_intersection_3d, bounds_surface_area };
