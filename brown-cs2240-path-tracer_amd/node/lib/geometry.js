'use strict';
// The subset of @toysinbox3dprinting/js-geometry the reference host uses
// (Vertex, Bounds, mat4/mat3 helpers, world_to_camera).  That package is not
// vendored and its version is unpinned (package.json:19, no lockfile), so the
// conventions here are an explicit choice (SURVEY.md §8c): 4x4 matrices are
// row-major arrays with column vectors (translation at [3], [7], [11]);
// camera matrices handed to the device are column-major WGSL mat4x4 arrays.

class Vertex {
    constructor(x, y, z) { this.x = x; this.y = y; this.z = z; }
    clone() { return new Vertex(this.x, this.y, this.z); }
    toArray() { return [this.x, this.y, this.z]; }
    sub_v(o) { return new Vertex(this.x - o.x, this.y - o.y, this.z - o.z); }
    normalize() {
        const l = Math.sqrt(this.x * this.x + this.y * this.y + this.z * this.z);
        return new Vertex(this.x / l, this.y / l, this.z / l);
    }
}

// js-geometry's Bounds fixes its strides when it is constructed: bvh.ts builds every child box
// as new Bounds(parent.min.clone(), parent.max.clone()) and only then moves one face to the
// split, so a node's stride_* (its split-axis choice, bvh.ts:46-52) is its PARENT's extent.
// The library's source is not in the reference; the reference's own renders decide it
// (scenes/student_outputs/final, DESIGN.md §4): with live strides CornellBox full_lighting and
// mirror differ from them beyond Monte Carlo noise (4x4-block L2 1.19x / 1.70x the noise),
// with construction-time strides they agree (0.97x / 1.00x).
class Bounds {
    constructor(min, max) {
        this.min = min; this.max = max;
        this.stride_x = max.x - min.x; this.stride_y = max.y - min.y; this.stride_z = max.z - min.z;
    }
}

const mat4_identity = () => [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1];
const mat4_scale = (x, y, z) => [x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1];
const mat4_translate = (x, y, z) => [1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1];

function mat4_matmul(a, b) {
    const r = new Array(16);
    for (let i = 0; i < 4; i++)
        for (let j = 0; j < 4; j++) {
            let s = 0;
            for (let k = 0; k < 4; k++) s += a[i * 4 + k] * b[k * 4 + j];
            r[i * 4 + j] = s;
        }
    return r;
}

// cofactor inverse (exact for translation / 0-degree rotation CTMs)
function mat4_invert(m) {
    const a = [m.slice(0, 4), m.slice(4, 8), m.slice(8, 12), m.slice(12, 16)];
    const minor = (r, c) => {
        const s = [];
        for (let i = 0; i < 4; i++) {
            if (i === r) continue;
            const row = [];
            for (let j = 0; j < 4; j++) if (j !== c) row.push(a[i][j]);
            s.push(row);
        }
        return s[0][0] * (s[1][1] * s[2][2] - s[1][2] * s[2][1])
            - s[0][1] * (s[1][0] * s[2][2] - s[1][2] * s[2][0])
            + s[0][2] * (s[1][0] * s[2][1] - s[1][1] * s[2][0]);
    };
    const cof = [];
    for (let r = 0; r < 4; r++) {
        cof.push([]);
        for (let c = 0; c < 4; c++) cof[r].push(((r + c) % 2 ? -1 : 1) * minor(r, c));
    }
    let det = 0;
    for (let c = 0; c < 4; c++) det += a[0][c] * cof[0][c];
    const out = new Array(16);
    for (let r = 0; r < 4; r++) for (let c = 0; c < 4; c++) out[r * 4 + c] = cof[c][r] / det;
    return out;
}

const mat4_to_mat3 = (m) => [m[0], m[1], m[2], m[4], m[5], m[6], m[8], m[9], m[10]];
const mat3_tranpose = (m) => [m[0], m[3], m[6], m[1], m[4], m[7], m[2], m[5], m[8]];
const mat3_vecmul = (m, v) => [
    m[0] * v[0] + m[1] * v[1] + m[2] * v[2],
    m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
    m[6] * v[0] + m[7] * v[1] + m[8] * v[2],
];
const mat4_vecmul = (m, v) => [
    m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3] * v[3],
    m[4] * v[0] + m[5] * v[1] + m[6] * v[2] + m[7] * v[3],
    m[8] * v[0] + m[9] * v[1] + m[10] * v[2] + m[11] * v[3],
    m[12] * v[0] + m[13] * v[1] + m[14] * v[2] + m[15] * v[3],
];

const cross = (a, b) => [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]];
const norm3 = (v) => { const l = Math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); return [v[0] / l, v[1] / l, v[2] / l]; };

/**
 * Look-at camera.  w = -look, v = up orthogonalised against w, u = v x w.
 * Returns column-major (WGSL mat4x4) arrays: cam_to_world has columns (u, v, w, pos);
 * world_to_camera is its inverse.  Matches the reference renders (SURVEY.md §8c).
 */
function camera_matrices(pos, look, up) {
    const P = pos.toArray(), Lk = look.toArray(), U = up.toArray();
    const w = norm3([-Lk[0], -Lk[1], -Lk[2]]);
    const d = U[0] * w[0] + U[1] * w[1] + U[2] * w[2];
    const v = norm3([U[0] - d * w[0], U[1] - d * w[1], U[2] - d * w[2]]);
    const u = cross(v, w);
    const cam_to_world = [u[0], u[1], u[2], 0, v[0], v[1], v[2], 0, w[0], w[1], w[2], 0, P[0], P[1], P[2], 1];
    const tx = -(u[0] * P[0] + u[1] * P[1] + u[2] * P[2]);
    const ty = -(v[0] * P[0] + v[1] * P[1] + v[2] * P[2]);
    const tz = -(w[0] * P[0] + w[1] * P[1] + w[2] * P[2]);
    const world_to_cam = [u[0], v[0], w[0], 0, u[1], v[1], w[1], 0, u[2], v[2], w[2], 0, tx, ty, tz, 1];
    return { world_to_cam, cam_to_world };
}

module.exports = {
    Vertex, Bounds, mat4_identity, mat4_scale, mat4_translate, mat4_matmul, mat4_invert,
    mat4_to_mat3, mat3_tranpose, mat3_vecmul, mat4_vecmul, camera_matrices,
};
