/* leaf_visit_stats.c — diagnostic (test infrastructure; not the product): how many ray queries of
 * a render visit each big leaf of the reference tree, against how many pass the exact box filter
 * that any visit needs (every child box on the root-to-leaf path has ray_bbox > 0).  The gap is
 * the waste of a leaf-major pass that resolves the big leaves for every filtered query before
 * the traversal.
 *   python3 scripts/leaf_visit_stats.py MedievalBoat 240 135 2   (dumps buffers, builds, runs this)
 * Includes the oracle with its diagnostic hooks defined (oracle/pt_oracle.c PO_*_HOOK). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXBIG 64
#define MAXPATH 40
static int g_nbig;
static int g_big_lp[MAXBIG], g_big_n[MAXBIG], g_path_len[MAXBIG];
static int g_path_node[MAXBIG][MAXPATH], g_path_side[MAXBIG][MAXPATH];
static int g_visited[MAXBIG];
static unsigned long long g_q, g_pass[MAXBIG], g_visit[MAXBIG], g_pass_any, g_visit_any, g_visit_multi;
static unsigned long long g_cnt_hist[8];

#define PO_LEAF_HOOK(s, ray, lp) leaf_hook(lp)
#define PO_INTERSECT_HOOK(s, ray, closest_t) isect_hook((const void *)(s), (const void *)(ray))
static void leaf_hook(int lp);
static void isect_hook(const void *sv, const void *rv);
#include "../oracle/pt_oracle.c"

static void leaf_hook(int lp) {
    for (int b = 0; b < g_nbig; ++b)
        if (g_big_lp[b] == lp) g_visited[b]++;
}
static void isect_hook(const void *sv, const void *rv) {
    const scene_t *s = sv;
    const ray_t *ray = rv;
    g_q++;
    int any_pass = 0, any_visit = 0, nvis = 0;
    for (int b = 0; b < g_nbig; ++b) {
        int pass = 1;
        for (int k = 0; k < g_path_len[b] && pass; ++k) {
            const int ptr = g_path_node[b][k], o = g_path_side[b][k] ? 11 : 5;
            v3 mn = V3(B(s, ptr + o), B(s, ptr + o + 1), B(s, ptr + o + 2));
            v3 mx = V3(B(s, ptr + o + 3), B(s, ptr + o + 4), B(s, ptr + o + 5));
            pass = 0.0f < ray_bbox(ray, mn, mx);
        }
        if (pass) { g_pass[b]++; any_pass = 1; }
        if (g_visited[b]) { g_visit[b]++; any_visit = 1; nvis++; if (!pass) { fprintf(stderr, "visit without filter pass!\n"); exit(1); } }
        g_visited[b] = 0;
    }
    g_pass_any += any_pass;
    g_visit_any += any_visit;
    g_visit_multi += nvis > 1;
    g_cnt_hist[nvis > 7 ? 7 : nvis]++;
}

static int *g_ent; /* every leaf entry's bvh index (probe rays start on them) */
static size_t g_nent, g_cap;

/* pre-order walk recording each leaf's path */
static void walk(const float *bvh, int ptr, int depth, int *pn, int *ps, int min_entries) {
    for (int side = 0; side < 2; ++side) {
        const int c = (int)bvh[ptr + 2 + side];
        pn[depth] = ptr;
        ps[depth] = side;
        if (bvh[c] == 1.0f) {
            const int n = (int)bvh[c + 4] / 4;
            for (int e = 0; e < n; ++e) {
                if (g_nent == g_cap) { g_cap = g_cap ? 2 * g_cap : 1024; g_ent = realloc(g_ent, g_cap * sizeof(int)); }
                g_ent[g_nent++] = c + 5 + 12 + 4 * e;
            }
            if (n >= min_entries && g_nbig < MAXBIG) {
                g_big_lp[g_nbig] = c; g_big_n[g_nbig] = n; g_path_len[g_nbig] = depth + 1;
                memcpy(g_path_node[g_nbig], pn, sizeof(int) * (depth + 1));
                memcpy(g_path_side[g_nbig], ps, sizeof(int) * (depth + 1));
                g_nbig++;
            }
        } else {
            walk(bvh, c, depth + 1, pn, ps, min_entries);
        }
    }
}

static float *load(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f) / 4;
    fseek(f, 0, SEEK_SET);
    float *p = malloc(*n * 4);
    if (fread(p, 4, *n, f) != *n) exit(1);
    fclose(f);
    return p;
}

/* a shadow ray from a hit toward a random point of a random light (radiance()'s NEE query) */
static void shadow(const scene_t *s, isect_t h, int32_t seed) {
    v4 off = V4(h.point.x + 1.0e-4f * h.normal.x, h.point.y + 1.0e-4f * h.normal.y, h.point.z + 1.0e-4f * h.normal.z, 1.0f);
    v4 sal = sample_area_lights(s, xyz(off), seed);
    ray_t r;
    r.p = off;
    r.d = V4(sal.x, sal.y, sal.z, 0.0f);
    r.d_inv = inv4(r.d);
    intersect(s, &r, NULL);
}
#define NEXT() (st ^= st << 13, st ^= st >> 7, st ^= st << 17, st)
#define UNIF() ((float)((double)(NEXT() >> 40) * (1.0 / 16777216.0)))
int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: dir frames depth min_entries rows_step [probe_rays]\n"); return 2; }
    char path[512];
    size_t ntri, nbvh, nmeta;
    snprintf(path, sizeof path, "%s/tri.bin", argv[1]); float *tri = load(path, &ntri);
    snprintf(path, sizeof path, "%s/bvh.bin", argv[1]); float *bvh = load(path, &nbvh);
    snprintf(path, sizeof path, "%s/meta.bin", argv[1]); float *meta = load(path, &nmeta);
    const int frames = atoi(argv[2]), depth = atoi(argv[3]), min_entries = atoi(argv[4]), step = atoi(argv[5]);
    int pn[MAXPATH], ps[MAXPATH];
    walk(bvh, 6, 0, pn, ps, min_entries);
    const uint32_t W = (uint32_t)meta[0], H = (uint32_t)meta[1];
    float *out = malloc(sizeof(float) * 3 * W);
    const int nprobe = argc > 6 ? atoi(argv[6]) : 0;
    if (nprobe > 0) { /* the library's probe rays instead (pt_leafbvh.cpp probe_pre_leaves): a random point of
                         a random leaf entry, a uniformly random direction */
        scene_t s = {tri, (uint32_t)ntri, bvh, (uint32_t)nbvh};
        unsigned long long st = 0x9e3779b97f4a7c15ull;
        const int v_start = (int)tri[2];
        double *cdf = malloc(g_nent * sizeof(double)), acc = 0.0; /* area-weighted entries */
        for (size_t e = 0; e < g_nent; ++e) {
            const int i = g_ent[e];
            const int i0 = ((int)bvh[i] - 1) * 3, i1 = ((int)bvh[i + 1] - 1) * 3, i2 = ((int)bvh[i + 2] - 1) * 3;
            v3 v0 = vert(&s, v_start, i0), e1 = sub3(vert(&s, v_start, i1), v0), e2 = sub3(vert(&s, v_start, i2), v0);
            v3 c = cross3(e1, e2);
            acc += sqrt((double)c.x * c.x + (double)c.y * c.y + (double)c.z * c.z);
            cdf[e] = acc;
        }
        for (int k = 0; k < nprobe; ++k) {
            const double x = (double)(NEXT() >> 11) * (1.0 / 9007199254740992.0) * acc;
            size_t lo = 0, hi = g_nent - 1;
            while (lo < hi) { size_t m = (lo + hi) / 2; if (cdf[m] <= x) lo = m + 1; else hi = m; }
            const int i = g_ent[lo];
            const int i0 = ((int)bvh[i] - 1) * 3, i1 = ((int)bvh[i + 1] - 1) * 3, i2 = ((int)bvh[i + 2] - 1) * 3;
            v3 v0 = vert(&s, v_start, i0), e1 = sub3(vert(&s, v_start, i1), v0), e2 = sub3(vert(&s, v_start, i2), v0);
            float a = UNIF(), b = UNIF();
            if (a + b > 1.0f) { a = 1.0f - a; b = 1.0f - b; }
            const float z = 2.0f * UNIF() - 1.0f, phi = 6.2831853f * UNIF(), r = sqrtf(fmaxf(0.0f, 1.0f - z * z));
            ray_t ray;
            ray.p = V4(v0.x + a * e1.x + b * e2.x, v0.y + a * e1.y + b * e2.y, v0.z + a * e1.z + b * e2.z, 1.0f);
            ray.d = V4(r * cosf(phi), r * sinf(phi), z, 0.0f);
            ray.d_inv = inv4(ray.d);
            intersect(&s, &ray, NULL);
        }
    }
    const int grid = argc > 7 ? atoi(argv[7]) : 0;
    if (grid > 0) { /* the library's camera probe (pt_leafbvh.cpp probe_pre_leaves): pixel-centre rays of a
                       grid x grid raster over the image, then one cosine bounce from each hit */
        scene_t s = {tri, (uint32_t)ntri, bvh, (uint32_t)nbvh};
        unsigned long long st = 0x9e3779b97f4a7c15ull;
        const float vhh = po_view_half_h(meta), vhw = vhh * meta[10];
        const float *M = meta + 28;
        for (int j = 0; j < grid; ++j)
            for (int i = 0; i < grid; ++i) {
                const float vx = vhw * ((i + 0.5f) / grid - 0.5f), vy = vhh * (0.5f - (j + 0.5f) / grid), pz = -meta[2];
                v4 pw = V4(M[12] + M[8] * pz + M[4] * vy + M[0] * vx, M[13] + M[9] * pz + M[5] * vy + M[1] * vx,
                           M[14] + M[10] * pz + M[6] * vy + M[2] * vx, 0.0f);
                v3 d = normalize3(V3(pw.x - meta[4], pw.y - meta[5], pw.z - meta[6]));
                ray_t ray;
                ray.p = V4(meta[4], meta[5], meta[6], 1.0f);
                ray.d = V4(d.x, d.y, d.z, 0.0f);
                ray.d_inv = inv4(ray.d);
                isect_t h = intersect(&s, &ray, NULL);
                if (!h.intersected) continue;
                shadow(&s, h, (int32_t)NEXT());
                v3 n = xyz(h.normal);
                if (dot3(n, d) > 0.0f) n = neg3(n);
                const float u1 = UNIF(), u2 = UNIF(), r = sqrtf(u1), phi = 6.2831853f * u2;
                v3 t = fabsf(n.x) > 0.5f ? V3(0.0f, 1.0f, 0.0f) : V3(1.0f, 0.0f, 0.0f);
                v3 b1 = normalize3(cross3(t, n)), b2 = cross3(n, b1);
                const float lx = r * cosf(phi), ly = r * sinf(phi), lz = sqrtf(fmaxf(0.0f, 1.0f - u1));
                v3 bd = normalize3(V3(b1.x * lx + b2.x * ly + n.x * lz, b1.y * lx + b2.y * ly + n.y * lz, b1.z * lx + b2.z * ly + n.z * lz));
                ray.p = V4(h.point.x + 0.001f * bd.x, h.point.y + 0.001f * bd.y, h.point.z + 0.001f * bd.z, 1.0f);
                ray.d = V4(bd.x, bd.y, bd.z, 0.0f);
                ray.d_inv = inv4(ray.d);
                h = intersect(&s, &ray, NULL);
                if (h.intersected) shadow(&s, h, (int32_t)NEXT());
            }
    }
    for (int f = 0; f < frames; ++f)
        for (uint32_t y = 0; y < H; y += (uint32_t)step)
            po_frame(tri, (uint32_t)ntri, bvh, (uint32_t)nbvh, meta, y, y + 1, (uint32_t)f, depth, out, NULL, 1);
    printf("queries %llu  any big-leaf filter pass %.4f  any visit %.4f  >1 visit %.4f\n", g_q,
           (double)g_pass_any / g_q, (double)g_visit_any / g_q, (double)g_visit_multi / g_q);
    printf("visits per query hist:");
    for (int i = 0; i < 8; ++i) printf(" %d:%.4f", i, (double)g_cnt_hist[i] / g_q);
    printf("\n%6s %8s %10s %10s %8s\n", "leaf", "entries", "pass/q", "visit/q", "v/pass");
    for (int b = 0; b < g_nbig; ++b)
        printf("%6d %8d %10.4f %10.4f %8.3f\n", b, g_big_n[b], (double)g_pass[b] / g_q, (double)g_visit[b] / g_q,
               g_pass[b] ? (double)g_visit[b] / g_pass[b] : 0.0);
    double fp = 0.0, fv = 0.0;
    for (int b = 0; b < g_nbig; ++b) { fp += (double)g_pass[b] * g_big_n[b]; fv += (double)g_visit[b] * g_big_n[b]; }
    printf("entry-weighted visited / filtered: %.3f\n", fp > 0.0 ? fv / fp : 0.0);
    return 0;
}
