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

/* pre-order walk recording each leaf's path */
static void walk(const float *bvh, int ptr, int depth, int *pn, int *ps, int min_entries) {
    for (int side = 0; side < 2; ++side) {
        const int c = (int)bvh[ptr + 2 + side];
        pn[depth] = ptr;
        ps[depth] = side;
        if (bvh[c] == 1.0f) {
            const int n = (int)bvh[c + 4] / 4;
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

int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: dir frames depth min_entries rows_step\n"); return 2; }
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
    return 0;
}
