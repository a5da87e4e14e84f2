"""A/B variant (not product code): path_after_shadow loads the shading point's material where each
part needs it (NEE, then the BSDF after a compiler memory barrier) instead of holding it across both
(the fused shadow kernel spills 20 B/lane at 64 VGPRs).  Writes a modified copy of csrc to argv[1]."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dst = sys.argv[1]
if os.path.exists(dst):
    shutil.rmtree(dst)
shutil.copytree(os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "csrc"), dst)
p = os.path.join(dst, "pt_path.h")
s = open(p).read()
old = """    const Mat m = load_mat(sc, ps.mat_id);
    if (rec >= 0) {
        Hit sh = hit_data(sc, ray, rec, t);
        Mat nm = load_mat(sc, sh.mat);
        if (sum3(nm.Ke) > 0.0f) ps.L = ps.L + nee_contrib(m, ps.wi, ps.hp, ps.hn, ray.d, ps.beta, sh, nm, sc.inv_ntri);
        if (fp.direct_only) return false;
    }
    if (hash1(ps.seed) > fp.rr_prob) return false;
    ray.d = ps.wi;
    bsdf_continue(m, ps.hp, ps.hn, ray, ps.beta, ps.spec, ps.seed, ps.depth, fp.rr_prob);"""
new = """    if (rec >= 0) {
        Hit sh = hit_data(sc, ray, rec, t);
        Mat nm = load_mat(sc, sh.mat);
        if (sum3(nm.Ke) > 0.0f) {
            const Mat m = load_mat(sc, ps.mat_id);
            ps.L = ps.L + nee_contrib(m, ps.wi, ps.hp, ps.hn, ray.d, ps.beta, sh, nm, sc.inv_ntri);
        }
        if (fp.direct_only) return false;
    }
    if (hash1(ps.seed) > fp.rr_prob) return false;
    ray.d = ps.wi;
    asm volatile("" ::: "memory");  // load the material again below rather than keep it live
    const Mat m = load_mat(sc, ps.mat_id);
    bsdf_continue(m, ps.hp, ps.hn, ray, ps.beta, ps.spec, ps.seed, ps.depth, fp.rr_prob);"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
