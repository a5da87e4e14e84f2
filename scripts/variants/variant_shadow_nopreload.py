"""A/B variant (not product code): the fused kernel's shadow batches load the path state after the
trace instead of before it (frees 8 VGPRs across phase 1, where the shadow instance spills 20 B/lane).
Writes a modified copy of csrc to argv[1]."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dst = sys.argv[1]
if os.path.exists(dst):
    shutil.rmtree(dst)
shutil.copytree(os.path.join(ROOT, "brown-cs2240-path-tracer_amd", "csrc"), dst)
p = os.path.join(dst, "pt_wavefront.hip")
s = open(p).read()
old = """        else { a1 = in.ray[2 * e + 1]; c2 = in.q2[e]; }
    }"""
new = """    }"""
assert old in s
s = s.replace(old, new)
old = """        } else {  // packed shadow entry
            unpack_dspec(__builtin_bit_cast(uint32_t, a1.x), ps);"""
new = """        } else {  // packed shadow entry
            a1 = in.ray[2 * e + 1];
            c2 = in.q2[e];
            unpack_dspec(__builtin_bit_cast(uint32_t, a1.x), ps);"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
