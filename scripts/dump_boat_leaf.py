# Writes the MedievalBoat reference tree's biggest leaf (7327 entries) as 48-byte pt_layout.h Tri
# records (v0, e1 = v1 - v0, e2 = v2 - v0 in f32, material, position, 0) for scripts/leafbvh_harness.cpp:
#   python3 scripts/dump_boat_leaf.py  ->  /tmp/lh/boat_leaf.bin  (oracle packing: test infrastructure)
import sys, os, struct
import numpy as np
sys.path.insert(0, 'oracle')
import scene_oracle as so
assets = 'scenes/scene_assets'
_, p = so.load_scene(os.path.join(assets, 'MedievalBoat.xml'), assets)
tri = p.triangle_data.astype(np.float32); bvh = p.bvh_data.astype(np.float32)
vs = int(tri[2])
leaves = []
def walk(ptr):
    stack=[ptr]
    while stack:
        q = stack.pop()
        for side in (2, 3):
            c = int(bvh[q + side])
            if bvh[c] == 1:
                n = int(bvh[c + 4]) // 4
                leaves.append((c, n))
            else:
                stack.append(c)
walk(6)
c, n = max(leaves, key=lambda x: x[1])
print('leaves', len(leaves), 'biggest', n)
out = bytearray()
base = c + 17
for k in range(n):
    i0, i1, i2, mat = bvh[base + 4*k: base + 4*k + 4]
    V = [tri[vs + (int(i) - 1) * 3: vs + (int(i) - 1) * 3 + 3] for i in (i0, i1, i2)]
    v0 = V[0]; e1 = (V[1] - V[0]).astype(np.float32); e2 = (V[2] - V[0]).astype(np.float32)
    rec = struct.pack('<9f3i', v0[0], v0[1], v0[2], e1[0], e1[1], e1[2], e2[0], e2[1], e2[2], int(mat), k, 0)
    out += rec
os.makedirs('/tmp/lh', exist_ok=True); open('/tmp/lh/boat_leaf.bin', 'wb').write(out)
print(len(out) // 48)
