"""The Node host (brown-cs2240-path-tracer_amd/node): the reference's scene pipeline re-hosted in
its own language.  Its packed buffers must equal the Python oracle's restatement bit for bit,
match the survey's independently derived counts, and keep the reference parsers' quirks."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import scene_oracle as so
from conftest import ALL_SCENES, PKG, SCENES, pack_with_node

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NODE_DIR = os.path.join(PKG, "node")


def node_eval(js: str):
    """Run a JS snippet with the host module loaded as `h`; returns the JSON it prints."""
    code = f"const h = require({json.dumps(NODE_DIR)});\n{js}"
    out = subprocess.run(["node", "-e", code], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError(out.stderr)
    return json.loads(out.stdout) if out.stdout.strip() else None


@pytest.mark.parametrize("scene", ALL_SCENES)
def test_node_packing_equals_oracle(packed, scene):
    cam, ps = so.load_scene(os.path.join(SCENES, "scene_assets", scene + ".xml"), os.path.join(SCENES, "scene_assets"))
    p = packed[scene]
    assert p.triangle_data.tobytes() == ps.triangle_data.tobytes()
    assert p.bvh_data.tobytes() == ps.bvh_data.tobytes()
    st = {"imageWidth": 512, "imageHeight": 512, "samplesPerPixel": 16, "pathContinuationProb": 0.9,
          "directLightingOnly": False}
    assert p.meta.tobytes() == so.make_meta(so.screen_dimension(st), cam, st).tobytes()


@pytest.mark.parametrize("scene", ALL_SCENES)
def test_packed_buffers_golden_sha(packed, scene):
    with open(os.path.join(GOLDEN, "packed_sha256.json")) as f:
        g = json.load(f)[scene]
    p = packed[scene]
    assert p.triangle_data.size == g["triangle_len"] and p.bvh_data.size == g["bvh_len"]
    assert hashlib.sha256(p.triangle_data.tobytes()).hexdigest() == g["triangle_sha256"]
    assert hashlib.sha256(p.bvh_data.tobytes()).hexdigest() == g["bvh_sha256"]


def tree_counts(bvh):
    nodes = leaves = refs = max_leaf = 0
    stack = [6]
    while stack:
        o = stack.pop()
        nodes += 1
        if bvh[o] == 1:
            leaves += 1
            n = int(bvh[o + 4]) // 4
            refs += n
            max_leaf = max(max_leaf, n)
        else:
            stack += [int(bvh[o + 2]), int(bvh[o + 3])]
    return nodes, leaves, refs, max_leaf


@pytest.mark.parametrize("scene", ["CornellBox", "CornellBox-Mirror", "CornellBox-Glossy", "MedievalBoat"])
def test_scene_counts_match_survey(packed, scene):
    """SURVEY.md §8 table, derived by the survey's own throwaway restatement: the triangle buffer
    (tree-independent) from the product, the tree from the oracle's builder under the survey's
    reading of Bounds.stride_* (each node's own extent).  The product's tree uses js-geometry's
    construction-time strides instead and is pinned by the next test."""
    import scene_oracle as so
    with open(os.path.join(GOLDEN, "survey_scene_stats.json")) as f:
        g = json.load(f)[scene]
    p = packed[scene]
    tri = p.triangle_data
    assert int(tri[0]) == g["verts"]
    assert (int(tri[4]) - int(tri[3])) // 4 == g["tris"]
    if "tri_len_no_vn_pad" in g:
        assert int(tri[5]) == g["tri_len_no_vn_pad"]
    if "vn_len" in g:
        assert int(tri[6]) == g["vn_len"]
    _, live = so.load_scene(os.path.join(SCENES, "scene_assets", scene + ".xml"), os.path.join(SCENES, "scene_assets"),
                            live_strides=True)
    assert live.bvh_data.size == g["bvh_len"]
    assert tree_counts(live.bvh_data) == (g["nodes"], g["leaves"], g["refs"], g["max_leaf"])


def test_product_tree_uses_construction_time_strides(packed):
    """CornellBox: the product's tree is the oracle's under js-geometry's construction-time
    strides (a node's split axis follows its parent's extent), not the survey's reading."""
    import scene_oracle as so
    p = packed["CornellBox"]
    _, ctor = so.load_scene(os.path.join(SCENES, "scene_assets", "CornellBox.xml"), os.path.join(SCENES, "scene_assets"))
    _, live = so.load_scene(os.path.join(SCENES, "scene_assets", "CornellBox.xml"), os.path.join(SCENES, "scene_assets"),
                            live_strides=True)
    assert p.bvh_data.tobytes() == ctor.bvh_data.tobytes() != live.bvh_data.tobytes()
    assert tree_counts(p.bvh_data) != tree_counts(live.bvh_data)


def test_ini_configs_meta(tmp_path):
    """Every reference .ini: resolution rounding, settings and meta block as the oracle computes them."""
    for d in ("final", "milestone"):
        for ini in sorted(os.listdir(os.path.join(SCENES, "scene_files", d))):
            path = os.path.join(SCENES, "scene_files", d, ini)
            p = pack_with_node(path, str(tmp_path / ini))
            sc = so.ini_file_to_ini_scene(so.parse_ini_file(open(path).read()))
            xml = os.path.join(SCENES, sc["IO"]["scene"].lstrip("/"))
            with open(xml) as f:
                cam, prims = so.load_scene_xml(f.read())
            meta = so.make_meta(so.screen_dimension(sc["Settings"]), cam, sc["Settings"])
            assert p.meta.tobytes() == meta.tobytes(), ini
            assert p.info["settings"]["samplesPerPixel"] == sc["Settings"]["samplesPerPixel"]


def test_parse_ini_semantics():
    r = node_eval(r'''
const f = h.parse_ini_file("[IO]\n  scene = /a.xml\n  output = o.png\n[Settings]\nimageWidth = 510\nimageHeight=300\n"
  + "samplesPerPixel = 7\npathContinuationProb = 0.25\ndirectLightingOnly = true\nnumDirectLightingSamples = 1\nnoequals\n");
const s = h.ini_file_to_ini_scene(f);
console.log(JSON.stringify({f, s, dim: h.screen_dimension(s.Settings)}));''')
    assert r["s"]["IO"]["scene"] == "/a.xml"
    assert r["s"]["Settings"] == {"directLightingOnly": True, "imageHeight": 300, "imageWidth": 510,
                                  "numDirectLightingSamples": 1, "pathContinuationProb": 0.25, "samplesPerPixel": 7}
    assert r["dim"] == [508, 300]  # round_4(510), round_4(510 / (510/300))
    with pytest.raises(RuntimeError, match="ini file to ini scene"):
        node_eval('h.ini_file_to_ini_scene(h.parse_ini_file("[IO]\\nscene=x\\n"));')


def test_parse_obj_quirks():
    """Tabs/comments, negative indices, quads split (0,1,2)(0,2,3), groups without faces dropped,
    usemtl creates objects even with repeated names, materials zero-initialised on newmtl."""
    obj = "v\t0 0 0 # c\nv 1 0 0\nv 1 1 0\nv 0 1 0\nusemtl empty\nusemtl a\nf -4 -3 -2 -1\nusemtl a\nf 1/1/1 2/2/2 3/3/3\n"
    mtl = "newmtl a\n  Kd 0.5 0.25 0.125 # x\n  Ke 1 2 3\nnewmtl b\nNs 7\n"
    r = node_eval(f'''
const g = h.parse_obj({json.dumps(obj)}, {json.dumps(mtl)}, [1,0,0,0, 0,1,0,0, 0,0,1,0, 0,0,0,1]);
console.log(JSON.stringify(g));''')
    assert r["vertices"] == [0, 0, 0, 1, 0, 0, 1, 1, 0, 0, 1, 0]
    assert [o["name"] for o in r["objects"]] == ["a", "a"]
    assert r["objects"][0]["indices"] == [1, 2, 3, 1, 3, 4]
    assert r["objects"][1]["indices"] == [1, 2, 3]
    assert r["objects"][0]["material"]["Kd"] == [0.5, 0.25, 0.125]
    assert r["objects"][0]["material"]["Ns"] == 0
    py = so.parse_obj(obj, mtl, so.mat4_identity())
    assert py["vertices"] == r["vertices"] and [o["indices"] for o in py["objects"]] == [o["indices"] for o in r["objects"]]
    with pytest.raises(RuntimeError, match="5\\+ sides"):
        node_eval('h.parse_obj("v 0 0 0\\nf 1 1 1 1 1\\n", "", [1,0,0,0,0,1,0,0,0,0,1,0,0,0,0,1]);')


def test_xml_compact_shape():
    r = node_eval(r'''
const x = h.xml2js('<?xml version="1.0"?><scenefile><!-- c --><a k="1"/><a k="2"><b v=\'x\'/></a><c/></scenefile>');
console.log(JSON.stringify(x));''')
    sf = r["scenefile"]
    assert isinstance(sf["a"], list) and sf["a"][0]["_attributes"] == {"k": "1"}
    assert sf["a"][1]["b"]["_attributes"] == {"v": "x"}
    assert sf["c"] == {}


def test_first_primitive_only_and_ctm_order():
    """index.ts:116 packs only the first primitive; CornellBox2.xml lists the box first."""
    r = node_eval(f'''
const s = h.load_scene_xml_file({json.dumps(os.path.join(SCENES, "scene_assets", "CornellBox2.xml"))});
const c = h.parse_scene_xml(require("fs").readFileSync({json.dumps(os.path.join(SCENES, "scene_assets", "CornellBox2.xml"))}, "utf8"));
console.log(JSON.stringify({{n: c.final_primitives.length, first: c.final_primitives[0].data.path,
  second_ctm: c.final_primitives[1].ctm, tri0: s.primitive_data[0].triangle_data[0]}}));''')
    assert r["n"] == 2 and r["first"].endswith("CornellBox-Original.obj") and r["tri0"] == 72
    # second primitive: translate(-1,0,0) . rotate(y, 90 "radians") . identity  (math.ts:3-12 takes radians)
    want = so.mat4_matmul(so.mat4_translate(-1, 0, 0), so.mat4_matmul(so.mat4_rot_axis(0, 1, 0, 90.0), so.mat4_scale(1, 1, 1)))
    assert np.allclose(r["second_ctm"], want, atol=0)


def test_missing_file_rejects():
    with pytest.raises(RuntimeError, match="file error"):
        node_eval('h.load_scene_xml_file("/nonexistent/scene_assets/x.xml");')


def test_addon_surface_without_gpu():
    r = node_eval('''
const pt = h.native();
let err = null;
try { pt.sceneCreate(new Float32Array(64), new Float32Array(64), 0); } catch (e) { err = e.message; }
let terr = null;
try { pt.render(1, 2); } catch (e) { terr = e.constructor.name; }
let oerr = null;
pt.setOption('kernel', 'wavefront'); pt.setOption('parts', 2); pt.setOption('kernel', null);
try { pt.setOption('nosuch', '1'); } catch (e) { oerr = e.message; }
console.log(JSON.stringify({abi: pt.abiVersion(), keys: Object.keys(pt).sort(), err, terr, oerr}));''')
    assert r["abi"] == 3
    assert r["oerr"] and "unknown option" in r["oerr"]
    assert r["keys"] == sorted(["abiVersion", "deviceCount", "sceneCreate", "sceneDestroy", "sceneInfo", "render",
                                "renderSync", "renderMulti", "frame",
                                "tonemap", "profileEnable", "profileRead", "bvhBuild", "renderImage",
                                "sceneSetVertexNormals", "setOption"])
    assert r["terr"] == "TypeError"
    assert r["err"] and "pt_hip error" in r["err"]


def test_png_writer_roundtrip(tmp_path):
    from PIL import Image
    out = tmp_path / "x.png"
    node_eval(f'''
const W = 5, H = 3, px = new Uint8ClampedArray(W * H * 4);
for (let i = 0; i < px.length; i++) px[i] = (i * 37) & 255;
require("fs").writeFileSync({json.dumps(str(out))}, h.encode_png(px, W, H));''')
    img = np.array(Image.open(out))
    assert img.shape == (3, 5, 4)
    assert np.array_equal(img.reshape(-1), (np.arange(60) * 37) & 255)


def test_multi_mesh_buffers_match_oracle(tmp_path):
    """--all-meshes: every primitive of CornellBox2.xml (the Cornell box and
    the MedievalBoat under its own CTM, parse-obj.ts:24's transform per mesh) merged into one scene,
    byte-identical to the oracle's restatement; without the flag only the first primitive, as
    index.ts:116."""
    import scene_oracle as so
    xml = os.path.join(SCENES, "scene_assets", "CornellBox2.xml")
    assets = os.path.join(SCENES, "scene_assets")
    multi = pack_with_node(xml, str(tmp_path / "multi"), "--all-meshes", "--native-bvh")
    first = pack_with_node(xml, str(tmp_path / "first"))
    _, om = so.load_scene(xml, assets, all_meshes=True)
    _, of = so.load_scene(xml, assets)
    assert multi.info["meshes"] == 2 and first.info["meshes"] == 1
    assert multi.triangle_data.tobytes() == om.triangle_data.tobytes()
    assert multi.bvh_data.tobytes() == om.bvh_data.tobytes()
    assert first.triangle_data.tobytes() == of.triangle_data.tobytes()
    assert first.bvh_data.tobytes() == of.bvh_data.tobytes()
    # the merged scene holds both meshes: 72 + 15222 vertices, 36 + 12573 triangles
    tri = multi.triangle_data
    assert int(tri[0]) == 72 + 15222 and (int(tri[4]) - int(tri[3])) // 4 == 36 + 12573


def test_merge_groups_large_mesh():
    """--all-meshes merge of a mesh far above V8's call-argument limit (no RangeError from a spread)."""
    r = node_eval('''
const scene = require(require('path').join(''' + json.dumps(NODE_DIR) + ''', 'lib', 'scene'));
const n = 600000;
const big = { vertices: new Array(3 * n).fill(0.5), vertex_normals: [], objects: [{ indices: [1, 2, 3] }] };
const small = { vertices: [0, 0, 0, 1, 0, 0, 0, 1, 0], vertex_normals: [], objects: [{ indices: [1, 2, 3] }] };
const m = scene.merge_groups([big, small]);
console.log(JSON.stringify({ nv: m.vertices.length, last: m.objects[1].indices }));''')
    assert r["nv"] == 3 * 600000 + 9 and r["last"] == [600001, 600002, 600003]
