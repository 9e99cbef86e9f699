"""Generate the mesh fixtures under tests/golden/meshes/ from the reference's mesh data.

Reads (as data) /root/reference/mesh_models/{agent_models,environment_models}/*.{dae,3ds}
and writes one Wavefront OBJ per mesh, one `o` group per Assimp-style submesh, in the
order the reference's AssimpMeshLoader (utilities/assimp_mesh_loader.hpp:20-60) would
see `scene->mMeshes`:

* COLLADA: one submesh per <triangles>/<polylist> element of each <geometry>, in
  document order; node transforms, <unit> and <up_axis> are ignored (the reference
  never reads mRootNode / mTransformation); <lines> produce no triangles.
* 3DS: one submesh per (object, material) with faces split by material, materials in
  file order (Assimp Discreet3DSImporter::ConvertMeshes); with no keyframer chunk the
  vertices are used as stored.

Vertex values are float32 (Assimp aiVector3D), written with 9 significant digits so
that (double)(float)strtod(text) reproduces them exactly.  This is a build-defined
convention: Assimp's own fast_atof may differ in the last float bit.

Usage: python tests/golden/make_meshes.py [reference_root]
"""
from __future__ import annotations

import json
import os
import struct
import sys
import xml.etree.ElementTree as ET

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "meshes")


def _strip(tag: str) -> str:
    return tag.split("}", 1)[-1]


def parse_dae(path):
    root = ET.parse(path).getroot()
    ns = {"c": root.tag.split("}")[0].strip("{")}
    sources = {}
    for src in root.iter("{%s}source" % ns["c"]):
        fa = src.find("c:float_array", ns)
        if fa is not None and fa.text:
            sources[src.get("id")] = np.array(fa.text.split(), dtype=np.float32)
    subs = []
    for geom in root.find("c:library_geometries", ns):
        mesh = geom.find("c:mesh", ns)
        if mesh is None:
            continue
        vmap = {}
        for v in mesh.findall("c:vertices", ns):
            for inp in v.findall("c:input", ns):
                if inp.get("semantic") == "POSITION":
                    vmap[v.get("id")] = inp.get("source").lstrip("#")
        for prim in mesh:
            kind = _strip(prim.tag)
            if kind not in ("triangles", "polylist"):
                continue
            inputs = prim.findall("c:input", ns)
            stride = max(int(i.get("offset")) for i in inputs) + 1
            voff = None
            vsrc = None
            for i in inputs:
                if i.get("semantic") == "VERTEX":
                    voff = int(i.get("offset"))
                    vsrc = vmap[i.get("source").lstrip("#")]
            pos = sources[vsrc].reshape(-1, 3)
            pe = prim.find("c:p", ns)
            idx = np.array(pe.text.split() if pe is not None and pe.text else [], dtype=np.int64)
            idx = idx.reshape(-1, stride)[:, voff]
            if kind == "polylist":
                vc = np.array(prim.find("c:vcount", ns).text.split(), dtype=np.int64)
                tris = []
                o = 0
                for c in vc:
                    if c == 3:
                        tris.append(idx[o:o + 3])
                    o += c
                tri = np.array(tris, dtype=np.int64).reshape(-1, 3)
            else:
                tri = idx.reshape(-1, 3)
            subs.append((prim.get("material") or "", pos[tri.reshape(-1)].reshape(-1, 9)))
    return subs


def parse_3ds(path):
    data = open(path, "rb").read()
    materials = []
    objects = []

    def walk(off, end, obj):
        while off + 6 <= end:
            cid, ln = struct.unpack_from("<HI", data, off)
            body = off + 6
            if cid in (0x4D4D, 0x3D3D, 0x4100, 0xAFFF):
                walk(body, off + ln, obj)
            elif cid == 0xA000:
                s = data[body:data.index(b"\0", body)]
                materials.append(s.decode("latin-1"))
            elif cid == 0x4000:
                s = data[body:data.index(b"\0", body)]
                o = {"name": s.decode("latin-1"), "verts": None, "faces": None, "mats": []}
                objects.append(o)
                walk(body + len(s) + 1, off + ln, o)
            elif cid == 0x4110:
                n = struct.unpack_from("<H", data, body)[0]
                obj["verts"] = np.frombuffer(data, np.float32, 3 * n, body + 2).reshape(n, 3).copy()
            elif cid == 0x4120:
                n = struct.unpack_from("<H", data, body)[0]
                f = np.frombuffer(data, np.uint16, 4 * n, body + 2).reshape(n, 4)[:, :3].astype(np.int64)
                obj["faces"] = f
                walk(body + 2 + 8 * n, off + ln, obj)
            elif cid == 0x4130:
                s = data[body:data.index(b"\0", body)]
                n = struct.unpack_from("<H", data, body + len(s) + 1)[0]
                fl = np.frombuffer(data, np.uint16, n, body + len(s) + 3).astype(np.int64)
                obj["mats"].append((s.decode("latin-1"), fl))
            off += ln

    walk(0, len(data), None)
    subs = []
    for o in objects:
        if o["verts"] is None or o["faces"] is None or len(o["faces"]) == 0:
            continue
        fmat = np.full(len(o["faces"]), len(materials), np.int64)  # default material last
        for name, fl in o["mats"]:
            fmat[fl] = materials.index(name)
        for m in range(len(materials) + 1):
            sel = np.nonzero(fmat == m)[0]
            if len(sel) == 0:
                continue
            tri = o["faces"][sel]
            name = materials[m] if m < len(materials) else "DefaultMaterial"
            subs.append((name, o["verts"][tri.reshape(-1)].reshape(-1, 9)))
    return subs


def write_obj(path, subs):
    with open(path, "w") as f:
        f.write("# generated by tests/golden/make_meshes.py (float32 values, %.9g)\n")
        base = 1
        for i, (mat, tris) in enumerate(subs):
            f.write("o sub%d %s\n" % (i, mat))
            v = tris.reshape(-1, 3)
            for x, y, z in v:
                f.write("v %.9g %.9g %.9g\n" % (x, y, z))
            for t in range(tris.shape[0]):
                a = base + 3 * t
                f.write("f %d %d %d\n" % (a, a + 1, a + 2))
            base += v.shape[0]


def main():
    os.makedirs(OUT, exist_ok=True)
    meta = {}
    jobs = [
        ("agent_unit_box", "mesh_models/agent_models/unit_box.dae", parse_dae),
        ("agent_blimp", "mesh_models/agent_models/blimp.3ds", parse_3ds),
        ("env_unit_box", "mesh_models/environment_models/unit_box.dae", parse_dae),
        ("env_model", "mesh_models/environment_models/model.dae", parse_dae),
    ]
    for name, rel, fn in jobs:
        subs = fn(os.path.join(REF, rel))
        write_obj(os.path.join(OUT, name + ".obj"), subs)
        meta[name] = {
            "source": rel,
            "submeshes": [{"material": m, "triangles": int(t.shape[0])} for m, t in subs],
            "triangles": int(sum(t.shape[0] for _, t in subs)),
        }
        print(name, meta[name]["triangles"], [s["triangles"] for s in meta[name]["submeshes"]])
    with open(os.path.join(OUT, "meshes.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
