"""Build-authored scene assets (committed outputs under scenes/).

  scenes/bunny.obj + bunny.mtl   C2/C5: the reference's resources/models/bunny.ply
                                 (binary PLY, read as data) re-emitted as OBJ WITHOUT `vn` (the PLY
                                 normals contain zero vectors, which the reference's interpolateNormal
                                 would turn into invisible faces), vertices printed with %.9g so the
                                 float32 values round-trip exactly; one material (Ka 0.1, Kd .8/.6/.4,
                                 Ks 0.3, Ns 32).
  scenes/cornell.obj + .mtl      C1: a 30-triangle Cornell-style box (open front/top), integer Ns.

Usage: python tools/make_scenes.py [--ply /root/reference/resources/models/bunny.ply]
"""
import argparse
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCENES = os.path.join(os.path.dirname(HERE), "scenes")


def read_ply(path):
    with open(path, "rb") as f:
        header = []
        while True:
            line = f.readline().decode("ascii").strip()
            header.append(line)
            if line == "end_header":
                break
        data = f.read()
    assert "format binary_little_endian 1.0" in header
    nv = int([h for h in header if h.startswith("element vertex")][0].split()[-1])
    nf = int([h for h in header if h.startswith("element face")][0].split()[-1])
    vprops = []
    in_v = False
    for h in header:
        if h.startswith("element vertex"):
            in_v = True
            continue
        if h.startswith("element") and in_v:
            break
        if in_v and h.startswith("property"):
            _, t, name = h.split()
            vprops.append((name, {"float": "<f4", "uchar": "u1", "int": "<i4"}[t]))
    vdt = np.dtype(vprops)
    verts = np.frombuffer(data, vdt, count=nv)
    off = vdt.itemsize * nv
    fdt = np.dtype([("n", "u1"), ("i", "<i4", 3)])
    faces = np.frombuffer(data, fdt, count=nf, offset=off)
    assert (faces["n"] == 3).all()
    v = np.stack([verts["x"], verts["y"], verts["z"]], 1).astype(np.float32)
    return v, faces["i"].astype(np.int64)


def write_bunny(ply):
    v, f = read_ply(ply)
    with open(os.path.join(SCENES, "bunny.mtl"), "w") as m:
        m.write("newmtl bunny\nNs 32\nKa 0.1 0.1 0.1\nKd 0.8 0.6 0.4\nKs 0.3 0.3 0.3\nNi 1\nd 1\nillum 2\n")
    with open(os.path.join(SCENES, "bunny.obj"), "w") as o:
        o.write("# Stanford bunny (from reference resources/models/bunny.ply), no vn; tools/make_scenes.py\n")
        o.write("mtllib bunny.mtl\n")
        for x, y, z in v:
            o.write("v %.9g %.9g %.9g\n" % (x, y, z))
        o.write("usemtl bunny\n")
        for a, b, c in f:
            o.write("f %d %d %d\n" % (a + 1, b + 1, c + 1))
    print("bunny:", len(v), "vertices", len(f), "faces")


def write_cornell():
    verts, groups = [], {}

    def quad(mat, a, b, c, d):
        base = len(verts) + 1
        verts.extend([a, b, c, d])
        groups.setdefault(mat, []).extend([(base, base + 1, base + 2), (base, base + 2, base + 3)])

    def block(mat, x0, x1, y0, y1, z0, z1):
        quad(mat, (x0, y1, z1), (x1, y1, z1), (x1, y1, z0), (x0, y1, z0))  # top   +y
        quad(mat, (x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1))  # front +z
        quad(mat, (x1, y0, z0), (x0, y0, z0), (x0, y1, z0), (x1, y1, z0))  # back  -z
        quad(mat, (x0, y0, z0), (x0, y0, z1), (x0, y1, z1), (x0, y1, z0))  # left  -x
        quad(mat, (x1, y0, z1), (x1, y0, z0), (x1, y1, z0), (x1, y1, z1))  # right +x

    quad("white", (0, 0, 1), (1, 0, 1), (1, 0, 0), (0, 0, 0))  # floor +y
    quad("white", (0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0))  # back wall +z
    quad("red", (0, 0, 1), (0, 0, 0), (0, 1, 0), (0, 1, 1))  # left wall +x
    quad("green", (1, 0, 0), (1, 0, 1), (1, 1, 1), (1, 1, 0))  # right wall -x
    quad("lamp", (0.35, 0.95, 0.35), (0.65, 0.95, 0.35), (0.65, 0.95, 0.65), (0.35, 0.95, 0.65))  # -y
    block("white", 0.55, 0.85, 0.0, 0.3, 0.45, 0.75)
    block("white", 0.15, 0.45, 0.0, 0.6, 0.2, 0.5)
    with open(os.path.join(SCENES, "cornell.mtl"), "w") as m:
        for name, kd, ka, ks, ns in [("white", "0.75 0.75 0.75", "0.1 0.1 0.1", "0.2 0.2 0.2", 16),
                                     ("red", "0.75 0.15 0.15", "0.1 0.1 0.1", "0.2 0.2 0.2", 16),
                                     ("green", "0.15 0.75 0.15", "0.1 0.1 0.1", "0.2 0.2 0.2", 16),
                                     ("lamp", "1 1 1", "1 1 1", "0 0 0", 1)]:
            m.write(f"newmtl {name}\nNs {ns}\nKa {ka}\nKd {kd}\nKs {ks}\nNi 1\nd 1\nillum 2\n\n")
    ntri = 0
    with open(os.path.join(SCENES, "cornell.obj"), "w") as o:
        o.write("# 30-triangle Cornell-style box (build-authored, tools/make_scenes.py)\nmtllib cornell.mtl\n")
        for v in verts:
            o.write("v %.9g %.9g %.9g\n" % v)
        for mat, tris in groups.items():
            o.write(f"usemtl {mat}\n")
            for t in tris:
                o.write("f %d %d %d\n" % t)
                ntri += 1
    print("cornell:", len(verts), "vertices", ntri, "faces")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--ply", default="/root/reference/resources/models/bunny.ply")
    a = ap.parse_args()
    os.makedirs(SCENES, exist_ok=True)
    if os.path.exists(a.ply):
        write_bunny(a.ply)
    write_cornell()
