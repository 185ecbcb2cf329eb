#!/usr/bin/env python3
"""Synthetic Sponza-class glTF scene (BASELINE.json configs[2]).

There is no network and no Sponza asset, so this writes an atrium of the same
class: ~262k world triangles (tessellated columns, arches, floor, walls,
drapes, a mirror ball and a glass ball), f32 POSITION + NORMAL, u32 indices,
one external .bin, nested nodes with TRS (exercises node propagation,
scene_builder.rs:145-169) and exactly one perspective camera node.  Every
material sets metallicFactor 0 (the glTF default 1.0 would make everything a
mirror, parser.rs:63-64); the light is an emissive ceiling quad
(emissiveFactor x KHR_materials_emissive_strength), because the glTF path has a
black background (scene_builder.rs:17).

    python scenes/gen_sponza_like.py [out_dir] [--scale S]
Deterministic (no randomness).  --scale multiplies the tessellation (1.0 = ~262k tris).
"""
import argparse
import json
import math
import os
import struct

import numpy as np


class Mesh:
    def __init__(self):
        self.pos, self.nrm, self.idx = [], [], []

    def add(self, pos, nrm, idx):
        base = sum(len(p) for p in self.pos)
        self.pos.append(np.asarray(pos, np.float32))
        self.nrm.append(np.asarray(nrm, np.float32))
        self.idx.append(np.asarray(idx, np.uint32) + base)

    def arrays(self):
        return np.concatenate(self.pos), np.concatenate(self.nrm), np.concatenate(self.idx)


def grid(nu, nv, f):
    """Parametric surface f(u, v) -> (pos, normal) on an (nu+1) x (nv+1) vertex grid."""
    us = np.linspace(0.0, 1.0, nu + 1)
    vs = np.linspace(0.0, 1.0, nv + 1)
    P, N = [], []
    for v in vs:
        for u in us:
            p, n = f(u, v)
            P.append(p)
            N.append(n)
    idx = []
    for j in range(nv):
        for i in range(nu):
            a = j * (nu + 1) + i
            b, c, d = a + 1, a + nu + 1, a + nu + 2
            idx += [a, b, d, a, d, c]
    return np.array(P), np.array(N), np.array(idx)


def quad(c, ex, ey, nu, nv, flip=False):
    c, ex, ey = (np.asarray(x, float) for x in (c, ex, ey))
    n = np.cross(ex, ey)
    n /= np.linalg.norm(n)
    if flip:
        n = -n
    P, N, I = grid(nu, nv, lambda u, v: (c + (u - 0.5) * ex + (v - 0.5) * ey, n))
    if flip:
        I = I.reshape(-1, 3)[:, ::-1].reshape(-1)
    return P, N, I


def cylinder(center, radius, height, nseg, nring):
    cx, cy, cz = center

    def f(u, v):
        a = 2 * math.pi * u
        r = radius * (1.0 + 0.08 * math.cos(16 * a))  # fluted column
        return (cx + r * math.cos(a), cy + v * height, cz + r * math.sin(a)), (math.cos(a), 0.0, math.sin(a))

    P, N, I = grid(nseg, nring, f)
    return P, N, I.reshape(-1, 3)[:, ::-1].reshape(-1)


def arch(c0, c1, y, thick, nseg, nring):
    """Half-torus tube spanning two column tops."""
    c0, c1 = np.asarray(c0, float), np.asarray(c1, float)
    mid = (c0 + c1) / 2
    span = np.linalg.norm(c1 - c0) / 2
    ax = (c1 - c0) / (2 * span)

    def f(u, v):
        t = math.pi * u
        centre = mid + ax * (-math.cos(t) * span) + np.array([0.0, y + math.sin(t) * span, 0.0])
        tang = ax * math.sin(t) + np.array([0.0, math.cos(t), 0.0])
        side = np.cross(tang, [0.0, 0.0, 1.0]) if abs(ax[2]) < 0.5 else np.cross(tang, [1.0, 0.0, 0.0])
        side /= np.linalg.norm(side)
        up = np.cross(side, tang)
        a = 2 * math.pi * v
        n = side * math.cos(a) + up * math.sin(a)
        return centre + thick * n, n

    return grid(nseg, nring, f)


def sphere(center, r, nseg, nring):
    def f(u, v):
        th, ph = 2 * math.pi * u, math.pi * v
        n = (math.sin(ph) * math.cos(th), math.cos(ph), math.sin(ph) * math.sin(th))
        return tuple(center[k] + r * n[k] for k in range(3)), n

    return grid(nseg, nring, f)


def drape(c, w, h, nu, nv, phase):
    cx, cy, cz = c

    def f(u, v):
        x = cx + (u - 0.5) * w
        z = cz + 0.15 * math.sin(10 * u + phase) * (1 - v)
        dz = 0.15 * 10 * math.cos(10 * u + phase) * (1 - v) / w
        n = np.array([-dz, 0.0, 1.0])
        return (x, cy + v * h, z), n / np.linalg.norm(n)

    return grid(nu, nv, f)


def build(scale):
    s = lambda n: max(2, int(round(n * math.sqrt(scale))))
    meshes = {k: Mesh() for k in ("floor", "walls", "columns", "arches", "red", "green", "blue", "mirror",
                                  "glass", "light")}
    meshes["floor"].add(*quad((0, 0, 0), (24, 0, 0), (0, 0, 12), s(128), s(64), flip=True))
    meshes["walls"].add(*quad((0, 6, 6), (24, 0, 0), (0, 12, 0), s(64), s(32), flip=True))
    meshes["walls"].add(*quad((0, 6, -6), (24, 0, 0), (0, 12, 0), s(64), s(32)))
    meshes["walls"].add(*quad((12, 6, 0), (0, 0, 12), (0, 12, 0), s(32), s(32), flip=True))
    meshes["walls"].add(*quad((-12, 6, 0), (0, 0, 12), (0, 12, 0), s(32), s(32)))
    xs = np.linspace(-10, 10, 12)
    for zc in (-3.0, 3.0):  # two colonnades, 12 columns each
        for x in xs:
            meshes["columns"].add(*cylinder((x, 0.0, zc), 0.35, 6.0, s(64), s(64)))
        for a, b in zip(xs[:-1], xs[1:]):
            meshes["arches"].add(*arch((a, 0, zc), (b, 0, zc), 6.0, 0.25, s(32), s(16)))
    for k, name in enumerate(("red", "green", "blue", "red")):
        meshes[name].add(*drape((-9 + 6 * k, 1.0, 5.7), 3.5, 4.5, s(48), s(24), phase=k))
    meshes["mirror"].add(*sphere((2.0, 1.0, 0.5), 1.0, s(64), s(32)))
    meshes["glass"].add(*sphere((-2.5, 0.8, -0.8), 0.8, s(48), s(24)))
    meshes["light"].add(*quad((0, 11.9, 0), (16, 0, 0), (0, 0, 6), 1, 1, flip=True))
    mats = {
        "floor": {"pbrMetallicRoughness": {"baseColorFactor": [0.7, 0.68, 0.62, 1.0], "metallicFactor": 0.0}},
        "walls": {"pbrMetallicRoughness": {"baseColorFactor": [0.8, 0.76, 0.66, 1.0], "metallicFactor": 0.0}},
        "columns": {"pbrMetallicRoughness": {"baseColorFactor": [0.75, 0.72, 0.6, 1.0], "metallicFactor": 0.0}},
        "arches": {"pbrMetallicRoughness": {"baseColorFactor": [0.7, 0.6, 0.5, 1.0], "metallicFactor": 0.0}},
        "red": {"pbrMetallicRoughness": {"baseColorFactor": [0.7, 0.12, 0.1, 1.0], "metallicFactor": 0.0}},
        "green": {"pbrMetallicRoughness": {"baseColorFactor": [0.12, 0.55, 0.15, 1.0], "metallicFactor": 0.0}},
        "blue": {"pbrMetallicRoughness": {"baseColorFactor": [0.1, 0.2, 0.65, 1.0], "metallicFactor": 0.0}},
        "mirror": {"pbrMetallicRoughness": {"baseColorFactor": [0.95, 0.95, 0.95, 1.0], "metallicFactor": 1.0}},
        "glass": {"pbrMetallicRoughness": {"baseColorFactor": [0.95, 1.0, 0.97, 0.3], "metallicFactor": 0.0}},
        "light": {"pbrMetallicRoughness": {"baseColorFactor": [1.0, 1.0, 1.0, 1.0], "metallicFactor": 0.0},
                  "emissiveFactor": [1.0, 0.95, 0.85],
                  "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 3.0}}},
    }
    return meshes, mats


def write(out_dir, name, meshes, mats, camera_trs):
    os.makedirs(out_dir, exist_ok=True)
    blob = bytearray()
    buffer_views, accessors, gl_meshes, gl_mats = [], [], [], []

    def view(data, target):
        while len(blob) % 4:
            blob.append(0)
        off = len(blob)
        blob.extend(data.tobytes())
        buffer_views.append({"buffer": 0, "byteOffset": off, "byteLength": data.nbytes, "target": target})
        return len(buffer_views) - 1

    ntris = 0
    for mname, mesh in meshes.items():
        P, N, I = mesh.arrays()
        ntris += len(I) // 3
        vp = view(P, 34962)
        vn = view(N, 34962)
        vi = view(I, 34963)
        accessors.append({"bufferView": vp, "componentType": 5126, "count": len(P), "type": "VEC3",
                          "min": P.min(0).tolist(), "max": P.max(0).tolist()})
        accessors.append({"bufferView": vn, "componentType": 5126, "count": len(N), "type": "VEC3"})
        accessors.append({"bufferView": vi, "componentType": 5125, "count": len(I), "type": "SCALAR"})
        gl_mats.append(mats[mname])
        gl_meshes.append({"name": mname, "primitives": [{
            "attributes": {"POSITION": len(accessors) - 3, "NORMAL": len(accessors) - 2},
            "indices": len(accessors) - 1, "material": len(gl_mats) - 1, "mode": 4}]})
    nodes = []
    children = []
    for k, m in enumerate(gl_meshes):  # mesh nodes under a root with an identity-ish TRS
        nodes.append({"mesh": k, "name": m["name"]})
        children.append(len(nodes) - 1)
    nodes.append({"camera": 0, "translation": camera_trs["t"], "rotation": camera_trs["r"]})
    cam_idx = len(nodes) - 1
    nodes.append({"name": "root", "children": children + [cam_idx], "translation": [0.0, 0.0, 0.0],
                  "scale": [1.0, 1.0, 1.0]})
    gltf = {
        "asset": {"version": "2.0", "generator": "gen_sponza_like.py"},
        "extensionsUsed": ["KHR_materials_emissive_strength"],
        "scene": 0, "scenes": [{"nodes": [len(nodes) - 1]}], "nodes": nodes,
        "cameras": [{"type": "perspective", "perspective": {"yfov": 0.9, "znear": 0.01}}],
        "meshes": gl_meshes, "materials": gl_mats, "accessors": accessors, "bufferViews": buffer_views,
        "buffers": [{"uri": name + ".bin", "byteLength": len(blob)}],
    }
    with open(os.path.join(out_dir, name + ".bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(out_dir, name + ".gltf"), "w") as f:
        json.dump(gltf, f)
    return ntris


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "gen"))
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--name", default="sponza_like")
    a = ap.parse_args()
    meshes, mats = build(a.scale)
    yaw = math.radians(97.0)  # look down the nave (-x), slightly across
    cam = {"t": [11.0, 2.6, 0.8], "r": [0.0, math.sin(yaw / 2), 0.0, math.cos(yaw / 2)]}
    n = write(a.out_dir, a.name, meshes, mats, cam)
    print(f"wrote {a.out_dir}/{a.name}.gltf with {n} triangles")


if __name__ == "__main__":
    main()
