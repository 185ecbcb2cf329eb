"""Small glTF fixtures for the glTF-row tests (written at test time into tmp dirs).

`write_room` makes a closed, lit room that exercises every branch of the
reader (scene_builder.rs:9-398):
  * nested nodes mixing TRS (rotation + non-uniform scale + translation) and a
    column-major `matrix` node, so propagation and cof() normals matter;
  * a second scene that also lists a node (TRS propagation runs over every
    scene, :155-161, but only `scene` is converted, :183);
  * interleaved POSITION/NORMAL in one strided bufferView (byteStride),
    accessor byteOffsets, u16 and u32 indices, and a non-indexed primitive;
  * materials: default (no material), metallicFactor omitted (=> Metallic),
    alpha < 1 (=> Dielectric 1.5), emissive x KHR_materials_emissive_strength,
    an `extensions` object without the strength extension;
  * the camera on a child of a rotated parent.
"""
import json
import math
import os

import numpy as np


def _box_faces(c, h, inward):
    """6 quads of an axis-aligned box: (positions[24,3], normals[24,3], u16 indices[36])."""
    P, N, I = [], [], []
    for axis in range(3):
        for sgn in (-1.0, 1.0):
            n = np.zeros(3)
            n[axis] = sgn
            u = np.zeros(3)
            u[(axis + 1) % 3] = h[(axis + 1) % 3]
            v = np.zeros(3)
            v[(axis + 2) % 3] = h[(axis + 2) % 3]
            centre = np.asarray(c, float) + n * np.asarray(h, float)
            base = len(P)
            for du, dv in ((-1, -1), (1, -1), (1, 1), (-1, 1)):
                P.append(centre + du * u + dv * v)
                N.append(-n if inward else n)
            tri = [0, 1, 2, 0, 2, 3] if (sgn > 0) != inward else [0, 2, 1, 0, 3, 2]
            I += [base + k for k in tri]
    return np.array(P, np.float32), np.array(N, np.float32), np.array(I, np.uint16)


def _sphere(nseg, nring):
    P, N = [], []
    for j in range(nring + 1):
        ph = math.pi * j / nring
        for i in range(nseg + 1):
            th = 2 * math.pi * i / nseg
            n = (math.sin(ph) * math.cos(th), math.cos(ph), math.sin(ph) * math.sin(th))
            P.append(n)
            N.append(n)
    I = []
    for j in range(nring):
        for i in range(nseg):
            a = j * (nseg + 1) + i
            b, c, d = a + 1, a + nseg + 2, a + nseg + 1
            I += [a, c, b, a, d, c]
    return np.array(P, np.float32), np.array(N, np.float32), np.array(I, np.uint32)


def write_room(out_dir, name="room", yfov=0.9):
    os.makedirs(out_dir, exist_ok=True)
    blob = bytearray()
    views, accs = [], []

    def align():
        while len(blob) % 4:
            blob.append(0)

    def add_view(data, stride=None, target=34962):
        align()
        off = len(blob)
        blob.extend(data)
        v = {"buffer": 0, "byteOffset": off, "byteLength": len(data), "target": target}
        if stride:
            v["byteStride"] = stride
        views.append(v)
        return len(views) - 1

    def add_acc(view, ctype, count, typ, byte_offset=0):
        a = {"bufferView": view, "componentType": ctype, "count": int(count), "type": typ}
        if byte_offset:
            a["byteOffset"] = byte_offset
        accs.append(a)
        return len(accs) - 1

    # room: inward box, interleaved pos/normal (stride 24), u16 indices
    P, N, I = _box_faces((0, 2, 0), (4, 2, 4), inward=True)
    inter = np.concatenate([P, N], axis=1).astype(np.float32)
    vi = add_view(inter.tobytes(), stride=24)
    room_pos = add_acc(vi, 5126, len(P), "VEC3", 0)
    room_nrm = add_acc(vi, 5126, len(P), "VEC3", 12)
    room_idx = add_acc(add_view(I.tobytes(), target=34963), 5123, len(I), "SCALAR")
    # sphere (unit), u32 indices, separate views; idx view has a leading pad used via accessor byteOffset
    SP, SN, SI = _sphere(16, 8)
    sp_pos = add_acc(add_view(SP.tobytes()), 5126, len(SP), "VEC3")
    sp_nrm = add_acc(add_view(SN.tobytes()), 5126, len(SN), "VEC3")
    sp_idx = add_acc(add_view(b"\0" * 8 + SI.tobytes(), target=34963), 5125, len(SI), "SCALAR", byte_offset=8)
    # light quad, non-indexed (6 vertices), facing down
    LP = np.array([[-1, 0, -1], [1, 0, 1], [1, 0, -1], [-1, 0, -1], [-1, 0, 1], [1, 0, 1]], np.float32)
    LN = np.tile(np.array([[0, -1, 0]], np.float32), (6, 1))
    l_pos = add_acc(add_view(LP.tobytes()), 5126, 6, "VEC3")
    l_nrm = add_acc(add_view(LN.tobytes()), 5126, 6, "VEC3")
    # a small cube, u16 indices, outward
    CP, CN, CI = _box_faces((0, 0, 0), (0.5, 0.5, 0.5), inward=False)
    c_pos = add_acc(add_view(CP.tobytes()), 5126, len(CP), "VEC3")
    c_nrm = add_acc(add_view(CN.tobytes()), 5126, len(CN), "VEC3")
    c_idx = add_acc(add_view(CI.tobytes(), target=34963), 5123, len(CI), "SCALAR")

    materials = [
        {"pbrMetallicRoughness": {"baseColorFactor": [0.75, 0.7, 0.65, 1.0], "metallicFactor": 0.0}},   # 0 walls
        {"pbrMetallicRoughness": {"baseColorFactor": [0.9, 0.9, 0.9, 1.0]}},                           # 1 metal
        {"pbrMetallicRoughness": {"baseColorFactor": [0.9, 1.0, 0.95, 0.4], "metallicFactor": 0.0}},   # 2 glass
        {"pbrMetallicRoughness": {"metallicFactor": 0.0}, "emissiveFactor": [1.0, 0.9, 0.7],
         "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 6.0}}},                 # 3 light
        {"pbrMetallicRoughness": {"baseColorFactor": [0.2, 0.5, 0.8, 1.0], "metallicFactor": 0.0},
         "extensions": {"SOME_other_extension": {}}},                                                   # 4 blue
    ]
    meshes = [
        {"primitives": [{"attributes": {"POSITION": room_pos, "NORMAL": room_nrm}, "indices": room_idx, "material": 0}]},
        {"primitives": [{"attributes": {"POSITION": sp_pos, "NORMAL": sp_nrm}, "indices": sp_idx, "material": 1},
                        {"attributes": {"POSITION": sp_pos, "NORMAL": sp_nrm}, "indices": sp_idx, "material": 2,
                         "mode": 4}]},
        {"primitives": [{"attributes": {"POSITION": l_pos, "NORMAL": l_nrm}, "material": 3}]},
        {"primitives": [{"attributes": {"POSITION": c_pos, "NORMAL": c_nrm}, "indices": c_idx, "material": 4},
                        {"attributes": {"POSITION": c_pos, "NORMAL": c_nrm}, "indices": c_idx}]},
    ]
    a = math.radians(25.0)
    b = math.radians(-20.0)
    nodes = [
        {"name": "root", "children": [1, 2, 3, 5, 7], "translation": [0.0, 0.0, 0.0]},               # 0
        {"mesh": 0},                                                                                 # 1 room
        {"mesh": 1, "translation": [1.2, 0.9, 0.4], "scale": [0.9, 0.9, 0.9]},                      # 2 spheres
        {"mesh": 2, "translation": [0.0, 3.98, 0.0]},                                               # 3 light
        {"mesh": 3, "matrix": [1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0,
                               -0.5, 0.0, 0.3, 1.0]},                                               # 4 cube (matrix)
        {"children": [4], "translation": [-1.4, 0.6, -0.8],
         "rotation": [0.0, math.sin(a / 2), 0.0, math.cos(a / 2)], "scale": [1.3, 0.8, 1.1]},       # 5 cube parent
        {"camera": 0, "translation": [0.0, 0.3, 0.0],
         "rotation": [math.sin(b / 2), 0.0, 0.0, math.cos(b / 2)]},                                 # 6 camera
        {"children": [6], "translation": [0.0, 2.2, 3.6]},                                          # 7 camera rig
        {"mesh": 3, "translation": [0.0, 1.0, 0.0]},                                                # 8 only in scene 1
    ]
    gltf = {
        "asset": {"version": "2.0"},
        "scene": 0,
        "scenes": [{"nodes": [0]}, {"nodes": [8, 1]}],
        "nodes": nodes,
        "cameras": [{"type": "perspective", "perspective": {"yfov": yfov, "znear": 0.01}}],
        "meshes": meshes, "materials": materials, "accessors": accs, "bufferViews": views,
        "buffers": [{"uri": name + ".bin", "byteLength": len(blob)}],
    }
    with open(os.path.join(out_dir, name + ".bin"), "wb") as f:
        f.write(bytes(blob))
    path = os.path.join(out_dir, name + ".gltf")
    with open(path, "w") as f:
        json.dump(gltf, f)
    return path, gltf


def write_variant(out_dir, mutate, name="variant"):
    """write_room, then apply `mutate(gltf_dict)` and rewrite the .gltf (for error cases)."""
    path, g = write_room(out_dir, name)
    mutate(g)
    with open(path, "w") as f:
        json.dump(g, f)
    return path
