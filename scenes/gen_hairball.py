#!/usr/bin/env python3
"""Synthetic hairball glTF (BASELINE.json configs[4]).

10,000,000 thin random triangles (seeded) inside a unit sphere, f32 POSITION +
NORMAL (geometric normals), no indices, one external .bin; three diffuse hair
tones plus one emissive quad above (the glTF path has a black background,
scene_builder.rs:17) and one perspective camera.  Triangles are ~6e-3 across so
|ba x ca| stays far above the 1e-11 determinant cull (triangle.rs:51).  The
working set (~1.7 GB of device BVH + triangles) is past the 256 MiB Infinity
Cache: the true-HBM traversal case.

    python scenes/gen_hairball.py [out_dir] [--tris N] [--seed S]
Deterministic for a given (N, seed); written in chunks so memory stays bounded.
"""
import argparse
import json
import math
import os

import numpy as np


def tri_chunk(rng, n):
    """n triangles: centre uniform in the unit ball, a random strand direction."""
    u = rng.random(n)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    centre = d * np.cbrt(u)[:, None] * 0.98
    t = rng.standard_normal((n, 3))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    w = rng.standard_normal((n, 3))
    w -= (w * t).sum(1, keepdims=True) * t
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    a = centre - t * 3e-3
    b = centre + t * 3e-3
    c = centre + w * 1.5e-3
    nrm = np.cross(b - a, c - a)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    P = np.stack([a, b, c], axis=1).astype(np.float32)          # [n, 3 verts, 3]
    N = np.repeat(nrm[:, None, :], 3, axis=1).astype(np.float32)
    return P.reshape(-1, 3), N.reshape(-1, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir", nargs="?", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "gen"))
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--name", default="hairball")
    a = ap.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    rng = np.random.default_rng(a.seed)
    n_groups = 3
    per = [a.tris // n_groups + (1 if g < a.tris % n_groups else 0) for g in range(n_groups)]
    bin_path = os.path.join(a.out_dir, a.name + ".bin")
    views, accs, prims = [], [], []
    off = 0
    with open(bin_path, "wb") as f:
        for g, cnt in enumerate(per):  # one primitive per hair tone: positions then normals
            pos_view, nrm_view = [], []
            mn = np.full(3, np.inf)
            mx = np.full(3, -np.inf)
            ppos = off
            # positions of this group, streamed in chunks (then normals with the same stream replayed)
            state = rng.bit_generator.state
            left = cnt
            while left:
                k = min(left, 1_000_000)
                P, _ = tri_chunk(rng, k)
                mn = np.minimum(mn, P.min(0)); mx = np.maximum(mx, P.max(0))
                f.write(P.tobytes()); off += P.nbytes
                left -= k
            pnorm = off
            rng.bit_generator.state = state
            left = cnt
            while left:
                k = min(left, 1_000_000)
                _, N = tri_chunk(rng, k)
                f.write(N.tobytes()); off += N.nbytes
                left -= k
            views.append({"buffer": 0, "byteOffset": ppos, "byteLength": pnorm - ppos, "target": 34962})
            views.append({"buffer": 0, "byteOffset": pnorm, "byteLength": off - pnorm, "target": 34962})
            accs.append({"bufferView": len(views) - 2, "componentType": 5126, "count": 3 * cnt, "type": "VEC3",
                         "min": mn.tolist(), "max": mx.tolist()})
            accs.append({"bufferView": len(views) - 1, "componentType": 5126, "count": 3 * cnt, "type": "VEC3"})
            prims.append({"attributes": {"POSITION": len(accs) - 2, "NORMAL": len(accs) - 1}, "material": g,
                          "mode": 4})
        # emissive quad above the ball, facing down (two triangles, non-indexed)
        L = np.array([[-1.2, 1.6, -1.2], [1.2, 1.6, 1.2], [1.2, 1.6, -1.2],
                      [-1.2, 1.6, -1.2], [-1.2, 1.6, 1.2], [1.2, 1.6, 1.2]], np.float32)
        LN = np.tile(np.array([[0, -1, 0]], np.float32), (6, 1))
        for arr in (L, LN):
            views.append({"buffer": 0, "byteOffset": off, "byteLength": arr.nbytes, "target": 34962})
            f.write(arr.tobytes()); off += arr.nbytes
        accs.append({"bufferView": len(views) - 2, "componentType": 5126, "count": 6, "type": "VEC3",
                     "min": L.min(0).tolist(), "max": L.max(0).tolist()})
        accs.append({"bufferView": len(views) - 1, "componentType": 5126, "count": 6, "type": "VEC3"})
        prims.append({"attributes": {"POSITION": len(accs) - 2, "NORMAL": len(accs) - 1}, "material": n_groups})
    mats = [{"pbrMetallicRoughness": {"baseColorFactor": c + [1.0], "metallicFactor": 0.0}}
            for c in ([0.55, 0.35, 0.2], [0.35, 0.22, 0.12], [0.7, 0.55, 0.35])]
    mats.append({"pbrMetallicRoughness": {"metallicFactor": 0.0}, "emissiveFactor": [1.0, 0.95, 0.9],
                 "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 4.0}}})
    pitch = math.radians(-12.0)
    gltf = {
        "asset": {"version": "2.0", "generator": "gen_hairball.py"},
        "extensionsUsed": ["KHR_materials_emissive_strength"],
        "scene": 0, "scenes": [{"nodes": [0, 1]}],
        "nodes": [{"mesh": 0, "name": "hairball"},
                  {"camera": 0, "translation": [0.0, 0.7, 3.2],
                   "rotation": [math.sin(pitch / 2), 0.0, 0.0, math.cos(pitch / 2)]}],
        "cameras": [{"type": "perspective", "perspective": {"yfov": 0.75, "znear": 0.01}}],
        "meshes": [{"name": "hair", "primitives": prims}], "materials": mats,
        "accessors": accs, "bufferViews": views,
        "buffers": [{"uri": a.name + ".bin", "byteLength": off}],
    }
    with open(os.path.join(a.out_dir, a.name + ".gltf"), "w") as f:
        json.dump(gltf, f)
    print(f"wrote {a.out_dir}/{a.name}.gltf with {a.tris + 2} triangles ({off / 1e6:.0f} MB .bin)")


if __name__ == "__main__":
    main()
