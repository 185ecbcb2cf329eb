"""Writes tests/golden/kats.json: the reference's 13 known-answer tests as data.

Inputs and expected outputs are transcribed from the reference's inline unit
tests (/root/reference/src, cited per vector).  Directions written as
`normalize(v)` in the reference are stored raw with "normalize": true; the
test applies cgmath's normalize (v * (1/|v|)) before the query.
Run: python tests/golden/make_kats.py
"""
import json
import os

BOX_MIN, BOX_MAX = [-1.0, -2.0, -1.0], [1.0, 2.0, 1.0]
RAYS = {  # aabb.rs:118-151 and primitives/box.rs:129-165 use the same five rays
    "a": ([0.0, 0.0, 2.0], [0.0, 0.0, 1.0]),
    "b": ([0.0, 0.0, -2.0], [0.0, 0.0, 1.0]),
    "c": ([2.0, 0.0, -2.0], [0.0, 0.0, 1.0]),
    "d": ([-2.0, 0.0, -2.0], [1.0, 0.0, 1.0]),
    "e": ([-1.0, 0.0, -2.0], [0.0, 0.0, 1.0]),
}
SQRT2 = 2.0 ** 0.5

kats = {
    "source": "/root/reference/src unit tests (#[cfg(test)]), transcribed as data",
    "aabb": [  # aabb.rs:118-151: AABB{min:(-1,-2,-1), max:(1,2,1)}.intersects(ray)
        {"name": f"aabb::{k}", "cite": f"aabb.rs:{line}", "min": BOX_MIN, "max": BOX_MAX,
         "origin": RAYS[k][0], "dir": RAYS[k][1], "normalize": True, "expected_t": exp}
        for k, line, exp in [("a", "118-123", None), ("b", "125-130", 1.0), ("c", "132-137", None),
                             ("d", "139-144", SQRT2), ("e", "146-151", 1.0)]
    ],
    "box": [  # primitives/box.rs:129-171: Box::new((1,2,1)).intersection(ray), exact t/normal/inside
        {"name": f"box::{k}", "cite": f"primitives/box.rs:{line}", "sizes": [1.0, 2.0, 1.0],
         "origin": RAYS[k][0], "dir": RAYS[k][1], "normalize": True, "expected": exp}
        for k, line, exp in [
            ("a", "130-134", None),
            ("b", "137-142", {"t": 1.0, "normal": [0.0, 0.0, -1.0], "inside": False}),
            ("c", "145-149", None),
            ("d", "152-157", {"t": SQRT2, "normal": [0.0, 0.0, -1.0], "inside": False}),
            ("e", "160-165", {"t": 1.0, "normal": [0.0, 0.0, -1.0], "inside": False}),
        ]
    ],
    "triangle_aaa": {  # primitives/triangle.rs:98-128
        "cite": "primitives/triangle.rs:98-128",
        "a": [-4.0, -2.0, 10.0], "ba": [1.0, 6.0, 0.0], "ca": [3.0, 0.0, 0.0],
        "position": [0.0, 0.0, -6.0], "u": 0.6, "v": 0.3, "pos": [-3.0, 2.0, 4.0],
        "note": "ray origin = pos, dir = normalize(world + pos) with world = ba'*u + ca'*v + a' of the "
                "TrianglePrimitive; intersect_lights over a 1-triangle light BVH must call back",
        "expected_called": True,
    },
    "triangle_bbb": {  # primitives/triangle.rs:130-144
        "cite": "primitives/triangle.rs:130-144",
        "a": [0.0, 0.0, 2.0], "b": [1.0, 0.0, 2.0], "c": [0.0, 1.0, 0.0],
        "origin": [0.1541891385674881, 0.7047585918803002, 0.5904828162393995],
        "dir": [-0.0759650747603601, -0.4459213624433466, 0.8918427248866934],
        "expected": None,
    },
    "cof_aaa": {  # gltf/scene_builder.rs:408-426
        "cite": "gltf/scene_builder.rs:408-426",
        "scales": [2.0, 3.0, 4.0], "angles_deg": [10.0, 20.0, 30.0],
        "normals": [[1.0, 2.0, 3.0], [-1.0, 2.0, 3.0], [-1.0, -2.0, 1.0]],
        "property": "normalize(cof(M) n) == normalize((M^T)^-1 n) within f64::EPSILON (approx default)",
    },
    "philox4x32_10": [  # Random123 kat_vectors (the RNG that replaces ThreadRng)
        {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
        {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
        {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
         "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
    ],
}

if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", path)
