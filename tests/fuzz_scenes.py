"""Seeded random scenes in the custom scene format (scene_parser.rs), for the fuzz
parity tests (test_oracle.py, test_gpu_fuzz.py).

Each seed draws a mix of the reference's primitive kinds, materials, rotations and
lights.  Some values are chosen to stress the exact paths rather than the average
ray:

- coordinates on a 1/8 grid, so sums are exact and every vertex and box is an
  exact f32 (the compact triangle layout), next to scenes with arbitrary f64
  values (the f64 layout);
- triangle meshes with shared vertices, and exact duplicate triangles, so the
  closest-hit update's strict `<` and the BVH's visit order decide ties
  (bvh.rs:213-222);
- boxes resting exactly on a plane (coplanar faces: ties across primitive kinds,
  intersections.rs order planes -> boxes -> ellipsoids -> triangles);
- flat boxes (a zero half size), degenerate (collinear) triangles, and
  non-normalised quaternions, which take the generic (guarded) code forms;
- scenes without lights, and scenes whose only lights are triangles or ellipsoids.
"""
import numpy as np

GRID = 0.125


def _g(rng, lo, hi):
    """A value on the 1/8 grid in [lo, hi]."""
    return float(np.round(rng.uniform(lo, hi) / GRID) * GRID)


def _v(rng, lo, hi, grid):
    if grid:
        return [_g(rng, lo, hi) for _ in range(3)]
    return [float(x) for x in rng.uniform(lo, hi, 3)]


def _fmt(xs):
    return " ".join(repr(float(x)) for x in xs)


def _quat(rng):
    """ROTATION x y z w (scene_parser.rs next_quat): unit about a random axis, about one
    coordinate axis, or (rarely) not normalised."""
    k = rng.integers(0, 4)
    if k == 0:
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
    elif k == 1:
        ax = rng.integers(0, 3)
        a = rng.uniform(-np.pi, np.pi) / 2
        q = np.zeros(4)
        q[ax] = np.sin(a)
        q[3] = np.cos(a)
    elif k == 2:
        q = rng.normal(size=4) * rng.uniform(0.5, 1.5)
    else:
        return None
    return [float(x) for x in q]


def _material(rng, lines, light_ok):
    lines.append("COLOR " + _fmt(rng.uniform(0.05, 1.0, 3)))
    m = rng.integers(0, 6)
    if m == 0:
        lines.append("METALLIC")
    elif m == 1:
        lines.append("DIELECTRIC")
        lines.append("IOR " + repr(float(rng.uniform(1.1, 2.2))))
    if light_ok and rng.random() < 0.35:
        lines.append("EMISSION " + _fmt(rng.uniform(0.5, 12.0, 3)))


def random_scene(seed, width=None, height=None, spp=2, depth=None, tri_only=False):
    """tri_only: triangles on the grid and nothing else (no planes, no mesh rotation),
    so the scene is triangle-only with every coordinate an exact f32 — the compact
    triangle layout and its pair lines (rt_layout.h) apply."""
    rng = np.random.default_rng(seed)
    grid = bool(rng.random() < 0.6) or tri_only
    w = width or int(rng.choice([8, 17, 24, 31, 64]))
    h = height or int(rng.choice([5, 12, 16, 40]))
    lines = [f"DIMENSIONS {w} {h}", f"SAMPLES {spp}", f"RAY_DEPTH {depth or int(rng.integers(1, 9))}",
             "BG_COLOR " + _fmt(rng.uniform(0, 0.3, 3)),
             "CAMERA_POSITION " + _fmt([_g(rng, -0.5, 0.5), _g(rng, -0.5, 0.5), -3.0]),
             "CAMERA_RIGHT 1 0 0", "CAMERA_UP 0 1 0",
             "CAMERA_FORWARD " + _fmt([_g(rng, -0.25, 0.25), _g(rng, -0.25, 0.25), 1.0]),
             "CAMERA_FOV_X " + repr(float(rng.uniform(0.6, 1.4)))]
    style = 1 if tri_only else rng.integers(0, 3)  # 0 shapes only, 1 triangles (+ planes), 2 both
    floor = -1.0
    # planes: an open room, axis-aligned or tilted
    for k in range(0 if tri_only else int(rng.integers(0, 6))):
        lines.append("NEW_PRIMITIVE")
        ax = k % 3
        n = [0.0, 0.0, 0.0]
        n[ax] = 1.0 if k < 3 else -1.0
        if rng.random() < 0.3:
            n = [x + float(rng.uniform(-0.2, 0.2)) for x in n]
        pos = [0.0, 0.0, 0.0]
        pos[ax] = floor if n[ax] > 0 else 1.5
        if ax == 2 and n[ax] > 0:
            pos[ax] = -4.0  # behind the camera
        lines.append("PLANE " + _fmt(n))
        lines.append("POSITION " + _fmt(pos))
        if rng.random() < 0.2:
            q = _quat(rng)
            if q:
                lines.append("ROTATION " + _fmt(q))
        _material(rng, lines, light_ok=False)
    has_floor = any(l == "POSITION 0.0 -1.0 0.0" for l in lines)
    if style in (0, 2):
        for _ in range(int(rng.integers(0, 6))):
            lines.append("NEW_PRIMITIVE")
            hs = _v(rng, 0.05, 0.5, grid)
            if rng.random() < 0.1:
                hs[int(rng.integers(0, 3))] = 0.0  # flat box
            pos = _v(rng, -0.9, 0.9, grid)
            rest = has_floor and rng.random() < 0.4
            if rest:
                pos[1] = floor + hs[1]  # bottom face on the floor plane, exactly on the grid
            lines.append("BOX " + _fmt(hs))
            lines.append("POSITION " + _fmt(pos))
            if not rest and rng.random() < 0.6:
                q = _quat(rng)
                if q:
                    lines.append("ROTATION " + _fmt(q))
            _material(rng, lines, light_ok=True)
        for _ in range(int(rng.integers(0, 5))):
            lines.append("NEW_PRIMITIVE")
            r = _v(rng, 0.05, 0.45, grid)
            if rng.random() < 0.4:
                r = [r[0]] * 3
            lines.append("ELLIPSOID " + _fmt(r))
            lines.append("POSITION " + _fmt(_v(rng, -0.9, 0.9, grid)))
            if rng.random() < 0.5:
                q = _quat(rng)
                if q:
                    lines.append("ROTATION " + _fmt(q))
            _material(rng, lines, light_ok=True)
    if style in (1, 2):
        tris = []
        # a height-field mesh with shared vertices (n x m quads, two triangles each)
        big = rng.random() < 0.15  # deep triangle BVH: the traversal stack's spill part
        n, m = (int(rng.integers(16, 33)), int(rng.integers(16, 33))) if big else \
            (int(rng.integers(2, 7)), int(rng.integers(2, 7)))
        x0, z0 = _g(rng, -1.0, 0.0), _g(rng, -0.5, 0.5)
        sx, sz = (0.0625, 0.0625) if big else (0.25, 0.25)
        hgt = {}
        for i in range(n + 1):
            for j in range(m + 1):
                hgt[i, j] = _g(rng, -0.9, -0.4) if grid else float(rng.uniform(-0.9, -0.4))
        for i in range(n):
            for j in range(m):
                p = [[x0 + (i + a) * sx, hgt[i + a, j + b], z0 + (j + b) * sz] for a, b in ((0, 0), (1, 0), (1, 1), (0, 1))]
                tris.append(p[0] + p[1] + p[2])
                tris.append(p[0] + p[2] + p[3])
        for _ in range(int(rng.integers(0, 12))):  # free triangles
            a = _v(rng, -0.9, 0.9, grid)
            tris.append(a + [a[k] + _g(rng, -0.5, 0.5) for k in range(3)] + [a[k] + _g(rng, -0.5, 0.5) for k in range(3)])
        if rng.random() < 0.5:  # a degenerate (collinear) triangle
            a = _v(rng, -0.5, 0.5, True)
            d = _v(rng, -0.25, 0.25, True)
            tris.append(a + [a[k] + d[k] for k in range(3)] + [a[k] + 2 * d[k] for k in range(3)])
        for _ in range(int(rng.integers(0, 4))):  # exact duplicates: ties at every hit
            tris.append(list(tris[int(rng.integers(0, len(tris)))]))
        order = rng.permutation(len(tris))
        mesh_q = _quat(rng) if rng.random() < 0.3 and not tri_only else None
        for k in order:
            lines.append("NEW_PRIMITIVE")
            lines.append("TRIANGLE " + _fmt(tris[k]))
            if mesh_q:
                lines.append("ROTATION " + _fmt(mesh_q))
            _material(rng, lines, light_ok=rng.random() < 0.15)
    return "\n".join(lines) + "\n"
