"""Dense-map outputs of the TSDF volume (after integration): the surface mesh
and the Euclidean signed distance field nvblox publishes (the reference runs nvblox on the RGB-D
topics, ``launch/thor_nvblox.launch.py:21-103``; nvblox itself is external and absent, so the rules
below are the spec, restated independently in ``oracle/numpy_dense.py``).

Mesh (marching cubes over the voxel centres):

* cube (i, j, k) has corners n = 0..7 at voxel (i + (n & 1), j + (n >> 1 & 1), k + (n >> 2 & 1));
  it is meshed only when all 8 corners have weight >= min_weight; corner n is *inside* when its
  tsdf < 0 and the cube's configuration is sum(inside_n << n);
* edge e = 4 a + m runs along axis a from the corner whose other two bits are m (bit a clear) to the
  corner with bit a set; it carries a vertex when exactly one end is inside, at
  p = centre(base) + t s e_a, t = tsdf(base) / (tsdf(base) - tsdf(end)) (f32 arithmetic);
* the triangles of a configuration come from the cube's faces: on each face, walked
  counter-clockwise about its outward normal, every maximal run of inside corners is cut off by one
  segment, from the vertex on the edge leaving the run to the vertex on the edge entering it (so
  diagonal inside corners are separated — the same decision from both cubes sharing the face, hence
  a watertight mesh).  The segments chain into closed loops, each listed from its smallest edge id
  not yet used and fanned from the first rotation of that list whose fan has no triangle with all
  three vertices on one cube face (an ambiguous face crossed twice by one loop would otherwise put
  a flat triangle on the face, doubled by the neighbouring cube); every triangle faces the outside
  (positive tsdf).
* triangles are emitted cube by cube in voxel storage order ([k][j][i] of the base corner), and in
  table order within a cube.

ESDF (exact, capped): sites are observed voxels (weight >= min_weight) with |tsdf| <= site_vox * s;
the distance of an observed voxel is the Euclidean distance (voxel units, integer squared) to the
nearest site, computed by three windowed passes min_{|d| <= R} (g + d^2) along x, y, z with
R = floor(max_dist / s) (exact for every distance <= R voxels), then s * sqrt(d^2) in f32, signed
negative when tsdf < 0 and the voxel is not itself a site; farther than R voxels -> +-max_dist;
unobserved voxels are NaN.  The 2-D slice marks a column (x, z) a site when any voxel of the height
band y in [y0, y1) is one (observed when any is observed) and runs the x and z passes.
"""

from __future__ import annotations

import numpy as np

N_CORNERS = 8
N_EDGES = 12


def _edge(a: int, base: int) -> int:
    """Edge id of the edge along axis a starting at corner `base` (bit a clear)."""
    others = [b for b in range(3) if b != a]
    m = ((base >> others[0]) & 1) | (((base >> others[1]) & 1) << 1)
    return 4 * a + m


def edge_corners() -> np.ndarray:
    """[12][2] (base corner, end corner) of each edge id."""
    out = np.zeros((N_EDGES, 2), dtype=np.int32)
    for a in range(3):
        others = [b for b in range(3) if b != a]
        for m in range(4):
            base = ((m & 1) << others[0]) | (((m >> 1) & 1) << others[1])
            out[4 * a + m] = (base, base | (1 << a))
    return out


def _faces() -> list[list[int]]:
    """Corner cycles of the 6 faces, counter-clockwise about the outward normal."""
    faces = []
    for a in range(3):
        u, v = (a + 1) % 3, (a + 2) % 3   # e_u x e_v = e_a
        for side in (0, 1):
            cyc = [(side << a) | (du << u) | (dv << v) for du, dv in ((0, 0), (1, 0), (1, 1), (0, 1))]
            faces.append(cyc if side == 1 else cyc[::-1])
    return faces


def _loops(cfg: int) -> list[list[int]]:
    """Closed vertex loops (edge ids) of configuration cfg, inside on the left seen from outside."""
    nxt: dict[int, int] = {}
    for cyc in _faces():
        inside = [(cfg >> c) & 1 for c in cyc]
        if all(inside) or not any(inside):
            continue
        for k in range(4):   # run of inside corners ending at corner k: inside[k] and not inside[k + 1]
            if not inside[k] or inside[(k + 1) % 4]:
                continue
            a = k
            while inside[(a - 1) % 4]:
                a = (a - 1) % 4
            out_e = _edge_between(cyc[k], cyc[(k + 1) % 4])
            in_e = _edge_between(cyc[(a - 1) % 4], cyc[a])
            assert out_e not in nxt
            nxt[out_e] = in_e
    loops, used = [], set()
    for e in sorted(nxt):
        if e in used:
            continue
        loop = [e]
        used.add(e)
        while nxt[loop[-1]] != e:
            loop.append(nxt[loop[-1]])
            used.add(loop[-1])
        loops.append(loop)
    return loops


def _edge_between(c0: int, c1: int) -> int:
    d = c0 ^ c1
    a = d.bit_length() - 1
    return _edge(a, min(c0, c1))


def _orientation_flip() -> bool:
    """True when a loop with inside on its left turns toward the inside corner (so triangles are
    reversed to face the outside)."""
    ec = edge_corners()
    loop = _loops(1)[0]   # corner 0 alone inside
    pts = []
    for e in loop:
        b, t = ec[e]
        pts.append((np.array([b & 1, b >> 1 & 1, b >> 2 & 1], float) + np.array([t & 1, t >> 1 & 1, t >> 2 & 1], float)) / 2)
    n = np.cross(pts[1] - pts[0], pts[2] - pts[0])
    return float(n.sum()) < 0.0   # the outside (corners 1..7) lies toward +(1, 1, 1)


def _edge_faces(e: int) -> set:
    b, t = (int(x) for x in edge_corners()[e])
    a = (b ^ t).bit_length() - 1
    return {(ax, (b >> ax) & 1) for ax in range(3) if ax != a}


def _fan_start(loop: list[int]) -> list[int]:
    """The first rotation of `loop` whose fan puts no triangle flat on a cube face."""
    for r in range(len(loop)):
        rot = loop[r:] + loop[:r]
        f0 = _edge_faces(rot[0])
        if not any(f0 & _edge_faces(rot[q]) & _edge_faces(rot[q + 1]) for q in range(1, len(rot) - 1)):
            return rot
    raise AssertionError("no flat-free fan")


def mc_triangle_table() -> tuple[np.ndarray, np.ndarray]:
    """(count [256] int32, tris [256][MAX][3] int8 edge ids, -1 padded) of every configuration."""
    flip = _orientation_flip()
    per = []
    for cfg in range(256):
        tris = []
        for loop in _loops(cfg):
            loop = _fan_start(loop)
            for q in range(1, len(loop) - 1):
                t = (loop[0], loop[q], loop[q + 1])
                tris.append((t[0], t[2], t[1]) if flip else t)
        per.append(tris)
    mx = max(len(t) for t in per)
    count = np.array([len(t) for t in per], dtype=np.int32)
    tab = np.full((256, mx, 3), -1, dtype=np.int8)
    for cfg, tris in enumerate(per):
        if tris:
            tab[cfg, :len(tris)] = np.array(tris, dtype=np.int8)
    return count, tab


def esdf_radius(max_dist: float, voxel: float) -> int:
    """Window R (voxels) of the capped ESDF passes."""
    return int(np.floor(max_dist / voxel + 1e-9))
