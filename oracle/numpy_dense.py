"""SURVEY.md §8f item 4 (after integration) — the dense-map outputs nvblox publishes from its TSDF
(surface mesh, Euclidean signed distance field, 2-D distance slice), CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for ``k_dense.hip``, never imported
by the product.  The reference runs nvblox (``launch/thor_nvblox.launch.py:21-103``) on the RGB-D
topics of ``scripts/run_pipeline.py:218-256``; nvblox is external and absent from
``/root/reference``, so the rules (``thor_slam_amd/dense.py``'s docstring) are the spec and parity
against nvblox itself is unpinned.  This file derives the marching-cubes configurations its own way
(crossings listed around each face, every leaving crossing joined to the entering crossing that
opened its run) and evaluates the ESDF with NumPy shifts; tests check both against the product's
table and kernels.

Volumes are [nz][ny][nx] f32 as ``numpy_tsdf``; voxel (i, j, k) has centre origin + s (i, j, k) +
s / 2, evaluated in f64 and rounded to f32.
"""

from __future__ import annotations

import numpy as np

CORNER_OFFSETS = np.array([(n & 1, (n >> 1) & 1, (n >> 2) & 1) for n in range(8)], dtype=np.int64)


def _edge_id(c0: int, c1: int) -> int:
    """Edge 4 a + m between corners differing in bit a; m = the two other bits of the lower corner, low axis first."""
    a = {1: 0, 2: 1, 4: 2}[c0 ^ c1]
    lo = min(c0, c1)
    o = [b for b in (0, 1, 2) if b != a]
    return 4 * a + ((lo >> o[0]) & 1) + 2 * ((lo >> o[1]) & 1)


def _face_cycles():
    """The 6 faces' corners, counter-clockwise about the outward normal (right-handed u, v, a)."""
    out = []
    for a, u, v in ((0, 1, 2), (1, 2, 0), (2, 0, 1)):
        ring = [(1 << u) * x + (1 << v) * y for x, y in ((0, 0), (1, 0), (1, 1), (0, 1))]
        out.append(list(reversed(ring)))                     # side 0: outward normal -e_a
        out.append([c | (1 << a) for c in ring])             # side 1: +e_a
    return out


def configuration_triangles(cfg: int) -> list[tuple[int, int, int]]:
    """Triangles (edge ids) of one configuration, facing the outside (positive tsdf)."""
    link = {}
    for ring in _face_cycles():
        ins = [bool((cfg >> c) & 1) for c in ring]
        crossings = []   # (edge, leaving?) in counter-clockwise order
        for k in range(4):
            if ins[k] != ins[(k + 1) % 4]:
                crossings.append((_edge_id(ring[k], ring[(k + 1) % 4]), ins[k]))
        for idx, (e, leaving) in enumerate(crossings):
            if leaving:   # the entering crossing just before it (cyclically) opened this run
                j = idx - 1
                while crossings[j % len(crossings)][1]:
                    j -= 1
                link[e] = crossings[j % len(crossings)][0]
    tris, seen = [], set()
    for start in sorted(link):
        if start in seen:
            continue
        loop, e = [], start
        while e not in seen:
            seen.add(e)
            loop.append(e)
            e = link[e]
        for r in range(len(loop)):   # first rotation without a triangle flat on a cube face
            rot = loop[r:] + loop[:r]
            fan = [(rot[0], rot[q + 1], rot[q]) for q in range(1, len(rot) - 1)]   # reversed: the loop turns inward
            if not any(_flat(t) for t in fan):
                tris.extend(fan)
                break
        else:
            raise AssertionError("no flat-free fan")
    return tris


def _midpoint(e: int) -> np.ndarray:
    a, m = divmod(e, 4)
    p = np.full(3, 0.5)
    o = [b for b in (0, 1, 2) if b != a]
    p[o[0]], p[o[1]] = m & 1, m >> 1
    return p


def _flat(tri) -> bool:
    """All three edge midpoints on one face of the unit cube."""
    P = np.array([_midpoint(e) for e in tri])
    return bool(np.any(np.all(P == 0.0, axis=0) | np.all(P == 1.0, axis=0)))


CONFIG_TRIANGLES = [configuration_triangles(c) for c in range(256)]


def _centres(origin, s, n, axis):
    return np.asarray(origin[axis] + s * (np.arange(n) + 0.5), dtype=np.float64).astype(np.float32)


def extract_mesh(tsdf: np.ndarray, weight: np.ndarray, origin, s: float, min_weight: float,
                 color: np.ndarray | None = None):
    """Triangle soup [n][3 vertices][xyz] f32 in cube order ([k][j][i] of the base corner); with a
    colour layer ``color`` [nz][ny][nx][3] also (triangles, colours [n][3][3] f32): each vertex
    takes the colour of its edge's voxel nearer to it (the base voxel when t < 1/2)."""
    nz, ny, nx = tsdf.shape
    if min(nx, ny, nz) < 2:
        empty = np.zeros((0, 3, 3), dtype=np.float32)
        return empty if color is None else (empty, empty.copy())
    sl = [(slice(dz, nz - 1 + dz), slice(dy, ny - 1 + dy), slice(dx, nx - 1 + dx)) for dx, dy, dz in CORNER_OFFSETS]
    obs = np.ones((nz - 1, ny - 1, nx - 1), dtype=bool)
    cfg = np.zeros((nz - 1, ny - 1, nx - 1), dtype=np.int64)
    for n in range(8):
        obs &= weight[sl[n]] >= np.float32(min_weight)
        cfg |= (tsdf[sl[n]] < 0).astype(np.int64) << n
    cfg[~obs] = 0
    k, j, i = np.nonzero(cfg)   # row-major: cube order
    cx, cy, cz = _centres(origin, s, nx, 0), _centres(origin, s, ny, 1), _centres(origin, s, nz, 2)
    sf = np.float32(s)
    out, cols = [], []
    for q in range(k.size):
        for tri in CONFIG_TRIANGLES[cfg[k[q], j[q], i[q]]]:
            v, vc = [], []
            for e in tri:
                a, m = divmod(e, 4)
                o = [b for b in (0, 1, 2) if b != a]
                off = [0, 0, 0]
                off[o[0]], off[o[1]] = m & 1, m >> 1
                bi, bj, bk = i[q] + off[0], j[q] + off[1], k[q] + off[2]
                ei, ej, ek = bi + (a == 0), bj + (a == 1), bk + (a == 2)
                va, vb = tsdf[bk, bj, bi], tsdf[ek, ej, ei]
                t = va / (va - vb)
                p = [cx[bi], cy[bj], cz[bk]]
                p[a] = p[a] + t * sf
                v.append(p)
                if color is not None:
                    vc.append(color[bk, bj, bi] if t < np.float32(0.5) else color[ek, ej, ei])
            out.append(v)
            cols.append(vc)
    tris = np.array(out, dtype=np.float32).reshape(-1, 3, 3)
    if color is None:
        return tris
    return tris, np.array(cols, dtype=np.float32).reshape(-1, 3, 3)


def _window_pass(g: np.ndarray, axis: int, R: int, cap: int) -> np.ndarray:
    """min over |d| <= R of g[x + d] + d^2 along `axis`, capped at `cap`."""
    out = g.copy()
    n = g.shape[axis]
    for d in range(1, min(R, n - 1) + 1):
        sh = [slice(None)] * g.ndim
        src = [slice(None)] * g.ndim
        sh[axis], src[axis] = slice(d, None), slice(None, n - d)       # from x - d
        out[tuple(sh)] = np.minimum(out[tuple(sh)], g[tuple(src)] + d * d)
        sh[axis], src[axis] = slice(None, n - d), slice(d, None)       # from x + d
        out[tuple(sh)] = np.minimum(out[tuple(sh)], g[tuple(src)] + d * d)
    return np.minimum(out, cap)


def radius(max_dist: float, s: float) -> int:
    return int(np.floor(max_dist / s + 1e-9))


def distance_table(R: int, s: float) -> np.ndarray:
    """f32 distance of every squared voxel distance 0..R^2: sqrt in f32, times s in f32."""
    return (np.sqrt(np.arange(R * R + 1, dtype=np.float32)) * np.float32(s)).astype(np.float32)


def _finish(d2, observed, negative, R, s, max_dist):
    tab = distance_table(R, s)
    far = d2 > R * R
    dist = np.where(far, np.float32(max_dist), tab[np.minimum(d2, R * R)])
    dist = np.where(negative, -dist, dist).astype(np.float32)
    return np.where(observed, dist, np.float32(np.nan)).astype(np.float32)


def esdf(tsdf: np.ndarray, weight: np.ndarray, s: float, max_dist: float, site_vox: float = 1.0,
         min_weight: float = 1e-4) -> np.ndarray:
    """Signed Euclidean distance field [nz][ny][nx] f32 (NaN = unobserved)."""
    R = radius(max_dist, s)
    cap = R * R + 1
    observed = weight >= np.float32(min_weight)
    site = observed & (np.abs(tsdf) <= np.float32(site_vox * s))
    g = np.where(site, 0, cap).astype(np.int64)
    for axis in (2, 1, 0):   # x, y, z
        g = _window_pass(g, axis, R, cap)
    return _finish(g, observed, observed & (tsdf < 0) & (g > 0), R, s, max_dist)


def esdf_slice(tsdf: np.ndarray, weight: np.ndarray, s: float, max_dist: float, y0: int, y1: int,
               site_vox: float = 1.0, min_weight: float = 1e-4) -> np.ndarray:
    """2-D distance map [nz][nx] f32 over the height band y0 <= j < y1 (unsigned; NaN = unobserved column)."""
    R = radius(max_dist, s)
    cap = R * R + 1
    t, w = tsdf[:, y0:y1, :], weight[:, y0:y1, :]
    observed = (w >= np.float32(min_weight)).any(axis=1)
    site = ((w >= np.float32(min_weight)) & (np.abs(t) <= np.float32(site_vox * s))).any(axis=1)
    g = np.where(site, 0, cap).astype(np.int64)
    for axis in (1, 0):   # x, z
        g = _window_pass(g, axis, R, cap)
    return _finish(g, observed, np.zeros_like(observed), R, s, max_dist)
