"""Dense-map outputs on the CPU (no GPU): the product's marching-cubes table (thor_slam_amd/dense.py)
equals the oracle's independent derivation and the generated header; the oracle's meshes are
watertight and face the outside (sphere, random sign volumes with every ambiguous face
configuration); the oracle ESDF / slice equal brute-force nearest-site distances."""

from __future__ import annotations

import importlib.util
from collections import Counter
from pathlib import Path

import numpy as np

from oracle import numpy_dense as D
from thor_slam_amd import dense

ROOT = Path(__file__).resolve().parents[1]


def _edge_balance(tris: np.ndarray) -> int:
    """Directed edges not matched by exactly one opposite edge (0 for a closed oriented surface)."""
    e = Counter()
    for t in tris:
        for a, b in ((0, 1), (1, 2), (2, 0)):
            e[(tuple(t[a]), tuple(t[b]))] += 1
    return sum(1 for (a, b), k in e.items() if k != 1 or e.get((b, a), 0) != 1)


def test_table_matches_oracle_derivation():
    count, tab = dense.mc_triangle_table()
    assert tab.shape[1] == 5 and count.max() == 5
    for cfg in range(256):
        assert [tuple(int(x) for x in t) for t in tab[cfg, :count[cfg]]] == D.CONFIG_TRIANGLES[cfg], cfg
        assert (tab[cfg, count[cfg]:] == -1).all()
    assert count[0] == 0 and count[255] == 0


def test_generated_header_is_current():
    spec = importlib.util.spec_from_file_location("gen_tables", ROOT / "tools" / "gen_tables.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert (ROOT / "thor-slam_amd" / "csrc" / "tslam_mc_table.h").read_text() == mod.render_mc(), "run tools/gen_tables.py"


def _sphere(n=24, s=0.1, r=0.7):
    origin = (-1.2, -1.2, -1.2)
    ax = origin[0] + s * (np.arange(n) + 0.5)
    Z, Y, X = np.meshgrid(ax, ax, ax, indexing="ij")
    return (np.sqrt(X ** 2 + Y ** 2 + Z ** 2) - r).astype(np.float32), origin, s


def test_sphere_mesh_closed_and_outward():
    sd, origin, s = _sphere()
    m = D.extract_mesh(sd, np.ones_like(sd), origin, s, 1e-4)
    assert m.shape[0] > 1000
    assert _edge_balance(m) == 0
    nrm = np.cross(m[:, 1] - m[:, 0], m[:, 2] - m[:, 0])
    assert (np.einsum("ij,ij->i", nrm, m.mean(axis=1)) > 0).all()      # away from the centre
    r = np.linalg.norm(m.reshape(-1, 3), axis=1)
    assert np.abs(r - 0.7).max() < 0.02                                 # on the sphere


def test_random_volumes_watertight():
    for seed in range(4):
        v = np.random.default_rng(seed).standard_normal((12, 12, 12)).astype(np.float32)
        v[[0, -1]] = 1.0
        v[:, [0, -1]] = 1.0
        v[:, :, [0, -1]] = 1.0                                          # closed by an outside border
        m = D.extract_mesh(v, np.ones_like(v), (0.0, 0.0, 0.0), 1.0, 1e-4)
        assert m.shape[0] > 1000 and _edge_balance(m) == 0, seed


def test_unobserved_cubes_are_skipped():
    sd, origin, s = _sphere(n=12, s=0.2)
    w = np.ones_like(sd)
    full = D.extract_mesh(sd, w, origin, s, 1e-4)
    w[:, :, :6] = 0.0
    half = D.extract_mesh(sd, w, origin, s, 1e-4)
    assert 0 < half.shape[0] < full.shape[0]
    assert (half[..., 0] >= origin[0] + s * 6.5 - 1e-6).all()


def _brute_esdf(tsdf, weight, s, max_dist, site_vox, min_weight):
    R = D.radius(max_dist, s)
    obs = weight >= np.float32(min_weight)
    site = obs & (np.abs(tsdf) <= np.float32(site_vox * s))
    pts = np.argwhere(site)
    idx = np.argwhere(np.ones_like(tsdf, dtype=bool))
    d2 = np.full(idx.shape[0], 10 ** 9, dtype=np.int64)
    for p in pts:
        d2 = np.minimum(d2, ((idx - p) ** 2).sum(axis=1))
    d2 = d2.reshape(tsdf.shape)
    tab = D.distance_table(R, s)
    dist = np.where(d2 > R * R, np.float32(max_dist), tab[np.minimum(d2, R * R)])
    dist = np.where(obs & (tsdf < 0) & (d2 > 0), -dist, dist)
    return np.where(obs, dist, np.float32(np.nan)).astype(np.float32)


def test_esdf_equals_brute_force():
    rng = np.random.default_rng(7)
    t = rng.uniform(-0.6, 0.6, (9, 11, 13)).astype(np.float32)
    w = (rng.random((9, 11, 13)) > 0.2).astype(np.float32)
    for max_dist in (0.35, 0.6, 5.0):          # R = 3, 6, 50 voxels of 0.1 m
        got = D.esdf(t, w, 0.1, max_dist, site_vox=1.0)
        want = _brute_esdf(t, w, 0.1, max_dist, 1.0, 1e-4)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    assert np.isnan(got[w == 0]).all() and (got[(w > 0) & (np.abs(t) <= np.float32(0.1))] == 0).all()


def test_esdf_slice_equals_brute_force():
    rng = np.random.default_rng(8)
    t = rng.uniform(-0.6, 0.6, (10, 6, 12)).astype(np.float32)
    w = (rng.random((10, 6, 12)) > 0.3).astype(np.float32)
    got = D.esdf_slice(t, w, 0.1, 0.5, 2, 4)
    band_t, band_w = t[:, 2:4], w[:, 2:4]
    site = ((band_w >= np.float32(1e-4)) & (np.abs(band_t) <= np.float32(0.1))).any(axis=1)
    obs = (band_w >= np.float32(1e-4)).any(axis=1)
    pts = np.argwhere(site)
    R = D.radius(0.5, 0.1)
    tab = D.distance_table(R, 0.1)
    for (k, i), val in np.ndenumerate(got):
        if not obs[k, i]:
            assert np.isnan(val)
            continue
        d2 = min(((pts - (k, i)) ** 2).sum(axis=1).min() if len(pts) else 10 ** 9, 10 ** 9)
        assert val == (np.float32(0.5) if d2 > R * R else tab[d2])
