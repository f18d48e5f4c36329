"""The oracle against independent brute-force definitions (it is the spec; pin it first)."""

import math

import numpy as np
import pytest

from helpers import scenario
from oracle import numpy_slam as O
from thor_slam_amd.params import HipSlamConfig, level_quotas, level_shapes


def _naive_fast(img, y, x):
    c = int(img[y, x])
    ring = [int(img[y + dy, x + dx]) - c for dx, dy in O.CIRCLE]
    best = -10**9
    for k in range(16):
        arc = [ring[(k + j) % 16] for j in range(9)]
        best = max(best, min(arc), min(-a for a in arc))
    return max(best, 0)


def test_fast_score_matches_definition():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(24, 31), dtype=np.uint8)
    img[5:12, 5:12] = 200  # a bright block gives real corners
    s = O.fast_scores(img)
    for y in range(3, 21):
        for x in range(3, 28):
            assert s[y, x] == _naive_fast(img, y, x), (y, x)
    assert (s[:3] == 0).all() and (s[:, -3:] == 0).all()


def test_fast_threshold_semantics():
    rng = np.random.default_rng(2)
    img = (rng.integers(0, 4, size=(40, 40)) * 60).astype(np.uint8)
    s = O.fast_scores(img)
    for t in (10, 40, 100):
        for y in range(3, 37):
            for x in range(3, 37):
                c = int(img[y, x])
                ring = [int(img[y + dy, x + dx]) for dx, dy in O.CIRCLE]
                corner = any(all(ring[(k + j) % 16] > c + t for j in range(9)) or
                             all(ring[(k + j) % 16] < c - t for j in range(9)) for k in range(16))
                assert (s[y, x] > t) == corner


def test_nms_keeps_independent_set_and_tiebreak():
    sc = np.zeros((30, 30), dtype=np.int32)
    sc[10, 10] = sc[10, 11] = 50  # tie: the earlier raster position survives
    sc[20, 20] = 60
    sc[21, 21] = 70
    keys = O.nms_keys(sc, 20, 4)
    x, y, s = O.decode_keys(keys)
    got = set(zip(y.tolist(), x.tolist()))
    assert got == {(10, 10), (21, 21)}
    rng = np.random.default_rng(3)
    sc = rng.integers(0, 40, size=(60, 70)).astype(np.int32)
    keys = O.nms_keys(sc, 20, 4)
    x, y, s = O.decode_keys(keys)
    pts = set(zip(y.tolist(), x.tolist()))
    for yy, xx in pts:  # no two survivors are 8-neighbours
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if (dy or dx) and (yy + dy, xx + dx) in pts:
                    pytest.fail("adjacent survivors")
    assert (s > 20).all()


def test_select_is_total_order():
    keys = np.array([(255 - 50) << 22 | 5 << 11 | 7, (255 - 50) << 22 | 5 << 11 | 3, (255 - 90) << 22 | 9 << 11 | 1], dtype=np.int64)
    sel = O.select_topk(keys, 2)
    x, y, s = O.decode_keys(sel)
    assert list(s) == [90, 50] and list(x) == [1, 3]


def test_orientation_bins_follow_the_centroid_angle():
    rng = np.random.default_rng(4)
    size = 64
    for _ in range(20):
        ang = rng.uniform(-math.pi, math.pi)
        yy, xx = np.mgrid[0:size, 0:size]
        ramp = (xx - 32) * math.cos(ang) + (yy - 32) * math.sin(ang)
        img = np.clip(128 + 6 * ramp, 0, 255).astype(np.uint8)
        b = O.orientation_bins(img, np.array([32]), np.array([32]))[0]
        deg = math.degrees(ang) % 360
        expect = int(round(deg / 12.0)) % 30
        assert b in (expect, (expect + 1) % 30, (expect - 1) % 30)


def test_brief_bit_layout():
    sm = np.zeros((64, 64), dtype=np.uint8)
    sm[32:, :] = 200  # bottom half bright
    desc = O.brief(sm, np.array([32]), np.array([31]), np.array([0]))
    pat = O.BRIEF_TABLE[0].astype(np.int64)
    for i in range(256):
        a = sm[31 + pat[i, 1], 32 + pat[i, 0]]
        b = sm[31 + pat[i, 3], 32 + pat[i, 2]]
        bit = (int(desc[0, i >> 5]) >> (i & 31)) & 1
        assert bit == int(a < b)


def _naive_match(q, t, cfg, mode):
    out = {}
    nq = sum(q["counts"])
    for l in range(cfg.n_levels):
        for ql in range(q["counts"][l]):
            i = q["offsets"][l] + ql
            cand = []
            for tl in range(t["counts"][l]):
                j = t["offsets"][l] + tl
                dx = q["kp"]["x"][i] - t["kp"]["x"][j]
                dy = q["kp"]["y"][i] - t["kp"]["y"][j]
                if mode == "stereo":
                    ok = abs(dy) <= cfg.stereo_row_tol and 1 <= dx <= (cfg.max_disparity >> l)
                else:
                    w = cfg.temporal_window >> l
                    ok = abs(dx) <= w and abs(dy) <= w
                if ok:
                    d = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(q["desc"][i], t["desc"][j]))
                    cand.append((d, j))
            out[i] = sorted(cand)
    return out, nq


def test_match_matches_naive_definition():
    cfg = HipSlamConfig(n_features=300, n_levels=2)
    sc = scenario(n=2, cfg_items=(("n_features", 300), ("n_levels", 2)))
    a, b = sc["oracle"][0]["cur"]["left"], sc["oracle"][0]["cur"]["right"]
    idx, dist, bj, second = O.match(a, b, cfg, "stereo")
    naive, _ = _naive_match(a, b, cfg, "stereo")
    rev, _ = _naive_match(b, a, cfg, "stereo_rev") if False else (None, None)
    for i, cand in naive.items():
        if not cand:
            assert bj[i] == -1
            continue
        assert (dist[i], bj[i]) == cand[0]
        assert second[i] == (cand[1][0] if len(cand) > 1 else 256)
    assert (idx >= 0).sum() > 50
    del rev


def test_level_helpers_agree():
    assert O.level_quotas(2000, 4) == level_quotas(2000, 4) == [1507, 376, 94, 23]
    assert O.level_shapes(640, 400, 4) == level_shapes(640, 400, 4)
    assert sum(level_quotas(4000, 4)) == 4000


def _random_pose(rng):
    from scipy.spatial.transform import Rotation

    r = Rotation.from_rotvec(rng.normal(0, 0.05, 3)).as_matrix()
    t = rng.normal(0, 0.05, 3)
    return r, t


def test_p3p_recovers_exact_pose():
    rng = np.random.default_rng(5)
    for _ in range(20):
        r, t = _random_pose(rng)
        pw = rng.uniform([-2, -1.5, 2], [2, 1.5, 6], size=(3, 3))
        pc = pw @ r.T + t
        f = pc / np.linalg.norm(pc, axis=1, keepdims=True)
        rot, trn, ok = O.p3p([[np.array([pw[k, i]]) for i in range(3)] for k in range(3)],
                             [[np.array([f[k, i]]) for i in range(3)] for k in range(3)])
        errs = [np.linalg.norm(rot[0, s] - r) + np.linalg.norm(trn[0, s] - t) for s in range(4) if ok[0, s]]
        assert errs and min(errs) < 1e-6


def test_ransac_and_refine_recover_pose_with_outliers():
    rng = np.random.default_rng(6)
    cfg = HipSlamConfig()
    r, t = _random_pose(rng)
    n = 400
    pw = rng.uniform([-3, -2, 2], [3, 2, 8], size=(n, 3))
    pc = pw @ r.T + t
    fx, fy, cx, cy = 384.0, 384.0, 319.5, 199.5
    u = fx * pc[:, 0] / pc[:, 2] + cx + rng.normal(0, 0.2, n)
    v = fy * pc[:, 1] / pc[:, 2] + cy + rng.normal(0, 0.2, n)
    out = rng.random(n) < 0.3
    u[out] += rng.uniform(-60, 60, out.sum())
    v[out] += rng.uniform(-60, 60, out.sum())
    corr = {"X": pw[:, 0], "Y": pw[:, 1], "Z": pw[:, 2], "du": cx - u, "dv": cy - v, "u": u, "v": v}
    est = O.estimate_pose(corr, (fx, fy, cx, cy), cfg, frame=7)
    assert est["status"] == 0
    assert np.linalg.norm(est["T"][:3, :3] - r) < 2e-3
    assert np.linalg.norm(est["T"][:3, 3] - t) < 5e-3
    assert abs(est["n_inliers"] - (~out).sum()) < 0.05 * n


def test_counter_rng_samples_are_distinct_and_deterministic():
    a = O.sample_triplets(0x5EED, 11, 256, 50)
    b = O.sample_triplets(0x5EED, 11, 256, 50)
    np.testing.assert_array_equal(a, b)
    assert (a[:, 0] != a[:, 1]).all() and (a[:, 0] != a[:, 2]).all() and (a[:, 1] != a[:, 2]).all()
    assert a.min() >= 0 and a.max() < 50
    assert not np.array_equal(a, O.sample_triplets(0x5EED, 12, 256, 50))


def test_tracker_follows_ground_truth():
    sc = scenario(n=4)
    src = sc["src"]
    gt0 = src.camera_pose(0, 0)
    for i, res in enumerate(sc["oracle"]):
        if i == 0:
            assert res["status"] == 2
            continue
        assert res["status"] == 0 and res["n_inliers"] > 500
        gt = np.linalg.inv(gt0) @ src.camera_pose(i, 0)
        # ~5 % drift budget on a fronto-parallel scene (yaw / x-translation ambiguity)
        assert np.linalg.norm(gt[:3, 3] - res["world_T_cam"][:3, 3]) < 0.08 * np.linalg.norm(gt[:3, 3]) + 1e-3
        assert np.linalg.norm(gt[:3, :3] - res["world_T_cam"][:3, :3]) < 2e-3


def test_rgbd_oracle_follows_ground_truth_and_record_layout():
    """RGB-D oracle (configs[4]): gray conversion, depth -> disparity and tracking vs the renderer."""
    from thor_slam_amd.calib import extract_cameras, rgbd_pairs, rgbd_undistort
    from thor_slam_amd.camera.rig import CameraRig
    from thor_slam_amd.params import HipSlamConfig
    from thor_slam_amd.rgbd import pack_rgbd
    from thor_slam_amd.synthetic import SyntheticRGBDSource

    src = SyntheticRGBDSource(width=320, height=240)
    bgr, depth = src.render_rgbd(0)
    rec = pack_rgbd(bgr, depth)
    assert rec.size == 5 * 320 * 240
    np.testing.assert_array_equal(rec[: bgr.size].reshape(bgr.shape), bgr)
    np.testing.assert_array_equal(rec[bgr.size:].view("<u2").reshape(depth.shape), depth)
    g = O.bgr_to_gray(np.array([[[255, 255, 255], [0, 0, 0], [0, 0, 255]]], dtype=np.uint8))
    assert g.tolist() == [[255, 0, (255 * 4899 + 8192) >> 14]]
    cams = extract_cameras(CameraRig([src]).calibration, 2)
    (ci, di), = rgbd_pairs(cams)
    r = rgbd_undistort(cams[ci])
    assert r.is_identity and r.baseline == 1.0
    cfg = HipSlamConfig(rgbd=True, n_features=500, n_levels=3)
    trk = O.OracleTracker(cfg, dict(fx=r.fx, fy=r.fy, cx=r.cx, cy=r.cy, baseline=r.baseline, map_l=r.map_left,
                                    map_r=r.map_right))
    for i in range(3):
        res = trk.step_rgbd(*src.render_rgbd(i))
    d = res["cur"]["disp"]
    ok = np.isfinite(d)
    assert ok.sum() > 100
    # the disparity is fx / Z of the rendered depth at the keypoint
    kp = res["cur"]["left"]["kp"]
    u, v = O.level0_coords(kp["x"][ok], kp["y"][ok], kp["level"][ok])
    _, dep = src.render_rgbd(2)
    z = dep[np.floor(v + 0.5).astype(int), np.floor(u + 0.5).astype(int)] * 0.001
    np.testing.assert_allclose(d[ok], r.fx / z, rtol=1e-12)
    gt = np.linalg.inv(src.camera_pose(0, 0)) @ src.camera_pose(2, 0)
    assert np.linalg.norm(res["world_T_cam"][:3, 3] - gt[:3, 3]) < 0.1 * np.linalg.norm(gt[:3, 3]) + 2e-3


def test_refine_rotation_prior_pulls_towards_prior():
    """IMU prior (§8f item 2): weight 0 leaves A7's refinement unchanged; a huge weight pins the
    rotation to the prior while the translation still fits the points."""
    from scipy.spatial.transform import Rotation

    rng = np.random.default_rng(5)
    n = 80
    X = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(3, 6, n)], 1)
    R = Rotation.from_rotvec([0.01, -0.02, 0.005]).as_matrix()
    t = np.array([0.02, 0.0, -0.01])
    Xc = X @ R.T + t
    fx = fy = 400.0
    cx, cy = 320.0, 200.0
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    corr = {"X": X[:, 0], "Y": X[:, 1], "Z": X[:, 2], "du": cx - u, "dv": cy - v, "u": u, "v": v}
    intr = (fx, fy, cx, cy)
    r0 = Rotation.from_rotvec([0.012, -0.018, 0.004]).as_matrix()
    a = O.refine(r0, t + 0.001, corr, intr, 4.0, 8)
    b = O.refine(r0, t + 0.001, corr, intr, 4.0, 8, prior=(np.eye(3), 0.0))
    np.testing.assert_array_equal(a[0], b[0])
    rp = Rotation.from_rotvec([0.011, -0.02, 0.005]).as_matrix()
    c = O.refine(r0, t + 0.001, corr, intr, 1e6, 8, prior=(rp, 1e12))
    assert np.abs(Rotation.from_matrix(c[0] @ rp.T).as_rotvec()).max() < 1e-6
