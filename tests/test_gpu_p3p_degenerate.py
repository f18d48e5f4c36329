"""A7's degenerate P3P samples: a crafted correspondence set whose RANSAC
hypotheses include exactly collinear world points, coincident points, points on one ray (identical
bearings) and near-collinear points, injected through ``TSLAM_BUF_CORR`` / ``TSLAM_BUF_STATS`` and
solved by ``TSLAM_KERNEL_POSE_SOLVE`` (k_p3p -> k_ransac / k_ransac_all -> k_refine).

The counter RNG's triplets are known in advance (``oracle.sample_triplets``), so the degenerate
configurations are placed exactly on chosen hypotheses.  Against ``oracle/numpy_slam.py`` p3p /
estimate_pose: every hypothesis' validity mask and every valid candidate's R, t bit for bit (the
NaN / inf the divisions by zero produce fail the same finiteness tests), the RANSAC winner and
counts identical, and the refined pose within 1e-9."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import make_source, rel_frobenius, rig_calibration
from oracle import numpy_slam as O
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.params import HipSlamConfig

pytestmark = pytest.mark.gpu

FRAME = 1        # the injected batch's global frame (seeds the RANSAC draw)
N_CORR = 200
KINDS = ("collinear", "coincident", "one_ray", "near_collinear")


def _rect():
    cams = extract_cameras(rig_calibration(make_source(0)), 2)
    (li, ri), = stereo_pairs(cams)
    return stereo_rectify(cams[li], cams[ri])


def crafted_set(cfg, intr, seed: int = 4):
    """(corr dict in keypoint order, {kind: [hypotheses]}): 8 hypotheses of each degenerate kind
    whose three samples are that configuration, the rest of the rows true inliers of one motion
    (80 %) or gross outliers."""
    fx, fy, cx, cy = intr
    rng = np.random.default_rng(seed)
    tri = O.sample_triplets(cfg.ransac_seed, FRAME, cfg.ransac_hypotheses, N_CORR)
    R = O.cayley(np.array([0.02, -0.03, 0.01]))
    t = np.array([0.05, -0.02, 0.1])
    X = np.full((N_CORR, 3), np.nan)
    uv_override = {}
    used = np.zeros(N_CORR, dtype=bool)
    targets = {k: [] for k in KINDS}
    kinds = [k for k in KINDS for _ in range(8)]
    for h in range(cfg.ransac_hypotheses):
        if not kinds:
            break
        idx = tri[h]
        if used[idx].any():
            continue
        kind = kinds.pop(0)
        targets[kind].append(h)
        used[idx] = True
        if kind == "collinear":   # one axis-parallel line: the differences are exact, their cross 0
            y0, z0 = rng.uniform(-1.0, 1.0), float(rng.integers(3, 7))
            for k, i in enumerate(idx):
                X[i] = [-1.0 + 0.75 * k + 0.125 * rng.integers(0, 4), y0, z0]
        elif kind == "coincident":   # the same point (and observation) two or three times
            p = [rng.uniform(-1.5, 1.5), rng.uniform(-1.0, 1.0), rng.uniform(3.0, 7.0)]
            q = [rng.uniform(-1.5, 1.5), rng.uniform(-1.0, 1.0), rng.uniform(3.0, 7.0)]
            X[idx[0]], X[idx[1]], X[idx[2]] = p, p, (p if h % 2 else q)
        elif kind == "one_ray":   # three depths along one viewing ray of the second camera
            u0, v0 = rng.uniform(100.0, 540.0), rng.uniform(80.0, 320.0)
            ray = np.array([(u0 - cx) / fx, (v0 - cy) / fy, 1.0])
            for k, i in enumerate(idx):
                xc = ray * (2.0 + 1.5 * k)
                X[i] = R.T @ (xc - t)
                uv_override[i] = (u0, v0)
        else:   # near-collinear: 1e-7 m off one line
            y0, z0 = rng.uniform(-1.0, 1.0), rng.uniform(3.0, 7.0)
            for k, i in enumerate(idx):
                X[i] = [-1.0 + 0.8 * k, y0 + 1e-7 * rng.standard_normal(), z0 + 1e-7 * rng.standard_normal()]
    assert all(len(v) == 8 for v in targets.values()), targets
    free = np.nonzero(~used)[0]
    X[free] = np.stack([rng.uniform(-2.0, 2.0, free.size), rng.uniform(-1.5, 1.5, free.size),
                        rng.uniform(2.0, 8.0, free.size)], 1)
    xc = X @ R.T + t
    u = fx * xc[:, 0] / xc[:, 2] + cx
    v = fy * xc[:, 1] / xc[:, 2] + cy
    for i, (a, b) in uv_override.items():
        u[i], v[i] = a, b
    out = rng.random(N_CORR) < 0.2
    out[used] = False
    u[out] += rng.uniform(10.0, 60.0, int(out.sum())) * rng.choice([-1.0, 1.0], int(out.sum()))
    v[out] += rng.uniform(10.0, 60.0, int(out.sum())) * rng.choice([-1.0, 1.0], int(out.sum()))
    corr = {"X": X[:, 0].copy(), "Y": X[:, 1].copy(), "Z": X[:, 2].copy(), "u": u, "v": v, "du": cx - u, "dv": cy - v}
    return corr, targets, tri


@pytest.mark.parametrize("mode", ["exhaustive", "bounded"])
def test_degenerate_p3p_samples_match_the_oracle(mode):
    import torch

    from thor_slam_amd._lib import Handle

    cfg = HipSlamConfig()
    rect = _rect()
    intr = (rect.fx, rect.fy, rect.cx, rect.cy)
    corr, targets, tri = crafted_set(cfg, intr)
    K, H = cfg.n_features, cfg.ransac_hypotheses
    bx, by, bz = O.bearings(corr, intr)
    rows = np.zeros((K, 8))
    rows[:N_CORR] = np.stack([corr["X"], corr["Y"], corr["Z"], corr["du"], corr["dv"], bx, by, bz], 1)
    stats = np.array([3, N_CORR, 0, 0, -1, FRAME, 0, 0], dtype=np.int32)   # 3 = to be solved

    h = Handle([rect], cfg, max_batch=1, ransac_mode=mode)
    img = torch.zeros((1, 2, rect.height, rect.width), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    h.submit(img.data_ptr(), 1, s)   # frame 0
    h.read_poses(1)
    h.begin_batch(img.data_ptr(), 1)   # frame 1: only the injected pose solve runs
    h.copy_in("corr", 0, rows)
    h.copy_in("stats", 0, stats)
    h.run_pose_solve(s)
    torch.cuda.synchronize()
    st = h.frame_block("stats", 0, np.int32)[:8]
    T = h.frame_block("pose", 0, np.float64)[:16].reshape(4, 4)
    hyp = h.frame_block("hyp", 0, np.float64)[:4 * H * 20].reshape(H, 4, 20)
    h.end_batch()
    h.close()

    # every hypothesis: the oracle's P3P on the same draw
    pw = [[corr["X"][tri[:, k]], corr["Y"][tri[:, k]], corr["Z"][tri[:, k]]] for k in range(3)]
    fb = [[bx[tri[:, k]], by[tri[:, k]], bz[tri[:, k]]] for k in range(3)]
    rot, trn, ok = O.p3p(pw, fb)
    dev_ok = ~np.isnan(hyp[:, :, 0])
    np.testing.assert_array_equal(dev_ok, ok)
    np.testing.assert_array_equal(hyp[:, :, :9][ok], rot.reshape(H, 4, 9)[ok])
    np.testing.assert_array_equal(hyp[:, :, 9:12][ok], trn[ok])
    # the degenerate kinds really were degenerate: collinear and coincident samples give no
    # candidate (0/0 in the frame or the quartic); one-ray samples (bearings equal up to rounding)
    # and near-collinear ones are solved, ill-conditioned but finite, by both for some hypotheses
    for kind in ("collinear", "coincident"):
        assert not ok[targets[kind]].any(), (kind, ok[targets[kind]])
    for kind in ("one_ray", "near_collinear"):
        assert ok[targets[kind]].any() and not ok[targets[kind]].all(), (kind, ok[targets[kind]])
    assert ok.sum() > H   # the regular hypotheses still give candidates
    # the RANSAC winner, counts and the refined pose
    o = O.estimate_pose(corr, intr, cfg, FRAME)
    assert (st[4], st[3]) == (o["best_hyp"], o["best_count"]), "RANSAC winner differs"
    assert st[0] == o["status"] == 0 and st[1] == N_CORR and st[2] == o["n_inliers"]
    assert o["best_hyp"] // 4 not in sum(targets.values(), [])
    assert rel_frobenius(T, o["T"]) < 1e-9
