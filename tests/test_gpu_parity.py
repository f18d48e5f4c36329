"""HIP path vs the NumPy oracle on identical synthetic frames (rows A2-A7).

Bar (BASELINE.json north_star): keypoints, descriptors and matches bit-exact; refined
disparities / sub-pixel positions / 3D correspondences bit-exact (same IEEE op sequence);
the RANSAC winner identical; relative and absolute poses within 1e-9 relative Frobenius
(the stated product tolerance is 1e-4; only the Gauss-Newton summation order differs).
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import rel_frobenius, scenario

pytestmark = pytest.mark.gpu

N_FRAMES = 4


@functools.lru_cache(maxsize=8)
def hip_run(seed: int = 0, batch: int = N_FRAMES, distorted: bool = False, n: int = N_FRAMES, cfg_items: tuple = (),
            splits: int = 0, width: int = 640, height: int = 400, mode: str = "auto", refine_block: int = 0):
    import torch

    from thor_slam_amd._lib import Handle

    sc = scenario(seed=seed, n=n, width=width, height=height, distorted=distorted, cfg_items=cfg_items)
    cfg = sc["cfg"]
    h = Handle([sc["rect"]], cfg, max_batch=batch, ransac_splits=splits, ransac_mode=mode, refine_block=refine_block)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    per = []
    K = cfg.n_features
    for b0 in range(0, n, batch):
        nb = min(batch, n - b0)
        h.submit(dev[b0:].data_ptr(), nb, torch.cuda.current_stream().cuda_stream)
        res = h.read_poses(nb)
        for f in range(nb):
            g = b0 + f
            slot = h.ring_slot(g)
            rec = {
                "pyr": h.frame_block("pyramid", slot, np.uint8).reshape(2, h.pyr_bytes),
                "kp": [h.keypoints(g, 0), h.keypoints(g, 1)],
                "stereo": h.frame_block("stereo", slot, np.int32)[:K],
                "disp": h.frame_block("disp", slot, np.float64)[:K],
                "temporal": h.frame_block("temporal", slot, np.int32)[:K],
                "tuv": h.frame_block("temporal_uv", f, np.float64)[: 2 * K].reshape(K, 2),
                "corr": h.frame_block("corr", f, np.float64)[: 8 * K].reshape(K, 8),
                "T_rel": res["T_rel"][f, 0], "T_abs": res["T_abs"][f, 0], "cov": res["cov"][f, 0],
                "stats": res["stats"][f, 0],
            }
            per.append(rec)
    h.close()
    return sc, per


def _levels(h_pyr, off, wh):
    return [h_pyr[o : o + w * hh].reshape(hh, w) for o, (w, hh) in zip(off, wh)]


def _check_image_features(ora_img: dict, got: dict, cfg, where: str):
    counts = np.array(ora_img["counts"])
    np.testing.assert_array_equal(got["counts"], counts, err_msg=f"{where}: per-level counts")
    valid = ora_img["valid"]
    for k in ("x", "y", "score", "level", "angle"):
        np.testing.assert_array_equal(got[k][valid], ora_img["kp"][k][valid], err_msg=f"{where}: keypoint {k}")
    np.testing.assert_array_equal(got["desc"][valid], ora_img["desc"][valid], err_msg=f"{where}: descriptors")


@pytest.mark.parametrize("distorted", [False, True])
def test_rectify_pyramid_bit_exact(distorted):
    from oracle import numpy_slam as O
    from thor_slam_amd.params import level_shapes

    sc, per = hip_run(distorted=distorted)
    cfg = sc["cfg"]
    wh = level_shapes(640, 400, cfg.n_levels)
    off = np.cumsum([0] + [w * h for w, h in wh])[:-1]
    for i, rec in enumerate(per):
        o = sc["oracle"][i]["cur"]
        for cam, side in ((0, "left"), (1, "right")):
            for l, lev in enumerate(_levels(rec["pyr"][cam], off, wh)):
                np.testing.assert_array_equal(lev, o[side]["levels"][l], err_msg=f"frame {i} cam {cam} level {l}")
        # smoothing is checked through the descriptors; spot-check level 0 directly too
        assert O.smooth(o["left"]["levels"][0]).shape == (400, 640)


@pytest.mark.parametrize("distorted", [False, True])
def test_keypoints_descriptors_bit_exact(distorted):
    sc, per = hip_run(distorted=distorted)
    for i, rec in enumerate(per):
        o = sc["oracle"][i]["cur"]
        _check_image_features(o["left"], rec["kp"][0], sc["cfg"], f"frame {i} left")
        _check_image_features(o["right"], rec["kp"][1], sc["cfg"], f"frame {i} right")


def test_matches_and_subpixel_bit_exact():
    sc, per = hip_run()
    for i, rec in enumerate(per):
        o = sc["oracle"][i]["cur"]
        np.testing.assert_array_equal(rec["stereo"], o["stereo"], err_msg=f"frame {i} stereo matches")
        np.testing.assert_array_equal(np.isnan(rec["disp"]), np.isnan(o["disp"]), err_msg=f"frame {i} disparity validity")
        ok = ~np.isnan(o["disp"])
        np.testing.assert_array_equal(rec["disp"][ok], o["disp"][ok], err_msg=f"frame {i} refined disparity")
        np.testing.assert_array_equal(rec["temporal"], o["temporal"], err_msg=f"frame {i} temporal matches")
        if i == 0:
            assert (rec["temporal"] == -1).all()
            continue
        corr = sc["oracle"][i]["corr"]
        np.testing.assert_array_equal(rec["tuv"][corr["j"], 0], corr["u"], err_msg=f"frame {i} refined u")
        np.testing.assert_array_equal(rec["tuv"][corr["j"], 1], corr["v"], err_msg=f"frame {i} refined v")


def test_correspondences_bit_exact():
    sc, per = hip_run()
    for i, rec in enumerate(per[1:], start=1):
        corr = sc["oracle"][i]["corr"]
        n = corr["X"].size
        assert rec["stats"][1] == n, f"frame {i}: n_corr {rec['stats'][1]} vs oracle {n}"
        got = rec["corr"][:n]
        for col, key in enumerate(("X", "Y", "Z", "du", "dv")):
            np.testing.assert_array_equal(got[:, col], corr[key], err_msg=f"frame {i} corr {key}")


def test_pose_parity():
    sc, per = hip_run()
    for i, rec in enumerate(per):
        o = sc["oracle"][i]
        st = rec["stats"]
        if i == 0:
            assert st[0] == 2
            np.testing.assert_array_equal(rec["T_abs"], np.eye(4))
            continue
        assert st[0] == o["status"] == 0, f"frame {i}: status {st[0]} vs {o['status']}"
        assert st[4] == o["best_hyp"] and st[3] == o["best_count"], f"frame {i}: RANSAC winner differs"
        assert st[2] == o["n_inliers"], f"frame {i}: inliers {st[2]} vs {o['n_inliers']}"
        assert rel_frobenius(rec["T_rel"], o["T"]) < 1e-9
        assert rel_frobenius(rec["T_abs"], o["world_T_cam"]) < 1e-9
        assert rel_frobenius(rec["cov"], o["cov"]) < 1e-6


def test_batch_size_invariance():
    _, a = hip_run(batch=N_FRAMES)
    _, b = hip_run(batch=1)
    for i, (x, y) in enumerate(zip(a, b)):
        for k in ("stereo", "temporal"):
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"frame {i} {k}")
        np.testing.assert_array_equal(x["stats"], y["stats"])
        np.testing.assert_array_equal(x["T_abs"], y["T_abs"])


@pytest.mark.parametrize("splits", [1, 3, 32])
def test_ransac_split_invariance(splits):
    """k_ransac_all (this size's automatic choice) at other split counts gives the same results."""
    _, a = hip_run()
    _, b = hip_run(splits=splits)
    for i, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(x["stats"], y["stats"], err_msg=f"frame {i}")
        np.testing.assert_array_equal(x["T_abs"], y["T_abs"], err_msg=f"frame {i}")


@pytest.mark.parametrize("splits", [0, 3])
def test_ransac_bounded_equals_exhaustive(splits):
    """The bounded kernel (k_ransac, forced) gives the same stats, winners and poses as the
    exhaustive one on the pipeline's own correspondences."""
    _, a = hip_run(mode="exhaustive")
    _, b = hip_run(splits=splits, mode="bounded")
    for i, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(x["stats"], y["stats"], err_msg=f"frame {i}")
        np.testing.assert_array_equal(x["T_abs"], y["T_abs"], err_msg=f"frame {i}")


def test_other_seeds_and_config():
    """Different scene seed and a smaller, single-level configuration stay bit-exact."""
    items = (("n_features", 700), ("n_levels", 1), ("ransac_hypotheses", 64))
    sc, per = hip_run(seed=5, n=3, cfg_items=items)
    for i, rec in enumerate(per):
        o = sc["oracle"][i]
        _check_image_features(o["cur"]["left"], rec["kp"][0], sc["cfg"], f"frame {i} left")
        np.testing.assert_array_equal(rec["stereo"], o["cur"]["stereo"])
        np.testing.assert_array_equal(rec["temporal"], o["cur"]["temporal"])
        if i:
            assert rec["stats"][4] == o["best_hyp"] and rec["stats"][2] == o["n_inliers"]
            assert rel_frobenius(rec["T_abs"], o["world_T_cam"]) < 1e-9


@pytest.mark.parametrize("mode", ["auto", "bounded"])
def test_c4_size_bit_exact(mode):
    """Config C4 geometry (1280x800, K=4000: the level-0 quota exceeds the counting-sort capacity,
    so select takes its bitonic path) stays bit-exact, with a distorted lens.  With the bounded
    RANSAC forced, correspondences past its LDS capacity (2048) come from global memory."""
    items = (("n_features", 4000),)
    sc, per = hip_run(seed=2, n=2, cfg_items=items, width=1280, height=800, distorted=True, mode=mode)
    if mode == "bounded":
        assert per[1]["stats"][1] > 2048, "the frame should exceed the LDS staging capacity"
    for i, rec in enumerate(per):
        o = sc["oracle"][i]
        _check_image_features(o["cur"]["left"], rec["kp"][0], sc["cfg"], f"frame {i} left")
        _check_image_features(o["cur"]["right"], rec["kp"][1], sc["cfg"], f"frame {i} right")
        np.testing.assert_array_equal(rec["stereo"], o["cur"]["stereo"])
        np.testing.assert_array_equal(rec["temporal"], o["cur"]["temporal"])
        if i:
            assert rec["stats"][4] == o["best_hyp"] and rec["stats"][2] == o["n_inliers"]
            assert rel_frobenius(rec["T_abs"], o["world_T_cam"]) < 1e-9


def test_two_stream_pipeline_bit_exact():
    """Front stages (rectify .. describe) on one stream, back stages (match .. pose) on another,
    so batch s + 1's front overlaps batch s's back (the library orders them with events; the ring
    keeps 2B + 1 frames): results identical to the oracle."""
    import torch

    from thor_slam_amd._lib import Handle

    n, batch = 8, 2
    sc = scenario(seed=0, n=n)
    cfg = sc["cfg"]
    h = Handle([sc["rect"]], cfg, max_batch=batch)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    fs, bs = torch.cuda.current_stream(), torch.cuda.Stream()
    for b0 in range(0, n, batch):   # no host synchronisation between batches: they overlap
        h.begin_batch(dev[b0:].data_ptr(), batch)
        for st in ("rectify", "detect", "describe"):
            h.run_stage(st, fs.cuda_stream)
        for st in ("match", "pose"):
            h.run_stage(st, bs.cuda_stream)
        h.end_batch()
    res = h.read_poses(batch)
    K = cfg.n_features
    for g in range(n - 2 * batch, n):   # the frames still in the ring (2B + 1)
        o = sc["oracle"][g]
        _check_image_features(o["cur"]["left"], h.keypoints(g, 0), cfg, f"frame {g} left")
        np.testing.assert_array_equal(h.frame_block("temporal", h.ring_slot(g), np.int32)[:K], o["cur"]["temporal"])
        np.testing.assert_array_equal(h.frame_block("stereo", h.ring_slot(g), np.int32)[:K], o["cur"]["stereo"])
    for f in range(batch):
        o = sc["oracle"][n - batch + f]
        assert res["stats"][f, 0, 4] == o["best_hyp"] and res["stats"][f, 0, 2] == o["n_inliers"]
        assert rel_frobenius(res["T_abs"][f, 0], o["world_T_cam"]) < 1e-9
    h.close()


def test_speculative_fast_threshold_exact_across_batches():
    """A4 speculative threshold: from the second batch on, detect scores exactly only
    the pixels that may reach a margin below the previous batch's K-th score per level.  Batches
    of 1 over 6 frames run it for frames 1..5: keypoints and descriptors stay bit-exact."""
    sc, per = hip_run(seed=0, batch=1, n=6)
    for i, (ora, got) in enumerate(zip(sc["oracle"], per)):
        for cam, side in enumerate(("left", "right")):
            _check_image_features(ora["cur"][side], got["kp"][cam], sc["cfg"], f"frame {i} {side}")


def test_speculative_fast_threshold_fallback_is_exact():
    """A low-contrast batch after a textured one: the learnt threshold leaves fewer than K
    candidates, select flags the images, and the flag-gated fallback (detect + select at t + 1)
    restores the exact keypoints."""
    import torch

    from oracle import numpy_slam as O
    from thor_slam_amd._lib import Handle

    sc = scenario(seed=0, n=4)
    cfg, rect = sc["cfg"], sc["rect"]
    frames = np.ascontiguousarray(sc["frames"]).copy()
    frames[2:] = (frames[2:].astype(np.int32) // 3 + 85).astype(np.uint8)   # contrast / 3
    h = Handle([rect], cfg, max_batch=2)
    dev = torch.from_numpy(frames).cuda()
    s = torch.cuda.current_stream().cuda_stream
    h.submit(dev[0].data_ptr(), 2, s)
    h.submit(dev[2].data_ptr(), 2, s)
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    ora = [trk.step(frames[i, 0], frames[i, 1]) for i in range(4)]
    for i in range(2, 4):
        for cam, side in enumerate(("left", "right")):
            _check_image_features(ora[i]["cur"][side], h.keypoints(i, cam), cfg, f"frame {i} {side}")
    # the low-contrast frames really have fewer strong corners than the learnt threshold admits
    assert min(ora[2]["cur"]["left"]["kp"]["score"][ora[2]["cur"]["left"]["valid"]]) < 40
    h.close()


@pytest.mark.slow
def test_c1_sequence_100_frames():
    """Config C1 (BASELINE.json configs[0]): the 100-frame 640x400 sequence end to end, in ragged
    batches of 32 (32, 32, 32, 4), against the oracle run frame by frame.  Every frame's keypoint
    counts, match and correspondence counts, RANSAC winner and inlier count are identical, and the
    chained absolute pose stays within 1e-9 relative Frobenius of the oracle's over the whole
    sequence (association or chaining drift would show up here, not in the 4-frame tests)."""
    n = 100
    sc, per = hip_run(seed=5, batch=32, n=n)
    n_tracked = 0
    for i, rec in enumerate(per):
        o = sc["oracle"][i]
        for cam, side in enumerate(("left", "right")):
            np.testing.assert_array_equal(rec["kp"][cam]["counts"], np.array(o["cur"][side]["counts"]),
                                          err_msg=f"frame {i} {side} counts")
        valid = o["cur"]["left"]["valid"]
        for k in ("x", "y", "angle"):
            np.testing.assert_array_equal(rec["kp"][0][k][valid], o["cur"]["left"]["kp"][k][valid],
                                          err_msg=f"frame {i} left {k}")
        np.testing.assert_array_equal(rec["kp"][0]["desc"][valid], o["cur"]["left"]["desc"][valid],
                                      err_msg=f"frame {i} left descriptors")
        st = rec["stats"]
        if i == 0:
            assert st[0] == 2
            continue
        assert st[0] == o["status"], f"frame {i}: status {st[0]} vs {o['status']}"
        assert st[1] == o["n_corr"], f"frame {i}: n_corr {st[1]} vs {o['n_corr']}"
        if o["status"] == 0:
            n_tracked += 1
            assert st[4] == o["best_hyp"] and st[3] == o["best_count"], f"frame {i}: RANSAC winner differs"
            assert st[2] == o["n_inliers"], f"frame {i}: inliers {st[2]} vs {o['n_inliers']}"
            assert rel_frobenius(rec["T_rel"], o["T"]) < 1e-9, f"frame {i}: T_rel"
        assert rel_frobenius(rec["T_abs"], o["world_T_cam"]) < 1e-9, f"frame {i}: T_abs"
    assert n_tracked >= 90, f"only {n_tracked} of {n - 1} frames tracked"


@pytest.mark.parametrize("splits,mode", [(0, "bounded"), (1, "bounded"), (7, "bounded"), (0, "exhaustive"), (0, "auto")])
def test_ransac_bounded_scoring_with_outliers(splits, mode):
    """k_ransac drops a pose as soon as its count cannot reach the block's best key.  With 35 % of
    the frame's refined positions moved 8-40 px (outliers to every pose), the RANSAC winner, its
    count, the inliers and the refined pose still equal the oracle's exhaustive scoring — with the
    bounded kernel forced, the exhaustive one (k_ransac_all) forced, and the automatic choice."""
    import torch

    from oracle import numpy_slam as O
    from thor_slam_amd._lib import Handle

    sc = scenario(seed=0, n=3)
    cfg, rect = sc["cfg"], sc["rect"]
    K = cfg.n_features
    h = Handle([rect], cfg, max_batch=1, ransac_splits=splits, ransac_mode=mode)
    dev = torch.from_numpy(np.ascontiguousarray(sc["frames"])).cuda()
    s = torch.cuda.current_stream().cuda_stream
    for g in range(2):
        h.submit(dev[g:].data_ptr(), 1, s)
    h.read_poses(1)
    h.begin_batch(dev[2:].data_ptr(), 1)
    for k in ("rectify_pyramid", "detect", "select", "describe", "match", "match_refine"):
        h.run_kernel(k, s)
    torch.cuda.synchronize()
    corr = {k: np.array(v, copy=True) for k, v in sc["oracle"][2]["corr"].items()}
    tuv = h.frame_block("temporal_uv", 0, np.float64)[: 2 * K].reshape(K, 2).copy()
    np.testing.assert_array_equal(tuv[corr["j"], 0], corr["u"])
    rng = np.random.default_rng(11)
    m = rng.random(corr["j"].size) < 0.35
    off = rng.uniform(8.0, 40.0, (int(m.sum()), 2)) * rng.choice([-1.0, 1.0], (int(m.sum()), 2))
    corr["u"][m] += off[:, 0]
    corr["v"][m] += off[:, 1]
    corr["du"], corr["dv"] = rect.cx - corr["u"], rect.cy - corr["v"]
    tuv[corr["j"], 0], tuv[corr["j"], 1] = corr["u"], corr["v"]
    h.copy_in("temporal_uv", 0, tuv)
    h.run_kernel("pose", s)
    torch.cuda.synchronize()
    st = h.frame_block("stats", 0, np.int32)[:5]
    T = h.frame_block("pose", 0, np.float64)[:16].reshape(4, 4)
    h.end_batch()
    h.close()
    o = O.estimate_pose(corr, (rect.fx, rect.fy, rect.cx, rect.cy), cfg, sc["oracle"][2]["frame"])
    assert st[1] == corr["j"].size and 0.5 < o["best_count"] / st[1] < 0.75
    assert (st[4], st[3]) == (o["best_hyp"], o["best_count"]), "RANSAC winner differs"
    assert st[0] == o["status"] == 0 and st[2] == o["n_inliers"]
    assert rel_frobenius(T, o["T"]) < 1e-9


def test_refine_block_128_parity():
    """k_refine<128> (the automatic choice from 1024 problems per launch) forced on a small batch:
    the oracle's pose within 1e-9, and bit-identical to k_refine<256> — both follow the same
    256-virtual-thread summation partition (k_pose.hip, RF_VIRT)."""
    sc, a = hip_run(refine_block=128)
    _, b = hip_run(refine_block=256)
    for i, (x, y) in enumerate(zip(a, b)):
        for k in ("stats", "T_rel", "T_abs", "cov"):
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"frame {i} {k}")
        if i:
            o = sc["oracle"][i]
            assert x["stats"][4] == o["best_hyp"] and x["stats"][2] == o["n_inliers"]
            assert rel_frobenius(x["T_rel"], o["T"]) < 1e-9
            assert rel_frobenius(x["T_abs"], o["world_T_cam"]) < 1e-9


def test_refine_512_frame_launch_invariance():
    """One launch of 512 frames (auto: k_refine<256>, the bounded RANSAC) against the same launch with
    k_refine<128> forced, and against launches of 64 frames: stats, poses and covariances
    bit-identical on every frame; the first frames also equal the oracle."""
    import torch

    from oracle import numpy_slam as O
    from thor_slam_amd._lib import Handle

    n, unique = 512, 16
    k = np.arange(n) % (2 * (unique - 1))
    tri = np.where(k < unique, k, 2 * (unique - 1) - k)   # consecutive frames stay consecutive
    sc = scenario(seed=0, n=4)
    cfg, rect = sc["cfg"], sc["rect"]
    distinct = sc["src"].render_stereo_sequence(unique)
    frames = np.ascontiguousarray(distinct[tri])
    dev = torch.from_numpy(frames).cuda()
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for name, batch, rb in (("auto", n, 0), ("128", n, 128), ("b64", 64, 0)):
        h = Handle([rect], cfg, max_batch=batch, refine_block=rb)
        recs = {k: [] for k in ("stats", "T_rel", "T_abs", "cov")}
        for b0 in range(0, n, batch):
            h.submit(dev[b0:].data_ptr(), batch, s)
            res = h.read_poses(batch)
            for k in recs:
                recs[k].append(np.array(res[k][:, 0], copy=True))
        h.close()
        out[name] = {k: np.concatenate(v) for k, v in recs.items()}
    for other in ("128", "b64"):
        for k in ("stats", "T_rel", "T_abs", "cov"):
            np.testing.assert_array_equal(out["auto"][k], out[other][k], err_msg=f"{other}: {k}")
    assert (out["auto"]["stats"][1:, 0] == 0).mean() > 0.95   # tracked
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    for i in range(4):
        o = trk.step(frames[i, 0], frames[i, 1])
        if i:
            assert out["auto"]["stats"][i, 4] == o["best_hyp"] and out["auto"]["stats"][i, 2] == o["n_inliers"]
            assert rel_frobenius(out["auto"]["T_rel"][i], o["T"]) < 1e-9



def test_blocked_chain_equals_serial_chain_over_300_frames():
    """k_chain's blocked product (T_abs(g) = A(j) Q(g) over global 64-frame blocks, k_pose.hip)
    against the oracle's serial left-to-right chain T_abs(t) = T_abs(t-1) inv(T_rel(t))
    (numpy_slam.py OracleTracker._advance) over 300 frames, so the comparison crosses four block
    boundaries: in batches of 37 (every batch but the first starts mid-block), of 300 (one launch,
    more than four blocks per round) and of 64.  Within 1e-9 relative Frobenius at every frame, and
    bit-identical across the three batchings."""
    import torch

    from thor_slam_amd._lib import Handle

    n, unique = 300, 16
    k = np.arange(n) % (2 * (unique - 1))
    tri = np.where(k < unique, k, 2 * (unique - 1) - k)   # consecutive frames stay consecutive
    sc = scenario(seed=0, n=4)
    cfg, rect = sc["cfg"], sc["rect"]
    frames = np.ascontiguousarray(sc["src"].render_stereo_sequence(unique)[tri])
    dev = torch.from_numpy(frames).cuda()
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for batch in (37, 300, 64):
        h = Handle([rect], cfg, max_batch=batch)
        recs = {k: [] for k in ("stats", "T_rel", "T_abs")}
        for b0 in range(0, n, batch):
            m = min(batch, n - b0)
            h.submit(dev[b0:].data_ptr(), m, s)
            res = h.read_poses(m)
            for key in recs:
                recs[key].append(np.array(res[key][:m, 0], copy=True))
        h.close()
        out[batch] = {key: np.concatenate(v) for key, v in recs.items()}
    for other in (300, 64):
        for key in ("stats", "T_rel", "T_abs"):
            np.testing.assert_array_equal(out[37][key], out[other][key], err_msg=f"batch {other}: {key}")
    st, t_rel, t_abs = out[37]["stats"], out[37]["T_rel"], out[37]["T_abs"]
    assert (st[1:, 0] == 0).mean() > 0.95
    serial = np.eye(4)
    for g in range(n):
        if g and st[g, 0] <= 0:
            t = t_rel[g]
            inv = np.eye(4)
            inv[:3, :3] = t[:3, :3].T
            inv[:3, 3] = -(t[:3, :3].T @ t[:3, 3])
            serial = serial @ inv
        assert rel_frobenius(t_abs[g], serial) < 1e-9, f"frame {g}: blocked chain vs serial chain"
