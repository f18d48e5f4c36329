"""SURVEY.md §8f item 3 — relocalisation in a saved map, CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for ``k_reloc.hip``.  The map is a
set of landmarks (world xyz + rBRIEF-256).  Spec:

* every valid keypoint of the frame's left image is matched against ALL map descriptors:
  best = lexicographic min of (Hamming distance, map index), second = min distance over the other
  map points; accepted iff best <= max_hamming and (no second or 100 * best < ratio_pct * second);
* the matches, in keypoint order, are 3D-2D correspondences (map point, level-0 keypoint
  position) and A7's ``estimate_pose`` (RNG seeded by the frame index) gives cam_T_world;
* a rig (``relocalize_rig``, SURVEY.md §8f items 1 + 3): the map lives in the rig's base frame;
  pair p matches its left image the same way and sees the map points in its frame E_p^-1 X (E_p =
  base_T_rect-left), A7 solves each pair, and ``numpy_rig.rig_pose`` (candidates E_p T_p E_p^-1,
  scored on every pair, joint Gauss-Newton) gives body_T_world.
"""

from __future__ import annotations

import numpy as np

from .numpy_rig import inv_rigid, rig_pose
from .numpy_slam import estimate_pose, level0_coords

_POP8 = np.array([bin(i).count("1") for i in range(256)], dtype=np.int64)


def hamming(q: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Distances between descriptor rows q [nq][8] u32 and m [nm][8] u32 -> [nq][nm]."""
    x = (q[:, None, :] ^ m[None, :, :]).view(np.uint8)
    return _POP8[x].sum(-1)


def match_map(feat: dict, map_desc: np.ndarray, cfg, chunk: int = 256) -> np.ndarray:
    K = feat["desc"].shape[0]
    out = np.full(K, -1, dtype=np.int64)
    qs = np.nonzero(feat["valid"])[0]
    M = map_desc.shape[0]
    if M == 0:
        return out
    for a in range(0, qs.size, chunk):
        q = qs[a:a + chunk]
        d = hamming(feat["desc"][q].astype(np.uint32), map_desc.astype(np.uint32))
        best = np.argmin(d, axis=1)                   # first minimum = lowest index
        bd = d[np.arange(q.size), best]
        if M > 1:
            d2 = d.copy()
            d2[np.arange(q.size), best] = 1 << 30
            sd = d2.min(axis=1)
            ok = (bd <= cfg.max_hamming) & (100 * bd < cfg.ratio_pct * sd)
        else:
            ok = bd <= cfg.max_hamming
        out[q[ok]] = best[ok]
    return out


def relocalize(feat: dict, map_xyz: np.ndarray, map_desc: np.ndarray, intr, cfg, frame: int) -> dict:
    fx, fy, cx, cy = intr
    m = match_map(feat, map_desc, cfg)
    j = np.nonzero(m >= 0)[0]
    kp = feat["kp"]
    u, v = level0_coords(kp["x"][j], kp["y"][j], kp["level"][j])
    xyz = map_xyz[m[j]]
    corr = {"X": xyz[:, 0], "Y": xyz[:, 1], "Z": xyz[:, 2], "du": cx - u, "dv": cy - v, "u": u, "v": v,
            "j": j, "i": m[j]}
    res = estimate_pose(corr, intr, cfg, frame)
    res["matches"] = m
    res["corr"] = corr
    return res


def relocalize_rig(feats: list[dict], map_xyz: np.ndarray, map_desc: np.ndarray, intrs: list, E: list[np.ndarray], cfg,
                   frame: int) -> dict:
    """``feats[p]``: pair p's left-image features of the frame; ``map_xyz`` in the base frame."""
    pairs = []
    for p, (feat, intr) in enumerate(zip(feats, intrs)):
        ei = inv_rigid(np.asarray(E[p], dtype=np.float64))
        x, y, z = map_xyz[:, 0], map_xyz[:, 1], map_xyz[:, 2]
        local = np.stack([((ei[r, 0] * x + ei[r, 1] * y) + ei[r, 2] * z) + ei[r, 3] for r in range(3)], axis=1)
        res = relocalize(feat, local, map_desc, intr, cfg, frame)
        corr = res.get("corr")
        pairs.append({"status": res["status"], "T": res["T"], "corr": corr, "intr": intr, "res": res})
    out = rig_pose([{k: v for k, v in q.items() if k != "res"} for q in pairs], E, cfg)
    out["pairs"] = [q["res"] for q in pairs]
    return out
