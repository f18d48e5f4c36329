"""SURVEY.md §8f item 1 — rig pose by generalised PnP over every stereo pair, CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for ``k_rig_pose`` (k_pose.hip),
never imported by the product.  cuVSLAM's multi-camera solve is closed, so this
file is the spec; parity against the reference is unpinned like rows A2-A8.

Spec (per frame; E_p = base_T_rect-left of pair p, E_p^-1 by the rigid-inverse formula below):

* candidates: for every pair whose own A7 pose succeeded, M_p = (E_p T_p) E_p^-1 (4x4 products
  with a fixed association, ``mul4``);
* each candidate is scored on the correspondences of ALL pairs: pair q tests A7's inlier rule
  with T_q = (E_q^-1 M) E_q in its own camera; most inliers wins, ties to the lowest pair;
* Gauss-Newton on the body motion over the inliers of all pairs, re-selected each iteration, with
  A7's left-multiplied Cayley update applied to M: for the body point Y = E_q Xc,
  d(res)/d(rho, omega) = [q, Y x q], q = (d pi / d Xc) R_e^T;
* status / covariance exactly as A7 (>= min_inliers, sigma^2 H^-1 with sigma^2 = SSE / (2n - 6));
* chaining T_abs(t) = T_abs(t-1) inv(T_rel(t)) like A7.
"""

from __future__ import annotations

import numpy as np

from .numpy_slam import cayley, count_inliers_mask, solve6


def mul4(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((4, 4))
    for i in range(4):
        for j in range(4):
            out[i, j] = ((a[i, 0] * b[0, j] + a[i, 1] * b[1, j]) + a[i, 2] * b[2, j]) + a[i, 3] * b[3, j]
    return out


def inv_rigid(e: np.ndarray) -> np.ndarray:
    out = np.zeros((4, 4))
    for i in range(3):
        for j in range(3):
            out[i, j] = e[j, i]
        out[i, 3] = -((e[0, i] * e[0, 3] + e[1, i] * e[1, 3]) + e[2, i] * e[2, 3])
    out[3, 3] = 1.0
    return out


def rig_pose(pairs: list[dict], E: list[np.ndarray], cfg) -> dict:
    """``pairs[q]``: {"status", "T" (4x4), "corr" (dict of X Y Z du dv u v, may be None),
    "intr" (fx, fy, cx, cy)}.  Returns {"T", "cov", "status", "n_corr", "n_inliers", "best"}."""
    P = len(pairs)
    Einv = [inv_rigid(e) for e in E]
    thr2 = float(cfg.ransac_thr_px) * float(cfg.ransac_thr_px)
    n_corr = sum(0 if pq["corr"] is None else pq["corr"]["X"].size for pq in pairs)
    out = {"T": np.eye(4), "cov": np.zeros((6, 6)), "status": 1, "n_corr": n_corr, "n_inliers": 0, "best": -1}
    cands = [mul4(mul4(E[p], pairs[p]["T"]), Einv[p]) for p in range(P) if pairs[p]["status"] == 0]
    if not cands:
        return out

    def per_pair(M):
        return [mul4(mul4(Einv[q], M), E[q]) for q in range(P)]

    def count(M):
        n = 0
        for q, T in enumerate(per_pair(M)):
            if pairs[q]["corr"] is not None:
                n += int(count_inliers_mask(T[:3, :3], T[:3, 3], pairs[q]["corr"], pairs[q]["intr"], thr2).sum())
        return n

    counts = [count(M) for M in cands]
    best = int(np.argmax(counts))   # first maximum = lowest pair
    out["best"] = best
    M = cands[best].copy()
    hm = None
    sq = 0.0
    fail = False
    for _ in range(cfg.refine_iters):
        jx_all, jy_all, rx_all, ry_all = [], [], [], []
        for q, T in enumerate(per_pair(M)):
            cr = pairs[q]["corr"]
            if cr is None:
                continue
            fx, fy, cx, cy = pairs[q]["intr"]
            rot, trn = T[:3, :3], T[:3, 3]
            m = count_inliers_mask(rot, trn, cr, pairs[q]["intr"], thr2)
            X, Y, Z = cr["X"][m], cr["Y"][m], cr["Z"][m]
            u, v = cx - cr["du"][m], cy - cr["dv"][m]
            xc = (rot[0, 0] * X + rot[0, 1] * Y) + rot[0, 2] * Z + trn[0]
            yc = (rot[1, 0] * X + rot[1, 1] * Y) + rot[1, 2] * Z + trn[1]
            zc = (rot[2, 0] * X + rot[2, 1] * Y) + rot[2, 2] * Z + trn[2]
            iz = 1.0 / zc
            rx_all.append((fx * xc) * iz + cx - u)
            ry_all.append((fy * yc) * iz + cy - v)
            a, b = fx * iz, fy * iz
            c = -(fx * xc) * (iz * iz)
            d = -(fy * yc) * (iz * iz)
            e = E[q]
            y0 = (e[0, 0] * xc + e[0, 1] * yc) + e[0, 2] * zc + e[0, 3]
            y1 = (e[1, 0] * xc + e[1, 1] * yc) + e[1, 2] * zc + e[1, 3]
            y2 = (e[2, 0] * xc + e[2, 1] * yc) + e[2, 2] * zc + e[2, 3]
            qx = [a * e[0, 0] + c * e[0, 2], a * e[1, 0] + c * e[1, 2], a * e[2, 0] + c * e[2, 2]]
            qy = [b * e[0, 1] + d * e[0, 2], b * e[1, 1] + d * e[1, 2], b * e[2, 1] + d * e[2, 2]]
            jx_all.append(np.stack(qx + [y1 * qx[2] - y2 * qx[1], y2 * qx[0] - y0 * qx[2], y0 * qx[1] - y1 * qx[0]]))
            jy_all.append(np.stack(qy + [y1 * qy[2] - y2 * qy[1], y2 * qy[0] - y0 * qy[2], y0 * qy[1] - y1 * qy[0]]))
        jx = np.concatenate(jx_all, axis=1)
        jy = np.concatenate(jy_all, axis=1)
        rx = np.concatenate(rx_all)
        ry = np.concatenate(ry_all)
        if rx.size < 6:
            fail = True
            break
        hm = jx @ jx.T + jy @ jy.T
        g = -(jx @ rx + jy @ ry)
        sol = solve6(hm, g)
        if sol is None:
            fail = True
            break
        dx = sol[0]
        ru = cayley(dx[3:])
        rot, trn = M[:3, :3].copy(), M[:3, 3].copy()
        M[:3, :3] = np.array([[(ru[i, 0] * rot[0, j] + ru[i, 1] * rot[1, j]) + ru[i, 2] * rot[2, j] for j in range(3)]
                              for i in range(3)])
        M[:3, 3] = np.array([((ru[i, 0] * trn[0] + ru[i, 1] * trn[1]) + ru[i, 2] * trn[2]) + dx[i] for i in range(3)])
        sq = float(rx @ rx + ry @ ry)
    if fail:
        return out
    n_in = count(M)
    out["n_inliers"] = n_in
    if n_in < cfg.min_inliers:
        return out
    out["status"] = 0
    out["T"] = M
    out["cov"] = np.linalg.inv(hm) * (sq / max(1, 2 * n_in - 6))
    return out


class RigChain:
    """world_T_base of the rig: T_abs(t) = T_abs(t-1) inv(T_rel(t)) for successful frames."""

    def __init__(self):
        self.world_T_base = np.eye(4)

    def step(self, res: dict) -> np.ndarray:
        if res["status"] == 0:
            self.world_T_base = self.world_T_base @ inv_rigid(res["T"])
        return self.world_T_base.copy()


def fuse_information(items: list[tuple], E: list[np.ndarray]) -> dict:
    """Rig fusion across ranks (the multi-GPU layout): ``items[q]`` =
    (status, T_rel 4x4, cov 6x6) of pair q.  Each tracked pair's body motion M_q = (E_q T_q) E_q^-1
    with information inv(R6 cov R6^T), R6 = blockdiag(R_e, R_e); combined in the tangent space of
    the first tracked pair: xi = (sum L)^-1 sum L xi_q, xi_q = (t, rotvec) of M_ref^-1 M_q,
    M = M_ref [exp(xi_w) | xi_rho]; covariance (sum L)^-1."""
    from scipy.spatial.transform import Rotation

    sum_l = np.zeros((6, 6))
    sum_lx = np.zeros(6)
    mref = None
    used = 0
    init = any(st == 2 for st, _, _ in items)
    for (st, T, cov), e in zip(items, E):
        if st != 0:
            continue
        M = mul4(mul4(e, T), inv_rigid(e))
        r6 = np.zeros((6, 6))
        r6[:3, :3] = r6[3:, 3:] = e[:3, :3]
        cb = r6 @ cov @ r6.T
        try:
            np.linalg.cholesky(cb)
        except np.linalg.LinAlgError:
            continue
        lam = np.linalg.inv(cb)
        if mref is None:
            mref = M
        d = mul4(inv_rigid(mref), M)
        xi = np.concatenate([d[:3, 3], Rotation.from_matrix(d[:3, :3]).as_rotvec()])
        sum_l += lam
        sum_lx += lam @ xi
        used += 1
    if not used:
        return {"status": 2 if init else 1, "T": np.eye(4), "cov": np.zeros((6, 6)), "used": 0}
    xi = np.linalg.solve(sum_l, sum_lx)
    x = np.eye(4)
    x[:3, :3] = Rotation.from_rotvec(xi[3:]).as_matrix()
    x[:3, 3] = xi[:3]
    return {"status": 0, "T": mul4(mref, x), "cov": np.linalg.inv(sum_l), "used": used}
