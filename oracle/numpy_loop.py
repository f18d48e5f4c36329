"""SURVEY.md §8f items 1 + 3 — keyframe pose graph and loop closure, CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``): the checker for ``k_loop.hip`` and
``k_posegraph.hip``, never imported by the product.  The reference exposes loop closure only as a
flag (``SlamConfig.enable_loop_closure``, ``thor_slam/slam/interface.py:155-156``) forwarded to
the closed cuVSLAM node, so this file is the spec and parity against the reference is unpinned
like rows A2-A8.

Keyframe database (one entry per keyframe, pair 0's rectified left camera):

* landmarks = the valid keypoints of the left image that have a stereo disparity d > 0 (finite),
  in keypoint order; camera-frame position z = fx*B / d, x = (u - cx) z / fx, y = (v - cy) z / fy
  with (u, v) the level-0 keypoint position (the A8 insertion formula);
* signature = the first ``S`` landmarks (keypoints are ordered by level, then by descending FAST
  score, so these are the strongest level-0 corners with depth).

Place recognition (``vote``): each signature descriptor of the query keyframe is matched against
a candidate's signature by brute-force Hamming: best = lexicographic min of (distance, index),
second = min distance over the others; a vote iff best <= max_hamming and (single entry or
100 * best < ratio_pct * second).  The candidate's score is its vote count.

Geometric verification (``verify``): the query frame's keypoints against the candidate's
landmarks with the relocalisation matcher and A7's P3P-RANSAC + Gauss-Newton
(``numpy_map.relocalize``), giving cam_q_T_cam_c.

Pose graph (``optimize``): nodes T_i = world_T_cam_i, edges (i, j, Z_ij, Omega_ij) with
Z_ij the measured T_i^-1 T_j.  se(3) vectors are xi = (rho, phi) (translation first);
Exp(xi) = [Exp_SO3(phi), V(phi) rho].  Residual e_ij = Log(Z_ij^-1 T_i^-1 T_j); right
perturbations T <- T Exp(delta) give

    J_j = Jr^-1(e),    J_i = -Jr^-1(e) Ad(T_j^-1 T_i),    Jr^-1(e) ~ I + ad(e) / 2,

Ad(R, t) = [[R, t^ R], [0, R]], ad(rho, phi) = [[phi^, rho^], [0, phi^]].  Each Gauss-Newton
iteration assembles H = sum J^T Omega J and g = sum J^T Omega e over the free nodes (node 0 is
the gauge and stays fixed), solves H delta = -g by Cholesky and applies T_i <- T_i Exp(delta_i).
The cost is sum e^T Omega e at the returned poses.
"""

from __future__ import annotations

import numpy as np

from .numpy_map import hamming, relocalize
from .numpy_slam import level0_coords

# --------------------------------------------------------------------------------------------
# keyframe database
# --------------------------------------------------------------------------------------------


def keyframe_landmarks(left: dict, disp: np.ndarray, intr) -> dict:
    """Compacted stereo landmarks of one keyframe: xyz [n][3] (camera frame), desc [n][8] u32,
    kp [n] (keypoint index)."""
    fx, fy, cx, cy, fxb = intr
    kp = left["kp"]
    K = left["desc"].shape[0]
    d = np.asarray(disp[:K], dtype=np.float64)
    ok = np.asarray(left["valid"][:K], dtype=bool) & np.isfinite(d)
    ok &= np.where(np.isfinite(d), d, 0.0) > 0.0
    ks = np.nonzero(ok)[0]
    u, v = level0_coords(kp["x"][ks], kp["y"][ks], kp["level"][ks])
    z = fxb / d[ks]
    xyz = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], axis=1) if ks.size else np.zeros((0, 3))
    return {"xyz": xyz, "desc": np.asarray(left["desc"][ks], dtype=np.uint32), "kp": ks}


def vote(q_desc: np.ndarray, c_desc: np.ndarray, S: int, max_hamming: int, ratio_pct: int) -> int:
    """Votes of the query signature (first S of q_desc) against a candidate signature."""
    q = np.asarray(q_desc[:S], dtype=np.uint32)
    c = np.asarray(c_desc[:S], dtype=np.uint32)
    if q.shape[0] == 0 or c.shape[0] == 0:
        return 0
    d = hamming(q, c)
    best = np.argmin(d, axis=1)
    bd = d[np.arange(q.shape[0]), best]
    if c.shape[0] > 1:
        d2 = d.copy()
        d2[np.arange(q.shape[0]), best] = 1 << 30
        sd = d2.min(axis=1)
        ok = (bd <= max_hamming) & (100 * bd < ratio_pct * sd)
    else:
        ok = bd <= max_hamming
    return int(ok.sum())


def verify(feat_q: dict, cand: dict, intr4, cfg, frame: int) -> dict:
    """cam_q_T_cam_c of keyframe q against candidate c's landmarks (relocalisation matcher)."""
    return relocalize(feat_q, cand["xyz"], cand["desc"], intr4, cfg, frame)


# --------------------------------------------------------------------------------------------
# SE(3) helpers (the formulas k_posegraph.hip follows)
# --------------------------------------------------------------------------------------------


def hat(w: np.ndarray) -> np.ndarray:
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def _abc(th2: float):
    """A = sin t / t, B = (1 - cos t) / t^2 = 2 sin^2(t/2) / t^2, C = (t - sin t) / t^3
    (four Taylor terms below t^2 = 1e-3, where C's direct form cancels)."""
    if th2 < 1e-3:
        t4, t6 = th2 * th2, th2 * th2 * th2
        return (1.0 - th2 / 6.0 + t4 / 120.0 - t6 / 5040.0, 0.5 - th2 / 24.0 + t4 / 720.0 - t6 / 40320.0,
                1.0 / 6.0 - th2 / 120.0 + t4 / 5040.0 - t6 / 362880.0)
    th = np.sqrt(th2)
    s, h = np.sin(th), np.sin(0.5 * th)
    return s / th, 2.0 * h * h / th2, (th - s) / (th2 * th)


def se3_exp(xi: np.ndarray) -> np.ndarray:
    rho, phi = xi[:3], xi[3:]
    th2 = float(phi @ phi)
    A, B, C = _abc(th2)
    W = hat(phi)
    W2 = W @ W
    T = np.eye(4)
    T[:3, :3] = np.eye(3) + A * W + B * W2
    T[:3, 3] = (np.eye(3) + B * W + C * W2) @ rho
    return T


def so3_log(R: np.ndarray) -> np.ndarray:
    """phi with |phi| < pi: theta = atan2(|v| / 2, (tr R - 1) / 2), v = vee(R - R^T) = 2 sin(theta) axis."""
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = 0.5 * np.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    c = (R[0, 0] + R[1, 1] + R[2, 2] - 1.0) * 0.5
    th = np.arctan2(s, c)
    if th < 1e-5:
        return v * (0.5 * (1.0 + th * th / 6.0))
    return v * (th / (2.0 * s))


def se3_log(T: np.ndarray) -> np.ndarray:
    phi = so3_log(T[:3, :3])
    th2 = float(phi @ phi)
    W = hat(phi)
    if th2 < 1e-3:   # k = (1 - A / 2B) / t^2
        k = 1.0 / 12.0 + th2 / 720.0 + th2 * th2 / 30240.0 + th2 * th2 * th2 / 1209600.0
    else:
        A, B, _ = _abc(th2)
        k = (1.0 - A / (2.0 * B)) / th2
    Vinv = np.eye(3) - 0.5 * W + k * (W @ W)
    return np.concatenate([Vinv @ T[:3, 3], phi])


def inv_se3(T: np.ndarray) -> np.ndarray:
    out = np.eye(4)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -(T[:3, :3].T @ T[:3, 3])
    return out


def adjoint(T: np.ndarray) -> np.ndarray:
    R, t = T[:3, :3], T[:3, 3]
    out = np.zeros((6, 6))
    out[:3, :3] = R
    out[:3, 3:] = hat(t) @ R
    out[3:, 3:] = R
    return out


def jr_inv(e: np.ndarray) -> np.ndarray:
    ad = np.zeros((6, 6))
    ad[:3, :3] = hat(e[3:])
    ad[:3, 3:] = hat(e[:3])
    ad[3:, 3:] = hat(e[3:])
    return np.eye(6) + 0.5 * ad


def edge_terms(Ti: np.ndarray, Tj: np.ndarray, Z: np.ndarray):
    """(e, J_i, J_j) of one edge."""
    Tij = inv_se3(Ti) @ Tj
    e = se3_log(inv_se3(Z) @ Tij)
    Jr = jr_inv(e)
    return e, -Jr @ adjoint(inv_se3(Tij)), Jr


def graph_cost(T: np.ndarray, edges: np.ndarray, Z: np.ndarray, info: np.ndarray) -> float:
    cost = 0.0
    for k, (i, j) in enumerate(edges):
        e, _, _ = edge_terms(T[i], T[j], Z[k])
        cost += float(e @ info[k] @ e)
    return cost


def optimize(T0: np.ndarray, edges: np.ndarray, Z: np.ndarray, info: np.ndarray, iters: int) -> dict:
    """Gauss-Newton on the pose graph (node 0 fixed); returns poses, cost, per-iteration |delta|."""
    T = np.array(T0, dtype=np.float64, copy=True)
    N = T.shape[0]
    n = 6 * (N - 1)
    steps = []
    for _ in range(iters):
        if n == 0:
            break
        H = np.zeros((n, n))
        g = np.zeros(n)
        for k, (i, j) in enumerate(edges):
            e, Ji, Jj = edge_terms(T[i], T[j], Z[k])
            W = info[k]
            for (a, Ja) in ((i, Ji), (j, Jj)):
                if a == 0:
                    continue
                ra = 6 * (a - 1)
                g[ra:ra + 6] += Ja.T @ W @ e
                for (b, Jb) in ((i, Ji), (j, Jj)):
                    if b == 0:
                        continue
                    rb = 6 * (b - 1)
                    H[ra:ra + 6, rb:rb + 6] += Ja.T @ W @ Jb
        L = np.linalg.cholesky(H)
        y = np.linalg.solve(L, -g)
        delta = np.linalg.solve(L.T, y)
        for a in range(1, N):
            T[a] = T[a] @ se3_exp(delta[6 * (a - 1):6 * a])
        steps.append(float(np.abs(delta).max()))
    return {"T": T, "cost": graph_cost(T, edges, Z, info), "steps": steps}


# --------------------------------------------------------------------------------------------
# the engine's loop-closure policy, restated (HipSlamEngine loop closure follows it)
# --------------------------------------------------------------------------------------------


def loop_information(sigma_t: float, sigma_r: float) -> np.ndarray:
    return np.diag([1.0 / sigma_t ** 2] * 3 + [1.0 / sigma_r ** 2] * 3)


def best_candidate(votes: np.ndarray, n_allowed: int, min_votes: int) -> int:
    """Highest vote among slots [0, n_allowed), ties to the oldest; -1 below min_votes."""
    if n_allowed <= 0:
        return -1
    v = np.asarray(votes[:n_allowed])
    j = int(np.argmax(v))
    return j if v[j] >= min_votes else -1


# --------------------------------------------------------------------------------------------
# the asynchronous loop-closure policy (HipSlamEngine with tslam_loop_auto follows it frame by
# frame)
# --------------------------------------------------------------------------------------------


def candidate_window(idx: int, cap_k: int, min_gap: int, latency: int, batch: int, interval: int) -> tuple[int, int]:
    """Database positions (= node indices: the i-th tracked keyframe takes position i) [lo, hi]
    the search of node ``idx`` votes against: at least ``min_gap`` nodes older, and still in the
    ring of cap_k positions while the search runs — which may be until frame g + latency, with up
    to two batches submitted past it whose tracked keyframes overwrite the oldest positions:
    margin M = (latency + 2 * batch - 1) // interval + 1."""
    margin = (latency + 2 * batch - 1) // interval + 1
    return max(0, idx - cap_k + margin), idx - min_gap


def best_vote(votes: list, n_pairs: int) -> tuple[int, int, int]:
    """(best votes, query pair q, candidate index j) over every query pair's votes [n * P]
    (candidate j = position lo + j // P, pair j % P): the most votes; ties go to the lower query
    pair, then the NEWEST position (the smallest loop span), then the lower pair."""
    best, q, j = -1, 0, 0
    for qq, v in enumerate(votes):
        v = np.asarray(v).reshape(-1, n_pairs)
        n = v.shape[0]
        r = int(np.argmax(v[::-1].reshape(-1)))   # newest position first, lower pair first within it
        jj = (n - 1 - r // n_pairs) * n_pairs + r % n_pairs
        if int(v.reshape(-1)[jj]) > best:
            best, q, j = int(v.reshape(-1)[jj]), qq, jj
    return best, q, j


def span_edges(edges: list, a: int, b: int) -> list[int]:
    """Indices of the edges (x, y), x < y, with both ends in the span [a, b], in the canonical
    order (y, x) — the solve's summation order does not depend on when a loop edge was recorded."""
    return sorted((e for e, (x, y) in enumerate(edges) if a <= x and y <= b), key=lambda e: (edges[e][1], edges[e][0]))


class SpanSolveFailed(Exception):
    """Raised by a LoopPolicy ``solve`` callable for a span solve that failed (the device's
    TSLAM_ESINGULAR); ``optimize``'s own failure is ``np.linalg.LinAlgError``."""


class LoopPolicy:
    """Keyframe pose graph + loop closure with a fixed latency.

    Frames are published in order; for frame g (status, raw = pair 0's rectified-left world_T_cam
    before loop correction):

    1. a tracked (status 0) frame with g % interval == 0 is a keyframe: node idx (T = T_prev @ Z
       with Z = raw_prev^-1 raw and the odometry edge (idx - 1, idx), or corr @ raw for the first),
       database position idx (entry (idx mod cap_k) * P + p per pair), and a search item due at
       frame g + latency;
    2. every item due at or before g completes, oldest first:
       * votes of pair q's entry of node idx against every pair's entry of the positions of
         ``candidate_window``; ``best_vote`` picks; below ``loop_min_votes`` nothing follows;
       * verification of the best candidate (node c, pair pc) on pair q's view (RANSAC seeded by
         g); a loop needs status 0 and ``loop_min_inliers``, and is not closed when the last
         closed loop's newer node is within ``loop_cooldown`` nodes of idx;
       * the loop edge (c, idx) with Z = M_pc T_qc^-1 M_q^-1 (M_p = rect0_T_rect_p), and the span
         solve: Gauss-Newton (``pg_iters``) on the nodes [c, idx] with node c fixed and the edges
         with both ends in the span (``span_edges``); the span takes the solution, later nodes
         are re-chained by their odometry (T_i = T_{i-1} Z_i), and corr = T_last raw_last^-1;
       * rejection: a span solve whose normal matrix is not positive definite (Cholesky fails: a
         pivot <= 0 or NaN — ``optimize`` raises ``LinAlgError``, the device returns
         TSLAM_ESINGULAR) or that returns a non-finite pose drops the loop: no edge, no
         correction, ``last_loop`` unchanged (the cooldown counts closed loops only), and
         (frame of c, g) goes to ``rejected``.  The session goes on: the reference's contract is
         a pose or None from ``process_frames`` (``interface.py:192-200``), and
         ``run_slam.py:314-321`` has no handler for an exception;
    3. the frame's corrected pose is corr @ raw.

    Relocalisation after a LOST run (``reloc_after_lost`` > 0; the reference's
    ``TrackingState.RELOCALIZING``, ``interface.py:16-23``, and cuVSLAM's
    ``enable_localization_n_mapping``, ``launch/thor_visual_slam.launch.py:42,74``): the device
    keeps chaining through LOST frames without their motion, so the poses after a long gap are
    off by whatever happened in it.

    * the ``reloc_after_lost``-th consecutive LOST frame (with at least one node) breaks the graph:
      state RELOCALIZING, ``anchor_end`` = the node count at the first break of the episode,
      ``seg_start`` = the next node (a later long LOST run inside the episode moves it again);
    * the first node of a segment gets no odometry edge (T = corr @ raw, provisional); nodes
      created while RELOCALIZING get a relocalisation item instead of a loop item, due at
      g + ``reloc_latency`` (items stay in order: an item is never due before the one before it);
    * a relocalisation item of node idx (skipped unless still RELOCALIZING and idx >= seg_start)
      votes against the positions [max(0, idx - cap_k + M), anchor_end - 1] (M of
      ``candidate_window``: still in the ring) with ``best_vote``, needs ``loop_min_votes`` and a
      verification with status 0 and ``loop_min_inliers``; then Z = M_pc T_qc^-1 M_q^-1, the
      segment's nodes move rigidly by D = T_c Z T_idx^-1 (T_i <- D T_i for i >= seg_start), the
      edge (c, idx) joins the graph, corr <- D corr, ``last_loop`` = idx, and tracking resumes
      (``relocs`` gets (frame of c, g, inliers));
    * span solves re-chain later nodes by odometry only up to a segment break; ``state`` is
      "relocalizing" for every frame of the episode (the engine publishes None), "lost" for other
      LOST frames, "tracking" otherwise.

    A session of any length keeps the newest cap_k keyframes searchable, and the span solve bounds
    a loop's cost by the ring (<= cap_k nodes).  ``vote(idx, q, lo, n)`` -> votes [n * P],
    ``verify(idx, g, q, c, pc)`` -> {"T", "stats"}, ``solve(T, edges, meas, info, iters)`` ->
    {"T", "cost"} are the device's operations (``vote`` / ``verify`` / ``optimize`` above restate
    them)."""

    def __init__(self, cfg, n_pairs: int, rect0_T_rect: list, vote, verify, solve):
        self.cfg, self.P = cfg, int(n_pairs)
        self.m = [np.asarray(x, dtype=np.float64) for x in rect0_T_rect]
        self.vote, self.verify, self.solve = vote, verify, solve
        self.cap_k = int(cfg.loop_max_keyframes)
        self.info = loop_information(cfg.pg_sigma_t, cfg.pg_sigma_r)
        self.frames, self.raw, self.T, self.odo = [], [], [], []
        self.edges, self.meas = [], []
        self.loops, self.loop_pairs = [], []
        self.rejected = []   # (frame of c, g) of loops whose span solve failed
        self.items = []   # [idx, g, due, kind] (kind "loop" or "reloc")
        self.corr = np.eye(4)
        self.cost = 0.0
        self.last_loop = None   # node of the last closed loop
        # relocalisation after a LOST run
        self.reloc_after = int(getattr(cfg, "reloc_after_lost", 0))
        self.reloc_latency = int(getattr(cfg, "reloc_latency", 0))
        self.lost_run = 0
        self.reloc = False        # RELOCALIZING
        self.anchor_end = 0       # candidates of the episode: nodes < anchor_end
        self.seg_start = 0        # first node of the unanchored segment
        self.relocs = []          # (frame of c, g, inliers)
        self.last_due = -1
        self.state = "tracking"

    def observe(self, g: int, status: int) -> None:
        """The LOST-run bookkeeping of frame g (first part of ``step``)."""
        if status == 1:
            self.lost_run += 1
            if self.reloc_after > 0 and self.lost_run == self.reloc_after and self.frames:
                if not self.reloc:
                    self.reloc = True
                    self.anchor_end = len(self.frames)
                self.seg_start = len(self.frames)
        else:
            self.lost_run = 0

    def step(self, g: int, status: int, raw: np.ndarray) -> np.ndarray:
        """Frame g -> its corrected pose (rect-left world_T_cam); ``state`` says how to publish it."""
        self.observe(g, status)
        if status == 0 and g % self.cfg.loop_kf_interval == 0:
            self._node(g, raw)
        while self.items and self.items[0][2] <= g:
            self._complete(*self.items.pop(0))
        self.state = "relocalizing" if self.reloc else "lost" if status == 1 else "tracking"
        return self.corr @ raw

    def finish(self) -> None:
        """Complete every pending item now (HipSlamEngine.settle)."""
        while self.items:
            self._complete(*self.items.pop(0))

    def _node(self, g: int, raw: np.ndarray) -> None:
        idx = len(self.frames)
        if idx == 0 or (self.reloc and idx == self.seg_start):   # the first node of a segment
            T, Z = self.corr @ raw, None
        else:
            Z = inv_se3(self.raw[-1]) @ raw
            T = self.T[-1] @ Z
            self.edges.append((idx - 1, idx))
            self.meas.append(Z)
        self.frames.append(g)
        self.raw.append(np.array(raw, dtype=np.float64, copy=True))
        self.T.append(T)
        self.odo.append(Z)
        kind = "reloc" if self.reloc else "loop"
        due = max(g + (self.reloc_latency if self.reloc else int(self.cfg.loop_latency)), self.last_due)
        self.last_due = due
        self.items.append([idx, g, due, kind])

    def _complete(self, idx: int, g: int, due: int = 0, kind: str = "loop") -> None:
        if kind == "reloc":
            self._relocate(idx, g)
            return
        cfg, P = self.cfg, self.P
        lo, hi = candidate_window(idx, self.cap_k, cfg.loop_min_gap, cfg.loop_latency, cfg.batch_size,
                                  cfg.loop_kf_interval)
        if hi < lo:
            return
        best, q, j = best_vote([self.vote(idx, qq, lo, hi - lo + 1) for qq in range(P)], P)
        if best < cfg.loop_min_votes:
            return
        c, pc = lo + j // P, j % P
        ver = self.verify(idx, g, q, c, pc)
        if int(ver["stats"][0]) != 0 or int(ver["stats"][2]) < cfg.loop_min_inliers:
            return
        if self.last_loop is not None and idx - self.last_loop <= int(getattr(cfg, "loop_cooldown", 0)):
            return
        edges = self.edges + [(c, idx)]
        meas = self.meas + [self.m[pc] @ inv_se3(ver["T"]) @ inv_se3(self.m[q])]
        sel = span_edges(edges, c, idx)
        try:
            sol = self.solve(np.stack(self.T[c:idx + 1]), np.array([edges[e] for e in sel]) - c,
                             np.stack([meas[e] for e in sel]), np.stack([self.info] * len(sel)), cfg.pg_iters)
            ok = bool(np.all(np.isfinite(sol["T"])))
        except (np.linalg.LinAlgError, SpanSolveFailed):
            ok = False
        if not ok:
            self.rejected.append((self.frames[c], g))
            return
        self.last_loop = idx
        self.edges, self.meas = edges, meas
        self.loops.append((self.frames[c], g, int(ver["stats"][2])))
        self.loop_pairs.append((pc, q))
        self.T[c:idx + 1] = list(sol["T"])
        for i in range(idx + 1, len(self.T)):
            if self.odo[i] is None:   # a segment break: the nodes after it are anchored otherwise
                break
            self.T[i] = self.T[i - 1] @ self.odo[i]
        self.corr = self.T[-1] @ inv_se3(self.raw[-1])
        self.cost = float(sol["cost"])

    def reloc_window(self, idx: int) -> tuple[int, int]:
        """Database positions [lo, hi] a relocalisation item of node idx votes against."""
        cfg = self.cfg
        margin = (cfg.loop_latency + 2 * cfg.batch_size - 1) // cfg.loop_kf_interval + 1
        return max(0, idx - self.cap_k + margin), self.anchor_end - 1

    def _relocate(self, idx: int, g: int) -> None:
        cfg, P = self.cfg, self.P
        if not self.reloc or idx < self.seg_start:
            return
        lo, hi = self.reloc_window(idx)
        if hi < lo:
            return
        best, q, j = best_vote([self.vote(idx, qq, lo, hi - lo + 1) for qq in range(P)], P)
        if best < cfg.loop_min_votes:
            return
        c, pc = lo + j // P, j % P
        ver = self.verify(idx, g, q, c, pc)
        if int(ver["stats"][0]) != 0 or int(ver["stats"][2]) < cfg.loop_min_inliers:
            return
        Z = self.m[pc] @ inv_se3(ver["T"]) @ inv_se3(self.m[q])
        D = self.T[c] @ Z @ inv_se3(self.T[idx])
        for i in range(self.seg_start, len(self.T)):
            self.T[i] = D @ self.T[i]
        self.edges.append((c, idx))
        self.meas.append(Z)
        self.corr = D @ self.corr
        self.relocs.append((self.frames[c], g, int(ver["stats"][2])))
        self.reloc = False
        self.last_loop = idx
