"""TEST INFRASTRUCTURE ONLY — NumPy restatement of the per-frame hot path (oracle).

See ``oracle/__init__.py`` for the import rule and the parity status.  Every function names
the SURVEY.md §8a row it defines; the reference anchors for the boundary semantics are cited
inline (``thor_slam/...:line``).  Integer stages (A2-A6) are bit-exact by construction; the
pose stage (A7) uses only IEEE +, -, *, / and sqrt in a fixed operation order (no BLAS, no
transcendental functions), so the HIP kernels — compiled with ``-ffp-contract=off`` — reproduce
the RANSAC decisions exactly and the refined pose to summation-order rounding.

Stages for one stereo frame (left L, right R):

  A2 rectify   integer bilinear remap with 1/32-px fixed-point tables
  A3 pyramid   2x2 box, (a+b+c+d+2)>>2, n_levels levels; 5x5 binomial smoothing per level
  A4 detect    FAST-9 score, threshold, 3x3 NMS with raster tie-break, per-level top-K by
               key = (255-score)<<22 | y<<11 | x (ascending)
  A5 describe  intensity-centroid orientation bin (integer wedge tests) + rotated BRIEF-256
  A6 match     brute-force Hamming per level: stereo (row band, positive disparity) and temporal
               (window) with ratio test + mutual check
  A7 pose      triangulate t-1 stereo matches, P3P-RANSAC with a counter RNG, Gauss-Newton refine

RGB-D frames (BASELINE configs[4], ``OracleTracker.step_rgbd``): the BGR colour image becomes
gray with fixed-point BT.601 weights, is undistorted like A2, and instead of A6 stereo every
keypoint reads the aligned depth (u16 mm) at its nearest raw pixel: disp = fx / Z, a virtual
1 m baseline, so A7 triangulates exactly as for stereo.
"""

from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation

# ----------------------------------------------------------------------------------------
# constants (independent derivation of thor_slam_amd.features; tests compare the two)
# ----------------------------------------------------------------------------------------
CIRCLE = np.array(
    [[0, -3], [1, -3], [2, -2], [3, -1], [3, 0], [3, 1], [2, 2], [1, 3],
     [0, 3], [-1, 3], [-2, 2], [-3, 1], [-3, 0], [-3, -1], [-2, -2], [-1, -3]],
    dtype=np.int64,
)
NBINS = 30
KEY_Y_SHIFT = 11
KEY_S_SHIFT = 22
RECT_BITS = 5
P3P_VMAX = 1000.0
P3P_BISECT = 60
U64 = np.uint64
MASK64 = (1 << 64) - 1


def _rhu(x):
    return np.floor(x + 0.5)


def make_brief_pattern() -> np.ndarray:
    rng = np.random.default_rng(0xB1EF)
    p = np.clip(_rhu(rng.normal(0.0, 31.0 / 5.0, size=(256, 4))), -13, 13).astype(np.int32)
    dup = (p[:, 0] == p[:, 2]) & (p[:, 1] == p[:, 3])
    p[dup, 2] = np.where(p[dup, 2] < 13, p[dup, 2] + 1, p[dup, 2] - 1)
    return p


def make_rotated_table() -> np.ndarray:
    pat = make_brief_pattern().astype(np.float64)
    tab = np.zeros((NBINS, 256, 4), dtype=np.int8)
    for b in range(NBINS):
        a = 2.0 * np.pi * b / NBINS
        c, s = np.cos(a), np.sin(a)
        tab[b, :, 0] = _rhu(c * pat[:, 0] - s * pat[:, 1])
        tab[b, :, 1] = _rhu(s * pat[:, 0] + c * pat[:, 1])
        tab[b, :, 2] = _rhu(c * pat[:, 2] - s * pat[:, 3])
        tab[b, :, 3] = _rhu(s * pat[:, 2] + c * pat[:, 3])
    return tab


def make_wedges() -> np.ndarray:
    ang = (np.arange(NBINS + 1) - 0.5) * (2.0 * np.pi / NBINS)
    w = np.stack([_rhu(np.cos(ang) * 16777216.0), _rhu(np.sin(ang) * 16777216.0)], 1).astype(np.int64)
    w[NBINS] = w[0]
    return w


DISC = np.array([(dx, dy) for dy in range(-15, 16) for dx in range(-15, 16) if dx * dx + dy * dy <= 225], dtype=np.int64)
BRIEF_TABLE = make_rotated_table()
WEDGES = make_wedges()


def level_shapes(w: int, h: int, n: int) -> list[tuple[int, int]]:
    s = [(w, h)]
    while len(s) < n:
        s.append((s[-1][0] // 2, s[-1][1] // 2))
    return s


def level_quotas(k: int, n: int) -> list[int]:
    tot = sum(0.25 ** l for l in range(n))
    q = [int(k * 0.25 ** l / tot) for l in range(n)]
    q[0] = k - sum(q[1:])
    return q


# ----------------------------------------------------------------------------------------
# A2 rectification maps + remap
# ----------------------------------------------------------------------------------------
def distort(x, y, coeffs):
    """Distortion models selected like isaac_ros.py:370-383 (rational_polynomial uses d[:8])."""
    d = list(np.asarray(coeffs, dtype=np.float64).flatten())
    if len(d) == 4:
        r = np.sqrt(x * x + y * y)
        th = np.arctan(r)
        t2 = th * th
        thd = th * (1 + t2 * (d[0] + t2 * (d[1] + t2 * (d[2] + t2 * d[3]))))
        sc = np.where(r > 1e-12, thd / np.where(r > 1e-12, r, 1.0), 1.0)
        return x * sc, y * sc
    if len(d) >= 8:
        d = d[:8]
    elif len(d) != 5:
        d = (d + [0.0] * 5)[:5]
    d = d + [0.0] * (8 - len(d))
    k1, k2, p1, p2, k3, k4, k5, k6 = d
    r2 = x * x + y * y
    rad = (1 + r2 * (k1 + r2 * (k2 + r2 * k3))) / (1 + r2 * (k4 + r2 * (k5 + r2 * k6)))
    return (x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x), y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y)


def rectification(k_l, d_l, w_T_l, k_r, d_r, w_T_r, width, height):
    """Bouguet rectification -> (fx, fy, cx, cy, baseline, map_l, map_r); maps (H, W, 2) int32."""
    r_T_l = np.linalg.inv(np.linalg.inv(w_T_l) @ w_T_r)
    rot, tr = r_T_l[:3, :3], r_T_l[:3, 3]
    half = Rotation.from_rotvec(-0.5 * Rotation.from_matrix(rot).as_rotvec()).as_matrix()
    t = half @ tr
    i = 0 if abs(t[0]) > abs(t[1]) else 1
    uu = np.zeros(3)
    uu[i] = 1.0 if t[i] > 0 else -1.0
    ww = np.cross(t, uu)
    nw = np.linalg.norm(ww)
    if nw > 0:
        ww = ww * (np.arccos(min(1.0, abs(t[i]) / np.linalg.norm(t))) / nw)
    wr = Rotation.from_rotvec(ww).as_matrix()
    rl, rr = wr @ half.T, wr @ half
    f = float(min(k_l[0, 0], k_l[1, 1], k_r[0, 0], k_r[1, 1]))
    cx = 0.5 * (k_l[0, 2] + k_r[0, 2])
    cy = 0.5 * (k_l[1, 2] + k_r[1, 2])

    def one(k, d, rect):
        v, u = np.mgrid[0:height, 0:width].astype(np.float64)
        ray = np.stack([(u - cx) / f, (v - cy) / f, np.ones_like(u)], -1) @ rect
        xd, yd = distort(ray[..., 0] / ray[..., 2], ray[..., 1] / ray[..., 2], d)
        su = k[0, 0] * xd + k[0, 1] * yd + k[0, 2]
        sv = k[1, 1] * yd + k[1, 2]
        mx = np.clip(np.floor(su * 32 + 0.5), -64, (width + 1) * 32).astype(np.int32)
        my = np.clip(np.floor(sv * 32 + 0.5), -64, (height + 1) * 32).astype(np.int32)
        return np.stack([mx, my], -1)

    return f, f, cx, cy, float(-(rr @ tr)[0]), one(k_l, d_l, rl), one(k_r, d_r, rr)


def remap(img: np.ndarray, mp: np.ndarray) -> np.ndarray:
    """A2: out = (sum of 4 taps x integer weights in 1/32 units + 512) >> 10, clamped taps."""
    h, w = img.shape
    mx, my = mp[..., 0].astype(np.int64), mp[..., 1].astype(np.int64)
    x0, y0 = mx >> RECT_BITS, my >> RECT_BITS
    fx, fy = mx & 31, my & 31
    im = img.astype(np.int64)

    def tap(xx, yy):
        return im[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)]

    acc = (tap(x0, y0) * (32 - fx) * (32 - fy) + tap(x0 + 1, y0) * fx * (32 - fy)
           + tap(x0, y0 + 1) * (32 - fx) * fy + tap(x0 + 1, y0 + 1) * fx * fy)
    return ((acc + 512) >> 10).astype(np.uint8)


def bgr_to_gray(bgr: np.ndarray) -> np.ndarray:
    """RGB-D input: (R*4899 + G*9617 + B*1868 + 8192) >> 14 on the BGR u8 image."""
    b = bgr[..., 0].astype(np.int64)
    g = bgr[..., 1].astype(np.int64)
    r = bgr[..., 2].astype(np.int64)
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)


def depth_disparity(feat: dict, depth_mm: np.ndarray, mp: np.ndarray | None, fx: float) -> np.ndarray:
    """RGB-D stand-in for A6 stereo: per keypoint, the depth at the raw pixel nearest to its level-0
    position (rounded, then through the undistortion table ``mp`` when given) as disp = fx / Z
    (Z = mm * 0.001; NaN for padding keypoints and zero depth)."""
    h, w = depth_mm.shape
    kp = feat["kp"]
    u, v = level0_coords(kp["x"], kp["y"], kp["level"])
    ix = np.clip(np.floor(u + 0.5).astype(np.int64), 0, w - 1)
    iy = np.clip(np.floor(v + 0.5).astype(np.int64), 0, h - 1)
    if mp is not None:
        m = mp[iy, ix].astype(np.int64)
        ix = np.clip((m[:, 0] + 16) >> RECT_BITS, 0, w - 1)
        iy = np.clip((m[:, 1] + 16) >> RECT_BITS, 0, h - 1)
    mm = depth_mm[iy, ix].astype(np.int64)
    ok = feat["valid"] & (mm > 0)
    with np.errstate(divide="ignore"):
        disp = fx / (mm.astype(np.float64) * 0.001)
    return np.where(ok, disp, np.nan)


# ----------------------------------------------------------------------------------------
# A3 pyramid + smoothing
# ----------------------------------------------------------------------------------------
def pyramid(img0: np.ndarray, n_levels: int) -> list[np.ndarray]:
    levels = [img0]
    for _ in range(1, n_levels):
        p = levels[-1].astype(np.int32)
        h, w = p.shape[0] // 2, p.shape[1] // 2
        q = p[0 : 2 * h : 2, 0 : 2 * w : 2] + p[0 : 2 * h : 2, 1 : 2 * w : 2] + p[1 : 2 * h : 2, 0 : 2 * w : 2] + p[1 : 2 * h : 2, 1 : 2 * w : 2]
        levels.append(((q + 2) >> 2).astype(np.uint8))
    return levels


def smooth(level: np.ndarray) -> np.ndarray:
    """5x5 binomial [1 4 6 4 1]^2 with replicated borders, (sum + 128) >> 8."""
    wts = np.array([1, 4, 6, 4, 1], dtype=np.int64)
    p = np.pad(level.astype(np.int64), 2, mode="edge")
    h, w = level.shape
    rows = sum(wts[k] * p[:, k : k + w] for k in range(5))
    full = sum(wts[k] * rows[k : k + h, :] for k in range(5))
    return ((full + 128) >> 8).astype(np.uint8)


# ----------------------------------------------------------------------------------------
# A4 FAST-9 + NMS + top-K
# ----------------------------------------------------------------------------------------
def fast_scores(level: np.ndarray) -> np.ndarray:
    """FAST-9 score for every pixel with the circle inside the image (else 0).

    score = max over 16 arcs of 9 contiguous circle pixels of max(min(I_c - I_p), min(I_p - I_c)).
    """
    h, w = level.shape
    im = level.astype(np.int16)
    c = im[3 : h - 3, 3 : w - 3]
    d = np.stack([im[3 + dy : h - 3 + dy, 3 + dx : w - 3 + dx] - c for dx, dy in CIRCLE])
    best = np.full(c.shape, -32768, dtype=np.int16)
    for sign in (1, -1):
        e = d * sign
        m2 = np.minimum(e, np.roll(e, -1, axis=0))
        m4 = np.minimum(m2, np.roll(m2, -2, axis=0))
        m8 = np.minimum(m4, np.roll(m4, -4, axis=0))
        m9 = np.minimum(m8, np.roll(e, -8, axis=0))
        best = np.maximum(best, m9.max(axis=0))
    out = np.zeros((h, w), dtype=np.int32)
    out[3 : h - 3, 3 : w - 3] = np.maximum(best, 0)
    return out


def nms_keys(scores: np.ndarray, threshold: int, margin: int) -> np.ndarray:
    """Keys of 3x3 NMS survivors inside the margin; ties go to the earlier raster position."""
    h, w = scores.shape
    s = np.where(scores > threshold, scores, 0)
    y0, y1, x0, x1 = margin, h - margin, margin, w - margin
    if y1 <= y0 or x1 <= x0:
        return np.zeros(0, dtype=np.int64)
    p = s[y0:y1, x0:x1]
    keep = p > 0
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy == 0 and dx == 0:
                continue
            q = s[y0 + dy : y1 + dy, x0 + dx : x1 + dx]
            after = dy > 0 or (dy == 0 and dx > 0)
            keep &= (q <= p) if after else (q < p)
    ys, xs = np.nonzero(keep)
    ys, xs = ys + y0, xs + x0
    sc = s[ys, xs].astype(np.int64)
    return ((255 - sc) << KEY_S_SHIFT) | (ys.astype(np.int64) << KEY_Y_SHIFT) | xs.astype(np.int64)


def select_topk(keys: np.ndarray, k: int) -> np.ndarray:
    return np.sort(keys)[:k]


def decode_keys(keys: np.ndarray):
    x = keys & 2047
    y = (keys >> KEY_Y_SHIFT) & 2047
    s = 255 - (keys >> KEY_S_SHIFT)
    return x.astype(np.int64), y.astype(np.int64), s.astype(np.int64)


# ----------------------------------------------------------------------------------------
# A5 orientation + rBRIEF
# ----------------------------------------------------------------------------------------
def orientation_bins(level: np.ndarray, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    if x.size == 0:
        return np.zeros(0, dtype=np.int64)
    im = level.astype(np.int64)
    vals = im[y[:, None] + DISC[None, :, 1], x[:, None] + DISC[None, :, 0]]
    m10 = (vals * DISC[None, :, 0]).sum(1)
    m01 = (vals * DISC[None, :, 1]).sum(1)
    cr = WEDGES[None, :, 0] * m01[:, None] - WEDGES[None, :, 1] * m10[:, None]  # cross(u_b, v)
    inside = (cr[:, :-1] >= 0) & (cr[:, 1:] < 0)
    found = inside.any(1)
    return np.where(found, inside.argmax(1), 0).astype(np.int64)


def brief(smoothed: np.ndarray, x: np.ndarray, y: np.ndarray, bins: np.ndarray) -> np.ndarray:
    """(N, 8) uint32 descriptors; bit i of word i>>5 is S(p_i) < S(q_i) under the rotated pattern."""
    if x.size == 0:
        return np.zeros((0, 8), dtype=np.uint32)
    t = BRIEF_TABLE[bins].astype(np.int64)  # (N, 256, 4)
    sm = smoothed.astype(np.int32)
    a = sm[y[:, None] + t[..., 1], x[:, None] + t[..., 0]]
    b = sm[y[:, None] + t[..., 3], x[:, None] + t[..., 2]]
    bits = (a < b).astype(np.uint32).reshape(-1, 8, 32)
    return (bits << np.arange(32, dtype=np.uint32)).sum(axis=2, dtype=np.uint64).astype(np.uint32)


# ----------------------------------------------------------------------------------------
# one image: A3-A5
# ----------------------------------------------------------------------------------------
def extract(img0: np.ndarray, cfg) -> dict:
    """Keypoints (level-segmented, fixed offsets) + descriptors of one rectified image."""
    levels = pyramid(img0, cfg.n_levels)
    quotas = level_quotas(cfg.n_features, cfg.n_levels)
    kmax = cfg.n_features
    kp = {k: np.zeros(kmax, dtype=np.int64) for k in ("x", "y", "score", "level", "angle")}
    for l in range(cfg.n_levels):  # padding entries keep their level (as the device layout does)
        kp["level"][sum(quotas[:l]) : sum(quotas[: l + 1])] = l
    valid = np.zeros(kmax, dtype=bool)
    desc = np.zeros((kmax, 8), dtype=np.uint32)
    counts, offs = [], []
    off = 0
    for l, lev in enumerate(levels):
        keys = select_topk(nms_keys(fast_scores(lev), cfg.fast_threshold, cfg.edge_margin), quotas[l])
        x, y, s = decode_keys(keys)
        n = keys.size
        ang = orientation_bins(lev, x, y)
        d = brief(smooth(lev), x, y, ang)
        sl = slice(off, off + n)
        kp["x"][sl], kp["y"][sl], kp["score"][sl], kp["level"][sl], kp["angle"][sl] = x, y, s, l, ang
        valid[sl] = True
        desc[sl] = d
        counts.append(n)
        offs.append(off)
        off += quotas[l]
    return {"kp": kp, "valid": valid, "desc": desc, "counts": counts, "offsets": offs, "quotas": quotas, "levels": levels}


def level0_coords(x, y, level):
    sc = np.left_shift(1, level).astype(np.float64)
    return (x + 0.5) * sc - 0.5, (y + 0.5) * sc - 0.5


# ----------------------------------------------------------------------------------------
# A6 matching
# ----------------------------------------------------------------------------------------
def match(q: dict, t: dict, cfg, mode: str):
    """Per query keypoint: (match index or -1, best distance).  ``mode`` is 'stereo' or 'temporal'."""
    kmax = cfg.n_features
    idx = np.full(kmax, -1, dtype=np.int64)
    dist = np.full(kmax, 256, dtype=np.int64)
    best_j = np.full(kmax, -1, dtype=np.int64)
    second = np.full(kmax, 256, dtype=np.int64)
    for l in range(cfg.n_levels):
        qo, qn = q["offsets"][l], q["counts"][l]
        to, tn = t["offsets"][l], t["counts"][l]
        if qn == 0 or tn == 0:
            continue
        qs, ts = slice(qo, qo + qn), slice(to, to + tn)
        qd = q["desc"][qs].view(np.uint64)
        td = t["desc"][ts].view(np.uint64)
        d = np.bitwise_count(qd[:, None, :] ^ td[None, :, :]).sum(-1).astype(np.int64)
        qx, qy = q["kp"]["x"][qs][:, None], q["kp"]["y"][qs][:, None]
        tx, ty = t["kp"]["x"][ts][None, :], t["kp"]["y"][ts][None, :]
        if mode == "stereo":
            disp = qx - tx
            elig = (np.abs(qy - ty) <= cfg.stereo_row_tol) & (disp >= 1) & (disp <= (cfg.max_disparity >> l))
        else:
            win = cfg.temporal_window >> l
            elig = (np.abs(qx - tx) <= win) & (np.abs(qy - ty) <= win)
        dm = np.where(elig, d, 1 << 20)
        bj = dm.argmin(1)
        bd = dm[np.arange(qn), bj]
        dm2 = dm.copy()
        dm2[np.arange(qn), bj] = 1 << 20
        sd = dm2.min(1)
        sd = np.where(sd >= (1 << 20), 256, sd)
        ti = dm.argmin(0)  # train side best query (first = lowest index among ties)
        has = bd < (1 << 20)
        ok = has & (bd <= cfg.max_hamming) & (bd * 100 < cfg.ratio_pct * sd) & (ti[bj] == np.arange(qn))
        idx[qs] = np.where(ok, bj + to, -1)
        dist[qs] = np.where(has, bd, 256)
        best_j[qs] = np.where(has, bj + to, -1)
        second[qs] = sd
    return idx, dist, best_j, second


# ----------------------------------------------------------------------------------------
# A7 pose: correspondences, counter RNG, P3P, RANSAC, Gauss-Newton
# ----------------------------------------------------------------------------------------
def splitmix64(x):
    x = (x + U64(0x9E3779B97F4A7C15)).astype(U64)
    x = ((x ^ (x >> U64(30))) * U64(0xBF58476D1CE4E5B9)).astype(U64)
    x = ((x ^ (x >> U64(27))) * U64(0x94D049BB133111EB)).astype(U64)
    return (x ^ (x >> U64(31))).astype(U64)


def sample_triplets(seed: int, frame: int, n_hyp: int, n: int) -> np.ndarray:
    """(H, 3) distinct correspondence indices from the counter-based RNG."""
    with np.errstate(over="ignore"):
        base = splitmix64(np.array([(seed ^ ((frame * 0x9E3779B97F4A7C15) & MASK64)) & MASK64], dtype=U64))[0]
        h = np.arange(n_hyp, dtype=U64)
        r = [(splitmix64(base ^ (h * U64(4) + U64(k))) >> U64(32)).astype(np.uint64) for k in range(3)]
    i0 = (r[0] % U64(n)).astype(np.int64)
    i1 = (r[1] % U64(n - 1)).astype(np.int64)
    i1 = i1 + (i1 >= i0)
    i2 = (r[2] % U64(n - 2)).astype(np.int64)
    lo, hi = np.minimum(i0, i1), np.maximum(i0, i1)
    i2 = i2 + (i2 >= lo)
    i2 = i2 + (i2 >= hi)
    return np.stack([i0, i1, i2], 1)


def _horner(c, v):
    p = c[-1]
    for k in range(len(c) - 2, -1, -1):
        p = p * v + c[k]
    return p


def _roots(c: list, lo: float, hi: float) -> np.ndarray:
    """Real roots in (lo, hi) of sum c_k v^k (coefficient arrays over hypotheses), ascending,
    NaN-padded to the degree.  Monotone intervals come from the derivative's roots; each interval
    with a sign change is bisected ``P3P_BISECT`` times."""
    deg = len(c) - 1
    nh = c[0].shape[0]
    if deg == 1:
        with np.errstate(divide="ignore", invalid="ignore"):
            r = -c[0] / c[1]
        ok = (c[1] != 0) & (r > lo) & (r < hi)
        return np.where(ok, r, np.nan)[:, None]
    dc = [c[k + 1] * float(k + 1) for k in range(deg)]
    crit = np.sort(_roots(dc, lo, hi), axis=1)
    crit = np.where(np.isnan(crit), hi, crit)
    pts = np.concatenate([np.full((nh, 1), lo), crit, np.full((nh, 1), hi)], 1)
    out = np.full((nh, deg), np.nan)
    for i in range(deg):
        a, b = pts[:, i].copy(), pts[:, i + 1].copy()
        sa = _horner(c, a) > 0
        sb = _horner(c, b) > 0
        has = (sa != sb) & (b > a)
        for _ in range(P3P_BISECT):
            m = 0.5 * (a + b)
            sm = _horner(c, m) > 0
            same = sm == sa
            a = np.where(same, m, a)
            b = np.where(same, b, m)
        out[:, i] = np.where(has, 0.5 * (a + b), np.nan)
    return np.sort(out, axis=1)


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def _sub(a, b):
    return [a[0] - b[0], a[1] - b[1], a[2] - b[2]]


def _normalize(a):
    n = np.sqrt(_dot(a, a))
    return [a[0] / n, a[1] / n, a[2] / n]


def _frame(p1, p2, p3):
    e1 = _normalize(_sub(p2, p1))
    e3 = _normalize(_cross(e1, _sub(p3, p1)))
    e2 = _cross(e3, e1)
    return e1, e2, e3


def p3p(pw: list, f: list):
    """Grunert P3P, vectorised over hypotheses.

    pw[k], f[k]: world points / unit bearings of the 3 samples, each a list of 3 arrays (H,).
    Returns R (H, 4, 3, 3), t (H, 4, 3) and a validity mask (H, 4), solutions ordered by the
    ascending root v = s3 / s1.  Degenerate samples (coincident or collinear points, coincident
    bearings) divide by zero and produce NaN / inf on purpose, as the kernel does: those
    solutions fail the finiteness tests (IEEE semantics, no warnings).
    """
    with np.errstate(all="ignore"):
        return _p3p(pw, f)


def _p3p(pw: list, f: list):
    a2 = _dot(_sub(pw[1], pw[2]), _sub(pw[1], pw[2]))
    b2 = _dot(_sub(pw[0], pw[2]), _sub(pw[0], pw[2]))
    c2 = _dot(_sub(pw[0], pw[1]), _sub(pw[0], pw[1]))
    ca = _dot(f[1], f[2])
    cb = _dot(f[0], f[2])
    cg = _dot(f[0], f[1])
    kk = (a2 - c2) / b2
    kc = c2 / b2
    n0, n1, n2 = 1.0 + kk, -2.0 * kk * cb, kk - 1.0
    d0, d1 = cg, -ca
    g0, g1, g2 = 1.0 - kc, 2.0 * kc * cb, -kc  # 1 - kc * M(v)
    # N^2
    q4 = n2 * n2
    q3 = 2.0 * n1 * n2
    q2 = n1 * n1 + 2.0 * n0 * n2
    q1 = 2.0 * n0 * n1
    q0 = n0 * n0
    # -4 cg N D
    m = -4.0 * cg
    q3 = q3 + m * (n2 * d1)
    q2 = q2 + m * (n1 * d1 + n2 * d0)
    q1 = q1 + m * (n0 * d1 + n1 * d0)
    q0 = q0 + m * (n0 * d0)
    # 4 D^2 G
    e0, e1, e2 = d0 * d0, 2.0 * d0 * d1, d1 * d1
    q4 = q4 + 4.0 * (e2 * g2)
    q3 = q3 + 4.0 * (e1 * g2 + e2 * g1)
    q2 = q2 + 4.0 * ((e0 * g2 + e1 * g1) + e2 * g0)
    q1 = q1 + 4.0 * (e0 * g1 + e1 * g0)
    q0 = q0 + 4.0 * (e0 * g0)
    roots = _roots([q0, q1, q2, q3, q4], 0.0, P3P_VMAX)
    nh = q0.shape[0]
    rot = np.full((nh, 4, 3, 3), np.nan)
    trn = np.full((nh, 4, 3), np.nan)
    ok = np.zeros((nh, 4), dtype=bool)
    fw = _frame(pw[0], pw[1], pw[2])
    for s in range(4):
        v = roots[:, s]
        num = (n0 + n1 * v) + n2 * (v * v)
        den = 2.0 * (cg - ca * v)
        u = num / den
        s1sq = b2 / ((1.0 + v * v) - 2.0 * cb * v)
        good = np.isfinite(v) & (u > 0) & (s1sq > 0) & np.isfinite(u) & np.isfinite(s1sq)
        s1 = np.sqrt(np.where(good, s1sq, 1.0))
        s2 = u * s1
        s3 = v * s1
        pc = [[f[0][k] * s1 for k in range(3)], [f[1][k] * s2 for k in range(3)], [f[2][k] * s3 for k in range(3)]]
        fc = _frame(pc[0], pc[1], pc[2])
        for i in range(3):
            for j in range(3):
                rot[:, s, i, j] = (fc[0][i] * fw[0][j] + fc[1][i] * fw[1][j]) + fc[2][i] * fw[2][j]
        for i in range(3):
            rp = (rot[:, s, i, 0] * pw[0][0] + rot[:, s, i, 1] * pw[0][1]) + rot[:, s, i, 2] * pw[0][2]
            trn[:, s, i] = pc[0][i] - rp
        good &= np.isfinite(rot[:, s]).all((1, 2)) & np.isfinite(trn[:, s]).all(1)
        ok[:, s] = good
    return rot, trn, ok


def count_inliers(rot, trn, corr, intr, thr2):
    """Inlier counts for poses rot (..., 3, 3) / trn (..., 3) over correspondences ``corr``."""
    fx, fy = intr[0], intr[1]
    X, Y, Z, du, dv = corr["X"], corr["Y"], corr["Z"], corr["du"], corr["dv"]
    r = rot[..., None]
    t = trn[..., None]
    xc = (r[..., 0, 0, :] * X + r[..., 0, 1, :] * Y) + r[..., 0, 2, :] * Z + t[..., 0, :]
    yc = (r[..., 1, 0, :] * X + r[..., 1, 1, :] * Y) + r[..., 1, 2, :] * Z + t[..., 1, :]
    zc = (r[..., 2, 0, :] * X + r[..., 2, 1, :] * Y) + r[..., 2, 2, :] * Z + t[..., 2, :]
    ex = fx * xc + du * zc
    ey = fy * yc + dv * zc
    e2 = ex * ex + ey * ey
    lim = thr2 * (zc * zc)
    with np.errstate(invalid="ignore"):
        return ((zc > 0) & (e2 < lim)).sum(-1)


def cayley(w):
    """Rotation with derivative [w]x at 0: I + 4/(4+|w|^2) ([w]x + [w]x^2 / 2)."""
    a = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    a2 = np.zeros((3, 3))
    for i in range(3):
        for j in range(3):
            a2[i, j] = (a[i, 0] * a[0, j] + a[i, 1] * a[1, j]) + a[i, 2] * a[2, j]
    n2 = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]
    s = 4.0 / (4.0 + n2)
    return np.eye(3) + s * (a + 0.5 * a2)


def solve6(hm: np.ndarray, g: np.ndarray):
    """Cholesky solve of the 6x6 normal equations (explicit loops, same order as the kernel)."""
    lm = np.zeros((6, 6))
    for j in range(6):
        s = hm[j, j]
        for k in range(j):
            s = s - lm[j, k] * lm[j, k]
        if not s > 0:
            return None
        lm[j, j] = np.sqrt(s)
        for i in range(j + 1, 6):
            s = hm[i, j]
            for k in range(j):
                s = s - lm[i, k] * lm[j, k]
            lm[i, j] = s / lm[j, j]
    y = np.zeros(6)
    for i in range(6):
        s = g[i]
        for k in range(i):
            s = s - lm[i, k] * y[k]
        y[i] = s / lm[i, i]
    x = np.zeros(6)
    for i in range(5, -1, -1):
        s = y[i]
        for k in range(i + 1, 6):
            s = s - lm[k, i] * x[k]
        x[i] = s / lm[i, i]
    return x, lm


def refine(rot, trn, corr, intr, thr2, iters, prior=None):
    """Gauss-Newton on the current inliers, re-selected every iteration.  Returns R, t, H, stats.

    ``prior`` = (R_prior, W) or (R_prior, W, t_prior, W_t): IMU prior, the
    term W/2 |w - delta|^2 with delta = vee of the antisymmetric part of R_prior R^T (small angle),
    and W_t/2 |t + rho - t_prior|^2 (accelerometer translation prediction)."""
    fx, fy, cx, cy = intr
    u = cx - corr["du"]
    v = cy - corr["dv"]
    hm = np.zeros((6, 6))
    n_in = 0
    sq = 0.0
    for _ in range(iters):
        m = count_inliers_mask(rot, trn, corr, intr, thr2)
        n_in = int(m.sum())
        if n_in < 6:
            return rot, trn, None, n_in, 0.0
        X, Y, Z = corr["X"][m], corr["Y"][m], corr["Z"][m]
        xc = (rot[0, 0] * X + rot[0, 1] * Y) + rot[0, 2] * Z + trn[0]
        yc = (rot[1, 0] * X + rot[1, 1] * Y) + rot[1, 2] * Z + trn[1]
        zc = (rot[2, 0] * X + rot[2, 1] * Y) + rot[2, 2] * Z + trn[2]
        iz = 1.0 / zc
        rx = (fx * xc) * iz + cx - u[m]
        ry = (fy * yc) * iz + cy - v[m]
        a, b = fx * iz, fy * iz
        c = -(fx * xc) * (iz * iz)
        d = -(fy * yc) * (iz * iz)
        # J rows: d(res)/d(rho, omega), with dXc/domega = -[Xc]x
        jx = [a, 0.0 * a, c, c * yc, a * zc - c * xc, -a * yc]
        jy = [0.0 * b, b, d, -b * zc + d * yc, -d * xc, b * xc]
        hm = np.zeros((6, 6))
        g = np.zeros(6)
        for i in range(6):
            g[i] = -(np.sum(jx[i] * rx) + np.sum(jy[i] * ry))
            for j in range(i, 6):
                hm[i, j] = np.sum(jx[i] * jx[j]) + np.sum(jy[i] * jy[j])
                hm[j, i] = hm[i, j]
        if prior is not None and prior[1] > 0:
            rp, w = prior[0], prior[1]
            mq = np.array([[(rp[i, 0] * rot[j, 0] + rp[i, 1] * rot[j, 1]) + rp[i, 2] * rot[j, 2] for j in range(3)]
                           for i in range(3)])
            dl = [0.5 * (mq[2, 1] - mq[1, 2]), 0.5 * (mq[0, 2] - mq[2, 0]), 0.5 * (mq[1, 0] - mq[0, 1])]
            for i in range(3):
                hm[3 + i, 3 + i] += w
                g[3 + i] += w * dl[i]
        if prior is not None and len(prior) > 2 and prior[3] > 0:
            tp, wt = prior[2], prior[3]
            for i in range(3):
                hm[i, i] += wt
                g[i] += wt * (tp[i] - trn[i])
        sol = solve6(hm, g)
        if sol is None:
            return rot, trn, None, n_in, 0.0
        dx = sol[0]
        ru = cayley(dx[3:])
        rot = np.array([[(ru[i, 0] * rot[0, j] + ru[i, 1] * rot[1, j]) + ru[i, 2] * rot[2, j] for j in range(3)] for i in range(3)])
        trn = np.array([((ru[i, 0] * trn[0] + ru[i, 1] * trn[1]) + ru[i, 2] * trn[2]) + dx[i] for i in range(3)])
        sq = float(np.sum(rx * rx) + np.sum(ry * ry))
    m = count_inliers_mask(rot, trn, corr, intr, thr2)
    return rot, trn, hm, int(m.sum()), sq


def count_inliers_mask(rot, trn, corr, intr, thr2):
    fx, fy = intr[0], intr[1]
    X, Y, Z = corr["X"], corr["Y"], corr["Z"]
    xc = (rot[0, 0] * X + rot[0, 1] * Y) + rot[0, 2] * Z + trn[0]
    yc = (rot[1, 0] * X + rot[1, 1] * Y) + rot[1, 2] * Z + trn[1]
    zc = (rot[2, 0] * X + rot[2, 1] * Y) + rot[2, 2] * Z + trn[2]
    ex = fx * xc + corr["du"] * zc
    ey = fy * yc + corr["dv"] * zc
    with np.errstate(invalid="ignore"):
        return (zc > 0) & ((ex * ex + ey * ey) < thr2 * (zc * zc))


SAD_HALF = 5
SAD_RANGE = 2


def _parabola(sm, s0, sp):
    """Sub-pixel offset of a discrete minimum from three integer costs (exact double division)."""
    den = 2.0 * (sm - 2 * s0 + sp).astype(np.float64)
    num = (sm - sp).astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(den > 0, num / den, 0.0)


def _patch_sad(ref: np.ndarray, rx, ry, img: np.ndarray, ix, iy) -> np.ndarray:
    """Sum |ref(rx+dx, ry+dy) - img(ix+dx, iy+dy)| over the 11x11 window (int64)."""
    d = np.arange(-SAD_HALF, SAD_HALF + 1)
    a = ref[ry[:, None, None] + d[None, :, None], rx[:, None, None] + d[None, None, :]].astype(np.int64)
    b = img[iy[:, None, None] + d[None, :, None], ix[:, None, None] + d[None, None, :]].astype(np.int64)
    return np.abs(a - b).sum((1, 2))


def stereo_subpixel(fl: dict, fr: dict, sidx: np.ndarray, levels_l, levels_r):
    """A6b: refined level-0 disparity per left keypoint (NaN when unmatched or rejected).

    For a stereo match (i -> r) at level l, the left 11x11 patch at (x_i, y_i) is compared with
    the right image along row y_i at x_r + k, k in [-2, 2]; the first minimum k* must be
    interior, then d0 = (x_i - (x_r + k* + delta)) * 2^l with the parabola delta.
    """
    disp = np.full(sidx.shape[0], np.nan)
    i = np.nonzero(sidx >= 0)[0]
    if i.size == 0:
        return disp
    r = sidx[i]
    lev = fl["kp"]["level"][i]
    for l in np.unique(lev):
        m = lev == l
        ii, rr = i[m], r[m]
        xi, yi = fl["kp"]["x"][ii], fl["kp"]["y"][ii]
        xr = fr["kp"]["x"][rr]
        cost = np.stack([_patch_sad(levels_l[l], xi, yi, levels_r[l], xr + k, yi) for k in range(-SAD_RANGE, SAD_RANGE + 1)], 1)
        ks = cost.argmin(1)
        inner = (ks > 0) & (ks < 2 * SAD_RANGE)
        kc = np.clip(ks, 1, 2 * SAD_RANGE - 1)
        rows = np.arange(ks.size)
        delta = _parabola(cost[rows, kc - 1], cost[rows, kc], cost[rows, kc + 1])
        d0 = (xi - ((xr + (ks - SAD_RANGE)) + delta)) * float(1 << int(l))
        disp[ii] = np.where(inner & (d0 > 0), d0, np.nan)
    return disp


def temporal_subpixel(fp: dict, fc: dict, i: np.ndarray, j: np.ndarray, levels_p, levels_c):
    """A7a: refined level-0 (u, v) at time t of each correspondence (i at t-1 -> j at t), plus
    a validity mask.  5x5 integer offsets, first minimum in raster order, must be interior."""
    u = np.full(i.size, np.nan)
    v = np.full(i.size, np.nan)
    ok = np.zeros(i.size, dtype=bool)
    lev = fc["kp"]["level"][j]
    for l in np.unique(lev):
        m = np.nonzero(lev == l)[0]
        xi, yi = fp["kp"]["x"][i[m]], fp["kp"]["y"][i[m]]
        xj, yj = fc["kp"]["x"][j[m]], fc["kp"]["y"][j[m]]
        n = 2 * SAD_RANGE + 1
        cost = np.stack([_patch_sad(levels_p[l], xi, yi, levels_c[l], xj + kx - SAD_RANGE, yj + ky - SAD_RANGE)
                         for ky in range(n) for kx in range(n)], 1)
        a = cost.argmin(1)
        ky, kx = a // n, a % n
        inner = (kx > 0) & (kx < n - 1) & (ky > 0) & (ky < n - 1)
        kxc, kyc = np.clip(kx, 1, n - 2), np.clip(ky, 1, n - 2)
        rows = np.arange(a.size)
        dx = _parabola(cost[rows, kyc * n + kxc - 1], cost[rows, kyc * n + kxc], cost[rows, kyc * n + kxc + 1])
        dy = _parabola(cost[rows, (kyc - 1) * n + kxc], cost[rows, kyc * n + kxc], cost[rows, (kyc + 1) * n + kxc])
        sc = float(1 << int(l))
        u[m] = ((xj + (kx - SAD_RANGE)) + dx + 0.5) * sc - 0.5
        v[m] = ((yj + (ky - SAD_RANGE)) + dy + 0.5) * sc - 0.5
        ok[m] = inner
    return u, v, ok


def build_correspondences(prev: dict, cur: dict, temporal_cur, rect) -> dict:
    """3D (t-1 refined stereo) <-> 2D (t refined) pairs, ordered by the t keypoint index."""
    fx, fy, cx, cy, fxb = rect
    j = np.nonzero(temporal_cur >= 0)[0]
    i = temporal_cur[j]
    disp = prev["disp"][i]
    keep = np.isfinite(disp)
    j, i, disp = j[keep], i[keep], disp[keep]
    lp = prev["left"]
    ul, vl = level0_coords(lp["kp"]["x"][i], lp["kp"]["y"][i], lp["kp"]["level"][i])
    uc, vc, ok = temporal_subpixel(lp, cur["left"], i, j, lp["levels"], cur["left"]["levels"])
    j, i, disp, ul, vl, uc, vc = j[ok], i[ok], disp[ok], ul[ok], vl[ok], uc[ok], vc[ok]
    z = fxb / disp
    x = (ul - cx) * z / fx
    y = (vl - cy) * z / fy
    return {"X": x, "Y": y, "Z": z, "du": cx - uc, "dv": cy - vc, "u": uc, "v": vc, "j": j, "i": i}


def bearings(corr, intr):
    fx, fy, cx, cy = intr
    bx = (corr["u"] - cx) / fx
    by = (corr["v"] - cy) / fy
    n = np.sqrt((bx * bx + by * by) + 1.0)
    return bx / n, by / n, 1.0 / n


def estimate_pose(corr: dict, intr, cfg, frame: int, prior=None) -> dict:
    """P3P-RANSAC + Gauss-Newton: T (4x4, cam_{t-1} -> cam_t), covariance, counts, status."""
    n = corr["X"].size
    thr2 = float(cfg.ransac_thr_px) * float(cfg.ransac_thr_px)
    out = {"T": np.eye(4), "cov": np.zeros((6, 6)), "n_corr": n, "n_inliers": 0, "status": 1, "best_hyp": -1, "best_count": 0}
    if n < max(6, cfg.min_inliers):
        return out
    tri = sample_triplets(cfg.ransac_seed, frame, cfg.ransac_hypotheses, n)
    bx, by, bz = bearings(corr, intr)
    pw = [[corr["X"][tri[:, k]], corr["Y"][tri[:, k]], corr["Z"][tri[:, k]]] for k in range(3)]
    fb = [[bx[tri[:, k]], by[tri[:, k]], bz[tri[:, k]]] for k in range(3)]
    rot, trn, ok = p3p(pw, fb)
    cnt = count_inliers(rot, trn, corr, intr, thr2)
    cnt = np.where(ok, cnt, -1)
    flat = cnt.reshape(-1)
    best = int(np.argmax(flat))  # first maximum = lowest (hypothesis, solution)
    out["best_hyp"], out["best_count"] = best, int(flat[best])
    if flat[best] < 3:
        return out
    r0 = rot.reshape(-1, 3, 3)[best]
    t0 = trn.reshape(-1, 3)[best]
    r1, t1, hm, n_in, sq = refine(r0, t0, corr, intr, thr2, cfg.refine_iters, prior)
    out["n_inliers"] = n_in
    if hm is None or n_in < cfg.min_inliers:
        return out
    t = np.eye(4)
    t[:3, :3], t[:3, 3] = r1, t1
    sigma2 = sq / max(1, 2 * n_in - 6)
    out["T"] = t
    out["cov"] = np.linalg.inv(hm) * sigma2
    out["sigma2"] = sigma2
    out["status"] = 0
    return out


# ----------------------------------------------------------------------------------------
# whole stereo frame + a sequence driver
# ----------------------------------------------------------------------------------------
class OracleTracker:
    """Stateful CPU tracker for one stereo pair: frame t uses frame t-1's stereo triangulation."""

    def __init__(self, cfg, rect_params: dict):
        self.cfg = cfg
        self.rect = rect_params  # fx, fy, cx, cy, baseline, map_l, map_r
        self.prev = None
        self.frame = 0
        self.world_T_cam = np.eye(4)

    def reset(self):
        self.prev = None
        self.frame = 0
        self.world_T_cam = np.eye(4)

    def step(self, left_raw: np.ndarray, right_raw: np.ndarray, prior=None) -> dict:
        cfg, rp = self.cfg, self.rect
        left = remap(left_raw, rp["map_l"])
        right = remap(right_raw, rp["map_r"])
        fl, fr = extract(left, cfg), extract(right, cfg)
        sm = match(fl, fr, cfg, "stereo")
        disp = stereo_subpixel(fl, fr, sm[0], fl["levels"], fr["levels"])
        cur = {"left": fl, "right": fr, "stereo": sm[0], "stereo_full": sm, "disp": disp,
               "rect_left": left, "rect_right": right}
        return self._advance(cur, prior)

    def step_rgbd(self, bgr: np.ndarray, depth_mm: np.ndarray) -> dict:
        """One RGB-D frame: colour -> gray -> undistort -> features; depth -> disparity."""
        cfg, rp = self.cfg, self.rect
        left = remap(bgr_to_gray(bgr), rp["map_l"])
        fl = extract(left, cfg)
        disp = depth_disparity(fl, depth_mm, rp["map_l"], rp["fx"])
        stereo = np.where(np.isfinite(disp), np.arange(cfg.n_features), -1)
        cur = {"left": fl, "right": None, "stereo": stereo, "disp": disp, "rect_left": left}
        return self._advance(cur)

    def _advance(self, cur: dict, prior=None) -> dict:
        cfg, rp = self.cfg, self.rect
        intr = (rp["fx"], rp["fy"], rp["cx"], rp["cy"])
        res = {"frame": self.frame, "cur": cur}
        if self.prev is None:
            res.update(T=np.eye(4), cov=np.zeros((6, 6)), status=2, n_corr=0, n_inliers=0)
            cur["temporal"] = np.full(cfg.n_features, -1, dtype=np.int64)
        else:
            tm = match(cur["left"], self.prev["left"], cfg, "temporal")
            cur["temporal"] = tm[0]
            cur["temporal_full"] = tm
            corr = build_correspondences(self.prev, cur, tm[0], (rp["fx"], rp["fy"], rp["cx"], rp["cy"], rp["fx"] * rp["baseline"]))
            est = estimate_pose(corr, intr, cfg, self.frame, prior)
            res.update(est)
            res["corr"] = corr
            if est["status"] != 0 and prior is not None and len(prior) > 2 and prior[3] > 0:
                # untracked frame with an accelerometer prediction: it moves by the IMU's T_rel
                t = np.eye(4)
                t[:3, :3], t[:3, 3] = prior[0], prior[2]
                res["T"] = t
                est = dict(est, status=-1)
            if est["status"] <= 0:
                t = res["T"]
                inv = np.eye(4)
                inv[:3, :3] = t[:3, :3].T
                inv[:3, 3] = -(t[:3, :3].T @ t[:3, 3])
                self.world_T_cam = self.world_T_cam @ inv
        res["world_T_cam"] = self.world_T_cam.copy()
        self.prev = cur
        self.frame += 1
        return res
