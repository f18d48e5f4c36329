"""Multi-GPU exchange for multi-camera rigs.

One process per GPU, one stereo source per rank.  After each batch, every rank packs its
keypoint + descriptor block on the device (``tslam_pack_features``).  It appends its per-frame
relative poses (same call), and the ranks all-gather the blocks over RCCL (``torch.distributed`` backend
``nccl`` = RCCL on ROCm; ``gloo`` on CPU for tests).  Every rank then holds the whole rig's
features for cross-camera matching, and the per-source motions for the rig-level solve
(``fuse_rig_motion``).

Block layout per (frame, camera), all little-endian:
``K*8`` bytes keypoints (u32 x|y<<16, u32 level|angle<<8|score<<16) | ``K*32`` bytes descriptors |
``L*4`` bytes per-level counts; then a pose trailer per (frame, stereo pair) of ``16 + 36`` f64
(T_rel, cov) plus 8 i32 (stats).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class BlockLayout:
    n_frames: int
    n_cams: int
    K: int
    L: int

    @property
    def cam_bytes(self) -> int:
        return self.K * 8 + self.K * 32 + self.L * 4

    @property
    def pose_bytes(self) -> int:
        return (16 + 36) * 8 + 8 * 4

    @property
    def feature_bytes(self) -> int:
        return self.n_frames * self.n_cams * self.cam_bytes

    @property
    def n_pairs(self) -> int:
        return self.n_cams // 2

    @property
    def rank_bytes(self) -> int:
        return self.feature_bytes + self.n_frames * self.n_pairs * self.pose_bytes


def pack_block(layout: BlockLayout, kps: np.ndarray, desc: np.ndarray, counts: np.ndarray,
               t_rel: np.ndarray, cov: np.ndarray, stats: np.ndarray) -> np.ndarray:
    """Host-side construction of one rank's block (the device writes the same bytes)."""
    K, L = layout.K, layout.L
    feats = np.zeros((layout.n_frames, layout.n_cams, layout.cam_bytes), dtype=np.uint8)
    feats[..., : K * 8] = np.ascontiguousarray(kps, np.uint32).reshape(layout.n_frames, layout.n_cams, -1).view(np.uint8)
    feats[..., K * 8 : K * 40] = np.ascontiguousarray(desc, np.uint32).reshape(layout.n_frames, layout.n_cams, -1).view(np.uint8)
    feats[..., K * 40 :] = np.ascontiguousarray(counts, np.int32).reshape(layout.n_frames, layout.n_cams, -1).view(np.uint8)
    n = layout.n_frames * layout.n_pairs
    trailer = np.zeros((n, layout.pose_bytes), dtype=np.uint8)
    t_rel = np.asarray(t_rel, np.float64).reshape(n, 16)
    cov = np.asarray(cov, np.float64).reshape(n, 36)
    trailer[:, : 52 * 8] = np.ascontiguousarray(np.concatenate([t_rel, cov], axis=1)).view(np.uint8)
    trailer[:, 52 * 8 :] = np.ascontiguousarray(np.asarray(stats, np.int32).reshape(n, 8)).view(np.uint8)
    return np.concatenate([feats.reshape(-1), trailer.reshape(-1)])


def unpack_rank_block(layout: BlockLayout, buf: np.ndarray) -> dict:
    """Decode one rank's block (uint8, rank_bytes) into per-frame/camera arrays."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    feats = buf[: layout.feature_bytes].reshape(layout.n_frames, layout.n_cams, layout.cam_bytes)
    K, L = layout.K, layout.L
    kp = feats[..., : K * 8].copy().view(np.uint32).reshape(layout.n_frames, layout.n_cams, K, 2)
    desc = feats[..., K * 8 : K * 40].copy().view(np.uint32).reshape(layout.n_frames, layout.n_cams, K, 8)
    counts = feats[..., K * 40 :].copy().view(np.int32).reshape(layout.n_frames, layout.n_cams, L)
    n = layout.n_frames * layout.n_pairs
    poses = buf[layout.feature_bytes :].reshape(n, layout.pose_bytes)
    dbl = poses[:, : 52 * 8].copy().view(np.float64).reshape(layout.n_frames, layout.n_pairs, 52)
    stats = poses[:, 52 * 8 :].copy().view(np.int32).reshape(layout.n_frames, layout.n_pairs, 8)
    return {
        "x": kp[..., 0] & 0xFFFF, "y": kp[..., 0] >> 16, "level": kp[..., 1] & 0xFF, "angle": (kp[..., 1] >> 8) & 0xFF,
        "score": kp[..., 1] >> 16, "desc": desc, "counts": counts,
        "T_rel": dbl[..., :16].reshape(layout.n_frames, layout.n_pairs, 4, 4),
        "cov": dbl[..., 16:].reshape(layout.n_frames, layout.n_pairs, 6, 6), "stats": stats,
    }


class FeatureExchange:
    """Owns the send/receive buffers of the per-step all-gather (device tensors for RCCL)."""

    def __init__(self, layout: BlockLayout, device, world: int):
        import torch

        self.layout = layout
        self.world = world
        self.device = device
        self.send = torch.zeros((layout.rank_bytes,), dtype=torch.uint8, device=device)
        self.recv = torch.zeros((world * layout.rank_bytes,), dtype=torch.uint8, device=device)

    def all_gather(self, async_op: bool = False):
        """All-gather ``send`` from every rank into ``recv`` ([world][rank_bytes]).

        With ``async_op`` (RCCL) the collective is queued behind the current stream's work (the
        pack kernel) and the call returns its work handle at once; ``handle.wait()`` makes the
        current stream wait for it, so the next batch's kernels overlap the transfer."""
        import torch.distributed as dist

        if self.world == 1:
            self.recv.copy_(self.send)
            return None
        if dist.get_backend() == "nccl":
            return dist.all_gather_into_tensor(self.recv, self.send, async_op=async_op)
        parts = list(self.recv.view(self.world, -1).unbind(0))  # gloo (CPU tensors)
        dist.all_gather(parts, self.send)
        return None

    def ranks(self) -> list[dict]:
        host = self.recv.view(self.world, -1).cpu().numpy()
        return [unpack_rank_block(self.layout, host[r]) for r in range(self.world)]


def _log_so3(r: np.ndarray) -> np.ndarray:
    from scipy.spatial.transform import Rotation

    return Rotation.from_matrix(r).as_rotvec()


def _exp_so3(w: np.ndarray) -> np.ndarray:
    from scipy.spatial.transform import Rotation

    return Rotation.from_rotvec(w).as_matrix()


def body_motion(base_T_cam: np.ndarray, cam_rel: np.ndarray) -> np.ndarray:
    """Relative camera motion (cam_{t-1} -> cam_t point map) as base_{t-1}_T_base_t."""
    cam_prev_T_cam = np.linalg.inv(cam_rel)
    return base_T_cam @ cam_prev_T_cam @ np.linalg.inv(base_T_cam)


def fuse_rig_motion(base_T_cams: list[np.ndarray], rels: list[np.ndarray], covs: list[np.ndarray], ok: list[bool]) -> np.ndarray | None:
    """Information-weighted fusion of the per-source body motions of one frame.

    Every source of a rigid rig observes the same body motion.  Each source's estimate is mapped
    to the body frame, and the estimates are averaged in the tangent space of the first valid
    one, weighted by the inverse of the rotated 6x6 covariance (diagonal approximation).
    """
    mots, wts = [], []
    for bt, rel, cov, good in zip(base_T_cams, rels, covs, ok):
        if not good:
            continue
        m = body_motion(bt, rel)
        rot6 = np.zeros((6, 6))
        rot6[:3, :3] = rot6[3:, 3:] = bt[:3, :3]
        c = rot6 @ np.asarray(cov) @ rot6.T
        w = 1.0 / np.maximum(np.diag(c), 1e-18)
        mots.append(m)
        wts.append(w)
    if not mots:
        return None
    ref = mots[0]
    num = np.zeros(6)
    den = np.zeros(6)
    for m, w in zip(mots, wts):
        d = np.linalg.inv(ref) @ m
        xi = np.concatenate([d[:3, 3], _log_so3(d[:3, :3])])
        num += w * xi
        den += w
    xi = num / den
    out = np.eye(4)
    out[:3, :3] = _exp_so3(xi[3:])
    out[:3, 3] = xi[:3]
    return ref @ out
