"""Shared fixtures-as-functions for the parity tests (cached per process)."""

from __future__ import annotations

import functools

import numpy as np

from oracle import numpy_slam as O
from thor_slam_amd.calib import extract_cameras, stereo_pairs, stereo_rectify
from thor_slam_amd.camera.rig import CameraRig
from thor_slam_amd.params import HipSlamConfig
from thor_slam_amd.synthetic import SyntheticStereoSource

DISTORTION = np.array([-0.05, 0.01, 0.0005, -0.0003, 0.0, 0.0, 0.0, 0.0])


def make_source(seed: int = 0, width: int = 640, height: int = 400, distorted: bool = False, n_frames: int = 200):
    return SyntheticStereoSource(seed=seed, width=width, height=height, n_frames=n_frames,
                                 distortion=DISTORTION if distorted else None)


def rig_calibration(src):
    return CameraRig([src]).calibration


@functools.lru_cache(maxsize=8)
def scenario(seed: int = 0, n: int = 4, width: int = 640, height: int = 400, distorted: bool = False,
             cfg_items: tuple = ()):
    """Rendered frames + product rectification + oracle run of one stereo sequence."""
    cfg = HipSlamConfig(**dict(cfg_items))
    src = make_source(seed, width, height, distorted)
    cal = rig_calibration(src)
    cams = extract_cameras(cal, 2)
    (li, ri), = stereo_pairs(cams)
    rect = stereo_rectify(cams[li], cams[ri])
    frames = src.render_stereo_sequence(n)
    trk = O.OracleTracker(cfg, dict(fx=rect.fx, fy=rect.fy, cx=rect.cx, cy=rect.cy, baseline=rect.baseline,
                                    map_l=rect.map_left, map_r=rect.map_right))
    results = [trk.step(frames[i, 0], frames[i, 1]) for i in range(n)]
    return {"cfg": cfg, "src": src, "rect": rect, "frames": frames, "oracle": results, "cams": cams}


C3_SOURCES = ("192.168.2.21", "192.168.2.22", "192.168.2.23", "192.168.2.25")   # run_slam.py:45-50 CAMERA_MAP


@functools.lru_cache(maxsize=4)
def rig_scene(names: tuple = ("192.168.2.21", "192.168.2.25"), n: int = 6, traj_len: int = 40, width: int = 640,
              height: int = 400):
    """A multi-source rig on the brackets.urdf joints (tests/golden/brackets_joints.json) in one
    shared room: product rectification, base_T_rect-left per pair, and frames [n][C][H][W] in the
    global camera order of isaac_ros.py:138-157 (sorted source names x cam_idx)."""
    import json
    from pathlib import Path

    from thor_slam_amd.camera import Extrinsics
    from thor_slam_amd.synthetic import RoomScene, circle_trajectory

    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    scene = RoomScene(seed=0)
    traj = circle_trajectory(traj_len)
    srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(mats[nm]), seed=k,
                                  width=width, height=height) for k, nm in enumerate(names)]
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(mats[nm])) for nm in names})
    cams = extract_cameras(rig.calibration, 2 * len(names))
    pairs = stereo_pairs(cams)
    rects = [stereo_rectify(cams[l], cams[r]) for l, r in pairs]
    E = [cams[l].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (l, _), r in zip(pairs, rects)]
    by_name = {s.name: s for s in srcs}
    frames = np.stack([np.stack([by_name[cams[l].source_name].render_image(i, c) for l, _ in pairs for c in (0, 1)])
                       for i in range(n)])
    return {"frames": frames, "rects": rects, "E": E, "traj": traj, "cams": cams, "pairs": pairs, "sources": srcs}


def rel_frobenius(a: np.ndarray, b: np.ndarray) -> float:
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


class ScriptedSource:
    """Duck-typed CameraSource with a scripted timestamp schedule (drives both rigs identically)."""

    def __init__(self, name: str, period: float, offset: float, jitter: float, n_cams: int = 2, imu: bool = False, seed: int = 0):
        self._name = name
        self.period, self.offset, self.jitter = period, offset, jitter
        self.n_cams = n_cams
        self.imu = imu
        self.rng = np.random.default_rng(seed)
        self.i = 0
        self.k = np.array([[400.0, 0, 319.5], [0, 400.0, 199.5], [0, 0, 1]])

    @property
    def name(self):
        return self._name

    def start(self):
        pass

    def stop(self):
        pass

    def _ts(self, i):
        return self.offset + i * self.period + float(self.rng.uniform(-self.jitter, self.jitter))

    def get_latest_frames(self):
        from thor_slam_amd.camera.types import CameraFrame

        t = self._ts(self.i)
        self.i += 1
        return [CameraFrame(image=np.zeros((2, 2), np.uint8), timestamp=t + 1e-4 * c, sequence_num=self.i, camera_name=f"{self._name}_{c}")
                for c in range(self.n_cams)]

    def try_get_latest_frames(self):
        return self.get_latest_frames()

    def get_intrinsics(self):
        from thor_slam_amd.camera.types import Intrinsics

        return [Intrinsics(640, 400, self.k.copy(), np.zeros(14)) for _ in range(self.n_cams)]

    def get_extrinsics(self):
        from thor_slam_amd.camera.types import Extrinsics

        out = []
        for c in range(self.n_cams):
            m = np.eye(4)
            m[0, 3] = (-0.0375 if c == 0 else 0.0375) if self.n_cams == 2 else 0.0
            out.append(Extrinsics.from_4x4_matrix(m))
        return out

    def get_sensor_extrinsics(self):
        return None

    def get_timestamped_sensor_data(self):
        if not self.imu:
            return None, None
        t = self.offset + self.i * self.period * 0.5
        return {"accelerometer": np.array([0.0, 9.81, 0.1 * self.i]), "gyroscope": np.array([0.01 * self.i, 0.0, 0.0])}, t

    def try_get_timestamped_sensor_data(self):
        return self.get_timestamped_sensor_data()

    @property
    def has_sensor_data(self):
        return self.imu


def scripted_sources():
    return [
        ScriptedSource("192.168.2.25", 1 / 30, 100.000, 0.004, imu=True, seed=1),
        ScriptedSource("192.168.2.21", 1 / 30, 100.011, 0.004, seed=2),
        ScriptedSource("192.168.2.23", 1 / 15, 100.020, 0.002, seed=3),
    ]


@functools.lru_cache(maxsize=2)
def rgbd_rig_scene(names: tuple = ("192.168.2.21", "192.168.2.22", "192.168.2.23", "192.168.2.25"), n: int = 5,
                   traj_len: int = 40, width: int = 1280, height: int = 720):
    """The 4-camera RGB-D rig of BASELINE.json configs[4] on the brackets.urdf joints: product
    undistortion, base_T_cam per camera and records [n][P][5*H*W] in the global camera order
    (sorted source names; per source the colour camera, its depth aligned)."""
    import json
    from pathlib import Path

    from thor_slam_amd.calib import rgbd_pairs, rgbd_undistort
    from thor_slam_amd.rgbd import pack_rgbd
    from thor_slam_amd.synthetic import synthetic_rgbd_rig

    mats = json.loads((Path(__file__).parent / "golden" / "brackets_joints.json").read_text())
    srcs, rig = synthetic_rgbd_rig(mats, names, width, height, traj_len)
    cams = extract_cameras(rig.calibration, 2 * len(names))
    pairs = rgbd_pairs(cams)
    rects = [rgbd_undistort(cams[c]) for c, _ in pairs]
    E = [cams[c].extrinsics.to_4x4_matrix() @ r.left_optical_T_rect() for (c, _), r in zip(pairs, rects)]
    by_name = {s.name: s for s in srcs}
    raw = [[by_name[cams[c].source_name].render_rgbd(i) for c, _ in pairs] for i in range(n)]
    records = np.stack([np.stack([pack_rgbd(b, d) for b, d in fr]) for fr in raw])
    return {"raw": raw, "records": records, "rects": rects, "E": E, "traj": srcs[0].trajectory,
            "cams": cams, "pairs": pairs, "sources": srcs}


def exact_inertial_record(Ti, vi, Tj, vj, gw, dt, b_true, rng, weights=(1e3, 1e5, 1e4, 1e2, 1e3), b_lin=None):
    """An inertial factor record (oracle/numpy_ba.py INE_N layout) between cameras cam_T_world Ti
    and Tj whose velocity, position and gyro-rotation residuals vanish at velocities vi, vj and the
    biases b_true = (ba, bg) of the earlier keyframe (linearised at b_lin, default 0), with random
    bias Jacobians; weights = (wv, wp, wR, w_ra, w_rg)."""
    from oracle import numpy_ba as B

    b_lin = np.zeros(6) if b_lin is None else np.asarray(b_lin, dtype=np.float64)
    f = np.zeros(B.INE_N)
    Jv, Jp = rng.normal(0, 0.2, (3, 3)) * dt, rng.normal(0, 0.02, (3, 3)) * dt
    Jvg, Jpg = rng.normal(0, 0.2, (3, 3)) * dt, rng.normal(0, 0.02, (3, 3)) * dt
    JRe = -np.eye(3) * dt + rng.normal(0, 0.01, (3, 3)) * dt
    dba, dbg = b_true[0:3] - b_lin[0:3], b_true[3:6] - b_lin[3:6]
    pi, pj = -Ti[:3, :3].T @ Ti[:3, 3], -Tj[:3, :3].T @ Tj[:3, 3]
    f[0:3] = Ti[:3, :3] @ (vj - vi - gw * dt) - Jv @ dba - Jvg @ dbg
    f[3:6] = Ti[:3, :3] @ (pj - pi - vi * dt - 0.5 * gw * dt * dt) - Jp @ dba - Jpg @ dbg
    t = -JRe @ dbg   # the gyro rotation M with vee-asym(M^T Q) = t
    nt = float(np.linalg.norm(t))
    A = B._exp_so3(t / max(nt, 1e-300) * np.arcsin(min(nt, 1.0)))
    M = (Tj[:3, :3] @ Ti[:3, :3].T) @ A.T
    f[6:15], f[15:24], f[24:27], f[27] = Jv.reshape(9), Jp.reshape(9), b_lin[0:3], dt
    f[28], f[29], f[30], f[31], f[71] = weights
    f[32:41], f[41:50], f[50:59], f[59:68], f[68:71] = M.reshape(9), JRe.reshape(9), Jvg.reshape(9), Jpg.reshape(9), b_lin[3:6]
    return f
