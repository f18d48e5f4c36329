"""Seeded synthetic stereo scenes and a fake ``CameraSource``.

The reference has no recorded dataset and no fake source; every benchmark and test here runs on
frames rendered by this module:

* a closed room (FLU world: x forward, y left, z up; walls at |x|,|y| = ``room_half``, floor and
  ceiling at z = -/+ ``room_height/2``) whose six planes carry seeded multi-octave noise
  textures contrast-stretched to 20..235;
* a body moving at ``speed`` m/s while yawing at ``yaw_rate`` deg/s (a circle around the room
  centre), sampled at ``fps`` timestamps;
* stereo cameras following Luxonis conventions: optical frames are RDF, ``get_extrinsics``
  returns [left_to_center, right_to_center] with the left camera at -baseline/2
  (luxonis.py:675-709), ``K = [[0.6 W, 0, (W-1)/2], [0, 0.6 W, (H-1)/2], [0, 0, 1]]``, 14
  rational-polynomial distortion coefficients (zero unless ``distortion`` is given);
* per-pixel N(0, 2^2) sensor noise, rounded and clipped to u8.

Rendering is plain NumPy (it produces test inputs; it is never on the timed path).
"""

from __future__ import annotations

import threading
from dataclasses import dataclass, field

import numpy as np

from .calib import RDF_TO_FLU_MATRIX, undistort_normalized
from scipy.spatial.transform import Rotation

from .camera.types import CameraFrame, CameraSource, Extrinsics, Intrinsics
from .rgbd import pack_rgbd

TEXTURE_SIZE = 1024
# OAK IMU axes (DRB: x down, y right, z back) -> camera RDF, as in run_slam.py:262-270
DRB_TO_RDF = np.array([[0, 1, 0, 0], [1, 0, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]], dtype=np.float64)
TEXEL_M = 0.01


def make_texture(seed: int, size: int = TEXTURE_SIZE) -> np.ndarray:
    """Multi-octave value noise, 3x3 box smoothed, stretched to [20, 235] (float32)."""
    rng = np.random.default_rng(seed)
    acc = np.zeros((size, size), dtype=np.float64)
    for octave, weight in ((1, 0.35), (2, 0.3), (3, 0.2), (4, 0.15)):
        step = 1 << octave
        n = size // step
        coarse = rng.random((n + 1, n + 1))
        coarse[n, :] = coarse[0, :]
        coarse[:, n] = coarse[:, 0]
        t = np.arange(size, dtype=np.float64) / step
        i0 = np.floor(t).astype(np.int64)
        f = t - i0
        rows = coarse[i0] * (1 - f)[:, None] + coarse[i0 + 1] * f[:, None]
        acc += weight * (rows[:, i0] * (1 - f)[None, :] + rows[:, i0 + 1] * f[None, :])
    pad = np.pad(acc, 1, mode="wrap")
    box = sum(pad[dy : dy + size, dx : dx + size] for dy in range(3) for dx in range(3)) / 9.0
    lo, hi = np.percentile(box, 0.5), np.percentile(box, 99.5)
    out = 20.0 + (np.clip(box, lo, hi) - lo) * (215.0 / (hi - lo))
    return out.astype(np.float32)


@dataclass
class RoomScene:
    seed: int = 0
    room_half: float = 4.0
    room_height: float = 3.0
    textures: list[np.ndarray] = field(default_factory=list)

    def __post_init__(self) -> None:
        if not self.textures:
            self.textures = [make_texture(self.seed * 16 + k) for k in range(6)]

    def render(self, world_T_cam: np.ndarray, intr: Intrinsics, noise_rng: np.random.Generator | None,
               return_depth: bool = False):
        """u8 HxW image seen by a camera whose RDF optical frame is at ``world_T_cam``
        (plus the optical-axis depth map in metres when ``return_depth``)."""
        w, h = intr.width, intr.height
        k = np.asarray(intr.matrix, dtype=np.float64)
        v, u = np.mgrid[0:h, 0:w].astype(np.float64)
        yd = (v - k[1, 2]) / k[1, 1]
        xd = (u - k[0, 2] - k[0, 1] * yd) / k[0, 0]
        coeffs = np.asarray(intr.coeffs, dtype=np.float64)
        if np.any(coeffs != 0):
            xn, yn = undistort_normalized(xd, yd, coeffs)
        else:
            xn, yn = xd, yd
        rays = np.stack([xn, yn, np.ones_like(xn)], axis=-1) @ world_T_cam[:3, :3].T
        origin = world_T_cam[:3, 3]
        bounds = np.array([self.room_half, self.room_half, 0.5 * self.room_height])
        with np.errstate(divide="ignore", invalid="ignore"):
            tb = np.where(rays > 0, (bounds - origin) / rays, (-bounds - origin) / rays)
        tb = np.where(np.isfinite(tb) & (tb > 0), tb, np.inf)
        axis = np.argmin(tb, axis=-1)
        t = np.take_along_axis(tb, axis[..., None], axis=-1)[..., 0]
        hit = origin + rays * t[..., None]
        positive = np.take_along_axis(rays, axis[..., None], axis=-1)[..., 0] > 0
        plane = axis * 2 + positive.astype(np.int64)
        # texture coordinates: the two in-plane axes
        a_idx = np.where(axis == 0, 1, 0)
        b_idx = np.where(axis == 2, 1, 2)
        ta = np.take_along_axis(hit, a_idx[..., None], axis=-1)[..., 0] / TEXEL_M
        tbb = np.take_along_axis(hit, b_idx[..., None], axis=-1)[..., 0] / TEXEL_M
        img = np.zeros((h, w), dtype=np.float64)
        for p in range(6):
            m = plane == p
            if np.any(m):
                img[m] = _bilinear_wrap(self.textures[p], ta[m], tbb[m])
        if noise_rng is not None:
            img += noise_rng.normal(0.0, 2.0, size=img.shape)
        out = np.clip(np.floor(img + 0.5), 0, 255).astype(np.uint8)
        if return_depth:
            return out, t  # rays have unit optical-axis component, so t is the z depth
        return out


def _bilinear_wrap(tex: np.ndarray, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    n = tex.shape[0]
    a0 = np.floor(a)
    b0 = np.floor(b)
    fa = a - a0
    fb = b - b0
    ia = a0.astype(np.int64) % n
    ib = b0.astype(np.int64) % n
    ia1 = (ia + 1) % n
    ib1 = (ib + 1) % n
    top = tex[ib, ia] * (1 - fa) + tex[ib, ia1] * fa
    bot = tex[ib1, ia] * (1 - fa) + tex[ib1, ia1] * fa
    return top * (1 - fb) + bot * fb


def circle_trajectory(n: int, fps: float = 30.0, speed: float = 0.5, yaw_rate_deg: float = 10.0,
                      pitch_amp_deg: float = 1.5, z0: float = 0.0) -> np.ndarray:
    """(n, 4, 4) world_T_body (FLU) poses on a circle around the room centre."""
    om = np.deg2rad(yaw_rate_deg)
    radius = speed / om
    out = np.zeros((n, 4, 4))
    for i in range(n):
        t = i / fps
        psi = om * t
        pitch = np.deg2rad(pitch_amp_deg) * np.sin(2 * np.pi * 0.25 * t)
        cz, sz = np.cos(psi), np.sin(psi)
        cp, sp = np.cos(pitch), np.sin(pitch)
        rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
        ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
        out[i] = np.eye(4)
        out[i, :3, :3] = rz @ ry
        # forward speed along the body heading: circle centred at the origin
        out[i, :3, 3] = [radius * np.sin(psi), radius * (1 - np.cos(psi)) - radius, z0]
    return out


def default_intrinsics(width: int = 640, height: int = 400, distortion: np.ndarray | None = None) -> Intrinsics:
    f = 0.6 * width
    k = np.array([[f, 0.0, (width - 1) / 2.0], [0.0, f, (height - 1) / 2.0], [0.0, 0.0, 1.0]])
    coeffs = np.zeros(14)
    if distortion is not None:
        d = np.asarray(distortion, dtype=np.float64).flatten()
        coeffs[: d.size] = d
    return Intrinsics(width=width, height=height, matrix=k, coeffs=coeffs)


class SyntheticStereoSource(CameraSource):
    """Renders [left, right] frames of a ``RoomScene`` along a trajectory (one source of a rig).

    ``rig_T_source`` is only used for rendering (where the source sits on the body); the
    calibration the engine sees comes from ``get_extrinsics`` + the rig's ``rig_extrinsics``,
    exactly like a real Luxonis source.
    """

    def __init__(
        self,
        name: str = "192.168.2.21",
        scene: RoomScene | None = None,
        trajectory: np.ndarray | None = None,
        width: int = 640,
        height: int = 400,
        baseline: float = 0.075,
        fps: float = 30.0,
        rig_T_source: np.ndarray | None = None,
        distortion: np.ndarray | None = None,
        seed: int = 0,
        t0: float = 1000.0,
        jitter_s: float = 0.0,
        n_frames: int = 100,
        imu: bool = False,
        gyro_noise: float = 0.0,
        accel_noise: float = 0.0,
        blackout: tuple[int, int] | None = None,
        gyro_bias: np.ndarray | None = None,
    ) -> None:
        self._name = name
        self.scene = scene or RoomScene(seed=seed)
        self.trajectory = trajectory if trajectory is not None else circle_trajectory(n_frames, fps)
        self.width, self.height = width, height
        self.baseline = baseline
        self.fps = fps
        self.rig_T_source = RDF_TO_FLU_MATRIX.copy() if rig_T_source is None else np.asarray(rig_T_source)
        self.seed = seed
        self.t0 = t0
        self.jitter_s = jitter_s
        self._intr = [default_intrinsics(width, height, distortion), default_intrinsics(width, height, distortion)]
        self._extr = []
        for sx in (-0.5, 0.5):
            m = np.eye(4)
            m[0, 3] = sx * baseline
            self._extr.append(Extrinsics.from_4x4_matrix(m))
        self.imu = imu
        self.gyro_noise = gyro_noise
        self.accel_noise = accel_noise
        self.gyro_bias = np.zeros(3) if gyro_bias is None else np.asarray(gyro_bias, dtype=np.float64).reshape(3)
        self.blackout = blackout   # frames [a, b) render as a uniform grey (a visual dropout)
        self._index = 0
        self._running = False
        self._lock = threading.Lock()

    # -- CameraSource API ------------------------------------------------------------
    @property
    def name(self) -> str:
        return self._name

    def start(self) -> None:
        self._running = True

    def stop(self) -> None:
        self._running = False

    def get_intrinsics(self) -> list[Intrinsics]:
        return list(self._intr)

    def get_extrinsics(self) -> list[Extrinsics]:
        return list(self._extr)

    def get_sensor_extrinsics(self) -> Extrinsics | None:
        """IMU -> source: the IMU sits at the source origin, axes in the OAK's DRB convention
        (the chain of run_slam.py:252-283 turns it into RDF with DRB_TO_RDF)."""
        return Extrinsics.from_4x4_matrix(np.eye(4)) if self.imu else None

    def imu_position(self, i: int) -> np.ndarray:
        """World position of the IMU (the source origin) at frame i."""
        return (self.trajectory[i % len(self.trajectory)] @ self.rig_T_source)[:3, 3]

    def imu_sample(self, i: int) -> dict:
        """The sample of the interval (i-1, i]: gyro = the source's rotation from frame i-1 to i over
        the frame interval (DRB axes) + gyro_bias + N(0, gyro_noise^2); accelerometer = the specific force
        R^T (a - g) in the IMU axes of frame i-1, with the world acceleration a the second
        difference of the IMU positions around frame i-1 (so p_i = p_{i-1} + v dt + a dt^2 / 2
        holds for the central-difference velocity v) and g = (0, 0, -9.81) (the renderer's world is
        z-up) + N(0, accel_noise^2).  A dict with the IMUData fields, the form the reference's rig
        carries (luxonis.py:1155-1158 casts to dict and indexes ["timestamp"]; its IMUData class has
        no constructor)."""
        dt = 1.0 / self.fps
        r0 = self.camera_pose(max(i - 1, 0), 0)[:3, :3]
        r1 = self.camera_pose(i, 0)[:3, :3]
        w_rdf = Rotation.from_matrix(r0.T @ r1).as_rotvec() / dt
        d = DRB_TO_RDF[:3, :3]
        w = d.T @ w_rdf + self.gyro_bias
        if self.gyro_noise:
            w = w + np.random.default_rng((self.seed, i, 99)).normal(0.0, self.gyro_noise, 3)
        if i == 0:
            a_w = np.zeros(3)   # the sequence starts at rest (the filter's gravity alignment)
        else:
            k = max(i - 1, 1)
            a_w = (self.imu_position(k + 1) - 2.0 * self.imu_position(k) + self.imu_position(k - 1)) / dt ** 2
        acc = d.T @ (r0.T @ (a_w + np.array([0.0, 0.0, 9.81])))
        if self.accel_noise:
            acc = acc + np.random.default_rng((self.seed, i, 98)).normal(0.0, self.accel_noise, 3)
        return {"accelerometer": acc, "gyroscope": w, "timestamp": self.timestamp(i), "sequence_num": i}

    def get_timestamped_sensor_data(self) -> tuple[dict | None, float | None]:
        if not self.imu:
            return None, None
        s = self.imu_sample(self._index)
        return s, s["timestamp"]

    def try_get_timestamped_sensor_data(self) -> tuple[dict | None, float | None]:
        return self.get_timestamped_sensor_data()

    @property
    def has_sensor_data(self) -> bool:
        return self.imu

    def get_latest_frames(self) -> list[CameraFrame]:
        if not self._running:
            raise RuntimeError("Camera source not started. Call start() first.")
        with self._lock:
            i = self._index
            self._index += 1
        return self.render_frames(i)

    def try_get_latest_frames(self) -> list[CameraFrame] | None:
        if not self._running:
            return None
        return self.get_latest_frames()

    # -- rendering -------------------------------------------------------------------
    def timestamp(self, i: int) -> float:
        jit = 0.0
        if self.jitter_s:
            jit = float(np.random.default_rng((self.seed, i, 7)).uniform(-self.jitter_s, self.jitter_s))
        return self.t0 + i / self.fps + jit

    def camera_pose(self, i: int, cam: int) -> np.ndarray:
        """world_T_cam (RDF optical frame) of camera ``cam`` at frame ``i``."""
        body = self.trajectory[i % len(self.trajectory)]
        return body @ self.rig_T_source @ self._extr[cam].to_4x4_matrix()

    def render_image(self, i: int, cam: int) -> np.ndarray:
        if self.blackout is not None and self.blackout[0] <= i < self.blackout[1]:
            return np.full((self.height, self.width), 128, dtype=np.uint8)
        rng = np.random.default_rng((self.seed, i, cam))
        return self.scene.render(self.camera_pose(i, cam), self._intr[cam], rng)

    def render_frames(self, i: int) -> list[CameraFrame]:
        ts = self.timestamp(i)
        return [
            CameraFrame(image=self.render_image(i, c), timestamp=ts, sequence_num=i, camera_name=f"{self._name}_{side}")
            for c, side in ((0, "left"), (1, "right"))
        ]

    def render_stereo_sequence(self, n: int, start: int = 0) -> np.ndarray:
        """(n, 2, H, W) u8 stack of frames start..start+n-1."""
        out = np.empty((n, 2, self.height, self.width), dtype=np.uint8)
        for k in range(n):
            for c in range(2):
                out[k, c] = self.render_image(start + k, c)
        return out

    def ground_truth_body(self, i: int) -> np.ndarray:
        return self.trajectory[i % len(self.trajectory)]


def synthetic_rig(joints: dict, names: list[str] | tuple[str, ...], width: int = 640, height: int = 400,
                  traj_len: int = 40, scene_seed: int = 0):
    """Stereo sources mounted on a rig's joints (``joints[name]`` = rig_T_source 4x4, e.g. the
    brackets.urdf joints of ``scripts/run_slam.py:45-50``'s CAMERA_MAP) in one shared room along
    one body trajectory -> (sources, CameraRig with those rig extrinsics)."""
    from .camera.rig import CameraRig

    scene = RoomScene(seed=scene_seed)
    traj = circle_trajectory(traj_len)
    srcs = [SyntheticStereoSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(joints[nm]), seed=k,
                                  width=width, height=height) for k, nm in enumerate(names)]
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(joints[nm])) for nm in names})
    return srcs, rig


class CachedStereoSource(SyntheticStereoSource):
    """A ``SyntheticStereoSource`` whose frames come from a pre-rendered cycle: frame i is
    ``frames[i % len(frames)]`` ([n][2][H][W] u8) — a trajectory that repeats with that period
    (``circle_trajectory`` of one full turn) replays without rendering, IMU samples included."""

    def __init__(self, frames: np.ndarray, **kw) -> None:
        super().__init__(**kw)
        self.frames = frames

    def render_image(self, i: int, cam: int) -> np.ndarray:
        return self.frames[i % len(self.frames), cam]


class SyntheticRGBDSource(SyntheticStereoSource):
    """An RGB-D source (BASELINE configs[4]): frames are [colour BGR u8, depth u16 mm] from one
    camera, the depth aligned to the colour image (same K and D, as Luxonis ``depth_align_to_rgb``,
    luxonis.py:1018-1030; frame order of ``get_latest_rgbd_frames``, :876-919).  Colour = the room
    texture through fixed channel gains; depth = the optical-axis distance in mm (0 beyond 65.535 m)."""

    def __init__(self, name: str = "192.168.2.21", width: int = 1280, height: int = 720, **kw) -> None:
        super().__init__(name=name, width=width, height=height, **kw)
        self._extr = [Extrinsics.from_4x4_matrix(np.eye(4)), Extrinsics.from_4x4_matrix(np.eye(4))]

    def render_rgbd(self, i: int) -> tuple[np.ndarray, np.ndarray]:
        rng = np.random.default_rng((self.seed, i, 0))
        g, z = self.scene.render(self.camera_pose(i, 0), self._intr[0], rng, return_depth=True)
        gf = g.astype(np.float64)
        bgr = np.stack([np.clip(np.floor(0.8 * gf + 30.5), 0, 255), gf, np.clip(np.floor(1.1 * gf - 9.5), 0, 255)],
                       axis=-1).astype(np.uint8)
        mm = np.floor(z * 1000.0 + 0.5)
        depth = np.where((mm > 0) & (mm <= 65535), mm, 0).astype(np.uint16)
        return bgr, depth

    def render_frames(self, i: int) -> list[CameraFrame]:
        ts = self.timestamp(i)
        bgr, depth = self.render_rgbd(i)
        return [CameraFrame(image=bgr, timestamp=ts, sequence_num=i, camera_name=f"{self._name}_rgb"),
                CameraFrame(image=depth, timestamp=ts, sequence_num=i, camera_name=f"{self._name}_depth")]

    def render_rgbd_sequence(self, n: int, start: int = 0) -> np.ndarray:
        """(n, 5*H*W) u8 device records: [BGR H*W*3 | depth u16 H*W little-endian] per frame."""
        out = np.empty((n, 5 * self.height * self.width), dtype=np.uint8)
        for k in range(n):
            out[k] = pack_rgbd(*self.render_rgbd(start + k))
        return out



def synthetic_rgbd_rig(joints: dict, names: list[str] | tuple[str, ...], width: int = 1280, height: int = 720,
                       traj_len: int = 40, scene_seed: int = 0):
    """RGB-D sources (colour + aligned depth at the source origin) on a rig's joints in one shared
    room along one body trajectory (the 4-camera nvblox-shaped rig of BASELINE.json configs[4],
    scripts/run_pipeline.py:218-256) -> (sources, CameraRig with those rig extrinsics)."""
    from .camera.rig import CameraRig

    scene = RoomScene(seed=scene_seed)
    traj = circle_trajectory(traj_len)
    srcs = [SyntheticRGBDSource(name=nm, scene=scene, trajectory=traj, rig_T_source=np.array(joints[nm]), seed=k,
                                width=width, height=height) for k, nm in enumerate(names)]
    rig = CameraRig(srcs, rig_extrinsics={nm: Extrinsics.from_4x4_matrix(np.array(joints[nm])) for nm in names})
    return srcs, rig
