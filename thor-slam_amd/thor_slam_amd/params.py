"""Engine configuration for the MI355X back end.

``HipSlamConfig`` extends the reference ``SlamConfig`` (interface.py:141-165) with the knobs of
the per-frame hot path (SURVEY.md §5 "Config / flags").  Every field has the same meaning in the
NumPy oracle and in the HIP kernels; ``to_c_params`` packs them for the C-ABI
(``include/tslam.h``: ``tslam_params``).
"""

from __future__ import annotations

from dataclasses import dataclass

from .slam.interface import SlamConfig

# Upper bounds baked into the kernels (checked on the host before any launch).
MAX_WIDTH = 2047
MAX_HEIGHT = 2047
MAX_LEVELS = 6
MAX_FEATURES = 8192
MAX_HYPOTHESES = 1024


@dataclass
class HipSlamConfig(SlamConfig):
    # A4 detect
    n_features: int = 2000          # K keypoints per image, split over pyramid levels by area
    n_levels: int = 4               # integer 2x2 box pyramid levels
    fast_threshold: int = 20        # FAST-9: corner iff score > threshold
    edge_margin: int = 19           # keypoints keep this distance from every level border
    # A6 match
    max_hamming: int = 64           # accept best distance <= this
    ratio_pct: int = 80             # accept best*100 < ratio_pct*second
    stereo_row_tol: int = 1         # |y_L - y_R| <= tol (level pixels) after rectification
    max_disparity: int = 128        # level-0 pixels; disparity range [1, max_disparity >> level]
    temporal_window: int = 80       # level-0 pixels; |dx|,|dy| <= window >> level between frames
    # A7 pose
    ransac_hypotheses: int = 128    # P3P minimal samples per frame
    ransac_thr_px: float = 2.0      # reprojection inlier threshold (level-0 pixels)
    ransac_seed: int = 0x5EED
    refine_iters: int = 8           # Gauss-Newton iterations on inliers
    min_inliers: int = 12           # fewer -> frame is LOST
    # A8 local bundle adjustment (config C4); ba_window = 0 disables it
    ba_window: int = 0              # keyframes in the sliding window
    ba_kf_interval: int = 5         # frame g is a keyframe iff g % ba_kf_interval == 0
    ba_iters: int = 5               # Gauss-Newton steps per window solve
    ba_lambda: float = 1.0          # Levenberg damping (px^2 units)
    ba_outlier_px: float = 3.0      # observations farther than this at the start are dropped
    # IMU fusion (thor_slam_amd/imu.py): the bias-corrected gyro rotation as a
    # prior in the pose Gauss-Newton, with a gyroscope-bias state; None = on when the calibration
    # carries the IMU extrinsics (the reference runs cuVSLAM with enable_imu_fusion:=true,
    # Makefile:81; launch/thor_visual_slam.launch.py:69)
    imu_fusion: bool | None = None
    # ... plus the accelerometer leg: velocity / gravity / accelerometer-bias state with the IMU
    # lever arm, a translation prior, and IMU chaining through visual dropouts (None = with
    # imu_fusion)
    imu_accel: bool | None = None
    # ... and, with local BA, the tightly coupled inertial factors: the IMU preintegrated between
    # BA keyframes, a velocity and accelerometer / gyroscope biases per keyframe (tied by the bias
    # random walks) inside the BA (oracle/numpy_ba.py inertial_system); floors of the velocity and
    # position weights' standard deviations (m/s, m)
    ba_inertial: bool = True
    ba_inertial_v_floor: float = 1e-2
    ba_inertial_p_floor: float = 1e-3
    # the record's gyro-rotation rows and the bias random walks between window keyframes (weights
    # from the gyroscope noise density and both random walks of launch/thor_visual_slam.launch.py:
    # 50-53,88-93, floored: rad, m/s^2, rad/s)
    ba_inertial_r_floor: float = 1e-3
    ba_inertial_ba_floor: float = 1e-3
    ba_inertial_bg_floor: float = 1e-3
    # noise model, launch/thor_visual_slam.launch.py:82-93 (calibrated on a 2.5 h rosbag, :97-104)
    gyroscope_noise_density: float = 8.27e-5        # rad/s/sqrt(Hz)   (launch:82)
    accelerometer_noise_density: float = 2.553e-3   # m/s^2/sqrt(Hz)   (launch:85)
    gyroscope_random_walk: float = 1e-8             # rad/s^2/sqrt(Hz) (launch:88)
    accelerometer_random_walk: float = 1.0493e-4    # m/s^3/sqrt(Hz)   (launch:91)
    imu_rot_floor: float = 2e-4     # rad, added in quadrature to the predicted rotation's std (sync, calibration)
    imu_vis_rot_floor: float = 1e-4  # rad, the vision's per-frame rotation error beyond its covariance
    imu_trans_floor: float = 1e-3   # m, added in quadrature to the predicted translation's std
    imu_gyro_bias_sigma: float = 0.01   # rad/s, initial gyroscope-bias std
    imu_accel_bias_sigma: float = 0.05  # m/s^2, initial accelerometer-bias std
    # batches whose vision the prior of the next batch may lack (oracle/numpy_imu.py lagged_priors):
    # the prior of batch s comes from the filter with the vision of batches <= s - 1 - lag absorbed,
    # coasted over the rest, so up to `lag` batches stay in flight; 0 = synchronous (each batch
    # waits for the previous one's vision)
    imu_prior_lag: int = 1
    # loop closure + keyframe pose graph; on when the reference's
    # SlamConfig.enable_loop_closure is (interface.py:155-156; single stereo pair / RGB-D camera)
    loop_kf_interval: int = 5       # frame g is a loop-closure keyframe iff g % loop_kf_interval == 0
    loop_max_keyframes: int = 1024  # keyframe database entries (= pose-graph nodes)
    loop_signature: int = 256       # place-recognition descriptors per keyframe
    loop_min_gap: int = 20          # candidates are at least this many keyframes older
    loop_min_votes: int = 40        # signature votes a candidate needs
    loop_min_inliers: int = 40      # verified RANSAC inliers a loop edge needs
    pg_iters: int = 8               # Gauss-Newton iterations per pose-graph solve
    pg_sigma_t: float = 0.01        # m, std of an edge's translation
    pg_sigma_r: float = 0.005       # rad, std of an edge's rotation
    # asynchronous loop closure (oracle/numpy_loop.py LoopPolicy): the search a keyframe g starts
    # (signature votes, verification, the pose-graph solve of the loop's span) runs on the device
    # beside tracking, and its correction applies from frame g + loop_latency on; 0 = at g itself
    loop_latency: int = 30
    # a verified loop is not closed (no edge, no solve) within this many keyframes after the last
    # closed loop: revisiting a known place would otherwise re-solve the span at every keyframe
    loop_cooldown: int = 5
    # relocalisation after a LOST run (the reference's TrackingState.RELOCALIZING, interface.py:16-23;
    # cuVSLAM's enable_localization_n_mapping, launch/thor_visual_slam.launch.py:42,74): the
    # reloc_after_lost-th consecutive LOST frame breaks the keyframe graph; each tracked keyframe
    # after it searches the keyframes from before the gap (loop-closure votes + verification,
    # due reloc_latency frames later) until one re-anchors the new segment; meanwhile the published
    # pose is None and the state RELOCALIZING (oracle/numpy_loop.py LoopPolicy).  0 = off.  Needs
    # the keyframe database of loop closure.
    reloc_after_lost: int = 3
    reloc_latency: int = 5
    # input kind: RGB-D (BASELINE configs[4]) = per source a colour camera (cam_idx 0, BGR) and a
    # depth image aligned to it (cam_idx 1, u16 mm); depth replaces stereo matching
    rgbd: bool = False
    # RGB-D dense mapping: the depth of pair 0 (the reference maps camera_0
    # only, launch/thor_nvblox.launch.py:50-56) integrated into a dense TSDF volume on the device
    # with the tracked poses; nvblox's parameters and defaults (thor_nvblox.launch.py:26-36)
    dense_map: bool = False
    voxel_size: float = 0.05
    tsdf_integrator_max_integration_distance_m: float = 10.0
    tsdf_integrator_truncation_distance_vox: float = 4.0
    tsdf_max_weight: float = 100.0
    # nvblox's colour layer: the RGB image averaged into the voxels near the surface (mesh colours)
    dense_color: bool = True
    # the volume, axis-aligned in the tracking world (rectified camera of the first frame, RDF:
    # x right, y down, z forward): corner (m) and voxel counts (x, y, z); 10 x 4 x 11 m by default
    tsdf_origin: tuple = (-5.0, -2.0, -1.0)
    tsdf_dims: tuple = (200, 80, 220)
    # dense-map outputs (get_mesh / get_esdf / get_esdf_slice; thor_slam_amd/dense.py): nvblox's
    # mesh / ESDF integrator parameters (its defaults: min weight 1e-4, ESDF max distance 2 m, site
    # distance 1 voxel) and the 2-D slice's height band (y down: metres in the tracking world)
    mesh_integrator_min_weight: float = 1e-4
    esdf_integrator_min_weight: float = 1e-4
    esdf_integrator_max_distance_m: float = 2.0
    esdf_integrator_max_site_distance_vox: float = 1.0
    esdf_slice_min_height: float = -0.5
    esdf_slice_max_height: float = 0.5
    # pipeline
    batch_size: int = 1             # frames per submission
    sync: bool = False              # wait for every batch before process_frames returns (latency mode)
    # one camera stream per GPU from one process (the rig cuVSLAM's multicam mode
    # takes, launch/thor_visual_slam.launch.py:49,81): the rig's cameras sharded over these devices,
    # rank r on devices[r] (empty = the engine's one device, unsharded).  shard_transport "rccl" =
    # an RCCL clique over the devices (one per rank), "copy" = device copies (ranks may share a device)
    devices: tuple = ()
    shard_transport: str = "rccl"

    def validate(self) -> None:
        if not 1 <= self.n_levels <= MAX_LEVELS:
            raise ValueError(f"n_levels must be in [1, {MAX_LEVELS}]")
        if not 1 <= self.n_features <= MAX_FEATURES:
            raise ValueError(f"n_features must be in [1, {MAX_FEATURES}]")
        if not 1 <= self.ransac_hypotheses <= MAX_HYPOTHESES:
            raise ValueError(f"ransac_hypotheses must be in [1, {MAX_HYPOTHESES}]")
        if self.edge_margin < 19:
            raise ValueError("edge_margin must be >= 19 (orientation radius 15, rotated BRIEF radius 19)")
        if not 0 <= self.fast_threshold <= 254:
            raise ValueError("fast_threshold must be in [0, 254]")
        if self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        if self.imu_accel and self.imu_fusion is False:
            raise ValueError("imu_accel needs IMU fusion (imu_fusion True or None)")
        if self.dense_map:
            if not self.rgbd:
                raise ValueError("dense_map needs rgbd=True (depth input)")
            if not (self.voxel_size > 0 and self.tsdf_integrator_max_integration_distance_m > 0
                    and self.tsdf_integrator_truncation_distance_vox > 0 and self.tsdf_max_weight >= 1):
                raise ValueError("voxel_size, integration distance, truncation must be > 0, max weight >= 1")
            if len(self.tsdf_dims) != 3 or min(self.tsdf_dims) < 1 or len(self.tsdf_origin) != 3:
                raise ValueError("tsdf_dims must be 3 positive voxel counts, tsdf_origin 3 coordinates")
        if not (self.ba_window == 0 or 2 <= self.ba_window <= 10):
            raise ValueError("ba_window must be 0 (off) or in [2, 10]")
        if self.ba_kf_interval < 1 or self.ba_iters < 1:
            raise ValueError("ba_kf_interval and ba_iters must be >= 1")
        if not (1 <= self.loop_max_keyframes <= 1024 and 1 <= self.loop_signature <= 256 and self.loop_kf_interval >= 1):
            raise ValueError("loop_max_keyframes must be in [1, 1024], loop_signature in [1, 256], loop_kf_interval >= 1")
        if self.loop_latency < 0 or self.imu_prior_lag < 0 or self.loop_cooldown < 0:
            raise ValueError("loop_latency, loop_cooldown and imu_prior_lag must be >= 0")
        if self.reloc_after_lost < 0 or self.reloc_latency < 0:
            raise ValueError("reloc_after_lost and reloc_latency must be >= 0")
        if self.devices:
            # local BA runs on rank 0 (state gather of a stereo rig); a camera-sharded RGB-D rig keeps
            # the TSDF on rank 0 (pair 0 is rank 0's camera) and has no local BA or loop closure
            if self.rgbd and self.ba_window:
                raise ValueError("a camera-sharded RGB-D rig (devices) runs without local BA")
            if self.shard_transport not in ("rccl", "copy"):
                raise ValueError("shard_transport must be 'rccl' or 'copy'")
        if not 0 <= self.max_hamming <= 253:
            raise ValueError("max_hamming must be in [0, 253] (the mutual check keeps distances as bytes)")


def level_shapes(width: int, height: int, n_levels: int) -> list[tuple[int, int]]:
    """(W_l, H_l) of every pyramid level: W_{l+1} = W_l >> 1, H_{l+1} = H_l >> 1."""
    out = [(width, height)]
    for _ in range(1, n_levels):
        w, h = out[-1]
        out.append((w >> 1, h >> 1))
    return out


def level_quotas(n_features: int, n_levels: int) -> list[int]:
    """Per-level keypoint budget proportional to level area (4^-l); level 0 takes the remainder."""
    total = sum(4.0 ** -l for l in range(n_levels))
    quotas = [int(n_features * (4.0 ** -l) / total) for l in range(n_levels)]
    quotas[0] = n_features - sum(quotas[1:])
    return quotas
