"""ctypes binding of ``libtslam_hip.so`` (C-ABI in ``include/tslam.h``).

The library is built in-tree (``make -C thor-slam_amd/csrc`` or ``__graft_entry__.build()``) and
loaded from this package directory.  There is deliberately no fallback: if the HIP library is
missing or fails to load, every engine constructor raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from .params import HipSlamConfig

LIB_NAME = "libtslam_hip.so"
LIB_PATH = Path(__file__).resolve().parent / LIB_NAME

# enum tslam_buffer
BUF = {
    "pyramid": 0, "smooth": 1, "keypoints": 2, "kcount": 3, "desc": 4, "stereo": 5, "disp": 6,
    "temporal": 7, "temporal_uv": 8, "corr": 9, "pose": 10, "stats": 11, "qbest": 12,
    "qsecond": 13, "tbest": 14, "ysorted": 15, "rowstart": 16, "desc_ys": 17, "det_thr": 18, "det_fail": 19,
    "hyp": 20,
}
STAGE = {"rectify": 0, "detect": 1, "describe": 2, "match": 3, "pose": 4, "all": 5, "ba": 6}
# single kernels, in pipeline order (bench.py times each with HIP events)
KERNELS = {
    "rectify_pyramid": 10, "detect": 11, "select": 12, "describe": 13,
    "match": 14, "match_refine": 15, "pose": 16, "chain": 17,
}
INE_RECORD = 80   # TSLAM_BA_INE_RECORD: doubles of an inertial factor record
RIG_KERNEL = 18   # rig pose (+ chain; sharded: the range's rig pose only)
POSE_SOLVE_KERNEL = 19   # P3P + RANSAC + refine on injected correspondences (parity tests)
TRANSPORT = {"rccl": 0, "copy": 1}   # tslam_group_create
SHARD_GATHER, SHARD_RESULTS, SHARD_PROFILE, SHARD_SERIAL, SHARD_PIPELINE, SHARD_SOLO, SHARD_PAIRS = 1, 2, 4, 8, 16, 32, 64   # tslam_shard_options
# tslam_shard_timing segments (enum tslam_segment), in order
SHARD_SEGMENTS = ("rectify_pyramid", "detect", "select", "describe", "pack", "exchange_wait", "import", "match",
                  "match_refine", "pose", "rig", "state", "pose_gather", "chain", "local_ba", "pair_blocks")
POSE_OK, POSE_LOST, POSE_INIT = 0, 1, 2


class StereoDesc(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cx", ctypes.c_double), ("cy", ctypes.c_double),
        ("baseline", ctypes.c_double),
        ("map_left", ctypes.POINTER(ctypes.c_int32)), ("map_right", ctypes.POINTER(ctypes.c_int32)),
    ]


class Params(ctypes.Structure):
    _fields_ = [
        ("n_features", ctypes.c_int32), ("n_levels", ctypes.c_int32), ("fast_threshold", ctypes.c_int32),
        ("edge_margin", ctypes.c_int32), ("max_hamming", ctypes.c_int32), ("ratio_pct", ctypes.c_int32),
        ("stereo_row_tol", ctypes.c_int32), ("max_disparity", ctypes.c_int32), ("temporal_window", ctypes.c_int32),
        ("ransac_hypotheses", ctypes.c_int32), ("refine_iters", ctypes.c_int32), ("min_inliers", ctypes.c_int32),
        ("ransac_thr_px", ctypes.c_double), ("ransac_seed", ctypes.c_uint64),
        ("max_batch", ctypes.c_int32), ("n_pairs", ctypes.c_int32), ("ransac_splits", ctypes.c_int32),
        ("ba_window", ctypes.c_int32), ("ba_kf_interval", ctypes.c_int32), ("ba_iters", ctypes.c_int32),
        ("ba_pad", ctypes.c_int32), ("ba_lambda", ctypes.c_double), ("ba_outlier_px", ctypes.c_double),
        ("rgbd", ctypes.c_int32), ("ransac_mode", ctypes.c_int32),
        ("refine_block", ctypes.c_int32), ("reserved0", ctypes.c_int32),
    ]


class CameraDesc(ctypes.Structure):
    """tslam_camera_desc: one raw camera (camera_info K/D + world extrinsics, isaac_ros.py:364-411)."""
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("K", ctypes.c_double * 9), ("D", ctypes.c_double * 14),
        ("n_coeffs", ctypes.c_int32), ("cam_idx", ctypes.c_int32), ("world_T_cam", ctypes.c_double * 16),
        ("source", ctypes.c_char_p),
    ]


class ImuState(ctypes.Structure):
    """tslam_imu_state: the IMU filter's state (orientation, velocity, biases, variances)."""
    _fields_ = [
        ("R", ctypes.c_double * 9), ("v", ctypes.c_double * 3), ("ba", ctypes.c_double * 3), ("var_v", ctypes.c_double),
        ("var_b", ctypes.c_double), ("bg", ctypes.c_double * 3), ("var_g", ctypes.c_double),
        ("w_prev", ctypes.c_double * 3), ("has_w_prev", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class ImuStep(ctypes.Structure):
    """tslam_imu_step: one frame interval's IMU prediction."""
    _fields_ = [
        ("dt", ctypes.c_double), ("gyro", ctypes.c_double * 3), ("w", ctypes.c_double * 3), ("R_rel", ctypes.c_double * 9),
        ("t_rel", ctypes.c_double * 3), ("w_rot", ctypes.c_double), ("w_trans", ctypes.c_double),
        ("v1", ctypes.c_double * 3), ("var_v1", ctypes.c_double), ("has_v1", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


def camera_desc(cam) -> CameraDesc:
    """A ``CameraConfig`` (intrinsics + world extrinsics) as a ``tslam_camera_desc``."""
    d = CameraDesc()
    intr = cam.intrinsics
    d.width, d.height = int(intr.width), int(intr.height)
    d.K[:] = [float(v) for v in np.asarray(intr.matrix, dtype=np.float64).reshape(9)]
    coeffs = np.asarray(intr.coeffs, dtype=np.float64).flatten()[:14]
    d.D[:len(coeffs)] = [float(v) for v in coeffs]
    d.n_coeffs = len(coeffs)
    d.cam_idx = int(cam.cam_idx)
    d.world_T_cam[:] = [float(v) for v in cam.extrinsics.to_4x4_matrix().reshape(16)]
    d.source = str(cam.source_name).encode()
    return d


_lib: ctypes.CDLL | None = None

# name -> (restype, argtypes); every symbol include/tslam.h declares
_P = ctypes.c_void_p
_SIGNATURES = {
    "tslam_imu_create": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "tslam_imu_destroy": (None, [_P]),
    "tslam_imu_reset": (ctypes.c_int, [_P]),
    "tslam_imu_begin": (ctypes.c_int, [_P, _P]),
    "tslam_imu_ready": (ctypes.c_int, [_P]),
    "tslam_imu_get_state": (ctypes.c_int, [_P, _P]),
    "tslam_imu_set_state": (ctypes.c_int, [_P, _P]),
    "tslam_imu_predict": (ctypes.c_int, [_P, _P, ctypes.c_double, _P, _P, _P]),
    "tslam_imu_coast": (ctypes.c_int, [_P, _P, _P, _P]),
    "tslam_imu_correct": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "tslam_imu_batch_priors": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P]),
    "tslam_imu_absorb": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P, _P]),
    "tslam_imu_vision_only": (ctypes.c_int, [_P, _P, ctypes.c_double, _P, _P, _P]),
    "tslam_imu_gravity": (ctypes.c_int, [_P, _P]),
    "tslam_imu_preintegrate": (ctypes.c_int, [_P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_double,
                                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _P]),
    "tslam_last_error": (ctypes.c_char_p, []),
    "tslam_abi_version": (ctypes.c_int, []),
    "tslam_create": (ctypes.c_int, [ctypes.POINTER(StereoDesc), ctypes.POINTER(Params), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "tslam_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "tslam_submit_sharded": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "tslam_shard_options": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_perturb_temporal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]),
    "tslam_shard_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tslam_create_rig": (ctypes.c_int, [ctypes.POINTER(CameraDesc), ctypes.c_int, ctypes.POINTER(Params), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "tslam_rig_pairs": (ctypes.c_int, [ctypes.POINTER(CameraDesc), ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "tslam_rectify_pair": (ctypes.c_int, [ctypes.POINTER(CameraDesc), ctypes.POINTER(CameraDesc), ctypes.POINTER(StereoDesc),
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_rgbd_undistort": (ctypes.c_int, [ctypes.POINTER(CameraDesc), ctypes.POINTER(StereoDesc), ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "tslam_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "tslam_begin_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tslam_run_stage": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "tslam_end_batch": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_detect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_describe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_match": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_pose": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_read_poses": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4),
    "tslam_reset": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_frames_done": (ctypes.c_int64, [ctypes.c_void_p]),
    "tslam_buffer_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "tslam_copy_out": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]),
    "tslam_copy_in": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]),
    "tslam_ring_slot": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "tslam_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_set_rig": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_set_motion_prior": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tslam_read_rig_poses": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4),
    "tslam_host_stage": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64)]),
    "tslam_submit_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "tslam_poll_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 9
                         + [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]),
    "tslam_poll_pose": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 5),
    "tslam_set_shard": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "tslam_exchange_sizes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "tslam_pack_streams": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_unpack_streams": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_import_raw": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p]),
    "tslam_stage_raw_peers": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_pack_streams_peers": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_import_peers": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_pair_block_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "tslam_pack_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_unpack_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_group_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "tslam_group_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "tslam_group_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "tslam_pack_poses": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_unpack_poses": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_ba_read_map": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_map_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "tslam_relocalize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64] + [ctypes.c_void_p] * 3),
    "tslam_relocalize_rig": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "tslam_ba_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6),
    "tslam_ba_replay_schur": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "tslam_ba_split_solve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_ba_defer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_ba_inertial": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                         ctypes.c_void_p, ctypes.c_double]),
    "tslam_ba_inertial_factor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "tslam_ba_read_inertial": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_ba_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "tslam_loop_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "tslam_loop_add_keyframe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "tslam_loop_read_keyframe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.POINTER(ctypes.c_int)]),
    "tslam_loop_query": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "tslam_loop_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int] + [ctypes.c_void_p] * 3),
    "tslam_tsdf_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double]),
    "tslam_tsdf_integrate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_tsdf_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_tsdf_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_ba_imu_factor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_double]),
    "tslam_tsdf_color": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_tsdf_integrate_rgbd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "tslam_tsdf_read_color": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_tsdf_write_color": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_mesh_read_colors": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "tslam_mesh_extract": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p]),
    "tslam_mesh_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "tslam_esdf_compute": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]),
    "tslam_esdf_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tslam_esdf_slice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_void_p]),
    "tslam_pose_graph": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "tslam_test_potrf_delay": (ctypes.c_int, [ctypes.c_int]),
    "tslam_ba_graph": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_loop_auto": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "tslam_loop_job_vote": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int64)]),
    "tslam_loop_job_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int64)]),
    "tslam_loop_job_pose_graph": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int64)]),
    "tslam_loop_job_poll": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double)]),
}


def load_library(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load (once) and type the HIP library.  Raises ``RuntimeError`` when it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is None and os.environ.get("TSLAM_LIBRARY"):
        path = os.environ["TSLAM_LIBRARY"]  # e.g. an experiment build; still cached as the one library
        p = Path(path)
        lib_is_default = True
    else:
        p = Path(path) if path is not None else LIB_PATH
        lib_is_default = path is None
    # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever loads first
    # is the one HIP runtime of the process; load torch's first so tensors and our kernels share
    # it (loading ours first leaves torch's HSA runtime unable to see the device).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise RuntimeError(
            f"{p} is missing: the MI355X hot path has no CPU fallback. "
            "Build it with `make -C thor-slam_amd/csrc` (or __graft_entry__.build())."
        )
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib_is_default:
        _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)


TSLAM_ESINGULAR = -5


class SingularSystemError(RuntimeError):
    """A pose-graph solve whose normal matrix was not positive definite (TSLAM_ESINGULAR)."""


def _check(rc: int) -> None:
    if rc != 0:
        msg = load_library().tslam_last_error()
        text = f"tslam error {rc}: {msg.decode() if msg else ''}"
        raise SingularSystemError(text) if rc == TSLAM_ESINGULAR else RuntimeError(text)


RANSAC_MODE = {"auto": 0, "exhaustive": 1, "bounded": 2}   # tslam_params.ransac_mode


def make_params(cfg: HipSlamConfig, max_batch: int, n_pairs: int, ransac_splits: int = 0,
                ransac_mode: str = "auto", refine_block: int = 0) -> Params:
    return Params(
        cfg.n_features, cfg.n_levels, cfg.fast_threshold, cfg.edge_margin, cfg.max_hamming, cfg.ratio_pct,
        cfg.stereo_row_tol, cfg.max_disparity, cfg.temporal_window, cfg.ransac_hypotheses, cfg.refine_iters,
        cfg.min_inliers, float(cfg.ransac_thr_px), int(cfg.ransac_seed) & ((1 << 64) - 1), int(max_batch), int(n_pairs),
        int(ransac_splits), int(cfg.ba_window), int(cfg.ba_kf_interval), int(cfg.ba_iters), 0, float(cfg.ba_lambda),
        float(cfg.ba_outlier_px), int(bool(cfg.rgbd)), RANSAC_MODE[ransac_mode], int(refine_block), 0,
    )


def native_rectify_pair(left, right=None, rgbd: bool = False) -> dict:
    """``tslam_rectify_pair`` (``tslam_rgbd_undistort`` with ``rgbd``) on two ``CameraConfig``:
    the library's C++ restatement of ``calib.stereo_rectify`` / ``calib.rgbd_undistort``."""
    lib = load_library()
    dl = camera_desc(left)
    h, w = int(dl.height), int(dl.width)
    desc = StereoDesc()
    ml = np.zeros((h, w, 2), np.int32)
    mr = np.zeros((h, w, 2), np.int32)
    base = np.zeros((4, 4))
    rot = np.zeros((2, 3, 3))
    if rgbd:
        _check(lib.tslam_rgbd_undistort(ctypes.byref(dl), ctypes.byref(desc), ml.ctypes.data, base.ctypes.data))
        mr[...] = ml
        rot[:] = np.eye(3)
    else:
        dr = camera_desc(right)
        _check(lib.tslam_rectify_pair(ctypes.byref(dl), ctypes.byref(dr), ctypes.byref(desc), ml.ctypes.data,
                                      mr.ctypes.data, base.ctypes.data, rot.ctypes.data))
    return {"width": desc.width, "height": desc.height, "fx": desc.fx, "fy": desc.fy, "cx": desc.cx, "cy": desc.cy,
            "baseline": desc.baseline, "map_left": ml, "map_right": mr, "base_T_rect": base,
            "rect_left": rot[0], "rect_right": rot[1]}


def comm_unique_id() -> bytes:
    """``tslam_comm_unique_id``: a fresh RCCL unique id (128 bytes) for ``Handle.comm_init``."""
    buf = (ctypes.c_uint8 * 128)()
    _check(load_library().tslam_comm_unique_id(buf))
    return bytes(buf)


class Handle:
    """Owns one ``tslam_handle`` (one device, ``n_pairs`` stereo pairs, batches <= ``max_batch``)."""

    def __init__(self, rects: list, cfg: HipSlamConfig, max_batch: int = 1, device: int = 0, ransac_splits: int = 0,
                 ransac_mode: str = "auto", refine_block: int = 0):
        self.lib = load_library()
        cfg.validate()
        self.cfg = cfg
        self.n_pairs = len(rects)
        self.cams_per_pair = 1 if cfg.rgbd else 2   # RGB-D: one colour camera (+ aligned depth) per "pair"
        self.n_cams = self.cams_per_pair * self.n_pairs
        self.max_batch = int(max_batch)
        self._maps = []  # keep host maps alive during create
        descs = (StereoDesc * self.n_pairs)()
        for i, r in enumerate(rects):
            ml = None if r.is_identity else np.ascontiguousarray(r.map_left, dtype=np.int32)
            mr = None if r.is_identity else np.ascontiguousarray(r.map_right, dtype=np.int32)
            self._maps += [ml, mr]
            descs[i] = StereoDesc(
                r.width, r.height, r.fx, r.fy, r.cx, r.cy, r.baseline,
                None if ml is None else ml.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                None if mr is None else mr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            )
        params = make_params(cfg, max_batch, self.n_pairs, ransac_splits, ransac_mode, refine_block)
        h = ctypes.c_void_p()
        _check(self.lib.tslam_create(descs, ctypes.byref(params), int(device), ctypes.byref(h)))
        self.h = h
        self._maps = []
        self._read_layout()

    @classmethod
    def from_cameras(cls, cams: list, cfg: HipSlamConfig, max_batch: int = 1, device: int = 0,
                     ransac_splits: int = 0) -> "Handle":
        """``tslam_create_rig``: the handle from raw per-camera calibration (``CameraConfig`` list),
        rectified and paired by the library's C++ host code; multi-pair rigs get ``tslam_set_rig``."""
        self = cls.__new__(cls)
        self.lib = load_library()
        cfg.validate()
        self.cfg = cfg
        descs = (CameraDesc * len(cams))(*[camera_desc(c) for c in cams])
        n_pairs = self.lib.tslam_rig_pairs(descs, len(cams), None, 0)
        _check(min(n_pairs, 0))
        self.n_pairs = n_pairs
        self.cams_per_pair = 1 if cfg.rgbd else 2
        self.n_cams = self.cams_per_pair * n_pairs
        self.max_batch = int(max_batch)
        params = make_params(cfg, max_batch, 0, ransac_splits)
        h = ctypes.c_void_p()
        _check(self.lib.tslam_create_rig(descs, len(cams), ctypes.byref(params), int(device), ctypes.byref(h)))
        self.h = h
        self._read_layout()
        return self

    def _read_layout(self) -> None:
        lay = (ctypes.c_int64 * 16)()
        lev = (ctypes.c_int32 * 18)()
        _check(self.lib.tslam_layout(self.h, lay, lev))
        self.width, self.height = int(lay[0]), int(lay[1])
        self.n_levels, self.K, self.ring, self.batch = int(lay[2]), int(lay[3]), int(lay[4]), int(lay[5])
        self.pyr_bytes = int(lay[7])
        self.pyr_off = [int(lay[8 + l]) for l in range(self.n_levels)]
        self.level_wh = [(int(lev[3 * l]), int(lev[3 * l + 1])) for l in range(self.n_levels)]
        self.quotas = [int(lev[3 * l + 2]) for l in range(self.n_levels)]
        self.koff = [sum(self.quotas[:l]) for l in range(self.n_levels)]

    # -- lifecycle -------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.tslam_destroy(self.h)
            self.h = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:
            pass

    def reset(self) -> None:
        _check(self.lib.tslam_reset(self.h))

    @property
    def frames_done(self) -> int:
        return int(self.lib.tslam_frames_done(self.h))

    # -- execution -------------------------------------------------------------------------
    def submit(self, images_dev_ptr: int, n_frames: int, stream: int = 0) -> None:
        _check(self.lib.tslam_submit(self.h, ctypes.c_void_p(images_dev_ptr), int(n_frames), ctypes.c_void_p(stream)))

    def begin_batch(self, images_dev_ptr: int, n_frames: int) -> None:
        _check(self.lib.tslam_begin_batch(self.h, ctypes.c_void_p(images_dev_ptr), int(n_frames)))

    def run_stage(self, stage: str, stream: int = 0) -> None:
        _check(self.lib.tslam_run_stage(self.h, STAGE[stage], ctypes.c_void_p(stream)))

    def run_kernel(self, name: str, stream: int = 0) -> None:
        _check(self.lib.tslam_run_stage(self.h, KERNELS[name], ctypes.c_void_p(stream)))

    def run_pose_solve(self, stream: int = 0) -> None:
        """``TSLAM_KERNEL_POSE_SOLVE`` (parity tests): P3P + RANSAC + refinement on the
        correspondences and counts already in the ``corr`` / ``stats`` buffers."""
        _check(self.lib.tslam_run_stage(self.h, POSE_SOLVE_KERNEL, ctypes.c_void_p(stream)))

    def perturb_temporal(self, percent: int, seed: int = 11, stream: int = 0) -> None:
        """``tslam_perturb_temporal`` (benchmark hook): outliers into the batch's refined temporal
        positions, between the match_refine and pose kernels."""
        _check(self.lib.tslam_perturb_temporal(self.h, int(percent), int(seed) & ((1 << 64) - 1), ctypes.c_void_p(stream)))

    def run_rig(self, stream: int = 0) -> None:
        _check(self.lib.tslam_run_stage(self.h, RIG_KERNEL, ctypes.c_void_p(stream)))

    def end_batch(self) -> None:
        _check(self.lib.tslam_end_batch(self.h))

    def sync(self) -> None:
        _check(self.lib.tslam_sync(self.h))

    def read_poses(self, n_frames: int) -> dict:
        n = n_frames * self.n_pairs
        t_rel = np.zeros((n, 4, 4))
        t_abs = np.zeros((n, 4, 4))
        cov = np.zeros((n, 6, 6))
        stats = np.zeros((n, 8), dtype=np.int32)
        _check(self.lib.tslam_read_poses(self.h, int(n_frames), t_rel.ctypes.data, t_abs.ctypes.data, cov.ctypes.data,
                                         stats.ctypes.data))
        shape = (n_frames, self.n_pairs)
        return {
            "T_rel": t_rel.reshape(shape + (4, 4)), "T_abs": t_abs.reshape(shape + (4, 4)),
            "cov": cov.reshape(shape + (6, 6)), "stats": stats.reshape(shape + (8,)),
        }

    def set_motion_prior(self, rot: np.ndarray, weight: np.ndarray, trans: np.ndarray | None = None,
                         trans_weight: np.ndarray | None = None) -> None:
        """Motion prior for the next batch: rot [n][P][3][3] (predicted T_rel rotations), weight
        [n][P]; optionally trans [n][P][3] (predicted T_rel translations) and trans_weight [n][P]."""
        rot = np.asarray(rot, dtype=np.float64)
        n = rot.shape[0]
        buf = np.zeros((n, self.n_pairs, 16))
        buf[..., :9] = rot.reshape(n, self.n_pairs, 9)
        buf[..., 9] = np.asarray(weight, dtype=np.float64).reshape(n, self.n_pairs)
        if trans is not None:
            buf[..., 10:13] = np.asarray(trans, dtype=np.float64).reshape(n, self.n_pairs, 3)
            buf[..., 13] = np.asarray(trans_weight, dtype=np.float64).reshape(n, self.n_pairs)
        _check(self.lib.tslam_set_motion_prior(self.h, np.ascontiguousarray(buf).ctypes.data, int(n)))

    def set_rig(self, base_T_rect: list) -> None:
        """Enable the rig pose: base_T_rect-left (4x4) of every pair, in pair order."""
        e = np.ascontiguousarray(np.stack([np.asarray(m, dtype=np.float64) for m in base_T_rect]))
        if e.shape != (self.n_pairs, 4, 4):
            raise ValueError(f"need {self.n_pairs} 4x4 matrices")
        _check(self.lib.tslam_set_rig(self.h, e.ctypes.data))

    def read_rig_poses(self, n_frames: int) -> dict:
        """Body-frame rig motion of the last batch (synchronises)."""
        t_rel = np.zeros((n_frames, 4, 4))
        t_abs = np.zeros((n_frames, 4, 4))
        cov = np.zeros((n_frames, 6, 6))
        stats = np.zeros((n_frames, 8), dtype=np.int32)
        _check(self.lib.tslam_read_rig_poses(self.h, int(n_frames), t_rel.ctypes.data, t_abs.ctypes.data, cov.ctypes.data,
                                             stats.ctypes.data))
        return {"T_rel": t_rel, "T_abs": t_abs, "cov": cov, "stats": stats}

    # -- asynchronous host boundary ------------------------------------------------------------
    def submit_host(self, images: np.ndarray, timestamps=None) -> None:
        """Host frames [n][...] (contiguous u8: [n][2P][H][W] gray or [n][P][5HW] RGB-D) -> the
        device, asynchronously (tslam_submit_host)."""
        images = np.ascontiguousarray(images, dtype=np.uint8)
        n = int(images.shape[0])
        ts = None if timestamps is None else np.ascontiguousarray(timestamps, dtype=np.float64)
        _check(self.lib.tslam_submit_host(self.h, images.ctypes.data, None if ts is None else ts.ctypes.data, n))

    def host_stage(self) -> np.ndarray:
        """The pinned staging buffer of the next submit_host as a [max_batch][frame_bytes] u8 view
        (tslam_host_stage: waits until its previous DMA finished); frames written there and passed
        back to submit_host skip the staging copy."""
        p, fb = ctypes.c_void_p(), ctypes.c_int64()
        _check(self.lib.tslam_host_stage(self.h, ctypes.byref(p), ctypes.byref(fb)))
        key = (p.value, fb.value)
        views = getattr(self, "_stage_views", None)
        if views is None:
            views = self._stage_views = {}
        if key not in views:
            buf = (ctypes.c_uint8 * (self.max_batch * fb.value)).from_address(p.value)
            views[key] = np.frombuffer(buf, dtype=np.uint8).reshape(self.max_batch, fb.value)
        return views[key]

    def _poll_buffers(self) -> tuple:
        """Result arrays of tslam_poll_batch, allocated once with their pointers (a non-blocking poll
        that finds nothing ready costs one C call, no allocation)."""
        if getattr(self, "_pb", None) is None:
            B, P = self.max_batch, self.n_pairs
            arrs = (np.zeros((B, P, 4, 4)), np.zeros((B, P, 4, 4)), np.zeros((B, P, 6, 6)),
                    np.zeros((B, P, 8), dtype=np.int32), np.zeros((B, 4, 4)), np.zeros((B, 4, 4)), np.zeros((B, 6, 6)),
                    np.zeros((B, 8), dtype=np.int32), np.zeros(B))
            g0, n = ctypes.c_int64(), ctypes.c_int()
            self._pb = (arrs, tuple(ctypes.c_void_p(a.ctypes.data) for a in arrs), g0, n, ctypes.byref(g0),
                        ctypes.byref(n))
        return self._pb

    def poll_batch(self, block: bool = False) -> dict | None:
        """Results of the oldest unread submitted batch (copies), or None when none is ready."""
        arrs, ptrs, g0, n, g0_ref, n_ref = self._poll_buffers()
        rc = self.lib.tslam_poll_batch(self.h, int(block), self.max_batch, *ptrs, g0_ref, n_ref)
        if rc < 0:
            _check(rc)
        if rc == 0:
            return None
        k = n.value
        t_rel, t_abs, cov, stats, r_rel, r_abs, r_cov, r_st, ts = (a[:k].copy() for a in arrs)
        out = {"T_rel": t_rel, "T_abs": t_abs, "cov": cov, "stats": stats, "timestamps": ts,
               "first_frame": int(g0.value), "n": k}
        out["rig"] = {"T_rel": r_rel, "T_abs": r_abs, "cov": r_cov, "stats": r_st}
        return out

    def poll_pose(self) -> dict | None:
        """Newest completed pose not returned before (non-blocking), or None."""
        T, cov = np.zeros((4, 4)), np.zeros((6, 6))
        ts, st, conf = ctypes.c_double(), ctypes.c_int32(), ctypes.c_float()
        rc = self.lib.tslam_poll_pose(self.h, T.ctypes.data, cov.ctypes.data, ctypes.addressof(ts), ctypes.addressof(st),
                                      ctypes.addressof(conf))
        if rc < 0:
            _check(rc)
        if rc == 0:
            return None
        return {"T": T, "cov": cov, "timestamp": ts.value, "state": st.value, "confidence": conf.value}

    # -- sharded rig (thor_slam_amd/shard.py drives these) --------------------
    def comm_init(self, unique_id: bytes, rank: int, world: int) -> None:
        """``tslam_comm_init``: join an RCCL communicator and own this rank's shard of the rig."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        _check(self.lib.tslam_comm_init(self.h, buf, int(rank), int(world)))

    def submit_sharded(self, images_dev_ptr: int, n_frames: int | None = None, stream: int = 0) -> None:
        """``tslam_submit_sharded``: one batch (default max_batch frames) of this rank's cameras,
        exchanges over RCCL."""
        n = self.max_batch if n_frames is None else int(n_frames)
        _check(self.lib.tslam_submit_sharded(self.h, ctypes.c_void_p(images_dev_ptr), n, ctypes.c_void_p(stream)))

    def shard_options(self, gather: bool = False, results: bool = False, profile: bool = False,
                      serial: bool = False, pipeline: bool = False, solo: bool = False, pairs: bool = False) -> None:
        """``tslam_shard_options`` of the driver behind this (sharded) handle (``pairs``:
        TSLAM_SHARD_PAIRS, the pair split of a one-camera-per-rank stereo rig)."""
        flags = ((SHARD_GATHER if gather else 0) | (SHARD_RESULTS if results else 0) | (SHARD_PROFILE if profile else 0)
                 | (SHARD_SERIAL if serial else 0) | (SHARD_PIPELINE if pipeline else 0) | (SHARD_SOLO if solo else 0)
                 | (SHARD_PAIRS if pairs else 0))
        _check(self.lib.tslam_shard_options(self.h, flags))

    def shard_timing(self) -> tuple[dict, int]:
        """``tslam_shard_timing``: average µs per batch of every segment of this rank (since the
        last call; synchronises) and the number of batches."""
        out = (ctypes.c_double * len(SHARD_SEGMENTS))()
        nb = self.lib.tslam_shard_timing(self.h, out, len(SHARD_SEGMENTS))
        _check(min(nb, 0))
        return {k: float(v) for k, v in zip(SHARD_SEGMENTS, out)}, int(nb)

    def set_shard(self, cam_lo: int, cam_hi: int, rank: int, world: int) -> None:
        _check(self.lib.tslam_set_shard(self.h, int(cam_lo), int(cam_hi), int(rank), int(world)))

    def exchange_sizes(self) -> tuple[int, int]:
        """(bytes of one stream block, bytes of one pose record)."""
        sb, pr = ctypes.c_int64(), ctypes.c_int64()
        _check(self.lib.tslam_exchange_sizes(self.h, ctypes.byref(sb), ctypes.byref(pr)))
        return int(sb.value), int(pr.value)

    def pack_streams(self, first_frame: int, n_frames: int, cam_lo: int, cam_hi: int, dst_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_pack_streams(self.h, int(first_frame), int(n_frames), int(cam_lo), int(cam_hi),
                                           ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream)))

    def unpack_streams(self, first_frame: int, n_frames: int, cam_lo: int, cam_hi: int, src_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_unpack_streams(self.h, int(first_frame), int(n_frames), int(cam_lo), int(cam_hi),
                                             ctypes.c_void_p(src_ptr), ctypes.c_void_p(stream)))

    def import_raw(self, images_ptr: int, first_frame: int, n_frames: int, cam_lo: int, cam_hi: int, stream: int = 0) -> None:
        _check(self.lib.tslam_import_raw(self.h, ctypes.c_void_p(images_ptr), int(first_frame), int(n_frames), int(cam_lo),
                                         int(cam_hi), ctypes.c_void_p(stream)))

    def stage_raw_peers(self, prev_raw_ptr: int, dst_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_stage_raw_peers(self.h, ctypes.c_void_p(prev_raw_ptr), ctypes.c_void_p(dst_ptr),
                                              ctypes.c_void_p(stream)))

    def pack_streams_peers(self, dst_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_pack_streams_peers(self.h, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream)))

    def import_peers(self, raw_ptr: int, streams_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_import_peers(self.h, ctypes.c_void_p(raw_ptr), ctypes.c_void_p(streams_ptr),
                                           ctypes.c_void_p(stream)))

    def pair_block_bytes(self) -> int:
        """Bytes of one RGB-D pair block (pose, stats, correspondences of one frame and camera)."""
        n = ctypes.c_int64()
        _check(self.lib.tslam_pair_block_bytes(self.h, ctypes.byref(n)))
        return int(n.value)

    def pack_pairs(self, f0: int, n_frames: int, pair_lo: int, pair_hi: int, dst_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_pack_pairs(self.h, int(f0), int(n_frames), int(pair_lo), int(pair_hi),
                                         ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream)))

    def unpack_pairs(self, f0: int, n_frames: int, pair_lo: int, pair_hi: int, src_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_unpack_pairs(self.h, int(f0), int(n_frames), int(pair_lo), int(pair_hi),
                                           ctypes.c_void_p(src_ptr), ctypes.c_void_p(stream)))

    def pack_poses(self, dst_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_pack_poses(self.h, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream)))

    def unpack_poses(self, src_ptr: int, stream: int = 0) -> None:
        _check(self.lib.tslam_unpack_poses(self.h, ctypes.c_void_p(src_ptr), ctypes.c_void_p(stream)))

    # -- buffer access (tests) -------------------------------------------------------------
    def buffer_info(self, which: str) -> tuple[int, int, int]:
        ptr = ctypes.c_void_p()
        tot = ctypes.c_int64()
        per = ctypes.c_int64()
        _check(self.lib.tslam_buffer_info(self.h, BUF[which], ctypes.byref(ptr), ctypes.byref(tot), ctypes.byref(per)))
        return int(ptr.value or 0), int(tot.value), int(per.value)

    def copy_out(self, which: str, offset: int, nbytes: int, dtype) -> np.ndarray:
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        _check(self.lib.tslam_copy_out(self.h, BUF[which], int(offset), out.ctypes.data, int(nbytes)))
        return out

    def copy_in(self, which: str, offset: int, data: np.ndarray) -> None:
        data = np.ascontiguousarray(data)
        _check(self.lib.tslam_copy_in(self.h, BUF[which], int(offset), data.ctypes.data, int(data.nbytes)))

    def ring_slot(self, global_frame: int) -> int:
        return int(self.lib.tslam_ring_slot(self.h, int(global_frame)))

    def frame_block(self, which: str, slot: int, dtype) -> np.ndarray:
        """All bytes of one frame slot of a buffer (ring slot or batch slot, per the layout)."""
        _, _, per = self.buffer_info(which)
        return self.copy_out(which, slot * per, per, dtype)

    def ba_read(self, pair: int = 0) -> dict:
        """A8 keyframe window of one pair (synchronises): slot-indexed frames, cam_T_world,
        landmark ids, landmark positions (by id), observations and the last solve's counts.
        On a rig (``set_rig``, several pairs) ``pair = n_pairs`` reads the body window of the
        rig-level solve: ``T_cw`` is body_T_world per slot, counts are the joint ones."""
        W, K = self.cfg.ba_window, self.K
        frames = np.zeros(W, dtype=np.int64)
        T = np.zeros((W, 4, 4))
        lm = np.zeros((W, K), dtype=np.int32)
        X = np.zeros((W * K, 3))
        uvd = np.zeros((3, W, K))
        cnt = np.zeros(4, dtype=np.int32)
        _check(self.lib.tslam_ba_read(self.h, int(pair), *(a.ctypes.data for a in (frames, T, lm, X, uvd, cnt))))
        return {"frames": frames, "T_cw": T, "lm": lm.astype(np.int64), "X": X, "u": uvd[0], "v": uvd[1],
                "d": uvd[2], "n_obs": int(cnt[0]), "n_lm": int(cnt[1]), "ok": bool(cnt[2])}

    def ba_read_map(self, pair: int = 0) -> dict:
        """Global landmark ids and keyframe-keypoint descriptors of the window (by landmark id)."""
        WK = self.cfg.ba_window * self.K
        gid = np.zeros(WK, dtype=np.int64)
        desc = np.zeros((WK, 8), dtype=np.uint32)
        _check(self.lib.tslam_ba_read_map(self.h, int(pair), gid.ctypes.data, desc.ctypes.data))
        return {"gid": gid, "desc": desc}

    def map_upload(self, xyz: np.ndarray, desc: np.ndarray) -> None:
        """Upload a relocalisation map: world points [n][3] f64 and rBRIEF descriptors [n][8] u32."""
        xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
        desc = np.ascontiguousarray(desc, dtype=np.uint32).reshape(-1, 8)
        if xyz.shape[0] != desc.shape[0]:
            raise ValueError("xyz and desc must have the same number of points")
        _check(self.lib.tslam_map_upload(self.h, xyz.ctypes.data, desc.ctypes.data, int(xyz.shape[0])))

    def relocalize(self, frame: int, pair: int = 0) -> dict:
        """cam_T_world of a resident frame's left camera in the uploaded map (synchronises)."""
        T = np.zeros((4, 4))
        cov = np.zeros((6, 6))
        st = np.zeros(8, dtype=np.int32)
        _check(self.lib.tslam_relocalize(self.h, int(pair), int(frame), T.ctypes.data, cov.ctypes.data, st.ctypes.data))
        return {"T": T, "cov": cov, "stats": st}

    def relocalize_rig(self, frame: int) -> dict:
        """body_T_world of a resident frame of the rig (``set_rig``) in the uploaded map (base-frame
        world points), from every pair's view (synchronises): T, cov, stats (the rig's), and
        pair_stats [P][8]."""
        T, cov = np.zeros((4, 4)), np.zeros((6, 6))
        st, pst = np.zeros(8, dtype=np.int32), np.zeros((self.n_pairs, 8), dtype=np.int32)
        _check(self.lib.tslam_relocalize_rig(self.h, int(frame), T.ctypes.data, cov.ctypes.data, st.ctypes.data,
                                             pst.ctypes.data))
        return {"T": T, "cov": cov, "stats": st, "pair_stats": pst}

    # -- loop closure + pose graph --------------------------------
    def loop_init(self, max_keyframes: int = 1024, signature: int = 256) -> None:
        _check(self.lib.tslam_loop_init(self.h, int(max_keyframes), int(signature)))

    def loop_add_keyframe(self, frame: int, pair: int = 0) -> tuple[int, int]:
        """Store a resident frame's stereo landmarks in the keyframe database -> (entry, landmarks)."""
        slot, n = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.tslam_loop_add_keyframe(self.h, int(pair), int(frame), ctypes.byref(slot), ctypes.byref(n)))
        return int(slot.value), int(n.value)

    def loop_read_keyframe(self, slot: int) -> dict:
        n = ctypes.c_int()
        _check(self.lib.tslam_loop_read_keyframe(self.h, int(slot), None, None, ctypes.byref(n)))
        xyz = np.zeros((max(n.value, 1), 3))
        desc = np.zeros((max(n.value, 1), 8), dtype=np.uint32)
        _check(self.lib.tslam_loop_read_keyframe(self.h, int(slot), xyz.ctypes.data, desc.ctypes.data, ctypes.byref(n)))
        return {"xyz": xyz[:n.value], "desc": desc[:n.value]}

    def loop_query(self, slot: int, n_candidates: int) -> np.ndarray:
        """Place-recognition votes of entry ``slot`` against entries [0, n_candidates)."""
        votes = np.zeros(max(int(n_candidates), 1), dtype=np.int32)
        _check(self.lib.tslam_loop_query(self.h, int(slot), int(n_candidates), votes.ctypes.data))
        return votes[:int(n_candidates)]

    def loop_verify(self, frame: int, slot: int, pair: int = 0) -> dict:
        """cam_q_T_cam_c of a resident frame against a database entry (synchronises)."""
        T = np.zeros((4, 4))
        cov = np.zeros((6, 6))
        st = np.zeros(8, dtype=np.int32)
        _check(self.lib.tslam_loop_verify(self.h, int(pair), int(frame), int(slot), T.ctypes.data, cov.ctypes.data,
                                          st.ctypes.data))
        return {"T": T, "cov": cov, "stats": st}

    # -- asynchronous loop closure (tslam_loop_auto / tslam_loop_job_*) -----------------------
    def loop_auto(self, interval: int) -> None:
        """Keyframes (g % interval == 0) stored by the submit path itself; 0 turns it off."""
        _check(self.lib.tslam_loop_auto(self.h, int(interval)))

    def loop_job_vote(self, query: int, k0: int, n_kf: int) -> "LoopJob":
        job = ctypes.c_int64()
        _check(self.lib.tslam_loop_job_vote(self.h, int(query), int(k0), int(n_kf), ctypes.byref(job)))
        return LoopJob(self, job.value, "vote", n=int(n_kf) * self.n_pairs)

    def loop_job_verify(self, frame: int, query: int, cand: int, pair: int = 0) -> "LoopJob":
        job = ctypes.c_int64()
        _check(self.lib.tslam_loop_job_verify(self.h, int(pair), int(frame), int(query), int(cand), ctypes.byref(job)))
        return LoopJob(self, job.value, "verify")

    def loop_job_pose_graph(self, T: np.ndarray, edges: np.ndarray, meas: np.ndarray, info: np.ndarray,
                            iters: int) -> "LoopJob":
        T = np.ascontiguousarray(np.array(T, dtype=np.float64).reshape(-1, 4, 4))
        edges = np.ascontiguousarray(np.asarray(edges, dtype=np.int32).reshape(-1, 2))
        meas = np.ascontiguousarray(np.asarray(meas, dtype=np.float64).reshape(-1, 4, 4))
        info = np.ascontiguousarray(np.asarray(info, dtype=np.float64).reshape(-1, 6, 6))
        job = ctypes.c_int64()
        _check(self.lib.tslam_loop_job_pose_graph(self.h, int(T.shape[0]), T.ctypes.data, int(edges.shape[0]),
                                                  edges.ctypes.data, meas.ctypes.data, info.ctypes.data, int(iters),
                                                  ctypes.byref(job)))
        return LoopJob(self, job.value, "pose_graph", n=int(T.shape[0]))

    def pose_graph(self, T: np.ndarray, edges: np.ndarray, meas: np.ndarray, info: np.ndarray, iters: int) -> dict:
        """Gauss-Newton on a keyframe pose graph (node 0 fixed) on the device -> poses, cost."""
        T = np.ascontiguousarray(np.array(T, dtype=np.float64).reshape(-1, 4, 4))
        edges = np.ascontiguousarray(np.asarray(edges, dtype=np.int32).reshape(-1, 2))
        meas = np.ascontiguousarray(np.asarray(meas, dtype=np.float64).reshape(-1, 4, 4))
        info = np.ascontiguousarray(np.asarray(info, dtype=np.float64).reshape(-1, 6, 6))
        cost = ctypes.c_double()
        _check(self.lib.tslam_pose_graph(self.h, int(T.shape[0]), T.ctypes.data, int(edges.shape[0]), edges.ctypes.data,
                                         meas.ctypes.data, info.ctypes.data, int(iters), ctypes.byref(cost)))
        return {"T": T, "cost": cost.value}

    # -- RGB-D dense mapping ------------------------------------------
    def tsdf_init(self, origin, dims, voxel_size: float = 0.05, trunc_vox: float = 4.0, max_dist: float = 10.0,
                  max_weight: float = 100.0) -> None:
        o = np.ascontiguousarray(origin, dtype=np.float64).reshape(3)
        d = np.ascontiguousarray(dims, dtype=np.int32).reshape(3)
        self._tsdf_dims = tuple(int(x) for x in d)
        _check(self.lib.tslam_tsdf_init(self.h, o.ctypes.data, d.ctypes.data, float(voxel_size), float(trunc_vox),
                                        float(max_dist), float(max_weight)))

    def tsdf_color(self, enable: bool = True) -> None:
        """The colour layer (call before tsdf_init)."""
        _check(self.lib.tslam_tsdf_color(self.h, int(bool(enable))))
        self._tsdf_color = bool(enable)

    def tsdf_integrate_rgbd(self, color_dev_ptr: int, depth_dev_ptr: int, stride_bytes: int, n_frames: int,
                            first_frame: int = 0, world_T_cam: np.ndarray | None = None, pair: int = 0,
                            stream: int = 0) -> None:
        """Depth + BGR colour of n frames (device, both ``stride_bytes`` apart) into the volume and
        its colour layer, with host poses or the last batch's tracked device poses."""
        poses = None
        if world_T_cam is not None:
            poses = np.ascontiguousarray(np.asarray(world_T_cam, dtype=np.float64).reshape(-1, 4, 4))
        _check(self.lib.tslam_tsdf_integrate_rgbd(self.h, int(pair), ctypes.c_void_p(color_dev_ptr),
                                                  ctypes.c_void_p(depth_dev_ptr), int(stride_bytes), int(n_frames),
                                                  int(first_frame), None if poses is None else poses.ctypes.data,
                                                  ctypes.c_void_p(stream)))

    def tsdf_read_color(self) -> tuple[np.ndarray, np.ndarray]:
        """(colour [nz][ny][nx][3] R, G, B f32, weight [nz][ny][nx] f32) of the colour layer."""
        nx, ny, nz = self._tsdf_dims
        c = np.zeros((nz, ny, nx, 3), dtype=np.float32)
        w = np.zeros((nz, ny, nx), dtype=np.float32)
        _check(self.lib.tslam_tsdf_read_color(self.h, c.ctypes.data, w.ctypes.data))
        return c, w

    def tsdf_write_color(self, color: np.ndarray, weight: np.ndarray) -> None:
        nx, ny, nz = self._tsdf_dims
        c = np.ascontiguousarray(color, dtype=np.float32)
        w = np.ascontiguousarray(weight, dtype=np.float32)
        if c.shape != (nz, ny, nx, 3) or w.shape != (nz, ny, nx):
            raise ValueError(f"colour layer must be {(nz, ny, nx, 3)} / {(nz, ny, nx)}")
        _check(self.lib.tslam_tsdf_write_color(self.h, c.ctypes.data, w.ctypes.data))

    def tsdf_integrate(self, depth_dev_ptr: int, stride_bytes: int, n_frames: int, first_frame: int = 0,
                       world_T_cam: np.ndarray | None = None, pair: int = 0, stream: int = 0) -> None:
        """Integrate n depth frames (device u16 mm, ``stride_bytes`` apart) with host poses
        world_T_cam [n][4][4], or the last batch's tracked device poses when None."""
        poses = None
        if world_T_cam is not None:
            poses = np.ascontiguousarray(np.asarray(world_T_cam, dtype=np.float64).reshape(-1, 4, 4))
        _check(self.lib.tslam_tsdf_integrate(self.h, int(pair), ctypes.c_void_p(depth_dev_ptr), int(stride_bytes),
                                             int(n_frames), int(first_frame),
                                             None if poses is None else poses.ctypes.data, ctypes.c_void_p(stream)))

    def tsdf_read(self) -> tuple[np.ndarray, np.ndarray]:
        """(tsdf, weight) as f32 [nz][ny][nx] (synchronises)."""
        nx, ny, nz = self._tsdf_dims
        t = np.zeros((nz, ny, nx), dtype=np.float32)
        w = np.zeros((nz, ny, nx), dtype=np.float32)
        _check(self.lib.tslam_tsdf_read(self.h, t.ctypes.data, w.ctypes.data))
        return t, w

    def tsdf_write(self, tsdf: np.ndarray, weight: np.ndarray) -> None:
        """Replace the volume (f32 [nz][ny][nx] each; synchronises)."""
        nx, ny, nz = self._tsdf_dims
        t = np.ascontiguousarray(tsdf, dtype=np.float32)
        w = np.ascontiguousarray(weight, dtype=np.float32)
        if t.shape != (nz, ny, nx) or w.shape != (nz, ny, nx):
            raise ValueError(f"volume must be {(nz, ny, nx)}")
        _check(self.lib.tslam_tsdf_write(self.h, t.ctypes.data, w.ctypes.data))

    # -- dense-map outputs (nvblox's mesh / ESDF / distance slice; thor_slam_amd/dense.py) -------
    def mesh(self, min_weight: float = 1e-4, stream: int = 0, colors: bool = False):
        """Marching-cubes triangle soup [n][3][3] f32 (metres), cube order (synchronises); with
        ``colors`` (colour layer) also the vertex colours [n][3][3] f32: (triangles, colours)."""
        n = ctypes.c_int64()
        _check(self.lib.tslam_mesh_extract(self.h, float(min_weight), ctypes.byref(n), ctypes.c_void_p(stream)))
        out = np.zeros((n.value, 3, 3), dtype=np.float32)
        _check(self.lib.tslam_mesh_read(self.h, out.ctypes.data, int(n.value)))
        if not colors:
            return out
        col = np.zeros((n.value, 3, 3), dtype=np.float32)
        if n.value:
            _check(self.lib.tslam_mesh_read_colors(self.h, col.ctypes.data, int(n.value)))
        return out, col

    def esdf(self, max_dist: float = 2.0, site_vox: float = 1.0, min_weight: float = 1e-4, stream: int = 0) -> np.ndarray:
        """Signed distance field f32 [nz][ny][nx] (NaN = unobserved; synchronises)."""
        nx, ny, nz = self._tsdf_dims
        _check(self.lib.tslam_esdf_compute(self.h, float(max_dist), float(site_vox), float(min_weight),
                                           ctypes.c_void_p(stream)))
        out = np.zeros((nz, ny, nx), dtype=np.float32)
        _check(self.lib.tslam_esdf_read(self.h, out.ctypes.data))
        return out

    def esdf_slice(self, y0: int, y1: int, max_dist: float = 2.0, site_vox: float = 1.0,
                   min_weight: float = 1e-4) -> np.ndarray:
        """2-D distance map f32 [nz][nx] over the height band y0 <= j < y1 (NaN = unobserved column)."""
        nx, ny, nz = self._tsdf_dims
        out = np.zeros((nz, nx), dtype=np.float32)
        _check(self.lib.tslam_esdf_slice(self.h, int(y0), int(y1), float(max_dist), float(site_vox), float(min_weight),
                                         out.ctypes.data))
        return out

    def ba_imu_factor(self, frame: int, M: np.ndarray, weight: float, pair: int = 0) -> None:
        """IMU rotation factor of keyframe ``frame`` (the rotation from the previous keyframe's
        camera, 3x3, and its weight) for the local BA window."""
        m = np.ascontiguousarray(M, dtype=np.float64).reshape(9)
        _check(self.lib.tslam_ba_imu_factor(self.h, int(pair), int(frame), m.ctypes.data, float(weight)))

    def ba_replay_schur(self, pair: int = 0, reps: int = 50, stream: int = 0) -> dict:
        """Average k_ba_schur duration (HIP events around ``reps`` replays) and flops per launch."""
        us, fl = ctypes.c_double(), ctypes.c_double()
        _check(self.lib.tslam_ba_replay_schur(self.h, int(pair), int(reps), ctypes.c_void_p(stream), ctypes.byref(us),
                                              ctypes.byref(fl)))
        return {"us": us.value, "flops": fl.value, "reps": int(reps)}

    def ba_inertial(self, gravity, ba_prior, ba_weight: float, bg_prior=None, bg_weight: float = 0.0,
                    pair: int = 0) -> None:
        """World gravity and the priors (value, weight) on the oldest window keyframe's
        accelerometer and gyroscope biases for pair's window (tslam.h)."""
        g = np.ascontiguousarray(gravity, dtype=np.float64).reshape(3)
        b = np.ascontiguousarray(ba_prior, dtype=np.float64).reshape(3)
        bg = np.ascontiguousarray(np.zeros(3) if bg_prior is None else bg_prior, dtype=np.float64).reshape(3)
        _check(self.lib.tslam_ba_inertial(self.h, int(pair), g.ctypes.data, b.ctypes.data, float(ba_weight),
                                          bg.ctypes.data, float(bg_weight)))

    def ba_inertial_factor(self, frame: int, record, v0, pair: int = 0) -> None:
        """Keyframe ``frame``'s inertial factor record (INE_RECORD doubles, oracle INE_N layout) and
        initial velocity, before its batch is submitted."""
        r = np.zeros(INE_RECORD)
        src = np.asarray(record, dtype=np.float64).reshape(-1)[:INE_RECORD]
        r[:src.size] = src
        v = np.ascontiguousarray(v0, dtype=np.float64).reshape(3)
        _check(self.lib.tslam_ba_inertial_factor(self.h, int(pair), int(frame), r.ctypes.data, v.ctypes.data))

    def ba_read_inertial(self, pair: int = 0) -> dict:
        """Velocities [W][3] and accelerometer / gyroscope biases [W][6] by slot (synchronises)."""
        vel = np.zeros((self.cfg.ba_window, 3))
        bias = np.zeros((self.cfg.ba_window, 6))
        _check(self.lib.tslam_ba_read_inertial(self.h, int(pair), vel.ctypes.data, bias.ctypes.data))
        return {"vel": vel, "bias": bias}

    def ba_defer(self, defer: bool) -> None:
        """``tslam_ba_defer``: a BA stage on its own stream is enqueued at the next flush point
        (the next batch's first back stage, or any state read) instead of inside the stage call."""
        _check(self.lib.tslam_ba_defer(self.h, int(bool(defer))))

    def ba_graph(self, enable: bool) -> None:
        """Pair windows' keyframe chains from captured hipGraphs (default) or direct launches (tslam.h)."""
        _check(self.lib.tslam_ba_graph(self.h, int(bool(enable))))

    def ba_split_solve(self, split: bool) -> None:
        """k_ba_reduce + k_ba_solve (kernel boundary) instead of k_ba_reduce_solve (tslam.h)."""
        _check(self.lib.tslam_ba_split_solve(self.h, int(bool(split))))

    def ba_profile(self, max_launches: int = 0) -> dict:
        """Schur-kernel HIP-event time / launches / algorithmic flops since the last call; re-arms
        timing for up to ``max_launches`` launches (0 = off).  Synchronises."""
        ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _check(self.lib.tslam_ba_profile(self.h, int(max_launches), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
        return {"ms": ms.value, "launches": int(n.value), "flops": fl.value}

    # -- decoding helpers (tests / map export) ---------------------------------------------
    def keypoints(self, global_frame: int, cam: int) -> dict:
        """Decoded keypoints of one camera at a global frame (must still be in the ring)."""
        slot = self.ring_slot(global_frame)
        C = self.n_cams
        kp = self.frame_block("keypoints", slot, np.uint32).reshape(C, self.K, 2)[cam]
        cnt = self.frame_block("kcount", slot, np.int32).reshape(C, self.n_levels)[cam]
        desc = self.frame_block("desc", slot, np.uint32).reshape(C, self.K, 8)[cam]
        return {
            "x": (kp[:, 0] & 0xFFFF).astype(np.int64), "y": (kp[:, 0] >> 16).astype(np.int64),
            "level": (kp[:, 1] & 0xFF).astype(np.int64), "angle": ((kp[:, 1] >> 8) & 0xFF).astype(np.int64),
            "score": (kp[:, 1] >> 16).astype(np.int64), "counts": cnt.astype(np.int64), "desc": desc,
        }


class LoopJob:
    """One ``tslam_loop_job_*`` on the handle's loop stream; ``result(block)`` returns its outputs
    once (None while it runs and ``block`` is False)."""

    def __init__(self, handle: Handle, job_id: int, kind: str, n: int = 0):
        self.handle, self.id, self.kind, self.n = handle, int(job_id), kind, int(n)
        self._res = None

    def result(self, block: bool = False):
        if self._res is not None:
            return self._res
        h = self.handle
        if self.kind == "vote":
            votes = np.zeros(max(self.n, 1), dtype=np.int32)
            rc = h.lib.tslam_loop_job_poll(h.h, self.id, int(block), votes.ctypes.data, None, None, None, None, None)
            out = votes[:self.n]
        elif self.kind == "verify":
            T, cov, st = np.zeros((4, 4)), np.zeros((6, 6)), np.zeros(8, dtype=np.int32)
            rc = h.lib.tslam_loop_job_poll(h.h, self.id, int(block), None, T.ctypes.data, cov.ctypes.data, st.ctypes.data,
                                           None, None)
            out = {"T": T, "cov": cov, "stats": st}
        else:
            T, cost = np.zeros((self.n, 4, 4)), ctypes.c_double()
            rc = h.lib.tslam_loop_job_poll(h.h, self.id, int(block), None, None, None, None, T.ctypes.data,
                                           ctypes.byref(cost))
            out = {"T": T, "cost": cost.value}
        if rc < 0:
            _check(rc)
        if rc == 0:
            return None
        self._res = out
        return out


class HandleGroup:
    """``tslam_group_create``: the handles (one per rank, the same rig) driven as one sharded rig
    by the library from this process — an RCCL clique over their devices (``transport="rccl"``,
    one device per handle) or device copies (``"copy"``, ranks may share a device)."""

    def __init__(self, handles: list, transport: str = "rccl"):
        self.lib = load_library()
        self.handles = list(handles)
        arr = (ctypes.c_void_p * len(handles))(*[h.h.value for h in handles])
        g = ctypes.c_void_p()
        _check(self.lib.tslam_group_create(arr, len(handles), TRANSPORT[transport], ctypes.byref(g)))
        self.g = g

    def submit(self, image_ptrs: list[int], n_frames: int | None = None, streams: list[int] | None = None) -> None:
        """One batch of ``n_frames`` (default max_batch; a multiple of the rank count): rank r's
        cameras at device pointer image_ptrs[r] (layout of tslam_submit_sharded)."""
        imgs = (ctypes.c_void_p * len(image_ptrs))(*[int(p) for p in image_ptrs])
        sts = None if streams is None else (ctypes.c_void_p * len(streams))(*[int(s) for s in streams])
        n = self.handles[0].max_batch if n_frames is None else int(n_frames)
        _check(self.lib.tslam_group_submit(self.g, imgs, n, sts))

    def close(self) -> None:
        if getattr(self, "g", None):
            self.lib.tslam_group_destroy(self.g)
            self.g = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:
            pass
