/*
 * tslam.h — C-ABI of libtslam_hip.so, the MI355X (gfx950) hot path of the thor-slam back end.
 *
 * The reference has no FFI for this path: its hot path is a separate closed process (cuVSLAM)
 * fed over ROS 2 topics by IsaacRosAdapter (thor_slam/slam/adapters/isaac_ros.py:327-430).
 * Each entry point below replaces one piece of that hop, and is bound from Python with ctypes by
 * thor_slam_amd/_lib.py (INTEGRATION.md shows the binding):
 *
 *   tslam_create        <- IsaacRosAdapter.initialize          isaac_ros.py:85-136 (publishers,
 *                          camera_info K/D/P per camera :364-411) — here: rectification tables,
 *                          rectified K and baseline of each stereo pair, device workspace
 *   tslam_submit        <- the per-camera image publish loop   isaac_ros.py:336-413 — here: one
 *                          batch of frames already in HBM, rectify -> detect -> describe ->
 *                          match -> pose on the caller's stream
 *   tslam_read_poses    <- IsaacRosAdapter._odom_cb            isaac_ros.py:308-325 (odometry +
 *                          covariance) — here: per-frame relative/absolute poses, 6x6 covariance
 *   tslam_reset         <- IsaacRosAdapter.reset               isaac_ros.py:438-442
 *   tslam_destroy       <- IsaacRosAdapter.shutdown            isaac_ros.py:444-450
 *   tslam_run_stage     stage-level entry points for parity tests (tslam_detect /
 *                          describe / match / pose); tslam_detect ... tslam_pose are aliases
 *   tslam_ba_read       <- the map/keyframe side of cuVSLAM (SlamEngine.get_map, interface.py:207) —
 *                          here: the A8 sliding keyframe window (poses, landmarks) of a pair
 *   tslam_set_shard ... one camera stream per GPU: the blocks a sharded rig
 *                          exchanges over RCCL (stream blocks, raw images, pair blocks, pose records)
 *   tslam_comm_init,    <- cuVSLAM's multicam mode (launch/thor_visual_slam.launch.py:49,81) for a
 *   tslam_group_create     rig spread over GPUs: the library's own driver of the sharded rig, one
 *                          process per GPU (RCCL) or one process for all of them (RCCL clique)
 *
 * Conventions: every function returns 0 on success or a negative TSLAM_E* code;
 * tslam_last_error() returns a thread-local message for the last failure.  A handle is not
 * thread-safe (one submitting thread per handle).  All device pointers are HIP device memory
 * on the handle's device; `stream` is a hipStream_t (NULL = default stream).  No function takes
 * or returns framework (torch) types.
 */
#ifndef TSLAM_H
#define TSLAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSLAM_ABI_VERSION 20

#define TSLAM_OK 0
#define TSLAM_EINVAL (-1)
#define TSLAM_EHIP (-2)
#define TSLAM_ENOMEM (-3)
#define TSLAM_ESTATE (-4)
#define TSLAM_ESINGULAR (-5)   /* a pose-graph solve whose normal matrix is not positive definite */

/* pose status per frame (tslam_read_poses stats[4*i + 0]) */
#define TSLAM_POSE_OK 0
#define TSLAM_POSE_LOST 1
#define TSLAM_POSE_INIT 2

typedef struct tslam_handle tslam_handle;

/* One rectified stereo pair (A1/A2 of SURVEY.md §8a). */
typedef struct {
    int32_t width, height;        /* raw == rectified image size, <= 2047 x 2047           */
    double fx, fy, cx, cy;        /* rectified intrinsics shared by both cameras              */
    double baseline;              /* metres, > 0                                              */
    const int32_t* map_left;      /* host (H*W*2) int32 source (x, y) in 1/32 px, or NULL =   */
    const int32_t* map_right;     /*   identity; copied to device at create                   */
} tslam_stereo_desc;

typedef struct {
    int32_t n_features;           /* K per image                                              */
    int32_t n_levels;             /* pyramid levels (1..6)                                    */
    int32_t fast_threshold;       /* corner iff FAST score > threshold                        */
    int32_t edge_margin;          /* >= 19                                                    */
    int32_t max_hamming;          /* A6 acceptance                                            */
    int32_t ratio_pct;
    int32_t stereo_row_tol;
    int32_t max_disparity;        /* level-0 px                                               */
    int32_t temporal_window;      /* level-0 px                                               */
    int32_t ransac_hypotheses;    /* <= 1024                                                  */
    int32_t refine_iters;
    int32_t min_inliers;
    double ransac_thr_px;
    uint64_t ransac_seed;
    int32_t max_batch;            /* frames per tslam_submit                                  */
    int32_t n_pairs;              /* stereo pairs per frame (cameras = 2 * n_pairs)           */
    int32_t ransac_splits;        /* RANSAC blocks per frame (0 = auto); never changes results */
    /* A8 local bundle adjustment (0 = off): keyframe window, frames between keyframes,
     * Gauss-Newton steps per solve, Levenberg damping, initial outlier gate (px) */
    int32_t ba_window;            /* keyframes in the sliding window (0 or 2..10)            */
    int32_t ba_kf_interval;       /* frame g is a keyframe iff g % ba_kf_interval == 0        */
    int32_t ba_iters;
    int32_t ba_pad;               /* reserved, 0                                              */
    double ba_lambda;
    double ba_outlier_px;
    /* RGB-D input (BASELINE configs[4]): each "pair" is one colour camera with a depth image
     * aligned to it; per frame and camera the submitted record is [BGR u8 H*W*3 | depth u16 mm
     * H*W] (images = [n][n_pairs][5*H*W] bytes; W*H even).  tslam_stereo_desc gives the colour
     * camera (baseline ignored, map_right unused); the stereo stage becomes a depth lookup. */
    int32_t rgbd;
    int32_t ransac_mode;          /* RANSAC scoring: 0 auto (bounded from 256 frames per launch),
                                     1 exhaustive, 2 bounded; never changes results             */
    int32_t refine_block;         /* k_refine threads per frame: 0 auto (128 from 512 frames per
                                     launch), 128 or 256; never changes results                  */
    int32_t reserved0;            /* 0                                                        */
} tslam_params;

/* One raw camera as IsaacRosAdapter publishes it (camera_info K/D + the rig extrinsics,
 * isaac_ros.py:364-411; CameraConfig of thor_slam/slam/interface.py).  Input of tslam_create_rig. */
typedef struct {
    int32_t width, height;        /* image size                                               */
    double K[9];                  /* camera matrix, row-major (camera_info.k)                  */
    double D[14];                 /* distortion coefficients (camera_info.d), n_coeffs valid;  */
    int32_t n_coeffs;             /*   >= 8 rational_polynomial[:8], 5 plumb_bob, 4 equidistant, else plumb_bob
                                       zero-padded (isaac_ros.py:370-383)                       */
    int32_t cam_idx;              /* index within its source: 0 = left / colour, 1 = right / depth */
    double world_T_cam[16];       /* RigCalibration.get_world_extrinsics (rig.py:35-70), row-major,
                                     optical (RDF) camera frame in the rig's base frame          */
    const char* source;           /* source name (NULL = "")                                   */
} tslam_camera_desc;

/* Buffers exposed for parity tests (tslam_buffer_info / tslam_copy_out / tslam_copy_in). */
enum tslam_buffer {
    TSLAM_BUF_PYRAMID = 0,   /* u8  [ring][cams][pyr_bytes]      rectified levels             */
    TSLAM_BUF_SMOOTH = 1,    /* u8  [batch][cams][pyr_bytes]     5x5 binomial per level       */
    TSLAM_BUF_KEYPOINTS = 2, /* u32 [ring][cams][K][2]           {x | y<<16, lvl | ang<<8 | score<<16} */
    TSLAM_BUF_KCOUNT = 3,    /* i32 [ring][cams][levels]                                      */
    TSLAM_BUF_DESC = 4,      /* u32 [ring][cams][K][8]                                        */
    TSLAM_BUF_STEREO = 5,    /* i32 [ring][pairs][K]             right index or -1            */
    TSLAM_BUF_DISP = 6,      /* f64 [ring][pairs][K]             refined level-0 disparity/NaN */
    TSLAM_BUF_TEMPORAL = 7,  /* i32 [ring][pairs][K]             left(t-1) index or -1        */
    TSLAM_BUF_TEMPORAL_UV = 8, /* f64 [batch][pairs][K][2]       refined (u, v) at t / NaN    */
    TSLAM_BUF_CORR = 9,      /* f64 [batch][pairs][K][8]         X Y Z du dv bx by bz         */
    TSLAM_BUF_POSE = 10,     /* f64 [batch][pairs][68]           T_rel[16] T_abs[16] cov[36]  */
    TSLAM_BUF_STATS = 11,    /* i32 [batch][pairs][8]            status n_corr n_inl best ... */
    TSLAM_BUF_QBEST = 12,    /* u32 [batch][pairs][2][K]         (dist<<16 | idx) stereo, temporal */
    TSLAM_BUF_QSECOND = 13,  /* u32 [batch][pairs][2][K]                                      */
    TSLAM_BUF_TBEST = 14,    /* u32 [batch][pairs][2][K]         train-side atomicMin         */
    TSLAM_BUF_YSORTED = 15,  /* u32 [ring][cams][K][4]           per level, by (y, rank): {x | y<<16, lvl | score<<16, kp index, valid} */
    TSLAM_BUF_ROWSTART = 16, /* u16 [ring][cams][sum(H_l+1)]     per level: first y-sorted position of row y */
    TSLAM_BUF_DESC_YS = 17,  /* u32 [ring][cams][K][8]           descriptors in the y-sorted order */
    TSLAM_BUF_DET_THR = 18,  /* u32 [1][cams][levels]            speculative FAST threshold te in use (0 = t + 1) */
    TSLAM_BUF_DET_FAIL = 19, /* u32 [batch][cams][levels]        1 = the last batch's image-level took the fallback */
    TSLAM_BUF_HYP = 20,      /* f64 [batch][pairs][n_hyp][4][20] P3P candidates of each RANSAC hypothesis, by
                                ascending root: R[9] t[3] (f64; R[0] NaN = no solution), then f32 copies */
    TSLAM_BUF_COUNT = 21
};

enum tslam_stage {
    TSLAM_STAGE_RECTIFY = 0, /* raw -> pyramid                                                  */
    TSLAM_STAGE_DETECT = 1,  /* pyramid -> smooth + candidates -> keypoints                     */
    TSLAM_STAGE_DESCRIBE = 2,/* keypoints -> orientation + descriptors                          */
    TSLAM_STAGE_MATCH = 3,   /* descriptors -> stereo/temporal matches + sub-pixel refinement   */
    TSLAM_STAGE_POSE = 4,    /* matches -> correspondences -> RANSAC -> refine -> chain         */
    TSLAM_STAGE_ALL = 5,     /* RECTIFY .. POSE, then BA when ba_window > 0                     */
    TSLAM_STAGE_BA = 6,      /* A8: insert the batch's keyframes into each pair's window + solve */
    /* single kernels (per-kernel timing in bench.py; same order as STAGE_ALL) */
    TSLAM_KERNEL_RECTIFY_PYRAMID = 10,
    TSLAM_KERNEL_DETECT = 11,       /* includes the histogram memset */
    TSLAM_KERNEL_SELECT = 12,
    TSLAM_KERNEL_DESCRIBE = 13,
    TSLAM_KERNEL_MATCH = 14,        /* includes the scratch memsets */
    TSLAM_KERNEL_MATCH_REFINE = 15,
    TSLAM_KERNEL_POSE = 16,
    TSLAM_KERNEL_CHAIN = 17,        /* every pair's chain, and the rig's after tslam_set_rig (one block each) */
    TSLAM_KERNEL_RIG = 18,          /* rig pose (after tslam_set_rig; sharded: the range's); run it before
                                       KERNEL_CHAIN */
    TSLAM_KERNEL_POSE_SOLVE = 19    /* parity tests: P3P + RANSAC + refinement alone, on the correspondences
                                       and counts in TSLAM_BUF_CORR / TSLAM_BUF_STATS (status 3 = to be
                                       solved, stats[1] = n) — crafted sets injected with tslam_copy_in */
};

/* Benchmark hook, never on the tracking path: inside a batch, after MATCH_REFINE, move `percent` %
 * of the batch's refined temporal positions (per frame, pair, keypoint by a hash of `seed`) by
 * 8..40 px per axis — outliers to every pose — so the pose stage can be timed on hard data. */
int tslam_perturb_temporal(tslam_handle* h, int percent, uint64_t seed, void* stream);

const char* tslam_last_error(void);
int tslam_abi_version(void);

int tslam_create(const tslam_stereo_desc* pairs, const tslam_params* params, int device, tslam_handle** out);
int tslam_destroy(tslam_handle* h);

/* Create a handle from raw calibration, doing on the host what HipSlamEngine.initialize does
 * through thor_slam_amd/calib.py (C++ restatement in tslam_calib.cpp, byte-identical tables):
 * cameras in extract_cameras order (sources sorted by name, isaac_ros.py:138-157), stereo pairs =
 * a cam_idx 1 camera directly after cam_idx 0 of its source, Bouguet rectification of each pair
 * (rgbd: undistortion of the colour camera), params->n_pairs = the pair count (0 = take it), and
 * for more than one pair tslam_set_rig with each pair's base_T_rect.
 * tslam_rig_pairs: the (left, right) indices into `cams` of the pairs (pairs[2*max_pairs] may be
 *   NULL); returns the pair count.
 * tslam_rectify_pair / tslam_rgbd_undistort: one pair's rectified intrinsics + baseline (the
 *   desc's map pointers are set to the given buffers), the [H][W][2] int32 1/32-px tables
 *   (NULL = skip), base_T_rect[16] = world_T_cam(left) * left_optical_T_rect (NULL = skip) and
 *   rect_rot[18] = the two 3x3 rectifying rotations (NULL = skip). */
int tslam_create_rig(const tslam_camera_desc* cams, int n_cams, const tslam_params* params, int device, tslam_handle** out);
int tslam_rig_pairs(const tslam_camera_desc* cams, int n_cams, int32_t* pairs, int max_pairs);
int tslam_rectify_pair(const tslam_camera_desc* left, const tslam_camera_desc* right, tslam_stereo_desc* desc,
                       int32_t* map_left, int32_t* map_right, double* base_T_rect, double* rect_rot);
int tslam_rgbd_undistort(const tslam_camera_desc* color, tslam_stereo_desc* desc, int32_t* map, double* base_T_rect);

/* Run the whole hot path on `n_frames` (<= max_batch) frames.  `images` is device memory laid out
 * [n_frames][2*n_pairs][H][W] u8 (left, right per pair).  Frames get consecutive global indices. */
int tslam_submit(tslam_handle* h, const uint8_t* images, int n_frames, void* stream);

/* Same, but stage by stage: set the batch, then run stages (parity tests inject/inspect buffers
 * between stages with tslam_copy_in / tslam_copy_out). */
int tslam_begin_batch(tslam_handle* h, const uint8_t* images, int n_frames);
int tslam_run_stage(tslam_handle* h, int stage, void* stream);
int tslam_end_batch(tslam_handle* h);

int tslam_detect(tslam_handle* h, void* stream);   /* RECTIFY + DETECT */
int tslam_describe(tslam_handle* h, void* stream);
int tslam_match(tslam_handle* h, void* stream);
int tslam_pose(tslam_handle* h, void* stream);

int tslam_sync(tslam_handle* h);

/* Asynchronous host boundary (what IsaacRosAdapter.process_frames + _odom_cb do over DDS,
 * isaac_ros.py:327-430 and :308-325; the pose may lag the frame, :429-430).
 *
 * tslam_submit_host: copy `n_frames` host frames ([n][2*n_pairs][H][W] gray, or RGB-D records
 *   [n][n_pairs][5*H*W]) into the handle's pinned staging buffer of the batch's parity (waiting
 *   only for that buffer's previous DMA), enqueue the DMA and the whole hot path on the handle's
 *   own streams (front stages on a high-priority stream overlapping the previous batch's back
 *   stages; with local BA, the BA on a third stream and the front / back streams CU-masked off
 *   64 CUs so its small dependent launches find free CUs) and the batch's results into a pinned
 *   slot (copied on the back stream right after the pose stage; with BA the slot completes after
 *   the BA, so the caller reads the window once it is polled); returns without waiting for the
 *   device.  Note: with local BA the CU-masked front / back streams come from
 *   hipExtStreamCreateWithCUMask, which gives default-flag, default-priority streams: they
 *   synchronise with the legacy null stream (null-stream work of the caller, e.g. a hipMemset or
 *   torch's default stream, serialises against the pipeline) and the front stream loses its high
 *   priority in that mode (the C4 bench runs in it).
 *   timestamps[n] (seconds, the frames' SynchronizedFrameSet.timestamp) may be NULL.  At most two
 *   batches' results are held: an unread batch s-2 is dropped when batch s is submitted.
 * tslam_poll_batch: results of the oldest unread submitted batch: returns 1 and fills the outputs
 *   (per frame and pair as tslam_read_poses, the rig's T_rel/T_abs/cov/stats when tslam_set_rig, the
 *   timestamps, its first global frame and frame count) when it has completed (or, with `block`,
 *   after waiting for it); 0 when no batch is ready / pending.  Pointers may be NULL.
 * tslam_poll_pose: non-blocking; the last frame of the newest completed batch not returned before:
 *   T[16] = its T_abs (the rig's world_T_base after tslam_set_rig, else the first pair's left-camera
 *   pose), cov[36], ts, state (TSLAM_POSE_*), conf = clamp(1 / (1 + tr(cov[:3,:3])), 0, 1)
 *   (isaac_ros.py:312; 1 when not tracked).  Returns 1 when a newer pose was written, else 0. */
int tslam_submit_host(tslam_handle* h, const uint8_t* host_images, const double* timestamps, int n_frames);
/* The pinned staging buffer the next tslam_submit_host copies from (max_batch frames of
 * frame_bytes each), after waiting until its previous DMA finished: a caller that assembles the
 * batch's frames there and passes this pointer as host_images saves the staging copy. */
int tslam_host_stage(tslam_handle* h, uint8_t** stage, int64_t* frame_bytes);
int tslam_poll_batch(tslam_handle* h, int block, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats,
                     double* rig_T_rel, double* rig_T_abs, double* rig_cov, int32_t* rig_stats, double* ts,
                     int64_t* first_frame, int* n_frames);
int tslam_poll_pose(tslam_handle* h, double* T, double* cov, double* ts, int32_t* state, float* conf);

/* Results of the last submitted batch (blocks until it is done).  Per frame f and pair p
 * (index f * n_pairs + p): T_rel[16] (cam_{t-1} -> cam_t), T_abs[16] (first left camera frame ->
 * current left camera frame, row-major), cov[36] (rho, omega), stats[8] = {status, n_corr,
 * n_inliers, best_count, best_hyp, global_frame, sigma^2 (f64 in stats[6..7]: the reprojection
 * variance that scales cov, 0 when not tracked)}.  Any pointer may be NULL.  The outputs
 * hold `max_frames` frames (TSLAM_EINVAL when the batch has more); TSLAM_ESTATE when no batch has
 * run since tslam_create / tslam_reset. */
int tslam_read_poses(tslam_handle* h, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats);

int tslam_reset(tslam_handle* h);
int64_t tslam_frames_done(tslam_handle* h);

int tslam_buffer_info(tslam_handle* h, int which, void** device_ptr, int64_t* bytes_total, int64_t* bytes_per_frame);
int tslam_copy_out(tslam_handle* h, int which, int64_t offset, void* host_dst, int64_t bytes);
int tslam_copy_in(tslam_handle* h, int which, int64_t offset, const void* host_src, int64_t bytes);
/* ring slot of global frame g (for ring-indexed buffers) */
int tslam_ring_slot(tslam_handle* h, int64_t global_frame);

/* Layout facts for host-side decoding: fills out[0..15] with
 * {W, H, n_levels, K, ring, batch, n_pairs, pyr_bytes, level offsets[6] (pyr), 0, 0}; and
 * level_info[0..17] with {W_l, H_l, K_l} for l < 6. */
int tslam_layout(tslam_handle* h, int64_t* out16, int32_t* level_info18);

/* IMU fusion (the gyro + accelerometer samples of
 * SynchronizedFrameSet.sensor_data, types.py:268-269, filled by rig.py:403-407, noise densities of
 * launch/thor_visual_slam.launch.py:82-93): a motion prior for each (frame, pair) of the NEXT
 * batch, prior[n][P][16] = {R[9], W_r, t[3], W_t, 0, 0}: the predicted rectified-left relative
 * pose T_rel = [R | t] (R row-major) with weights W_r (px^2 / rad^2) and W_t (px^2 / m^2), 0 = none.
 * A7's Gauss-Newton then minimises sum |reprojection|^2 + W_r |log(R_prior R^T)|^2 (small-angle
 * form) + W_t |t - t_prior|^2; RANSAC is unchanged.  A frame that is not tracked (LOST) but has
 * W_t > 0 is chained with the prediction (its T_rel record becomes [R | t]; status stays LOST),
 * so the trajectory continues through visual dropouts.  The tslam_imu_* filter below computes the
 * priors from the samples (gyro integration, velocity / gravity / accelerometer-bias filter). */
int tslam_set_motion_prior(tslam_handle* h, const double* prior, int n_frames);

/* The IMU filter behind those priors (host-side, native; the fusion cuVSLAM runs inside its
 * library with enable_imu_fusion:=true, Makefile:81, on the IMUData of each
 * SynchronizedFrameSet, types.py:268-269 / rig.py:403-407).  State: the rectified-left camera's
 * orientation in the filter's world, the world velocity, gravity, the accelerometer and gyroscope
 * biases (IMU axes) and their variances.  Noise (TSLAM_IMU_NOISE doubles): gyroscope noise
 * density and random walk, accelerometer noise density and random walk
 * (launch/thor_visual_slam.launch.py:82-90), rotation / translation prior floors, initial
 * velocity / accelerometer-bias / gyroscope-bias sigmas, the vision's rotation floor.
 *   tslam_imu_create: rect_R_imu (row-major), lever = the IMU's position in the camera frame (m),
 *     accel = 0 for the gyro-only filter.  tslam_imu_begin: anchor at rest (accel: one sample in
 *     IMU axes; NULL when gyro-only).
 *   tslam_imu_predict / _coast / _correct: one frame interval's prediction from a state, the state
 *     after an untracked interval, the state after a tracked one (T_rel row-major 4x4 mapping frame
 *     k points to frame k + 1, cov the 6x6 (rho, omega) covariance).
 *   tslam_imu_batch_priors: the next batch's predictions (dt[k] NaN = no sample -> valid[k] = 0),
 *     the state coasted over the batch's earlier frames; tslam_imu_absorb: the batch's tracked
 *     motions (status 0 = tracked) into the filter's state.
 *   tslam_imu_vision_only: the vision-only motion and covariance behind a solution the device
 *     weighted with a step's prior (one Gauss-Newton step on the vision alone; sigma2 from the pose
 *     stats); T / cov copied through when no prior acted or the vision's normal matrix is not
 *     positive definite.
 * Spec: oracle/numpy_imu.py. */
#define TSLAM_IMU_NOISE 10
typedef struct tslam_imu tslam_imu;
typedef struct tslam_imu_state {
    double R[9];          /* world_R_cam */
    double v[3];          /* world velocity, m/s */
    double ba[3];         /* accelerometer bias, IMU axes */
    double var_v, var_b;
    double bg[3];         /* gyroscope bias, IMU axes */
    double var_g;
    double w_prev[3];     /* previous interval's camera-axes rate (valid when has_w_prev) */
    int32_t has_w_prev, reserved;
} tslam_imu_state;
typedef struct tslam_imu_step {
    double dt;
    double gyro[3];
    double w[3];          /* bias-corrected rate, camera axes */
    double R_rel[9];
    double t_rel[3];
    double w_rot, w_trans;
    double v1[3];         /* predicted velocity (valid when has_v1) */
    double var_v1;
    int32_t has_v1, reserved;
} tslam_imu_step;
int tslam_imu_create(const double* rect_R_imu, const double* noise, const double* lever, int accel, tslam_imu** out);
void tslam_imu_destroy(tslam_imu* f);
int tslam_imu_reset(tslam_imu* f);
int tslam_imu_begin(tslam_imu* f, const double* accel);
int tslam_imu_ready(const tslam_imu* f);
int tslam_imu_get_state(const tslam_imu* f, tslam_imu_state* st);
int tslam_imu_set_state(tslam_imu* f, const tslam_imu_state* st);
int tslam_imu_predict(const tslam_imu* f, const tslam_imu_state* st, double dt, const double* gyro, const double* accel,
                   tslam_imu_step* out);
int tslam_imu_coast(const tslam_imu* f, const tslam_imu_state* st, const tslam_imu_step* s, tslam_imu_state* out);
int tslam_imu_correct(const tslam_imu* f, const tslam_imu_state* st, const tslam_imu_step* s, const double* t_rel,
                      const double* cov, tslam_imu_state* out);
int tslam_imu_batch_priors(const tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                           tslam_imu_step* out, int32_t* valid);
int tslam_imu_absorb(tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                     const int32_t* status, const double* t_rel, const double* cov);
int tslam_imu_vision_only(const double* T, const double* cov, double sigma2, const tslam_imu_step* s, double* T_out,
                          double* cov_out);
/* The filter's world gravity (zero before tslam_imu_begin / for the gyro-only filter). */
int tslam_imu_gravity(const tslam_imu* f, double* gravity);
/* The inertial factor record of tslam_ba_inertial_factor (record[TSLAM_BA_INE_RECORD], layout
 * there) from the n frame intervals between two keyframes: dt[n], gyro[n][3], accel[n][3] (IMU
 * axes), the filter's biases bg[3], ba[3] (they become bg_lin, ba_lin), w_prev[3] = the factor
 * frame's rate over the interval before the first (NULL: none), the factor's frame: frame_R_imu[9]
 * (row-major; NULL = the filter's rect_R_imu, i.e. pair 0's rectified-left camera; a rig's body
 * window passes base_R_imu) and lever[3] (the IMU's position in that frame; NULL = the filter's),
 * and the weights' floors: wv = 1 / (n_a^2 T + v_floor^2), wp = 1 / (n_a^2 T^3 / 3 + p_floor^2),
 * wR = 1 / (n_g^2 T + r_floor^2), the bias random walks w_ra = 1 / (s_a^2 T + ba_floor^2),
 * w_rg = 1 / (s_g^2 T + bg_floor^2) (n_a, n_g, s_a, s_g: the filter's noise densities and random
 * walks, launch/thor_visual_slam.launch.py:82-93; a zero density or walk gives weight 0).  Spec:
 * oracle/numpy_ba.py preintegrate. */
#define TSLAM_BA_INE_RECORD 80
int tslam_imu_preintegrate(const tslam_imu* f, int n, const double* dt, const double* gyro, const double* accel,
                           const double* bg, const double* ba, const double* w_prev, const double* frame_R_imu,
                           const double* lever, double v_floor, double p_floor, double r_floor, double ba_floor,
                           double bg_floor, double* record);

/* Rig pose (replaces the multi-camera fusion cuVSLAM does for the rig of
 * isaac_ros.py:364-411): base_T_rect[P][16] = the rectified-left frame of each pair in the rig's
 * base frame (RigCalibration.get_world_extrinsics, rig.py:35-70, composed with the
 * rectification).  Afterwards every POSE stage also solves one body motion per frame from ALL
 * pairs' correspondences (generalised PnP: per-pair RANSAC winners as candidates scored on every
 * pair, then a joint Gauss-Newton) and chains it. */
int tslam_set_rig(tslam_handle* h, const double* base_T_rect);
/* Body-frame results of the last batch (synchronises): per frame T_rel (body_{t-1} -> body_t
 * point map), T_abs (world_T_base, world = base at frame 0), 6x6 covariance, stats
 * {status, n_corr (all pairs), n_inliers, best candidate count, best candidate, frame, 0, 0}.
 * Capacity and state errors as tslam_read_poses. */
int tslam_read_rig_poses(tslam_handle* h, int max_frames, double* T_rel, double* T_abs, double* cov, int32_t* stats);

/* Sharded rig: one camera stream per GPU (replaces cuVSLAM's multicam mode,
 * launch/thor_visual_slam.launch.py:49,81, whose rig is RigCalibration.get_world_extrinsics,
 * rig.py:35-70).  Every rank creates the same handle for the whole rig (all pairs, tslam_set_rig
 * for a multi-pair rig), then tslam_set_shard(h, cam_lo, cam_hi, rank, world):
 *   - its front stages (RECTIFY, DETECT, DESCRIBE) process cameras [cam_lo, cam_hi) of every frame
 *     of a batch; tslam_begin_batch then takes images [n][cam_hi - cam_lo][H][W];
 *   - its back stages (MATCH, POSE) process frames [rank*n/world, (rank+1)*n/world) of the batch
 *     for every pair (plus the rig pose), after the other cameras of frames lo-1 .. hi-1 were
 *     brought in: tslam_unpack_streams (the exchanged stream blocks) + tslam_import_raw (their raw
 *     images, rectified into the ring);
 *   - CHAIN chains the whole batch after tslam_unpack_poses of every rank's records.
 * Per batch (s = the caller's stream order; collectives are the caller's, e.g. RCCL all-to-all /
 * all-gather through torch.distributed):
 *   begin_batch -> RECTIFY, DETECT, DESCRIBE -> pack_streams(frames lo_q-1.. for every rank q)
 *   -> all-to-all (raw images + stream blocks) -> import_raw + unpack_streams -> MATCH, POSE
 *   -> pack_poses -> all-gather -> unpack_poses -> KERNEL_CHAIN -> end_batch.
 * Every rank then holds the same per-pair and rig poses as an unsharded handle fed all cameras.
 * Requires n % world == 0 per batch (tslam_begin_batch rejects other n) and ba_window == 0.
 *
 * RGB-D rigs (params.rgbd; each "pair" is one colour camera + its aligned depth, so a camera's
 * back end needs no other camera) shard by camera only, and no image moves: begin_batch takes the
 * rank's records [n][cam_hi - cam_lo][5*H*W]; RECTIFY .. DESCRIBE, MATCH and POSE track the rank's
 * cameras over the whole batch; tslam_pack_pairs (its cameras, each peer's frame range) ->
 * all-to-all -> tslam_unpack_pairs (the peers' cameras, its own range); KERNEL_RIG solves the rig
 * pose of its range; then pack_poses -> all-gather -> unpack_poses -> KERNEL_CHAIN as above. */
int tslam_set_shard(tslam_handle* h, int cam_lo, int cam_hi, int rank, int world);
/* Bytes of one pair block (RGB-D sharding and the stereo pair split; per batch frame and pair:
 * pose f64[68], stats i32[8], correspondences f64[K][5] — the columns the rig pose reads:
 * X, Y, Z, cx - u, cy - v; rows past stats[1] are not copied). */
int tslam_pair_block_bytes(tslam_handle* h, int64_t* bytes);
/* Pair blocks of batch frames f0 .. f0+n_frames-1 x pairs [pair_lo, pair_hi) (frame-major) to / from
 * device memory, inside a batch (pack after POSE, unpack before KERNEL_RIG). */
int tslam_pack_pairs(tslam_handle* h, int f0, int n_frames, int pair_lo, int pair_hi, void* dst, void* stream);
int tslam_unpack_pairs(tslam_handle* h, int f0, int n_frames, int pair_lo, int pair_hi, const void* src, void* stream);
/* Bytes of one stream block (per frame and camera) and of one pose record (per frame). */
int tslam_exchange_sizes(tslam_handle* h, int64_t* stream_block, int64_t* pose_record);
/* Stream blocks of frames first_frame .. +n_frames-1 (global indices, ring-resident; frames < 0
 * pack as zeros / are skipped on unpack) x cameras [cam_lo, cam_hi), frame-major, device memory. */
int tslam_pack_streams(tslam_handle* h, int64_t first_frame, int n_frames, int cam_lo, int cam_hi, void* dst, void* stream);
int tslam_unpack_streams(tslam_handle* h, int64_t first_frame, int n_frames, int cam_lo, int cam_hi, const void* src,
                         void* stream);
/* Rectify + pyramid raw images [n_frames][cam_hi - cam_lo][H][W] (device) of global frames
 * first_frame.. into the ring (frames < 0 skipped). */
int tslam_import_raw(tslam_handle* h, const uint8_t* images, int64_t first_frame, int n_frames, int cam_lo, int cam_hi,
                     void* stream);
/* The all-to-all's peers, one launch each (stereo, world > 1, cameras [rank*S, (rank+1)*S); the
 * layouts of an all-to-all of [world][B/world + 1][S][...] slots, slot q for / from rank q):
 * tslam_stage_raw_peers: this rank's raw images of every peer q's frames lo_q-1 .. hi_q-1 (frame -1
 *   = prev_raw [S][H][W], the previous batch's last frame) -> dst [world][nr][S][H][W];
 * tslam_pack_streams_peers: their stream blocks -> dst [world][nr][S][stream_block];
 * tslam_import_peers: every peer's raw images and stream blocks of this rank's frames lo-1 .. hi-1
 *   (as received) -> rectified into the ring + unpacked (tslam_import_raw + tslam_unpack_streams
 *   per peer in two launches). */
int tslam_stage_raw_peers(tslam_handle* h, const uint8_t* prev_raw, void* dst, void* stream);
int tslam_pack_streams_peers(tslam_handle* h, void* dst, void* stream);
int tslam_import_peers(tslam_handle* h, const uint8_t* raw, const void* streams, void* stream);
/* Pose records (per frame: pose f64[P][68], rig pose f64[68], stats i32[P][8], rig stats i32[8])
 * of this rank's frame range of the current batch -> dst; all n frames <- src (frame order). */
int tslam_pack_poses(tslam_handle* h, void* dst, void* stream);
int tslam_unpack_poses(tslam_handle* h, const void* src, void* stream);

/* Multi-GPU without a host framework (tslam_comm_init): the sharded rig above,
 * driven by the library over RCCL (librccl, ncclSend / ncclRecv / ncclAllGather on xGMI).
 * tslam_comm_unique_id: a fresh ncclUniqueId (128 bytes); rank 0 makes it and hands it to the
 *   other ranks over the host's own channel.
 * tslam_comm_init: this handle (the whole rig: tslam_create_rig, or tslam_create + tslam_set_rig)
 *   joins the `world`-rank communicator as `rank` (one rank per GPU, the handle's device) and owns
 *   cameras [rank*C/world, (rank+1)*C/world) and, of an n-frame batch, frames
 *   [rank*n/world, (rank+1)*n/world) (C divisible by world, world <= max_batch; a stereo rig may
 *   run local BA: rank 0 solves it, see TSLAM_SHARD_GATHER; RGB-D rigs without local BA).
 * tslam_submit_sharded: one batch of n_frames (1 .. max_batch; ranges may be uneven or empty) of
 *   this rank's cameras ([n][C/world][H][W] u8 in HBM; RGB-D records [n][C/world][5*H*W]) once
 *   `stream` has them: front end of its cameras; raw images (straight from the input) + stream
 *   blocks of the frames every other rank solves sent point to point (RGB-D: its cameras' pair
 *   blocks); back end (+ rig pose) of its frame range; pose records all-gathered; the chain.  The
 *   library runs the phases on streams of its own — front (high priority), exchange, back — with
 *   double-buffered exchange buffers, so batch s's image exchange overlaps its front end; `stream`
 *   then waits for the batch (with TSLAM_SHARD_PIPELINE only for its input: batch s+1's front end
 *   then overlaps batch s's back end).  Every rank then
 *   reads the whole rig's poses with tslam_read_poses / tslam_read_rig_poses, identical to one
 *   handle fed all cameras.  Nothing synchronises the host. */
int tslam_comm_unique_id(void* id128);
int tslam_comm_init(tslam_handle* h, const void* id128, int rank, int world);
int tslam_submit_sharded(tslam_handle* h, const uint8_t* images, int n_frames, void* stream);

/* Options of the driver behind a sharded handle (tslam_comm_init, or any handle of a group):
 *   TSLAM_SHARD_GATHER   every rank sends rank 0 the temporal matches + refined disparities of its
 *                        frame range and the keypoints + descriptors of its left cameras, so rank
 *                        0's ring holds what local BA, loop closure (tslam_loop_*) and
 *                        relocalisation (tslam_relocalize) read, as on one handle; rank 0 solves
 *                        the local BA window (implied when ba_window > 0);
 *   TSLAM_SHARD_RESULTS  every batch's poses go to the handle's pinned result slots, so
 *                        tslam_poll_batch / tslam_poll_pose work on a sharded handle (the
 *                        asynchronous boundary: submit, then poll);
 *   TSLAM_SHARD_PROFILE  HIP events around every kernel and exchange of this rank's batches;
 *                        tslam_shard_timing returns the average µs per batch of each segment
 *                        (TSLAM_SEG_*) since its last call (synchronises) and the batch count;
 *   TSLAM_SHARD_SERIAL   (profiling aid) every rank's work on one stream per device, shared by the
 *                        ranks on it: with all ranks of a group on one GPU, each kernel and copy
 *                        runs alone, so the profile gives isolated per-rank durations;
 *   TSLAM_SHARD_PIPELINE the caller's stream waits only until the batch has read its input and
 *                        receive buffers (the caller may refill the input), not for the whole
 *                        batch: the next batch's front end overlaps this one's back end.  Results
 *                        are then read after a device synchronisation or through the result
 *                        slots (TSLAM_SHARD_RESULTS + tslam_poll_*);
 *   TSLAM_SHARD_SOLO     (profiling aid, groups only) rank 0 alone runs its work and every exchange
 *                        is skipped (its receive buffers keep the last full batch's data): the
 *                        per-GPU step of one rank of an N-GPU node with the exchange hidden, timed
 *                        on one GPU.  Results are not meaningful; reset the handles afterwards;
 *   TSLAM_SHARD_PAIRS    pair split of a stereo rig with one camera per rank (world = cameras, no
 *                        local BA / gather): rank r's back end solves pair r/2 over half r&1 of
 *                        the batch, so its raw images and stream blocks go to its partner r^1
 *                        only, and rank r's rig range (range (r&1)*world/2 + r/2 of the world-way
 *                        split, inside its half) collects the other pairs' pair blocks (pose,
 *                        stats, correspondences) from the ranks of its half before the rig pose.
 *                        Every rank of the rig must set it alike.  Results are identical.
 * Setting options waits for the work enqueued so far. */
#define TSLAM_SHARD_GATHER 1
#define TSLAM_SHARD_RESULTS 2
#define TSLAM_SHARD_PROFILE 4
#define TSLAM_SHARD_SERIAL 8
#define TSLAM_SHARD_PIPELINE 16
#define TSLAM_SHARD_SOLO 32
#define TSLAM_SHARD_PAIRS 64
enum tslam_segment {
    TSLAM_SEG_RECTIFY = 0, TSLAM_SEG_DETECT, TSLAM_SEG_SELECT, TSLAM_SEG_DESCRIBE, TSLAM_SEG_PACK,
    TSLAM_SEG_EXCHANGE_WAIT,   /* front end done -> the peers' images and stream blocks landed */
    TSLAM_SEG_IMPORT, TSLAM_SEG_MATCH, TSLAM_SEG_MATCH_REFINE, TSLAM_SEG_POSE, TSLAM_SEG_RIG,
    TSLAM_SEG_STATE,           /* state blocks packed (senders) / unpacked (rank 0) */
    TSLAM_SEG_POSE_GATHER, TSLAM_SEG_CHAIN, TSLAM_SEG_BA,
    TSLAM_SEG_PAIR_BLOCKS,     /* pair split: pair blocks packed, exchanged, unpacked */
    TSLAM_SEG_COUNT
};
int tslam_shard_options(tslam_handle* h, int flags);
int tslam_shard_timing(tslam_handle* h, double* out_us, int n_out);

/* One process driving the whole sharded rig (the SlamEngine boundary on several GPUs): handles[r]
 * (the same rig on every handle, one per rank, created on the rank's device) become ranks
 * 0 .. n-1 of one driver, as after tslam_comm_init.
 *   TSLAM_TRANSPORT_RCCL: an RCCL clique over the handles' devices (ncclCommInitAll; one device per
 *     handle), all ranks' sends / receives issued inside one ncclGroupStart / ncclGroupEnd;
 *   TSLAM_TRANSPORT_COPY: device-to-device copies (hipMemcpyAsync) instead of RCCL, same buffers and
 *     ordering; several ranks may share a device (tests world > 1 on one GPU).
 * tslam_group_submit: one batch of n_frames (1 .. max_batch); images[r] = rank r's
 *   cameras as for tslam_submit_sharded, streams[r] (NULL array or entries = each device's null
 *   stream) orders the input and then waits for the batch.
 * tslam_group_destroy before destroying the handles (they return to unsharded). */
#define TSLAM_TRANSPORT_RCCL 0
#define TSLAM_TRANSPORT_COPY 1
typedef struct tslam_group tslam_group;
int tslam_group_create(tslam_handle* const* handles, int n, int transport, tslam_group** out);
int tslam_group_submit(tslam_group* g, const uint8_t* const* images, int n_frames, void* const* streams);
int tslam_group_destroy(tslam_group* g);

/* A8 window of stereo pair `pair` after the last enqueued solve (synchronises the device),
 * indexed by slot (slot = keyframe number mod ba_window): frames[W] (global frame, -1 = empty),
 * cam_T_world[W][16] (BA estimate), landmark[W][K] (id = home slot * K + keypoint, or -1),
 * points[W*K][3] (world position by id), obs_uvd[3][W][K] (u, v, disparity; NaN = none),
 * counts[4] (observations, landmarks, last solve ok, 0).  Any output pointer may be NULL.
 * Rig-level A8: on a handle with tslam_set_rig over several pairs the keyframes of all pairs are
 * solved as ONE window of body poses (every pair's reduced camera system moved into the body frame
 * by the adjoint of E_p^-1 and summed; the pairs' cameras are E_p^-1 B); pair = n_pairs then reads
 * that body window: cam_T_world[W][16] = body_T_world (base_link), counts = the joint ones,
 * landmark / points / obs_uvd filled with -1 / 0 / NaN (the landmarks live in the pairs' windows). */
/* IMU rotation factor of keyframe `frame` of `pair` for its local BA window (before the batch that
 * contains the frame is submitted): M (row-major 3x3) = the gyro-integrated rotation from the
 * previous keyframe's rectified-left camera to this one's (frame g - ba_kf_interval points to
 * frame g), weight (1 / rad^2; 0 = none).  Every Gauss-Newton step of the window then adds the
 * residual vee((M^T R_c R_{c-1}^T - ...) / 2) between window-consecutive keyframes (spec:
 * oracle/numpy_ba.py imu_terms).  Pair windows only (a rig's body window ignores it). */
int tslam_ba_imu_factor(tslam_handle* h, int pair, int64_t frame, const double* M, double weight);
/* Tightly coupled inertial factors (spec: oracle/numpy_ba.py inertial_system; ABI 19: gyroscope
 * bias and bias random walks, the noise model of launch/thor_visual_slam.launch.py:50-53,88-93).
 * tslam_ba_inertial: world gravity [3] (the tracking world: pair 0's rectified-left camera at frame
 *   0) and priors on the oldest window keyframe's biases: accelerometer [3] with its weight
 *   (1 / (m/s^2)^2), gyroscope [3] with its weight (1 / (rad/s)^2), for the next solves of `pair`'s
 *   window.
 * tslam_ba_inertial_factor: keyframe `frame`'s IMU preintegration from the previous keyframe
 *   (before the batch holding it is submitted): record[TSLAM_BA_INE_RECORD] = dv[3], dp[3]
 *   (previous keyframe's camera axes), Jv[9], Jp[9] (row-major, d/d ba), ba_lin[3], dt, wv
 *   (1 / (m/s)^2, 0 = no factor), wp (1 / m^2), wR (1 / rad^2: the gyro rotation rows), w_ra
 *   (accelerometer-bias random walk), M[9] (the gyro rotation, previous camera points -> this
 *   camera), JRe[9] (d r_R / d bg), Jvg[9], Jpg[9] (d/d bg), bg_lin[3], w_rg (gyroscope-bias random
 *   walk), 8 unused — tslam_imu_preintegrate writes it — and v0[3], the keyframe camera's initial
 *   world velocity.  Every window keyframe then carries a velocity and accelerometer / gyroscope
 *   biases (a new keyframe's start at its record's linearisation point, or the previous keyframe's);
 *   every Gauss-Newton step eliminates these 9 unknowns per keyframe into the reduced camera system
 *   (k_ba_reduce_solve_ine) and updates them after the camera solve.  A window with no factor
 *   between two of its keyframes solves as before.  A factor's rotation rows replace the separate
 *   tslam_ba_imu_factor of that keyframe: give one or the other.
 * tslam_ba_read_inertial (synchronises): velocity[W][3] and bias[W][6] (accelerometer, gyroscope) by slot.
 * On a rig (tslam_set_rig over several pairs, rig-level A8) the factors act on the body window:
 * pair = n_pairs, record in the earlier keyframe's body (base_link) axes, velocities of the body
 * origin, gravity in the body window's world (base_link at frame 0); pair windows are refused. */
int tslam_ba_inertial(tslam_handle* h, int pair, const double* gravity, const double* ba_prior, double ba_weight,
                      const double* bg_prior, double bg_weight);
int tslam_ba_inertial_factor(tslam_handle* h, int pair, int64_t frame, const double* record, const double* v0);
int tslam_ba_read_inertial(tslam_handle* h, int pair, double* velocity, double* bias);
int tslam_ba_read(tslam_handle* h, int pair, int64_t* frames, double* cam_T_world, int32_t* landmark,
                  double* points, double* obs_uvd, int32_t* counts);

/* A8 profiling (synchronises): returns the total HIP-event time and count of the Schur-product
 * kernel (k_ba_schur) launches timed since the previous call and their algorithmic flops
 * (2 (6n+1)^2 3L per launch, n keyframes, L landmarks), then re-arms timing for up to
 * `max_launches` further launches (0 = off). */
int tslam_ba_profile(tslam_handle* h, int max_launches, double* schur_ms, int64_t* schur_launches, double* schur_flops);
/* Verification of the in-launch hand-off: split = 1 runs every later pair-window
 * Gauss-Newton step as k_ba_reduce + k_ba_solve (a kernel boundary between the reduction and the
 * solve) instead of k_ba_reduce_solve; both sum in the same order, so the windows agree bit for
 * bit.  0 (default) restores the fused launch. */
int tslam_ba_split_solve(tslam_handle* h, int split);
/* Issue of a stereo pair window's keyframe chain (ABI 19).  enable = 1: each keyframe's ~16 BA
 * launches replay a captured hipGraph of that chain shape whose kernels read the keyframe's
 * arguments from a device record (one node update + one graph launch per keyframe and pair);
 * 0 (default): direct launches with by-value arguments — on this ROCm the replay is the slower
 * issue (162 against 80 us of host time per keyframe).  Same kernels, same sums:
 * the windows agree bit for bit.  Rig body windows and BA profiling always launch directly. */
int tslam_ba_graph(tslam_handle* h, int enable);
/* Deferred BA issue for stage-API callers that pipeline batches (defer = 1; 0, the default,
 * issues the BA inside tslam_run_stage(TSLAM_STAGE_BA)).  With a BA stage on a stream of its own,
 * the stage call only takes the pose snapshot and makes that stream wait for the batch's back end;
 * the ~16 launches per keyframe are enqueued at the next flush point: the next batch's first back
 * stage (so its front stages are already on the GPU), the next BA stage, or any call that reads or
 * changes BA, pose or map state (tslam_sync, tslam_poll_*, tslam_read_*, tslam_ba_*, tslam_copy_*,
 * loop / relocalisation / map / TSDF calls, tslam_reset, tslam_destroy).  tslam_submit_host never
 * defers.  Results are identical; only the host's enqueue order changes. */
int tslam_ba_defer(tslam_handle* h, int defer);
/* Measurement: `reps` back-to-back k_ba_schur launches on pair `pair`'s last solved window (the
 * kernel only rewrites its own outputs), between two HIP events on `stream`: the average launch
 * duration and the algorithmic flops per launch (for the FP64 MFMA roofline, without per-launch
 * events inside the timed steps). */
int tslam_ba_replay_schur(tslam_handle* h, int pair, int reps, void* stream, double* us_per_launch,
                          double* flops_per_launch);

/* Map side of A8 for persistence (synchronises): per landmark id of pair `pair`'s window the
 * global landmark id (creation frame * K + keypoint; -1 / stale where no landmark lives) and the
 * rBRIEF descriptor of the keyframe keypoint the id names: gid[W*K], desc[W*K][8]. */
int tslam_ba_read_map(tslam_handle* h, int pair, int64_t* gid, uint32_t* desc);

/* Relocalisation (SlamEngine.load_map / relocalize, interface.py:239-256): upload a map of n
 * landmarks (world xyz f64 [n][3], rBRIEF-256 [n][8]; n < 2^20), then solve cam_T_world of a
 * resident frame's left camera of `pair` by brute-force Hamming matching of its keypoints against
 * the map (ratio + max_hamming as A6) and A7's P3P-RANSAC + Gauss-Newton.  stats as
 * tslam_read_poses (status 0 = relocalised); cam_T_world = identity when it fails. */
int tslam_map_upload(tslam_handle* h, const double* xyz, const uint32_t* desc, int64_t n);
int tslam_relocalize(tslam_handle* h, int pair, int64_t frame, double* cam_T_world, double* cov, int32_t* stats);
/* Relocalisation of a whole rig (tslam_set_rig; map uploaded in the rig's base / world frame):
 * every pair matches its left image of `frame` against the map, A7 solves each pair on the map
 * points seen in its frame (E_p^-1 X), and the rig pose (candidates from every pair, scored on all
 * pairs, joint Gauss-Newton) gives body_T_world[16] (+ cov[36] in the body frame, stats[8] as the
 * rig's; pair_stats[P][8] per pair).  A map seen by any one pair relocalises the rig. */
int tslam_relocalize_rig(tslam_handle* h, int64_t frame, double* body_T_world, double* cov, int32_t* stats,
                         int32_t* pair_stats);

/* Loop closure + keyframe pose graph (the reference only forwards
 * SlamConfig.enable_loop_closure, thor_slam/slam/interface.py:155-156, to cuVSLAM).  Spec and CPU
 * restatement: oracle/numpy_loop.py.  All of these synchronise the handle's stream.
 *
 * tslam_loop_init: a keyframe database of `max_keyframes` entries (ring: entry = count mod
 *   max_keyframes) with `signature` (<= 256) descriptors per keyframe for place recognition;
 *   tslam_reset empties it.
 * tslam_loop_add_keyframe: store resident `frame` of `pair`: its valid left keypoints with a stereo
 *   disparity d > 0, in keypoint order, as camera-frame landmarks (z = fx*B/d, x = (u-cx) z/fx,
 *   y = (v-cy) z/fy; u, v level-0) + rBRIEF-256; returns the entry and its landmark count.
 * tslam_loop_read_keyframe: copy entry `slot` out (xyz[n][3], desc[n][8]; NULL skips).
 * tslam_loop_query: votes[j] for entries j < n_candidates: the query entry's first `signature`
 *   descriptors matched by brute-force Hamming against entry j's (A6 max_hamming + ratio rule).
 * tslam_loop_verify: cam_q_T_cam_c of resident `frame` against entry `slot`'s landmarks by the
 *   relocalisation matcher and A7's P3P-RANSAC + Gauss-Newton; stats as tslam_read_poses.
 * tslam_pose_graph: `iters` Gauss-Newton iterations on nodes world_T_node[n_nodes][16] (in/out,
 *   node 0 fixed; n_nodes <= 1024) with edges[n_edges][2] = (a, b), meas[n_edges][16] = measured
 *   T_a^-1 T_b, info[n_edges][36]; residual Log(meas^-1 T_a^-1 T_b) in (rho, phi) order, dense
 *   normal equations factored by blocked Cholesky (FP64 MFMA trailing updates); *cost = sum of
 *   e^T info e at the returned poses (cost may be NULL). */
int tslam_loop_init(tslam_handle* h, int max_keyframes, int signature);
int tslam_loop_add_keyframe(tslam_handle* h, int pair, int64_t frame, int* slot, int* n_landmarks);
int tslam_loop_read_keyframe(tslam_handle* h, int slot, double* xyz, uint32_t* desc, int* n);
int tslam_loop_query(tslam_handle* h, int slot, int n_candidates, int32_t* votes);
int tslam_loop_verify(tslam_handle* h, int pair, int64_t frame, int slot, double* T_qc, double* cov, int32_t* stats);
int tslam_pose_graph(tslam_handle* h, int n_nodes, double* world_T_node, int n_edges, const int32_t* edges,
                     const double* meas, const double* info, int iters, double* cost);
/* Test hook (process-wide, 0 = off, the default): every later k_pg_potrf launch holds its blocks
 * >= 1 back by `spins` x 127 x 64 cycles before they read the diagonal tile, forcing the read
 * order of a late block (the panel's stores of block 0 have landed).  Results never change. */
int tslam_test_potrf_delay(int spins);

/* Asynchronous loop closure (ABI 15): the reference's default deployment path runs with loop
 * closure on at batch 1 (HipSlamEngine(num_cameras=N) + initialize, scripts/run_slam.py:299-300;
 * SlamConfig.enable_loop_closure defaults to True, interface.py:156), so nothing of it may wait on
 * the host per frame.  Spec of the policy on top: oracle/numpy_loop.py LoopPolicy.
 *
 * tslam_loop_auto: with interval > 0 every tracked keyframe of every later batch (frame g with
 *   g % interval == 0 and pose status 0: the rig's after tslam_set_rig, pair 0's otherwise) is
 *   stored by the submit path itself, on the batch's back stream right after its pose stage (no
 *   host round trip, no ring-residency condition).  The i-th tracked keyframe since the call (or
 *   tslam_reset) takes database position i, entry (i mod cap_k) * P + p for each pair p, cap_k =
 *   max_keyframes / P of tslam_loop_init: the database is a ring over tracked keyframes, so a
 *   session of any length keeps the newest cap_k, and untracked stretches take no entries.  Each
 *   entry also holds a snapshot of its image's keypoint records, level counts and descriptors (the
 *   query side of a later verification).  interval 0 turns it off.  tslam_loop_add_keyframe (the
 *   manual slot counter) is refused while it is on.  Unsharded handles only.
 * Jobs: run in submission order on the handle's loop stream (beside the tracking streams), results
 * in pinned memory; at most 64 jobs may be unreturned.  Each returns a job id (> 0).
 * tslam_loop_job_vote: votes of entry `query` against the entries of database positions
 *   [k0, k0 + n_kf): votes[(k - k0) * P + p] for pair p's entry of position k (tslam_loop_query's
 *   rule).
 * tslam_loop_job_verify: cam_q_T_cam_c of entry `query`'s snapshot (its pair's left image, the
 *   RANSAC seeded by `frame`, the keyframe's frame index) against entry `cand`'s landmarks, as
 *   tslam_loop_verify on the resident frame.
 * tslam_loop_job_pose_graph: tslam_pose_graph's solve (inputs copied at the call).
 * tslam_loop_job_poll: 0 while job `id` runs (block = 0), else 1 and its results once:
 *   vote -> votes[n_kf * P]; verify -> T_qc[16], cov[36], stats[8]; pose graph -> world_T_node
 *   [n_nodes][16] and *cost (NULL skips any output).  TSLAM_ESTATE for an unknown or returned id;
 *   TSLAM_ESINGULAR (also from tslam_pose_graph) when the solve's normal matrix was not positive
 *   definite (a pivot <= 0 or NaN: some pose came back non-finite) — the loop policy then rejects
 *   that loop (oracle/numpy_loop.py LoopPolicy). */
int tslam_loop_auto(tslam_handle* h, int interval);
int tslam_loop_job_vote(tslam_handle* h, int query, int64_t k0, int n_kf, int64_t* job);
int tslam_loop_job_verify(tslam_handle* h, int pair, int64_t frame, int query, int cand, int64_t* job);
int tslam_loop_job_pose_graph(tslam_handle* h, int n_nodes, const double* world_T_node, int n_edges, const int32_t* edges,
                              const double* meas, const double* info, int iters, int64_t* job);
int tslam_loop_job_poll(tslam_handle* h, int64_t job, int block, int32_t* votes, double* T_qc, double* cov,
                        int32_t* stats, double* world_T_node, double* cost);

/* RGB-D dense mapping (the reference runs nvblox on the RGB + u16 depth
 * topics, scripts/run_pipeline.py:218-256, voxel 0.05 m / truncation 4 voxels / 10 m,
 * launch/thor_nvblox.launch.py:26-36).  Spec and CPU restatement: oracle/numpy_tsdf.py.
 *
 * tslam_tsdf_init: a dense volume of dims[3] = (nx, ny, nz) voxels of voxel_size metres with its
 *   corner at origin[3] (tracking world frame = rectified left camera of frame 0); tsdf f32 (m)
 *   and weight f32, zeroed (also by tslam_reset).
 * tslam_tsdf_integrate: integrate n_frames depth images (device u16 mm [H][W] of pair `pair`'s
 *   camera, frames stride_bytes apart; for RGB-D records [BGR | depth] pass record + 3*H*W and the
 *   record stride) with camera poses world_T_cam[n][16] (host; a NaN pose skips its frame) or, when world_T_cam is NULL, the
 *   device-resident tracked poses of frames first_frame.. of the last batch (untracked frames are
 *   skipped).  Enqueued on `stream` (NULL: the handle's last stream).
 * tslam_tsdf_read: copy the volume out (synchronises); tsdf / weight may be NULL.
 * tslam_tsdf_write: replace the volume (a saved dense map reloaded; synchronises).
 * Colour layer (nvblox's colour integration of the RGB image aligned with the depth):
 * tslam_tsdf_color(h, 1) before tslam_tsdf_init adds a running colour (R, G, B f32 in [0, 255])
 * and its weight per voxel; tslam_tsdf_integrate_rgbd integrates the BGR images `color` with the
 * depth (both frames stride_bytes apart: an RGB-D record's colour and depth parts), the colour of
 * the depth pixel into every updated voxel inside the truncation band;
 * tslam_tsdf_read_color / _write_color copy it ([nz][ny][nx][3] and [nz][ny][nx]). */
int tslam_tsdf_init(tslam_handle* h, const double* origin, const int32_t* dims, double voxel_size, double trunc_vox,
                    double max_dist, double max_weight);
int tslam_tsdf_integrate(tslam_handle* h, int pair, const void* depth, int64_t stride_bytes, int n_frames,
                         int64_t first_frame, const double* world_T_cam, void* stream);
int tslam_tsdf_read(tslam_handle* h, float* tsdf, float* weight);
int tslam_tsdf_write(tslam_handle* h, const float* tsdf, const float* weight);
int tslam_tsdf_color(tslam_handle* h, int enable);
int tslam_tsdf_integrate_rgbd(tslam_handle* h, int pair, const void* color, const void* depth, int64_t stride_bytes,
                              int n_frames, int64_t first_frame, const double* world_T_cam, void* stream);
int tslam_tsdf_read_color(tslam_handle* h, float* rgb, float* weight);
int tslam_tsdf_write_color(tslam_handle* h, const float* rgb, const float* weight);

/* Dense-map outputs of the TSDF volume — what nvblox publishes after integration (its mesh and
 * ESDF / distance-slice outputs; launch/thor_nvblox.launch.py:21-103 starts the node the reference
 * feeds).  Spec: thor_slam_amd/dense.py; CPU restatement: oracle/numpy_dense.py.  Every value
 * follows from the volume alone (f32 tsdf / weight [nz][ny][nx]).
 *
 * tslam_mesh_extract: marching cubes over the voxel centres (cubes whose 8 voxels have weight >=
 *   min_weight; inside = tsdf < 0) into the handle's triangle buffer, on `stream` (NULL: the
 *   handle's last stream); waits for the triangle count only (*n_tris).
 * tslam_mesh_read: copy the first min(max_tris, count) triangles out, 9 f32 each (three xyz
 *   vertices in metres, facing positive tsdf), in cube order (synchronises).
 * tslam_mesh_read_colors: with the colour layer, the vertices' colours (9 f32 per triangle: each
 *   vertex takes the colour of its edge's voxel nearer to it).
 * tslam_esdf_compute: exact Euclidean signed distance (m) of every observed voxel (weight >=
 *   min_weight) to the nearest site (observed, |tsdf| <= site_vox * voxel), negative inside (tsdf
 *   < 0), +-max_dist beyond floor(max_dist / voxel) voxels (<= 2048), NaN unobserved; enqueued on
 *   `stream` into the handle's ESDF volume.
 * tslam_esdf_read: copy the ESDF volume out (synchronises).
 * tslam_esdf_slice: 2-D unsigned distance map out[nz][nx] over the height band y0 <= j < y1 (a
 *   column is a site / observed when any of its band's voxels is; synchronous). */
int tslam_mesh_extract(tslam_handle* h, double min_weight, int64_t* n_tris, void* stream);
int tslam_mesh_read(tslam_handle* h, float* tris, int64_t max_tris);
int tslam_mesh_read_colors(tslam_handle* h, float* colors, int64_t max_tris);
int tslam_esdf_compute(tslam_handle* h, double max_dist, double site_vox, double min_weight, void* stream);
int tslam_esdf_read(tslam_handle* h, float* esdf);
int tslam_esdf_slice(tslam_handle* h, int y0, int y1, double max_dist, double site_vox, double min_weight, float* out);

#ifdef __cplusplus
}
#endif

#endif /* TSLAM_H */
