// tslam_ba.h — A8 local bundle adjustment: device storage and launch arguments (k_ba.hip).
//
// Per stereo pair p (persistent, W = ba_window slots, K keypoints per image):
//   T    f64 [P][W][16]     cam_T_world of each keyframe (BA estimate)
//   Tfe  f64 [P][W][16]     world_T_cam of the front end (tracking chain) at insertion
//   u v d f64 [P][W][K]     level-0 observation of every keypoint, disparity (NaN = none)
//   lm   i32 [P][W][K]      landmark id (home slot * K + keypoint) or -1
//   X    f64 [P][W*K][3]    landmark positions (world), indexed by id
// Per solve (scratch, one set per pair: the rig-level solve keeps every pair's linearisation alive
// across an iteration): observation lists, the camera x landmark observation table, Jacobian
// blocks and the split-K partials of the 64 x 64 Schur product C.  The camera system is 64 wide:
// 6 rows per keyframe (<= 10 keyframes = 60 rows) and row 60 = the landmark
// right-hand side.
// Rig-level A8 (a handle with tslam_set_rig and P > 1; oracle RigKeyframeWindow): storage pair P
// is the BODY window — T[P] = body_T_world per slot, Tfe[P] = the rig front end's world_T_body at
// insertion, and its C / cam_U / dc / counts hold the combined body system of an iteration; every
// pair's cameras are E_p^-1 T[P].
#pragma once

#include "tslam_common.h"

#define TS_BA_MAXD 54   // 6 * (TS_BA_MAXW - 1): the reduced camera system without the gauge
// inertial factor record per slot (oracle/numpy_ba.py INE_N): dv 0-2, dp 3-5, Jv 6-14, Jp 15-23
// (d/d ba, row-major), ba_lin 24-26, dt 27, wv 28 (0 = no factor), wp 29, wR 30, w_ra 31, M 32-40
// (gyro rotation, camera i points -> camera j), JRe 41-49 (d r_R / d bg), Jvg 50-58, Jpg 59-67
// (d/d bg), bg_lin 68-70, w_rg 71, 72-79 unused
#define TS_BA_INE 80
#define TS_BA_INEY 9   // inertial unknowns per keyframe: velocity, accelerometer bias, gyroscope bias
#define TS_BA_MAXY (TS_BA_INEY * TS_BA_MAXW)
#define TS_BA_SPLIT 256 // blocks of the Schur product (32-landmark chunks dealt over them; 8192 landmarks in one round)
#define TS_BA_TILES 128 // scan tiles of a solve's compaction (landmark + observation tiles)
// at the largest window and K (n_features <= 8192, tslam_create): landmark tiles W K / 2048 plus
// W K / 2048 observation tiles fit (k_ba_tilescatter's LDS counts, tc_fl / tc_ids)
static_assert(2 * TS_BA_MAXW * (8192 / 2048) <= TS_BA_TILES, "compaction tiles at W = 10, K = 8192");
#define TS_BA_PART (4096 + 288) // doubles per Schur block partial: C [64][64], then the camera blocks [MAXW][27]

static_assert(6 * TS_BA_MAXW + 1 <= 64, "the BA camera system (6 rows per keyframe + rhs) is 64 wide");
static_assert(TS_BA_MAXW * 27 <= 288, "a Schur partial holds every window camera's 27 sums");

struct BaStore {
    // persistent, pair 0 (pair stride: W*16 doubles for T/Tfe, W*K for u/v/d/lm, W*K*3 for X)
    double* T;
    double* Tfe;
    double* u;
    double* v;
    double* d;
    int32_t* lm;
    double* X;
    uint32_t* kf_desc;  // [P][W*K][8] descriptor of every keyframe keypoint (a landmark id's descriptor)
    int64_t* gid;       // [P][W*K] global landmark id (creation frame * K + keypoint), kept on re-homing
    // scratch (sizes for W*K landmarks/observations)
    int32_t* remap;    // [K] (0x7F7F7F7F between evictions: k_ba_insert refills it)
    int32_t* cnt;      // [WK] observations per landmark id (after the gate; zero between solves)
    int32_t* lm_id;    // [WK] id per compact index
    uint8_t* keep;     // [W*K] gate result per (window camera, keypoint)
    // per landmark tile (k_ba_tilecount): the ids' flags (>= 2 gated observations), 32 per word,
    // and the flagged ids of the tile before each word — the compact index of any id in O(1)
    uint32_t* lmask;   // [WK / 32 + 64]
    int32_t* lpre;     // [WK / 32 + 64]
    // k_ba_tilecount's per-thread results for k_ba_tilescatter: each thread's 8 flags (a byte) and,
    // in observation tiles, its 8 landmark ids — the scatter reads them instead of re-deriving them
    uint8_t* tc_fl;    // [TS_BA_TILES][256]
    int32_t* tc_ids;   // [TS_BA_TILES][2048]
    int32_t* cam_off;  // [W+1]
    int32_t* counts;   // [P][4] n_obs, L, solve ok, pad
    int32_t* tiles;    // [2][TS_BA_TILES] tile counts, tile offsets
    int32_t* done;     // [P] blocks of k_ba_reduce_solve counted in (zero between launches)
    // per (compact landmark r, window camera ci) slot s = r * TS_BA_MAXW + ci (k_ba_tilescatter):
    // the observation index or -1, its (u, v, d), and W_o of the last linearisation — every per-
    // iteration read of the Schur pass is one level of indexing
    int32_t* lo_o;     // [WK * MAXW] (all -1 outside a solve's rows: k_ba_insert_gate clears the last solve's)
    double* lo_uvd;    // [WK * MAXW][4]  u, v, d, 0
    double* lo_W;      // [WK * MAXW][18] W_o = J_c^T J_p (6x3, row-major)
    double* Xc;        // [WK][3] position of compact landmark r during the solve (X[lm_id[r]] after it)
    double* obs_Vg;    // [WK][9]   J_p^T J_p (upper 6) | J_p^T r (3), gathered per landmark
    double* lm_L;      // [6][WK]   (structure-of-arrays)   Cholesky factor of V_i (1/L00 L10 1/L11 L20 L21 1/L22: diagonal inverted)
    double* lm_gp;     // [3][WK]
    double* part;      // [TS_BA_SPLIT][TS_BA_PART] per Schur block: C partial, then [camera][27] partial
    double* C;         // [64][64]
    double* cam_U;     // [W][27]
    double* dc;        // [W][6]
    double* flops;     // [1] algorithmic Schur-product flops accumulated (profiling)
    double* fe_pose;   // [2][B][P][16] front-end world_T_cam of the batch (snapshot per batch parity)
    double* fe_body;   // [2][B][16] rig front end's world_T_body of the batch (rig-level A8)
    int32_t* kf_assoc; // [2][B][P][K] a keyframe's keypoint chained by the temporal matches back to
                       // frame g - interval (or -1), written beside the pose snapshot (k_ba_kf_assoc)
    double* imu;       // [P][W][10] IMU rotation factor per slot: M (row-major 9), weight (0 = none)
    double* ine;       // [P][W][TS_BA_INE] inertial factor per slot (from the previous keyframe)
    double* vel;       // [P][W][3] world velocity of each slot's camera
    double* bias;      // [P][W][6] accelerometer and gyroscope biases (IMU axes) per slot
};

struct BaArgs {
    BaStore st;
    int W;                      // window slots
    int pair;
    int slot;                   // insert / evict: the keyframe's slot
    int prev;                   // insert: slot of the previous (newest) keyframe or -1
    int64_t frame;              // insert: global frame
    int interval;               // frames between keyframes
    int n_order;                // keyframes in `order`
    int order[TS_BA_MAXW];      // evict: remaining slots; gather/solve: occupied slots, oldest first
    int iters, nsplit;
    int fused_backsub;          // schur: first apply the previous iteration's landmark back substitution
    int pose_given;             // insert: the slot's cam_T_world is already set (rig-level A8)
    double lam, outlier_px;
    const double* fe;           // insert: this batch's front-end pose snapshot [B][P][16]
    const double* fe_body;      // rig insert: the rig front end's snapshot [B][16]
    const int32_t* kf_assoc;    // insert: this batch's chained temporal matches [B][P][K]
    double imu[10];             // insert: the keyframe's IMU rotation factor (M 9, weight; 0 = none)
    double ine[TS_BA_INE];      // insert: the keyframe's inertial factor (wv = 0: none)
    double vel0[3];             // insert: its camera's initial world velocity
    double icfg[12];            // solve: world gravity 0-2, priors on the oldest keyframe's biases:
                                // accelerometer 3-5 with weight 6, gyroscope 7-9 with weight 10
};

// Per-pair view (the scratch pointers are shared).
struct BaPair {
    double* T;
    double* Tfe;
    double* u;
    double* v;
    double* d;
    int32_t* lm;
    double* X;
    uint32_t* kf_desc;
    int64_t* gid;
    int32_t *remap, *cnt, *lm_id, *lpre, *cam_off, *counts, *tiles, *lo_o, *done;
    uint32_t* lmask;
    uint8_t* tc_fl;
    int32_t* tc_ids;
    uint8_t* keep;
    double *lo_uvd, *lo_W, *Xc, *obs_Vg, *lm_L, *lm_gp, *part, *C, *cam_U, *dc, *flops;
    double* imu;
    double *ine, *vel, *bias;
};

__device__ __forceinline__ BaPair ba_pair(const BatchCtx& c, const BaArgs& a, int p) {
    const size_t W = (size_t)a.W, K = (size_t)c.g.K, WK = W * K, M = TS_BA_MAXW;
    const BaStore& s = a.st;
    BaPair q;
    q.T = s.T + (size_t)p * a.W * 16;
    q.Tfe = s.Tfe + (size_t)p * a.W * 16;
    q.u = s.u + p * WK;
    q.v = s.v + p * WK;
    q.d = s.d + p * WK;
    q.lm = s.lm + p * WK;
    q.X = s.X + p * WK * 3;
    q.kf_desc = s.kf_desc + p * WK * 8;
    q.gid = s.gid + p * WK;
    // per-pair scratch (strides: ba_scratch_sizes in tslam_api.cpp)
    q.remap = s.remap + p * K; q.cnt = s.cnt + p * WK; q.lm_id = s.lm_id + p * WK;
    q.keep = s.keep + p * WK;
    q.lmask = s.lmask + p * (WK / 32 + 64); q.lpre = s.lpre + p * (WK / 32 + 64);
    q.tc_fl = s.tc_fl + p * (size_t)TS_BA_TILES * 256; q.tc_ids = s.tc_ids + p * (size_t)TS_BA_TILES * 2048;
    q.cam_off = s.cam_off + p * (W + 1);
    q.counts = s.counts + 4 * p;
    q.tiles = s.tiles + p * 2 * TS_BA_TILES;
    q.done = s.done + p;
    q.lo_o = s.lo_o + p * WK * M; q.lo_uvd = s.lo_uvd + p * WK * M * 4; q.lo_W = s.lo_W + p * WK * M * 18;
    q.Xc = s.Xc + p * WK * 3; q.obs_Vg = s.obs_Vg + p * WK * 9;
    q.lm_L = s.lm_L + p * WK * 6; q.lm_gp = s.lm_gp + p * WK * 3;
    q.part = s.part + p * (size_t)TS_BA_SPLIT * TS_BA_PART; q.C = s.C + p * 4096;
    q.cam_U = s.cam_U + p * W * 27; q.dc = s.dc + p * W * 6; q.flops = s.flops;
    q.imu = s.imu + p * W * 10;
    q.ine = s.ine + p * W * TS_BA_INE;
    q.vel = s.vel + p * W * 3;
    q.bias = s.bias + p * W * 6;
    return q;
}

void launch_ba_snapshot(const BatchCtx& c, double* dst, hipStream_t s);
// the batch's keyframes' temporal-match chains back to the previous keyframe frame (interval iv)
void launch_ba_kf_assoc(const BatchCtx& c, int32_t* dst, int iv, hipStream_t s);
void launch_ba_keyframe(const BatchCtx& c, const BaArgs& a, bool evict, hipStream_t s);
// timing: when non-null, an event pair is recorded around every k_ba_schur launch (profiling)
struct BaTiming {
    hipEvent_t* ev;   // 2 * cap events
    int cap, used;
};
// split: k_ba_reduce + k_ba_solve per iteration instead of k_ba_reduce_solve (same sums, bit for bit);
// inertial: the solve kernels with the window's inertial factors (velocities + accelerometer bias)
void launch_ba_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s, BaTiming* timing, bool split = false,
                     bool inertial = false);
// rig-level A8: the body snapshot of the batch, a keyframe's body pose (and every pair's camera at
// E_p^-1 B), and the joint solve over all pairs (storage pair c.P = the body window)
void launch_ba_snapshot_rig(const BatchCtx& c, double* dst, hipStream_t s);
void launch_ba_rig_keyframe(const BatchCtx& c, const BaArgs& a, hipStream_t s);
void launch_ba_rig_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s, BaTiming* timing, bool inertial = false);
// one k_ba_schur launch on the window state `a` (measurement replays)
void launch_ba_schur(const BatchCtx& c, const BaArgs& a, hipStream_t s);

// A pair window's keyframe as a device-resident record: the batch context, the eviction's
// arguments (remaining slots) and the solve's.  The *_rec kernels read it through two pointers,
// so one captured hipGraph per chain shape replays every keyframe of that shape: its first node
// (k_ba_setrec, the record by value) is the only one whose parameters change per replay.
struct BaRec {
    BatchCtx c;
    BaArgs evict;
    BaArgs a;
};
// The keyframe's chain on the record d (grids from the host copy `r`): eviction (when `evict`),
// gate / tile count / scatter, a.iters x (Schur + reduce-and-solve, or reduce + solve when
// `split`), back substitution — the launches of launch_ba_keyframe + launch_ba_solve, by pointer.
void launch_ba_chain_rec(const BaRec& r, const BaRec* d, bool evict, bool split, bool inertial, hipStream_t s);
// k_ba_setrec: copies the record (by value) to d
void launch_ba_setrec(const BaRec& r, BaRec* d, hipStream_t s);
// points graph node `node` (a captured k_ba_setrec) of `exec` at record r / destination d
hipError_t ba_graph_set_record(hipGraphExec_t exec, hipGraphNode_t node, const BaRec& r, BaRec* d);
