// tslam_ba.h — A8 local bundle adjustment: device storage and launch arguments (k_ba.hip).
//
// Per stereo pair p (persistent, W = ba_window slots, K keypoints per image):
//   T    f64 [P][W][16]     cam_T_world of each keyframe (BA estimate)
//   Tfe  f64 [P][W][16]     world_T_cam of the front end (tracking chain) at insertion
//   u v d f64 [P][W][K]     level-0 observation of every keypoint, disparity (NaN = none)
//   lm   i32 [P][W][K]      landmark id (home slot * K + keypoint) or -1
//   X    f64 [P][W*K][3]    landmark positions (world), indexed by id
// Per solve (scratch, shared by the pairs: their solves are ordered on one stream):
//   observation lists, per-landmark CSR, Jacobian blocks, the Schur columns Qt [3L][64] and the
//   split-K partials of C = Qt^T Qt.  The camera system is 64 wide: 6 rows per keyframe
//   (<= 10 keyframes = 60 rows) and row 60 = the landmark right-hand side.
#pragma once

#include "tslam_common.h"

#define TS_BA_MAXD 54   // 6 * (TS_BA_MAXW - 1): the reduced camera system without the gauge
#define TS_BA_SPLIT 128 // split-K blocks of the Schur GEMM

static_assert(6 * TS_BA_MAXW + 1 <= 64, "the BA camera system (6 rows per keyframe + rhs) is 64 wide");

struct BaStore {
    // persistent, pair 0 (pair stride: W*16 doubles for T/Tfe, W*K for u/v/d/lm, W*K*3 for X)
    double* T;
    double* Tfe;
    double* u;
    double* v;
    double* d;
    int32_t* lm;
    double* X;
    // scratch (sizes for W*K landmarks/observations)
    int32_t* remap;    // [K]
    int32_t* cnt;      // [WK] observations per landmark id (after the gate)
    int32_t* li;       // [WK] compact index per id or -1
    int32_t* lm_id;    // [WK] id per compact index
    int32_t* lm_off;   // [WK+1] CSR offsets
    int32_t* fill;     // [WK]
    int32_t* lm_obs;   // [WK] observation indices grouped by landmark
    int32_t* obs_cam;  // [WK] window position of the observing keyframe (0 = oldest)
    int32_t* obs_k;    // [WK]
    int32_t* obs_id;   // [WK]
    int32_t* cam_off;  // [W+1]
    int32_t* counts;   // [P][4] n_obs, L, solve ok, pad
    double* obs_W;     // [WK][18]  W_o = J_c^T J_p (6x3)
    double* obs_Ug;    // [WK][27]  J_c^T J_c (upper 21) | J_c^T r (6)
    double* lm_L;      // [WK][9]   Cholesky factor of V_i
    double* lm_gp;     // [WK][3]
    double* Qt;        // [3WK+4][64]
    double* part;      // [TS_BA_SPLIT][64][64]
    double* cam_U;     // [W][27]
    double* dc;        // [W][6]
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
    double lam, outlier_px;
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
    int32_t *remap, *cnt, *li, *lm_id, *lm_off, *fill, *lm_obs, *obs_cam, *obs_k, *obs_id, *cam_off, *counts;
    double *obs_W, *obs_Ug, *lm_L, *lm_gp, *Qt, *part, *cam_U, *dc;
};

__device__ __forceinline__ BaPair ba_pair(const BatchCtx& c, const BaArgs& a, int p) {
    const size_t WK = (size_t)a.W * c.g.K;
    const BaStore& s = a.st;
    BaPair q;
    q.T = s.T + (size_t)p * a.W * 16;
    q.Tfe = s.Tfe + (size_t)p * a.W * 16;
    q.u = s.u + p * WK;
    q.v = s.v + p * WK;
    q.d = s.d + p * WK;
    q.lm = s.lm + p * WK;
    q.X = s.X + p * WK * 3;
    q.remap = s.remap; q.cnt = s.cnt; q.li = s.li; q.lm_id = s.lm_id; q.lm_off = s.lm_off; q.fill = s.fill;
    q.lm_obs = s.lm_obs; q.obs_cam = s.obs_cam; q.obs_k = s.obs_k; q.obs_id = s.obs_id; q.cam_off = s.cam_off;
    q.counts = s.counts + 4 * p;
    q.obs_W = s.obs_W; q.obs_Ug = s.obs_Ug; q.lm_L = s.lm_L; q.lm_gp = s.lm_gp; q.Qt = s.Qt; q.part = s.part;
    q.cam_U = s.cam_U; q.dc = s.dc;
    return q;
}

void launch_ba_keyframe(const BatchCtx& c, const BaArgs& a, bool evict, hipStream_t s);
void launch_ba_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s);
