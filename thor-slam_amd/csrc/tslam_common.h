// tslam_common.h — device-side layout shared by the gfx950 kernels and the C-ABI host code.
//
// HBM layout (one handle = one device, P stereo pairs, C = 2P cameras, K keypoints/image,
// batch B frames, ring R = 2B + 1 frames (+ the keyframe interval with BA) so frame t-1 of a
// batch's first frame is still resident while the next batch's front stages run):
//
//   pyramid  u8  [R][C][pyr_bytes]   rectified level 0 + 2x2 box levels, each level dense (pitch W_l)
//   smooth   u8  [B][C][pyr_bytes]   5x5 binomial of every level (BRIEF sampling image)
//   cand     u32 [B][C][cand_total]  per (level, 16-row band) fixed-capacity key segments
//   ccount   u32 [B][C][total_bands] keys written per band
//   hist     u32 [B][C][L][256]      survivor histogram in key order (bin = 255 - score)
//   kps      u32 [R][C][K][2]        {x | y<<16, level | angle<<8 | score<<16}
//   kcount   i32 [R][C][L]
//   desc     u32 [R][C][K][8]        rBRIEF-256
//   ys       u32x4 [R][C][K]  desc_ys u32 [R][C][K][8]  per level, keypoints sorted by (y, rank):
//            {xy, level | score<<16, kp index, valid} and their descriptors (contiguous match staging)
//   rowstart u16 [R][C][sum(H_l+1)]  per level: first y-sorted position of row y
//   qbest/qsecond/tbest u32 [B][P][2][K]   matching scratch (mode 0 stereo, 1 temporal)
//   stereo   i32 [R][P][K]  disp f64 [R][P][K]        stereo match + refined disparity of left kps
//            (RGB-D: disp = fx / Z from the aligned depth, a virtual 1 m baseline; stereo = k or -1)
//   temporal i32 [R][P][K]  tuv  f64 [B][P][K][2]     temporal match + refined (u, v) at t
//   corr     f64 [B][P][K][8]        X Y Z du dv bx by bz (ordered by t keypoint index)
//   pose     f64 [B][P][68]          T_rel, T_abs, cov;  stats i32 [B][P][8];  state f64 [P][16]
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TS_MAX_LEVELS 6
// detect band height: 32 rows while the band's LDS (2 * rows + 10 rows of W bytes) stays <= 48 KiB
// (3 blocks per CU; fewer halo rows and barriers per pixel), else 24 or 16 (LevelGeom::band_rows)
#define TS_BAND_ROWS_MAX 32
#define TS_DET_HALO 4
#define TS_RECT_BAND 32
#define TS_MATCH_CHUNK 512
#define TS_SAD_HALF 5
#define TS_SAD_RANGE 2
#define TS_POSE_DOUBLES 68
#define TS_STATS_INTS 8
#define TS_CORR_DOUBLES 8
#define TS_MAX_HYP 1024
// one P3P candidate pose: [R 9 | t 3] f64, then f32 R 9, t 3, max |R_ij|, max |t_i| and 2 pad
// (the scoring pass reads the f32 record through scalar loads as operands of its inlier test)
#define TS_HYP_DOUBLES 20
#define TS_MAX_SPLITS 32   // RANSAC blocks per frame
#define TS_RANSAC_WORDS 26 // per split: key + pad + 12 doubles
#define TS_PRIOR_DOUBLES 16 // per (frame, pair): IMU prior R (row-major 3x3), W_r, t[3], W_t, 0, 0
#define TS_BA_CU_RESERVE 96   // CUs the front / back streams leave to the BA stream (tslam_submit_host;
                              // bench.py --front-cu-reserve sweep)
// Wave issue priority of the back kernels (match .. chain, rig pose): latency-bound waves that share
// the SIMDs with the next batch's front-end waves (detect, describe: throughput-bound) get served
// first (C2 234.7-235.3k -> 235.6-235.9k frames/s, C3 59.75k -> 60.05k; the front kernels at
// priority 1 or 2 instead were 1 % slower).  The local BA's kernels use 3 (k_ba.hip).
#define TS_BACK_PRIO __builtin_amdgcn_s_setprio(2)
#define TS_BA_MAXW 10      // keyframes per BA window (6 camera rows each in the 64-wide system)

struct LevelGeom {
    int n_levels;
    int W[TS_MAX_LEVELS], H[TS_MAX_LEVELS];
    int pyr_off[TS_MAX_LEVELS];
    int pyr_bytes;
    int K;
    int Kq[TS_MAX_LEVELS], koff[TS_MAX_LEVELS];
    int band_rows[TS_MAX_LEVELS];  // detect band height per level (LevelGeom rule in build_geometry)
    int smooth_groups[TS_MAX_LEVELS];   // detect smoothing: row groups per band (items = groups x quads)
    int det_lds;                   // detect dynamic LDS bytes: max over levels of (2 rows + 10) x W
    int nbands[TS_MAX_LEVELS], band_start[TS_MAX_LEVELS];
    int total_bands;
    int cand_cap[TS_MAX_LEVELS];   // keys per band at level l
    int cand_off[TS_MAX_LEVELS];   // u32 offset of level l's first band segment (per image)
    int cand_total;                // u32 per image
    int qtiles[TS_MAX_LEVELS], qtile_start[TS_MAX_LEVELS];  // 128-query k_match tiles per level
    int total_qtiles;
    int rs_off[TS_MAX_LEVELS];     // u16 offset of level l's row-start table (H_l + 1 entries)
    int rs_total;                  // u16 per image
    int dt_nx[TS_MAX_LEVELS], dt_start[TS_MAX_LEVELS];   // describe tiles: per row of level l, first tile
    int dt_total;                  // describe tiles per image
};

struct PairCalib {
    double fx, fy, cx, cy, fxb;     // fxb = fx * baseline
};

struct MatchParams {
    int max_hamming, ratio_pct, row_tol, max_disp, window;
};

struct PoseParams {
    int n_hyp, iters, min_inliers, splits;
    int mode;   // RANSAC scoring: 0 auto, 1 exhaustive (k_ransac_all), 2 bounded (k_ransac)
    int refine_block;   // k_refine threads per frame: 0 auto, 128, 256
    double thr2;
    uint64_t seed;
};

// Everything a batch launch needs; built by the host per stage call.
struct BatchCtx {
    LevelGeom g;
    int C, P, B, R;
    int cpp;               // cameras per pair: 2 (stereo), 1 (RGB-D: colour camera + aligned depth)
    int rgbd;
    int n;                 // frames in this batch
    // camera view of the front-end kernels (rectify .. describe): cameras cam0 .. cam0+ncam-1 of
    // every frame, images [n][ncam][H][W] (the whole rig: 0, C; a sharded rig: the rank's streams)
    int cam0, ncam;
    // pair view of the back-end kernels (match .. pose): pairs pair0 .. pair0+npair-1 of every
    // frame (the whole rig: 0, P; a camera-sharded RGB-D rig: the rank's cameras); batch buffers
    // keep their [n][P] layout
    int pair0, npair;
    int match_modes;       // k_match: 3 = temporal + stereo, 1 = stereo only (sharded pre-pass)
    int reloc;             // k_rig_pose solves a relocalisation (frame 0 is not a first frame)
    // peer layout of a sharded import (tslam_import_peers): images [world][nbuf][S][H][W] as the
    // all-to-all delivers them; the launch covers the world-1 peers' slots (not peer_me's), frames
    // peer_skip .. nbuf-1 of each (peer_S = 0: the plain [n][ncam] view above)
    int peer_S, peer_me, peer_nbuf, peer_skip;
    int64_t g0;            // global index of the batch's first frame
    int W, H;              // level-0 size
    // inputs
    const uint8_t* images; // [n][C][H][W] gray (RGB-D: the converted staging buffer)
    const uint8_t* rgbd_in; // RGB-D only: [n][P][BGR u8 H*W*3 | depth u16 mm H*W]
    const int32_t* maps;   // [C][H][W][2] or nullptr
    uint32_t map_mask;     // bit c set -> camera c has a map (else identity)
    // buffers
    uint8_t* pyr;
    uint8_t* smo;
    uint32_t* cand;
    uint32_t* ccount;
    uint32_t* hist;
    uint32_t* kps;
    int32_t* kcount;
    uint32_t* desc;
    uint4* ys;             // [R][C][K] y-sorted keypoint records
    uint32_t* desc_ys;     // [R][C][K][8] y-sorted descriptors
    uint16_t* rowstart;    // [R][C][rs_total]
    uint32_t* qbest;
    uint32_t* qsecond;
    uint32_t* tbest;
    int32_t* stereo;
    double* disp;
    int32_t* temporal;
    double* tuv;
    double* corr;
    double* pose;
    double* ransac;        // [B][P][TS_MAX_SPLITS][13] split winners (key word + pose)
    double* hyp;           // [B][P][4 * n_hyp][TS_HYP_DOUBLES] P3P candidate poses (k_p3p -> k_ransac)
    int32_t* stats;
    double* state;
    const double* prior;   // [B][P][16] IMU prior of the batch (tslam_set_motion_prior) or null
    // rig: base_T_rect-left of each pair and its inverse, body-frame results
    const double* rig_E;   // [P][16]
    const double* rig_Einv;
    double* rig_pose;      // [B][68]  body T_rel, T_abs, cov
    int32_t* rig_stats;    // [B][8]
    double* rig_state;     // [32]: the rig chain's (A, Q), two row-major 4x4 (k_pose.hip blocked chain)
    double* rig_prior;     // [B][16] body-frame IMU prior (k_rig_prior, from the pairs' priors) or null
    // A4 speculative FAST threshold (DESIGN.md §5 "detect"): te[cam][l] in use, its running
    // minimum for the next batch, per (frame, cam, level) fallback flags, launch mode
    // (0: te = max(t + 1, det_thr), flags set by select; 1: te = t + 1 for flagged images only)
    const uint32_t* det_thr;      // [C][L]
    uint32_t* det_thr_acc;        // [C][L]
    uint32_t* det_fail;           // [B][C][L]

    const uint32_t* brief_table;  // [30][256] LDS patch byte offsets of the two points (lo | hi << 16)
    const int64_t* wedges;        // [31][2]
    PairCalib calib[8];
    MatchParams mp;
    PoseParams pp;
    int fast_threshold, margin;
};

static inline __host__ __device__ int ring_slot(const BatchCtx& c, int64_t g) { return (int)(g % c.R); }

// sharded rig: frame ranges of the ranks (tslam_ranges.h)
#include "tslam_ranges.h"
// front-end image index (f * ncam + view camera) -> frame, rig camera; in the peer layout the
// index runs over (peer, frame, camera) of the world-1 peers
__device__ __forceinline__ void view_image(const BatchCtx& c, int img, int* f, int* cam) {
    if (c.peer_S) {
        const int per = c.n * c.peer_S, qq = img / per, q = qq < c.peer_me ? qq : qq + 1;
        const int r = img - qq * per;
        *f = r / c.peer_S;
        *cam = q * c.peer_S + (r - *f * c.peer_S);
        return;
    }
    *f = img / c.ncam;
    *cam = c.cam0 + (img - *f * c.ncam);
}
// the input image of view index img (its offset in c.images, in images)
__device__ __forceinline__ size_t view_src(const BatchCtx& c, int img) {
    if (c.peer_S) {
        const int per = c.n * c.peer_S, qq = img / per, q = qq < c.peer_me ? qq : qq + 1;
        const int r = img - qq * per, f = r / c.peer_S;
        return ((size_t)q * c.peer_nbuf + c.peer_skip + f) * c.peer_S + (r - f * c.peer_S);
    }
    return (size_t)img;
}

// host launchers (one per stage kernel set)
void launch_rectify_pyramid(const BatchCtx& c, hipStream_t s);
void launch_detect(const BatchCtx& c, hipStream_t s);
void launch_select(const BatchCtx& c, hipStream_t s);
void launch_describe(const BatchCtx& c, hipStream_t s);
void launch_match(const BatchCtx& c, hipStream_t s);
void launch_match_refine(const BatchCtx& c, hipStream_t s);
void launch_match_stereo(const BatchCtx& c, hipStream_t s);
void launch_pose(const BatchCtx& c, hipStream_t s);
void launch_chains(const BatchCtx& c, bool rig, hipStream_t s);   // every pair's chain (+ the rig's)
void launch_rig_pose(const BatchCtx& c, hipStream_t s);
// sharded rig exchange (k_exchange.hip): stream blocks (per frame x camera) and pose records (per frame)
int64_t stream_block_bytes(const LevelGeom& g);
int64_t pose_record_bytes(int P);
void launch_stream_blocks(const BatchCtx& c, bool pack, int64_t first, int n_frames, int cam_lo, int ncam, uint8_t* blk,
                          hipStream_t s);
// all peers at once (alltoall layout [world][cap][S][block], cap = peer_cap): pack this rank's
// cameras of every peer q's frames lo_q - 1 .. hi_q - 1 (slot q), or unpack every peer's cameras
// of frames lo_me - 1 .. hi_me - 1 (slot q <- cameras q*S ..); slot `me` untouched
void launch_stream_blocks_peers(const BatchCtx& c, bool pack, int64_t g0, int n, int world, int cap, int me, int S,
                                uint8_t* blk, hipStream_t s);
void launch_stage_raw_peers(const uint8_t* images, const uint8_t* prev, uint8_t* dst, int n, int world, int cap, int me,
                            int S, int64_t img_bytes, hipStream_t s);
void launch_pose_records(const BatchCtx& c, bool pack, int f0, int n, uint8_t* rec, hipStream_t s);
// every frame of the batch from the all-gather's padded layout [world][peer_records][record]
// (`pairs`: rank q's slot holds rig range rig_slot(q), tslam_ranges.h)
void launch_pose_records_gathered(const BatchCtx& c, int world, bool pairs, const uint8_t* rec, hipStream_t s);
// state blocks a sharded rank sends to rank 0 so that rank 0's ring holds what local BA, loop
// closure and relocalisation read (k_exchange.hip): per (frame of the sender's range, pair) the
// temporal matches + refined disparities, per (batch frame, left camera of the sender's streams)
// keypoints + level counts + descriptors; pack on the sender, unpack on rank 0 (per sender)
int64_t state_range_block_bytes(const LevelGeom& g);
int64_t state_camera_block_bytes(const LevelGeom& g);
void launch_state_blocks(const BatchCtx& c, bool pack, int n, int world, int rank, int cam_lo, int cam_hi, uint8_t* blk,
                         hipStream_t s);
// camera-sharded RGB-D rig: pair blocks (per batch frame x pair: pose, stats, correspondences)
int64_t pair_block_bytes(const LevelGeom& g);
void launch_pair_blocks(const BatchCtx& c, bool pack, int f0, int n_frames, int p0, int np, uint8_t* blk, hipStream_t s);
void launch_pose_solve(const BatchCtx& c, hipStream_t s);
void launch_perturb_uv(const BatchCtx& c, int percent, uint64_t seed, hipStream_t s);   // benchmark hook
void launch_reloc(const BatchCtx& c, int pair, int64_t frame, const double* map_xyz, const uint32_t* map_desc, int M,
                  int32_t* match, double* corr, int32_t* stats, double* pose, double* ransac, double* hyp, hipStream_t s);
void launch_reloc_rig(const BatchCtx& c, int64_t frame, const double* map_xyz, const uint32_t* map_desc, int M,
                      int32_t* match, double* corr, int32_t* stats, double* pose, double* ransac, double* hyp,
                      double* rig_pose, int32_t* rig_stats, hipStream_t s);
// relocalisation query image: keypoint records [K][2], level counts [L], descriptors [K][8] of one
// camera image (a ring slot's, or a keyframe database entry's snapshot)
struct RelocQuery {
    const uint32_t* kps;
    const int32_t* kcount;
    const uint32_t* desc;
};
static inline RelocQuery reloc_query_ring(const BatchCtx& c, int cam, int64_t frame) {
    const size_t ib = (size_t)ring_slot(c, frame) * c.C + cam;
    return {c.kps + ib * c.g.K * 2, c.kcount + ib * c.g.n_levels, c.desc + ib * c.g.K * 8};
}
// `dM` (device, may be null): the map size read on the device instead of M
void launch_reloc_query(const BatchCtx& c, int pair, int64_t frame, RelocQuery q, const double* map_xyz,
                        const uint32_t* map_desc, int M, const int32_t* dM, int32_t* match, double* corr, int32_t* stats,
                        double* pose, double* ransac, double* hyp, hipStream_t s);
// keyframe database (tslam_loop_*): entry e holds landmarks xyz [K][3] + desc [K][8] + count, and
// the snapshot of its image (kps [K][2], kcount [TS_MAX_LEVELS], desc [K][8])
struct LoopDb {
    double* xyz;
    uint32_t* desc;
    int32_t* n;
    uint32_t* snap_kps;
    int32_t* snap_kcount;
    uint32_t* snap_desc;
};
void launch_loop_store(const BatchCtx& c, int pair, int64_t frame, double* xyz, uint32_t* desc, int32_t* n_out,
                       hipStream_t s);
void launch_loop_store_auto(const BatchCtx& c, int interval, const LoopDb& db, int capk, bool rig, int64_t* count,
                            hipStream_t s);
void launch_loop_vote(const uint32_t* db_desc, const int32_t* db_n, int K, int S, int q_slot, int64_t k0, int capk, int P,
                      int n_cand, int max_hamming, int ratio_pct, int32_t* votes, hipStream_t s);
void launch_pose_graph_iteration(double* T, const int32_t* edges, const double* Z, const double* info, int N, int E,
                                 const int32_t* adj_off, const int32_t* adj, const int32_t* ftile, double* terms,
                                 double* H, double* g, double* delta, double* Ld, hipStream_t s);
// test hook: blocks >= 1 of every k_pg_potrf launch sleep `spins` x 127 x 64 cycles first
void pose_graph_test_delay(int spins);
void launch_pose_graph_cost(const double* T, const int32_t* edges, const double* Z, const double* info, int E,
                            double* terms, double* cost, hipStream_t s);
// TSDF volume + one integration launch (k_tsdf.hip)
#define TSDF_MAX_FRAMES 256
#define TSDF_POSE 13   // cam_T_world R (9), t (3), use flag
struct TsdfArgs {
    float* tsdf;
    float* weight;
    int nx, ny, nz;
    double ox, oy, oz, s;
    double trunc, max_dist, max_weight;
    const uint8_t* depth;      // frame 0's depth (u16 mm), frames `stride` bytes apart
    int64_t stride;
    int n;                     // frames
    int W, H;
    double fx, fy, cx, cy;
    const int32_t* map;        // [H][W][2] undistortion table (fixed point, 5 bits) or null
    const double* poses;       // [n][TSDF_POSE]
    // colour layer (null when off): frame 0's BGR image (frames `stride` bytes apart, as the
    // depth), the running colour [nv][3] (R, G, B) f32 and its weight f32
    const uint8_t* color;
    float* col;
    float* col_w;
};
void launch_tsdf(const BatchCtx& c, int pair, int f0, const double* host_wTc_dev, const TsdfArgs& a, double* poses,
                 hipStream_t s);
// dense-map outputs of the TSDF volume (k_dense.hip): marching-cubes mesh, capped exact ESDF
struct DenseArgs {
    const float* tsdf;
    const float* weight;
    int nx, ny, nz;
    uint32_t n_cubes;          // (nx - 1)(ny - 1)(nz - 1)
    int64_t n_voxels;
    double ox, oy, oz, s;      // volume corner and voxel size (voxel centres in f64, rounded to f32)
    float sf;                  // (float)s
    float min_weight;          // observed: weight >= min_weight
    float site_dist;           // ESDF site: |tsdf| <= site_dist
    float max_dist;            // ESDF value beyond R voxels
    int32_t cap;               // R^2 + 1
    const float* color;        // mesh: the colour layer [nv][3] or null (no vertex colours)
};
void launch_mesh_count(const DenseArgs& a, uint8_t* cfg, uint32_t* block_sums, uint64_t* block_off, uint64_t* total,
                       hipStream_t s);
void launch_mesh_emit(const DenseArgs& a, const uint8_t* cfg, const uint64_t* block_off, float* tris, float* cols,
                      int64_t cap, hipStream_t s);
void launch_esdf(const DenseArgs& a, int R, const float* tab, int32_t* g0, int32_t* g1, float* out, hipStream_t s);
void launch_esdf_slice(const DenseArgs& a, int y0, int y1, int R, const float* tab, int32_t* g0, int32_t* g1,
                       uint8_t* obs, float* out, hipStream_t s);
void launch_rgbd_gray(const BatchCtx& c, uint8_t* gray, hipStream_t s);
void launch_rgbd_depth(const BatchCtx& c, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

// Wave-uniform minimum via DPP row reductions (quad perms, half-row and row mirrors: VALU
// latency, no LDS crossbar) and four readlanes.  Requires all 64 lanes active.
__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false));  // row_mirror
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

// Wave-uniform sum via the same DPP row reduction (result in an SGPR).
__device__ __forceinline__ int wave_sum_dpp(int v) {
    // old = 0 (the identity) lets each step fuse into one v_add_u32_dpp; after the 4 row steps
    // every lane holds its row's sum, row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) fold
    // the rows into lane 63 — 6 VALU + 1 readlane instead of 4 DPP moves, 4 adds and 4 readlanes
    // (exact: integer sums, every lane of the wave active)
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return __builtin_amdgcn_readlane(v, 63);
}

// f64 DPP move (both halves) for the row reductions below.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
    switch (ctrl_sel) {   // constant after inlining
        case 0: lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false); break;
        case 1: lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false); break;
        case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, false); break;
        default: lo = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xF, 0xF, false); break;
    }
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// f64 DPP move with a compile-time control (e.g. quad_perm broadcasts 0x00/0x55/0xAA/0xFF).
template <int CTRL>
__device__ __forceinline__ double dpp_f64c(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// Wave-uniform f64 sum: DPP row reductions (no LDS crossbar) + four readlanes.  Requires all 64
// lanes active.  The summation order is fixed (deterministic run to run).
__device__ __forceinline__ double wave_sum_f64(double v) {
    v = v + dpp_f64(v, 0);
    v = v + dpp_f64(v, 1);
    v = v + dpp_f64(v, 2);
    v = v + dpp_f64(v, 3);
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// Wave sums of N <= 32 f64 values at once (a transposing butterfly): at the exchange with lane
// distance d = 32, 16, .., 2 every lane keeps half of its values (the upper half when lane & d)
// and adds its partner's copy of that half, so value k ends in lanes 2k and 2k + 1 after a last
// exchange at distance 1.  31 shuffles for 32 values instead of 32 separate reductions; a fixed
// order, so deterministic.  Returns the sum of value lane >> 1 (lanes past 2N hold zeros).
template <int N>
__device__ __forceinline__ double wave_multi_sum(const double (&in)[N]) {
    static_assert(N <= 32, "at most 32 values");
    double v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = k < N ? in[k] : 0.0;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int h = 16; h >= 1; h >>= 1) {   // values per lane after this exchange
        const int d = 2 * h;              // lane distance 32, 16, 8, 4, 2
        const bool upper = (lane & d) != 0;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            const double keep = upper ? v[h + j] : v[j];
            const double send = upper ? v[j] : v[h + j];
            v[j] = keep + __shfl_xor(send, d, 64);
        }
    }
    return v[0] + __shfl_xor(v[0], 1, 64);
}

// XCD-aware 1-D block mapping: blocks are dealt round-robin over the 8 XCDs, so block b runs on the
// XCD labelled b % 8.  Give all `bpi` blocks of one image the same label, so that image's pyramid
// lines are fetched into one L2 only.  Speed only: correctness never depends on placement.
// Launch with xcd_grid(n_img, bpi) blocks; returns false for the padding blocks.
static inline __host__ int xcd_grid(int n_img, int bpi) { return ((n_img + 7) / 8) * 8 * bpi; }
__device__ __forceinline__ bool xcd_image_block(int b, int n_img, int bpi, int* img, int* local) {
    const int k = b >> 3;
    *img = (k / bpi) * 8 + (b & 7);
    *local = k % bpi;
    return *img < n_img;
}

// Level of y-sorted position `pos` (levels are laid out back to back, koff[l] .. koff[l+1]).
__device__ __forceinline__ int pos_level(const LevelGeom& g, int pos) {
    int l = 0;
    while (l + 1 < g.n_levels && pos >= g.koff[l + 1]) ++l;
    return l;
}
