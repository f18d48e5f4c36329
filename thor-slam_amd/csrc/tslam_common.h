// tslam_common.h — device-side layout shared by the gfx950 kernels and the C-ABI host code.
//
// HBM layout (one handle = one device, P stereo pairs, C = 2P cameras, K keypoints/image,
// batch B frames, ring R = 2B frames so frame t-1 of a batch's first frame is still resident):
//
//   pyramid  u8  [R][C][pyr_bytes]   rectified level 0 + 2x2 box levels, each level dense (pitch W_l)
//   smooth   u8  [B][C][pyr_bytes]   5x5 binomial of every level (BRIEF sampling image)
//   cand     u32 [B][C][cand_total]  per (level, 16-row band) fixed-capacity key segments
//   ccount   u32 [B][C][total_bands] keys written per band
//   hist     u32 [B][C][L][256]      survivor histogram in key order (bin = 255 - score)
//   kps      u32 [R][C][K][2]        {x | y<<16, level | angle<<8 | score<<16}
//   kcount   i32 [R][C][L]
//   desc     u32 [R][C][K][8]        rBRIEF-256
//   qbest/qsecond/tbest u32 [B][P][2][K]   matching scratch (mode 0 stereo, 1 temporal)
//   stereo   i32 [R][P][K]  disp f64 [R][P][K]        stereo match + refined disparity of left kps
//   temporal i32 [B][P][K]  tuv  f64 [B][P][K][2]     temporal match + refined (u, v) at t
//   corr     f64 [B][P][K][8]        X Y Z du dv bx by bz (ordered by t keypoint index)
//   pose     f64 [B][P][68]          T_rel, T_abs, cov;  stats i32 [B][P][8];  state f64 [P][16]
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TS_MAX_LEVELS 6
#define TS_BAND_ROWS 16
#define TS_DET_HALO 4
#define TS_RECT_BAND 32
#define TS_MATCH_CHUNK 1024
#define TS_SAD_HALF 5
#define TS_SAD_RANGE 2
#define TS_POSE_DOUBLES 68
#define TS_STATS_INTS 8
#define TS_CORR_DOUBLES 8
#define TS_MAX_HYP 1024

struct LevelGeom {
    int n_levels;
    int W[TS_MAX_LEVELS], H[TS_MAX_LEVELS];
    int pyr_off[TS_MAX_LEVELS];
    int pyr_bytes;
    int K;
    int Kq[TS_MAX_LEVELS], koff[TS_MAX_LEVELS];
    int nbands[TS_MAX_LEVELS], band_start[TS_MAX_LEVELS];
    int total_bands;
    int cand_cap[TS_MAX_LEVELS];   // keys per band at level l
    int cand_off[TS_MAX_LEVELS];   // u32 offset of level l's first band segment (per image)
    int cand_total;                // u32 per image
    int qtiles[TS_MAX_LEVELS], qtile_start[TS_MAX_LEVELS];  // 256-query tiles per level
    int total_qtiles;
};

struct PairCalib {
    double fx, fy, cx, cy, fxb;     // fxb = fx * baseline
};

struct MatchParams {
    int max_hamming, ratio_pct, row_tol, max_disp, window;
};

struct PoseParams {
    int n_hyp, iters, min_inliers;
    double thr2;
    uint64_t seed;
};

// Everything a batch launch needs; built by the host per stage call.
struct BatchCtx {
    LevelGeom g;
    int C, P, B, R;
    int n;                 // frames in this batch
    int64_t g0;            // global index of the batch's first frame
    int W, H;              // level-0 size
    // inputs
    const uint8_t* images; // [n][C][H][W]
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
    uint32_t* qbest;
    uint32_t* qsecond;
    uint32_t* tbest;
    int32_t* stereo;
    double* disp;
    int32_t* temporal;
    double* tuv;
    double* corr;
    double* pose;
    int32_t* stats;
    double* state;
    const uint32_t* brief_table;  // [30][256] packed int8x4 (px, py, qx, qy)
    const int64_t* wedges;        // [31][2]
    PairCalib calib[8];
    MatchParams mp;
    PoseParams pp;
    int fast_threshold, margin;
};

static inline __host__ __device__ int ring_slot(const BatchCtx& c, int64_t g) { return (int)(g % c.R); }

// host launchers (one per stage kernel set)
void launch_rectify_pyramid(const BatchCtx& c, hipStream_t s);
void launch_detect(const BatchCtx& c, hipStream_t s);
void launch_select(const BatchCtx& c, hipStream_t s);
void launch_describe(const BatchCtx& c, hipStream_t s);
void launch_match(const BatchCtx& c, hipStream_t s);
void launch_match_refine(const BatchCtx& c, hipStream_t s);
void launch_pose(const BatchCtx& c, hipStream_t s);
void launch_chain(const BatchCtx& c, hipStream_t s);

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

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
