// k_reloc.hip — relocalisation in a loaded map (SlamEngine.relocalize,
// reference thor_slam/slam/interface.py:250-256).
//
// The map is a set of landmarks (world position f64 x3 + rBRIEF-256 descriptor), uploaded once.
// For one resident frame: every valid left keypoint is matched against ALL map descriptors by
// brute-force Hamming (best = lexicographic min of (distance, index), second = min over the
// others; accepted iff best <= max_hamming and 100 * best < ratio_pct * second), the matches
// become 3D-2D correspondences (world point, level-0 keypoint position) in keypoint order, and
// A7's P3P-RANSAC + Gauss-Newton solve cam_T_world (RNG seeded by the frame index).
#include "tslam_common.h"

#define RL_CHUNK 512   // map descriptors staged per LDS pass (16 KB)

// One thread per query keypoint; the block stages the map descriptors chunk by chunk (LDS
// broadcasts: every thread reads the same descriptor) and keeps best / second per query.
__global__ __launch_bounds__(256) void k_reloc_match(BatchCtx c, RelocQuery qi, const uint32_t* map_desc, int M_arg,
                                                     const int32_t* dM, int32_t* match) {
    __shared__ uint4 s_d[RL_CHUNK][2];
    const int K = c.g.K;
    const int M = dM ? *dM : M_arg;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = false;
    uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q < K) {
        const uint32_t meta = qi.kps[(size_t)q * 2 + 1];
        const int l = (int)(meta & 0xFF);
        valid = q - c.g.koff[l] < qi.kcount[l];
        const uint4* src = reinterpret_cast<const uint4*>(qi.desc + (size_t)q * 8);
        const uint4 a = src[0], b = src[1];
        d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    }
    uint32_t best = 0xFFFFFFFFu, second = 0xFFFFFFFFu;   // (distance << 20) | index
    for (int m0 = 0; m0 < M; m0 += RL_CHUNK) {
        const int nm = min(RL_CHUNK, M - m0);
        __syncthreads();
        for (int i = threadIdx.x; i < nm * 2; i += blockDim.x)
            s_d[i >> 1][i & 1] = reinterpret_cast<const uint4*>(map_desc + (size_t)(m0 + (i >> 1)) * 8)[i & 1];
        __syncthreads();
        if (!valid) continue;
        for (int j = 0; j < nm; ++j) {
            const uint4 a = s_d[j][0], b = s_d[j][1];
            const uint32_t dist = __builtin_popcount(d[0] ^ a.x) + __builtin_popcount(d[1] ^ a.y) +
                                  __builtin_popcount(d[2] ^ a.z) + __builtin_popcount(d[3] ^ a.w) +
                                  __builtin_popcount(d[4] ^ b.x) + __builtin_popcount(d[5] ^ b.y) +
                                  __builtin_popcount(d[6] ^ b.z) + __builtin_popcount(d[7] ^ b.w);
            const uint32_t key = (dist << 20) | (uint32_t)(m0 + j);
            if (key < best) {
                second = best;
                best = key;
            } else if (key < second) {
                second = key;
            }
        }
    }
    if (q >= K) return;
    int out = -1;
    if (valid && best != 0xFFFFFFFFu) {
        const uint32_t bd = best >> 20, sd = second >> 20;   // second: 4095 when absent
        if ((int)bd <= c.mp.max_hamming && (second == 0xFFFFFFFFu || 100u * bd < (uint32_t)c.mp.ratio_pct * sd))
            out = (int)(best & 0xFFFFFu);
    }
    match[q] = out;
}

// One block: the matches in keypoint order -> correspondence rows (A7 layout) + stats.  `xf`
// (row-major 3x4, or null): the map point enters as xf * X (the rig's per-pair frame E_p^-1).
__global__ __launch_bounds__(256) void k_reloc_corr(BatchCtx c, RelocQuery qi, int pair, const double* map_xyz,
                                                    const double* xf, const int32_t* match, double* corr, int32_t* stats,
                                                    double* pose, int64_t frame) {
    __shared__ int s_tmp[32];
    const int K = c.g.K;
    // the pose record starts as k_corr leaves it (identity T_rel, zeros): k_refine writes the 3x4
    // part only, and k_rig_pose reads the whole 4x4
    for (int i = threadIdx.x; i < TS_POSE_DOUBLES; i += blockDim.x) pose[i] = (i < 16 && (i % 5) == 0) ? 1.0 : 0.0;
    const PairCalib cal = c.calib[pair];
    const double fx = cal.fx, fy = cal.fy, cx = cal.cx, cy = cal.cy;
    int n = 0;
    for (int base = 0; base < K; base += blockDim.x) {
        const int q = base + threadIdx.x;
        const int m = q < K ? match[q] : -1;
        const int flag = m >= 0;
        // block exclusive scan of the flags
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        int x = flag;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_tmp[wave] = x;
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            if (w < wave) off += s_tmp[w];
            tot += s_tmp[w];
        }
        if (flag) {
            const uint32_t xy = qi.kps[(size_t)q * 2], meta = qi.kps[(size_t)q * 2 + 1];
            const double sc = (double)(1 << (meta & 0xFF));
            const double u = ((double)(xy & 0xFFFF) + 0.5) * sc - 0.5;
            const double v = ((double)(xy >> 16) + 0.5) * sc - 0.5;
            const double bx = (u - cx) / fx;
            const double by = (v - cy) / fy;
            const double nn = sqrt((bx * bx + by * by) + 1.0);
            double* cr = corr + (size_t)(n + off + x - flag) * TS_CORR_DOUBLES;
            const double X = map_xyz[(size_t)m * 3], Y = map_xyz[(size_t)m * 3 + 1], Z = map_xyz[(size_t)m * 3 + 2];
            if (xf) {
                for (int e = 0; e < 3; ++e) cr[e] = ((xf[4 * e] * X + xf[4 * e + 1] * Y) + xf[4 * e + 2] * Z) + xf[4 * e + 3];
            } else {
                cr[0] = X;
                cr[1] = Y;
                cr[2] = Z;
            }
            cr[3] = cx - u;
            cr[4] = cy - v;
            cr[5] = bx / nn;
            cr[6] = by / nn;
            cr[7] = 1.0 / nn;
        }
        n += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        stats[0] = n < max(6, c.pp.min_inliers) ? 1 : 3;   // 3 = "to be solved" (A7 convention)
        stats[1] = n;
        stats[2] = stats[3] = stats[6] = stats[7] = 0;
        stats[4] = -1;
        stats[5] = (int)frame;
    }
}

void launch_reloc(const BatchCtx& c, int pair, int64_t frame, const double* map_xyz, const uint32_t* map_desc, int M,
                  int32_t* match, double* corr, int32_t* stats, double* pose, double* ransac, double* hyp, hipStream_t s) {
    launch_reloc_query(c, pair, frame, reloc_query_ring(c, c.cpp * pair, frame), map_xyz, map_desc, M, nullptr, match, corr,
                       stats, pose, ransac, hyp, s);
}

// The same from an explicit query image (a keyframe database snapshot: loop verification jobs
// that run after the frame's ring slot was reused); frame = the RANSAC seed.
void launch_reloc_query(const BatchCtx& c, int pair, int64_t frame, RelocQuery q, const double* map_xyz,
                        const uint32_t* map_desc, int M, const int32_t* dM, int32_t* match, double* corr, int32_t* stats,
                        double* pose, double* ransac, double* hyp, hipStream_t s) {
    hipLaunchKernelGGL(k_reloc_match, dim3((c.g.K + 255) / 256), dim3(256), 0, s, c, q, map_desc, M, dM, match);
    hipLaunchKernelGGL(k_reloc_corr, dim3(1), dim3(256), 0, s, c, q, pair, map_xyz, (const double*)nullptr, match,
                       corr, stats, pose, frame);
    BatchCtx r = c;   // A7's RANSAC + refinement on the relocalisation scratch: one frame, one "pair"
    r.n = 1;
    r.P = 1;
    r.pair0 = 0;
    r.npair = 1;
    r.g0 = frame;
    r.prior = nullptr;   // no IMU prior: the solve is the map's alone
    r.rig_prior = nullptr;
    r.calib[0] = c.calib[pair];
    r.corr = corr;
    r.stats = stats;
    r.pose = pose;
    r.ransac = ransac;
    r.hyp = hyp;
    launch_pose_solve(r, s);
}

// Relocalisation of a rig (tslam_relocalize_rig): every pair matches its left image of the frame
// against the map (world = the rig's base frame) and sees the map points in its frame E_p^-1 X, so
// that A7 per pair gives T_p = cam_p_T(E_p^-1 world) and k_rig_pose's model X_c = E_q^-1 M E_q X'
// solves M = body_T_world from every pair's correspondences (candidates E_p T_p E_p^-1, scored on
// all pairs, joint Gauss-Newton).  Scratch per pair: match [P][K], and a one-frame, P-pair batch
// context (corr, stats, pose, ransac, hyp) + the rig record (rig_pose, rig_stats).
void launch_reloc_rig(const BatchCtx& c, int64_t frame, const double* map_xyz, const uint32_t* map_desc, int M,
                      int32_t* match, double* corr, int32_t* stats, double* pose, double* ransac, double* hyp,
                      double* rig_pose, int32_t* rig_stats, hipStream_t s) {
    const int K = c.g.K;
    for (int p = 0; p < c.P; ++p) {
        int32_t* mp = match + (size_t)p * K;
        const RelocQuery q = reloc_query_ring(c, c.cpp * p, frame);
        hipLaunchKernelGGL(k_reloc_match, dim3((K + 255) / 256), dim3(256), 0, s, c, q, map_desc, M, (const int32_t*)nullptr,
                           mp);
        hipLaunchKernelGGL(k_reloc_corr, dim3(1), dim3(256), 0, s, c, q, p, map_xyz, c.rig_Einv + 16 * p, mp,
                           corr + (size_t)p * K * TS_CORR_DOUBLES, stats + (size_t)p * TS_STATS_INTS,
                           pose + (size_t)p * TS_POSE_DOUBLES, frame);
    }
    BatchCtx r = c;   // one frame, every pair
    r.n = 1;
    r.pair0 = 0;
    r.npair = c.P;
    r.g0 = frame;
    r.corr = corr;
    r.stats = stats;
    r.pose = pose;
    r.ransac = ransac;
    r.hyp = hyp;
    r.prior = nullptr;
    r.rig_prior = nullptr;
    r.rig_pose = rig_pose;
    r.rig_stats = rig_stats;
    r.reloc = 1;
    launch_pose_solve(r, s);
    launch_rig_pose(r, s);
}
