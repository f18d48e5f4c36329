// k_tsdf.hip — RGB-D dense mapping: projective TSDF integration (nvblox
// parameters of launch/thor_nvblox.launch.py:26-36).  CPU restatement and spec:
// oracle/numpy_tsdf.py.
//
// The volume is a dense voxel grid resident in HBM (tsdf f32 + weight f32, [nz][ny][nx]) in the
// tracking world frame.  One launch integrates a whole batch of depth frames: thread per voxel of a 16x4x4 brick,
// the batch's camera poses in LDS, and the voxel's (tsdf, weight) loaded on its first update and
// stored once after the last frame — the per-voxel update order is the frame order, so a batch
// equals one call per frame, while the voxel read-modify-write traffic is paid once per batch.
//
//   k_tsdf_poses      per frame: cam_T_world (3x4) + a use flag, from the host's world_T_cam or
//                     from the batch's device-resident chained poses (tracked frames only);
//   k_tsdf_integrate  per 16x4x4 brick: the frames whose view can reach the brick (bounding
//                     sphere vs the frustum, one frame per thread, ballot), then per voxel for
//                     each of those frames project the centre (f64), nearest depth pixel through
//                     the undistortion table, truncated signed distance, weighted average;
//                     with the colour layer, the same pixel's colour averaged into the voxels
//                     inside the truncation band (nvblox's colour integration).
#include "tslam_common.h"

// host poses: world_T_cam [n][16] -> cam_T_world; device poses: T_abs of batch frames (f0 + i)
__global__ void k_tsdf_poses(BatchCtx c, int pair, int f0, const double* host_wTc, int n, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* T;
    double use = 1.0;
    if (host_wTc) {
        T = host_wTc + 16 * (size_t)i;
        use = __builtin_isfinite(T[0]) ? 1.0 : 0.0;   // NaN pose: skip the frame
    } else {
        const size_t o = (size_t)(f0 + i) * c.P + pair;
        T = c.pose + o * TS_POSE_DOUBLES + 16;
        const int st = c.stats[o * TS_STATS_INTS];
        use = (st == 0 || (st == 2 && c.g0 + f0 + i == 0)) ? 1.0 : 0.0;   // tracked, or the first frame
    }
    double* q = out + (size_t)i * TSDF_POSE;
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k) q[3 * r + k] = T[4 * k + r];   // R^T
        q[9 + r] = -((T[r] * T[3] + T[4 + r] * T[7]) + T[8 + r] * T[11]);
    }
    q[12] = use;
}

// Bricks of 16 x 4 x 4 voxels, one per 256-thread block (x rows of 64 B stay coalesced).  Before
// touching a voxel the block decides, one frame per thread, which frames can see ANY voxel of its
// brick: the brick's bounding sphere against the conditions the per-voxel test applies
// (p_z > 0, p_z <= max_dist + trunc, 0 <= floor(u + 1/2) < W, same for v — the four image
// borders are planes through the camera centre).  The cull is conservative (radius inflated by 1 %
// + 1 um against rounding), so every update the exact per-voxel test would make still happens,
// in frame order: results are unchanged, while (brick, frame) pairs outside the view cost one
// sphere test per block instead of a projection per voxel (nvblox's "blocks in view" step).
#define TSDF_BX 16
#define TSDF_BY 4
#define TSDF_BZ 4

__device__ __forceinline__ bool tsdf_brick_visible(const TsdfArgs& a, const double* q, double X, double Y, double Z,
                                                   double R) {
    if (q[12] == 0.0) return false;
    const double pz = ((q[6] * X + q[7] * Y) + q[8] * Z) + q[11];
    if (pz + R <= 0.0) return false;                      // every voxel has p_z <= 0
    if (pz - R > a.max_dist + a.trunc) return false;      // p_z > d + trunc for every valid depth
    const double px = ((q[0] * X + q[1] * Y) + q[2] * Z) + q[9];
    const double py = ((q[3] * X + q[4] * Y) + q[5] * Z) + q[10];
    // u + 1/2 >= 0  <=>  fx p_x + (cx + 1/2) p_z >= 0;  u + 1/2 < W  <=>  fx p_x + (cx + 1/2 - W) p_z < 0
    const double cl = a.cx + 0.5, cr = a.cx + 0.5 - a.W, ct = a.cy + 0.5, cb = a.cy + 0.5 - a.H;
    if (a.fx * px + cl * pz + R * sqrt(a.fx * a.fx + cl * cl) < 0.0) return false;
    if (a.fx * px + cr * pz - R * sqrt(a.fx * a.fx + cr * cr) >= 0.0) return false;
    if (a.fy * py + ct * pz + R * sqrt(a.fy * a.fy + ct * ct) < 0.0) return false;
    if (a.fy * py + cb * pz - R * sqrt(a.fy * a.fy + cb * cb) >= 0.0) return false;
    return true;
}

__global__ __launch_bounds__(256) void k_tsdf_integrate(TsdfArgs a, int nbx, int nby) {
    __shared__ double s_p[TSDF_MAX_FRAMES * TSDF_POSE];
    __shared__ uint64_t s_mask[TSDF_MAX_FRAMES / 64];
    for (int i = threadIdx.x; i < a.n * TSDF_POSE; i += blockDim.x) s_p[i] = a.poses[i];
    const int b = blockIdx.x;
    const int i0 = (b % nbx) * TSDF_BX, j0 = ((b / nbx) % nby) * TSDF_BY, k0 = (b / (nbx * nby)) * TSDF_BZ;
    const int ex = min(TSDF_BX, a.nx - i0), ey = min(TSDF_BY, a.ny - j0), ez = min(TSDF_BZ, a.nz - k0);
    __syncthreads();
    {   // frames that may see the brick: thread t tests frame t (t < TSDF_MAX_FRAMES = blockDim)
        const int t = threadIdx.x;
        bool vis = false;
        if (t < a.n) {
            const double BX = a.ox + a.s * (i0 + 0.5 * ex), BY = a.oy + a.s * (j0 + 0.5 * ey),
                         BZ = a.oz + a.s * (k0 + 0.5 * ez);
            const double R = 0.5 * a.s * sqrt((double)(ex * ex + ey * ey + ez * ez)) * 1.01 + 1e-6;
            vis = tsdf_brick_visible(a, s_p + t * TSDF_POSE, BX, BY, BZ, R);
        }
        const uint64_t m = __ballot(vis);
        if ((t & 63) == 0) s_mask[t >> 6] = m;
    }
    __syncthreads();
    const int ti = threadIdx.x % TSDF_BX, tj = (threadIdx.x / TSDF_BX) % TSDF_BY, tk = threadIdx.x / (TSDF_BX * TSDF_BY);
    if (ti >= ex || tj >= ey || tk >= ez) return;
    const int i = i0 + ti, j = j0 + tj, k = k0 + tk;
    const int64_t v = ((int64_t)k * a.ny + j) * a.nx + i;
    const double X = a.ox + a.s * (i + 0.5), Y = a.oy + a.s * (j + 0.5), Z = a.oz + a.s * (k + 0.5);
    bool loaded = false;
    double ts = 0.0, w = 0.0;
    double cr = 0.0, cg = 0.0, cb = 0.0, cw = 0.0;   // colour layer (loaded with the voxel)
    for (int wd = 0; wd < (a.n + 63) / 64; ++wd) {
        uint64_t m = s_mask[wd];   // wave-uniform: frames in order
        while (m) {
            const int f = wd * 64 + __builtin_ctzll(m);
            m &= m - 1;
            const double* q = s_p + f * TSDF_POSE;   // LDS broadcast
            const double pz = ((q[6] * X + q[7] * Y) + q[8] * Z) + q[11];
            if (!(pz > 0.0)) continue;
            const double px = ((q[0] * X + q[1] * Y) + q[2] * Z) + q[9];
            const double py = ((q[3] * X + q[4] * Y) + q[5] * Z) + q[10];
            const double u = a.fx * px / pz + a.cx, vv = a.fy * py / pz + a.cy;
            const double fu = floor(u + 0.5), fv = floor(vv + 0.5);
            if (!(fu >= 0.0 && fu < a.W && fv >= 0.0 && fv < a.H)) continue;
            int ix = (int)fu, iy = (int)fv;
            if (a.map) {
                const int32_t* mp = a.map + ((size_t)iy * a.W + ix) * 2;
                ix = min(max((mp[0] + 16) >> 5, 0), a.W - 1);
                iy = min(max((mp[1] + 16) >> 5, 0), a.H - 1);
            }
            const uint16_t mm = reinterpret_cast<const uint16_t*>(a.depth + (size_t)f * a.stride)[(size_t)iy * a.W + ix];
            const double d = (double)mm * 0.001;
            if (!(d > 0.0 && d <= a.max_dist)) continue;
            const double sdf = d - pz;
            if (sdf < -a.trunc) continue;
            const double obs = fmin(sdf, a.trunc);
            if (!loaded) {
                ts = (double)a.tsdf[v];
                w = (double)a.weight[v];
                if (a.col) {
                    cr = (double)a.col[3 * v];
                    cg = (double)a.col[3 * v + 1];
                    cb = (double)a.col[3 * v + 2];
                    cw = (double)a.col_w[v];
                }
                loaded = true;
            }
            const double w1 = w + 1.0;
            ts = (double)(float)((ts * w + obs) / w1);   // stored as f32 after every frame (as the oracle)
            w = (double)(float)fmin(w1, a.max_weight);
            if (a.col && sdf <= a.trunc) {   // colour inside the truncation band: the same pixel's BGR
                const uint8_t* px = a.color + (size_t)f * a.stride + ((size_t)iy * a.W + ix) * 3;
                const double c1 = cw + 1.0;
                cr = (double)(float)((cr * cw + (double)px[2]) / c1);
                cg = (double)(float)((cg * cw + (double)px[1]) / c1);
                cb = (double)(float)((cb * cw + (double)px[0]) / c1);
                cw = (double)(float)fmin(c1, a.max_weight);
            }
        }
    }
    if (loaded) {
        a.tsdf[v] = (float)ts;
        a.weight[v] = (float)w;
        if (a.col) {
            a.col[3 * v] = (float)cr;
            a.col[3 * v + 1] = (float)cg;
            a.col[3 * v + 2] = (float)cb;
            a.col_w[v] = (float)cw;
        }
    }
}

void launch_tsdf(const BatchCtx& c, int pair, int f0, const double* host_wTc_dev, const TsdfArgs& a, double* poses,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_tsdf_poses, dim3((a.n + 63) / 64), dim3(64), 0, s, c, pair, f0, host_wTc_dev, a.n, poses);
    TsdfArgs b = a;
    b.poses = poses;
    const int nbx = (a.nx + TSDF_BX - 1) / TSDF_BX, nby = (a.ny + TSDF_BY - 1) / TSDF_BY,
              nbz = (a.nz + TSDF_BZ - 1) / TSDF_BZ;
    hipLaunchKernelGGL(k_tsdf_integrate, dim3((unsigned)((int64_t)nbx * nby * nbz)), dim3(256), 0, s, b, nbx, nby);
}
