// k_tsdf.hip — RGB-D dense mapping: projective TSDF integration (nvblox
// parameters of launch/thor_nvblox.launch.py:26-36).  CPU restatement and spec:
// oracle/numpy_tsdf.py.
//
// The volume is a dense voxel grid resident in HBM (tsdf f32 + weight f32, [nz][ny][nx]) in the
// tracking world frame.  One launch integrates a whole batch of depth frames: thread per voxel,
// the batch's camera poses in LDS, and the voxel's (tsdf, weight) loaded on its first update and
// stored once after the last frame — the per-voxel update order is the frame order, so a batch
// equals one call per frame, while the voxel read-modify-write traffic is paid once per batch.
//
//   k_tsdf_poses      per frame: cam_T_world (3x4) + a use flag, from the host's world_T_cam or
//                     from the batch's device-resident chained poses (tracked frames only);
//   k_tsdf_integrate  per voxel: for each frame project the centre (f64), nearest depth pixel
//                     through the undistortion table, truncated signed distance, weighted average.
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

__global__ __launch_bounds__(256) void k_tsdf_integrate(TsdfArgs a) {
    __shared__ double s_p[TSDF_MAX_FRAMES * TSDF_POSE];
    for (int i = threadIdx.x; i < a.n * TSDF_POSE; i += blockDim.x) s_p[i] = a.poses[i];
    __syncthreads();
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nv = (int64_t)a.nx * a.ny * a.nz;
    if (v >= nv) return;
    const int i = (int)(v % a.nx), j = (int)((v / a.nx) % a.ny), k = (int)(v / ((int64_t)a.nx * a.ny));
    const double X = a.ox + a.s * (i + 0.5), Y = a.oy + a.s * (j + 0.5), Z = a.oz + a.s * (k + 0.5);
    bool loaded = false;
    double ts = 0.0, w = 0.0;
    for (int f = 0; f < a.n; ++f) {
        const double* q = s_p + f * TSDF_POSE;   // LDS broadcast
        if (q[12] == 0.0) continue;
        const double pz = ((q[6] * X + q[7] * Y) + q[8] * Z) + q[11];
        if (!(pz > 0.0)) continue;
        const double px = ((q[0] * X + q[1] * Y) + q[2] * Z) + q[9];
        const double py = ((q[3] * X + q[4] * Y) + q[5] * Z) + q[10];
        const double u = a.fx * px / pz + a.cx, vv = a.fy * py / pz + a.cy;
        const double fu = floor(u + 0.5), fv = floor(vv + 0.5);
        if (!(fu >= 0.0 && fu < a.W && fv >= 0.0 && fv < a.H)) continue;
        int ix = (int)fu, iy = (int)fv;
        if (a.map) {
            const int32_t* m = a.map + ((size_t)iy * a.W + ix) * 2;
            ix = min(max((m[0] + 16) >> 5, 0), a.W - 1);
            iy = min(max((m[1] + 16) >> 5, 0), a.H - 1);
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
            loaded = true;
        }
        const double w1 = w + 1.0;
        ts = (double)(float)((ts * w + obs) / w1);   // stored as f32 after every frame (as the oracle)
        w = (double)(float)fmin(w1, a.max_weight);
    }
    if (loaded) {
        a.tsdf[v] = (float)ts;
        a.weight[v] = (float)w;
    }
}

void launch_tsdf(const BatchCtx& c, int pair, int f0, const double* host_wTc_dev, const TsdfArgs& a, double* poses,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_tsdf_poses, dim3((a.n + 63) / 64), dim3(64), 0, s, c, pair, f0, host_wTc_dev, a.n, poses);
    TsdfArgs b = a;
    b.poses = poses;
    const int64_t nv = (int64_t)a.nx * a.ny * a.nz;
    hipLaunchKernelGGL(k_tsdf_integrate, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, b);
}
