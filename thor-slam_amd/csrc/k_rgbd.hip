// k_rgbd.hip — RGB-D input (BASELINE.json configs[4]): a colour camera with a
// depth image aligned to it (the Luxonis RGB-D stream, luxonis.py:876-919: BGR u8 + u16 mm, depth
// aligned to CAM_A with the colour camera's K and D, :1018-1030).
//
// Each "pair" of the handle is then one colour camera (cameras per pair = 1).  Per frame and
// camera the input record is [BGR u8 H*W*3 | depth u16 H*W].  The colour image becomes the gray
// image of the usual path (same fixed-point BT.601 weights as HipSlamEngine.bgr_to_gray), and
// instead of stereo matching every keypoint reads the depth at its nearest raw pixel (through the
// undistortion map) and stores disp = fx / Z: with a virtual 1 m baseline (fx*B = fx) the pose
// stage's Z = fx*B / disp and the BA's disparity row are unchanged.
#include "tslam_common.h"

// BGR -> gray, 4 pixels per thread (3 dword loads, 1 dword store) when W*H is a multiple of 4.
__global__ __launch_bounds__(256) void k_rgbd_gray(BatchCtx c, uint8_t* gray) {
    const int img = blockIdx.y;   // view image f * ncam + (camera - cam0): input and output [n][ncam]
    const size_t npx = (size_t)c.W * c.H;
    const uint8_t* src = c.rgbd_in + (size_t)img * npx * 5;
    uint8_t* dst = gray + (size_t)img * npx;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((npx & 3) == 0) {
        if (4 * i >= npx) return;
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src) + 3 * i;
        const uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];
        const uint8_t px[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                                (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                                (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
        uint32_t out = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = px[3 * k], g = px[3 * k + 1], r = px[3 * k + 2];
            out |= ((r * 4899u + g * 9617u + b * 1868u + 8192u) >> 14) << (8 * k);
        }
        reinterpret_cast<uint32_t*>(dst)[i] = out;
    } else {
        for (size_t k = 4 * i; k < 4 * i + 4 && k < npx; ++k) {
            const uint32_t b = src[3 * k], g = src[3 * k + 1], r = src[3 * k + 2];
            dst[k] = (uint8_t)((r * 4899u + g * 9617u + b * 1868u + 8192u) >> 14);
        }
    }
}

// One thread per (frame, camera, keypoint): disp = fx / (depth_mm * 0.001) at the raw pixel nearest
// to the keypoint (level-0 position rounded, then mapped through the undistortion table), NaN when
// the keypoint is padding or the depth is 0.  stereo = the keypoint itself (or -1).
__global__ __launch_bounds__(256) void k_rgbd_depth(BatchCtx c) {
    const int K = c.g.K;
    const int fl = blockIdx.y, p = c.pair0 + fl % c.npair, f = fl / c.npair;   // camera p = pair p
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int slot = ring_slot(c, c.g0 + f);
    const size_t ib = (size_t)slot * c.C + p;
    const uint32_t* kp = c.kps + (ib * K + k) * 2;
    const int l = (int)(kp[1] & 0xFF);
    const bool valid = k - c.g.koff[l] < c.kcount[ib * c.g.n_levels + l];
    double disp = __builtin_nan("");
    if (valid) {
        const double sc = (double)(1 << l);
        const double u = ((double)(kp[0] & 0xFFFF) + 0.5) * sc - 0.5;
        const double v = ((double)(kp[0] >> 16) + 0.5) * sc - 0.5;
        int ix = min(max((int)floor(u + 0.5), 0), c.W - 1);
        int iy = min(max((int)floor(v + 0.5), 0), c.H - 1);
        if (c.maps && ((c.map_mask >> p) & 1u)) {
            const int32_t* m = c.maps + (((size_t)p * c.H + iy) * c.W + ix) * 2;
            ix = min(max((m[0] + 16) >> 5, 0), c.W - 1);
            iy = min(max((m[1] + 16) >> 5, 0), c.H - 1);
        }
        const size_t npx = (size_t)c.W * c.H;
        // the input records are the front-end view's, [n][ncam] from camera cam0
        const uint16_t* depth = reinterpret_cast<const uint16_t*>(c.rgbd_in + ((size_t)f * c.ncam + (p - c.cam0)) * npx * 5 + npx * 3);
        const uint32_t mm = depth[(size_t)iy * c.W + ix];
        if (mm) disp = c.calib[p].fx / ((double)mm * 0.001);
    }
    const size_t o = ((size_t)slot * c.P + p) * K + k;
    c.disp[o] = disp;
    c.stereo[o] = __builtin_isfinite(disp) ? k : -1;
}

void launch_rgbd_gray(const BatchCtx& c, uint8_t* gray, hipStream_t s) {
    const size_t groups = ((size_t)c.W * c.H + 3) / 4;
    hipLaunchKernelGGL(k_rgbd_gray, dim3((unsigned)((groups + 255) / 256), c.n * c.ncam), dim3(256), 0, s, c, gray);
}

void launch_rgbd_depth(const BatchCtx& c, hipStream_t s) {
    hipLaunchKernelGGL(k_rgbd_depth, dim3((c.g.K + 255) / 256, c.n * c.npair), dim3(256), 0, s, c);
}
