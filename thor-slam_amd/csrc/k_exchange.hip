// k_exchange.hip — the per-batch block of SURVEY.md §8e that the ranks all-gather over RCCL:
// per (frame, camera) K*8 B keypoints | K*32 B descriptors | L*4 B level counts, then per
// (frame, pair) T_rel (16 f64) | covariance (36 f64) | stats (8 i32).  One kernel gathers it from
// the ring buffers with 16-byte copies (a memcpy per piece would be ~2,300 API calls per batch).
#include "tslam_common.h"

__global__ __launch_bounds__(256) void k_pack(BatchCtx c, uint8_t* dst) {
    const int64_t K = c.g.K, L = c.g.n_levels;
    const int64_t per_cam = K * 40 + L * 4;
    const int item = blockIdx.x;   // f * C + cam, then trailer blocks
    if (item < c.n * c.C) {
        const int f = item / c.C, cam = item % c.C;
        const int slot = ring_slot(c, c.g0 + f);
        const size_t sc = (size_t)slot * c.C + cam;
        uint8_t* o = dst + (int64_t)item * per_cam;
        const uint4* kp = reinterpret_cast<const uint4*>(c.kps + sc * K * 2);
        const uint4* de = reinterpret_cast<const uint4*>(c.desc + sc * K * 8);
        // keypoints: K*8 B = K/2 uint4 (K even) ; descriptors: K*32 B = 2K uint4
        if ((K & 1) == 0 && (per_cam & 15) == 0) {
            uint4* ok = reinterpret_cast<uint4*>(o);
            for (int64_t i = threadIdx.x; i < K / 2; i += blockDim.x) ok[i] = kp[i];
            uint4* od = reinterpret_cast<uint4*>(o + K * 8);
            for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) od[i] = de[i];
        } else {
            const uint32_t* k32 = c.kps + sc * K * 2;
            const uint32_t* d32 = c.desc + sc * K * 8;
            for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) reinterpret_cast<uint32_t*>(o)[i] = k32[i];
            for (int64_t i = threadIdx.x; i < 8 * K; i += blockDim.x) reinterpret_cast<uint32_t*>(o + K * 8)[i] = d32[i];
        }
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x)
            reinterpret_cast<int32_t*>(o + K * 40)[i] = c.kcount[sc * L + i];
        return;
    }
    // pose trailer: one block covers up to 256 (frame, pair) records, 52 doubles + 8 ints each
    const int64_t feat = (int64_t)c.n * c.C * per_cam;
    const int nrec = c.n * c.P;
    const int r0 = (item - c.n * c.C) * 4;
    for (int r = r0; r < min(r0 + 4, nrec); ++r) {
        uint8_t* o = dst + feat + (int64_t)r * (52 * 8 + TS_STATS_INTS * 4);
        const double* pz = c.pose + (size_t)r * TS_POSE_DOUBLES;
        for (int i = threadIdx.x; i < 52; i += blockDim.x)
            reinterpret_cast<double*>(o)[i] = i < 16 ? pz[i] : pz[32 + (i - 16)];
        for (int i = threadIdx.x; i < TS_STATS_INTS; i += blockDim.x)
            reinterpret_cast<int32_t*>(o + 52 * 8)[i] = c.stats[(size_t)r * TS_STATS_INTS + i];
    }
}

void launch_pack(const BatchCtx& c, uint8_t* dst, hipStream_t s) {
    const int trailer_blocks = (c.n * c.P + 3) / 4;
    hipLaunchKernelGGL(k_pack, dim3(c.n * c.C + trailer_blocks), dim3(256), 0, s, c, dst);
}
