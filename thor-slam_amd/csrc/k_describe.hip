// k_describe.hip — row A5 of SURVEY.md §8a: intensity-centroid orientation + rotated BRIEF-256.
// One wave64 per keypoint: the 31-row orientation disc is read two rows per wave instruction
// (coalesced), the moments are reduced with cross-lane shuffles, and the 256 binary tests are
// four wave ballots (lane i of ballot k = test 64k + i), i.e. the descriptor is assembled in
// registers with no LDS and no atomics.  Bit-exact with oracle.orientation_bins / oracle.brief.
#include "tslam_common.h"

__global__ __launch_bounds__(256) void k_describe(BatchCtx c) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int img, local;
    if (!xcd_image_block(blockIdx.x, c.n * c.C, (c.g.K + 3) / 4, &img, &local)) return;
    const int pos = local * 4 + wave;          // y-sorted walk of the image (L1/L2 locality)
    const int cam = img % c.C;
    const int f = img / c.C;
    const int slot = ring_slot(c, c.g0 + f);
    if (pos >= c.g.K) return;
    int l;
    bool valid;
    const int kp_idx = ysorted_kp(c, c.yperm + ((size_t)slot * c.C + cam) * c.g.K,
                                  c.kcount + ((size_t)slot * c.C + cam) * c.g.n_levels, pos, &l, &valid);
    uint32_t* kp = c.kps + (((size_t)slot * c.C + cam) * c.g.K + kp_idx) * 2;
    const uint32_t meta = kp[1];
    uint32_t* dst = c.desc + (((size_t)slot * c.C + cam) * c.g.K + kp_idx) * 8;
    if (!valid) {
        if (lane < 8) dst[lane] = 0u;
        return;
    }
    const uint32_t xy = kp[0];
    const int x = xy & 0xFFFF, y = xy >> 16;
    const int W = c.g.W[l];
    const uint8_t* lev = c.pyr + ((size_t)slot * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l];
    const uint8_t* sm = c.smo + ((size_t)f * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l];

    // orientation moments over dx^2 + dy^2 <= 225
    int m10 = 0, m01 = 0;
    const int dx = (lane & 31) - 15;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int dy = -15 + 2 * it + (lane >> 5);
        if (dy <= 15 && dx <= 15 && dx * dx + dy * dy <= 225) {
            const int v = lev[(size_t)(y + dy) * W + (x + dx)];
            m10 += dx * v;
            m01 += dy * v;
        }
    }
    // integer sums are order-independent: DPP row sums + readlanes leave them in SGPRs, so the
    // wedge search below runs on the scalar unit
    m10 = __builtin_amdgcn_readfirstlane(wave_sum_dpp(m10));
    m01 = __builtin_amdgcn_readfirstlane(wave_sum_dpp(m01));
    // bin b: cross(u_b, v) >= 0 and cross(u_{b+1}, v) < 0, v = (m10, m01)
    int bin = 0;
    {
        int64_t prev = c.wedges[0] * (int64_t)m01 - c.wedges[1] * (int64_t)m10;
        for (int b = 0; b < 30; ++b) {
            const int64_t nxt = c.wedges[2 * (b + 1)] * (int64_t)m01 - c.wedges[2 * (b + 1) + 1] * (int64_t)m10;
            if (prev >= 0 && nxt < 0) {
                bin = b;
                break;
            }
            prev = nxt;
        }
    }
    // rotated BRIEF: test 64k + lane
    const uint32_t* tab = c.brief_table + bin * 256;
    uint32_t words[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t = tab[64 * k + lane];
        const int px = (int8_t)(t & 0xFF), py = (int8_t)((t >> 8) & 0xFF);
        const int qx = (int8_t)((t >> 16) & 0xFF), qy = (int8_t)(t >> 24);
        const int a = sm[(size_t)(y + py) * W + (x + px)];
        const int b = sm[(size_t)(y + qy) * W + (x + qx)];
        const uint64_t m = __ballot(a < b);
        words[2 * k] = (uint32_t)m;
        words[2 * k + 1] = (uint32_t)(m >> 32);
    }
    if (lane < 8) {
        uint32_t w = words[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
            if (lane == k) w = words[k];
        dst[lane] = w;
    }
    if (lane == 0) kp[1] = (meta & ~0xFF00u) | ((uint32_t)bin << 8);
}

void launch_describe(const BatchCtx& c, hipStream_t s) {
    const int bpi = (c.g.K + 3) / 4;
    hipLaunchKernelGGL(k_describe, dim3(xcd_grid(c.n * c.C, bpi)), dim3(256), 0, s, c);
}
