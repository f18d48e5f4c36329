// k_describe.hip — row A5 of SURVEY.md §8a: intensity-centroid orientation + rotated BRIEF-256.
//
// One wave64 handles TS_DESC_KPW consecutive keypoints of the y-sorted walk of one image.  The
// kernel is latency-bound (each keypoint needs an index chain, then pixels, then the table row
// of its orientation bin), so a wave resolves all its keypoints' indices in one round trip,
// issues the pixel loads of all of them before using any, computes every orientation, then
// loads all table rows at once: 3 exposed memory latencies per wave instead of ~5 per keypoint.
// Only coalesced dword loads touch global memory (byte gathers cost one address cycle per cache
// line): the orientation disc is reduced straight from registers, and the 37x37 BRIEF patch is
// staged in the wave's own LDS slice, where the 512 rotated samples are byte reads.  The 256
// binary tests are four wave ballots (lane i of ballot k = test 64k + i); no atomics, no block
// barriers.  Bit-exact with oracle.orientation_bins / oracle.brief.
#include "tslam_common.h"

#define TS_BRIEF_ROWS 37   // rotated pattern offsets lie in [-18, 18]
#define TS_BRIEF_WORDS 10  // 40 bytes per staged row (37 columns at any alignment)
#define TS_ORIENT_WORDS 9  // 36 bytes per disc row (31 columns at any alignment)
#define TS_DESC_KPW 4      // keypoints per wave

// Round down to a dword boundary by pointer arithmetic (an integer round trip would turn the
// loads into flat loads, which the compiler then drains together with every scalar load).
__device__ __forceinline__ const uint8_t* align4(const uint8_t* p) { return p - ((uintptr_t)p & 3u); }

__global__ __launch_bounds__(256) void k_describe(BatchCtx c) {
    __shared__ uint32_t s_patch[4][TS_BRIEF_ROWS * TS_BRIEF_WORDS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int img, local;
    const int bpi = (c.g.K + 4 * TS_DESC_KPW - 1) / (4 * TS_DESC_KPW);
    if (!xcd_image_block(blockIdx.x, c.n * c.C, bpi, &img, &local)) return;
    const int pos0 = (local * 4 + wave) * TS_DESC_KPW;   // y-sorted walk (L1/L2 locality)
    if (pos0 >= c.g.K) return;
    const int cam = img % c.C;
    const int f = img / c.C;
    const int slot = ring_slot(c, c.g0 + f);
    const size_t ib = (size_t)slot * c.C + cam;
    uint32_t* kps = c.kps + ib * c.g.K * 2;
    uint32_t* desc = c.desc + ib * c.g.K * 8;

    // (1) index chain: lane k resolves position pos0 + k
    int my_idx = 0, my_lev = 0, my_ok = 0;
    uint32_t my_xy = 0, my_meta = 0;
    if (lane < TS_DESC_KPW && pos0 + lane < c.g.K) {
        bool v;
        my_idx = ysorted_kp(c, c.yperm + ib * c.g.K, c.kcount + ib * c.g.n_levels, pos0 + lane, &my_lev, &v);
        my_ok = v ? 1 : 2;   // 2 = padding slot (zero descriptor)
        if (v) {
            const uint2 e = *reinterpret_cast<const uint2*>(kps + (size_t)my_idx * 2);
            my_xy = e.x;
            my_meta = e.y;
        }
    }
    int kidx[TS_DESC_KPW], kok[TS_DESC_KPW], kx[TS_DESC_KPW], ky[TS_DESC_KPW], kW[TS_DESC_KPW];
    uint32_t kmeta[TS_DESC_KPW];
    const uint8_t* lev[TS_DESC_KPW];
    const uint8_t* q0[TS_DESC_KPW];
#pragma unroll
    for (int k = 0; k < TS_DESC_KPW; ++k) {
        kidx[k] = __builtin_amdgcn_readlane(my_idx, k);
        kok[k] = __builtin_amdgcn_readlane(my_ok, k);
        const uint32_t xy = (uint32_t)__builtin_amdgcn_readlane((int)my_xy, k);
        kmeta[k] = (uint32_t)__builtin_amdgcn_readlane((int)my_meta, k);
        const int l = __builtin_amdgcn_readlane(my_lev, k);
        kx[k] = xy & 0xFFFF;
        ky[k] = xy >> 16;
        kW[k] = c.g.W[l];
        lev[k] = c.pyr + ib * c.g.pyr_bytes + c.g.pyr_off[l] + (size_t)(ky[k] - 15) * kW[k] + (kx[k] - 15);
        q0[k] = c.smo + ((size_t)f * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l] + (size_t)(ky[k] - 18) * kW[k] + (kx[k] - 18);
    }

    // (2) every pixel load of the wave's keypoints before any use: the 31-row disc as 9 aligned
    // words per row (5 wave loads) and the 37-row patch as 10 words per row (6 wave loads)
    uint32_t od[TS_DESC_KPW][5], pd[TS_DESC_KPW][6];
#pragma unroll
    for (int k = 0; k < TS_DESC_KPW; ++k) {
        if (kok[k] != 1) continue;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int s = lane + 64 * i;
            const int r = s / TS_ORIENT_WORDS, w = s - TS_ORIENT_WORDS * r;
            od[k][i] = s < 31 * TS_ORIENT_WORDS ? *(const uint32_t*)(align4(lev[k] + (size_t)r * kW[k]) + 4 * w) : 0u;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int s = lane + 64 * i;
            const int r = s / TS_BRIEF_WORDS, w = s - TS_BRIEF_WORDS * r;
            pd[k][i] = s < TS_BRIEF_ROWS * TS_BRIEF_WORDS ? *(const uint32_t*)(align4(q0[k] + (size_t)r * kW[k]) + 4 * w) : 0u;
        }
    }

    // (3) orientation moments over dx^2 + dy^2 <= 225 from registers; the integer sums are
    // order-independent (DPP row sums + readlanes leave them in SGPRs).  Bin b: cross(u_b, v) >= 0
    // and cross(u_{b+1}, v) < 0 with v = (m10, m01); lane b tests wedge b, the lowest hit wins
    // (== the sequential first-match scan), no hit -> bin 0.
    int bin[TS_DESC_KPW];
    const int64_t wa0 = lane < 30 ? c.wedges[2 * lane] : 0, wa1 = lane < 30 ? c.wedges[2 * lane + 1] : 0;
    const int64_t wb0 = lane < 30 ? c.wedges[2 * lane + 2] : 0, wb1 = lane < 30 ? c.wedges[2 * lane + 3] : 0;
#pragma unroll
    for (int k = 0; k < TS_DESC_KPW; ++k) {
        bin[k] = 0;
        if (kok[k] != 1) continue;
        int m10 = 0, m01 = 0;
        const uintptr_t base = (uintptr_t)lev[k];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int s = lane + 64 * i;
            if (s < 31 * TS_ORIENT_WORDS) {
                const int r = s / TS_ORIENT_WORDS, w = s - TS_ORIENT_WORDS * r;
                const uintptr_t rp = base + (uintptr_t)r * kW[k];
                const int dx0 = (int)(((rp & ~(uintptr_t)3) + 4 * w) - rp) - 15, dy = r - 15;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int dx = dx0 + j, v = (od[k][i] >> (8 * j)) & 0xFF;
                    if (dx * dx + dy * dy <= 225) {
                        m10 += dx * v;
                        m01 += dy * v;
                    }
                }
            }
        }
        m10 = __builtin_amdgcn_readfirstlane(wave_sum_dpp(m10));
        m01 = __builtin_amdgcn_readfirstlane(wave_sum_dpp(m01));
        const bool hit = lane < 30 && (wa0 * (int64_t)m01 - wa1 * (int64_t)m10) >= 0 &&
                         (wb0 * (int64_t)m01 - wb1 * (int64_t)m10) < 0;
        const uint64_t m = __ballot(hit);
        bin[k] = m ? (int)__builtin_ctzll(m) : 0;
    }

    // (4) the table rows of all bins at once, then BRIEF per keypoint out of the LDS patch
    uint32_t tab[TS_DESC_KPW][4];
#pragma unroll
    for (int k = 0; k < TS_DESC_KPW; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) tab[k][j] = kok[k] == 1 ? c.brief_table[bin[k] * 256 + 64 * j + lane] : 0u;
    uint8_t* patch = (uint8_t*)s_patch[wave];
#pragma unroll
    for (int k = 0; k < TS_DESC_KPW; ++k) {
        if (kok[k] == 0) continue;
        uint32_t* dst = desc + (size_t)kidx[k] * 8;
        if (kok[k] == 2) {
            if (lane < 8) dst[lane] = 0u;
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // previous keypoint's reads first
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int s = lane + 64 * i;
            if (s < TS_BRIEF_ROWS * TS_BRIEF_WORDS) s_patch[wave][s] = pd[k][i];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // patch writes before reads
        const uintptr_t base = (uintptr_t)q0[k];
        uint32_t words[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t t = tab[k][j];
            const int px = (int8_t)(t & 0xFF), py = (int8_t)((t >> 8) & 0xFF);
            const int qx = (int8_t)((t >> 16) & 0xFF), qy = (int8_t)(t >> 24);
            const uintptr_t ra = base + (uintptr_t)(py + 18) * kW[k], rb = base + (uintptr_t)(qy + 18) * kW[k];
            const int a = patch[(py + 18) * (4 * TS_BRIEF_WORDS) + (int)(ra & 3) + px + 18];
            const int b = patch[(qy + 18) * (4 * TS_BRIEF_WORDS) + (int)(rb & 3) + qx + 18];
            const uint64_t m = __ballot(a < b);
            words[2 * j] = (uint32_t)m;
            words[2 * j + 1] = (uint32_t)(m >> 32);
        }
        if (lane < 8) {
            uint32_t w = words[0];
#pragma unroll
            for (int j = 1; j < 8; ++j)
                if (lane == j) w = words[j];
            dst[lane] = w;
        }
        if (lane == 0) kps[(size_t)kidx[k] * 2 + 1] = (kmeta[k] & ~0xFF00u) | ((uint32_t)bin[k] << 8);
    }
}

void launch_describe(const BatchCtx& c, hipStream_t s) {
    const int bpi = (c.g.K + 4 * TS_DESC_KPW - 1) / (4 * TS_DESC_KPW);
    hipLaunchKernelGGL(k_describe, dim3(xcd_grid(c.n * c.C, bpi)), dim3(256), 0, s, c);
}
